"""Data model mirroring the reference's types on the DoLimit path.

pb.RateLimitRequest / RateLimitDescriptor / RateLimitResponse_DescriptorStatus
(go-control-plane v0.9.7 rls.proto), config.RateLimit (src/config/config.go:19-25),
stats.RateLimitStats (src/stats/manager.go:47-55).
"""
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

UNKNOWN, OK, OVER_LIMIT = 0, 1, 2
SECOND, MINUTE, HOUR, DAY = 1, 2, 3, 4


@dataclass
class RateLimitStats:
    key: str
    total_hits: int = 0
    over_limit: int = 0
    near_limit: int = 0
    over_limit_with_local_cache: int = 0
    within_limit: int = 0
    shadow_mode: int = 0


@dataclass
class Limit:
    requests_per_unit: int
    unit: int


@dataclass
class RateLimit:
    full_key: str
    stats: RateLimitStats
    limit: Limit
    unlimited: bool = False
    shadow_mode: bool = False


@dataclass
class Descriptor:
    entries: List[Tuple[str, str]]
    limit: Optional[Limit] = None


@dataclass
class RateLimitRequest:
    domain: str
    descriptors: List[Descriptor]
    hits_addend: int = 0


@dataclass
class DescriptorStatus:
    code: int
    current_limit: Optional[Limit]
    limit_remaining: int
    duration_until_reset: Optional[int]


def new_rate_limit(requests_per_unit: int, unit: int, stats_key: str, unlimited=False, shadow_mode=False):
    """config.NewRateLimit (src/config/config_impl.go:67-71)."""
    return RateLimit(stats_key, RateLimitStats(stats_key), Limit(requests_per_unit, unit), unlimited, shadow_mode)
