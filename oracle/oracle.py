"""CPU restatement of the reference's fixed-window hot path (TEST INFRASTRUCTURE ONLY).

This module is the parity oracle. It is imported only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, and only as
the checker: the product path (``ratelimit_amd``) never imports it.

It is a sequential, pure-Python restatement of the Go code, read as text
(the Go toolchain is absent here and on the GPU box, see DESIGN.md "Oracle"):

* ``CacheKeyGenerator.GenerateCacheKey``   src/limiter/cache_key.go:48-80
* ``BaseRateLimiter.GenerateCacheKeys``    src/limiter/base_limiter.go:45-60
* ``BaseRateLimiter.IsOverLimitWithLocalCache`` base_limiter.go:63-72
* ``BaseRateLimiter.GetResponseDescriptorStatus`` base_limiter.go:76-135
* ``checkOverLimitThreshold`` / ``checkNearLimitThreshold`` base_limiter.go:150-179
* ``generateResponseDescriptorStatus``      base_limiter.go:181-197
* ``fixedRateLimitCacheImpl.DoLimit``       src/redis/fixed_cache_impl.go:33-113
* ``utils.UnitToDivider`` / ``CalculateReset`` / ``Max``  src/utils/utilities.go:17-43

External stores are modelled from their published semantics:

* redis-server ``INCRBY``/``EXPIRE`` (unpinned version; pinned at the boundary by
  test/redis/driver_impl_test.go:122-134 "INCRBY on a missing key returns hits,
  then +hits").  A key whose TTL has passed reads as missing.  Redis expires a
  key when ``now_ms > expire_ms``; with integer simulated seconds (sub-second
  part 0) a key written at ``t`` with ``EXPIRE ttl`` is live while
  ``now <= t + ttl``.
* freecache v1.1.0 local cache (go.mod:9): ``Set(key, ttl)`` stores
  ``expireAt = now + ttl``; ``Get`` misses once ``expireAt <= now``.  Capacity
  eviction is unpinned (parity assumes a cache large enough to never evict).
* radix v3.5.1 decodes the INCRBY reply into ``*uint32``: counts are kept
  modulo 2**32 (behaviour for counts >= 2**32 is "parity unpinned").

Simulated clock: every clock read inside one request returns that request's
``now`` (as every reference unit test does with ``UnixNow().Return(c)``).
Expiration jitter is modelled with a Go ``rand.Int63n`` restatement over an
injectable ``Int63`` source; the GPU backend fixes the draw at 0.
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

# go-control-plane v0.9.7 rls.proto enums (third-party, not in the container).
UNKNOWN, OK, OVER_LIMIT = 0, 1, 2  # RateLimitResponse_Code
UNIT_UNKNOWN, SECOND, MINUTE, HOUR, DAY = 0, 1, 2, 3, 4  # RateLimit_Unit
UNIT_NAMES = {"second": SECOND, "minute": MINUTE, "hour": HOUR, "day": DAY}

U32 = 0xFFFFFFFF
STAT_FIELDS = ("total_hits", "over_limit", "near_limit",
               "over_limit_with_local_cache", "within_limit", "shadow_mode")


def unit_to_divider(unit: int) -> int:
    """utils.UnitToDivider, src/utils/utilities.go:17-30 (panics on UNKNOWN)."""
    if unit == SECOND:
        return 1
    if unit == MINUTE:
        return 60
    if unit == HOUR:
        return 60 * 60
    if unit == DAY:
        return 60 * 60 * 24
    raise RuntimeError("should not get here")


def calculate_reset(unit: int, now: int) -> int:
    """utils.CalculateReset, src/utils/utilities.go:32-36 (Go % truncates)."""
    sec = unit_to_divider(unit)
    return sec - int(math.fmod(now, sec))


def go_max_u32(a: int, b: int) -> int:
    """utils.Max, src/utils/utilities.go:38-43."""
    return a if a > b else b


def f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def go_float64_to_uint32(x: float) -> int:
    """Go ``uint32(float64)`` on amd64: CVTTSD2SQ (truncate to int64) then keep
    the low 32 bits.  Out-of-int64-range inputs give 0x8000000000000000."""
    if not (-9.2233720368547758e18 <= x < 9.2233720368547758e18) or x != x:
        v = -(1 << 63)
    else:
        v = int(x)  # truncation toward zero
    return v & U32


def near_limit_threshold(limit: int, ratio: float) -> int:
    """``uint32(math.Floor(float64(float32(limit) * nearLimitRatio)))``,
    base_limiter.go:94: one IEEE fp32 multiply, then floor in float64."""
    prod = f32(f32(float(limit)) * f32(ratio))
    return go_float64_to_uint32(math.floor(prod))


class GoInt63n:
    """Restatement of Go ``(*rand.Rand).Int63n`` (math/rand) over an Int63 source."""

    def __init__(self, int63: Callable[[], int]):
        self.int63 = int63

    def int63n(self, n: int) -> int:
        if n <= 0:
            raise ValueError("invalid argument to Int63n")
        if n & (n - 1) == 0:
            return self.int63() & (n - 1)
        mx = (1 << 63) - 1 - ((1 << 63) % n)
        v = self.int63()
        while v > mx:
            v = self.int63()
        return v % n


# --------------------------------------------------------------------------
# Data model mirroring the Go types the hot path touches.
# --------------------------------------------------------------------------
@dataclass
class RateLimitStats:
    """stats.RateLimitStats, src/stats/manager.go:47-55 (6 counters per rule)."""
    key: str
    total_hits: int = 0
    over_limit: int = 0
    near_limit: int = 0
    over_limit_with_local_cache: int = 0
    within_limit: int = 0
    shadow_mode: int = 0

    def as_tuple(self) -> Tuple[int, ...]:
        return tuple(getattr(self, f) for f in STAT_FIELDS)


@dataclass
class Limit:
    """pb.RateLimitResponse_RateLimit {RequestsPerUnit, Unit}."""
    requests_per_unit: int
    unit: int


@dataclass
class RateLimit:
    """config.RateLimit, src/config/config.go:19-25; NewRateLimit config_impl.go:67-71."""
    full_key: str
    stats: RateLimitStats
    limit: Limit
    unlimited: bool = False
    shadow_mode: bool = False


def new_rate_limit(requests_per_unit: int, unit: int, stats_key: str,
                   unlimited: bool = False, shadow_mode: bool = False) -> RateLimit:
    st = RateLimitStats(stats_key)
    return RateLimit(stats_key, st, Limit(requests_per_unit, unit), unlimited, shadow_mode)


@dataclass
class Descriptor:
    """pb_struct.RateLimitDescriptor: entries plus optional per-request Limit override."""
    entries: List[Tuple[str, str]]
    limit: Optional[Limit] = None


@dataclass
class RateLimitRequest:
    """pb.RateLimitRequest {Domain, Descriptors, HitsAddend}."""
    domain: str
    descriptors: List[Descriptor]
    hits_addend: int = 0


def new_rate_limit_request(domain: str, descriptors: Sequence[Sequence[Tuple[str, str]]],
                           hits_addend: int) -> RateLimitRequest:
    """test/common/common.go:51-65 NewRateLimitRequest."""
    return RateLimitRequest(domain, [Descriptor([(k, v) for k, v in d]) for d in descriptors],
                            hits_addend)


@dataclass
class DescriptorStatus:
    """pb.RateLimitResponse_DescriptorStatus as produced by generateResponseDescriptorStatus."""
    code: int
    current_limit: Optional[Limit]
    limit_remaining: int
    duration_until_reset: Optional[int]  # seconds; None when CurrentLimit is nil

    def as_tuple(self):
        cl = None if self.current_limit is None else (self.current_limit.requests_per_unit,
                                                       self.current_limit.unit)
        return (self.code, cl, self.limit_remaining, self.duration_until_reset)


@dataclass
class CacheKey:
    key: str
    per_second: bool


# --------------------------------------------------------------------------
# Stores
# --------------------------------------------------------------------------
class FakeRedis:
    """INCRBY/EXPIRE with lazy TTL expiry in simulated seconds."""

    def __init__(self):
        self.data: Dict[str, List[int]] = {}  # key -> [count_u32, expire_at or -1]
        self.log: List[Tuple] = []

    def _live(self, key: str, now: int):
        e = self.data.get(key)
        if e is None:
            return None
        if e[1] >= 0 and now > e[1]:
            del self.data[key]
            return None
        return e

    def incrby(self, key: str, h: int, now: int) -> int:
        self.log.append(("INCRBY", key, h))
        e = self._live(key, now)
        if e is None:
            e = [0, -1]
            self.data[key] = e
        e[0] = (e[0] + h) & U32
        return e[0]

    def expire(self, key: str, ttl: int, now: int) -> None:
        self.log.append(("EXPIRE", key, ttl))
        e = self._live(key, now)
        if e is not None:
            e[1] = now + ttl

    def seed(self, key: str, count: int, expire_at: int) -> None:
        self.data[key] = [count & U32, expire_at]

    def purge(self, now: int) -> None:
        dead = [k for k, e in self.data.items() if e[1] >= 0 and now > e[1]]
        for k in dead:
            del self.data[k]


class FakeFreecache:
    """freecache Get/Set with expireAt = now + ttl; miss once expireAt <= now."""

    def __init__(self):
        self.data: Dict[str, int] = {}
        self.hit_count = 0
        self.miss_count = 0

    def get(self, key: str, now: int) -> bool:
        e = self.data.get(key)
        if e is not None and now < e:
            self.hit_count += 1
            return True
        self.miss_count += 1
        return False

    def set(self, key: str, ttl: int, now: int) -> None:
        self.data[key] = now + ttl

    def entry_count(self, now: int) -> int:
        """Entries whose TTL has not passed at ``now`` (the live part of EntryCount)."""
        return sum(1 for e in self.data.values() if now < e)

    def purge(self, now: int) -> None:
        for k in [k for k, e in self.data.items() if e <= now]:
            del self.data[k]


# --------------------------------------------------------------------------
# The limiter
# --------------------------------------------------------------------------
class OracleFixedRateLimitCache:
    """redis.fixedRateLimitCacheImpl + limiter.BaseRateLimiter, sequential.

    ``do_limit(request, limits, now)`` returns the per-descriptor statuses and
    adds the stats deltas into ``limits[i].stats`` exactly like the Go code.
    """

    def __init__(self, near_limit_ratio: float = 0.8, local_cache: bool = False,
                 cache_key_prefix: str = "", per_second: bool = False,
                 expiration_jitter_max_seconds: int = 0,
                 jitter_int63: Optional[Callable[[], int]] = None):
        self.near_limit_ratio = f32(near_limit_ratio)
        self.prefix = cache_key_prefix
        self.client = FakeRedis()
        self.per_second_client = FakeRedis() if per_second else None
        self.local_cache = FakeFreecache() if local_cache else None
        self.jitter_max = expiration_jitter_max_seconds
        self.jitter = GoInt63n(jitter_int63 or (lambda: 0))

    # cache_key.go:48-80
    def generate_cache_key(self, domain: str, descriptor: Descriptor,
                           limit: Optional[RateLimit], now: int) -> CacheKey:
        if limit is None:
            return CacheKey("", False)
        parts = [self.prefix, domain, "_"]
        for k, v in descriptor.entries:
            parts += [k, "_", v, "_"]
        divider = unit_to_divider(limit.limit.unit)
        parts.append(str(go_div(now, divider) * divider))  # strconv.FormatInt((now/d)*d, 10)
        return CacheKey("".join(parts), limit.limit.unit == SECOND)

    # base_limiter.go:45-60
    def generate_cache_keys(self, request: RateLimitRequest, limits, hits: int, now: int):
        assert len(request.descriptors) == len(limits)
        keys = []
        for d, lim in zip(request.descriptors, limits):
            keys.append(self.generate_cache_key(request.domain, d, lim, now))
            if lim is not None:
                lim.stats.total_hits += hits
        return keys

    # base_limiter.go:63-72
    def is_over_limit_with_local_cache(self, key: str, now: int) -> bool:
        if self.local_cache is not None:
            return self.local_cache.get(key, now)
        return False

    # base_limiter.go:76-135
    def get_response_descriptor_status(self, key: str, limit: Optional[RateLimit], before: int,
                                       after: int, is_over_limit_with_local_cache: bool,
                                       hits: int, now: int) -> DescriptorStatus:
        if key == "":
            return DescriptorStatus(OK, None, 0, None)
        st = limit.stats
        over = False
        if is_over_limit_with_local_cache:
            over = True
            st.over_limit += hits
            st.over_limit_with_local_cache += hits
            status = self._gen(OVER_LIMIT, limit.limit, 0, now)
        else:
            thr = limit.limit.requests_per_unit
            near = near_limit_threshold(thr, self.near_limit_ratio)
            if after > thr:
                over = True
                status = self._gen(OVER_LIMIT, limit.limit, 0, now)
                # checkOverLimitThreshold, base_limiter.go:150-165
                if before >= thr:
                    st.over_limit += hits
                else:
                    st.over_limit += (after - thr) & U32
                    st.near_limit += (thr - go_max_u32(near, before)) & U32
                if self.local_cache is not None:
                    self.local_cache.set(key, unit_to_divider(limit.limit.unit), now)
            else:
                status = self._gen(OK, limit.limit, (thr - after) & U32, now)
                # checkNearLimitThreshold, base_limiter.go:167-179
                if after > near:
                    if before >= near:
                        st.near_limit += hits
                    else:
                        st.near_limit += (after - near) & U32
                st.within_limit += hits
        if over and limit.shadow_mode:
            status.code = OK
            st.shadow_mode += hits
        return status

    # base_limiter.go:181-197
    def _gen(self, code: int, limit: Optional[Limit], remaining: int, now: int) -> DescriptorStatus:
        if limit is not None:
            return DescriptorStatus(code, limit, remaining, calculate_reset(limit.unit, now))
        return DescriptorStatus(code, None, remaining, None)

    # fixed_cache_impl.go:33-113
    def do_limit(self, request: RateLimitRequest, limits: List[Optional[RateLimit]],
                 now: int) -> List[DescriptorStatus]:
        hits = go_max_u32(1, request.hits_addend)
        keys = self.generate_cache_keys(request, limits, hits, now)
        n = len(request.descriptors)
        lc_flags = [False] * n
        results = [0] * n
        main_pipe: List[Tuple[int, str, int]] = []
        ps_pipe: List[Tuple[int, str, int]] = []
        for i, ck in enumerate(keys):
            if ck.key == "":
                continue
            if self.is_over_limit_with_local_cache(ck.key, now):
                if not limits[i].shadow_mode:
                    lc_flags[i] = True
                continue
            ttl = unit_to_divider(limits[i].limit.unit)
            if self.jitter_max > 0:
                ttl += self.jitter.int63n(self.jitter_max)
            if self.per_second_client is not None and ck.per_second:
                ps_pipe.append((i, ck.key, ttl))
            else:
                main_pipe.append((i, ck.key, ttl))
        # PipeDo: the main pipeline, then the per-second one; commands run in order.
        for client, pipe in ((self.client, main_pipe), (self.per_second_client, ps_pipe)):
            for i, key, ttl in pipe:
                results[i] = client.incrby(key, hits, now)
                client.expire(key, ttl, now)
        out = []
        for i, ck in enumerate(keys):
            after = results[i]
            before = (after - hits) & U32
            out.append(self.get_response_descriptor_status(ck.key, limits[i], before, after,
                                                           lc_flags[i], hits, now))
        return out

    def seed(self, key: str, count: int, expire_at: int, per_second: bool = False) -> None:
        """Test hook standing in for the mocked INCRBY reply of the reference unit tests."""
        (self.per_second_client if per_second else self.client).seed(key, count, expire_at)


def go_div(a: int, b: int) -> int:
    """Go integer division truncates toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q
