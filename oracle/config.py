"""CPU restatement of the config lookup and the service step around DoLimit
(TEST INFRASTRUCTURE ONLY: imported by ``tests/`` as the checker, never by
the product path).

Followed line by line from the Go source read as text:

* ``rateLimitConfigImpl.loadConfig``      src/config/config_impl.go:200-231
* ``rateLimitDescriptor.loadDescriptors`` config_impl.go:96-150
* ``validateYamlKeys``                    config_impl.go:155-197
* ``rateLimitConfigImpl.GetLimit``        config_impl.go:243-298
* ``descriptorKey``                       config_impl.go:300-312
* ``service.constructLimitsToCheck``      src/service/ratelimit.go:104-143
* ``service.shouldRateLimitWorker``       ratelimit.go:147-208 (no custom headers)

Stats counters are looked up by name in one store (gostats: ``NewStats(key)``
returns the same counters for the same key), so an override's per-value
stats key accumulates across calls (test/config/config_test.go:201-262).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import yaml

from .oracle import (DAY, HOUR, MINUTE, OK, OVER_LIMIT, SECOND, U32, Descriptor, DescriptorStatus, Limit,
                     OracleFixedRateLimitCache, RateLimit, RateLimitRequest, RateLimitStats)

# pb.RateLimitResponse_RateLimit_Unit_value (rls.proto): strings.ToUpper(unit) -> enum
UNIT_VALUE = {"UNKNOWN": 0, "SECOND": SECOND, "MINUTE": MINUTE, "HOUR": HOUR, "DAY": DAY}
# config_impl.go:57-65
VALID_KEYS = {"domain", "key", "value", "descriptors", "rate_limit", "unit", "requests_per_unit", "unlimited",
              "shadow_mode"}


class RateLimitConfigError(Exception):
    """newRateLimitConfigError (config_impl.go:73-76): "<file>: <text>"."""


class StatsStore:
    """The gostats store behind stats.Manager.NewStats (src/stats/manager_impl.go)."""

    def __init__(self):
        self.by_key: Dict[str, RateLimitStats] = {}

    def new_stats(self, key: str) -> RateLimitStats:
        if key not in self.by_key:
            self.by_key[key] = RateLimitStats(key)
        return self.by_key[key]


class _Node:
    """rateLimitDescriptor (config_impl.go:45-48)."""

    def __init__(self, limit: Optional[RateLimit]):
        self.descriptors: Dict[str, "_Node"] = {}
        self.limit = limit


def _validate_yaml_keys(name: str, m) -> None:
    """config_impl.go:155-197."""
    for k, v in m.items():
        if not isinstance(k, str):
            raise RateLimitConfigError("%s: config error, key is not of type string: %s" % (name, k))
        if k not in VALID_KEYS:
            raise RateLimitConfigError("%s: config error, unknown key '%s'" % (name, k))
        if isinstance(v, list):
            for e in v:
                if not isinstance(e, dict):
                    raise RateLimitConfigError(
                        "%s: config error, yaml file contains list of type other than map: %s" % (name, e))
                _validate_yaml_keys(name, e)
        elif isinstance(v, dict):
            _validate_yaml_keys(name, v)
        elif v is None or isinstance(v, (str, int, bool)):
            pass
        else:
            raise RateLimitConfigError("%s: error checking config" % name)


class RateLimitConfig:
    """rateLimitConfigImpl: NewRateLimitConfigImpl over (name, yaml text) files (config_impl.go:318-330)."""

    def __init__(self, files: Sequence[Tuple[str, str]], store: Optional[StatsStore] = None):
        self.store = store or StatsStore()
        self.domains: Dict[str, _Node] = {}
        for name, text in files:
            self._load(name, text)

    def _load(self, name: str, text: str) -> None:  # loadConfig :200-231
        try:
            any_ = yaml.safe_load(text)
        except yaml.YAMLError as e:
            raise RateLimitConfigError("%s: error loading config file: %s" % (name, e))
        if not isinstance(any_, dict):
            any_ = {}
        _validate_yaml_keys(name, any_)
        domain = any_.get("domain") or ""
        if domain == "":
            raise RateLimitConfigError("%s: config file cannot have empty domain" % name)
        if domain in self.domains:
            raise RateLimitConfigError("%s: duplicate domain '%s' in config file" % (name, domain))
        root = _Node(None)
        self._load_descriptors(name, root, domain + ".", any_.get("descriptors") or [])
        self.domains[domain] = root

    def _load_descriptors(self, name, node: _Node, parent_key: str, descriptors) -> None:  # :96-150
        for dc in descriptors:
            key = str(dc.get("key") or "")
            if key == "":
                raise RateLimitConfigError("%s: descriptor has empty key" % name)
            value = str(dc.get("value") or "")
            final_key = key + ("_" + value if value != "" else "")
            new_parent_key = parent_key + final_key
            if final_key in node.descriptors:
                raise RateLimitConfigError("%s: duplicate descriptor composite key '%s'" % (name, new_parent_key))
            rate_limit = None
            rl = dc.get("rate_limit")
            if rl is not None:
                unlimited = bool(rl.get("unlimited") or False)
                uname = str(rl.get("unit") or "").upper()
                value_u = UNIT_VALUE.get(uname)
                valid = value_u is not None and value_u != 0
                if unlimited:
                    if valid:
                        raise RateLimitConfigError("%s: should not specify rate limit unit when unlimited" % name)
                elif not valid:
                    raise RateLimitConfigError("%s: invalid rate limit unit '%s'" % (name, rl.get("unit") or ""))
                rate_limit = RateLimit(new_parent_key, self.store.new_stats(new_parent_key),
                                       Limit(int(rl.get("requests_per_unit") or 0) & U32, value_u or 0),
                                       unlimited, bool(dc.get("shadow_mode") or False))
            child = _Node(rate_limit)
            self._load_descriptors(name, child, new_parent_key + ".", dc.get("descriptors") or [])
            node.descriptors[final_key] = child

    def get_limit(self, domain: str, descriptor: Descriptor) -> Optional[RateLimit]:
        """GetLimit, config_impl.go:243-298."""
        value = self.domains.get(domain)
        if value is None:
            return None
        if descriptor.limit is not None:
            key = descriptor_key(domain, descriptor)
            return RateLimit(key, self.store.new_stats(key),
                             Limit(descriptor.limit.requests_per_unit, descriptor.limit.unit), False, False)
        rate_limit = None
        descriptors_map = value.descriptors
        for i, (k, v) in enumerate(descriptor.entries):
            nxt = descriptors_map.get(k + "_" + v)
            if nxt is None:
                nxt = descriptors_map.get(k)
            if nxt is not None and nxt.limit is not None and i == len(descriptor.entries) - 1:
                rate_limit = nxt.limit
            if nxt is not None and len(nxt.descriptors) > 0:
                descriptors_map = nxt.descriptors
            else:
                break
        return rate_limit


def descriptor_key(domain: str, descriptor: Descriptor) -> str:
    """descriptorKey, config_impl.go:300-312."""
    key = ""
    for k, v in descriptor.entries:
        if key != "":
            key += "."
        key += k
        if v != "":
            key += "_" + v
    return domain + "." + key


class OracleService:
    """The service step around DoLimit (ratelimit.go:104-208) over the oracle cache."""

    def __init__(self, config: RateLimitConfig, cache: OracleFixedRateLimitCache, global_shadow_mode=False):
        self.config = config
        self.cache = cache
        self.global_shadow_mode = global_shadow_mode

    def construct_limits_to_check(self, request: RateLimitRequest):  # :104-143
        limits: List[Optional[RateLimit]] = []
        unlimited: List[bool] = []
        for d in request.descriptors:
            rl = self.config.get_limit(request.domain, d)
            if rl is not None and rl.unlimited:
                unlimited.append(True)
                rl = None
            else:
                unlimited.append(False)
            limits.append(rl)
        return limits, unlimited

    def should_rate_limit(self, request: RateLimitRequest, now: int):
        """-> (overall code, statuses, matched limits); ratelimit.go:147-208."""
        if request.domain == "":
            raise ValueError("rate limit domain must not be empty")
        if len(request.descriptors) == 0:
            raise ValueError("rate limit descriptor list must not be empty")
        limits, unlimited = self.construct_limits_to_check(request)
        sts = self.cache.do_limit(request, limits, now)
        out = []
        final = OK
        for i, s in enumerate(sts):
            if unlimited[i]:
                out.append(DescriptorStatus(OK, None, U32, None))
            else:
                out.append(s)
                if s.code == OVER_LIMIT:
                    final = OVER_LIMIT
        if final == OVER_LIMIT and self.global_shadow_mode:
            final = OK
        return final, out, limits
