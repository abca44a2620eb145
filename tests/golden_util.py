"""Helpers that turn tests/golden/*.json fixtures into request/limit objects.

Shared by the oracle tests (CPU) and the GPU parity tests; the objects are the
oracle's data model, which the product's Python mirror (ratelimit_amd.limiter)
shares field-for-field.
"""
import glob
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


def names(kind=None):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.json"))):
        n = os.path.splitext(os.path.basename(p))[0]
        if kind is None or load(n)["kind"] == kind:
            out.append(n)
    return out


class StatsRegistry:
    """gostats store: NewCounter(name) returns the existing counter (same key -> same stats)."""

    def __init__(self, mod):
        self.mod = mod
        self.by_key = {}

    def get(self, key):
        if key not in self.by_key:
            self.by_key[key] = self.mod.RateLimitStats(key)
        return self.by_key[key]


def make_limit(mod, reg, d):
    """Fixture limit dict -> mod.RateLimit sharing stats by key (config.NewRateLimit)."""
    if d is None:
        return None
    return mod.RateLimit(d["stats_key"], reg.get(d["stats_key"]),
                         mod.Limit(d["rpu"], d["unit"]), False, bool(d.get("shadow", False)))


def make_request(mod, r):
    return mod.RateLimitRequest(r["domain"], [mod.Descriptor([tuple(e) for e in d]) for d in r["descriptors"]],
                                r["hits_addend"])


def status_tuple(s):
    """(code, (rpu, unit) or None, remaining, reset or None) from any status object."""
    cl = None if s.current_limit is None else (s.current_limit.requests_per_unit, s.current_limit.unit)
    return (s.code, cl, s.limit_remaining, s.duration_until_reset)


def expect_tuple(e):
    return (e["code"], None if e["limit"] is None else tuple(e["limit"]), e["remaining"], e["reset"])


def check_stats(reg, expect_stats):
    for key, fields in expect_stats.items():
        st = reg.get(key)
        for f, v in fields.items():
            assert getattr(st, f) == v, "%s.%s = %d, expected %d" % (key, f, getattr(st, f), v)


GAUGES = ("hit_count", "miss_count", "lookup_count", "entry_count")


def check_gauges(got, expect):
    """localCacheStats gauges (local_cache_stats.go:36-43) against a step's expect_gauges."""
    for g in GAUGES:
        if g in expect:
            assert got[g] == expect[g], "%s = %d, expected %d (%s)" % (g, got[g], expect[g], expect["source_line"])


def oracle_gauges(cache, now):
    lc = cache.local_cache
    if lc is None:
        return dict.fromkeys(GAUGES, 0)
    return {"hit_count": lc.hit_count, "miss_count": lc.miss_count, "lookup_count": lc.hit_count + lc.miss_count,
            "entry_count": lc.entry_count(now)}
