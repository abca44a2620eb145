"""Write tests/golden/ref_*.json: known answers transcribed from the reference's tests.

The reference (Go) cannot be built here (no Go toolchain, no module cache, no
network), so its own unit/integration tests are the pin.  Every
expected value below is copied by hand from the cited test line; nothing here
is computed by the oracle.  Re-run with ``python tests/golden/make_golden.py``.

Fixture schema (one JSON file per reference test):
  config:  near_limit_ratio, local_cache, prefix, per_second, jitter_max, jitter_int63
  steps[]: now, seed[] (mocked INCRBY reply N is restated as a stored count N-hits),
           request{domain, descriptors[[[k,v],..],..], hits_addend},
           limits[] (null = nil limit, i.e. no rule), expect_commands (the mock's
           PipeAppend expectations, per client), expect_statuses[], expect_stats{}
           (cumulative counter values asserted by the test; absent fields unasserted).
"decide" fixtures call GetResponseDescriptorStatus directly with (before, after).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OK, OVER = 1, 2
SEC, MIN, HOUR, DAY = 1, 2, 3, 4


def lim(rpu, unit, key, shadow=False):
    return {"rpu": rpu, "unit": unit, "stats_key": key, "shadow": shadow}


def st(code, limit=None, rem=0, reset=None):
    return {"code": code, "limit": limit, "remaining": rem, "reset": reset}


def stats(**kw):
    return kw


def req(domain, descs, hits):
    return {"domain": domain, "descriptors": descs, "hits_addend": hits}


def cfg(ratio=0.8, local_cache=False, prefix="", per_second=False, jitter_max=0, jitter=None):
    return {"near_limit_ratio": ratio, "local_cache": local_cache, "prefix": prefix,
            "per_second": per_second, "jitter_max": jitter_max, "jitter_int63": jitter or []}


def reset(unit, now):
    # CalculateReset (utilities.go:32-36) is evaluated by the reference test itself
    # (``utils.CalculateReset(&limits[0].Limit.Unit, timeSource)``); restated here.
    d = {SEC: 1, MIN: 60, HOUR: 3600, DAY: 86400}[unit]
    return d - now % d


fixtures = {}

# ---------------------------------------------------------------- testRedis
# test/redis/fixed_cache_impl_test.go:37-141, run WithoutPerSecondRedis / WithPerSecondRedis (:28-31)
for per_second in (False, True):
    steps = []
    # :55-76
    steps.append({
        "now": 1234,
        "seed": [{"key": "domain_key_value_1234", "count": 4, "per_second": per_second}],
        "request": req("domain", [[["key", "value"]]], 1),
        "limits": [lim(10, SEC, "key_value")],
        "expect_commands": {("per_second" if per_second else "main"): [
            ["INCRBY", "domain_key_value_1234", 1], ["EXPIRE", "domain_key_value_1234", 1]]},
        "expect_statuses": [st(OK, [10, SEC], 5, reset(SEC, 1234))],
        "expect_stats": {"key_value": stats(total_hits=1, over_limit=0, near_limit=0, within_limit=1)},
    })
    # :78-104
    steps.append({
        "now": 1234,
        "seed": [{"key": "domain_key2_value2_subkey2_subvalue2_1200", "count": 10}],
        "request": req("domain", [[["key2", "value2"]], [["key2", "value2"], ["subkey2", "subvalue2"]]], 1),
        "limits": [None, lim(10, MIN, "key2_value2_subkey2_subvalue2")],
        "expect_commands": {"main": [
            ["INCRBY", "domain_key2_value2_subkey2_subvalue2_1200", 1],
            ["EXPIRE", "domain_key2_value2_subkey2_subvalue2_1200", 60]]},
        "expect_statuses": [st(OK, None, 0, None), st(OVER, [10, MIN], 0, reset(MIN, 1234))],
        "expect_stats": {"key2_value2_subkey2_subvalue2":
                         stats(total_hits=1, over_limit=1, near_limit=0, within_limit=0)},
    })
    # :106-139
    steps.append({
        "now": 1000000,
        "seed": [{"key": "domain_key3_value3_997200", "count": 10},
                 {"key": "domain_key3_value3_subkey3_subvalue3_950400", "count": 12}],
        "request": req("domain", [[["key3", "value3"]], [["key3", "value3"], ["subkey3", "subvalue3"]]], 1),
        "limits": [lim(10, HOUR, "key3_value3"), lim(10, DAY, "key3_value3_subkey3_subvalue3")],
        "expect_commands": {"main": [
            ["INCRBY", "domain_key3_value3_997200", 1], ["EXPIRE", "domain_key3_value3_997200", 3600],
            ["INCRBY", "domain_key3_value3_subkey3_subvalue3_950400", 1],
            ["EXPIRE", "domain_key3_value3_subkey3_subvalue3_950400", 86400]]},
        "expect_statuses": [st(OVER, [10, HOUR], 0, reset(HOUR, 1000000)),
                            st(OVER, [10, DAY], 0, reset(DAY, 1000000))],
        "expect_stats": {"key3_value3": stats(total_hits=1, over_limit=1, near_limit=0, within_limit=0)},
    })
    name = "ref_redis_%s" % ("per_second" if per_second else "single")
    fixtures[name] = {"source": "test/redis/fixed_cache_impl_test.go:37-141", "kind": "do_limit",
                      "config": cfg(per_second=per_second), "steps": steps}


# ------------------------------------------------- over limit with local cache
def key4_steps(shadow, local_cache):
    """The shared key4 sequence: replies 11, 13, 16 then a local-cache hit."""
    s = []
    lm = lim(15, HOUR, "key4_value4", shadow)
    for n, (reply, code, rem, st_exp) in enumerate([
        (11, OK, 4, stats(total_hits=1, over_limit=0, near_limit=0, within_limit=1)),
        (13, OK, 2, stats(total_hits=2, over_limit=0, near_limit=1, within_limit=2)),
        (16, OK if shadow else OVER, 0, stats(total_hits=3, over_limit=1, near_limit=1, within_limit=2)),
    ]):
        if local_cache:
            st_exp["over_limit_with_local_cache"] = 0
        s.append({
            "now": 1000000,
            "seed": [{"key": "domain_key4_value4_997200", "count": reply - 1}],
            "request": req("domain", [[["key4", "value4"]]], 1),
            "limits": [lm],
            "expect_commands": {"main": [["INCRBY", "domain_key4_value4_997200", 1],
                                         ["EXPIRE", "domain_key4_value4_997200", 3600]]},
            "expect_statuses": [st(code, [15, HOUR], rem, reset(HOUR, 1000000))],
            "expect_stats": {"key4_value4": st_exp},
        })
    return s


lc = key4_steps(False, True)
# :262-276: local cache hit, no INCRBY/EXPIRE
lc.append({
    "now": 1000000, "seed": [],
    "request": req("domain", [[["key4", "value4"]]], 1),
    "limits": [lim(15, HOUR, "key4_value4")],
    "expect_commands": {"main": []},
    "expect_statuses": [st(OVER, [15, HOUR], 0, reset(HOUR, 1000000))],
    "expect_stats": {"key4_value4": stats(total_hits=4, over_limit=2, over_limit_with_local_cache=1,
                                          near_limit=1, within_limit=2)},
})
# localCacheStats gauges after each step (testLocalCacheStats(hit, miss, lookup,
# expired, entry), fixed_cache_impl_test.go:218,239,260,279). freecache v1.1.0
# (go.mod:9, not vendored) counts LookupCount = HitCount + MissCount, and every
# DoLimit of a non-empty key makes one Get (IsOverLimitWithLocalCache,
# base_limiter.go:63-72). The vector at :260, (0, 2, 3, 0, 1), is not reachable:
# its lookup 3 needs hit + miss = 3, and :279's (1, 3, 4) needs miss 3 already.
# testLocalCacheStats returns a func(*testing.T) that the test never runs
# (:143-145), so the reference never checks it; the executed semantics give
# (0, 3, 3, 0, 1), kept here with the transcribed vector beside it.
# expiredCount is freecache's own bookkeeping (entries found stale on access),
# 0 in every vector; the backend reports entry/lookup/hit/miss.
KEY4_GAUGES = [((0, 1, 1, 0, 0), None), ((0, 2, 2, 0, 0), None), ((0, 3, 3, 0, 1), (0, 2, 3, 0, 1)),
               ((1, 3, 4, 0, 1), None)]


def with_gauges(steps, lines):
    for step, ((h, m, lk, ex, en), ref), line in zip(steps, KEY4_GAUGES, lines):
        g = {"hit_count": h, "miss_count": m, "lookup_count": lk, "entry_count": en, "source_line": line}
        if ref is not None:
            g["reference_vector"] = list(ref)
            g["note"] = "unreachable as transcribed (lookup != hit + miss); never executed by the reference"
        step["expect_gauges"] = g
    return steps


fixtures["ref_over_limit_with_local_cache"] = {
    "source": "test/redis/fixed_cache_impl_test.go:179-280", "kind": "do_limit",
    "config": cfg(local_cache=True),
    "steps": with_gauges(lc, ["fixed_cache_impl_test.go:%d" % x for x in (218, 239, 260, 279)])}

lcs = key4_steps(True, True)
# :569-586: shadow rule in the local cache: INCRBY skipped, result 0 -> OK with the full limit
lcs.append({
    "now": 1000000, "seed": [],
    "request": req("domain", [[["key4", "value4"]]], 1),
    "limits": [lim(15, HOUR, "key4_value4", True)],
    "expect_commands": {"main": []},
    "expect_statuses": [st(OK, [15, HOUR], 15, reset(HOUR, 1000000))],
    "expect_stats": {"key4_value4": stats(total_hits=4, over_limit=1, over_limit_with_local_cache=0,
                                          near_limit=1, within_limit=3)},
})
fixtures["ref_over_limit_with_local_cache_shadow_rule"] = {
    "source": "test/redis/fixed_cache_impl_test.go:485-590", "kind": "do_limit",
    "config": cfg(local_cache=True),
    "steps": with_gauges(lcs, ["fixed_cache_impl_test.go:%d" % x for x in (524, 545, 567, 589)])}

# ---------------------------------------------------------------- near limit
nl = key4_steps(False, False)
for key, hits, limit, reply, code, rem, exp in [
    # (:351-367) all under limit, under near
    ("5", 3, 20, 5, OK, 15, stats(total_hits=3, over_limit=0, near_limit=0, within_limit=3)),
    # (:369-384) all under limit, some over near
    ("6", 2, 8, 7, OK, 1, stats(total_hits=2, over_limit=0, near_limit=1, within_limit=2)),
    # (:386-401) all under limit, all over near
    ("7", 3, 20, 19, OK, 1, stats(total_hits=3, over_limit=0, near_limit=3, within_limit=3)),
    # (:403-418) some over limit, all over near
    ("8", 3, 20, 22, OVER, 0, stats(total_hits=3, over_limit=2, near_limit=1, within_limit=0)),
    # (:420-435) some in all three places
    ("9", 7, 20, 22, OVER, 0, stats(total_hits=7, over_limit=2, near_limit=4, within_limit=0)),
    # (:437-452) all over limit
    ("10", 3, 10, 30, OVER, 0, stats(total_hits=3, over_limit=3, near_limit=0, within_limit=0)),
]:
    k = "domain_key%s_value%s_1234" % (key, key)
    nl.append({
        "now": 1234,
        "seed": [{"key": k, "count": reply - hits}],
        "request": req("domain", [[["key" + key, "value" + key]]], hits),
        "limits": [lim(limit, SEC, "key%s_value%s" % (key, key))],
        "expect_commands": {"main": [["INCRBY", k, hits], ["EXPIRE", k, 1]]},
        "expect_statuses": [st(code, [limit, SEC], rem, reset(SEC, 1234))],
        "expect_stats": {"key%s_value%s" % (key, key): exp},
    })
fixtures["ref_near_limit"] = {"source": "test/redis/fixed_cache_impl_test.go:282-453", "kind": "do_limit",
                              "config": cfg(), "steps": nl}

# ---------------------------------------------------------------- jitter
fixtures["ref_redis_with_jitter"] = {
    "source": "test/redis/fixed_cache_impl_test.go:455-483", "kind": "do_limit",
    "config": cfg(jitter_max=3600, jitter=[100]),
    "steps": [{
        "now": 1234,
        "seed": [{"key": "domain_key_value_1234", "count": 4}],
        "request": req("domain", [[["key", "value"]]], 1),
        "limits": [lim(10, SEC, "key_value")],
        "expect_commands": {"main": [["INCRBY", "domain_key_value_1234", 1],
                                     ["EXPIRE", "domain_key_value_1234", 101]]},
        "expect_statuses": [st(OK, [10, SEC], 5, reset(SEC, 1234))],
        "expect_stats": {"key_value": stats(total_hits=1, over_limit=0, near_limit=0, within_limit=1)},
    }]}

# ---------------------------------------------------------------- key generation
# test/limiter/base_limiter_test.go:21-57
fixtures["ref_generate_cache_keys"] = {
    "source": "test/limiter/base_limiter_test.go:21-57", "kind": "cache_keys",
    "cases": [
        {"prefix": "", "now": 1234, "request": req("domain", [[["key", "value"]]], 1),
         "limits": [lim(10, SEC, "key_value")], "expect_keys": ["domain_key_value_1234"],
         "expect_stats": {"key_value": stats(total_hits=1)}},
        {"prefix": "prefix:", "now": 1234, "request": req("domain", [[["key", "value"]]], 1),
         "limits": [lim(10, SEC, "key_value")], "expect_keys": ["prefix:domain_key_value_1234"],
         "expect_stats": {"key_value": stats(total_hits=1)}},
        # fixed_cache_impl_test.go:80,108,111 (minute / hour / day windows)
        {"prefix": "", "now": 1234,
         "request": req("domain", [[["key2", "value2"]], [["key2", "value2"], ["subkey2", "subvalue2"]]], 1),
         "limits": [None, lim(10, MIN, "k2")], "expect_keys": ["", "domain_key2_value2_subkey2_subvalue2_1200"]},
        {"prefix": "", "now": 1000000,
         "request": req("domain", [[["key3", "value3"]], [["key3", "value3"], ["subkey3", "subvalue3"]]], 1),
         "limits": [lim(10, HOUR, "k3"), lim(10, DAY, "k3s")],
         "expect_keys": ["domain_key3_value3_997200", "domain_key3_value3_subkey3_subvalue3_950400"]},
    ]}

# ---------------------------------------------------------------- decision logic
# test/limiter/base_limiter_test.go:85-231 (GetResponseDescriptorStatus called directly)
fixtures["ref_base_limiter_decide"] = {
    "source": "test/limiter/base_limiter_test.go:85-231", "kind": "decide",
    "cases": [
        # :85-94 empty key
        {"key": "", "limit": None, "before": 0, "after": 0, "lc": False, "hits": 1, "now": 1234,
         "ratio": 0.8, "local_cache": False,
         "expect": {"code": OK, "remaining": 0}, "expect_stats": {}},
        # :96-116 over limit with local cache
        {"key": "key", "limit": lim(5, SEC, "key_value"), "before": 2, "after": 6, "lc": True, "hits": 2,
         "now": 1234, "ratio": 0.8, "local_cache": False,
         "expect": {"code": OVER, "remaining": 0, "limit": [5, SEC]},
         "expect_stats": {"key_value": stats(over_limit=2, over_limit_with_local_cache=2, shadow_mode=0)}},
        # :118-140 same, shadow mode
        {"key": "key", "limit": lim(5, SEC, "key_value", True), "before": 2, "after": 6, "lc": True,
         "hits": 2, "now": 1234, "ratio": 0.8, "local_cache": False,
         "expect": {"code": OK, "remaining": 0, "limit": [5, SEC]},
         "expect_stats": {"key_value": stats(over_limit=2, shadow_mode=2, over_limit_with_local_cache=2)}},
        # :142-165 over limit populates the local cache
        {"key": "key", "limit": lim(5, SEC, "key_value"), "before": 2, "after": 7, "lc": False, "hits": 1,
         "now": 1234, "ratio": 0.8, "local_cache": True,
         "expect": {"code": OVER, "remaining": 0, "limit": [5, SEC], "local_cache_set": True},
         "expect_stats": {"key_value": stats(over_limit=2, near_limit=1, shadow_mode=0)}},
        # :167-189 same, shadow mode (local cache still populated)
        {"key": "key", "limit": lim(5, SEC, "key_value", True), "before": 2, "after": 7, "lc": False,
         "hits": 1, "now": 1234, "ratio": 0.8, "local_cache": True,
         "expect": {"code": OK, "remaining": 0, "limit": [5, SEC], "local_cache_set": True},
         "expect_stats": {"key_value": stats(over_limit=2, near_limit=1)}},
        # :191-210 below limit
        {"key": "key", "limit": lim(10, SEC, "key_value"), "before": 2, "after": 6, "lc": False, "hits": 1,
         "now": 1234, "ratio": 0.8, "local_cache": False,
         "expect": {"code": OK, "remaining": 4, "limit": [10, SEC]},
         "expect_stats": {"key_value": stats(near_limit=0, within_limit=1, shadow_mode=0)}},
        # :212-231 below limit, shadow mode
        {"key": "key", "limit": lim(10, SEC, "key_value", True), "before": 2, "after": 6, "lc": False,
         "hits": 1, "now": 1234, "ratio": 0.8, "local_cache": False,
         "expect": {"code": OK, "remaining": 4, "limit": [10, SEC]},
         "expect_stats": {"key_value": stats(near_limit=0, within_limit=1, shadow_mode=0)}},
    ]}

# ---------------------------------------------------------------- INCRBY counting
# test/redis/driver_impl_test.go:122-134 and :170-183 (miniredis): INCRBY a 1 -> 1, then -> 2
fixtures["ref_driver_incrby"] = {
    "source": "test/redis/driver_impl_test.go:122-134,170-183", "kind": "incrby",
    "ops": [["a", 1, 1], ["a", 1, 2]]}


# ---------------------------------------------------------------- integration (real redis)
def integration_steps(local_cache):
    """test/integration/integration_test.go:371-597 testBasicBaseConfig, with the
    config of test/integration/runtime/current/ratelimit/config/{basic,another}.yaml
    resolved per descriptor (GetLimit is out of scope; stats keys are the rule FullKeys).
    The random descriptor values (r.Int(), :436,:499) are fixed to "rand1"/"rand2".
    All calls share one simulated second (the test runs within one minute window)."""
    now = 1_700_000_100
    s = []
    # :383-393 unknown domain "foo" -> nil limit
    s.append({"now": now, "seed": [], "request": req("foo", [[["hello", "world"]]], 1), "limits": [None],
              "expect_statuses": [st(OK, None, 0, None)], "expect_stats": {},
              "expect_gauges": {"hit_count": 0, "miss_count": 0, "source_line": "integration_test.go:397-401"}})
    # :405-420 basic/key1 (second, 50)
    s.append({"now": now, "seed": [], "request": req("basic", [[["key1", "foo"]]], 1),
              "limits": [lim(50, SEC, "basic.key1")],
              "expect_statuses": [st(OK, [50, SEC], 49, reset(SEC, now))],
              "expect_stats": {"basic.key1": stats(total_hits=1)},
              "expect_gauges": {"hit_count": 0, "miss_count": 1 if local_cache else 0,
                                "source_line": "integration_test.go:425-433"}})
    # :434-496 25x another/key2 (minute, 20)
    for i in range(25):
        code, rem = (OVER, 0) if i >= 20 else (OK, 20 - (i + 1))
        e = stats(total_hits=i + 1, over_limit=(i - 19) if i >= 20 else 0,
                  over_limit_with_local_cache=(i - 20) if (local_cache and i >= 20) else 0)
        s.append({"now": now, "seed": [], "request": req("another", [[["key2", "rand1"]]], 1),
                  "limits": [lim(20, MIN, "another.key2")],
                  "expect_statuses": [st(code, [20, MIN], rem, reset(MIN, now))],
                  "expect_stats": {"another.key2": e},
                  "expect_gauges": {"hit_count": (i - 20) if (local_cache and i >= 20) else 0,
                                    "miss_count": ((i + 2) if i < 20 else 22) if local_cache else 0,
                                    "source_line": "integration_test.go:479-495"}})
    # :498-583 15x another/{key2 (minute, 20), key3 (hour, 10)}
    for i in range(15):
        code3, rem3 = (OVER, 0) if i >= 10 else (OK, 10 - (i + 1))
        s.append({"now": now, "seed": [],
                  "request": req("another", [[["key2", "rand2"]], [["key3", "rand2"]]], 1),
                  "limits": [lim(20, MIN, "another.key2"), lim(10, HOUR, "another.key3")],
                  "expect_statuses": [st(OK, [20, MIN], 20 - (i + 1), reset(MIN, now)),
                                      st(code3, [10, HOUR], rem3, reset(HOUR, now))],
                  "expect_stats": {
                      "another.key2": stats(total_hits=i + 26, over_limit=5,
                                            over_limit_with_local_cache=4 if local_cache else 0),
                      "another.key3": stats(total_hits=i + 1, over_limit=(i - 9) if i >= 10 else 0,
                                            over_limit_with_local_cache=(i - 10) if (local_cache and i >= 10) else 0)},
                  "expect_gauges": {"hit_count": ((4 if i < 10 else i - 6) if local_cache else 0),
                                    "miss_count": ((i * 2 + 24 if i < 10 else i + 34) if local_cache else 0),
                                    "source_line": "integration_test.go:559-582"}})
    # :585-596 DurationUntilReset decreases between two hits 2 s apart (day unit, 20)
    s.append({"now": now, "seed": [], "request": req("another", [[["key4", "durTest"]]], 1),
              "limits": [lim(20, DAY, "another.key4")],
              "expect_statuses": [st(OK, [20, DAY], 19, reset(DAY, now))], "expect_stats": {}})
    s.append({"now": now + 2, "seed": [], "request": req("another", [[["key4", "durTest"]]], 1),
              "limits": [lim(20, DAY, "another.key4")],
              "expect_statuses": [st(OK, [20, DAY], 18, reset(DAY, now + 2))], "expect_stats": {}})
    return s


# integration_test.go:77-90: the five settings combinations of TestBasicConfig
for name, per_second, local_cache, prefix in [
    ("single", False, False, ""), ("per_second", True, False, ""),
    ("single_local_cache", False, True, ""), ("per_second_local_cache", True, True, ""),
    ("single_prefix", False, False, "prefix:")]:
    fixtures["ref_integration_%s" % name] = {
        "source": "test/integration/integration_test.go:77-90,371-597", "kind": "do_limit",
        "config": cfg(local_cache=local_cache, per_second=per_second, prefix=prefix),
        "steps": integration_steps(local_cache)}

# ---------------------------------------------------------------- near-limit threshold known answers
# SURVEY.md §8c "known-answer extras" (numpy fp32, the build's own checks, NOT reference vectors)
fixtures["own_near_threshold"] = {
    "source": "SURVEY.md §8c known-answer extras (build's own fp32 checks)", "kind": "near",
    "cases": [[5, 0.8, 4], [8, 0.8, 6], [10, 0.8, 8], [15, 0.8, 12], [20, 0.8, 16], [50, 0.8, 40],
              [500, 0.8, 400], [16777217, 0.8, 13421773], [4294967295, 0.8, 3435973888],
              [10, 0.9, 9], [33, 0.9, 29], [10, 0.75, 7], [33, 0.75, 24], [10, 0.7, 7], [7, 0.7, 4]]}


def main():
    for name, fx in fixtures.items():
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
    print("wrote %d fixtures" % len(fixtures))


if __name__ == "__main__":
    main()
