"""Pin the CPU oracle against the reference's own known answers (tests/golden/ref_*.json)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle import oracle as O  # noqa: E402
import golden_util as G  # noqa: E402


@pytest.mark.parametrize("name", G.names("do_limit"))
def test_oracle_do_limit_fixture(name):
    fx = G.load(name)
    c = fx["config"]
    jit = list(c["jitter_int63"])
    cache = O.OracleFixedRateLimitCache(
        near_limit_ratio=c["near_limit_ratio"], local_cache=c["local_cache"],
        cache_key_prefix=c["prefix"], per_second=c["per_second"],
        expiration_jitter_max_seconds=c["jitter_max"],
        jitter_int63=(lambda: jit.pop(0)) if jit else None)
    reg = G.StatsRegistry(O)
    for step in fx["steps"]:
        for sd in step["seed"]:
            cache.seed(sd["key"], sd["count"], -1, sd.get("per_second", False))
        req = G.make_request(O, step["request"])
        limits = [G.make_limit(O, reg, l) for l in step["limits"]]
        cache.client.log.clear()
        if cache.per_second_client is not None:
            cache.per_second_client.log.clear()
        out = cache.do_limit(req, limits, step["now"])
        assert [G.status_tuple(s) for s in out] == [G.expect_tuple(e) for e in step["expect_statuses"]]
        G.check_stats(reg, step["expect_stats"])
        if "expect_gauges" in step:
            G.check_gauges(G.oracle_gauges(cache, step["now"]), step["expect_gauges"])
        for client_name, cmds in step.get("expect_commands", {}).items():
            client = cache.client if client_name == "main" else cache.per_second_client
            assert [list(x) for x in client.log] == cmds


def test_oracle_cache_keys():
    fx = G.load("ref_generate_cache_keys")
    for case in fx["cases"]:
        cache = O.OracleFixedRateLimitCache(cache_key_prefix=case["prefix"])
        reg = G.StatsRegistry(O)
        req = G.make_request(O, case["request"])
        limits = [G.make_limit(O, reg, l) for l in case["limits"]]
        keys = cache.generate_cache_keys(req, limits, 1, case["now"])
        assert [k.key for k in keys] == case["expect_keys"]
        G.check_stats(reg, case.get("expect_stats", {}))


def test_oracle_decide():
    fx = G.load("ref_base_limiter_decide")
    for case in fx["cases"]:
        cache = O.OracleFixedRateLimitCache(near_limit_ratio=case["ratio"], local_cache=case["local_cache"])
        reg = G.StatsRegistry(O)
        limit = G.make_limit(O, reg, case["limit"])
        s = cache.get_response_descriptor_status(case["key"], limit, case["before"], case["after"],
                                                 case["lc"], case["hits"], case["now"])
        e = case["expect"]
        assert s.code == e["code"] and s.limit_remaining == e["remaining"]
        if "limit" in e:
            assert (s.current_limit.requests_per_unit, s.current_limit.unit) == tuple(e["limit"])
        if e.get("local_cache_set"):
            assert cache.local_cache.get(case["key"], case["now"])
        G.check_stats(reg, case["expect_stats"])


def test_oracle_incrby():
    fx = G.load("ref_driver_incrby")
    r = O.FakeRedis()
    for key, h, expect in fx["ops"]:
        assert r.incrby(key, h, 0) == expect


def test_oracle_near_threshold():
    for limit, ratio, expect in G.load("own_near_threshold")["cases"]:
        assert O.near_limit_threshold(limit, ratio) == expect, (limit, ratio)


def test_oracle_unknown_unit_panics():
    with pytest.raises(RuntimeError):
        O.unit_to_divider(O.UNIT_UNKNOWN)


def test_gauge_vectors_present_and_the_unreachable_one_explained():
    """integration_test.go:397-582 and fixed_cache_impl_test.go:218-279 / :524-589
    are transcribed; the one vector that breaks lookup = hit + miss keeps its
    transcription beside the executed value."""
    n = 0
    for name in G.names("do_limit"):
        for step in G.load(name)["steps"]:
            g = step.get("expect_gauges")
            if g is None:
                continue
            n += 1
            if "lookup_count" in g:
                assert g["lookup_count"] == g["hit_count"] + g["miss_count"]
            if "reference_vector" in g:
                h, m, lk = g["reference_vector"][:3]
                assert lk != h + m and g["source_line"].endswith((":260", ":567"))
    assert n == 5 * 42 + 2 * 4
