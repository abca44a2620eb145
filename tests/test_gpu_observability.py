"""GPU: local-cache gauges (localCacheStats, src/limiter/local_cache_stats.go:20-43)
and table snapshot / restore, against the oracle.

The stream gives every stem one unit (so a freecache key is exactly one window
record), small limits so the local cache fills, Zipf-skewed stems, hits 1..4
and a clock that crosses second and minute boundaries.
"""
import random

import numpy as np
import pytest

from oracle import oracle as O
from ratelimit_amd.limiter import GpuRateLimitCache, FixedTimeSource, RedisError

pytestmark = pytest.mark.gpu

SMALL = dict(table_slots=1 << 16, max_batch=1 << 14, max_rules=1 << 10)


def stream(seed, n_calls=3000, n_stems=60):
    rng = random.Random(seed)
    reg = {}
    w = [1.0 / (i + 1) ** 1.1 for i in range(n_stems)]
    units = [rng.choice([O.SECOND, O.MINUTE]) for _ in range(n_stems)]
    calls = []
    now = 1_700_000_030
    for i in range(n_calls):
        if rng.random() < 0.01:
            now += rng.randint(1, 25)
        descs, limits = [], []
        for _ in range(rng.randint(1, 3)):
            s = rng.choices(range(n_stems), w)[0]
            key = "rule%d" % (s % 7)
            if key + str(units[s]) not in reg:
                reg[key + str(units[s])] = O.new_rate_limit(5 + 3 * (s % 7), units[s], key + "_u%d" % units[s],
                                                            shadow_mode=(s % 11 == 0))
            descs.append(O.Descriptor([("stem", "s%03d" % s)]))
            limits.append(reg[key + str(units[s])])
        calls.append((O.RateLimitRequest("obs", descs, rng.randint(1, 4)), limits, now))
    return calls


def st(s):
    cl = None if s.current_limit is None else (s.current_limit.requests_per_unit, s.current_limit.unit)
    return (s.code, cl, s.limit_remaining, s.duration_until_reset)


def run_gpu(cache, calls, chunk):
    out = []
    for i in range(0, len(calls), chunk):
        out += cache.do_limit_batch(calls[i:i + chunk])
    return out


@pytest.mark.parametrize("local_cache", [True, False])
def test_gpu_local_cache_gauges_match_oracle(local_cache):
    calls = stream(7)
    oc = O.OracleFixedRateLimitCache(0.8, local_cache)
    cache = GpuRateLimitCache(FixedTimeSource(0), 0.8, local_cache, **SMALL)
    try:
        for i in range(0, len(calls), 500):
            part = calls[i:i + 500]
            want = [oc.do_limit(r, l, now) for r, l, now in part]
            got = cache.do_limit_batch(part)
            assert [[st(s) for s in g] for g in got] == [[st(s) for s in w] for w in want]
            now = part[-1][2]
            info = cache.backend.local_cache_info(now)
            if local_cache:
                lc = oc.local_cache
                assert info["hit_count"] == lc.hit_count
                assert info["miss_count"] == lc.miss_count
                assert info["lookup_count"] == lc.hit_count + lc.miss_count
                assert info["entry_count"] == lc.entry_count(now)
            else:
                assert info == {"entry_count": 0, "lookup_count": 0, "hit_count": 0, "miss_count": 0}
        assert not local_cache or oc.local_cache.hit_count > 100  # the stream exercises the cache
    finally:
        cache.close()


def test_gpu_snapshot_restore_continues_exactly():
    calls = stream(8)
    oc = O.OracleFixedRateLimitCache(0.8, True)
    want = [oc.do_limit(r, l, now) for r, l, now in calls]
    half = len(calls) // 2
    a = GpuRateLimitCache(FixedTimeSource(0), 0.8, True, **SMALL)
    b = GpuRateLimitCache(FixedTimeSource(0), 0.8, True, **SMALL)
    try:
        got = run_gpu(a, calls[:half], 300)
        img = a.backend.snapshot()
        a.close()
        b.backend.load_snapshot(img)
        got += run_gpu(b, calls[half:], 300)
        assert [[st(s) for s in g] for g in got] == [[st(s) for s in w] for w in want]
        small = GpuRateLimitCache(FixedTimeSource(0), 0.8, True, table_slots=1 << 15, max_batch=1 << 14,
                                  max_rules=1 << 10)
        try:
            with pytest.raises(RedisError, match="table_slots"):
                small.backend.load_snapshot(img)
            bad = img.copy()
            bad[0] ^= 0xFF
            with pytest.raises(RedisError, match="not a table snapshot"):
                small.backend.load_snapshot(bad)
        finally:
            small.close()
    finally:
        b.close()


def test_gpu_profile_sampling_counts_and_leaves_results_unchanged():
    """rl_profile(ctx, k) times every k-th batch, the k-th submitted after the
    call first (bench --prof-every), and does not change any decision."""
    calls = stream(11, n_calls=1400)
    oc = O.OracleFixedRateLimitCache(0.8, True)
    cache = GpuRateLimitCache(FixedTimeSource(0), 0.8, True, **SMALL)
    try:
        cache.backend.profile(True, 3)
        cache.backend.profile_read()
        n_batches = 0
        for i in range(0, len(calls), 200):
            part = calls[i:i + 200]
            want = [oc.do_limit(r, l, now) for r, l, now in part]
            got = cache.do_limit_batch(part)
            assert [[st(s) for s in g] for g in got] == [[st(s) for s in w] for w in want]
            n_batches += 1
        ms, nb = cache.backend.profile_read()
        assert nb == n_batches // 3
        assert all(v >= 0.0 for v in ms.values()) and ms["table"] > 0.0
        # k_table's own run time per sampled batch (device clock)
        assert 0.0 < ms["table_kernel"] < 10.0
        cache.backend.profile(False)
        cache.do_limit_batch(calls[-10:])
        assert cache.backend.profile_read()[1] == 0
    finally:
        cache.close()


def test_gpu_cache_health_check_follows_device_failures():
    """GpuRateLimitCache's health monitor on the real library: batches keep
    the check quiet, a request-level failure (a clock past 32 bits: RL_E_TIME)
    too; a device-level failure of a batch (RL_E_HIP, injected at the backend
    call: a dead device cannot be made on demand) fails it and the next
    answered batch marks it OK."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_health_cpu import FakeServer
    from oracle import oracle as O
    from ratelimit_amd.limiter import FixedTimeSource, GpuRateLimitCache
    from ratelimit_amd import abi
    srv = FakeServer()
    cache = GpuRateLimitCache(FixedTimeSource(1_700_000_000), health_server=srv, table_slots=1 << 12,
                              max_batch=1 << 10, max_rules=8)
    req = O.RateLimitRequest("d", [O.Descriptor([("k", "v")])], 1)
    lim = [O.RateLimit("d.k_v", O.RateLimitStats("d.k_v"), O.Limit(5, O.SECOND))]
    try:
        cache.do_limit(None, req, lim)
        cache.time_source = FixedTimeSource(1 << 33)  # a clock past the table's 32 bits: RL_E_TIME
        with pytest.raises(RedisError, match="RL_E_TIME"):
            cache.do_limit(None, req, lim)
        cache.time_source = FixedTimeSource(1_700_000_000)
        assert srv.calls == []
        real = cache.backend.do_limit_packed

        def dead(*a, **k):
            raise RedisError("gpu: hipErrorLaunchFailure [RL_E_HIP]", abi.RL_E_HIP)
        cache.backend.do_limit_packed = dead
        with pytest.raises(RedisError):
            cache.do_limit(None, req, lim)
        assert srv.calls == ["fail"]
        cache.backend.do_limit_packed = real
        assert cache.do_limit(None, req, lim)[0].limit_remaining == 3
        assert srv.calls == ["fail", "ok"]
    finally:
        cache.close()
