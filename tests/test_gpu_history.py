"""Time moving back: the history log (rl_device.h).

Redis keeps a window key div + jitter seconds after its last hit
(src/redis/fixed_cache_impl.go:71-74), so a request whose clock is behind
others (it waited in a batcher) still finds its window's count. The table
answers exactly every request whose window is at most 8 back from the newest
one written for its (stem, unit), and every request whose clock is within
div + J (expiration_jitter_max_seconds) of it; an older one whose window the
key may have had fails with RL_E_TIME. These streams revisit windows 2-8
back, and at J = 300 / 600 windows 9-300 s back (SECOND) and 9-11 back
(MINUTE), on the short-run, long-run (parallel) and multi-unit (exact) paths,
against the C and Python oracles, which model Redis keys without any window
limit.
"""
import numpy as np
import pytest

from oracle import c_oracle
from oracle import oracle as O
from ratelimit_amd import abi, workloads as W
from ratelimit_amd.limiter import Backend, GpuRateLimitCache, RedisError
import golden_util as G
import streams

pytestmark = pytest.mark.gpu

SMALL = dict(table_slots=1 << 16, max_batch=1 << 14, max_rules=1 << 10)


def _compare(batches, lc, isolate=False, jitter=0):
    be = Backend(0.8, lc, table_slots=1 << 18, max_batch=1 << 16, max_rules=8, jitter=jitter)
    co = c_oracle.COracle(0.8, lc, horizon=jitter)
    try:
        for i, (a, n, nq, nr) in enumerate(batches):
            g = be.do_limit_arrays(a, n, nq, nr, isolate=isolate)
            o = co.do_limit(a, n, nq, nr)
            if isolate:
                assert (g["status"] == 0).all(), np.unique(g["status"])
            for k in ("code", "limit_remaining", "reset_s", "stats"):
                if not np.array_equal(g[k], o[k]):
                    bad = np.nonzero(g[k] != o[k])[0][:5]
                    raise AssertionError("batch %d %s differs at %s: gpu %s oracle %s" % (i, k, bad, g[k][bad],
                                                                                          o[k][bad]))
    finally:
        be.close()
        co.close()


def _drop(a, n, nq, keep):
    return streams.drop_descriptors(a, n, nq, keep)


def _stream(seed, n_tenants, nq, batches, step, max_back, unit=None, multi=False, hot=0):
    """C1-shaped batches; batch k's clock is NOW0 + k*step and each request
    lags it by a uniform 0..max_back seconds. unit forces every descriptor's
    unit; multi gives every 4th tenant one stem under both units; hot adds a
    long run (the parallel path) of one tenant, every other batch in an
    older window."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(batches):
        base = W.NOW0 + k * step
        ten = rng.integers(0, n_tenants, nq)
        now = base - rng.integers(0, max_back + 1, nq)
        if hot and k >= 1:  # one tenant nobody else draws: forward on even batches, back on odd ones
            ten = np.r_[ten, np.full(hot, n_tenants + 7)]
            now = np.r_[now, np.full(hot, base - (max_back if k % 2 else 0))]
        a, n, q, nr = W.c1_batch(ten, now, rng.integers(1, 4, ten.size).astype(np.uint32))
        if unit is not None:
            a["unit"][:] = unit
        if multi:  # the minute descriptor of tenants % 4 == 0 uses the second descriptor's stem
            L = int(a["stem_off"][1])
            st = a["stem_bytes"].reshape(n, L)
            m = np.repeat(ten % 4 == 0, 2) & (np.arange(n) % 2 == 1)
            st[m] = st[np.nonzero(m)[0] - 1]
            a["limit"][:] = np.tile(np.array([6, 20], np.uint32), q)  # low limits: shared keys go over
        out.append((a, n, q, nr))
    return out


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_second_windows_up_to_7_back_vs_c_oracle(lc):
    _compare(_stream(1, 3_000, 6_000, 8, 3, 7, hot=200), lc, isolate=True)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_minute_windows_up_to_8_back_vs_c_oracle(lc):
    _compare(_stream(2, 3_000, 6_000, 8, 150, 479, unit=2, hot=200), lc, isolate=True)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_multi_unit_stems_moving_back_vs_c_oracle(lc):
    _compare(_stream(3, 2_000, 4_000, 8, 2, 5, multi=True), lc, isolate=True)


def test_gpu_history_default_path_no_statuses():
    """Without per-descriptor statuses (a failure would fail the whole batch)."""
    _compare(_stream(4, 1_000, 3_000, 6, 4, 7), False)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_calls_revisit_windows_vs_python_oracle(lc):
    """Call-level (the reference's DoLimit per RPC, one batch per chunk): a
    SECOND key revisits windows 2..7 back and a MINUTE key windows 2..5 back."""
    reg = {}

    def L(rpu, unit, key):
        reg.setdefault(key, O.RateLimitStats(key))
        return O.RateLimit(key, reg[key], O.Limit(rpu, unit))

    t = 1_700_000_030
    sec = [t, t + 1, t + 6, t + 4, t + 2, t + 7, t + 1, t, t + 8, t + 2, t + 3, t + 8]
    mn = [t, t + 60, t + 300, t + 120, t + 180, t + 61, t + 310, t + 100, t + 301, t + 62]
    calls = []
    for now in sec:
        calls.append((O.RateLimitRequest("d", [O.Descriptor([("k", "a")])], 1), [L(4, O.SECOND, "s")], now))
    for now in mn:
        calls.append((O.RateLimitRequest("d", [O.Descriptor([("k", "b")]), O.Descriptor([("k", "c")])], 2),
                      [L(5, O.MINUTE, "m"), L(3, O.MINUTE, "m2")], now))
    py_out, py_stats = streams.python_oracle_run(calls, 0.8, lc, "", False)
    streams.reset_stats(calls)
    cache = GpuRateLimitCache(None, 0.8, lc, "", False, **SMALL)
    outs = []
    for q0, q1 in ((0, 5), (5, 12), (12, 15), (15, len(calls))):
        outs.extend(cache.do_limit_batch(calls[q0:q1]))
    cache.close()
    stats = {l.stats.key: tuple(getattr(l.stats, f) for f in O.STAT_FIELDS) for _, ls, _ in calls for l in ls}
    assert [[G.status_tuple(s) for s in o] for o in outs] == [[s.as_tuple() for s in o] for o in py_out]
    assert stats == py_stats


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_second_windows_9_to_300_back_at_jitter_300_vs_c_oracle(lc):
    """Clocks up to 299 s behind the batch's newest (J = 300): windows far
    beyond the 8 always kept, every one answered exactly (no RL_E_TIME)."""
    _compare(_stream(7, 3_000, 6_000, 8, 40, 299, unit=1, hot=200), lc, isolate=True, jitter=300)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_minute_windows_9_to_11_back_at_jitter_600_vs_c_oracle(lc):
    _compare(_stream(8, 3_000, 6_000, 8, 200, 659, unit=2, hot=200), lc, isolate=True, jitter=600)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_multi_unit_stems_300_s_back_at_jitter_300_vs_c_oracle(lc):
    _compare(_stream(9, 2_000, 4_000, 8, 30, 299, multi=True), lc, isolate=True, jitter=300)


def test_gpu_beyond_the_history_fails_alone():
    """At J = 0, a SECOND window 9 back from a key's newest is beyond the
    history: RL_E_TIME for that descriptor only; 8 back is still exact."""
    be = Backend(0.8, False, **SMALL)
    co = c_oracle.COracle(0.8, False)
    t0 = W.NOW0
    for now in (t0, t0 + 8):
        b = W.c1_batch(np.arange(10), now)
        be.do_limit_arrays(*b, isolate=True)
        co.do_limit(*b)
    a, n, nq, nr = W.c1_batch(np.arange(10), np.r_[np.full(5, t0 - 1), np.full(5, t0)])
    g = be.do_limit_arrays(a, n, nq, nr, isolate=True)
    failed = np.zeros(n, bool)
    failed[0:10:2] = True  # SECOND descriptors at t0 - 1 (9 back from t0 + 8)
    assert (g["status"][failed] == abi.RL_E_TIME).all() and (g["status"][~failed] == 0).all()
    keep = ~failed
    o = co.do_limit(*_drop(a, n, nq, keep), nr)
    for k in ("code", "limit_remaining", "reset_s"):
        assert np.array_equal(g[k][keep], o[k]), k
    with pytest.raises(RedisError, match="RL_E_TIME"):
        be.do_limit_arrays(*W.c1_batch(np.arange(2), t0 - 2))
    be.close()
    co.close()


def test_gpu_jitter_horizon_bound():
    """J = 300: a SECOND key hit at t0 and t0 + 400. A request 300 s behind
    (t0 + 100, a window never written) is exact; 350 s behind, or the record
    of t0 itself (dead and dropped), is RL_E_TIME."""
    be = Backend(0.8, False, jitter=300, **SMALL)
    co = c_oracle.COracle(0.8, False, horizon=300)
    t0 = W.NOW0
    for now in (t0, t0 + 400):
        b = W.c1_batch(np.arange(4), now)
        be.do_limit_arrays(*b, isolate=True)
        co.do_limit(*b)
    a, n, nq, nr = W.c1_batch(np.arange(4), np.array([t0 + 100, t0 + 50, t0, t0 + 399]))
    g = be.do_limit_arrays(a, n, nq, nr, isolate=True)
    failed = np.zeros(n, bool)
    failed[[2, 4]] = True  # the SECOND descriptors of t0 + 50 and t0
    assert (g["status"][failed] == abi.RL_E_TIME).all(), g["status"]
    assert (g["status"][~failed] == 0).all(), g["status"]
    o = co.do_limit(*_drop(a, n, nq, ~failed), nr)
    for k in ("code", "limit_remaining", "reset_s"):
        assert np.array_equal(g[k][~failed], o[k]), k
    be.close()
    co.close()


@pytest.mark.parametrize("history_entries", [0, 1 << 16])
def test_gpu_snapshot_keeps_the_history(history_entries):
    """rl_snapshot_save/load carry the history log: a restored ctx answers
    older windows exactly like the one it was taken from."""
    bs = _stream(5, 500, 1_000, 6, 20, 150)
    kw = dict(table_slots=1 << 14, max_batch=1 << 12, max_rules=8, history_entries=history_entries, jitter=300)
    be = Backend(0.8, True, **kw)
    co = c_oracle.COracle(0.8, True, horizon=300)
    for a, n, nq, nr in bs[:4]:
        be.do_limit_arrays(a, n, nq, nr)
        co.do_limit(a, n, nq, nr)
    assert be.table_info()["history_appended"] > 0
    snap = be.snapshot()
    be.close()
    be2 = Backend(0.8, True, **kw)
    be2.load_snapshot(snap)
    for a, n, nq, nr in bs[4:]:
        g = be2.do_limit_arrays(a, n, nq, nr)
        o = co.do_limit(a, n, nq, nr)
        for k in ("code", "limit_remaining", "reset_s", "stats"):
            assert np.array_equal(g[k], o[k]), k
    be2.close()
    co.close()


def test_gpu_snapshot_rejects_a_bad_slot_image():
    """A slot image whose long stem points past the used arena is refused
    (RL_E_INVALID), not uploaded."""
    kw = dict(table_slots=1 << 12, max_batch=1 << 10, max_rules=8)
    be = Backend(0.8, False, **kw)
    a, n, nq, nr = W.c1_batch(np.arange(4), W.NOW0)
    be.do_limit_arrays(a, n, nq, nr)
    snap = bytearray(be.snapshot())
    slots = np.frombuffer(snap, np.uint8, count=64 * (1 << 12), offset=64).reshape(-1, 64)
    live = np.nonzero(slots[:, :4].view(np.uint32)[:, 0] >= 2)[0]
    assert live.size == 8
    i = 64 + 64 * int(live[0])
    snap[i + 4:i + 6] = np.uint16(200).tobytes()   # key_len 200: a long stem...
    snap[i + 60:i + 64] = np.uint32(1 << 30).tobytes()  # ...whose tail lies far past the arena
    with pytest.raises(RedisError, match="RL_E_INVALID"):
        be.load_snapshot(np.frombuffer(bytes(snap), np.uint8))
    be.close()


@pytest.mark.parametrize("tenants,nq", [(3_000, 4_000), (100_000, 150_000)])
def test_gpu_round4_pool_exhaustion_streams_are_exact(tenants, nq):
    """The streams that exhausted round 4's ring-line pool (64 lines, and 64
    partitions of 1024): with the history log at its default size every
    descriptor is answered, oracle-exact, none RL_E_TIME."""
    be = Backend(0.8, False, table_slots=1 << 19, max_batch=1 << 19, max_rules=8)
    co = c_oracle.COracle(0.8, False)
    try:
        for a, n, nq_, nr in _stream(6, tenants, nq, 8, 3, 7):
            g = be.do_limit_arrays(a, n, nq_, nr, isolate=True)
            o = co.do_limit(a, n, nq_, nr)
            assert (g["status"] == 0).all(), np.unique(g["status"])
            for k in ("code", "limit_remaining", "reset_s", "stats"):
                assert np.array_equal(g[k], o[k]), k
        info = be.table_info()
        assert info["history_lost"] == 0 and info["history_appended"] > 0
    finally:
        be.close()
        co.close()


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_history_log_overwritten_fails_never_miscounts(lc):
    """A log far too small for J = 300 (64 x 1024 entries against ~16k
    appends a batch): a lookup that reaches an overwritten entry fails with
    RL_E_TIME (counted in history_lost); every descriptor that succeeds
    matches the oracle fed only the descriptors that succeeded. Then the same
    keys, far ahead in time and moving back within their reach, are answered
    exactly again (their new history is walked before the broken part)."""
    be = Backend(0.8, lc, table_slots=1 << 16, max_batch=1 << 14, max_rules=8, history_entries=1, jitter=300)
    co = c_oracle.COracle(0.8, lc, horizon=300)
    failed_total = ok_total = 0
    try:
        assert be.table_info()["history_entries"] == 64 * 1024
        for a, n, nq, nr in _stream(10, 3_000, 8_000, 12, 20, 299, unit=1):
            g = be.do_limit_arrays(a, n, nq, nr, isolate=True)
            failed = g["status"] != 0
            assert (g["status"][failed] == abi.RL_E_TIME).all(), np.unique(g["status"])
            keep = ~failed
            o = co.do_limit(*_drop(a, n, nq, keep), nr)
            for k in ("code", "limit_remaining", "reset_s"):
                assert np.array_equal(g[k][keep], o[k]), k
            failed_total += int(failed.sum())
            ok_total += int(keep.sum())
        info = be.table_info()
        assert info["history_lost"] > 0 and failed_total > 0 and ok_total > failed_total
        assert info["history_appended"] > info["history_entries"]
        for k in range(4):  # 10 000 s later: forward, then up to 5 windows back
            t = W.NOW0 + 10_000 + 10 * k
            ten = np.arange(1_000)
            b = W.c1_batch(ten, t - (ten % 6) * (k % 2))
            g = be.do_limit_arrays(*b, isolate=True)
            o = co.do_limit(*b)
            assert (g["status"] == 0).all(), np.unique(g["status"])
            for f in ("code", "limit_remaining", "reset_s"):
                assert np.array_equal(g[f], o[f]), f
    finally:
        be.close()
        co.close()


def test_gpu_sweep_evicts_keys_with_history():
    """rl_sweep evicts a slot once its cur and every logged record are dead;
    a second and third generation of keys moving back are exact again."""
    be = Backend(0.8, False, table_slots=1 << 14, max_batch=1 << 14, max_rules=8)
    try:
        for gen in range(3):
            co = c_oracle.COracle(0.8, False)
            t = W.NOW0 + gen * 100_000
            for k in range(4):  # 400 keys, each one's cur moves forward then back
                ten = np.arange(400) + gen * 1000
                now = np.full(400, t + (3 if k % 2 else 0) + k)
                b = W.c1_batch(ten, now)
                g = be.do_limit_arrays(*b, isolate=True)
                o = co.do_limit(*b)
                assert (g["status"] == 0).all(), np.unique(g["status"])
                for f in ("code", "limit_remaining", "reset_s"):
                    assert np.array_equal(g[f], o[f]), f
            co.close()
            info = be.table_info()
            assert info["history_lost"] == 0 and info["history_slots"] > 0
            assert be.sweep(t + 50_000) > 0
            info = be.table_info()
            assert info["history_slots"] == 0 and info["live_slots"] == 0
    finally:
        be.close()
