"""Stems seen under several units (per-request overrides) on the parallel path.

A per-request override (config_impl.go:254-265) can give a descriptor a unit
other than its rule's, so one stem is counted under SECOND and MINUTE. The
Redis key is stem ‖ windowStart (cache_key.go:73-74): at t % 60 == 0 both
units hit the same key, otherwise two independent ones. k_split orders such a
stem's descriptors into one group per key and k_table's alias_setup sets the
groups up for the parallel path with write-back to every unit slot holding a
record of the key; until round 3 a hot stem like that was replayed by one lane
on every batch. Every answer must equal the C oracle's (full Redis semantics),
including the fallbacks to the exact path (clocks differing inside a batch,
one window in both stores of the per-second split, forced sort-key
collisions)."""
import numpy as np
import pytest

from oracle import c_oracle
from ratelimit_amd import workloads
from ratelimit_amd.limiter import Backend

pytestmark = pytest.mark.gpu

NOW0 = workloads.NOW0  # NOW0 % 60 == 20: NOW0 + 40 starts a minute


def _check(batches, lc, ps=False, isolate=False, **kw):
    cfg = dict(table_slots=1 << 17, max_batch=1 << 16, max_rules=8)
    cfg.update(kw)
    be = Backend(0.8, lc, ps, **cfg)
    co = c_oracle.COracle(0.8, lc, ps)
    try:
        for i, (a, n, nq, nr) in enumerate(batches):
            g = be.do_limit_arrays(a, n, nq, nr, isolate=isolate)
            o = co.do_limit(a, n, nq, nr)
            if isolate:
                assert not g["status"].any(), "batch %d: statuses %s" % (i, np.unique(g["status"]))
            for k in ("code", "limit_remaining", "reset_s", "stats"):
                assert np.array_equal(g[k], o[k]), "batch %d: %s differs at %s" % (
                    i, k, np.nonzero(np.asarray(g[k]) != np.asarray(o[k]))[0][:8])
    finally:
        be.close()
        co.close()


def _stream(now_rel, p_override=0.5, tenants=2000, rpb=20_000, seed=5, now_per_request=None):
    z = workloads.ZipfSampler(tenants, 1.1)
    rng = np.random.default_rng(seed)
    out = []
    for k, t0 in enumerate(now_rel):
        t = z.sample(rng, rpb)
        h = rng.integers(1, 9, rpb).astype(np.uint32)
        now = NOW0 + t0 if now_per_request is None else now_per_request(k, t0, rpb)
        p = p_override[k % len(p_override)] if isinstance(p_override, (list, tuple)) else p_override
        out.append(workloads.c2u_batch(t, now, h, rng, 16, p))
    return out


@pytest.mark.parametrize("lc", [False, True])
@pytest.mark.parametrize("isolate", [False, True])
def test_gpu_hot_override_stream_vs_c_oracle(lc, isolate):
    """Hot tenants with half their sec descriptors overridden to MINUTE: runs of
    ~1-3k descriptors of one stem under two units (split_long_body and
    k_split), across a minute boundary (one shared key at +40)."""
    _check(_stream([37, 38, 39, 40, 41, 42]), lc, isolate=isolate)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_override_on_and_off_vs_c_oracle(lc):
    """Batches with and without overrides, repeated and backward clocks: stems
    flagged multi-unit in the table take alias_setup alone (records of the
    other unit read as shared keys at +40, +60, +100, +120)."""
    _check(_stream([38, 40, 40, 41, 59, 60, 61, 60, 100, 100, 101, 120, 121],
                   p_override=[0.5, 0.0, 0.0, 0.3]), lc)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_override_per_second_split_vs_c_oracle(lc):
    """REDIS_PERSECOND: SECOND keys in their own store, the local-cache entry
    shared; one window in both stores (+40) stays on the exact path."""
    _check(_stream([38, 39, 40, 41, 100]), lc, ps=True)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_override_clock_changes_inside_batch_vs_c_oracle(lc):
    """The clock moves by a second halfway through each batch (over the minute
    boundary at +40): multi-unit stems without one `now` take the exact path,
    merged back into arrival order."""
    def npr(k, t0, nq):
        return NOW0 + t0 + (np.arange(nq) >= nq // 2).astype(np.int64)
    _check(_stream([38, 39, 40, 60, 61], now_per_request=npr), lc)


@pytest.mark.parametrize("bits", [6, 10])
def test_gpu_override_with_colliding_sort_keys_vs_c_oracle(bits):
    """Forced sort-key collisions (test-only hash width): multi-unit stems and
    other stems in one run, split into families and groups together."""
    for lc in (False, True):
        _check(_stream([39, 40, 41], tenants=3000, rpb=8000), lc, debug_hash_bits=bits)


def test_gpu_override_small_runs_vs_c_oracle():
    """Short multi-unit runs (uniform tenants, many overridden): groups of one
    and two descriptors stay with their head."""
    rng = np.random.default_rng(9)
    batches = []
    for k, t0 in enumerate([39, 40, 41, 100]):
        t = rng.integers(0, 40, 300)
        h = rng.integers(1, 4, 300).astype(np.uint32)
        batches.append(workloads.c2u_batch(t, NOW0 + t0, h, rng, hot=40, p_override=0.5))
    for lc in (False, True):
        _check(batches, lc)
