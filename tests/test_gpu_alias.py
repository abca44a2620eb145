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
from ratelimit_amd import abi, workloads
from ratelimit_amd.limiter import Backend
import streams

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


@pytest.mark.parametrize("lc,ps", [(False, False), (True, False), (True, True)])
def test_gpu_hot_override_whole_minute_vs_c_oracle(lc, ps):
    """Every second of a minute and into the next: the MINUTE key of a hot
    overridden stem is also the SECOND key of the minute's first second, whose
    record sits in the SECOND slot's cur at +41 (rolled away by that batch's
    SECOND group: read from the roll's log entry) and in its history log from
    +42 on (read there, written back to a new version). Both stay on the
    parallel path (until round 5 the exact path replayed the stem by one lane
    for the rest of the minute: C2U at 0.005 G decisions/s after 200 s)."""
    _check(_stream(list(range(38, 104)), rpb=4_000, tenants=500, seed=13), lc, ps)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_hot_override_ten_thousand_element_runs_vs_c_oracle(lc):
    """60k requests per batch: the hottest stems' runs (~10k and ~5k
    descriptors under two units, the size class of C2U's 58k-element runs)
    through split_long_body's chunked wave walks, across a minute boundary
    (+40: one shared key, a lone alias group)."""
    _check(_stream([38, 39, 40, 41], rpb=60_000, seed=9), lc, table_slots=1 << 17, max_batch=1 << 17)


@pytest.mark.parametrize("mode", ["0", "2"])
def test_gpu_long_splits_inline_and_on_the_long_kernel_vs_c_oracle(monkeypatch, mode):
    """The runs over 1024 elements walked by k_split's own 256-lane workgroups
    (RL_SPLIT_LONG=0) and by k_split_long's 1024-lane ones for every batch (2);
    the default (1) switches between the two after the first such batch. Also
    forced sort-key collisions, whose long runs of many stems end on the exact
    path from either kernel."""
    monkeypatch.setenv("RL_SPLIT_LONG", mode)
    _check(_stream([38, 39, 40, 41], rpb=60_000, seed=9), True, table_slots=1 << 17, max_batch=1 << 17)
    _check(_stream([39, 40, 41], tenants=3000, rpb=8000), False, debug_hash_bits=6)


@pytest.mark.parametrize("mode", ["0", "2"])
def test_gpu_long_runs_on_full_and_scanning_late_grids_vs_c_oracle(monkeypatch, mode):
    """k_late's long-run part on one workgroup per 256 sorted positions for
    every batch (RL_LATE_CUE=0) and on the few workgroups that walk k_table's
    bitmap for every batch (2); the default (1) uses the second until a batch
    has long runs. Hot keys under two units (alias groups), local cache on."""
    monkeypatch.setenv("RL_LATE_CUE", mode)
    _check(_stream([38, 39, 40, 41], rpb=20_000, seed=5), True, table_slots=1 << 17, max_batch=1 << 17)
    _check(_stream(list(range(38, 50)), rpb=4_000, tenants=500, seed=13), False)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_sort_keys_at_the_top_of_the_range_vs_c_oracle(lc):
    """debug_hash_bits=33: every stem's sort key is 0x7FFFFFFF or 0xFFFFFFFF,
    and the second is KEY_DUP, k_run_check's duplicate mark in the
    arrival-order keys, so k_prepare files those stems under 0xFFFFFFFE. Batches
    of one request (its two stems seen once, or a collision pair) and batches
    of 300 (two sort keys for every stem: mixed-stem runs through k_split and
    the exact path)."""
    _check(_stream(list(range(38, 68)), tenants=30, rpb=1, p_override=0.3), lc, debug_hash_bits=33)
    _check(_stream([39, 40, 41], tenants=40, rpb=300, p_override=0.3), lc, debug_hash_bits=33)


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


@pytest.mark.parametrize("n_shards,lc", [(2, False), (3, True)])
def test_gpu_override_multishard_ctx_vs_c_oracle(n_shards, lc):
    """A ctx hash-sharded over n_shards tables on cuda:0: each owner's routed
    batch (per-descriptor clocks and global request labels) goes through the
    same groups and alias_setup."""
    _check(_stream([38, 39, 40, 41]), lc, n_shards=n_shards, shard_devices=[0] * n_shards, hash_seed=77,
           max_rules=16)  # (routed owners keep stats per source: shards x rules)


@pytest.mark.parametrize("world", [2, 4])
def test_gpu_override_loopback_router_vs_c_oracle(world):
    """The library router at world 2 and 4 over the loopback transport: slices
    of hot overridden tenants routed to their owners."""
    from test_gpu_loopback import _check as lb_check, run_world
    cfg = (0.8, True, False)
    batches = _stream([39, 40, 41], rpb=6000)
    out = run_world(world, batches, cfg)
    for r in range(world):
        assert out[r][0] == "ok", out[r][1]
    lb_check(out, batches, cfg, world)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_override_bad_descriptor_in_hot_stem_fails_alone(lc):
    """A failed descriptor (unknown unit) inside a hot overridden stem's run:
    with statuses it fails alone; its run goes to the exact path and every
    other answer stays oracle-exact."""
    from test_gpu_robustness import _drop
    (a, n, nq, nr), = _stream([40], rpb=8000)
    hot = np.nonzero((a["unit"] == 2) & (a["rule_id"] == 2))[0]  # overridden sec descriptors
    bad = {k: v.copy() for k, v in a.items()}
    i = int(hot[len(hot) // 2])
    bad["unit"][i] = 9
    be = Backend(0.8, lc, table_slots=1 << 17, max_batch=1 << 16, max_rules=8)
    g = be.do_limit_arrays(bad, n, nq, nr, isolate=True)
    keep = np.ones(n, bool)
    keep[i] = False
    assert g["status"][i] == abi.RL_E_INVALID and (g["status"][keep] == 0).all()
    co = c_oracle.COracle(0.8, lc)
    o = co.do_limit(*_drop(bad, n, nq, keep), nr)
    co.close()
    be.close()
    for k in ("code", "limit_remaining", "reset_s"):
        assert np.array_equal(g[k][keep], o[k]), k
    assert np.array_equal(g["stats"], o["stats"])


def test_gpu_override_restore_then_limit_vs_c_oracle():
    """rl_restore seeding one stem under SECOND and MINUTE at a shared window
    (restore batches run the same grouping; a multi-unit stem there takes the
    exact path, merged in arrival order), then override batches on top."""
    stems = [b"bench_tenant_t%010d_tier_sec_" % t for t in range(8)]
    units = [1, 2] * 4
    nows = [NOW0 + 40] * 8
    counts = [5, 7, 0, 3, 90, 95, 1, 1]
    lcs = [0, 0, 0, 0, 1, 0, 0, 0]
    for lc in (False, True):
        be = Backend(0.8, lc, table_slots=1 << 16, max_batch=1 << 15, max_rules=8)
        co = c_oracle.COracle(0.8, lc)
        be.restore([stems[k // 2 * 2] for k in range(8)], units, nows, counts, lcs)
        co.restore([stems[k // 2 * 2] for k in range(8)], units, nows, counts, lcs)
        rng = np.random.default_rng(3)
        for t0 in (40, 40, 41, 60):
            t = rng.integers(0, 8, 400)
            h = rng.integers(1, 4, 400).astype(np.uint32)
            a, n, nq, nr = workloads.c2u_batch(t, NOW0 + t0, h, rng, hot=8, p_override=0.5)
            g = be.do_limit_arrays(a, n, nq, nr)
            o = co.do_limit(a, n, nq, nr)
            for k in ("code", "limit_remaining", "reset_s", "stats"):
                assert np.array_equal(g[k], o[k]), (t0, k)
        be.close()
        co.close()


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_c2u_bench_scale_vs_c_oracle(lc):
    """BASELINE-scale C2U batches (1M descriptors; the hottest tenant's stem runs
    tens of thousands of descriptors under two units: split_long_body's wave
    walks over many 16-step rounds), across a minute boundary (+40: SECOND and
    MINUTE share the key), against the C oracle."""
    z = workloads.ZipfSampler(2_000_000, 1.1)
    bs = list(workloads.c2u_stream(n_tenants=2_000_000, requests_per_batch=500_000, batches=4, now0=NOW0 + 38,
                                   sampler=z))
    _check(bs, lc, table_slots=1 << 23, max_batch=1 << 20)


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_hot_override_far_too_small_log_fails_never_miscounts(lc):
    """the alias groups' records in a history log far too small
    (64 x 1024 entries, wrapping every few batches, J = 300): k_late writes a
    group's count back into the log entry alias_setup appended in the same
    batch, which no append of that batch may overwrite (log_append refuses
    instead). Every descriptor is RL_E_TIME or equal to the oracle fed only
    the descriptors that succeeded."""
    be = Backend(0.8, lc, table_slots=1 << 17, max_batch=1 << 14, max_rules=8, history_entries=1, jitter=300)
    co = c_oracle.COracle(0.8, lc, horizon=300)
    failed_total = ok_total = 0
    try:
        assert be.table_info()["history_entries"] == 64 * 1024
        for a, n, nq, nr in _stream(list(range(38, 98)) + list(range(40, 70)), rpb=8_000, tenants=30_000, seed=21):
            g = be.do_limit_arrays(a, n, nq, nr, isolate=True)
            failed = g["status"] != 0
            assert (g["status"][failed] == abi.RL_E_TIME).all(), np.unique(g["status"])
            keep = ~failed
            o = co.do_limit(*streams.drop_descriptors(a, n, nq, keep), nr)
            for k in ("code", "limit_remaining", "reset_s"):
                assert np.array_equal(g[k][keep], o[k]), k
            failed_total += int(failed.sum())
            ok_total += int(keep.sum())
        info = be.table_info()
        assert info["history_appended"] > info["history_entries"]  # the log wrapped
        assert ok_total > failed_total
    finally:
        be.close()
        co.close()
