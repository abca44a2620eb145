"""One rl_ctx hash-sharding its table over several GPUs (rl_config.n_shards).

The multi-GPU path behind the C ABI: one process, one ctx,
n_shards engines, each with a router (rl_comm.hip) on its own worker thread,
the routers joined in an in-process loopback world. A host batch is cut into
request-aligned slices, one per shard, each crossing its shard's own PCIe link
(rl_do_limit, rl_do_limit_host_async); a device batch is taken whole by shard
0 (rl_do_limit_async). Either way every descriptor goes to its owner shard
and back, and the shards' stats are summed. Here all shards sit on cuda:0
(shard_device = [0, 0, ...]: the routing, per-owner pipelines, stats sums and
slices are the same code as across devices; only the copies are plain device
copies instead of xGMI peer copies).

Answers and stats of every entry point must equal the single-table oracles
(Python oracle for random streams, C oracle for C2 batches), and the table
maintenance calls (sweep, table_info, restore, snapshot) must act on the union
of the shards exactly as on one table.
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from ratelimit_amd import abi, workloads
from ratelimit_amd.limiter import Backend, GpuRateLimitCache, RedisError
import golden_util as G
import streams

pytestmark = pytest.mark.gpu

SMALL = dict(table_slots=1 << 16, max_batch=1 << 15, max_rules=1 << 10, hash_seed=0x5EED)


def _shards(n):
    return dict(n_shards=n, shard_devices=[0] * n)


def _c2(n_batches=4, tenants=20_000, per_batch=6_000, seed=3):
    z = workloads.ZipfSampler(tenants, 1.1)
    return list(workloads.c2_stream(seed=seed, n_tenants=tenants, requests_per_batch=per_batch, batches=n_batches,
                                    sampler=z))


def _to_dev(a):
    return {k: torch.from_numpy(np.ascontiguousarray(v).view({np.dtype(np.uint32): np.int32}.get(v.dtype, v.dtype)))
            .to("cuda") for k, v in a.items()}


@pytest.mark.parametrize("n_shards", [2, 3])
@pytest.mark.parametrize("lc", [False, True])
def test_gpu_multishard_random_stream_vs_python_oracle(n_shards, lc):
    calls = streams.random_stream(40 + n_shards, n_calls=500, zipf=True)
    py_out, py_stats = streams.python_oracle_run(calls, 0.8, lc, "", False)
    streams.reset_stats(calls)
    cache = GpuRateLimitCache(None, 0.8, lc, "", False, **SMALL, **_shards(n_shards))
    outs = []
    try:
        i = 0
        for k in (100, 1, 0, 150, 249):
            outs += cache.do_limit_batch(calls[i:i + k])
            i += k
    finally:
        cache.close()
    got = [[G.status_tuple(s) for s in o] for o in outs]
    exp = [[s.as_tuple() for s in o] for o in py_out]
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g == e, "call %d: gpu %s oracle %s" % (i, g, e)
    stats = {}
    for _, limits, _ in calls:
        for l in limits:
            if l is not None:
                stats[l.stats.key] = tuple(getattr(l.stats, f) for f in abi.STAT_FIELDS)
    assert stats == py_stats


@pytest.mark.parametrize("n_shards,lc,ps", [(2, False, False), (2, True, False), (4, True, True)])
def test_gpu_multishard_c2_host_path_vs_c_oracle(n_shards, lc, ps):
    be = Backend(0.8, lc, ps, table_slots=1 << 17, max_batch=1 << 15, max_rules=8, hash_seed=99,
                 **_shards(n_shards))
    co = c_oracle.COracle(0.8, lc, ps)
    for a, n, nq, nr in _c2():
        g = be.do_limit_arrays(a, n, nq, nr)
        o = co.do_limit(a, n, nq, nr)
        for k in ("code", "limit_remaining", "reset_s", "stats"):
            assert np.array_equal(g[k], o[k]), k
    # every shard holds part of the keys; the sum is the whole table
    infos = [be.table_info(shard=j) for j in range(n_shards)]
    assert all(i["live_slots"] > 0 for i in infos)
    assert sum(i["live_slots"] for i in infos) == be.table_info()["live_slots"]
    be.close()
    co.close()


@pytest.mark.parametrize("n_shards", [2, 3])
def test_gpu_multishard_max_rules_equal_to_batch_rules(n_shards):
    """max_rules == n_rules: the owners keep stats per source
    slice, so each shard holds n_shards x max_rules rows; a batch carrying all
    max_rules rules answers and sums its stats like one table, through the host,
    the pipelined host and the device entry points."""
    be = Backend(0.8, True, table_slots=1 << 17, max_batch=1 << 15, max_rules=2, hash_seed=7,
                 **_shards(n_shards))
    co = c_oracle.COracle(0.8, True)
    batches = _c2(n_batches=3, seed=11)
    for a, n, nq, nr in batches[:2]:
        assert nr == 2
        g = be.do_limit_arrays(a, n, nq, nr)
        o = co.do_limit(a, n, nq, nr)
        for k in ("code", "limit_remaining", "reset_s", "stats"):
            assert np.array_equal(g[k], o[k]), k
    a, n, nq, nr = batches[2]
    dev = _to_dev(a)
    out = {"code": torch.zeros(n, dtype=torch.uint8, device="cuda"),
           "limit_remaining": torch.zeros(n, dtype=torch.int32, device="cuda"),
           "reset_s": torch.zeros(n, dtype=torch.int32, device="cuda"),
           "stats": torch.zeros(nr * abi.RL_NUM_STATS, dtype=torch.int64, device="cuda")}
    torch.cuda.synchronize()
    be.do_limit_device(dev, out, n, nq, nr)
    be.synchronize()
    o = co.do_limit(a, n, nq, nr)
    assert np.array_equal(out["code"].cpu().numpy(), o["code"])
    assert np.array_equal(out["limit_remaining"].cpu().numpy().view(np.uint32), o["limit_remaining"])
    assert np.array_equal(out["stats"].cpu().numpy().view(np.uint64), o["stats"])
    be.close()
    co.close()


def test_gpu_multishard_async_device_path_pipelined_vs_c_oracle():
    """rl_do_limit_async with device arrays: every batch submitted before one
    synchronize (RSLOTS routed batches in flight)."""
    batches = _c2(n_batches=6, per_batch=5_000)
    be = Backend(0.8, True, table_slots=1 << 17, max_batch=1 << 15, max_rules=8, hash_seed=5, **_shards(2))
    co = c_oracle.COracle(0.8, True)
    want = [co.do_limit(*b) for b in batches]
    co.close()
    outs = []
    for a, n, nq, nr in batches:
        d_in = _to_dev(a)
        d_out = {"code": torch.zeros(n, dtype=torch.uint8, device="cuda"),
                 "limit_remaining": torch.zeros(n, dtype=torch.int32, device="cuda"),
                 "reset_s": torch.zeros(n, dtype=torch.int32, device="cuda"),
                 "stats": torch.zeros(nr * abi.RL_NUM_STATS, dtype=torch.int64, device="cuda")}
        be.do_limit_device(d_in, d_out, n, nq, nr)
        outs.append((d_in, d_out))
    be.synchronize()
    for (d_in, d_out), w in zip(outs, want):
        assert np.array_equal(d_out["code"].cpu().numpy(), w["code"])
        assert np.array_equal(d_out["limit_remaining"].cpu().numpy().view(np.uint32), w["limit_remaining"])
        assert np.array_equal(d_out["reset_s"].cpu().numpy().view(np.uint32), w["reset_s"])
        assert np.array_equal(d_out["stats"].cpu().numpy().view(np.uint64), w["stats"])
    be.close()


def test_gpu_multishard_one_bad_descriptor_fails_alone():
    (a, n, nq, nr), = _c2(n_batches=1, tenants=3_000, per_batch=4_000)
    bad = {k: v.copy() for k, v in a.items()}
    bad["unit"][7] = 9
    bad["rule_id"][1001] = 99
    be = Backend(0.8, True, **SMALL, **_shards(2))
    with pytest.raises(RedisError, match="RL_E_INVALID"):
        be.do_limit_arrays(bad, n, nq, nr)
    g = be.do_limit_arrays(bad, n, nq, nr, isolate=True)
    failed = np.zeros(n, bool)
    failed[[7, 1001]] = True
    assert (g["status"][failed] == abi.RL_E_INVALID).all() and (g["status"][~failed] == 0).all()
    idx = np.nonzero(~failed)[0]
    off = bad["stem_off"]
    stems = [bad["stem_bytes"][off[i]:off[i + 1]] for i in idx]
    o_off = np.zeros(idx.size + 1, np.uint32)
    o_off[1:] = np.cumsum([s.size for s in stems])
    kept = {"stem_bytes": np.concatenate(stems), "stem_off": o_off, "now": bad["now"]}
    for k in ("req_idx", "unit", "flags", "limit", "hits", "rule_id"):
        kept[k] = bad[k][idx]
    co = c_oracle.COracle(0.8, True)
    o = co.do_limit(kept, idx.size, nq, nr)
    co.close()
    for k in ("code", "limit_remaining", "reset_s"):
        assert np.array_equal(g[k][~failed], o[k]), k
    assert np.array_equal(g["stats"], o["stats"])
    be.close()


def test_gpu_multishard_maintenance_matches_one_table():
    """sweep / table_info / local_cache_info / restore / snapshot on 3 shards act
    like the same calls on one table, and a snapshot reloads into a fresh
    3-shard ctx that answers the rest of the stream exactly."""
    batches = _c2(n_batches=4, tenants=8_000, per_batch=4_000)
    one = Backend(0.8, True, **SMALL)
    three = Backend(0.8, True, **SMALL, **_shards(3))
    for b in batches[:2]:
        g1, g3 = one.do_limit_arrays(*b), three.do_limit_arrays(*b)
        for k in g1:
            assert np.array_equal(g1[k], g3[k]), k
    t = workloads.NOW0
    for f in ("live_slots", "arena_bytes_used"):
        assert one.table_info()[f] == three.table_info()[f], f
    assert one.local_cache_info(t + 1) == three.local_cache_info(t + 1)
    # restore a few keys into both (owner routing on the host for 3 shards)
    stems = [b"restored_%d" % i for i in range(50)]
    units = [2] * 50  # RL_UNIT_MINUTE
    one.restore(stems, units, [t] * 50, list(range(50)))
    three.restore(stems, units, [t] * 50, list(range(50)))
    assert one.table_info()["live_slots"] == three.table_info()["live_slots"]
    snap = three.snapshot()
    fresh = Backend(0.8, True, **dict(SMALL, hash_seed=1), **_shards(3))  # adopts the snapshot's key
    fresh.load_snapshot(snap)
    for b in batches[2:]:
        g1, g3 = one.do_limit_arrays(*b), fresh.do_limit_arrays(*b)
        for k in g1:
            assert np.array_equal(g1[k], g3[k]), k
    # sweeping far in the future evicts the same keys
    assert one.sweep(t + 10 * 86400) == fresh.sweep(t + 10 * 86400)
    assert fresh.table_info()["live_slots"] == one.table_info()["live_slots"] == 0
    for be in (one, three, fresh):
        be.close()


def test_gpu_multishard_bad_config():
    with pytest.raises(ValueError):
        Backend(0.8, False, **SMALL, n_shards=17, shard_devices=[0] * 17)
    with pytest.raises(ValueError):
        Backend(0.8, False, **SMALL, n_shards=2, shard_devices=[0])


def test_gpu_multishard_long_and_ragged_stems_vs_c_oracle():
    """Stems of 1..300 bytes, Zipf-repeated: partition tiles whose stems do not
    fit the LDS staging area take the direct byte-copy path, short ones the
    staged dword path; unaligned chunk boundaries on every owner."""
    from ratelimit_amd.packing import arrays_from_lists
    rng = np.random.default_rng(9)
    pool = [bytes(rng.integers(33, 127, int(L)).astype(np.uint8)) for L in
            np.r_[rng.integers(1, 40, 2000), rng.integers(80, 300, 2000)]]
    z = workloads.ZipfSampler(len(pool), 1.1)
    batches = []
    for k in range(3):
        nq = 5000
        ids = z.sample(rng, nq)
        if k == 1:  # one tile of only long stems, one of only short ones
            ids[:512] = rng.integers(2000, 4000, 512)
            ids[512:1024] = rng.integers(0, 2000, 512)
        stems = [pool[i] for i in ids]
        a = arrays_from_lists(stems, np.full(nq, workloads.NOW0 + k, np.int64), np.arange(nq),
                              rng.integers(1, 5, nq), np.zeros(nq), rng.integers(1, 50, nq), rng.integers(1, 4, nq),
                              rng.integers(0, 4, nq))
        pad = (-a["stem_bytes"].size) % 4  # (device stems: 4-byte aligned, whole dwords)
        a["stem_bytes"] = np.r_[a["stem_bytes"], np.zeros(pad + 4, np.uint8)]
        batches.append((a, nq, nq, 4))
    for n_shards in (1, 3):
        be = Backend(0.8, True, table_slots=1 << 16, max_batch=1 << 14, max_rules=16, hash_seed=3,
                     **_shards(n_shards))
        co = c_oracle.COracle(0.8, True)
        for b in batches:
            g, o = be.do_limit_arrays(*b), co.do_limit(*b)
            for key in ("code", "limit_remaining", "reset_s", "stats"):
                assert np.array_equal(g[key], o[key]), (n_shards, key)
        be.close()
        co.close()


@pytest.mark.parametrize("n_shards,lc,isolate", [(2, False, False), (3, True, True), (4, True, False)])
def test_gpu_multishard_host_async_pipelined_vs_c_oracle(n_shards, lc, isolate):
    """rl_do_limit_host_async on a multi-shard ctx: every slice crosses its own
    shard's link; eight batches (more than the routers keep in flight, so the
    stats of the oldest are summed before its slot is reused) submitted before
    one synchronize, from page-locked buffers."""
    from ratelimit_amd.limiter import PinnedArena
    from ratelimit_amd.packing import PackedBatch
    batches = _c2(n_batches=8, per_batch=5_000, seed=17)
    co = c_oracle.COracle(0.8, lc)
    want = [co.do_limit(*b) for b in batches]
    co.close()
    be = Backend(0.8, lc, table_slots=1 << 17, max_batch=1 << 15, max_rules=16, hash_seed=7, **_shards(n_shards))
    arena = PinnedArena()
    keep = []
    for a, n, nq, nr in batches:
        pb = PackedBatch({k: arena.like(v) for k, v in a.items()}, n, nq, nr)
        out = {k: arena.like(v) for k, v in pb.alloc_result(isolate).items()}
        keep.append((pb, out, be.do_limit_host_async(pb, out)))
    be.synchronize()
    for (pb, out, _), w in zip(keep, want):
        n = pb.n
        for k in ("code", "limit_remaining", "reset_s"):
            assert np.array_equal(out[k][:n], w[k]), k
        assert np.array_equal(out["stats"][:pb.n_rules * abi.RL_NUM_STATS], w["stats"])
        if isolate:
            assert not out["status"][:n].any()
    be.close()
    arena.close()


def test_gpu_multishard_host_async_rejects_and_recovers():
    """A host batch larger than max_batch is refused at the call (no shard
    takes any of it); the next batches are answered exactly."""
    from ratelimit_amd.limiter import PinnedArena
    from ratelimit_amd.packing import PackedBatch
    batches = _c2(n_batches=3, per_batch=3_000, seed=23)
    big = workloads.concat_batches(_c2(n_batches=2, per_batch=3_000, seed=24))
    be = Backend(0.8, True, table_slots=1 << 16, max_batch=8_192, max_rules=16, hash_seed=7, **_shards(2))
    co = c_oracle.COracle(0.8, True)
    arena = PinnedArena()

    def run(a, n, nq, nr):
        pb = PackedBatch({k: arena.like(v) for k, v in a.items()}, n, nq, nr)
        out = {k: arena.like(v) for k, v in pb.alloc_result().items()}
        ref = be.do_limit_host_async(pb, out)
        return pb, out, ref

    r0 = run(*batches[0])
    be.synchronize()
    w0 = co.do_limit(*batches[0])
    assert np.array_equal(r0[1]["code"][:r0[0].n], w0["code"])
    with pytest.raises(RedisError, match="RL_E_CAPACITY"):
        run(*big)  # 12000 descriptors > max_batch: taken by no shard
    for b in batches[1:]:
        pb, out, _ = run(*b)
        be.synchronize()
        w = co.do_limit(*b)
        for k in ("code", "limit_remaining", "reset_s", "stats"):
            assert np.array_equal(out[k][:pb.n if k != "stats" else pb.n_rules * abi.RL_NUM_STATS], w[k]), k
    be.close()
    co.close()
    arena.close()
