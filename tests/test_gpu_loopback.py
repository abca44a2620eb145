"""The library's multi-rank router (rl_comm.hip) at world 2-4 on ONE GPU.

rl_comm_loopback_id gives an in-process world: each rank is a host thread with
its own single-shard Backend on cuda:0, and the exchanges (counts, records and
stems, results and stats) are device copies through the loopback transport
with the RCCL transport's grouped send/recv contract (rl_transport.h). This is
the code path an 8-GPU node runs (bench.py --gpus 8): partition by owner,
counts with n_rules and flags, per-peer offsets, receive-buffer growth, owner
parts cut at request boundaries, per-source stats blocks, scatter to arrival
order. RCCL itself refuses two ranks on one device, so on a one-GPU machine
this is the only way the W > 1 exchange runs.

Every batch is the node batch split into per-rank request slices (uneven,
sometimes empty); the concatenation of the ranks' answers in rank order must
equal the C oracle over the whole batch, and the ranks' stats must sum to its
stats. Reference: the Redis cluster client's key-slot routing inside one
service process (src/redis/driver_impl.go:108-126) with the sequential INCRBY
order of fixed_cache_impl.go:51-110 across the whole node batch.
"""
import threading
import traceback

import numpy as np
import pytest

from oracle.c_oracle import COracle
from ratelimit_amd import abi, workloads as W
from ratelimit_amd._lib import RedisError
from ratelimit_amd.limiter import Backend
from ratelimit_amd.packing import RuleInterner, pack_calls, slice_requests
import streams
from test_sharded_cpu import _split_points

pytestmark = pytest.mark.gpu
SEED = 0x5EED


def _random_batches(seed, per=60, n_calls=480):
    calls = streams.random_stream(seed, n_calls=n_calls, zipf=True)
    interner = RuleInterner()
    pbs = [pack_calls(calls[k:k + per], "", interner) for k in range(0, len(calls), per)]
    nr = max(len(interner.keys), 1)
    return [(pb.arrays, pb.n, pb.n_requests, nr) for pb in pbs]


def _c2_batches(seed, requests=6_000, batches=4):
    return list(W.c2_stream(seed=seed, n_tenants=20_000, requests_per_batch=requests, batches=batches))


def _dev(a, dev):
    import torch
    return {k: torch.from_numpy(np.ascontiguousarray(v).view({np.dtype(np.uint32): np.int32}.get(v.dtype, v.dtype)))
            .to(dev) for k, v in a.items()}


def run_world(world, batches, cfg, *, max_batch=1 << 15, max_rules=64, slices=None, isolate=(), n_rules_of=None,
              serial=False, table_slots=1 << 18, after=None, before=None):
    """Drive `world` loopback ranks over `batches`. slices(k) -> request cut
    points (default: uneven random); isolate: ranks passing out.status;
    n_rules_of(rank, k) overrides a rank's n_rules. Returns per rank either
    ("ok", [(n, results dict) per batch]) or ("err", message)."""
    import os
    import torch
    from ratelimit_amd.sharded import LibRouter, loopback_id
    os.environ.setdefault("RL_LOOPBACK_TIMEOUT_S", "30")  # (read at join: a stuck peer fails, never hangs)
    uid = loopback_id()
    bes = [Backend(*cfg, table_slots=table_slots, max_batch=max_batch, max_rules=max_rules, device=0, hash_seed=SEED)
           for _ in range(world)]
    routers = [LibRouter(be, world, r, uid) for r, be in enumerate(bes)]
    out = [None] * world

    def body(r):
        dev = torch.device("cuda", 0)
        keep = []
        try:
            if before:
                before(r, bes[r])
            for k, (arrays, n, nq, n_rules) in enumerate(batches):
                cuts = slices(k) if slices else _split_points(nq, world, k)
                sub, sn, snq = slice_requests(arrays, n, nq, cuts[r], cuts[r + 1])
                nr = n_rules_of(r, k) if n_rules_of else n_rules
                dev_in = _dev(sub, dev)
                m = max(sn, 1)
                dev_out = {"code": torch.zeros(m, dtype=torch.uint8, device=dev),
                           "limit_remaining": torch.zeros(m, dtype=torch.int32, device=dev),
                           "reset_s": torch.zeros(m, dtype=torch.int32, device=dev),
                           "stats": torch.zeros(max(nr, 1) * abi.RL_NUM_STATS, dtype=torch.int64, device=dev)}
                if r in isolate:
                    dev_out["status"] = torch.zeros(m, dtype=torch.uint8, device=dev)
                routers[r].submit(dev_in, sn, snq, nr, dev_out)
                keep.append((sn, nr, dev_in, dev_out))
                if serial:
                    routers[r].finish()
            routers[r].finish()
            if after:
                after(r, bes[r])
            res = []
            for sn, nr, _, o in keep:
                d = {"code": o["code"][:sn].cpu().numpy(),
                     "limit_remaining": o["limit_remaining"][:sn].cpu().numpy().view(np.uint32),
                     "reset_s": o["reset_s"][:sn].cpu().numpy().view(np.uint32),
                     "stats": o["stats"][:nr * abi.RL_NUM_STATS].cpu().numpy().view(np.uint64)}
                if "status" in o:
                    d["status"] = o["status"][:sn].cpu().numpy()
                res.append((sn, d))
            out[r] = ("ok", res)
        except RedisError as e:
            out[r] = ("err", str(e))
            try:  # a failed rank still completes the collective steps it owes
                routers[r].finish()
            except RedisError:
                pass
        except Exception:
            out[r] = ("exc", traceback.format_exc())

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=90)
    alive = [t.is_alive() for t in ts]
    for be in bes if not any(alive) else []:
        be.close()
    assert not any(alive), "a loopback rank hung"
    for r in range(world):
        assert out[r][0] != "exc", out[r][1]
    return out


def _check(out, batches, cfg, world, ranks=None):
    co = COracle(*cfg)
    for k, (arrays, n, nq, n_rules) in enumerate(batches):
        exp = co.do_limit(arrays, n, nq, n_rules)
        rs = range(world) if ranks is None else ranks
        for f in ("code", "limit_remaining", "reset_s"):
            got = np.concatenate([out[r][1][k][1][f] for r in rs])
            bad = np.nonzero(got != exp[f])[0]
            assert bad.size == 0, (k, f, bad.size, bad[:8].tolist(), got[bad[:8]].tolist(), exp[f][bad[:8]].tolist())
        tot = sum(out[r][1][k][1]["stats"].astype(np.uint64) for r in rs)
        assert np.array_equal(tot, exp["stats"]), k
    co.close()


@pytest.mark.parametrize("world,kind,lc,serial", [
    (2, "random", True, False), (3, "random", False, True), (4, "random", True, False),
    (2, "c2", False, False), (3, "c2", True, False), (4, "c2", False, True)])
def test_gpu_loopback_router_matches_oracle(world, kind, lc, serial):
    cfg = (0.8, lc, False)
    batches = _random_batches(7 + world) if kind == "random" else _c2_batches(11 + world)
    out = run_world(world, batches, cfg, serial=serial)
    for r in range(world):
        assert out[r][0] == "ok", out[r][1]
    _check(out, batches, cfg, world)


@pytest.mark.parametrize("world", [2, 4])
def test_gpu_loopback_owner_parts(world, monkeypatch):
    """RL_DEBUG_OWNER_PART: an owner answers what it received in parts of 2500
    records cut at request boundaries (stats summed over the parts)."""
    monkeypatch.setenv("RL_DEBUG_OWNER_PART", "2500")
    cfg = (0.8, True, False)
    batches = _c2_batches(21)
    out = run_world(world, batches, cfg)
    _check(out, batches, cfg, world)


def test_gpu_loopback_skewed_owner_over_max_batch():
    """One hot tenant carries 80% of the node batch: its owner receives more
    than max_batch records (every slice fits) and answers them in parts; its
    receive buffers grow on the way."""
    cfg = (0.8, True, False)
    rng = np.random.default_rng(5)
    batches = []
    for k in range(3):
        t = np.where(rng.random(12_000) < 0.8, 7, rng.integers(0, 5_000, 12_000))
        batches.append(W.c1_batch(t, W.NOW0 + k, rng.integers(1, 4, 12_000).astype(np.uint32)))
    even = lambda k: [0, 4_000, 8_000, 12_000]  # 8000 descriptors per rank
    out = run_world(3, batches, cfg, max_batch=1 << 13, slices=even)
    _check(out, batches, cfg, 3)


def _with_bad(arrays, n, nq):
    bad = {k: v.copy() for k, v in arrays.items()}
    bad["unit"][7] = 9                # unknown unit
    bad["rule_id"][1001] = 99         # rule id >= n_rules
    bad["now"][2500] = -5             # both descriptors of request 2500
    failed = np.zeros(n, bool)
    failed[[7, 1001, 5000, 5001]] = True
    return bad, failed


def _drop(a, n, nq, keep):
    idx = np.nonzero(keep[:n])[0]
    off = a["stem_off"]
    stems = [a["stem_bytes"][off[i]:off[i + 1]] for i in idx]
    o = np.zeros(idx.size + 1, np.uint32)
    o[1:] = np.cumsum([s.size for s in stems])
    out = {"stem_bytes": np.concatenate(stems), "stem_off": o, "now": a["now"]}
    for k in ("req_idx", "unit", "flags", "limit", "hits", "rule_id"):
        out[k] = a[k][idx]
    return out, idx.size, nq


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_loopback_isolation(lc):
    """Per-descriptor statuses across ranks: the bad descriptors fail alone
    wherever their owners are; everything else equals the oracle over the
    batch without them."""
    cfg = (0.8, lc, False)
    (a, n, nq, nr), = _c2_batches(31, requests=4_000, batches=1)
    bad, failed = _with_bad(a, n, nq)
    out = run_world(3, [(bad, n, nq, nr)], cfg, isolate=(0, 1, 2), slices=lambda k: [0, 1_000, 2_600, 4_000])
    st = np.concatenate([out[r][1][0][1]["status"] for r in range(3)])
    code = np.concatenate([out[r][1][0][1]["code"] for r in range(3)])
    assert st[7] == abi.RL_E_INVALID and st[1001] == abi.RL_E_INVALID
    assert st[5000] == abi.RL_E_TIME and st[5001] == abi.RL_E_TIME
    assert (st[~failed] == 0).all() and (code[failed] == 0).all()
    co = COracle(*cfg)
    o = co.do_limit(*_drop(bad, n, nq, ~failed), nr)
    co.close()
    for f in ("code", "limit_remaining", "reset_s"):
        got = np.concatenate([out[r][1][0][1][f] for r in range(3)])
        assert np.array_equal(got[~failed], o[f]), f
    tot = sum(out[r][1][0][1]["stats"].astype(np.uint64) for r in range(3))
    assert np.array_equal(tot, o["stats"])


def test_gpu_loopback_isolation_requested_by_one_rank():
    """Only rank 0 passes out.status: owners still answer per descriptor (the
    isolate flag travels with the counts), so rank 1's bad descriptor fails
    rank 1's batch at synchronize while rank 0's answers stay exact."""
    cfg = (0.8, False, False)
    (a, n, nq, nr), = _c2_batches(33, requests=4_000, batches=1)
    bad = {k: v.copy() for k, v in a.items()}
    bad["unit"][5001] = 9  # request 2500: rank 1's slice
    out = run_world(2, [(bad, n, nq, nr)], cfg, isolate=(0,), slices=lambda k: [0, 2_000, 4_000])
    assert out[0][0] == "ok" and (out[0][1][0][1]["status"] == 0).all()
    assert out[1][0] == "err" and "RL_E_INVALID" in out[1][1]
    keep = np.ones(n, bool)
    keep[5001] = False
    co = COracle(*cfg)
    o = co.do_limit(*_drop(bad, n, nq, keep), nr)
    co.close()
    for f in ("code", "limit_remaining", "reset_s"):
        assert np.array_equal(out[0][1][0][1][f], o[f][:4_000]), f


def test_gpu_loopback_rejected_slice_fails_alone():
    """A slice larger than max_batch is rejected on its rank's host: that rank
    still takes part in every exchange (zero counts) and its batch fails at
    synchronize; no rank hangs, and the other ranks' answers equal the oracle
    over the node batch without the rejected slice. The next batches run
    normally on every rank."""
    cfg = (0.8, True, False)
    batches = _c2_batches(41, requests=3_000, batches=3)
    cuts = lambda k: [0, 1_000, 2_000, 3_000] if k != 1 else [0, 200, 2_800, 3_000]  # rank 1: 5200 > 4096
    out = run_world(3, batches, cfg, max_batch=1 << 12, slices=cuts)
    assert out[0][0] == "ok" and out[2][0] == "ok", (out[0], out[2])
    assert out[1][0] == "err" and "RL_E_CAPACITY" in out[1][1], out[1]
    co = COracle(*cfg)
    for k, (a, n, nq, nr) in enumerate(batches):
        c = cuts(k)
        if k == 1:  # the node batch without rank 1's slice
            keep = np.ones(n, bool)
            keep[2 * c[1]:2 * c[2]] = False
            exp = co.do_limit(*_drop(a, n, nq, keep), nr)
            got = {f: np.concatenate([out[0][1][k][1][f], out[2][1][k][1][f]]) for f in ("code", "reset_s",
                                                                                           "limit_remaining")}
            for f in got:
                assert np.array_equal(got[f], exp[f]), (k, f)
            assert np.array_equal(out[0][1][k][1]["stats"] + out[2][1][k][1]["stats"], exp["stats"])
        else:
            exp = co.do_limit(a, n, nq, nr)
            assert np.array_equal(out[0][1][k][1]["code"], exp["code"][:2 * c[1]]), k
    co.close()


def test_gpu_loopback_ranks_with_different_n_rules():
    """Ranks may pass different n_rules: owners keep per-source stats with the
    largest as stride, each rank gets its own rules' deltas."""
    cfg = (0.8, False, False)
    batches = _c2_batches(51, requests=3_000, batches=2)
    out = run_world(3, batches, cfg, n_rules_of=lambda r, k: 2 + 3 * r)
    co = COracle(*cfg)
    for k, (a, n, nq, nr) in enumerate(batches):
        exp = co.do_limit(a, n, nq, nr)
        tot = np.zeros(2 * abi.RL_NUM_STATS, np.uint64)
        for r in range(3):
            s = out[r][1][k][1]["stats"]
            assert s.size == (2 + 3 * r) * abi.RL_NUM_STATS and not s[2 * abi.RL_NUM_STATS:].any()
            tot += s[:2 * abi.RL_NUM_STATS]
        assert np.array_equal(tot, exp["stats"]), k
    co.close()


def test_gpu_loopback_sweep_and_table_info_are_collective():
    """rl_sweep / rl_table_info_get on a routed ctx complete the pending batch
    first: the live keys summed over ranks equal the oracle's after the last
    batch, and a sweep one day later evicts them all."""
    cfg = (0.8, False, False)
    batches = _c2_batches(61, requests=2_000, batches=2)
    info = {}

    def after(r, be):
        info[r] = (be.table_info()["live_slots"], be.sweep(W.NOW0 + 2 * 86_400), be.table_info()["live_slots"])

    out = run_world(2, batches, cfg, after=after)
    _check(out, batches, cfg, 2)
    keys = set()  # the table keeps one slot per (stem, unit)
    for a, n, nq, nr in batches:
        off = a["stem_off"]
        keys |= {(a["stem_bytes"][off[i]:off[i + 1]].tobytes(), int(a["unit"][i])) for i in range(n)}
    live = sum(info[r][0] for r in range(2))
    assert live == len(keys), (live, len(keys))
    assert sum(info[r][1] for r in range(2)) == live and all(info[r][2] == 0 for r in range(2))


def test_gpu_loopback_sweep_floor_is_the_least_over_ranks():
    """A routed rl_sweep applies one floor on every rank, the least `now` the
    ranks passed: rank 0 sweeps at NOW0 + 3 and rank 1 at NOW0 - 100, so the
    batches at NOW0 .. NOW0 + 2 that rank 1 sends to owner 0 are answered (a
    floor of rank 0's own would refuse them with RL_E_TIME); a third rank
    passing an out-of-range time fails its own sweep and does not vote."""
    cfg = (0.8, False, False)
    batches = _c2_batches(71, requests=2_000, batches=3)
    swept = {}

    def before(r, be):
        t = {0: W.NOW0 + 3, 1: W.NOW0 - 100, 2: -1}[r]
        try:
            swept[r] = be.sweep(t)
        except RedisError as e:
            swept[r] = e.status

    out = run_world(3, batches, cfg, before=before)
    assert swept[0] == 0 and swept[1] == 0 and swept[2] == abi.RL_E_TIME, swept
    for r in range(3):
        assert out[r][0] == "ok", out[r][1]
    _check(out, batches, cfg, 3)


def test_gpu_loopback_missing_peer_times_out(monkeypatch):
    """A rank whose peer never calls fails with RL_E_COMM after
    RL_LOOPBACK_TIMEOUT_S instead of waiting forever."""
    import torch
    from ratelimit_amd.sharded import LibRouter, loopback_id
    monkeypatch.setenv("RL_LOOPBACK_TIMEOUT_S", "3")
    uid = loopback_id()
    bes = [Backend(0.8, False, table_slots=1 << 16, max_batch=1 << 12, max_rules=16, device=0, hash_seed=SEED)
           for _ in range(2)]
    rr = [LibRouter(be, 2, r, uid) for r, be in enumerate(bes)]
    (a, n, nq, nr), = _c2_batches(71, requests=500, batches=1)
    dev = torch.device("cuda", 0)
    dev_in = _dev(a, dev)
    dev_out = {"code": torch.zeros(n, dtype=torch.uint8, device=dev),
               "limit_remaining": torch.zeros(n, dtype=torch.int32, device=dev),
               "reset_s": torch.zeros(n, dtype=torch.int32, device=dev)}
    with pytest.raises(RedisError, match="RL_E_COMM"):
        rr[0].submit(dev_in, n, nq, nr, dev_out)  # rank 1 never arrives
    with pytest.raises(RedisError, match="RL_E_COMM"):
        rr[0].finish()  # the router stays failed
    for be in bes:
        be.close()


@pytest.mark.parametrize("world,lc", [(2, True), (3, False)])
def test_gpu_loopback_prefixed_host_batches_go_rules(world, lc):
    """One process per GPU through the Go adapter's own entry point: every
    rank packs ITS requests (an uneven, sometimes empty slice of each node
    batch) with the Go batcher's rules into a pinned prefix-shared batch and
    submits it with rl_do_limit_prefixed_async on its routed ctx (collective,
    as the batcher's tick); results in pinned host memory after the collective
    rl_synchronize. Rank-order concatenation == the C oracle over the node
    batch, stats summed over ranks; a rank whose batch is malformed (bad tile
    index) takes part with no records and fails alone at rl_synchronize."""
    import os
    from ratelimit_amd.limiter import PinnedArena
    from ratelimit_amd.packing import go_prefixed_batch, go_statuses
    from ratelimit_amd.sharded import LibRouter, loopback_id
    os.environ.setdefault("RL_LOOPBACK_TIMEOUT_S", "30")
    cfg = (0.8, lc, False)
    calls = streams.random_stream(31 + world, n_calls=900, zipf=True, p_nil=0.15)
    per = 150
    node = [calls[k:k + per] for k in range(0, len(calls), per)]
    uid = loopback_id()
    bes = [Backend(*cfg, table_slots=1 << 18, max_batch=1 << 15, max_rules=256, device=0, hash_seed=SEED)
           for _ in range(world)]
    routers = [LibRouter(be, world, r, uid) for r, be in enumerate(bes)]
    interner = RuleInterner()  # (one rule-id space for the node, as the config's)
    for req, lims, _ in calls:
        for l in lims:
            if l is not None:
                interner.intern(l.stats.key)
    nr = len(interner.keys)
    out = [None] * world
    bad_rank, bad_batch = world - 1, 2

    def body(r):
        arena = PinnedArena()
        try:
            res = []
            for k, part in enumerate(node):
                cuts = _split_points(len(part), world, k)
                mine = part[cuts[r]:cuts[r + 1]]
                pb, where = go_prefixed_batch(mine, "", interner, n_rules=nr,
                                              alloc=lambda nb: arena.array(nb, np.uint8))
                if r == bad_rank and k == bad_batch and pb.n_requests:
                    ix = np.frombuffer(pb.buf, np.uint32, count=4, offset=pb.offsets["index"])
                    ix[0] = 7  # the index no longer starts at zero: rejected at the call
                o = {kk: arena.like(v) for kk, v in pb.alloc_result(reset=True).items()}
                rc = bes[r].do_limit_prefixed_async(pb, o)
                res.append((mine, where, o, rc, pb))
            err = None
            try:
                bes[r].synchronize()
            except RedisError as e:
                err = str(e)
            out[r] = ("ok", res, err)
        except Exception:
            out[r] = ("exc", traceback.format_exc(), None)
            try:
                bes[r].synchronize()
            except Exception:
                pass
        finally:
            out[r] = out[r] + (arena,)

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=90)
    assert not any(t.is_alive() for t in ts), "a loopback rank hung"
    try:
        for r in range(world):
            assert out[r][0] == "ok", out[r][1]
        # the malformed rank failed alone, at rl_synchronize
        assert out[bad_rank][2] is not None and "index" in out[bad_rank][2]
        for r in range(world - 1):
            assert out[r][2] is None, out[r][2]
        co = COracle(*cfg)
        for k, part in enumerate(node):
            cuts = _split_points(len(part), world, k)
            keep = [c for r in range(world) for c in (part[cuts[r]:cuts[r + 1]]
                                                       if not (r == bad_rank and k == bad_batch) else [])]
            pk = pack_calls(keep, "", interner, n_rules=nr)
            exp = co.do_limit(pk.arrays, pk.n, pk.n_requests, pk.n_rules)
            got_code, got_rem, got_rst = [], [], []
            tot = np.zeros(nr * abi.RL_NUM_STATS, np.uint64)
            for r in range(world):
                if r == bad_rank and k == bad_batch:
                    continue
                mine, where, o, _, pb = out[r][1][k]
                got_code.append(o["code"][:pb.n])
                got_rem.append(o["limit_remaining"][:pb.n])
                got_rst.append(o["reset_s"][:pb.n])
                tot += o["stats"][:nr * abi.RL_NUM_STATS].astype(np.uint64)
            for f, g in (("code", got_code), ("limit_remaining", got_rem), ("reset_s", got_rst)):
                g = np.concatenate(g) if g else np.zeros(0)
                assert np.array_equal(g, exp[f][:pk.n]), (k, f)
            assert np.array_equal(tot, exp["stats"]), k
        co.close()
    finally:
        for r in range(world):
            if out[r] is not None:
                out[r][-1].close()
        for be in bes:
            be.close()
