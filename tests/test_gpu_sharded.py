"""Multi-GPU routing through the C ABI (rl_route_*) on the GPU box.

World size 1 (RCCL) and 2 (two ranks sharing cuda:0, gloo exchange staged
through host memory; the 8-GPU RCCL run is the driver's) run
ShardedRateLimitCache with DeviceRouteOps: hash -> owner partition, wire
packing, owner-side unpack + the normal HIP pipeline, inverse routing. Results
of all ranks' slices in rank order must equal the C
oracle over the whole stream; the ranks' per-source stats sum to the oracle's.
The pipelined cases submit every batch before one finish() (two process
groups: forward and return).
"""
import os
import sys

import numpy as np
import pytest

from oracle.c_oracle import COracle
from ratelimit_amd import abi, workloads as W
from ratelimit_amd.packing import RuleInterner, pack_calls, slice_requests
import streams
from test_sharded_cpu import _free_port, _split_points

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu


def _batches(kind, seed):
    if kind == "random":
        calls = streams.random_stream(seed, n_calls=480, zipf=True)
        interner = RuleInterner()
        pbs = [pack_calls(calls[k:k + 60], "", interner) for k in range(0, len(calls), 60)]
        nr = max(len(interner.keys), 1)
        return [(pb.arrays, pb.n, pb.n_requests, nr) for pb in pbs]
    return list(W.c2_stream(seed=seed, n_tenants=20_000, requests_per_batch=6_000, batches=4))


def _worker(rank, world, port, backend, batches, cfg, q, pipelined=False, impl="python", max_batch=1 << 15):
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ratelimit_amd.limiter import Backend
    from ratelimit_amd.sharded import DeviceRouteOps, Exchange, RcclRouter, ShardedRateLimitCache
    try:
        dist.init_process_group(backend, rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        be = Backend(*cfg, table_slots=1 << 18, max_batch=max_batch, max_rules=64, device=0, hash_seed=0x5EED)
        if impl == "rccl":  # the routed step inside the library (rl_comm.hip)
            rr = RcclRouter(be)
        else:
            rx = Exchange(dist.new_group(backend=backend)) if pipelined else None
            sc = ShardedRateLimitCache(DeviceRouteOps(be), Exchange(), max_batch=1 << 15, max_stem_bytes=1 << 21,
                                       device=dev, ret_exchange=rx)
        res = []
        pending = []
        for k, (arrays, n, nq, n_rules) in enumerate(batches):
            cuts = _split_points(nq, world, k)
            sub, sn, snq = slice_requests(arrays, n, nq, cuts[rank], cuts[rank + 1])
            dev_in = {key: torch.from_numpy(np.ascontiguousarray(v).view(
                {np.dtype(np.uint32): np.int32}.get(v.dtype, v.dtype))).to(dev) for key, v in sub.items()}
            dev_out = {"code": torch.zeros(max(sn, 1), dtype=torch.uint8, device=dev),
                       "limit_remaining": torch.zeros(max(sn, 1), dtype=torch.int32, device=dev),
                       "reset_s": torch.zeros(max(sn, 1), dtype=torch.int32, device=dev)}
            if impl == "rccl":
                dev_out["stats"] = torch.zeros(n_rules * abi.RL_NUM_STATS, dtype=torch.int64, device=dev)
                rr.submit(dev_in, sn, snq, n_rules, dev_out)
                if not pipelined:
                    rr.finish()
                pending.append((sn, dev_out, dev_out["stats"]))
                continue
            if pipelined:
                pending.append((sn, dev_out, sc.submit(dev_in, sn, snq, n_rules, dev_out)))
                continue
            stats = sc.do_limit(dev_in, sn, snq, n_rules, dev_out)
            res.append((dev_out["code"][:sn].cpu().numpy(), dev_out["limit_remaining"][:sn].cpu().numpy().view(np.uint32),
                        dev_out["reset_s"][:sn].cpu().numpy().view(np.uint32), stats.cpu().numpy().view(np.uint64)))
        if impl == "rccl":
            rr.finish()
            for sn, dev_out, stats in pending:
                res.append((dev_out["code"][:sn].cpu().numpy(),
                            dev_out["limit_remaining"][:sn].cpu().numpy().view(np.uint32),
                            dev_out["reset_s"][:sn].cpu().numpy().view(np.uint32), stats.cpu().numpy().view(np.uint64)))
        elif pipelined:
            sc.finish()
            for sn, dev_out, stats in pending:
                res.append((dev_out["code"][:sn].cpu().numpy(),
                            dev_out["limit_remaining"][:sn].cpu().numpy().view(np.uint32),
                            dev_out["reset_s"][:sn].cpu().numpy().view(np.uint32), stats.cpu().numpy().view(np.uint64)))
        be.close()
        q.put((rank, res, None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _run(world, backend, batches, cfg, pipelined=False, impl="python", max_batch=1 << 15):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, backend, batches, cfg, q, pipelined, impl, max_batch)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=100)
            assert err is None, err
            out[rank] = res
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.parametrize("world,backend,kind,local_cache,pipelined", [
    (1, "nccl", "random", True, False), (2, "gloo", "random", True, False), (2, "gloo", "c2", False, False),
    (1, "nccl", "c2", False, True), (2, "gloo", "random", True, True)])
def test_gpu_sharded_matches_oracle(world, backend, kind, local_cache, pipelined):
    cfg = (0.8, local_cache, False)
    batches = _batches(kind, 7)
    out = _run(world, backend, batches, cfg, pipelined)
    co = COracle(*cfg)
    for k, (arrays, n, nq, n_rules) in enumerate(batches):
        exp = co.do_limit(arrays, n, nq, n_rules)
        for f, i in (("code", 0), ("limit_remaining", 1), ("reset_s", 2)):
            got = np.concatenate([out[r][k][i] for r in range(world)])
            assert np.array_equal(got, exp[f]), (k, f)
        tot = sum(out[r][k][3].astype(np.uint64) for r in range(world))  # per-source stats
        assert np.array_equal(tot, exp["stats"][:n_rules * abi.RL_NUM_STATS]), k


@pytest.mark.parametrize("kind,local_cache,pipelined,part,alias", [
    ("random", True, False, 0, True), ("random", True, False, 0, False), ("c2", False, True, 0, True),
    ("c2", False, True, 2500, False), ("c2", True, True, 2500, True)])
def test_gpu_rccl_router_matches_oracle(kind, local_cache, pipelined, part, alias, monkeypatch):
    """rl_comm_init + rl_do_limit_routed_async at world 1. alias: the owner
    reads the partition in place (the world-1 fast path); otherwise
    (RL_DEBUG_ROUTE_NOALIAS) the exchange path with its own-chunk device
    copies and offsets. part 2500 (RL_DEBUG_OWNER_PART) < the 12k-descriptor
    C2 batches: the owner answers a received batch in parts, cut at request
    boundaries, as it does when skew sends it more than max_batch records."""
    if part:
        monkeypatch.setenv("RL_DEBUG_OWNER_PART", str(part))
    if not alias:
        monkeypatch.setenv("RL_DEBUG_ROUTE_NOALIAS", "1")
    cfg = (0.8, local_cache, False)
    batches = _batches(kind, 11)
    out = _run(1, "nccl", batches, cfg, pipelined, impl="rccl")
    co = COracle(*cfg)
    for k, (arrays, n, nq, n_rules) in enumerate(batches):
        exp = co.do_limit(arrays, n, nq, n_rules)
        for f, i in (("code", 0), ("limit_remaining", 1), ("reset_s", 2)):
            bad = np.nonzero(out[0][k][i] != exp[f])[0]
            assert bad.size == 0, (k, f, bad.size, bad[:8].tolist(), out[0][k][i][bad[:8]].tolist(),
                                   exp[f][bad[:8]].tolist(), arrays["req_idx"][bad[:8]].tolist())
        assert np.array_equal(out[0][k][3], exp["stats"][:n_rules * abi.RL_NUM_STATS]), k


def test_gpu_rccl_router_many_large_batches_pipelined():
    """24 C2 batches of 120k descriptors submitted back to back before one
    finish(): partitions of consecutive batches run on different pipeline
    streams, concurrently (round 5), each on its slot's own scratch (a shared
    one gave a bench run garbage counts), and RL_ROUTED_LAG batches are
    pending at any time. Every answer and stat equals the C oracle's."""
    cfg = (0.8, True, False)
    batches = list(W.c2_stream(seed=23, n_tenants=50_000, requests_per_batch=60_000, batches=24))
    out = _run(1, "nccl", batches, cfg, True, impl="rccl", max_batch=1 << 18)
    co = COracle(*cfg)
    for k, (arrays, n, nq, n_rules) in enumerate(batches):
        exp = co.do_limit(arrays, n, nq, n_rules)
        for f, i in (("code", 0), ("limit_remaining", 1), ("reset_s", 2)):
            assert np.array_equal(out[0][k][i], exp[f]), (k, f)
        assert np.array_equal(out[0][k][3], exp["stats"][:n_rules * abi.RL_NUM_STATS]), k
