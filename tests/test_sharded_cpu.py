"""Multi-rank exchange protocol of ratelimit_amd.sharded over gloo (CPU).

World sizes 2 and 3 run ShardedRateLimitCache with the CPU stand-in ops
(tests/route_cpu.py: numpy packing + the C oracle as each owner's table). The
per-descriptor results of every rank's slice, concatenated in rank order, and
the sum of the ranks' per-source stats must equal one sequential oracle over the whole batch
sequence: the routing preserves the global arrival order per key.
"""
import os
import socket
import sys

import numpy as np
import pytest

from oracle.c_oracle import COracle
from ratelimit_amd import abi
from ratelimit_amd.packing import RuleInterner, pack_calls, slice_requests
import streams

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    """A bindable port below the ephemeral range: an OS-assigned port could be
    handed to another socket (RCCL's bootstrap binds ephemeral ones) between
    this probe and the rendezvous store's bind."""
    import random
    for _ in range(200):
        p = random.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port")


def _batches(seed, n_batches=6, calls_per_batch=40, local_cache=False):
    calls = streams.random_stream(seed, n_calls=n_batches * calls_per_batch, zipf=True)
    interner = RuleInterner()
    out = []
    pbs = [pack_calls(calls[k:k + calls_per_batch], "", interner) for k in range(0, len(calls), calls_per_batch)]
    n_rules = max(len(interner.keys), 1)
    for pb in pbs:
        out.append((pb.arrays, pb.n, pb.n_requests, n_rules))
    return out


def _split_points(nq, world, k):
    # uneven, sometimes empty slices
    cuts = sorted({0, nq} | {int(x) for x in np.random.default_rng(k).integers(0, nq + 1, world - 1)})
    while len(cuts) < world + 1:
        cuts.insert(1, cuts[0])
    return cuts


def _worker(rank, world, port, batches, cfg, q, poison_rank=-1, pipelined=False):
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ratelimit_amd.sharded import Exchange, ShardedRateLimitCache
    from route_cpu import CpuRouteOps
    from ratelimit_amd._lib import RedisError
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ops = CpuRouteOps(*cfg)
        rx = Exchange(dist.new_group(backend="gloo")) if pipelined else None
        sc = ShardedRateLimitCache(ops, Exchange(), max_batch=4096, max_stem_bytes=1 << 18,
                                   device=torch.device("cpu"), ret_exchange=rx)
        res = []
        pending = []
        for k, (arrays, n, nq, n_rules) in enumerate(batches):
            cuts = _split_points(nq, world, k)
            sub, sn, snq = slice_requests(arrays, n, nq, cuts[rank], cuts[rank + 1])
            if rank == poison_rank and sn:
                sub["unit"] = sub["unit"].copy()
                sub["unit"][0] = 9
            dev_in = {key: torch.from_numpy(np.ascontiguousarray(v).view(
                {np.dtype(np.uint32): np.int32}.get(v.dtype, v.dtype))) for key, v in sub.items()}
            dev_out = {"code": torch.zeros(max(sn, 1), dtype=torch.uint8),
                       "limit_remaining": torch.zeros(max(sn, 1), dtype=torch.int32),
                       "reset_s": torch.zeros(max(sn, 1), dtype=torch.int32)}
            if pipelined:  # submit everything, one finish at the end
                pending.append((sn, dev_out, sc.submit(dev_in, sn, snq, n_rules, dev_out)))
                continue
            try:
                stats = sc.do_limit(dev_in, sn, snq, n_rules, dev_out)
            except RedisError as e:
                res.append(("RedisError", str(e)))
                continue
            res.append((dev_out["code"][:sn].numpy().copy(),
                        dev_out["limit_remaining"][:sn].numpy().view(np.uint32).copy(),
                        dev_out["reset_s"][:sn].numpy().view(np.uint32).copy(),
                        stats.numpy().view(np.uint64).copy()))
        if pipelined:
            sc.finish()
            for sn, dev_out, stats in pending:
                res.append((dev_out["code"][:sn].numpy().copy(),
                            dev_out["limit_remaining"][:sn].numpy().view(np.uint32).copy(),
                            dev_out["reset_s"][:sn].numpy().view(np.uint32).copy(),
                            stats.numpy().view(np.uint64).copy()))
        q.put((rank, res, None))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _run(world, batches, cfg, poison_rank=-1, pipelined=False):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, batches, cfg, q, poison_rank, pipelined)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=240)
        assert err is None, err
        out[rank] = res
    for p in ps:
        p.join(timeout=60)
    return out


@pytest.mark.parametrize("world,seed,local_cache,per_second,pipelined", [
    (2, 1, False, False, False), (2, 2, True, False, False), (3, 3, True, True, False), (3, 4, True, False, True)])
def test_sharded_exchange_matches_sequential_oracle(world, seed, local_cache, per_second, pipelined):
    cfg = (0.8, local_cache, per_second)
    batches = _batches(seed, local_cache=local_cache)
    out = _run(world, batches, cfg, pipelined=pipelined)
    co = COracle(*cfg)
    for k, (arrays, n, nq, n_rules) in enumerate(batches):
        exp = co.do_limit(arrays, n, nq, n_rules)
        got_code = np.concatenate([out[r][k][0] for r in range(world)])
        got_rem = np.concatenate([out[r][k][1] for r in range(world)])
        got_reset = np.concatenate([out[r][k][2] for r in range(world)])
        assert np.array_equal(got_code, exp["code"]), k
        assert np.array_equal(got_rem, exp["limit_remaining"]), k
        assert np.array_equal(got_reset, exp["reset_s"]), k
        # per-source stats: each rank counts its own requests; the sum is the node's
        tot = sum(out[r][k][3].astype(np.uint64) for r in range(world))
        assert np.array_equal(tot, exp["stats"][:n_rules * abi.RL_NUM_STATS]), k


def test_sharded_error_on_one_rank_fails_the_batch_everywhere():
    batches = _batches(5, n_batches=2)
    out = _run(2, batches[:1], (0.8, False, False), poison_rank=1)
    for r in range(2):
        assert out[r][0][0] == "RedisError", out[r][0]
    assert "malformed" in out[1][0][1] and "peer shard" in out[0][0][1]
