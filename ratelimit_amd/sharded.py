"""Hash-sharded multi-GPU DoLimit: one process and one rl_ctx per GPU.

SURVEY.md §8e. The reference scales by pointing many service replicas at
sharded Redis (cluster / sentinel pools, src/redis/driver_impl.go:66-142): a key
lives on exactly one shard. Here every GPU owns the keys whose stem hash maps
to it (rl_route.hip), and each batch makes one exchange:

1. each rank packs its slice of the node's batch by owner (rl_route_pack);
2. RCCL all_to_all_single: counts, then wire records and stem bytes;
3. the owner runs the normal pipeline over the chunks, concatenated in source
   rank order (= global arrival order, so the sequential-INCRBY contract holds
   across ranks) (rl_route_do_limit);
4. all_to_all_single returns the packed results (ret), which each source
   scatters back to arrival order (rl_route_scatter);
5. per-rule stats deltas are summed with all_reduce.

Rank r's slice precedes rank r+1's in the global order. An error on any rank
(validation, table full, ...) keeps the exchange well-formed (zero counts) and
raises RedisError on every rank after the step, like the reference's backend
failure path (driver_impl.go:60-64).
"""
import contextlib
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import abi
from ._lib import RedisError, check, lib

WIRE_BYTES = 32  # RL_WIRE_BYTES


class Exchange:
    """all_to_all / all_reduce over a process group. NCCL (= RCCL) groups move
    device tensors directly over xGMI; gloo groups (CPU tests, or several ranks
    sharing one GPU) stage through host memory."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.staged = dist.get_backend(group) != "nccl"

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None):
        if self.staged and out.is_cuda:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def all_reduce_sum(self, t: torch.Tensor):
        if self.staged and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)


class DeviceRouteOps:
    """The device halves of the exchange, through the C ABI (rl_route_*)."""

    def __init__(self, backend):
        if not backend.cfg.hash_seed:
            raise ValueError("a sharded table needs an explicit hash_seed shared by every shard (owner = stem hash)")
        self.be = backend
        self.device = torch.device("cuda", backend.cfg.device)
        # One explicit stream for the library kernels AND the collectives (a NULL
        # handle would mean the ctx's own non-blocking stream, unordered with RCCL).
        self.torch_stream = torch.cuda.Stream(self.device)

    def stream(self):
        return self.torch_stream.cuda_stream

    @contextlib.contextmanager
    def stream_ctx(self):
        caller = torch.cuda.current_stream(self.device)
        self.torch_stream.wait_stream(caller)
        with torch.cuda.stream(self.torch_stream):
            yield
        caller.wait_stream(self.torch_stream)

    def pack(self, dev_in, n, n_requests, n_rules, world, rank, send_rec, send_stem, perm):
        b = abi.make_batch_struct(dev_in, n, n_requests, n_rules)
        counts = np.zeros(2 * world, np.uint64)
        check(self.be.ctx, lib().rl_route_pack(self.be.ctx, b, world, rank, abi.ptr(send_rec), abi.ptr(send_stem),
                                               abi.ptr(perm), abi.ptr(counts), self.stream()))
        return counts.reshape(world, 2)

    def owner(self, n, recv_rec, recv_stem, stem_bytes, src_base, world, n_rules, ret, stats):
        base = np.ascontiguousarray(src_base, np.uint64)
        check(self.be.ctx, lib().rl_route_do_limit(self.be.ctx, n, abi.ptr(recv_rec), abi.ptr(recv_stem), stem_bytes,
                                                   abi.ptr(base), world, n_rules, abi.ptr(ret), abi.ptr(stats),
                                                   self.stream()))

    def scatter(self, n, perm, back, dev_out):
        r = abi.make_result_struct({"stats": None, **dev_out})
        check(self.be.ctx, lib().rl_route_scatter(self.be.ctx, n, abi.ptr(perm), abi.ptr(back), r, self.stream()))

    def synchronize(self):
        self.be.synchronize()


class ShardedRateLimitCache:
    """DoLimit over a hash-sharded table spanning every rank of `exchange`.

    Each call takes this rank's slice of the node batch as device arrays (the
    rl_batch layout, torch tensors) and fills dev_out in arrival order. The
    returned stats tensor (int64, n_rules x RL_NUM_STATS) holds the deltas of
    the WHOLE node batch (all ranks), identical on every rank.
    """

    def __init__(self, ops, exchange: Exchange, max_batch: int, max_stem_bytes: int, device: torch.device,
                 max_recv: Optional[int] = None, max_recv_stem: Optional[int] = None):
        self.ops = ops
        self.ex = exchange
        self.device = device
        self.max_batch = max_batch
        self.max_recv = max_recv or max_batch
        self.max_recv_stem = max_recv_stem or max_stem_bytes
        u8 = dict(dtype=torch.uint8, device=device)
        self.send_rec = torch.empty(max_batch * WIRE_BYTES, **u8)
        self.send_stem = torch.empty(max_stem_bytes + 4, **u8)
        self.perm = torch.empty(max_batch, dtype=torch.int32, device=device)
        self.recv_rec = torch.empty(self.max_recv * WIRE_BYTES, **u8)
        self.recv_stem = torch.empty(self.max_recv_stem + 4, **u8)
        self.ret = torch.empty(self.max_recv, dtype=torch.int64, device=device)
        self.back = torch.empty(max_batch, dtype=torch.int64, device=device)
        self.last_recv = 0

    def do_limit(self, dev_in: dict, n: int, n_requests: int, n_rules: int, dev_out: dict) -> torch.Tensor:
        ctx = getattr(self.ops, "stream_ctx", contextlib.nullcontext)
        with ctx():
            return self._do_limit(dev_in, n, n_requests, n_rules, dev_out)

    def _do_limit(self, dev_in, n, n_requests, n_rules, dev_out):
        world, rank = self.ex.world, self.ex.rank
        err: Optional[Exception] = None
        if n > self.max_batch:
            raise RedisError("gpu: batch exceeds max_batch [RL_E_CAPACITY]")
        # 1. pack by owner
        try:
            counts = self.ops.pack(dev_in, n, n_requests, n_rules, world, rank, self.send_rec, self.send_stem,
                                   self.perm)
        except RedisError as e:
            err, counts = e, np.zeros((world, 2), np.uint64)
        # 2. exchange counts, then records and stems
        cs = torch.from_numpy(counts.astype(np.int64).reshape(-1)).to(self.device)
        cr = torch.empty_like(cs)
        self.ex.all_to_all(cr, cs)
        rc = cr.cpu().numpy().reshape(world, 2)
        n_recv, stem_recv = int(rc[:, 0].sum()), int(rc[:, 1].sum())
        if n_recv > self.max_recv or stem_recv > self.max_recv_stem:
            # every rank computes the same totals for its own receive side; an
            # overflowing owner still takes part in the exchange (zero-sized) below
            err = err or RedisError("gpu: routed batch exceeds the owner's capacity [RL_E_CAPACITY]")
        send_n = [int(x) for x in counts[:, 0]]
        send_b = [int(x) for x in counts[:, 1]]
        recv_n = [int(x) for x in rc[:, 0]]
        recv_b = [int(x) for x in rc[:, 1]]
        self.ex.all_to_all(self.recv_rec[:n_recv * WIRE_BYTES] if n_recv <= self.max_recv else
                           torch.empty(n_recv * WIRE_BYTES, dtype=torch.uint8, device=self.device),
                           self.send_rec[:sum(send_n) * WIRE_BYTES],
                           [x * WIRE_BYTES for x in recv_n], [x * WIRE_BYTES for x in send_n])
        self.ex.all_to_all(self.recv_stem[:stem_recv] if stem_recv <= self.max_recv_stem else
                           torch.empty(stem_recv, dtype=torch.uint8, device=self.device),
                           self.send_stem[:sum(send_b)], recv_b, send_b)
        # 3. owner pipeline over the global-order concatenation
        src_base = np.zeros(world, np.uint64)
        src_base[1:] = np.cumsum(rc[:-1, 1])
        stats = torch.zeros(n_rules * abi.RL_NUM_STATS + 1, dtype=torch.int64, device=self.device)
        ret = self.ret[:n_recv] if n_recv <= self.max_recv else torch.zeros(n_recv, dtype=torch.int64,
                                                                            device=self.device)
        if err is None:
            try:
                self.ops.owner(n_recv, self.recv_rec, self.recv_stem, stem_recv, src_base, world, n_rules, ret,
                               stats)
            except RedisError as e:
                err = e
        self.last_recv = n_recv
        # 4. results back to their sources, then to arrival order
        self.ex.all_to_all(self.back[:sum(send_n)], ret, send_n, recv_n)
        if err is None:
            try:
                self.ops.scatter(n, self.perm, self.back, dev_out)
                self.ops.synchronize()
            except RedisError as e:
                err = e
        # 5. node-wide stats and error agreement
        if err is not None:
            stats.zero_()
            stats[-1] = 1
        self.ex.all_reduce_sum(stats)
        if err is not None:
            raise err
        if int(stats[-1].item()):
            raise RedisError("gpu: a peer shard failed this batch [RL_E_COMM]")
        return stats[:-1]
