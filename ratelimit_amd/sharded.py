"""Hash-sharded multi-GPU DoLimit: one process and one rl_ctx per GPU.

Two drivers of the same exchange:

* LibRouter / RcclRouter (production): the whole routed step inside the
  library (rl_comm_init + rl_do_limit_routed_async, rl_comm.hip): partition,
  RCCL send/recv over xGMI, owner pipeline, return, scatter, with one host
  wait per batch (its partition counts) and no Python on the per-batch path
  beyond one ctypes call. The same library router runs W ranks inside one
  process over its loopback transport (loopback_id(): threads, one Backend
  each, several on one GPU), which is how the multi-rank protocol is
  exercised on a one-GPU machine.
* ShardedRateLimitCache (below): the same protocol with the collectives issued
  from Python (torch.distributed all_to_all_single) around the device halves
  rl_route_pack / rl_route_do_limit / rl_route_scatter. It runs over gloo as
  well (CPU tests with tests/route_cpu.py, several ranks sharing one GPU),
  which RCCL cannot (one rank per device).

SURVEY.md §8e. The reference scales by pointing many service replicas at
sharded Redis (cluster / sentinel pools, src/redis/driver_impl.go:66-142): a key
lives on exactly one shard. Here every GPU owns the keys whose stem hash maps
to it (rl_route.hip), and each batch makes one exchange:

1. each rank packs its slice of the node's batch by owner (rl_route_pack);
2. all_to_all_single: counts, then wire records and stem bytes ("forward"
   process group, forward stream);
3. the owner runs the normal pipeline over the chunks, concatenated in source
   rank order (= global arrival order, so the sequential-INCRBY contract holds
   across ranks) (rl_route_do_limit), its stats attributed per source rank;
4. all_to_all_single returns the packed results and each source's stats block
   ("return" process group, return stream), and each source scatters the
   results back to arrival order (rl_route_scatter).

Pipelining (`submit` / `finish`): the forward side of batch t+1 runs while the
owner pipeline and the return side of batch t are still on the GPU. The only
host wait per batch is the 2 x world counts the split sizes of step 2 need
(all_to_all_single takes host split sizes); it waits for rl_route_pack of that
batch only. `depth` slots of receive / result buffers rotate; a slot is
reused once the owner batch that read it is done (HIP events, no host wait).

Stats are per source, like a replica's own Prometheus counters in the
reference (ratelimit.go stats scope per process): the tensor returned for a
batch holds the deltas of THIS rank's requests; the sum over ranks is the
node-wide total.

Rank r's slice precedes rank r+1's in the global order. An error on any rank
(validation, table full, ...) keeps the exchange well-formed (zero counts) and
raises RedisError on every rank at `finish`, like the reference's backend
failure path (driver_impl.go:60-64); `do_limit` = submit + finish.
"""
import collections
import contextlib
import time
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import abi
from ._lib import RedisError, check, lib

WIRE_BYTES = 32  # RL_WIRE_BYTES


def loopback_id() -> np.ndarray:
    """The id of a new in-process loopback world (rl_comm_loopback_id): its
    ranks are threads of this process, one Backend each (they may share one
    GPU), exchanging by device copies with the RCCL router's protocol."""
    uid = np.zeros(abi.RL_COMM_ID_BYTES, np.uint8)
    check(None, lib().rl_comm_loopback_id(abi.ptr(uid)))
    return uid


class LibRouter:
    """DoLimit over a table hash-sharded across `world` ranks, routed by the
    library (rl_comm_init + rl_do_limit_routed_async, rl_comm.hip).

    Every rank builds one Backend (hash_seed shared by all ranks, max_rules >=
    world x n_rules), joins the world `uid` (RCCL: rl_comm_unique_id handed to
    every process; loopback: loopback_id(), ranks as threads), then calls
    submit() once per node batch with its slice (device tensors, the rl_batch /
    rl_result layout; a rank may pass n = 0). Results land in dev_out in
    arrival order; dev_out["stats"] (optional) receives the deltas of this
    rank's requests. A submit completes the previous batch (the library never
    waits for work it just issued); dev_out is final after finish(), which
    every rank calls together: it completes the last batch and raises
    RedisError if one failed on this rank. The library reads a batch's inputs
    until RL_ROUTED_INFLIGHT later submits have returned (its own chunk is read
    in place): submit holds them that long, and finish releases them. Output
    tensors must stay alive until finish.
    """

    def __init__(self, backend, world: int, rank: int, uid: np.ndarray):
        if not backend.cfg.hash_seed:
            raise ValueError("a sharded table needs an explicit hash_seed shared by every shard (owner = stem hash)")
        self.be = backend
        self.world, self.rank = world, rank
        uid = np.ascontiguousarray(uid, np.uint8)
        check(backend.ctx, lib().rl_comm_init(backend.ctx, world, rank, abi.ptr(uid)))
        self.device = torch.device("cuda", backend.cfg.device)
        # the batch's inputs are ordered through a stream of our own: torch's
        # default stream has the NULL handle, which the library reads as
        # "inputs complete at the call"
        self.stream = torch.cuda.Stream(self.device)
        self._held = collections.deque()  # the inputs of the batches the library may still read

    def submit(self, dev_in: dict, n: int, n_requests: int, n_rules: int, dev_out: dict):
        b = abi.make_batch_struct(dev_in, n, n_requests, n_rules)
        r = abi.make_result_struct(dev_out)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        check(self.be.ctx, lib().rl_do_limit_routed_async(self.be.ctx, b, r, self.stream.cuda_stream))
        self._held.append(dev_in)
        while len(self._held) > abi.RL_ROUTED_INFLIGHT:
            self._held.popleft()

    def finish(self):
        self.be.synchronize()
        self._held.clear()

    def do_limit(self, dev_in: dict, n: int, n_requests: int, n_rules: int, dev_out: dict):
        self.submit(dev_in, n, n_requests, n_rules, dev_out)
        self.finish()


class RcclRouter(LibRouter):
    """LibRouter over RCCL across every rank of a torch.distributed group (one
    process per GPU): rank 0's rl_comm_unique_id is broadcast to the others."""

    def __init__(self, backend, group=None):
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        uid = np.zeros(abi.RL_COMM_ID_BYTES, np.uint8)
        if rank == 0:
            check(None, lib().rl_comm_unique_id(abi.ptr(uid)))
        box = [uid.tobytes()]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        super().__init__(backend, world, rank, np.frombuffer(box[0], np.uint8).copy())


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
    """The device halves of the exchange, through the C ABI (rl_route_*), and
    the streams / events that pipeline them.

    Streams: `fwd` (pack + forward collectives), one `own[slot]` per buffer
    slot (the owner call: its inputs-ready point and the copy of the packed
    results), `ret` (return collectives + scatter). Events: `recv_free[slot]`
    (the owner batch that read slot's receive buffers is done) and
    `stats_free[slot]` (the return side read slot's result / stats buffers).
    """

    def __init__(self, backend, depth: int = 3):
        if not backend.cfg.hash_seed:
            raise ValueError("a sharded table needs an explicit hash_seed shared by every shard (owner = stem hash)")
        self.be = backend
        self.device = torch.device("cuda", backend.cfg.device)
        self.depth = depth
        self.fwd = torch.cuda.Stream(self.device)
        self.ret = torch.cuda.Stream(self.device)
        self.own = [torch.cuda.Stream(self.device) for _ in range(depth)]
        self.recv_free = [None] * depth
        self.stats_free = [None] * depth

    # -- stream phases -----------------------------------------------------
    @contextlib.contextmanager
    def phase(self, name: str, slot: int):
        if name == "fwd":
            st = self.fwd
        elif name == "own":
            st = self.own[slot]
            st.wait_stream(self.fwd)  # the received chunks
            if self.stats_free[slot] is not None:
                st.wait_event(self.stats_free[slot])  # the slot's previous results were sent back
        else:
            st = self.ret
            st.wait_stream(self.own[slot])
        with torch.cuda.stream(st):
            yield

    def begin(self, dev_in: dict, dev_out: dict):
        caller = torch.cuda.current_stream(self.device)
        self.fwd.wait_stream(caller)
        self.ret.wait_stream(caller)  # dev_out may still be read by the caller's earlier work
        for t in dev_in.values():
            t.record_stream(self.fwd)
        for t in dev_out.values():
            if t is not None:
                t.record_stream(self.ret)

    def before_pack(self, slot: int):
        # the partition rewrites slot's permutation: the scatter of the slot's
        # previous batch (return side) must have read it
        if self.stats_free[slot] is not None:
            self.fwd.wait_event(self.stats_free[slot])

    def before_payload(self, slot: int):
        if self.recv_free[slot] is not None:
            self.fwd.wait_event(self.recv_free[slot])

    def after_owner(self, slot: int):
        ev = torch.cuda.Event()
        ev.record(self.own[slot])  # own[slot] waited for the owner batch (b_done) before its copy
        self.recv_free[slot] = ev

    def after_return(self, slot: int):
        ev = torch.cuda.Event()
        ev.record(self.ret)
        self.stats_free[slot] = ev

    def join(self):
        torch.cuda.current_stream(self.device).wait_stream(self.ret)
        torch.cuda.current_stream(self.device).wait_stream(self.fwd)

    # -- library calls ------------------------------------------------------
    def pack(self, dev_in, n, n_requests, n_rules, world, rank, send_rec, send_stem, perm, counts):
        b = abi.make_batch_struct(dev_in, n, n_requests, n_rules)
        check(self.be.ctx, lib().rl_route_pack(self.be.ctx, b, world, rank, abi.ptr(send_rec), abi.ptr(send_stem),
                                               abi.ptr(perm), abi.ptr(counts), self.fwd.cuda_stream))

    def owner(self, n, recv_rec, recv_stem, stem_bytes, src_base, world, n_rules, ret, stats, isolate, slot):
        base = np.ascontiguousarray(src_base, np.uint64)
        check(self.be.ctx, lib().rl_route_do_limit(self.be.ctx, n, abi.ptr(recv_rec), abi.ptr(recv_stem), stem_bytes,
                                                   abi.ptr(base), world, n_rules, n_rules, abi.ptr(ret),
                                                   abi.ptr(stats), int(isolate), self.own[slot].cuda_stream))

    def scatter(self, n, perm, back, dev_out):
        r = abi.make_result_struct({"stats": None, **dev_out})
        check(self.be.ctx, lib().rl_route_scatter(self.be.ctx, n, abi.ptr(perm), abi.ptr(back), r,
                                                  self.ret.cuda_stream))

    def synchronize(self):
        self.fwd.synchronize()
        self.ret.synchronize()
        self.be.synchronize()


class _Slot:
    def __init__(self, max_recv, max_recv_stem, device):
        u8 = dict(dtype=torch.uint8, device=device)
        self.perm = None  # (allocated by the cache: sized by max_batch)
        self.recv_rec = torch.empty(max_recv * WIRE_BYTES, **u8)
        self.recv_stem = torch.empty(max_recv_stem + 4, **u8)
        self.ret = torch.empty(max_recv, dtype=torch.int64, device=device)
        self.stats = None


class ShardedRateLimitCache:
    """DoLimit over a hash-sharded table spanning every rank of `exchange`.

    Each call takes this rank's slice of the node batch as device arrays (the
    rl_batch layout, torch tensors) and fills dev_out (code, limit_remaining,
    reset_s, optional status) in arrival order. The stats of a batch (int64,
    n_rules x RL_NUM_STATS) are the deltas of this rank's requests.

    `ret_exchange` (a second process group over the same ranks) lets the
    return collectives of batch t run while the forward ones of batch t+1 do;
    with one group both directions share one communicator and serialise.
    """

    def __init__(self, ops, exchange: Exchange, max_batch: int, max_stem_bytes: int, device: torch.device,
                 max_recv: Optional[int] = None, max_recv_stem: Optional[int] = None,
                 ret_exchange: Optional[Exchange] = None):
        self.ops = ops
        self.ex = exchange
        self.rx = ret_exchange or exchange
        if self.rx.world != self.ex.world or self.rx.rank != self.ex.rank:
            raise ValueError("ret_exchange must span the same ranks as exchange")
        self.device = device
        self.max_batch = max_batch
        self.max_recv = max_recv or max_batch
        self.max_recv_stem = max_recv_stem or max_stem_bytes
        self.depth = getattr(ops, "depth", 1)
        u8 = dict(dtype=torch.uint8, device=device)
        self.send_rec = torch.empty(max_batch * WIRE_BYTES, **u8)
        self.send_stem = torch.empty(max_stem_bytes + 4, **u8)
        self.counts = torch.zeros(2 * self.ex.world, dtype=torch.int64, device=device)
        self.back = torch.empty(max_batch, dtype=torch.int64, device=device)
        self.slots = [_Slot(self.max_recv, self.max_recv_stem, device) for _ in range(self.depth)]
        for s in self.slots:
            s.perm = torch.empty(max_batch, dtype=torch.int32, device=device)
        self.t = 0
        self.last_recv = 0
        self.recv_log: List[int] = []
        self._err: Optional[Exception] = None
        # host seconds per phase of submit() (bench diagnostics)
        self.host_s = {"pack": 0.0, "counts_wait": 0.0, "payload": 0.0, "owner": 0.0, "return": 0.0}

    def _phase(self, name, slot):
        ph = getattr(self.ops, "phase", None)
        return ph(name, slot) if ph else contextlib.nullcontext()

    def _hook(self, name, *a):
        f = getattr(self.ops, name, None)
        if f:
            f(*a)

    def do_limit(self, dev_in: dict, n: int, n_requests: int, n_rules: int, dev_out: dict,
                 isolate: bool = False) -> torch.Tensor:
        stats = self.submit(dev_in, n, n_requests, n_rules, dev_out, isolate)
        self.finish()
        return stats

    def submit(self, dev_in: dict, n: int, n_requests: int, n_rules: int, dev_out: dict,
               isolate: bool = False) -> torch.Tensor:
        """Enqueue one batch; returns its stats tensor (valid after finish())."""
        world, rank = self.ex.world, self.ex.rank
        hs, t0 = self.host_s, time.perf_counter()
        slot = self.t % self.depth
        S = self.slots[slot]
        self.t += 1
        nst = n_rules * abi.RL_NUM_STATS
        self._hook("begin", dev_in, dev_out)
        self._hook("before_pack", slot)
        with self._phase("fwd", slot):
            # 1. pack by owner
            self.counts.zero_()
            try:
                if n > self.max_batch:
                    raise RedisError("gpu: batch exceeds max_batch [RL_E_CAPACITY]")
                self.ops.pack(dev_in, n, n_requests, n_rules, world, rank, self.send_rec, self.send_stem, S.perm,
                              self.counts)
            except RedisError as e:
                self._err = self._err or e
                self.counts.zero_()
            # 2. exchange counts (the one host wait), then records and stems
            cr = torch.empty_like(self.counts)
            self.ex.all_to_all(cr, self.counts)
            t1 = time.perf_counter()
            both = torch.cat([self.counts, cr]).cpu().numpy()
            t2 = time.perf_counter()
            sc, rc = both[:2 * world].reshape(world, 2), both[2 * world:].reshape(world, 2)
            n_recv, stem_recv = int(rc[:, 0].sum()), int(rc[:, 1].sum())
            fits = n_recv <= self.max_recv and stem_recv <= self.max_recv_stem
            if not fits:
                # every rank computes the totals of its own receive side; an
                # overflowing owner still takes part in the exchange below
                self._err = self._err or RedisError("gpu: routed batch exceeds the owner's capacity [RL_E_CAPACITY]")
            send_n, send_b = [int(x) for x in sc[:, 0]], [int(x) for x in sc[:, 1]]
            recv_n, recv_b = [int(x) for x in rc[:, 0]], [int(x) for x in rc[:, 1]]
            self._hook("before_payload", slot)
            u8 = dict(dtype=torch.uint8, device=self.device)
            self.ex.all_to_all(S.recv_rec[:n_recv * WIRE_BYTES] if fits else torch.empty(n_recv * WIRE_BYTES, **u8),
                               self.send_rec[:sum(send_n) * WIRE_BYTES],
                               [x * WIRE_BYTES for x in recv_n], [x * WIRE_BYTES for x in send_n])
            self.ex.all_to_all(S.recv_stem[:stem_recv] if fits else torch.empty(stem_recv, **u8),
                               self.send_stem[:sum(send_b)], recv_b, send_b)
        t3 = time.perf_counter()
        # 3. owner pipeline over the global-order concatenation
        src_base = np.zeros(world, np.uint64)
        src_base[1:] = np.cumsum(rc[:-1, 1])
        if S.stats is None or S.stats.numel() != world * nst:
            S.stats = torch.zeros(max(world * nst, 1), dtype=torch.int64, device=self.device)
        ret = S.ret[:n_recv] if fits else torch.zeros(n_recv, dtype=torch.int64, device=self.device)
        with self._phase("own", slot):
            if self._err is None:
                try:
                    self.ops.owner(n_recv, S.recv_rec, S.recv_stem, stem_recv, src_base, world, n_rules, ret,
                                   S.stats, isolate, slot)
                except RedisError as e:
                    self._err = e
            if self._err is not None:
                ret.zero_()
                S.stats.zero_()
        self._hook("after_owner", slot)
        t4 = time.perf_counter()
        self.last_recv = n_recv
        self.recv_log.append(n_recv)
        # 4. results and per-source stats back to their sources, then arrival order
        with self._phase("ret", slot):
            self.rx.all_to_all(self.back[:sum(send_n)], ret, send_n, recv_n)
            rs = torch.empty(world * nst, dtype=torch.int64, device=self.device)
            if nst:
                self.rx.all_to_all(rs, S.stats[:world * nst])
            stats = rs.view(world, nst).sum(0)
            if self._err is None:
                try:
                    self.ops.scatter(n, S.perm, self.back, dev_out)
                except RedisError as e:
                    self._err = e
        self._hook("after_return", slot)
        t5 = time.perf_counter()
        hs["pack"] += t1 - t0
        hs["counts_wait"] += t2 - t1
        hs["payload"] += t3 - t2
        hs["owner"] += t4 - t3
        hs["return"] += t5 - t4
        return stats

    def finish(self):
        """Wait for every submitted batch; raise RedisError on every rank if any
        rank failed one (the exchange stayed well-formed meanwhile)."""
        err, self._err = self._err, None
        try:
            self.ops.synchronize()
        except RedisError as e:
            err = err or e
        self._hook("join")
        flag = torch.tensor([1 if err is not None else 0], dtype=torch.int64,
                            device=self.device if not self.ex.staged else "cpu")
        self.ex.all_reduce_sum(flag)
        if err is not None:
            raise err
        if int(flag.item()):
            raise RedisError("gpu: a peer shard failed this batch [RL_E_COMM]")
