"""Host-side mirror of the reference's RateLimitCache interface over the C ABI.

``GpuRateLimitCache`` is what a user of the reference's
``limiter.RateLimitCache`` (src/limiter/cache.go:11-29) switches to:

    cache = GpuRateLimitCache(time_source, near_limit_ratio=0.8, local_cache=True,
                              cache_key_prefix="", per_second=False)
    statuses = cache.do_limit(ctx, request, limits)   # DoLimit
    cache.flush()                                     # Flush

Same argument meaning and error behaviour as
``redis.NewFixedRateLimitCacheImpl`` / ``fixedRateLimitCacheImpl.DoLimit``
(src/redis/fixed_cache_impl.go:33-125): nil limits answer {OK, nil, 0}; the
per-rule stats counters (limit.stats) are incremented; backend failures raise
``RedisError`` (the reference panics with redis.RedisError).  ``do_limit_batch``
is the batcher's entry point: many in-flight calls, one GPU launch sequence.
"""
import ctypes as C
import time
from typing import List, Optional, Sequence

import numpy as np

from . import abi
from ._lib import RedisError, check, lib, load
from .packing import PackedBatch, RuleInterner, pack_calls
from .types import OK, DescriptorStatus, Limit  # noqa: F401  (re-exported data model)

# rl_profile stages (include/ratelimit_hip.h RL_NUM_STAGES)
STAGES = ("prepare", "sort", "segment", "table", "finish")
PROFILE_FIELDS = STAGES + ("table_kernel",)  # + k_table's own run time (device clock)

__all__ = ["GpuRateLimitCache", "GpuRateLimitService", "RedisError", "TimeSource"]


class TimeSource:
    """utils.TimeSource (src/utils/utilities.go:9-12)."""

    def unix_now(self) -> int:
        return int(time.time())


class FixedTimeSource(TimeSource):
    def __init__(self, now: int):
        self.now = now

    def unix_now(self) -> int:
        return self.now


def _config(near_limit_ratio, local_cache, per_second, jitter, table_slots, max_batch, max_rules, device,
            arena_bytes, max_stem_bytes, hash_seed=0, debug_hash_bits=0, n_shards=1, shard_devices=None,
            history_entries=0):
    cfg = abi.RlConfig()
    cfg.history_entries = history_entries
    cfg.table_slots = table_slots
    cfg.arena_bytes = arena_bytes
    cfg.max_batch = max_batch
    cfg.max_requests = max_batch
    cfg.max_rules = max_rules
    cfg.max_stem_bytes = max_stem_bytes
    cfg.near_limit_ratio = near_limit_ratio
    cfg.local_cache_enabled = 1 if local_cache else 0
    cfg.per_second_split = 1 if per_second else 0
    cfg.device = device
    cfg.expiration_jitter_max_seconds = jitter
    cfg.hash_seed = hash_seed
    cfg.debug_hash_bits = debug_hash_bits
    cfg.n_shards = n_shards
    devs = list(shard_devices) if shard_devices is not None else [device] * n_shards
    if len(devs) != n_shards or n_shards > 16:
        raise ValueError("shard_devices must name n_shards (<= 16) devices")
    for j, d in enumerate(devs):
        cfg.shard_device[j] = d
    return cfg


class PinnedArena:
    """Page-locked host arrays from the library (rl_alloc_host): numpy views
    whose PCIe copies run asynchronously (rl_do_limit_host_async)."""

    def __init__(self):
        self.ptrs = []

    def array(self, n: int, dtype) -> np.ndarray:
        dt = np.dtype(dtype)
        nbytes = max(int(n), 1) * dt.itemsize
        p = lib().rl_alloc_host(nbytes)
        if not p:
            raise MemoryError("rl_alloc_host(%d) failed" % nbytes)
        self.ptrs.append(p)
        buf = (C.c_uint8 * nbytes).from_address(p)
        return np.frombuffer(buf, dtype=dt, count=max(int(n), 1))

    def like(self, a: np.ndarray) -> np.ndarray:
        out = self.array(a.size, a.dtype)
        out[:a.size] = a
        return out

    def close(self):
        for p in self.ptrs:
            lib().rl_free_host(p)
        self.ptrs = []


class Backend:
    """Owns one rl_ctx (one GPU's table)."""

    def __init__(self, near_limit_ratio=0.8, local_cache=False, per_second=False, jitter=0,
                 table_slots=1 << 20, max_batch=1 << 16, max_rules=1 << 12, device=0, arena_bytes=0,
                 max_stem_bytes=0, hash_seed=0, debug_hash_bits=0, n_shards=1, shard_devices=None, history_entries=0,
                 library=None):
        """n_shards > 1: one ctx hash-shards its table over shard_devices (default:
        all on `device`) and routes every batch between them (rl_config.n_shards).
        history_entries: 32-B history log entries (0 = table_slots; rl_config.history_entries).
        jitter: EXPIRATION_JITTER_MAX_SECONDS (the history horizon: older windows kept div + jitter s).
        library: a path to another build of the library (tests: the RL_LOG_TEAR build); default the product's."""
        L = self.L = lib() if library is None else load(library)
        err = C.create_string_buffer(512)
        self.cfg = _config(near_limit_ratio, local_cache, per_second, jitter, table_slots, max_batch, max_rules,
                           device, arena_bytes, max_stem_bytes, hash_seed, debug_hash_bits, n_shards, shard_devices,
                           history_entries)
        self.ctx = L.rl_create(C.byref(self.cfg), err, 512)
        if not self.ctx:
            raise RedisError(err.value.decode())

    def _check(self, rc):
        check(self.ctx, rc, self.L)

    def close(self):
        if getattr(self, "ctx", None):
            self.L.rl_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- raw packed-batch entry points
    def do_limit_packed(self, pb: PackedBatch, isolate: bool = False):
        """rl_do_limit. isolate: per-descriptor statuses (result "status"): a
        descriptor that cannot be answered fails alone instead of the batch."""
        out = pb.alloc_result(isolate)
        b = pb.batch_struct()
        r = abi.make_result_struct(out)
        self._check(self.L.rl_do_limit(self.ctx, C.byref(b), C.byref(r)))
        n, nr = pb.n, pb.n_rules
        res = {"code": out["code"][:n], "limit_remaining": out["limit_remaining"][:n],
               "reset_s": out["reset_s"][:n], "stats": out["stats"][:nr * abi.RL_NUM_STATS]}
        if isolate:
            res["status"] = out["status"][:n]
        return res

    def do_limit_arrays(self, arrays, n, n_requests, n_rules, isolate: bool = False):
        return self.do_limit_packed(PackedBatch(arrays, n, n_requests, n_rules), isolate)

    def do_limit_device(self, dev_in: dict, dev_out: dict, n, n_requests, n_rules, stream=None):
        """All arrays are torch CUDA tensors (device memory); asynchronous and
        pipelined; dev_out is read after synchronize(). `stream` (a hipStream_t
        handle; default: torch's current stream) orders the batch after the
        work producing its inputs. torch's default stream has the NULL handle,
        which the library cannot order against cheaply: under it, the inputs
        must be complete at the call."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream().cuda_stream
        b = abi.make_batch_struct(dev_in, n, n_requests, n_rules)
        r = abi.make_result_struct(dev_out)
        self._check(self.L.rl_do_limit_async(self.ctx, C.byref(b), C.byref(r),
                                                C.c_void_p(stream) if stream else None))

    def do_limit_structs(self, b, r, stream=None):
        """rl_do_limit_async with prebuilt rl_batch / rl_result structs (device
        arrays; the structs are read during the call only): what a C or Go
        caller does per batch. stream: a hipStream_t handle, or None (the
        inputs are complete at the call)."""
        self._check(self.L.rl_do_limit_async(self.ctx, C.byref(b), C.byref(r), C.c_void_p(stream) if stream else None))

    def do_limit_host_async(self, pb: PackedBatch, out: dict):
        """rl_do_limit_host_async: host arrays in (pb) and out (dict of numpy
        arrays: code, limit_remaining, reset_s, stats[, status]), nothing waited
        for; out is final after synchronize(). Both must stay alive and
        untouched until then; pinned arrays (PinnedArena) make the copies
        asynchronous."""
        b = pb.batch_struct()
        r = abi.make_result_struct(out)
        self._check(self.L.rl_do_limit_host_async(self.ctx, C.byref(b), C.byref(r)))
        return b, r  # (the structs the call read; kept by the caller with the arrays)

    def do_limit_compact_async(self, cb, out: dict):
        """rl_do_limit_compact_async: a CompactBatch (packing.compact_batch; its
        buffer pinned for an asynchronous copy) in, out as do_limit_host_async;
        final after synchronize()."""
        r = abi.make_result_struct(out)
        s = cb.struct()
        self._check(self.L.rl_do_limit_compact_async(self.ctx, C.byref(s), C.byref(r)))
        return s, r

    def batch_progress(self):
        """rl_batch_progress: (batches submitted, batches complete), never waits."""
        a, b = C.c_uint64(), C.c_uint64()
        self._check(self.L.rl_batch_progress(self.ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def do_limit_prefixed_async(self, pb, out: dict):
        """rl_do_limit_prefixed_async: a PrefixedBatch (packing.prefixed_batch;
        its buffer pinned for an asynchronous copy) in, out as
        do_limit_host_async; final after synchronize()."""
        r = abi.make_result_struct(out)
        s = pb.struct()
        self._check(self.L.rl_do_limit_prefixed_async(self.ctx, C.byref(s), C.byref(r)))
        return s, r

    # ---- config match + DoLimit on raw requests (rl_match.hip)
    def load_config(self, tree) -> None:
        """rl_config_load: ``tree`` is a ratelimit_amd.config.ConfigTree."""
        nodes, kb, pre = tree.arrays()
        t = abi.RlConfigTree()
        t.n_nodes = len(nodes)
        t.cache_key_prefix_len = len(tree.prefix.encode())
        t.nodes = C.c_void_p(nodes.ctypes.data)
        t.key_bytes = abi.ptr(kb)
        t.key_bytes_len = sum(len(k) for k in tree.keys)
        t.cache_key_prefix = abi.ptr(pre)
        self._check(self.L.rl_config_load(self.ctx, C.byref(t)))

    def do_limit_requests(self, arrays: dict, n_rules: int) -> dict:
        """rl_do_limit_requests on pack_requests() arrays -> per-descriptor results + stats."""
        n = len(arrays["req_idx"])
        b = abi.RlRequestBatch()
        b.n_requests, b.n_descriptors, b.n_entries, b.n_rules = len(arrays["hits"]), n, len(arrays["key_len"]), n_rules
        for k in abi.REQUEST_ARRAYS:
            setattr(b, k, abi.ptr(arrays[k]))
        return self.do_limit_request_batch(b)

    def do_limit_request_batch(self, b) -> dict:
        """rl_do_limit_requests on a filled RlRequestBatch (e.g. from RequestPacker.pack)."""
        n, n_rules = b.n_descriptors, b.n_rules
        out = {k: np.zeros(max(n, 1), dt) for k, dt in abi.REQUEST_RESULT_DTYPES.items()}
        out["stats"] = np.zeros(max(n_rules, 1) * abi.RL_NUM_STATS, np.uint64)
        r = abi.RlRequestResult()
        for k in out:
            setattr(r, k, abi.ptr(out[k]))
        self._check(self.L.rl_do_limit_requests(self.ctx, C.byref(b), C.byref(r)))
        res = {k: v[:n] for k, v in out.items() if k != "stats"}
        res["stats"] = out["stats"][:n_rules * abi.RL_NUM_STATS]
        return res

    def profile(self, enable: bool, every: int = 1):
        """Time every ``every``-th batch's stages with HIP events (rl_profile)."""
        self._check(self.L.rl_profile(self.ctx, max(int(every), 1) if enable else 0))

    def profile_read(self):
        """-> ({prepare, sort, segment, table, finish} summed ms over the timed batches, and
        table_kernel: k_table's device-clock run time averaged per batch}, batches timed);
        resets the sums."""
        ms = (C.c_double * len(PROFILE_FIELDS))()
        nb = C.c_uint64(0)
        self._check(self.L.rl_profile_read(self.ctx, ms, len(PROFILE_FIELDS), C.byref(nb)))
        return dict(zip(PROFILE_FIELDS, list(ms))), nb.value

    def synchronize(self):
        self._check(self.L.rl_synchronize(self.ctx))

    def restore(self, stems: Sequence[bytes], units, nows, counts, lc=None):
        from .packing import arrays_from_lists
        n = len(stems)
        a = arrays_from_lists(list(stems), [], [0] * n, units, [0] * n, [0] * n, [0] * n, [0] * n)
        nowa = np.asarray(nows, np.int64)
        cnt = np.asarray(counts, np.uint32)
        lca = np.asarray(lc if lc is not None else [0] * n, np.uint8)
        rb = abi.RlRestoreBatch()
        rb.n = n
        rb.stem_bytes, rb.stem_off, rb.unit = abi.ptr(a["stem_bytes"]), abi.ptr(a["stem_off"]), abi.ptr(a["unit"])
        rb.now, rb.count, rb.lc = abi.ptr(nowa), abi.ptr(cnt), abi.ptr(lca)
        self._check(self.L.rl_restore(self.ctx, C.byref(rb)))

    def sweep(self, now: int) -> int:
        ev = C.c_uint64(0)
        self._check(self.L.rl_sweep(self.ctx, now, C.byref(ev)))
        return ev.value

    def table_info(self, shard=None) -> dict:
        """Table counters summed over shards (or of one shard)."""
        info = abi.RlTableInfo()
        if shard is None:
            self._check(self.L.rl_table_info_get(self.ctx, C.byref(info)))
        else:
            self._check(self.L.rl_table_info_shard(self.ctx, shard, C.byref(info)))
        return {f: getattr(info, f) for f, _ in abi.RlTableInfo._fields_}

    def local_cache_info(self, now: int) -> dict:
        """localCacheStats gauges (src/limiter/local_cache_stats.go:20-43)."""
        info = abi.RlLocalCacheInfo()
        self._check(self.L.rl_local_cache_info_get(self.ctx, now, C.byref(info)))
        return {f: getattr(info, f) for f, _ in abi.RlLocalCacheInfo._fields_}

    def snapshot(self) -> np.ndarray:
        """Exact table image (counters, local cache, arena, time floor) as host bytes."""
        nb = C.c_uint64(0)
        self._check(self.L.rl_snapshot_size(self.ctx, C.byref(nb)))
        buf = np.empty(nb.value, np.uint8)
        self._check(self.L.rl_snapshot_save(self.ctx, abi.ptr(buf), nb.value))
        return buf

    def load_snapshot(self, buf: np.ndarray) -> None:
        buf = np.ascontiguousarray(buf, np.uint8)
        self._check(self.L.rl_snapshot_load(self.ctx, abi.ptr(buf), buf.size))

    def debug_keys(self, pb: PackedBatch) -> List[str]:
        cap = int(pb.arrays["stem_off"][-1]) + 24 * pb.n + 1
        buf = np.zeros(cap, np.uint8)
        off = np.zeros(pb.n + 1, np.uint32)
        b = pb.batch_struct()
        self._check(self.L.rl_debug_keys(self.ctx, C.byref(b), abi.ptr(buf), abi.ptr(off), cap))
        return [bytes(buf[off[i]:off[i + 1]]).decode() for i in range(pb.n)]

    def debug_decide(self, before, after, lc_hit, hits, limit, unit, flags, now):
        n = len(before)
        a = [np.ascontiguousarray(x, dt) for x, dt in
             ((before, np.uint32), (after, np.uint32), (lc_hit, np.uint8), (hits, np.uint32), (limit, np.uint32),
              (unit, np.uint8), (flags, np.uint8), (now, np.int64))]
        code = np.zeros(n, np.uint8)
        rem = np.zeros(n, np.uint32)
        reset = np.zeros(n, np.uint32)
        deltas = np.zeros(n * abi.RL_NUM_STATS, np.uint64)
        lc_set = np.zeros(n, np.uint8)
        self._check(self.L.rl_debug_decide(self.ctx, n, *[abi.ptr(x) for x in a], abi.ptr(code), abi.ptr(rem),
                                              abi.ptr(reset), abi.ptr(deltas), abi.ptr(lc_set)))
        return code, rem, reset, deltas.reshape(n, abi.RL_NUM_STATS), lc_set


# rl_status of a device-level failure: the GPU or its runtime, not a request
DEVICE_FAILURES = (abi.RL_E_HIP, abi.RL_E_COMM, abi.RL_E_INTERNAL)


class HealthMonitor:
    """The batcher's health monitor (go/src/gpu/cache_impl.go healthMonitor):
    a device-level failure fails the server's health check once, the next
    success marks it OK again — what the Redis pool does on its connections
    (src/redis/driver_impl.go:31-52, server.HealthCheckFail / HealthCheckOK,
    src/server/server.go:47-48). Request-level failures (RL_E_TIME,
    RL_E_INVALID, RL_E_CAPACITY, a full table) leave it as it is. `server`:
    an object with health_check_fail() and health_check_ok() (None: off)."""

    def __init__(self, server=None):
        self.server = server
        self.unhealthy = False

    def observe(self, err):
        if self.server is None:
            return
        if isinstance(err, RedisError) and err.status in DEVICE_FAILURES:
            if not self.unhealthy:
                self.server.health_check_fail()
                self.unhealthy = True
        elif err is None and self.unhealthy:
            self.server.health_check_ok()
            self.unhealthy = False


class GpuRateLimitCache:
    """limiter.RateLimitCache backed by libratelimit_hip.so (BACKEND_TYPE=gpu).
    health_server (GPU_HEALTH_CHECK_DEVICE): the server whose health check a
    device failure fails (HealthMonitor)."""

    def __init__(self, time_source: Optional[TimeSource] = None, near_limit_ratio: float = 0.8,
                 local_cache: bool = False, cache_key_prefix: str = "", per_second: bool = False,
                 expiration_jitter_max_seconds: int = 0, health_server=None, **backend_kw):
        self.time_source = time_source or TimeSource()
        self.prefix = cache_key_prefix
        self.interner = RuleInterner()
        self.health = HealthMonitor(health_server)
        self.backend = Backend(near_limit_ratio, local_cache, per_second, expiration_jitter_max_seconds,
                               **backend_kw)

    def close(self):
        self.backend.close()

    def do_limit(self, ctx, request, limits) -> List[DescriptorStatus]:
        """fixedRateLimitCacheImpl.DoLimit semantics for one request."""
        return self.do_limit_batch([(request, limits, self.time_source.unix_now())])[0]

    def do_limit_batch(self, calls, isolate: bool = False) -> list:
        """Many in-flight DoLimit calls (request, limits, now) as one GPU batch, in arrival order.

        isolate=False: any failure raises RedisError for the whole batch.
        isolate=True: a call holding a descriptor the backend could not answer
        gets a RedisError object in place of its statuses (the batcher panics
        that RPC only, as checkError does per DoLimit, fixed_cache_impl.go:90-95);
        every other call is answered."""
        pb = pack_calls(calls, self.prefix, self.interner)
        try:
            res = self.backend.do_limit_packed(pb, isolate)
        except RedisError as e:
            self.health.observe(e)
            raise
        self.health.observe(None)
        outs = [[DescriptorStatus(OK, None, 0, None) for _ in req.descriptors] for req, _, _ in calls]
        code, rem, rst = res["code"], res["limit_remaining"], res["reset_s"]
        failed = {}
        for j, (c, i) in enumerate(pb.origin):
            lim = calls[c][1][i]
            if isolate and res["status"][j]:
                failed.setdefault(c, int(res["status"][j]))
            outs[c][i] = DescriptorStatus(int(code[j]), lim.limit, int(rem[j]), int(rst[j]))
        for c, st in failed.items():
            outs[c] = RedisError("gpu: descriptor failed [%s]" % abi.STATUS_NAMES.get(st, st))
        st = res["stats"].reshape(-1, abi.RL_NUM_STATS)
        # apply the per-rule deltas to the gostats counters (limit.Stats)
        seen = {}
        for request, limits, _ in calls:
            for lim in limits:
                if lim is not None:
                    seen[lim.stats.key] = lim.stats
        for key, stats in seen.items():
            row = st[self.interner.ids[key]]
            for f, v in zip(abi.STAT_FIELDS, row):
                if v:
                    setattr(stats, f, getattr(stats, f) + int(v))
        return outs

    def flush(self):
        """Flush(): nothing is asynchronous on the host path."""
        return None


class GpuRateLimitService:
    """The service step around DoLimit with the config lookup on the GPU:
    constructLimitsToCheck + DoLimit + shouldRateLimitWorker's statuses
    (src/service/ratelimit.go:104-208; no custom headers) for many requests at
    once through ``rl_do_limit_requests``. Config is YAML text as
    ``NewRateLimitConfigImpl`` takes it (src/config/config_impl.go:318-330)."""

    def __init__(self, config_files, near_limit_ratio: float = 0.8, local_cache: bool = False,
                 cache_key_prefix: str = "", per_second: bool = False, global_shadow_mode: bool = False,
                 **backend_kw):
        from .config import ConfigTree
        self.interner = RuleInterner()
        self.tree = ConfigTree.from_yaml(config_files, cache_key_prefix, self.interner)
        self.global_shadow_mode = global_shadow_mode
        self.backend = Backend(near_limit_ratio, local_cache, per_second, **backend_kw)
        self.backend.load_config(self.tree)
        self.stats = {}  # stats key -> [6 counters] (the gostats store)

    def close(self):
        self.backend.close()

    def should_rate_limit_batch(self, requests, nows):
        """-> [(overall code, [DescriptorStatus])] per request, arrival order."""
        from .config import pack_requests
        for r in requests:  # checkServiceErr (ratelimit.go:151-152)
            if r.domain == "":
                raise ValueError("rate limit domain must not be empty")
            if not r.descriptors:
                raise ValueError("rate limit descriptor list must not be empty")
        a = pack_requests(requests, nows, self.interner)
        n_rules = max(len(self.interner.keys), 1)
        res = self.backend.do_limit_requests(a, n_rules)
        st = res["stats"].reshape(-1, abi.RL_NUM_STATS)
        for i in np.nonzero(st.any(axis=1))[0]:
            row = self.stats.setdefault(self.interner.keys[i], [0] * abi.RL_NUM_STATS)
            for j in range(abi.RL_NUM_STATS):
                row[j] += int(st[i, j])
        out = []
        d = 0
        OVER = 2
        for r in requests:
            sts = []
            final = OK
            for _ in r.descriptors:
                m = int(res["match"][d])
                if m == abi.RL_MATCH_LIMIT:
                    s_ = DescriptorStatus(int(res["code"][d]),
                                          Limit(int(res["requests_per_unit"][d]), int(res["unit"][d])),
                                          int(res["limit_remaining"][d]), int(res["reset_s"][d]))
                    if s_.code == OVER:
                        final = OVER
                else:  # nil limit {OK, nil, 0}; unlimited {OK, nil, MaxUint32}
                    s_ = DescriptorStatus(OK, None, int(res["limit_remaining"][d]), None)
                sts.append(s_)
                d += 1
            if final == OVER and self.global_shadow_mode:
                final = OK
            out.append((final, sts))
        return out
