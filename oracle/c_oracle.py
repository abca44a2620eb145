"""ctypes wrapper for oracle/librl_oracle.so (TEST INFRASTRUCTURE ONLY).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline. Build with ``make -C oracle``.
"""
import ctypes as C
import os

import numpy as np

from ratelimit_amd import abi  # data layout only (no product code runs)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librl_oracle.so")
_lib = None


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.rlo_create.restype = C.c_void_p
        L.rlo_create.argtypes = [C.c_float, C.c_int, C.c_int]
        L.rlo_destroy.argtypes = [C.c_void_p]
        L.rlo_mt_create.restype = C.c_void_p
        L.rlo_mt_create.argtypes = [C.c_float, C.c_int, C.c_int, C.c_int]
        L.rlo_mt_destroy.argtypes = [C.c_void_p]
        L.rlo_mt_do_limit.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.POINTER(abi.RlResult)]
        L.rlo_do_limit.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.POINTER(abi.RlResult)]
        L.rlo_restore.argtypes = [C.c_void_p, C.POINTER(abi.RlRestoreBatch)]
        L.rlo_keys.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.c_void_p, C.c_void_p, C.c_uint32]
        L.rlo_near_threshold.restype = C.c_uint32
        L.rlo_near_threshold.argtypes = [C.c_uint32, C.c_float]
        L.rlo_set_horizon.restype = None
        L.rlo_set_horizon.argtypes = [C.c_void_p, C.c_int64]
        L.rlo_live_keys.restype = C.c_uint64
        L.rlo_live_keys.argtypes = [C.c_void_p]
        _lib = L
    return _lib


class COracle:
    def __init__(self, near_limit_ratio=0.8, local_cache=False, per_second=False, horizon=0):
        """horizon: keep keys for requests lagging up to horizon s + 2 windows
        (the GPU ctx's expiration_jitter_max_seconds; GC slack only)."""
        self.h = lib().rlo_create(near_limit_ratio, int(local_cache), int(per_second))
        if horizon:
            lib().rlo_set_horizon(self.h, horizon)

    def close(self):
        if self.h:
            lib().rlo_destroy(self.h)
            self.h = None

    __del__ = close

    def do_limit(self, arrays, n, n_requests, n_rules):
        """Returns dict of result arrays for a packed batch (numpy arrays)."""
        b = abi.make_batch_struct(arrays, n, n_requests, n_rules)
        out = {"code": np.zeros(max(n, 1), np.uint8), "limit_remaining": np.zeros(max(n, 1), np.uint32),
               "reset_s": np.zeros(max(n, 1), np.uint32),
               "stats": np.zeros(max(n_rules, 1) * abi.RL_NUM_STATS, np.uint64)}
        r = abi.make_result_struct(out)
        rc = lib().rlo_do_limit(self.h, C.byref(b), C.byref(r))
        if rc:
            raise RuntimeError("oracle rlo_do_limit: %s" % abi.STATUS_NAMES.get(rc, rc))
        return {k: v[:n] if k != "stats" else v[:n_rules * abi.RL_NUM_STATS] for k, v in out.items()}

    def restore(self, stems, unit, now, count, lc=None):
        from ratelimit_amd.packing import arrays_from_lists
        n = len(stems)
        a = arrays_from_lists(stems, [], [0] * n, unit, [0] * n, [0] * n, [0] * n, [0] * n)
        nowa = np.asarray(now, np.int64)
        cnt = np.asarray(count, np.uint32)
        lca = np.asarray(lc if lc is not None else [0] * n, np.uint8)
        rb = abi.RlRestoreBatch()
        rb.n = n
        rb.stem_bytes, rb.stem_off, rb.unit = abi.ptr(a["stem_bytes"]), abi.ptr(a["stem_off"]), abi.ptr(a["unit"])
        rb.now, rb.count, rb.lc = abi.ptr(nowa), abi.ptr(cnt), abi.ptr(lca)
        rc = lib().rlo_restore(self.h, C.byref(rb))
        if rc:
            raise RuntimeError("oracle restore failed %d" % rc)

    def keys(self, arrays, n, n_requests):
        b = abi.make_batch_struct(arrays, n, n_requests, 0)
        cap = int(arrays["stem_off"][-1]) + 24 * n + 1
        buf = np.zeros(cap, np.uint8)
        off = np.zeros(n + 1, np.uint32)
        rc = lib().rlo_keys(self.h, C.byref(b), abi.ptr(buf), abi.ptr(off), cap)
        if rc:
            raise RuntimeError("oracle keys failed %d" % rc)
        return [bytes(buf[off[i]:off[i + 1]]).decode() for i in range(n)]

    def live_keys(self):
        return lib().rlo_live_keys(self.h)


def near_threshold(limit, ratio):
    return lib().rlo_near_threshold(limit, ratio)


class COracleMT:
    """The C restatement sharded by stem hash over `threads` independent stores,
    one thread per shard (the multi-core CPU baseline; equal to COracle)."""

    def __init__(self, near_limit_ratio=0.8, local_cache=False, per_second=False, threads=1):
        self.threads = threads
        self.h = lib().rlo_mt_create(near_limit_ratio, int(local_cache), int(per_second), threads)

    def close(self):
        if self.h:
            lib().rlo_mt_destroy(self.h)
            self.h = None

    __del__ = close

    def do_limit(self, arrays, n, n_requests, n_rules):
        b = abi.make_batch_struct(arrays, n, n_requests, n_rules)
        out = {"code": np.zeros(max(n, 1), np.uint8), "limit_remaining": np.zeros(max(n, 1), np.uint32),
               "reset_s": np.zeros(max(n, 1), np.uint32),
               "stats": np.zeros(max(n_rules, 1) * abi.RL_NUM_STATS, np.uint64)}
        r = abi.make_result_struct(out)
        rc = lib().rlo_mt_do_limit(self.h, C.byref(b), C.byref(r))
        if rc:
            raise RuntimeError("oracle rlo_mt_do_limit: %s" % abi.STATUS_NAMES.get(rc, rc))
        return {k: v[:n] if k != "stats" else v[:n_rules * abi.RL_NUM_STATS] for k, v in out.items()}
