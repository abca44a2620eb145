"""ctypes mirror of include/ratelimit_hip.h (data layout only; loads no library)."""
import ctypes as C

import numpy as np

RL_OK, RL_E_INVALID, RL_E_TABLE_FULL, RL_E_ARENA_FULL, RL_E_HIP, RL_E_CAPACITY, RL_E_TIME, \
    RL_E_COMM, RL_E_INTERNAL = range(9)
STATUS_NAMES = {0: "RL_OK", 1: "RL_E_INVALID", 2: "RL_E_TABLE_FULL", 3: "RL_E_ARENA_FULL",
                4: "RL_E_HIP", 5: "RL_E_CAPACITY", 6: "RL_E_TIME", 7: "RL_E_COMM", 8: "RL_E_INTERNAL"}
RL_FLAG_SHADOW = 1
RL_NUM_STATS = 6
STAT_FIELDS = ("total_hits", "over_limit", "near_limit", "over_limit_with_local_cache",
               "within_limit", "shadow_mode")

P = C.c_void_p


class RlConfig(C.Structure):
    _fields_ = [("table_slots", C.c_uint64), ("arena_bytes", C.c_uint64),
                ("max_batch", C.c_uint32), ("max_requests", C.c_uint32),
                ("max_rules", C.c_uint32), ("max_stem_bytes", C.c_uint32),
                ("near_limit_ratio", C.c_float), ("local_cache_enabled", C.c_int32),
                ("per_second_split", C.c_int32), ("device", C.c_int32),
                ("expiration_jitter_max_seconds", C.c_int64), ("reserved", C.c_int32 * 8)]


class RlBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_requests", C.c_uint32), ("n_rules", C.c_uint32),
                ("reserved", C.c_uint32), ("stem_bytes", P), ("stem_off", P), ("now", P),
                ("req_idx", P), ("unit", P), ("flags", P), ("limit", P), ("hits", P),
                ("rule_id", P)]


class RlResult(C.Structure):
    _fields_ = [("code", P), ("limit_remaining", P), ("reset_s", P), ("stats", P)]


class RlRestoreBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("reserved", C.c_uint32), ("stem_bytes", P), ("stem_off", P),
                ("unit", P), ("now", P), ("count", P), ("lc", P)]


class RlTableInfo(C.Structure):
    _fields_ = [("table_slots", C.c_uint64), ("live_slots", C.c_uint64), ("tombstones", C.c_uint64),
                ("arena_bytes_used", C.c_uint64), ("exact_stems", C.c_uint64),
                ("batches", C.c_uint64), ("decisions", C.c_uint64)]


def ptr(a):
    """Address of a numpy array (host) or a torch tensor (device) as c_void_p."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return C.c_void_p(a.ctypes.data)
    return C.c_void_p(a.data_ptr())  # torch.Tensor


BATCH_ARRAYS = ("stem_bytes", "stem_off", "now", "req_idx", "unit", "flags", "limit", "hits", "rule_id")
BATCH_DTYPES = {"stem_bytes": np.uint8, "stem_off": np.uint32, "now": np.int64, "req_idx": np.uint32,
                "unit": np.uint8, "flags": np.uint8, "limit": np.uint32, "hits": np.uint32,
                "rule_id": np.uint32}
RESULT_DTYPES = {"code": np.uint8, "limit_remaining": np.uint32, "reset_s": np.uint32, "stats": np.uint64}


def make_batch_struct(arrays, n, n_requests, n_rules):
    b = RlBatch()
    b.n, b.n_requests, b.n_rules = n, n_requests, n_rules
    for k in BATCH_ARRAYS:
        setattr(b, k, ptr(arrays[k]))
    return b


def make_result_struct(arrays):
    r = RlResult()
    for k in ("code", "limit_remaining", "reset_s", "stats"):
        setattr(r, k, ptr(arrays[k]))
    return r
