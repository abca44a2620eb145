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
                ("expiration_jitter_max_seconds", C.c_int64), ("hash_seed", C.c_uint64),
                ("n_shards", C.c_uint32), ("debug_hash_bits", C.c_uint32), ("shard_device", C.c_int32 * 16),
                ("history_entries", C.c_uint64), ("reserved", C.c_int32 * 6)]


class RlBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_requests", C.c_uint32), ("n_rules", C.c_uint32),
                ("reserved", C.c_uint32), ("stem_bytes", P), ("stem_off", P), ("now", P),
                ("req_idx", P), ("unit", P), ("flags", P), ("limit", P), ("hits", P),
                ("rule_id", P)]


# rl_limit (12 B): one entry of a compact batch's limit table
LIMIT_DTYPE = np.dtype([("requests_per_unit", np.uint32), ("rule_id", np.uint32), ("unit", np.uint8),
                        ("flags", np.uint8), ("reserved", np.uint16)])


class RlLimit(C.Structure):
    _fields_ = [("requests_per_unit", C.c_uint32), ("rule_id", C.c_uint32), ("unit", C.c_uint8),
                ("flags", C.c_uint8), ("reserved", C.c_uint16)]


assert LIMIT_DTYPE.itemsize == C.sizeof(RlLimit)


class RlBatchCompact(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_requests", C.c_uint32), ("n_rules", C.c_uint32), ("n_limits", C.c_uint32),
                ("buf", P), ("buf_bytes", C.c_uint64), ("stem_bytes", C.c_uint64), ("stem_off", C.c_uint64),
                ("limit_idx", C.c_uint64), ("req_first", C.c_uint64), ("now", C.c_uint64), ("hits", C.c_uint64),
                ("limits", C.c_uint64)]


RL_PREFIXED_TILE = 256  # include/ratelimit_hip.h: requests per index tile


class RlBatchPrefixed(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_requests", C.c_uint32), ("n_rules", C.c_uint32), ("n_limits", C.c_uint32),
                ("buf", P), ("buf_bytes", C.c_uint64), ("req", C.c_uint64), ("now", C.c_uint64),
                ("hits", C.c_uint64), ("desc", C.c_uint64), ("prefix_bytes", C.c_uint64),
                ("suffix_bytes", C.c_uint64), ("limits", C.c_uint64), ("index", C.c_uint64)]


class RlResult(C.Structure):
    _fields_ = [("code", P), ("limit_remaining", P), ("reset_s", P), ("stats", P), ("status", P)]


class RlRestoreBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("reserved", C.c_uint32), ("stem_bytes", P), ("stem_off", P),
                ("unit", P), ("now", P), ("count", P), ("lc", P)]


class RlTableInfo(C.Structure):
    _fields_ = [("table_slots", C.c_uint64), ("live_slots", C.c_uint64), ("tombstones", C.c_uint64),
                ("arena_bytes_used", C.c_uint64), ("exact_stems", C.c_uint64),
                ("batches", C.c_uint64), ("decisions", C.c_uint64),
                ("history_entries", C.c_uint64), ("history_appended", C.c_uint64),
                ("history_lost", C.c_uint64), ("history_slots", C.c_uint64), ("history_refused", C.c_uint64)]


class RlLogTear(C.Structure):
    """rl_log_tear (include/ratelimit_hip.h): rl_debug_log_tear's armed tear and its outcome."""
    _fields_ = [("armed", C.c_uint32), ("protocol", C.c_uint32), ("sched", C.c_uint32 * 3),
                ("entry", C.c_uint32 * 8), ("before", C.c_uint32 * 8), ("seen", C.c_uint32 * 12),
                ("verdict", C.c_int32), ("reserved", C.c_uint32)]


class RlConfigNode(C.Structure):
    _fields_ = [("parent", C.c_int32), ("key_off", C.c_uint32), ("key_len", C.c_uint32),
                ("requests_per_unit", C.c_uint32), ("rule_id", C.c_uint32), ("unit", C.c_uint8),
                ("has_limit", C.c_uint8), ("unlimited", C.c_uint8), ("shadow_mode", C.c_uint8)]


# numpy view of rl_config_node (24 B), for building the node array in one go
CONFIG_NODE_DTYPE = np.dtype([("parent", np.int32), ("key_off", np.uint32), ("key_len", np.uint32),
                              ("requests_per_unit", np.uint32), ("rule_id", np.uint32), ("unit", np.uint8),
                              ("has_limit", np.uint8), ("unlimited", np.uint8), ("shadow_mode", np.uint8)])


class RlConfigTree(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("cache_key_prefix_len", C.c_uint32), ("nodes", P),
                ("key_bytes", P), ("key_bytes_len", C.c_uint64), ("cache_key_prefix", P)]


class RlRequestBatch(C.Structure):
    _fields_ = [("n_requests", C.c_uint32), ("n_descriptors", C.c_uint32), ("n_entries", C.c_uint32),
                ("n_rules", C.c_uint32), ("domain_bytes", P), ("domain_off", P), ("now", P), ("hits", P),
                ("req_idx", P), ("entry_first", P), ("desc_off", P), ("desc_bytes", P), ("key_len", P),
                ("value_len", P), ("override_flags", P), ("override_rpu", P), ("override_unit", P),
                ("override_rule", P)]


class RlRequestResult(C.Structure):
    _fields_ = [("code", P), ("limit_remaining", P), ("reset_s", P), ("match", P), ("rule_id", P),
                ("requests_per_unit", P), ("unit", P), ("stats", P)]


class RlLocalCacheInfo(C.Structure):
    _fields_ = [("entry_count", C.c_uint64), ("lookup_count", C.c_uint64), ("hit_count", C.c_uint64),
                ("miss_count", C.c_uint64)]


RL_MATCH_NONE, RL_MATCH_UNLIMITED, RL_MATCH_LIMIT = 0, 1, 2
REQUEST_ARRAYS = ("domain_bytes", "domain_off", "now", "hits", "req_idx", "entry_first", "desc_off", "desc_bytes",
                  "key_len", "value_len", "override_flags", "override_rpu", "override_unit", "override_rule")
REQUEST_DTYPES = {"domain_bytes": np.uint8, "domain_off": np.uint32, "now": np.int64, "hits": np.uint32,
                  "req_idx": np.uint32, "entry_first": np.uint32, "desc_off": np.uint32, "desc_bytes": np.uint8,
                  "key_len": np.uint16, "value_len": np.uint16, "override_flags": np.uint8,
                  "override_rpu": np.uint32, "override_unit": np.uint8, "override_rule": np.uint32}
REQUEST_RESULT_DTYPES = {"code": np.uint8, "limit_remaining": np.uint32, "reset_s": np.uint32, "match": np.uint8,
                         "rule_id": np.uint32, "requests_per_unit": np.uint32, "unit": np.uint8}


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
RESULT_DTYPES = {"code": np.uint8, "limit_remaining": np.uint32, "reset_s": np.uint32, "stats": np.uint64,
                 "status": np.uint8}
ABI_VERSION = 6
RL_COMM_ID_BYTES = 128  # include/ratelimit_hip.h
RL_ROUTED_INFLIGHT = 6  # include/ratelimit_hip.h (routed batches in flight: the input-reuse distance)
RL_ROUTED_LAG = 3  # include/ratelimit_hip.h (calls between a routed batch's partition and its owner pipeline)


def make_batch_struct(arrays, n, n_requests, n_rules):
    b = RlBatch()
    b.n, b.n_requests, b.n_rules = n, n_requests, n_rules
    for k in BATCH_ARRAYS:
        setattr(b, k, ptr(arrays[k]))
    return b


def make_result_struct(arrays):
    r = RlResult()
    for k in ("code", "limit_remaining", "reset_s", "stats", "status"):
        setattr(r, k, ptr(arrays.get(k)))
    return r
