"""Loads the in-tree libratelimit_hip.so (the HIP product library) via ctypes.

There is deliberately no fallback: if the library is missing or cannot be
loaded, every entry point raises. Build it with ``python -m ratelimit_amd.build``.
"""
import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RL_LIB_PATH") or os.path.join(HERE, "libratelimit_hip.so")  # override: profiling builds
TEAR_LIB_PATH = os.path.join(HERE, "libratelimit_hip_tear.so")  # RL_LOG_TEAR build (tests/test_gpu_log_tear.py)

EXPORTS = ["rl_abi_version", "rl_create", "rl_destroy", "rl_last_error", "rl_do_limit", "rl_do_limit_async",
           "rl_synchronize", "rl_sweep", "rl_restore", "rl_table_info_get", "rl_table_info_shard", "rl_alloc_host",
           "rl_free_host",
           "rl_debug_keys", "rl_debug_decide", "rl_profile", "rl_profile_read", "rl_route_pack",
           "rl_route_do_limit", "rl_route_scatter", "rl_config_load", "rl_do_limit_requests",
           "rl_local_cache_info_get", "rl_snapshot_size", "rl_snapshot_save", "rl_snapshot_load",
           "rl_packer_create", "rl_packer_destroy", "rl_packer_pack", "rl_packer_rules", "rl_packer_rule_key",
           "rl_packer_last_error", "rl_comm_unique_id", "rl_comm_loopback_id", "rl_comm_init", "rl_do_limit_routed_async",
           "rl_do_limit_host_async", "rl_do_limit_compact_async", "rl_do_limit_prefixed_async", "rl_batch_progress",
           "rl_debug_log_tear"]

_libs = {}


class RedisError(RuntimeError):
    """Mirror of redis.RedisError (src/redis/driver.go:6-10): backend failure.
    status: the library's rl_status (None: raised by the host code)."""

    def __init__(self, msg, status=None):
        super().__init__(msg)
        self.status = status


def lib():
    """The product library (or RL_LIB_PATH's build)."""
    return load(LIB_PATH)


def load(path):
    """A build of the library at `path`, loaded once per process."""
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError("libratelimit_hip.so not built (%s): run `python -m ratelimit_amd.build`" % path)
    # One HIP runtime per process: torch ships its own libamdhip64.so.7. Loaded
    # first, it also serves this library (same soname); loaded after ours, torch
    # would bring a second runtime that finds no GPU. Device tensors handed to
    # the *_async / rl_route_* entry points must come from the same runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    L.rl_abi_version.restype = C.c_uint32
    L.rl_create.restype = C.c_void_p
    L.rl_create.argtypes = [C.POINTER(abi.RlConfig), C.c_char_p, C.c_size_t]
    L.rl_destroy.argtypes = [C.c_void_p]
    L.rl_last_error.restype = C.c_char_p
    L.rl_last_error.argtypes = [C.c_void_p]
    L.rl_do_limit.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.POINTER(abi.RlResult)]
    L.rl_do_limit_async.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.POINTER(abi.RlResult), C.c_void_p]
    L.rl_do_limit_host_async.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.POINTER(abi.RlResult)]
    if hasattr(L, "rl_do_limit_compact_async"):  # (A/B runs load libraries built before it existed)
        L.rl_do_limit_compact_async.argtypes = [C.c_void_p, C.POINTER(abi.RlBatchCompact), C.POINTER(abi.RlResult)]
    if hasattr(L, "rl_do_limit_prefixed_async"):
        L.rl_do_limit_prefixed_async.argtypes = [C.c_void_p, C.POINTER(abi.RlBatchPrefixed), C.POINTER(abi.RlResult)]
    L.rl_synchronize.argtypes = [C.c_void_p]
    if hasattr(L, "rl_batch_progress"):
        L.rl_batch_progress.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.rl_sweep.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_uint64)]
    L.rl_restore.argtypes = [C.c_void_p, C.POINTER(abi.RlRestoreBatch)]
    L.rl_table_info_get.argtypes = [C.c_void_p, C.POINTER(abi.RlTableInfo)]
    L.rl_table_info_shard.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(abi.RlTableInfo)]
    L.rl_alloc_host.restype = C.c_void_p
    L.rl_alloc_host.argtypes = [C.c_size_t]
    L.rl_free_host.argtypes = [C.c_void_p]
    L.rl_debug_keys.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.c_void_p, C.c_void_p, C.c_uint32]
    L.rl_debug_decide.argtypes = [C.c_void_p, C.c_uint32] + [C.c_void_p] * 13
    L.rl_profile.argtypes = [C.c_void_p, C.c_int]
    L.rl_profile_read.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_uint32, C.POINTER(C.c_uint64)]
    L.rl_route_pack.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                                C.c_void_p, C.c_void_p, C.c_void_p]
    L.rl_route_do_limit.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                    C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.rl_route_scatter.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(abi.RlResult),
                                   C.c_void_p]
    L.rl_comm_unique_id.argtypes = [C.c_void_p]
    L.rl_comm_loopback_id.argtypes = [C.c_void_p]
    L.rl_comm_init.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.rl_do_limit_routed_async.argtypes = [C.c_void_p, C.POINTER(abi.RlBatch), C.POINTER(abi.RlResult), C.c_void_p]
    L.rl_config_load.argtypes = [C.c_void_p, C.POINTER(abi.RlConfigTree)]
    L.rl_do_limit_requests.argtypes = [C.c_void_p, C.POINTER(abi.RlRequestBatch), C.POINTER(abi.RlRequestResult)]
    L.rl_local_cache_info_get.argtypes = [C.c_void_p, C.c_int64, C.POINTER(abi.RlLocalCacheInfo)]
    L.rl_snapshot_size.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.rl_snapshot_save.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    L.rl_snapshot_load.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    L.rl_packer_create.restype = C.c_void_p
    L.rl_packer_create.argtypes = [C.c_uint32]
    L.rl_packer_destroy.argtypes = [C.c_void_p]
    L.rl_packer_pack.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                 C.POINTER(abi.RlRequestBatch)]
    L.rl_packer_rules.restype = C.c_uint32
    L.rl_packer_rules.argtypes = [C.c_void_p]
    L.rl_packer_rule_key.restype = C.c_char_p
    L.rl_packer_rule_key.argtypes = [C.c_void_p, C.c_uint32]
    L.rl_packer_last_error.restype = C.c_char_p
    L.rl_packer_last_error.argtypes = [C.c_void_p]
    if hasattr(L, "rl_debug_log_tear"):
        L.rl_debug_log_tear.argtypes = [C.c_void_p, C.POINTER(abi.RlLogTear), C.POINTER(abi.RlLogTear)]
    if L.rl_abi_version() != abi.ABI_VERSION:
        raise RuntimeError("libratelimit_hip.so ABI mismatch")
    _libs[path] = L
    return L


def check(ctx, rc, L=None):
    if rc != 0:
        msg = (L or lib()).rl_last_error(ctx).decode(errors="replace")
        raise RedisError("%s [%s]" % (msg, abi.STATUS_NAMES.get(rc, rc)), rc)
