"""CPU-side checks of the boundary: the C-ABI library loads and exports every
symbol include/ratelimit_hip.h declares; struct layouts agree; the host packer
builds the reference's key stems. No compute calls (no GPU here)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from ratelimit_amd import abi, packing, workloads
from ratelimit_amd import types as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ratelimit_hip.h")
LIB = os.path.join(ROOT, "ratelimit_amd", "libratelimit_hip.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rl_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_api():
    fns = declared_functions()
    for f in ["rl_create", "rl_destroy", "rl_do_limit", "rl_do_limit_async", "rl_synchronize", "rl_sweep",
              "rl_restore", "rl_last_error", "rl_alloc_host", "rl_free_host", "rl_table_info_get"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        from ratelimit_amd import build
        build.build()
    lib = C.CDLL(LIB)
    for f in declared_functions():
        assert hasattr(lib, f), f
    lib.rl_abi_version.restype = C.c_uint32
    assert lib.rl_abi_version() == abi.ABI_VERSION


def test_product_loader_lists_all_exports():
    from ratelimit_amd import _lib
    assert sorted(_lib.EXPORTS) == declared_functions()


def test_struct_layout_matches_header():
    # sizes as laid out by the C compiler for include/ratelimit_hip.h (x86-64 / gfx950 host)
    assert C.sizeof(abi.RlConfig) == 8 + 8 + 4 * 4 + 4 + 4 * 3 + 8 + 8 + 4 + 4 + 4 * 16 + 4 * 8
    assert C.sizeof(abi.RlBatch) == 16 + 9 * 8
    assert C.sizeof(abi.RlResult) == 5 * 8
    assert C.sizeof(abi.RlRestoreBatch) == 8 + 6 * 8


def test_stem_matches_cache_key_generator():
    # cache_key.go:62-71: prefix ‖ domain ‖ '_' ‖ Σ(key ‖ '_' ‖ value ‖ '_')
    assert packing.stem_of("", "domain", [("key", "value")]) == b"domain_key_value_"
    assert packing.stem_of("prefix:", "domain", [("key", "value")]) == b"prefix:domain_key_value_"
    assert packing.stem_of("", "d", [("a", ""), ("b", "c")]) == b"d_a__b_c_"


def test_pack_calls_drops_nil_and_interns_rules():
    lim = T.new_rate_limit(10, T.MINUTE, "r1")
    req = T.RateLimitRequest("dom", [T.Descriptor([("k", "v")]), T.Descriptor([("x", "y")])], 0)
    it = packing.RuleInterner()
    pb = packing.pack_calls([(req, [None, lim], 1234), (req, [lim, lim], 1235)], "", it)
    assert pb.n == 3 and pb.n_requests == 2 and pb.n_rules == 1
    assert pb.origin == [(0, 1), (1, 0), (1, 1)]
    assert list(pb.arrays["req_idx"]) == [0, 1, 1]
    assert list(pb.arrays["now"]) == [1234, 1235]
    assert bytes(pb.arrays["stem_bytes"][:pb.arrays["stem_off"][1]]) == b"dom_x_y_"


def test_pack_rejects_unknown_unit():
    lim = T.new_rate_limit(10, 0, "r1")
    req = T.RateLimitRequest("dom", [T.Descriptor([("k", "v")])], 1)
    with pytest.raises(RuntimeError):
        packing.pack_calls([(req, [lim], 1)], "", packing.RuleInterner())


def test_c1_workload_shape():
    a, n, nq, nr = workloads.c1_batch(np.array([1234, 7]), 1_700_000_000)
    assert n == 4 and nq == 2 and nr == 2
    s = bytes(a["stem_bytes"][a["stem_off"][0]:a["stem_off"][1]])
    assert s == b"bench_tenant_t0000001234_tier_sec_" and len(s) == 34
    s = bytes(a["stem_bytes"][a["stem_off"][3]:a["stem_off"][4]])
    assert s == b"bench_tenant_t0000000007_tier_min_"
    assert list(a["unit"]) == [1, 2, 1, 2] and list(a["req_idx"]) == [0, 0, 1, 1]


def test_c1_device_generator_equals_host_generator():
    """c1_batch_dev (torch, used to fill C3-sized tables on the GPU) builds the
    same bytes and arrays as c1_batch; checked here on the CPU device."""
    t = np.array([0, 1234, 9_999_999_999, 62_499_999], np.int64)
    h = np.array([1, 2, 3, 8], np.uint32)
    a, n, nq, nr = workloads.c1_batch(t, 1_700_000_000, h)
    d, dn, dq, dr = workloads.c1_batch_dev(t, 1_700_000_000, h, device="cpu")
    assert (n, nq, nr) == (dn, dq, dr)
    for k, v in a.items():
        got = d[k].numpy()
        assert np.array_equal(got.view(v.dtype) if got.dtype != v.dtype else got, v), k


def test_concat_batches_rebases():
    b1 = workloads.c1_batch(np.array([1]), 10)
    b2 = workloads.c1_batch(np.array([2, 3]), 11)
    a, n, nq, nr = workloads.concat_batches([b1, b2])
    assert n == 6 and nq == 3
    assert list(a["req_idx"]) == [0, 0, 1, 1, 2, 2]
    assert list(a["now"]) == [10, 11, 11]
    assert a["stem_off"][-1] == 6 * 34
