"""The C ABI proven from C99 (tests/c_abi/): no Go, no Python in the call path.

* CPU: include/ratelimit_hip.h compiles as strict C99 (`gcc -x c -std=c99
  -pedantic -Werror`); every struct's size and every field's offset and size,
  as that compiler lays them out, equal the ctypes mirror in
  ratelimit_amd/abi.py field for field (the layout the Python adapter and the
  cgo sketch in INTEGRATION.md rely on); the ABI constants agree; and
  abi_run.c links against libratelimit_hip.so.
* GPU: abi_run (plain C: rl_create, rl_do_limit per batch, rl_destroy) answers
  the reference's own golden DoLimit steps (tests/golden/ref_*.json,
  transcribed from integration_test.go / fixed_cache_impl_test.go), one
  rl_do_limit per RPC, with the reference's expected statuses and stats.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from ratelimit_amd import abi
from ratelimit_amd.packing import RuleInterner, pack_calls
from ratelimit_amd.sharded import WIRE_BYTES
import golden_util as G

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "c_abi")
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "ratelimit_amd")
CFLAGS = ["gcc", "-x", "c", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I" + INC]

MIRROR = {"rl_config": abi.RlConfig, "rl_batch": abi.RlBatch, "rl_result": abi.RlResult,
          "rl_restore_batch": abi.RlRestoreBatch, "rl_table_info": abi.RlTableInfo,
          "rl_config_node": abi.RlConfigNode, "rl_config_tree": abi.RlConfigTree,
          "rl_request_batch": abi.RlRequestBatch, "rl_request_result": abi.RlRequestResult,
          "rl_local_cache_info": abi.RlLocalCacheInfo, "rl_limit": abi.RlLimit,
          "rl_batch_compact": abi.RlBatchCompact, "rl_batch_prefixed": abi.RlBatchPrefixed,
          "rl_log_tear": abi.RlLogTear}


def _build(src, out, extra=()):
    subprocess.run(CFLAGS + [os.path.join(SRC, src), "-o", out] + list(extra), check=True,
                   capture_output=True, text=True)
    return out


def test_header_is_c99_and_matches_the_ctypes_mirror(tmp_path):
    exe = _build("abi_layout.c", str(tmp_path / "abi_layout"))
    lines = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    sizes, fields, consts = {}, {}, {}
    for ln in lines:
        p = ln.split()
        if not p:
            continue
        if p[0] == "S":
            sizes[p[1]] = int(p[2])
        elif p[0] == "F":
            fields.setdefault(p[1], []).append((p[2], int(p[3]), int(p[4])))
        elif p[0] == "C":
            consts[p[1]] = int(p[2])
    import ctypes as C
    assert set(sizes) == set(MIRROR)
    for name, cls in MIRROR.items():
        assert C.sizeof(cls) == sizes[name], name
        mirror = [(f, getattr(cls, f).offset, getattr(cls, f).size) for f, _ in cls._fields_]
        assert mirror == fields[name], name  # same fields, same order, offsets and sizes
    assert consts == {"RL_ABI_VERSION": abi.ABI_VERSION, "RL_NUM_STATS": abi.RL_NUM_STATS,
                      "RL_WIRE_BYTES": WIRE_BYTES, "RL_COMM_ID_BYTES": abi.RL_COMM_ID_BYTES}


def _lib():
    lib = os.path.join(LIBDIR, "libratelimit_hip.so")
    if not os.path.exists(lib):
        pytest.skip("libratelimit_hip.so not built")
    return ["-L" + LIBDIR, "-lratelimit_hip", "-Wl,-rpath," + LIBDIR]


def test_c_program_links_against_the_library(tmp_path):
    _build("abi_run.c", str(tmp_path / "abi_run"), _lib())


# --------------------------------------------------------------------------- GPU
def _fixture_cases():
    out = []
    for name in G.names("do_limit"):
        fx = G.load(name)
        if fx["config"]["jitter_max"] or any(s["seed"] for s in fx["steps"]):
            continue  # (jitter draws and mocked INCRBY replies: test_gpu_parity covers them)
        out.append(name)
    return out


def _write_fixture(path, fx):
    """One packed batch per golden step (one rl_do_limit per RPC)."""
    c = fx["config"]
    reg = G.StatsRegistry(O)
    interner = RuleInterner()
    steps = []
    with open(path, "wb") as f:
        f.write(b"RLFX" + struct.pack("<IIfII", 1, len(fx["steps"]), c["near_limit_ratio"], int(c["local_cache"]),
                                      int(c["per_second"])))
        for st in fx["steps"]:
            req = G.make_request(O, st["request"])
            limits = [G.make_limit(O, reg, l) for l in st["limits"]]
            pb = pack_calls([(req, limits, st["now"])], c["prefix"], interner, n_rules=64)
            a, n = pb.arrays, pb.n
            f.write(struct.pack("<IIII", n, pb.n_requests, 64, int(a["stem_off"][n])))
            f.write(a["stem_bytes"][:int(a["stem_off"][n])].tobytes())
            for k, dt in (("stem_off", np.uint32), ("now", np.int64), ("req_idx", np.uint32), ("unit", np.uint8),
                          ("flags", np.uint8), ("limit", np.uint32), ("hits", np.uint32), ("rule_id", np.uint32)):
                m = n + 1 if k == "stem_off" else (pb.n_requests if k == "now" else n)
                f.write(np.ascontiguousarray(a[k][:m], dt).tobytes())
            steps.append((n, [l is not None for l in limits]))
    return steps, interner


@pytest.mark.gpu
@pytest.mark.parametrize("name", _fixture_cases())
def test_gpu_c_program_answers_golden_steps(name, tmp_path):
    fx = G.load(name)
    exe = _build("abi_run.c", str(tmp_path / "abi_run"), _lib())
    steps, interner = _write_fixture(str(tmp_path / "in.bin"), fx)
    r = subprocess.run([exe, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    buf = open(str(tmp_path / "out.bin"), "rb").read()
    pos = 0
    totals = {}
    for st, (n, present) in zip(fx["steps"], steps):
        code = np.frombuffer(buf, np.uint8, n, pos)
        pos += n
        rem = np.frombuffer(buf, np.uint32, n, pos)
        pos += 4 * n
        reset = np.frombuffer(buf, np.uint32, n, pos)
        pos += 4 * n
        stats = np.frombuffer(buf, np.uint64, 64 * abi.RL_NUM_STATS, pos).reshape(64, abi.RL_NUM_STATS)
        pos += 8 * 64 * abi.RL_NUM_STATS
        exp = [e for e, p in zip(st["expect_statuses"], present) if p]
        got = [{"code": int(code[j]), "remaining": int(rem[j]), "reset": int(reset[j])} for j in range(n)]
        assert got == [{"code": e["code"], "remaining": e["remaining"], "reset": e["reset"]} for e in exp], st
        for rid, key in enumerate(interner.keys):
            t = totals.setdefault(key, np.zeros(abi.RL_NUM_STATS, np.uint64))
            t += stats[rid]
        for key, want in st["expect_stats"].items():
            got_s = dict(zip(abi.STAT_FIELDS, (int(x) for x in totals.get(key, np.zeros(abi.RL_NUM_STATS)))))
            for fld, v in want.items():
                assert got_s[fld] == v, (key, fld)
    assert pos == len(buf)
