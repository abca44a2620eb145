"""The host C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer
(the reference's counterpart is `go test -race`,
Makefile:66-72): the protobuf wire parser that takes untrusted RPC payloads
(ratelimit_amd/csrc/rl_pack.cpp) and the C oracle everything is checked
against (oracle/rl_oracle.c, sequential and thread-sharded), built with
-fsanitize=address,undefined -fno-sanitize-recover=all into
tests/c_abi/san_run.c and fed valid, truncated, byte-flipped and
hand-malformed messages and C1/C2/C2U-shaped batches. Any finding aborts the
program; its answers must equal the unsanitized builds' (the product
library's packer, oracle/librl_oracle.so)."""
import os
import random
import shutil
import struct
import subprocess

import numpy as np
import pytest

from oracle.c_oracle import COracle, COracleMT
from ratelimit_amd import workloads as W
from ratelimit_amd._lib import RedisError
from ratelimit_amd.config import RequestPacker
import pbwire
from test_packer_cpu import random_requests

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.fixture(scope="module")
def san_run(tmp_path_factory):
    if not shutil.which("gcc") or not shutil.which("g++"):
        pytest.skip("no gcc")
    d = tmp_path_factory.mktemp("san")
    inc = "-I" + os.path.join(ROOT, "include")
    objs = []
    for src, cc, std in ((os.path.join(ROOT, "ratelimit_amd", "csrc", "rl_pack.cpp"), "g++", "-std=c++17"),
                         (os.path.join(ROOT, "oracle", "rl_oracle.c"), "gcc", "-std=c11"),
                         (os.path.join(HERE, "c_abi", "san_run.c"), "gcc", "-std=c11")):
        o = str(d / (os.path.basename(src) + ".o"))
        subprocess.run([cc, std, inc, "-Wall", "-c", src, "-o", o] + SAN, check=True, capture_output=True, text=True)
        objs.append(o)
    exe = str(d / "san_run")
    subprocess.run(["g++", "-o", exe] + objs + SAN + ["-lpthread", "-lm"], check=True, capture_output=True, text=True)
    syms = subprocess.run(["nm", "-u", exe], capture_output=True, text=True).stdout
    assert "__asan_report_load" in syms and "__ubsan_handle" in syms  # (instrumented)
    return exe, d


def _group(msgs, nows):
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return (struct.pack("<I", len(msgs)) + off.tobytes() + b"".join(msgs) + np.asarray(nows, np.int64).tobytes())


def _malformed():
    """Hand-built bad messages: field number 0 and 2^29, a length past the
    end, an 11-byte varint, a nested descriptor longer than its parent, a
    wire type 3/4 group, an entry whose key length overflows."""
    v = pbwire.field_varint
    out = [
        bytes([0x00, 0x01]),                         # field 0
        bytes([0x80, 0x80, 0x80, 0x80, 0x10, 0x01]),  # field 2^29 (varint)
        bytes([0x0a, 0x7f]) + b"ab",                 # domain length 127, 2 bytes there
        bytes([0x18]) + b"\xff" * 10 + b"\x01",      # hits: an 11-byte varint
        bytes([0x12, 0x04, 0x0a, 0x10, 0x0a, 0x01]),  # descriptor of 4 holding an entry of 16
        bytes([0x1b, 0x1c]),                         # wire types 3 / 4 (groups)
        bytes([0x12, 0x06, 0x0a, 0x04, 0x0a, 0xff, 0xff, 0x03]),  # key length 65535 inside 4 bytes
        bytes([0x0a, 0xff, 0xff, 0xff, 0xff, 0x0f]) + b"x",       # domain length 2^32 - 1
        v(3, 1 << 40),                               # hits past 32 bits
        bytes([0x2d]) + b"\x01\x02",                 # fixed32 unknown field, truncated
        bytes([0x29]) + b"\x01" * 8,                 # fixed64 unknown field (valid, skipped)
    ]
    return out


def _packer_inputs(seed=3):
    rng = random.Random(seed)
    reqs = random_requests(seed, 600)
    msgs = [pbwire.encode_request(r, extra_unknown=(i % 4 == 0)) for i, r in enumerate(reqs)]
    groups = []
    for i in range(0, 600, 60):  # valid groups
        groups.append((msgs[i:i + 60], [1_700_000_000 + j for j in range(60)]))
    for m in msgs[:6]:  # every truncation of a few messages
        for k in range(len(m)):
            groups.append(([m[:k]], [1_700_000_000]))
    for _ in range(300):  # byte flips
        m = bytearray(rng.choice(msgs))
        if not m:
            continue
        for _ in range(rng.randint(1, 3)):
            m[rng.randrange(len(m))] = rng.randrange(256)
        groups.append(([bytes(m)], [1_700_000_000]))
    for m in _malformed():
        groups.append(([m], [1_700_000_000]))
        groups.append(([msgs[0], m, msgs[1]], [1_700_000_000] * 3))
    return groups


def _fnv(h, a):
    for b in np.ascontiguousarray(a).view(np.uint8).tobytes():
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def _oracle_inputs():
    rng = np.random.default_rng(9)
    z = W.ZipfSampler(5_000, 1.1)
    out = []
    for k in range(8):
        if k % 3 == 0:
            a, n, nq, nr = W.c1_batch(rng.integers(0, 5_000, 3_000), W.NOW0 + k)
        elif k % 3 == 1:
            a, n, nq, nr = W.c1_batch(z.sample(rng, 3_000), W.NOW0 + k, rng.integers(1, 9, 3_000).astype(np.uint32))
        else:
            a, n, nq, nr = W.c2u_batch(z.sample(rng, 3_000), W.NOW0 + k, rng.integers(1, 9, 3_000).astype(np.uint32),
                                       rng)
            nr = 3
        out.append((a, n, nq, nr, k % 2))
    return out


def test_host_code_is_clean_under_asan_and_ubsan(san_run):
    exe, d = san_run
    groups = _packer_inputs()
    (d / "packer.bin").write_bytes(b"".join(_group(m, t) for m, t in groups))
    batches = _oracle_inputs()
    blob = b""
    for a, n, nq, nr, mt in batches:
        blob += struct.pack("<4I", n, nq, nr, mt) + a["stem_off"].astype(np.uint32).tobytes() + \
            a["stem_bytes"].tobytes() + a["now"].astype(np.int64).tobytes()
        for k, t in (("req_idx", np.uint32), ("unit", np.uint8), ("flags", np.uint8), ("limit", np.uint32),
                     ("hits", np.uint32), ("rule_id", np.uint32)):
            blob += a[k].astype(t).tobytes()
    (d / "oracle.bin").write_bytes(blob)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(d / "packer.bin"), str(d / "oracle.bin")], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.split("\n")
    plines = [l.split() for l in lines if l.startswith("P ")]
    olines = [l.split() for l in lines if l.startswith("O ")]
    assert len(plines) == len(groups) and len(olines) == len(batches)
    # the packer: the same verdict as the product library's (unsanitized) build
    pk = RequestPacker(first_override_rule=7)
    bad = 0
    try:
        for (msgs, nows), p in zip(groups, plines):
            try:
                b = pk.pack(msgs, nows)
                want = (0, b.n_requests, b.n_descriptors)
            except RedisError:
                want = None
            if want is None:
                assert int(p[2]) != 0, p
                bad += 1
            else:
                assert (int(p[2]), int(p[3]), int(p[4])) == want, (p, want)
    finally:
        pk.close()
    assert bad > 100  # (the malformed groups were rejected, not parsed)
    # the oracle: the same answers as oracle/librl_oracle.so
    seq, mt = COracle(0.8, True), COracleMT(0.8, True, False, 3)
    try:
        for (a, n, nq, nr, use_mt), o in zip(batches, olines):
            g = (mt if use_mt else seq).do_limit(a, n, nq, nr)
            h = 0xcbf29ce484222325
            for k in ("code", "limit_remaining", "reset_s", "stats"):
                h = _fnv(h, g[k])
            assert int(o[2]) == 0 and o[3] == "%016x" % h, (o, "%016x" % h)
    finally:
        seq.close()
        mt.close()
