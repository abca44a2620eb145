"""Host packer throughput (rl_packer, one thread): C1-shaped gRPC payloads
(serialized RateLimitRequest: domain "bench", descriptors [(tenant, t), (tier,
sec)] and [(tenant, t), (tier, min)], hits 1) -> rl_request_batch. CPU only.

    python scripts/bench_packer.py [--requests N] [--reps K]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pbwire  # noqa: E402
from ratelimit_amd.config import RequestPacker  # noqa: E402
from ratelimit_amd.types import Descriptor, RateLimitRequest  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=500_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(0xC1)
    tenants = rng.integers(0, 10_000_000, a.requests)
    msgs = [pbwire.encode_request(RateLimitRequest("bench", [
        Descriptor([("tenant", "t%010d" % t), ("tier", "sec")]),
        Descriptor([("tenant", "t%010d" % t), ("tier", "min")])], 1)) for t in tenants]
    nows = np.full(a.requests, 1_700_000_000, np.int64)
    pk = RequestPacker(2)
    pk.pack(msgs, nows)  # warm the packer's buffers
    t0 = time.perf_counter()
    for _ in range(a.reps):
        b = pk.pack(msgs, nows)
    dt = (time.perf_counter() - t0) / a.reps
    # the native call alone, on payloads already in one buffer (what a gRPC
    # server's receive ring hands the batcher); the figure above adds Python's
    # b"".join of the per-message bytes objects
    import ctypes as C
    from ratelimit_amd import abi
    buf = np.frombuffer(b"".join(msgs), np.uint8)
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    rb = abi.RlRequestBatch()
    L = pk._lib
    t0 = time.perf_counter()
    for _ in range(a.reps):
        rc = L.rl_packer_pack(pk.h, abi.ptr(buf), abi.ptr(off), len(msgs), abi.ptr(nows), C.byref(rb))
        assert rc == 0
    dn = (time.perf_counter() - t0) / a.reps
    print(json.dumps({"path": "rl_packer_pack, 1 thread", "requests": a.requests,
                      "descriptors": int(b.n_descriptors), "payload_bytes_per_request": sum(map(len, msgs)) / a.requests,
                      "native_ms_per_batch": dn * 1e3, "native_descriptors_per_s": b.n_descriptors / dn,
                      "with_python_join_ms_per_batch": dt * 1e3, "with_python_join_descriptors_per_s": b.n_descriptors / dt}))
    pk.close()


if __name__ == "__main__":
    main()
