"""Isolated timing of the routing partition (rl_route_pack) on one GPU.

Measurement tool, not part of the library: packs one C1 batch (1M
descriptors, 34-byte stems) for n_shards owners `reps` times on one stream and
prints the mean time per call (HIP events), with the algorithmic bytes moved
(inputs read once, wire records + stems + perm written once).

    python tools/route_pack_bench.py [n_shards ...]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ratelimit_amd import abi, workloads as W  # noqa: E402
from ratelimit_amd._lib import check, lib  # noqa: E402
from ratelimit_amd.limiter import Backend  # noqa: E402
from ratelimit_amd.sharded import WIRE_BYTES  # noqa: E402


def main():
    shards = [int(x) for x in sys.argv[1:]] or [1, 8]
    nq = 500_000
    be = Backend(0.8, False, table_slots=1 << 20, max_batch=2 * nq, max_rules=8, hash_seed=7)
    a, n, _, _ = W.c1_batch(np.random.default_rng(1).integers(0, 10_000_000, nq), W.NOW0)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v).view({np.dtype(np.uint32): np.int32}.get(v.dtype, v.dtype)))
           .cuda() for k, v in a.items()}
    stem_bytes = int(a["stem_off"][n])
    send_rec = torch.empty(n * WIRE_BYTES, dtype=torch.uint8, device="cuda")
    send_stem = torch.empty(stem_bytes + 64, dtype=torch.uint8, device="cuda")
    perm = torch.empty(n, dtype=torch.int32, device="cuda")
    counts = torch.empty(2 * 256, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    b = abi.make_batch_struct(dev, n, nq, 2)
    out = {}
    for ns in shards:
        def call():
            check(be.ctx, lib().rl_route_pack(be.ctx, b, ns, 0, abi.ptr(send_rec), abi.ptr(send_stem), abi.ptr(perm),
                                               abi.ptr(counts), st.cuda_stream))
        for _ in range(5):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record(st)
        for _ in range(reps):
            call()
        e1.record(st)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        byts = n * (4 + 4 + 1 + 1 + 4 + 4 + 4 + 4) + nq * 8 + stem_bytes  # inputs
        byts += n * (WIRE_BYTES + 4) + stem_bytes                                  # wire, perm, stems
        c = counts[:2 * ns].cpu().numpy()
        assert int(c[0::2].sum()) == n and int(c[1::2].sum()) == stem_bytes, c
        out[ns] = {"us": round(us, 1), "GBps": round(byts / us / 1e3, 1)}
    be.synchronize()
    print(json.dumps({"tool": "route_pack_bench", "descriptors": n, "per_n_shards": out}))


if __name__ == "__main__":
    main()
