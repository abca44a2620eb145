"""Host submission rate of the pipelined path: enqueue K batches without
synchronising (C1 shapes), then synchronise. If the enqueue time per batch is
close to the GPU time per batch, the host is the limiter."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ratelimit_amd import workloads as W
from ratelimit_amd.limiter import Backend
from bench import to_dev
nq = 500_000; n = 2 * nq
be = Backend(0.8, False, table_slots=1 << 26, max_batch=n, max_rules=8, device=0, max_stem_bytes=64 * n)
rng = np.random.default_rng(1)
a, bn, bq, br = W.c1_batch(rng.integers(0, 10_000_000, nq), W.NOW0)
a.pop("now")
dev = to_dev(a, torch)
nows = [torch.full((nq,), W.NOW0 + s, dtype=torch.int64, device="cuda") for s in range(400)]
out = {"code": torch.empty(n, dtype=torch.uint8, device="cuda"), "limit_remaining": torch.empty(n, dtype=torch.int32, device="cuda"),
       "reset_s": torch.empty(n, dtype=torch.int32, device="cuda"), "stats": torch.zeros(12, dtype=torch.int64, device="cuda")}
s = [0]
def step():
    inp = dict(dev); inp["now"] = nows[s[0]]; s[0] += 1
    be.do_limit_device(inp, out, n, nq, 2)
for _ in range(10): step()
be.synchronize(); torch.cuda.synchronize()
K = 100
t0 = time.perf_counter()
for _ in range(K): step()
t1 = time.perf_counter()
be.synchronize(); torch.cuda.synchronize()
t2 = time.perf_counter()
print("enqueue %.1f us/batch, total %.1f us/batch" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6))
# Python-side overhead alone: build the rl_batch without launching
import ratelimit_amd.limiter as LM
t0 = time.perf_counter()
for _ in range(K):
    inp = dict(dev); inp["now"] = nows[0]
    from ratelimit_amd import abi
    b = abi.make_batch_struct(inp, n, nq, 2); r = abi.make_result_struct(out)
t1 = time.perf_counter()
print("python dict+batch build %.1f us/batch" % ((t1 - t0) / K * 1e6))
