"""Request-path throughput (rl_do_limit_requests): C1 / C2 batches as raw
requests (domain + entry bytes), matched against the C1 config on the GPU
(GetLimit trie walk), compacted into DoLimit and mapped back.

Host buffers (pinned, rl_alloc_host), synchronous: the number is PCIe-inclusive
(raw request bytes in, per-descriptor results out) and includes the one
mid-call count readback. The same batches through the packed DoLimit path
(rl_do_limit, also host buffers) are timed beside it, and both results are
checked equal (the request path must give DoLimit's answers).

    python scripts/bench_requests.py [--config c1|c2] [--steps K]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ratelimit_amd import abi, workloads as W  # noqa: E402
from ratelimit_amd._lib import lib  # noqa: E402
from ratelimit_amd.config import ConfigTree  # noqa: E402
from ratelimit_amd.limiter import Backend  # noqa: E402


def pinned(a):
    """Copy a numpy array into pinned host memory (rl_alloc_host)."""
    if a is None:
        return None
    p = lib().rl_alloc_host(max(a.nbytes, 1))
    out = np.ctypeslib.as_array((C.c_uint8 * max(a.nbytes, 1)).from_address(p)).view(a.dtype)[:a.size]
    out[...] = a
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1", choices=["c1", "c2"])
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--requests", type=int, default=500_000)
    ap.add_argument("--tenants", type=int, default=10_000_000)
    args = ap.parse_args()
    nq, T = args.requests, args.tenants
    rng = np.random.default_rng(0xC1 if args.config == "c1" else 0xC2)
    zs = W.ZipfSampler(T, 1.1) if args.config == "c2" else None
    kw = dict(table_slots=1 << 26, max_batch=2 * nq, max_rules=16)
    be_req = Backend(0.8, False, **kw)
    be_pk = Backend(0.8, False, **kw)
    tree = ConfigTree.from_yaml([("c1.yaml", W.C1_CONFIG_YAML)])
    be_req.load_config(tree)
    batches = []
    for b in range(4):
        t = zs.sample(rng, nq) if zs is not None else rng.integers(0, T, nq)
        h = rng.integers(1, 9, nq) if args.config == "c2" else None
        raw = {k: pinned(v) for k, v in W.c1_requests(t, W.NOW0 + b, h).items()}
        pk, n, _, nr = W.c1_batch(t, W.NOW0 + b, h)
        batches.append((raw, {k: pinned(v) for k, v in pk.items()}, n))
    n = batches[0][2]
    # results (pinned)
    rr = {k: pinned(np.zeros(n, dt)) for k, dt in abi.REQUEST_RESULT_DTYPES.items()}
    rr["stats"] = pinned(np.zeros(2 * abi.RL_NUM_STATS, np.uint64))
    pr = {k: pinned(np.zeros(n, dt)) for k, dt in abi.RESULT_DTYPES.items() if k != "stats"}
    pr["stats"] = pinned(np.zeros(2 * abi.RL_NUM_STATS, np.uint64))

    def req_call(raw):
        b = abi.RlRequestBatch()
        b.n_requests, b.n_descriptors, b.n_entries, b.n_rules = nq, n, 2 * n, 2
        for k in abi.REQUEST_ARRAYS:
            setattr(b, k, abi.ptr(raw[k]))
        r = abi.RlRequestResult()
        for k in rr:
            setattr(r, k, abi.ptr(rr[k]))
        rc = lib().rl_do_limit_requests(be_req.ctx, C.byref(b), C.byref(r))
        assert rc == 0, lib().rl_last_error(be_req.ctx)

    def pk_call(pk):
        b = abi.make_batch_struct(pk, n, nq, 2)
        r = abi.make_result_struct(pr)
        rc = lib().rl_do_limit(be_pk.ctx, C.byref(b), C.byref(r))
        assert rc == 0, lib().rl_last_error(be_pk.ctx)

    # warm-up + equality of the two paths on the same stream (clock +1 s per step)
    for s in range(8):
        raw, pk, _ = batches[s % 4]
        now = W.NOW0 + s
        raw["now"][:] = now
        pk["now"][:] = now
        req_call(raw)
        pk_call(pk)
        for k in ("code", "limit_remaining", "reset_s"):
            assert np.array_equal(rr[k], pr[k]), k
        assert np.array_equal(rr["stats"], pr["stats"])
        assert (rr["match"] == abi.RL_MATCH_LIMIT).all()
    res = {}
    for name, fn, idx in (("requests", req_call, 0), ("packed", pk_call, 1)):
        t0 = time.perf_counter()
        for s in range(args.steps):
            bt = batches[s % 4][idx]
            bt["now"][:] = W.NOW0 + 8 + s
            fn(bt)
        res[name] = time.perf_counter() - t0
    out = {"path": "rl_do_limit_requests (host buffers, PCIe-inclusive)", "config": args.config.upper(),
           "descriptors_per_batch": n, "steps": args.steps,
           "requests_decisions_per_s": n * args.steps / res["requests"],
           "requests_ms_per_batch": 1e3 * res["requests"] / args.steps,
           "packed_decisions_per_s": n * args.steps / res["packed"],
           "packed_ms_per_batch": 1e3 * res["packed"] / args.steps,
           "raw_bytes_per_descriptor": sum(v.nbytes for v in batches[0][0].values() if v is not None) / n,
           "packed_bytes_per_descriptor": sum(v.nbytes for v in batches[0][1].values()) / n,
           "parity": "request path == packed DoLimit path on 8 warm-up batches"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
