"""BASELINE configs[3] (C3) at its per-GPU shard on one MI355X: 1B keys over 8
GPUs is 125M live keys per GPU = 62.5M tenants x {sec, min} in a 2^28-slot
(17 GB of 64-B slots + 8.6 GB of ring lines) table. The table is filled through the normal pipeline with batches
generated on the GPU, then C1-shaped 1M-descriptor batches run against it.

Checked at full size (size-independent properties): every key is one live slot;
SECOND windows are fresh each batch, so remaining = 100 - rank of the tenant in
the batch; MINUTE windows carry the fill's INCRBY and every earlier batch's, so
remaining = 3000 - (1 + earlier hits + rank); stats conserve hits. Checked
against the C oracle on the tenants below SUBSET (the oracle holds those keys
only; keys are independent, so the GPU's answer for a descriptor of a subset
tenant equals the oracle's on the subset-only stream).
"""
import numpy as np
import pytest

from oracle import c_oracle
from ratelimit_amd import workloads as W
from ratelimit_amd.limiter import Backend

pytestmark = pytest.mark.gpu

TENANTS = 62_500_000
SLOTS = 1 << 28
NQ = 500_000
SUBSET = 1_000_000


def _rank_in_batch(t):
    """1-based arrival rank of each request's tenant among equal tenants."""
    order = np.argsort(t, kind="stable")
    ts = t[order]
    start = np.r_[True, ts[1:] != ts[:-1]]
    grp = np.cumsum(start) - 1
    first = np.nonzero(start)[0]
    rank = np.empty(t.size, np.int64)
    rank[order] = np.arange(t.size) - first[grp] + 1
    return rank


def test_gpu_c3_shard_125m_live_keys():
    import torch
    be = Backend(0.8, False, table_slots=SLOTS, max_batch=1 << 20, max_rules=8, max_stem_bytes=64 << 20)
    out = {"code": torch.empty(2 * NQ, dtype=torch.uint8, device="cuda"),
           "limit_remaining": torch.empty(2 * NQ, dtype=torch.int32, device="cuda"),
           "reset_s": torch.empty(2 * NQ, dtype=torch.int32, device="cuda"),
           "stats": torch.zeros(12, dtype=torch.int64, device="cuda")}
    try:
        # ---- fill: all 125M keys at NOW0 - 1 (one INCRBY each)
        for s0 in range(0, TENANTS, NQ):
            a, n, nq, nr = W.c1_batch_dev(torch.arange(s0, min(s0 + NQ, TENANTS), device="cuda"), W.NOW0 - 1)
            be.do_limit_device(a, out, n, nq, nr)
        be.synchronize()
        info = be.table_info()
        assert info["live_slots"] == 2 * TENANTS and info["tombstones"] == 0 and info["exact_stems"] == 0

        co = c_oracle.COracle(0.8, False)
        for s0 in range(0, SUBSET, NQ):
            co.do_limit(*W.c1_batch(np.arange(s0, min(s0 + NQ, SUBSET)), W.NOW0 - 1))

        rng = np.random.default_rng(0xC3)
        seen_min = np.zeros(0, np.int64)  # tenants hit by earlier batches (minute window NOW0-1 .. NOW0+39)
        for k in range(3):
            t = rng.integers(0, TENANTS, NQ)
            a, n, nq, nr = W.c1_batch_dev(t, W.NOW0 + k)
            be.do_limit_device(a, out, n, nq, nr)
            be.synchronize()
            code = out["code"].cpu().numpy()
            rem = out["limit_remaining"].cpu().numpy().view(np.uint32).astype(np.int64)
            reset = out["reset_s"].cpu().numpy()
            stats = out["stats"].cpu().numpy().reshape(2, 6)
            assert (code == 1).all()
            rank = _rank_in_batch(t)
            assert np.array_equal(rem[0::2], 100 - rank)
            srt = np.sort(seen_min)
            prior = np.searchsorted(srt, t, side="right") - np.searchsorted(srt, t, side="left")
            assert np.array_equal(rem[1::2], 3000 - (1 + prior + rank))
            assert (reset[0::2] == 1).all() and (reset[1::2] == 60 - (W.NOW0 + k) % 60).all()
            assert stats[:, 0].tolist() == [NQ, NQ] and stats[:, 4].tolist() == [NQ, NQ]
            assert stats[:, 1].sum() == 0 and stats[:, 2].sum() == 0
            seen_min = np.concatenate([seen_min, t])
            # C oracle on the subset tenants
            m = t < SUBSET
            o = co.do_limit(*W.c1_batch(t[m], W.NOW0 + k))
            dm = np.repeat(m, 2)
            assert np.array_equal(code[dm], o["code"])
            assert np.array_equal(rem[dm].astype(np.uint32), o["limit_remaining"])
            assert np.array_equal(reset[dm].view(np.uint32), o["reset_s"])
        co.close()
        info = be.table_info()
        assert info["live_slots"] == 2 * TENANTS
        # SECOND keys moved 1-3 windows forward: their old cur went to the history log
        assert 0 < info["history_appended"] <= 3 * NQ and info["history_lost"] == 0
    finally:
        be.close()
