"""The Go batcher's exact packing rules through the GPU (round-4 review item 5a).

go/src/gpu/cache_impl.go packs every in-flight DoLimit call into a
prefix-shared batch (gpu.go PrefixedBatch): its entry-level shared prefix cut
at 255 bytes, nil limits skipped, the limit table deduplicated on (limit, rule,
unit, shadow) in first-seen order, sections in its own order; then answers
each call with DurationUntilReset from the call's clock and fails a whole call
when one of its descriptors failed. ratelimit_amd.packing.go_prefixed_batch /
go_statuses restate those rules; here their batches run through
rl_do_limit_prefixed_async from pinned memory and every call's statuses and
the per-rule stats must equal the oracle's sequential replay: C1- and
C2-shaped calls (vs the C oracle), the random structured streams with nil
limits and overrides and C4's nested descriptors (vs the Python oracle)."""
import random

import numpy as np
import pytest

import streams
from oracle import c_oracle
from oracle import oracle as O
from ratelimit_amd import abi, workloads
from ratelimit_amd.limiter import Backend, PinnedArena
from ratelimit_amd.packing import RuleInterner, go_prefixed_batch, go_statuses, pack_calls

pytestmark = pytest.mark.gpu


def _run_go(calls_batches, prefix="", lc=False, ps=False, max_rules=1 << 10, **kw):
    """Every batch of calls packed by the Go rules, queued back to back from
    pinned buffers (two in flight, as the batcher alternates them); -> per
    batch go_statuses and the stats deltas by rule key."""
    be = Backend(0.8, lc, ps, table_slots=kw.get("table_slots", 1 << 18), max_batch=kw.get("max_batch", 1 << 17),
                 max_rules=max_rules)
    arena = PinnedArena()
    it = RuleInterner()
    keep, res = [], []
    try:
        for calls in calls_batches:
            pb, where = go_prefixed_batch(calls, prefix, it, n_rules=max_rules,
                                          alloc=lambda nb: arena.array(nb, np.uint8))
            out = {k: arena.like(v) for k, v in pb.alloc_result(isolate=True, reset=False).items()}
            keep.append((pb, out, be.do_limit_prefixed_async(pb, out)))
            res.append((calls, where, out))
        be.synchronize()
        got, stats = [], {}
        for calls, where, out in res:
            got.append(go_statuses(calls, where, out))
            st = out["stats"].reshape(-1, abi.RL_NUM_STATS)
            for key, rid in it.ids.items():
                if st[rid].any():
                    stats[key] = tuple(int(x) + y for x, y in zip(st[rid], stats.get(key, (0,) * 6)))
        return got, stats
    finally:
        be.close()
        arena.close()


def _oracle_statuses(calls, lc=False, prefix="", ps=False):
    outs, stats = streams.python_oracle_run(calls, 0.8, lc, prefix, ps)
    want = []
    for (req, lims, now), o in zip(calls, outs):
        want.append([(s.code, s.limit_remaining, s.duration_until_reset) for s in o])
    return want, {k: v for k, v in stats.items() if any(v)}


@pytest.mark.parametrize("lc", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_go_rules_random_streams_nil_limits_overrides(seed, lc):
    calls = streams.random_stream(seed, n_calls=1200, p_nil=0.2, p_override=0.15, max_desc=5)
    want, wstats = _oracle_statuses(calls, lc, "go:")
    parts = [calls[i:i + 300] for i in range(0, len(calls), 300)]
    got, gstats = _run_go(parts, prefix="go:", lc=lc)
    flat = [s for g in got for s in g]
    assert flat == want
    assert gstats == wstats


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_go_rules_c4_nested(lc):
    calls = streams.c4_stream(7, n_calls=2400)
    want, wstats = _oracle_statuses(calls, lc)
    got, gstats = _run_go([calls[i:i + 600] for i in range(0, len(calls), 600)], lc=lc)
    assert [s for g in got for s in g] == want
    assert gstats == wstats


def _tenant_calls(tenants, now, hits, rules, reg, nil_every=0):
    """C1/C2-shaped calls: per request [(tenant,t),(tier,sec)] and
    [(tenant,t),(tier,min)]; every nil_every-th request also carries a
    descriptor without a limit."""
    calls = []
    for i, (t, h) in enumerate(zip(tenants, hits)):
        ent = ("tenant", "t%010d" % t)
        descs = [O.Descriptor([ent, ("tier", "sec")]), O.Descriptor([ent, ("tier", "min")])]
        lims = [rules["sec"], rules["min"]]
        if nil_every and i % nil_every == 0:
            descs.insert(1, O.Descriptor([ent, ("tier", "none")]))
            lims.insert(1, None)
        calls.append((O.RateLimitRequest("bench", descs, int(h)), lims, now))
    return calls


def _c_oracle_statuses(batches, lc=False):
    """The same calls through pack_calls arrays into the C oracle."""
    it = RuleInterner()
    co = c_oracle.COracle(0.8, lc)
    want, stats = [], {}
    try:
        for calls in batches:
            pk = pack_calls(calls, "", it, n_rules=1 << 10)
            o = co.do_limit(pk.arrays, pk.n, pk.n_requests, pk.n_rules)
            per = [[(1, 0, None) for _ in req.descriptors] for req, _, _ in calls]
            for j, (c, i) in enumerate(pk.origin):
                per[c][i] = (int(o["code"][j]), int(o["limit_remaining"][j]), int(o["reset_s"][j]))
            want += per
            st = o["stats"].reshape(-1, abi.RL_NUM_STATS)
            for key, rid in it.ids.items():
                if st[rid].any():
                    stats[key] = tuple(int(x) + y for x, y in zip(st[rid], stats.get(key, (0,) * 6)))
    finally:
        co.close()
    return want, stats


@pytest.mark.parametrize("shape", ["c1", "c2"])
def test_gpu_go_rules_tenant_shapes_vs_c_oracle(shape):
    reg = {}
    rules = {u: O.RateLimit("bench.tenant.tier_" + u, O.RateLimitStats("bench.tenant.tier_" + u),
                            O.Limit(lim, unit), False, False)
             for u, lim, unit in (("sec", 100, O.SECOND), ("min", 3000, O.MINUTE))}
    rng = np.random.default_rng(0xC1 if shape == "c1" else 0xC2)
    batches = []
    z = workloads.ZipfSampler(20_000, 1.1) if shape == "c2" else None
    for b in range(3):
        nq = 8000
        ten = z.sample(rng, nq) if z else rng.integers(0, 50_000, nq)
        hits = rng.integers(1, 9, nq) if z else np.ones(nq, np.int64)
        batches.append(_tenant_calls(ten, workloads.NOW0 + b, hits, rules, reg, nil_every=7))
    want, wstats = _c_oracle_statuses(batches)
    got, gstats = _run_go(batches)
    assert [s for g in got for s in g] == want
    assert gstats == wstats


def test_gpu_go_rules_failed_descriptor_fails_its_call_only():
    """A call whose clock is before the last sweep's time floor: its
    descriptor comes back with RL_E_TIME, so the batcher panics that RPC
    alone (cache_impl.go finish) and answers every other call of the batch."""
    calls = streams.random_stream(21, n_calls=400, p_nil=0.1, start_now=1_700_000_100)
    be = Backend(0.8, False, table_slots=1 << 16, max_batch=1 << 14, max_rules=1 << 10)
    arena = PinnedArena()
    try:
        be.sweep(1_700_000_100)  # the time floor
        stale = (O.RateLimitRequest("stale", [O.Descriptor([("only", "here")])], 1),
                 [O.RateLimit("stale.only", O.RateLimitStats("stale.only"), O.Limit(5, O.SECOND), False, False)],
                 1_700_000_050)
        mixed = calls[:200] + [stale] + calls[200:]
        it = RuleInterner()
        pb, where = go_prefixed_batch(mixed, "", it, n_rules=1 << 10, alloc=lambda nb: arena.array(nb, np.uint8))
        out = {k: arena.like(v) for k, v in pb.alloc_result(isolate=True, reset=False).items()}
        keep = be.do_limit_prefixed_async(pb, out)
        be.synchronize()
        got = go_statuses(mixed, where, out)
        assert isinstance(got[200], str) and "rl_status %d" % abi.RL_E_TIME in got[200]
        want, _ = _oracle_statuses(calls)
        assert got[:200] + got[201:] == want
        del keep
    finally:
        be.close()
        arena.close()
