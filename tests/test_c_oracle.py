"""The C restatement oracle agrees with the golden vectors and with the Python oracle."""
import numpy as np
import pytest

from oracle import c_oracle
from oracle import oracle as O
from ratelimit_amd import abi
from ratelimit_amd.packing import RuleInterner, pack_calls
import golden_util as G
import streams


def run_packed(co, calls, prefix, interner):
    pb = pack_calls(calls, prefix, interner)
    return pb, co.do_limit(pb.arrays, pb.n, pb.n_requests, pb.n_rules)


def unpack_statuses(calls, pb, res):
    """Scatter packed results back to per-call status tuples (nil limits -> OK,None,0,None)."""
    outs = [[(O.OK, None, 0, None)] * len(req.descriptors) for req, _, _ in calls]
    for j, (c, i) in enumerate(pb.origin):
        lim = calls[c][1][i]
        outs[c][i] = (int(res["code"][j]), (lim.limit.requests_per_unit, lim.limit.unit),
                      int(res["limit_remaining"][j]), int(res["reset_s"][j]))
    return outs


@pytest.mark.parametrize("name", G.names("do_limit"))
def test_c_oracle_golden(name):
    fx = G.load(name)
    c = fx["config"]
    co = c_oracle.COracle(c["near_limit_ratio"], c["local_cache"], c["per_second"])
    reg = G.StatsRegistry(O)
    interner = RuleInterner()
    for step in fx["steps"]:
        req = G.make_request(O, step["request"])
        limits = [G.make_limit(O, reg, l) for l in step["limits"]]
        calls = [(req, limits, step["now"])]
        pb = pack_calls(calls, c["prefix"], interner)
        # seeds: find the packed descriptor whose full key is the seeded key
        if step["seed"]:
            keys = co.keys(pb.arrays, pb.n, pb.n_requests)
            for sd in step["seed"]:
                j = keys.index(sd["key"])
                s0, s1 = pb.arrays["stem_off"][j], pb.arrays["stem_off"][j + 1]
                co.restore([bytes(pb.arrays["stem_bytes"][s0:s1])], [pb.arrays["unit"][j]],
                           [step["now"]], [sd["count"]])
        res = co.do_limit(pb.arrays, pb.n, pb.n_requests, pb.n_rules)
        got = unpack_statuses(calls, pb, res)[0]
        assert got == [G.expect_tuple(e) for e in step["expect_statuses"]]
        st = res["stats"].reshape(-1, abi.RL_NUM_STATS)
        for r, key in enumerate(interner.keys):
            s = reg.get(key)
            for f, v in zip(abi.STAT_FIELDS, st[r]):
                setattr(s, f, getattr(s, f) + int(v))
        G.check_stats(reg, step["expect_stats"])


def test_c_oracle_keys_golden():
    fx = G.load("ref_generate_cache_keys")
    for case in fx["cases"]:
        co = c_oracle.COracle()
        reg = G.StatsRegistry(O)
        req = G.make_request(O, case["request"])
        limits = [G.make_limit(O, reg, l) for l in case["limits"]]
        pb = pack_calls([(req, limits, case["now"])], case["prefix"], RuleInterner())
        keys = co.keys(pb.arrays, pb.n, pb.n_requests)
        assert keys == [k for k in case["expect_keys"] if k]


def test_c_oracle_near_threshold():
    for limit, ratio, expect in G.load("own_near_threshold")["cases"]:
        assert c_oracle.near_threshold(limit, ratio) == expect


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("local_cache,per_second,prefix", [(False, False, ""), (True, False, "p:"),
                                                           (False, True, ""), (True, True, "")])
def test_c_oracle_matches_python_oracle(seed, local_cache, per_second, prefix):
    calls = streams.random_stream(seed, n_calls=250, zipf=seed % 2 == 0)
    py_out, py_stats = streams.python_oracle_run(calls, 0.8, local_cache, prefix, per_second)
    co = c_oracle.COracle(0.8, local_cache, per_second)
    interner = RuleInterner()
    totals = {}
    # feed in variable-size batches: a batch is a sequential replay of its calls
    rng = np.random.default_rng(seed)
    i = 0
    while i < len(calls):
        k = int(rng.integers(1, 40))
        chunk = calls[i:i + k]
        pb, res = run_packed(co, chunk, prefix, interner)
        got = unpack_statuses(chunk, pb, res)
        exp = [[s.as_tuple() for s in o] for o in py_out[i:i + k]]
        assert got == exp, "mismatch in calls %d..%d" % (i, i + k)
        st = res["stats"].reshape(-1, abi.RL_NUM_STATS)
        for r, key in enumerate(interner.keys):
            totals[key] = tuple(a + int(b) for a, b in zip(totals.get(key, (0,) * 6), st[r]))
        i += k
    for key, v in py_stats.items():
        assert totals.get(key, (0,) * 6) == v, key


@pytest.mark.parametrize("ratio,local_cache,prefix", [(0.8, False, ""), (0.8, True, "prefix:"), (0.9, True, ""),
                                                      (0.9, False, "prefix:")])
def test_c4_stream_c_oracle_matches_python_oracle(ratio, local_cache, prefix):
    """C4 (nested 4-entry descriptors, shadow, unlimited, overrides, rollover):
    the two restatements agree, so the GPU C4 test has a consistent checker."""
    calls = streams.c4_stream(11, n_calls=1500)
    assert any(l is None for _, ls, _ in calls for l in ls)              # unlimited -> nil
    assert any(l is not None and l.shadow_mode for _, ls, _ in calls for l in ls)
    assert any(d.limit is not None for r, _, _ in calls for d in r.descriptors)  # overrides
    assert {now % 60 for _, _, now in calls} >= {59, 0, 1}                # minute rollover
    py_out, py_stats = streams.python_oracle_run(calls, ratio, local_cache, prefix, False)
    co = c_oracle.COracle(ratio, local_cache, False)
    interner = RuleInterner()
    totals = {}
    i = 0
    for k in (1, 7, 300, 64, 500, 628):
        chunk = calls[i:i + k]
        pb, res = run_packed(co, chunk, prefix, interner)
        got = unpack_statuses(chunk, pb, res)
        exp = [[s.as_tuple() for s in o] for o in py_out[i:i + k]]
        assert got == exp, "mismatch in calls %d..%d" % (i, i + k)
        st = res["stats"].reshape(-1, abi.RL_NUM_STATS)
        for r, key in enumerate(interner.keys):
            totals[key] = tuple(a + int(b) for a, b in zip(totals.get(key, (0,) * 6), st[r]))
        i += k
    assert i == len(calls)
    for key, v in py_stats.items():
        assert totals.get(key, (0,) * 6) == v, key
    co.close()


@pytest.mark.parametrize("threads", [2, 7])
@pytest.mark.parametrize("local_cache,per_second,prefix", [(False, False, ""), (True, False, "p:"),
                                                           (True, True, "")])
def test_sharded_multithreaded_oracle_equals_sequential(threads, local_cache, per_second, prefix):
    """The multi-core CPU baseline (key-sharded stores, one thread each) replays
    exactly what the sequential restatement does: random structured streams
    (shared keys across units, shadow, per-second split) and a Zipf C2 stream."""
    from ratelimit_amd import workloads as W
    seq = c_oracle.COracle(0.8, local_cache, per_second)
    mt = c_oracle.COracleMT(0.8, local_cache, per_second, threads)
    interner = RuleInterner()
    calls = streams.random_stream(threads, n_calls=400, zipf=True)
    for i in range(0, len(calls), 50):
        pb = pack_calls(calls[i:i + 50], prefix, interner)
        a = seq.do_limit(pb.arrays, pb.n, pb.n_requests, pb.n_rules)
        b = mt.do_limit(pb.arrays, pb.n, pb.n_requests, pb.n_rules)
        for k in a:
            assert np.array_equal(a[k], b[k]), k
    z = W.ZipfSampler(5000, 1.1)
    for arr, n, nq, nr in W.c2_stream(n_tenants=5000, requests_per_batch=20000, batches=3, sampler=z):
        a = seq.do_limit(arr, n, nq, nr)
        b = mt.do_limit(arr, n, nq, nr)
        for k in a:
            assert np.array_equal(a[k], b[k]), k
    seq.close()
    mt.close()
