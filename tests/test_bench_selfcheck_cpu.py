"""bench.py's self-check (verify) on the CPU: answers produced by the C oracle
over the whole stream pass it; a single wrong answer, or stats that lose
hits, fail it — so a wrong-answer fast path cannot post a bench line.
The "GPU" here is the oracle itself replaying every tenant: the check replays
only a tenant subset, and keys are independent, so the two must agree."""
import argparse

import numpy as np
import pytest

import bench
from oracle.c_oracle import COracle
from ratelimit_amd import workloads as W


def _args(config, distinct=3):
    return argparse.Namespace(requests=3_000, distinct_batches=distinct, config=config, no_fill=False,
                              n_rules=3 if config == "c2u" else 2)


def _full_run(args, T, world, steps, sampler):
    """Every rank's batches through one oracle (global order: fill, then per
    step rank-major); returns each rank's answers at the last step."""
    co = COracle(0.8, False, False)
    ranks = [bench.make_batches(args, W, q, world * T, sampler) for q in range(world)]
    co.do_limit(*W.c1_batch(np.arange(world * T), W.NOW0 - 1))
    last = {}
    for s in range(steps):
        for q in range(world):
            a, n, nq, _ = ranks[q][s % len(ranks[q])]
            b = dict(a, now=np.full(nq, W.NOW0 + s, np.int64))
            o = co.do_limit(b, n, nq, args.n_rules)
            if s == steps - 1:
                last[q] = {k: np.array(v) for k, v in o.items()}
    co.close()
    return last, ranks[0][0][1]


@pytest.mark.parametrize("config,world", [("c1", 1), ("c2", 1), ("c2u", 1), ("c1", 2)])
def test_selfcheck_passes_on_exact_answers(config, world):
    args, T, steps = _args(config), 20_000, 7
    sampler = W.ZipfSampler(world * T, 1.1) if config != "c1" else None
    last, n = _full_run(args, T, world, steps, sampler)
    for rank in range(world):
        chk = bench.verify(args, W, last[rank], steps - 1, n, world, rank, T, W.NOW0, sampler, modulus=16)
        assert chk["verified"] and chk["checked"] > 0, chk


@pytest.mark.parametrize("field", ["limit_remaining", "code", "stats"])
def test_selfcheck_fails_on_one_wrong_answer(field):
    args, T, steps = _args("c2"), 20_000, 5
    sampler = W.ZipfSampler(T, 1.1)
    last, n = _full_run(args, T, 1, steps, sampler)
    got = {k: v.copy() for k, v in last[0].items()}
    a, _, _, ten = bench.make_batches(args, W, 0, T, sampler)[(steps - 1) % args.distinct_batches]
    i = int(np.nonzero((ten % 16 == 77 % 16)[a["req_idx"]])[0][-1])  # a descriptor of the checked subset
    if field == "limit_remaining":
        got[field][i] ^= 1
    elif field == "code":
        got[field][i] = 3 - got[field][i]
    else:
        got["stats"][0] -= 1  # one hit lost
    chk = bench.verify(args, W, got, steps - 1, n, 1, 0, T, W.NOW0, sampler, modulus=16)
    assert not chk["verified"] and chk["mismatches"], chk


def test_cpu_share_reports_a_basis():
    s = bench.cpu_share()
    assert s["cores"] >= 1 and s["cores"] <= s["affinity_cpus"] and s["basis"]
