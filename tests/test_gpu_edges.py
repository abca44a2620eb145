"""Edge cases of the boundary, each against the C oracle: empty batches on
every entry point, requests without descriptors, the longest stem the ABI
takes (65535 bytes) and one past it (that descriptor's RL_E_INVALID), a batch
of exactly max_batch descriptors and one more (RL_E_CAPACITY at the call),
and the stats paths on both sides of the LDS rule table (512 rules: block
tables in LDS; 513: global atomics)."""
import numpy as np
import pytest

from oracle import c_oracle
from ratelimit_amd import abi, workloads
from ratelimit_amd.limiter import Backend, PinnedArena, RedisError
from ratelimit_amd.packing import PackedBatch, compact_batch

pytestmark = pytest.mark.gpu

NOW0 = workloads.NOW0


def _batch(stems, req, nq, units=None, limits=None, hits=None, rules=None, now=NOW0):
    n = len(stems)
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum([len(s) for s in stems])
    return {"stem_bytes": np.frombuffer(b"".join(stems) or b"\0\0\0\0", np.uint8).copy(), "stem_off": off,
            "now": np.full(nq, now, np.int64), "req_idx": np.asarray(req, np.uint32),
            "unit": np.asarray(units if units is not None else [1] * n, np.uint8), "flags": np.zeros(n, np.uint8),
            "limit": np.asarray(limits if limits is not None else [5] * n, np.uint32),
            "hits": np.asarray(hits if hits is not None else [1] * n, np.uint32),
            "rule_id": np.asarray(rules if rules is not None else [0] * n, np.uint32)}


def _same(g, o, keep=None):
    keep = slice(None) if keep is None else keep
    for k in ("code", "limit_remaining", "reset_s"):
        assert np.array_equal(np.asarray(g[k])[keep], o[k]), k
    assert np.array_equal(g["stats"], o["stats"])


def test_gpu_empty_batches_on_every_entry_point():
    be = Backend(0.8, True, table_slots=1 << 14, max_batch=1 << 12, max_rules=8)
    a = _batch([], [], 0)
    g = be.do_limit_arrays(a, 0, 0, 2)
    assert g["stats"].sum() == 0
    arena = PinnedArena()
    pb = PackedBatch({k: arena.like(v) for k, v in a.items()}, 0, 0, 2)
    out = {k: arena.like(v) for k, v in pb.alloc_result().items()}
    keep = [be.do_limit_host_async(pb, out)]
    cb = compact_batch(a, 0, 0, 2, alloc=lambda nb: arena.array(nb, np.uint8))
    cout = {k: arena.like(v) for k, v in cb.alloc_result().items()}
    keep.append(be.do_limit_compact_async(cb, cout))
    be.synchronize()
    assert out["stats"].sum() == 0 and cout["stats"].sum() == 0
    # and the table still answers afterwards
    b, n, nq, nr = workloads.c1_batch(np.arange(100), NOW0)
    co = c_oracle.COracle(0.8, True)
    _same(be.do_limit_arrays(b, n, nq, nr), co.do_limit(b, n, nq, nr))
    co.close()
    be.close()
    arena.close()


def test_gpu_requests_without_descriptors():
    """Requests 0, 3 and 4 carry no descriptor (their limits were nil:
    answered host-side, base_limiter.go:78-81); the others' clocks differ."""
    stems = [b"dom_k_%d_" % (i % 5) for i in range(12)]
    req = [1, 1, 2, 2, 2, 5, 5, 6, 6, 6, 6, 7]
    a = _batch(stems, req, 8, hits=[2] * 12)
    a["now"] = NOW0 + np.arange(8, dtype=np.int64)
    for lc in (False, True):
        be = Backend(0.8, lc, table_slots=1 << 14, max_batch=1 << 12, max_rules=8)
        co = c_oracle.COracle(0.8, lc)
        for _ in range(3):
            _same(be.do_limit_arrays(a, 12, 8, 1), co.do_limit(a, 12, 8, 1))
        be.close()
        co.close()


def test_gpu_longest_stem_and_one_past_it():
    long_ok = bytes(np.random.default_rng(1).integers(97, 123, 65535).astype(np.uint8))
    too_long = long_ok + b"z"
    stems = [b"short_a_", long_ok, too_long, long_ok, b"short_a_"]
    a = _batch(stems, [0, 1, 2, 3, 4], 5, limits=[1] * 5)
    be = Backend(0.8, False, table_slots=1 << 14, max_batch=1 << 12, max_rules=8, max_stem_bytes=1 << 19)
    co = c_oracle.COracle(0.8, False)
    g = be.do_limit_arrays(a, 5, 5, 1, isolate=True)
    keep = np.array([True, True, False, True, True])
    assert g["status"][2] == abi.RL_E_INVALID and (g["status"][keep] == 0).all()
    from test_gpu_robustness import _drop
    o = co.do_limit(*_drop(a, 5, 5, keep), 1)
    _same(g, o, keep)
    assert list(g["code"][keep]) == [1, 1, 2, 2]  # OK, OK, OVER_LIMIT, OVER_LIMIT (RateLimitResponse_Code)
    be.close()
    co.close()


def test_gpu_max_batch_exactly_and_one_more():
    mb = 1 << 12
    be = Backend(0.8, False, table_slots=1 << 14, max_batch=mb, max_rules=8)
    co = c_oracle.COracle(0.8, False)
    a, n, nq, nr = workloads.c1_batch(np.arange(mb // 2), NOW0)
    assert n == mb
    _same(be.do_limit_arrays(a, n, nq, nr), co.do_limit(a, n, nq, nr))
    b, n2, nq2, _ = workloads.c1_batch(np.arange(mb // 2 + 1), NOW0)
    with pytest.raises(RedisError) as e:
        be.do_limit_arrays(b, n2, nq2, nr)
    assert "max_batch" in str(e.value)
    # the ctx keeps working after the refused call
    _same(be.do_limit_arrays(a, n, nq, nr), co.do_limit(a, n, nq, nr))
    be.close()
    co.close()


@pytest.mark.parametrize("n_rules", [512, 513])
def test_gpu_stats_on_both_sides_of_the_lds_rule_table(n_rules):
    """Per-rule stats for n_rules = 512 (block tables in LDS, striped) and 513
    (global atomics), every rule hit, hot and cold stems mixed."""
    rng = np.random.default_rng(n_rules)
    n, nq = 20_000, 10_000
    ten = rng.integers(0, 3000, n)
    stems = [b"tenant_%d_" % t for t in ten]
    req = np.sort(rng.integers(0, nq, n)).astype(np.uint32)
    rules = rng.integers(0, n_rules, n).astype(np.uint32)
    rules[:n_rules] = np.arange(n_rules)
    a = _batch(stems, req, nq, units=rng.integers(1, 3, n), limits=rng.integers(0, 20, n),
               hits=rng.integers(0, 4, n), rules=rules)
    be = Backend(0.8, True, table_slots=1 << 16, max_batch=1 << 15, max_rules=1024)
    co = c_oracle.COracle(0.8, True)
    for k in range(2):
        a["now"] = np.full(nq, NOW0 + k, np.int64)
        _same(be.do_limit_arrays(a, n, nq, n_rules), co.do_limit(a, n, nq, n_rules))
    be.close()
    co.close()
