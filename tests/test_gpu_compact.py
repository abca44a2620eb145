"""rl_do_limit_compact_async: the host-fed batch in its PCIe layout.

One contiguous buffer per batch (per request: clock, HitsAddend, first
descriptor; per descriptor: stem and a 16-bit index into the batch's table of
distinct limits) must answer exactly like the same batch as rl_batch arrays
(the C oracle), pipelined with other batches, with per-descriptor statuses,
and must reject a malformed request layout."""
import numpy as np
import pytest

from oracle import c_oracle
from ratelimit_amd import abi, workloads
from ratelimit_amd.limiter import Backend, PinnedArena, RedisError
from ratelimit_amd.packing import compact_batch

pytestmark = pytest.mark.gpu


def _want(batches, lc, ps=False):
    co = c_oracle.COracle(0.8, lc, ps)
    out = [co.do_limit(a, n, nq, nr) for a, n, nq, nr in batches]
    co.close()
    return out


def _check(got, want, batches, isolate=()):
    for i, (g, w) in enumerate(zip(got, want)):
        n, nr = batches[i][1], batches[i][3]
        for k in ("code", "limit_remaining", "reset_s"):
            assert np.array_equal(g[k][:n], w[k]), "batch %d: %s differs" % (i, k)
        assert np.array_equal(g["stats"][:nr * abi.RL_NUM_STATS], w["stats"]), (i, g["stats"][:nr * abi.RL_NUM_STATS],
                                                                                w["stats"])
        if i in isolate:
            assert (g["status"][:n] == 0).all()


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_compact_pipeline_matches_oracle(lc):
    """C2 and C2U batches (hot keys, overrides: three limits per batch) queued
    back to back from pinned buffers, with an rl_batch host-fed batch and a
    status batch mid-stream."""
    z = workloads.ZipfSampler(20_000, 1.1)
    batches = list(workloads.c2_stream(n_tenants=20_000, requests_per_batch=30_000, batches=3, sampler=z))
    batches += list(workloads.c2u_stream(seed=3, n_tenants=20_000, requests_per_batch=30_000, batches=4,
                                         now0=workloads.NOW0 + 3, sampler=z))
    want = _want(batches, lc)
    be = Backend(0.8, lc, table_slots=1 << 18, max_batch=1 << 17, max_rules=8)
    arena = PinnedArena()
    keep, got = [], []
    for i, (a, n, nq, nr) in enumerate(batches):
        out = {k: arena.like(v) for k, v in
               compact_batch(a, n, nq, nr).alloc_result(isolate=(i == 5)).items()}
        if i == 2:
            from ratelimit_amd.packing import PackedBatch
            pb = PackedBatch({k: arena.like(v) for k, v in a.items()}, n, nq, nr)
            keep.append((pb, out, be.do_limit_host_async(pb, out)))
        else:
            cb = compact_batch(a, n, nq, nr, alloc=lambda nb: arena.array(nb, np.uint8))
            assert cb.buf.size <= 46.1 * n + 256 or i >= 3  # (C2: 34-B stems, 2 per request)
            keep.append((cb, out, be.do_limit_compact_async(cb, out)))
        got.append(out)
    be.synchronize()
    _check(got, want, batches, isolate=(5,))
    be.close()
    arena.close()


def test_gpu_compact_ragged_requests_and_long_stems():
    """Requests of 0..5 descriptors, stems from 1 to 200 bytes (the arena),
    hits per request, shadow flags: against the C oracle from unpinned memory."""
    rng = np.random.default_rng(7)
    stems, req, unit, flags, limit, hits, rule = [], [], [], [], [], [], []
    nq = 3000
    h = rng.integers(0, 6, nq).astype(np.uint32)
    for q in range(nq):
        for _ in range(rng.integers(0, 6)):
            L = int(rng.choice([1, 7, 34, 80, 81, 200]))
            stems.append(bytes(rng.integers(97, 100, L).astype(np.uint8)))
            req.append(q)
            u = int(rng.integers(1, 5))
            unit.append(u)
            flags.append(int(rng.random() < 0.2))
            limit.append(int(rng.integers(0, 30)))
            hits.append(int(h[q]))
            rule.append(u - 1)
    n = len(stems)
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum([len(s) for s in stems])
    a = {"stem_bytes": np.frombuffer(b"".join(stems), np.uint8).copy(), "stem_off": off,
         "now": np.full(nq, workloads.NOW0, np.int64) + np.arange(nq) // 1000,
         "req_idx": np.array(req, np.uint32), "unit": np.array(unit, np.uint8), "flags": np.array(flags, np.uint8),
         "limit": np.array(limit, np.uint32), "hits": np.array(hits, np.uint32), "rule_id": np.array(rule, np.uint32)}
    batches = [(a, n, nq, 4)]
    for lc in (False, True):
        want = _want(batches, lc)
        be = Backend(0.8, lc, table_slots=1 << 16, max_batch=1 << 15, max_rules=8)
        cb = compact_batch(a, n, nq, 4)
        out = cb.alloc_result()
        keep = be.do_limit_compact_async(cb, out)
        be.synchronize()
        _check([out], want, batches)
        del keep
        be.close()


def test_gpu_compact_bad_limit_index_fails_alone_and_bad_layout_fails_batch():
    a, n, nq, nr = workloads.c1_batch(np.arange(2000), workloads.NOW0)
    want = _want([(a, n, nq, nr)], False)[0]
    be = Backend(0.8, False, table_slots=1 << 16, max_batch=1 << 14, max_rules=8)
    # a limit index past the table: that descriptor's RL_E_INVALID, the rest answered
    cb = compact_batch(a, n, nq, nr)
    li = cb.buf[cb.offsets["limit_idx"]:cb.offsets["limit_idx"] + 2 * n].view(np.uint16)
    li[10] = 7
    out = cb.alloc_result(isolate=True)
    keep = be.do_limit_compact_async(cb, out)
    be.synchronize()
    assert out["status"][10] == abi.RL_E_INVALID and out["code"][10] == 0
    ok = np.ones(n, bool)
    ok[10] = False
    assert (out["status"][ok] == 0).all()
    assert np.array_equal(out["code"][ok], want["code"][ok])
    del keep
    # request ranges that do not cover [0, n): the batch fails at synchronize
    cb = compact_batch(a, n, nq, nr)
    rf = cb.buf[cb.offsets["req_first"]:cb.offsets["req_first"] + 4 * (nq + 1)].view(np.uint32)
    rf[5], rf[6] = rf[6], rf[5]
    out = cb.alloc_result()
    keep = be.do_limit_compact_async(cb, out)
    with pytest.raises(RedisError):
        be.synchronize()
    del keep
    # a section outside the buffer: refused at the call
    cb = compact_batch(a, n, nq, nr)
    cb.offsets["stem_bytes"] = cb.buf.size
    with pytest.raises(RedisError):
        be.do_limit_compact_async(cb, cb.alloc_result())
    be.close()


@pytest.mark.parametrize("n_shards,lc", [(2, False), (3, True)])
def test_gpu_compact_multishard_matches_oracle(n_shards, lc):
    """A ctx hash-sharded over 2-3 tables on cuda:0: each compact batch is cut
    into request-aligned slices, each shard copies and unpacks its slice and
    routes it (C2 and C2U batches, a status batch, ragged slices at the
    request cuts) — answers and summed stats equal the C oracle's."""
    z = workloads.ZipfSampler(20_000, 1.1)
    batches = list(workloads.c2_stream(n_tenants=20_000, requests_per_batch=30_001, batches=2, sampler=z))
    batches += list(workloads.c2u_stream(seed=5, n_tenants=20_000, requests_per_batch=29_999, batches=3,
                                         now0=workloads.NOW0 + 38, sampler=z))
    want = _want(batches, lc)
    be = Backend(0.8, lc, table_slots=1 << 18, max_batch=1 << 17, max_rules=32, n_shards=n_shards,
                 shard_devices=[0] * n_shards, hash_seed=91)
    arena = PinnedArena()
    keep, got = [], []
    for i, (a, n, nq, nr) in enumerate(batches):
        cb = compact_batch(a, n, nq, nr, alloc=lambda nb: arena.array(nb, np.uint8))
        out = {k: arena.like(v) for k, v in cb.alloc_result(isolate=(i == 3)).items()}
        keep.append((cb, out, be.do_limit_compact_async(cb, out)))
        got.append(out)
    be.synchronize()
    _check(got, want, batches, isolate=(3,))
    # a request layout that does not cover [0, n): refused or failed at synchronize, on every shard count
    a, n, nq, nr = batches[0]
    cb = compact_batch(a, n, nq, nr)
    rf = cb.buf[cb.offsets["req_first"]:cb.offsets["req_first"] + 4 * (nq + 1)].view(np.uint32)
    rf[nq // 2], rf[nq // 2 + 1] = rf[nq // 2 + 1], rf[nq // 2]
    bad_out = cb.alloc_result()  # (kept until synchronize, like every output)
    with pytest.raises(RedisError):
        keep.append(be.do_limit_compact_async(cb, bad_out))
        be.synchronize()
    be.close()
    arena.close()
