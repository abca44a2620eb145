"""rl_do_limit_prefixed_async: the prefix-shared host batch (the fed path's
densest PCIe layout, include/ratelimit_hip.h).

Each request's shared stem prefix is stored once and each descriptor carries
its suffix; the GPU rebuilds the stems tile by tile from the batcher's index.
Every batch must answer exactly like the same batch as rl_batch arrays (the C
oracle): C1, C2, C2U and C4 streams pipelined from pinned buffers on one and
on 2-3 shards, ragged requests with long stems and capped prefixes, statuses;
a malformed index or reserved bits fail the batch, a section outside the
buffer is refused at the call."""
import numpy as np
import pytest

import streams
from oracle import c_oracle
from ratelimit_amd import abi, workloads
from ratelimit_amd.limiter import Backend, PinnedArena, RedisError
from ratelimit_amd.packing import RuleInterner, pack_calls, prefixed_batch

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
        assert np.array_equal(g["stats"][:nr * abi.RL_NUM_STATS], w["stats"]), i
        if i in isolate:
            assert (g["status"][:n] == 0).all()


def _c4_batches(n_batches=4, n_calls=1500):
    calls = streams.c4_stream(11, n_calls=n_calls)
    interner = RuleInterner()
    step = len(calls) // n_batches
    out = []
    for k in range(n_batches):
        pb = pack_calls(calls[k * step:(k + 1) * step], "", interner)
        out.append((pb.arrays, pb.n, pb.n_requests, None))
    return [(a, n, nq, len(interner.keys)) for a, n, nq, _ in out]


def _mixed_batches():
    z = workloads.ZipfSampler(20_000, 1.1)
    batches = list(workloads.c1_stream(n_tenants=40_000, requests_per_batch=20_003, batches=2))
    batches += list(workloads.c2_stream(n_tenants=20_000, requests_per_batch=30_000, batches=2, sampler=z,
                                        now0=workloads.NOW0 + 2))
    batches += list(workloads.c2u_stream(seed=3, n_tenants=20_000, requests_per_batch=30_000, batches=3,
                                         now0=workloads.NOW0 + 4, sampler=z))
    return batches


def test_gpu_prefixed_c1_layout_is_under_32_bytes_per_decision():
    a, n, nq, nr = workloads.c1_batch(np.arange(100_000), workloads.NOW0)
    pb = prefixed_batch(a, n, nq, nr)
    assert pb.buf.size / n <= 32.0, pb.buf.size / n


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_prefixed_pipeline_matches_oracle(lc):
    """C1, C2 and C2U batches (hot keys, overrides) queued back to back from
    pinned buffers, with a status batch mid-stream."""
    batches = _mixed_batches()
    want = _want(batches, lc)
    be = Backend(0.8, lc, table_slots=1 << 18, max_batch=1 << 17, max_rules=8)
    arena = PinnedArena()
    keep, got = [], []
    for i, (a, n, nq, nr) in enumerate(batches):
        pb = prefixed_batch(a, n, nq, nr, alloc=lambda nb: arena.array(nb, np.uint8))
        # batch 2 without reset_s (not copied back): the caller's CalculateReset
        out = {k: arena.like(v) for k, v in pb.alloc_result(isolate=(i == 4), reset=(i != 2)).items()}
        keep.append((pb, out, be.do_limit_prefixed_async(pb, out)))
        got.append(out)
    be.synchronize()
    a, n = batches[2][0], batches[2][1]
    div = np.where(a["unit"][:n] == 1, 1, 60)
    now = a["now"][a["req_idx"][:n]]
    got[2]["reset_s"] = (div - now % div).astype(np.uint32)  # utils.CalculateReset (utilities.go:32-36)
    _check(got, want, batches, isolate=(4,))
    be.close()
    arena.close()


@pytest.mark.parametrize("lc", [False, True])
def test_gpu_prefixed_c4_nested_descriptors(lc):
    """C4: nested 4-entry descriptors (shared leading entries), duplicates
    inside a request, shadow, overrides, window rollover."""
    batches = _c4_batches()
    want = _want(batches, lc)
    be = Backend(0.8, lc, table_slots=1 << 16, max_batch=1 << 14, max_rules=64)
    keep, got = [], []
    for a, n, nq, nr in batches:
        pb = prefixed_batch(a, n, nq, nr)
        out = pb.alloc_result()
        keep.append((pb, out, be.do_limit_prefixed_async(pb, out)))
        got.append(out)
    be.synchronize()
    _check(got, want, batches)
    be.close()


def _ragged(seed, nq, lengths, max_desc=5):
    rng = np.random.default_rng(seed)
    stems, req, unit, flags, limit, hits, rule = [], [], [], [], [], [], []
    h = rng.integers(0, 6, nq).astype(np.uint32)
    for q in range(nq):
        head = bytes(rng.integers(97, 100, int(rng.choice(lengths))).astype(np.uint8))
        for _ in range(rng.integers(0, max_desc + 1)):
            tail = bytes(rng.integers(97, 100, int(rng.choice(lengths))).astype(np.uint8))
            s = (head + tail)[:max(1, int(rng.choice(lengths)))] if rng.random() < 0.7 else tail or b"x"
            stems.append(s)
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
    return a, n, nq, 4


@pytest.mark.parametrize("lengths,max_prefix", [((1, 7, 34, 80, 81, 200), 255), ((300, 400, 600), 255),
                                                ((1, 34, 120), 0), ((1, 34, 120), 17)])
def test_gpu_prefixed_ragged_requests_long_stems(lengths, max_prefix):
    """Requests of 0..5 descriptors, stems from 1 to 1200 bytes (long-stem
    arena; tiles whose stems overflow the kernel's LDS assembly), prefixes
    capped at 0 / 17 / 255 bytes, hits per request, shadow flags."""
    batches = [_ragged(7, 3000, lengths)]
    for lc in (False, True):
        want = _want(batches, lc)
        be = Backend(0.8, lc, table_slots=1 << 16, max_batch=1 << 15, max_rules=8, max_stem_bytes=1 << 24)
        a, n, nq, nr = batches[0]
        pb = prefixed_batch(a, n, nq, nr, max_prefix=max_prefix)
        out = pb.alloc_result()
        keep = be.do_limit_prefixed_async(pb, out)
        be.synchronize()
        _check([out], want, batches)
        del keep
        be.close()


def test_gpu_prefixed_bad_limit_index_alone_bad_index_fails_batch():
    a, n, nq, nr = workloads.c1_batch(np.arange(2000), workloads.NOW0)
    want = _want([(a, n, nq, nr)], False)[0]
    be = Backend(0.8, False, table_slots=1 << 16, max_batch=1 << 14, max_rules=8)
    # a limit index past the table: that descriptor's RL_E_INVALID, the rest answered
    pb = prefixed_batch(a, n, nq, nr)
    dw = pb.buf[pb.offsets["desc"]:pb.offsets["desc"] + 4 * n].view(np.uint32)
    dw[10] = (dw[10] & 0xFFFF0000) | 7
    out = pb.alloc_result(isolate=True)
    keep = be.do_limit_prefixed_async(pb, out)
    be.synchronize()
    assert out["status"][10] == abi.RL_E_INVALID and out["code"][10] == 0
    ok = np.ones(n, bool)
    ok[10] = False
    assert (out["status"][ok] == 0).all()
    assert np.array_equal(out["code"][ok], want["code"][ok])
    del keep

    def corrupt(section, word, value):
        pb = prefixed_batch(a, n, nq, nr)
        w = pb.buf[pb.offsets[section]:].view(np.uint32)
        w[word] = value
        return pb

    T = (nq + abi.RL_PREFIXED_TILE - 1) // abi.RL_PREFIXED_TILE
    be.close()
    be = Backend(0.8, False, table_slots=1 << 16, max_batch=1 << 14, max_rules=8)  # (an untouched table)
    bad = [corrupt("index", 4 * 2 + 0, 5),                  # a tile's first descriptor
           corrupt("index", 4 * 3 + 2, 1 << 30),            # a tile's suffix offset past the totals
           corrupt("req", 7, (3 << 16) | 2),                # a request's descriptor count / prefix
           corrupt("req", 9, (1 << 24) | (30 << 16) | 2),   # reserved bits
           corrupt("desc", 11, (5 << 16) | 1)]              # a suffix length (the sums no longer match)
    for pb in bad:
        out = pb.alloc_result()
        keep = be.do_limit_prefixed_async(pb, out)
        with pytest.raises(RedisError):
            be.synchronize()
        del keep
    # the ctx stays usable and the failed batches left the table untouched
    pb = prefixed_batch(a, n, nq, nr)
    out = pb.alloc_result()
    keep = be.do_limit_prefixed_async(pb, out)
    be.synchronize()
    for k in ("code", "limit_remaining", "reset_s"):
        assert np.array_equal(out[k][:n], want[k]), k
    del keep
    # refused at the call: totals that do not end at n, a section outside the buffer
    pb = corrupt("index", 4 * T, n + 1)
    with pytest.raises(RedisError):
        be.do_limit_prefixed_async(pb, pb.alloc_result())
    pb = prefixed_batch(a, n, nq, nr)
    pb.offsets["suffix_bytes"] = pb.buf.size
    with pytest.raises(RedisError):
        be.do_limit_prefixed_async(pb, pb.alloc_result())
    be.close()


@pytest.mark.parametrize("n_shards,lc", [(2, False), (3, True)])
def test_gpu_prefixed_multishard_matches_oracle(n_shards, lc):
    """A ctx hash-sharded over 2-3 tables on cuda:0: each batch is cut at
    request tiles, each shard copies and unpacks its tiles and routes them
    (C1, C2, C2U, C4, a status batch) — answers and summed stats equal the C
    oracle's; a malformed index fails the batch on every shard count."""
    batches = _mixed_batches() + _c4_batches(2, 800)
    want = _want(batches, lc)
    be = Backend(0.8, lc, table_slots=1 << 18, max_batch=1 << 17, max_rules=256, n_shards=n_shards,
                 shard_devices=[0] * n_shards, hash_seed=91)
    arena = PinnedArena()
    keep, got = [], []
    for i, (a, n, nq, nr) in enumerate(batches):
        pb = prefixed_batch(a, n, nq, nr, alloc=lambda nb: arena.array(nb, np.uint8))
        out = {k: arena.like(v) for k, v in pb.alloc_result(isolate=(i == 3)).items()}
        keep.append((pb, out, be.do_limit_prefixed_async(pb, out)))
        got.append(out)
    be.synchronize()
    _check(got, want, batches, isolate=(3,))
    a, n, nq, nr = batches[0]
    pb = prefixed_batch(a, n, nq, nr)
    w = pb.buf[pb.offsets["req"]:].view(np.uint32)
    w[nq // 2] += 1  # one more descriptor in a request than the index holds
    bad_out = pb.alloc_result()
    with pytest.raises(RedisError):
        keep.append(be.do_limit_prefixed_async(pb, bad_out))
        be.synchronize()
    be.close()
    arena.close()


def test_gpu_prefixed_empty_requests_and_empty_batch():
    """Requests without descriptors (their clocks only), a batch of no
    descriptors, and a batch of no requests."""
    a, n, nq, nr = _ragged(3, 700, (5, 40), max_desc=1)
    be = Backend(0.8, True, table_slots=1 << 16, max_batch=1 << 14, max_rules=8)
    want = _want([(a, n, nq, nr)], True)
    pb = prefixed_batch(a, n, nq, nr)
    out = pb.alloc_result()
    keep = [be.do_limit_prefixed_async(pb, out)]
    empty = {k: v[:0] if k not in ("stem_off", "now") else v[:1] for k, v in a.items()}
    empty["stem_off"] = np.zeros(1, np.uint32)
    for nq0 in (0, 5):
        e = dict(empty, now=np.full(max(nq0, 1), workloads.NOW0, np.int64))
        pe = prefixed_batch(e, 0, nq0, nr)
        oe = pe.alloc_result()
        keep.append((pe, oe, be.do_limit_prefixed_async(pe, oe)))
    be.synchronize()
    _check([out], want, [(a, n, nq, nr)])
    be.close()
