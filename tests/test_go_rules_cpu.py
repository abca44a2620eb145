"""The Go batcher's packing rules (go/src/gpu/cache_impl.go shared / pack,
gpu.go PrefixedBatch.Begin / Add / Seal), restated in
ratelimit_amd.packing.go_prefixed_batch, on the CPU: the batch they build
stands for exactly the rl_batch arrays pack_calls builds (same stems, units,
limits, rules, request indices), with the Go layout's own choices — the shared
prefix cut at entry boundaries and capped at 255 bytes, the limit table in
first-seen order, Go's section order. test_gpu_go_rules.py runs the same
batches on the GPU."""
import numpy as np

import streams
from oracle import oracle as O
from ratelimit_amd import abi
from ratelimit_amd.packing import RuleInterner, go_prefixed_batch, pack_calls, unprefix


def _same_arrays(calls, prefix=""):
    pk = pack_calls(calls, prefix, RuleInterner())
    pb, where = go_prefixed_batch(calls, prefix, RuleInterner())
    u, a, n = unprefix(pb), pk.arrays, pk.n
    assert (pb.n, pb.n_requests) == (n, pk.n_requests)
    for k in ("req_idx", "unit", "flags", "limit", "rule_id"):
        assert np.array_equal(u[k][:n], a[k][:n]), k
    assert np.array_equal(u["stem_off"][:n + 1], a["stem_off"][:n + 1])
    assert bytes(u["stem_bytes"][:u["stem_off"][n]]) == bytes(a["stem_bytes"][:a["stem_off"][n]])
    hq = pb.section("hits", np.uint32, pb.n_requests)
    assert list(hq) == [int(r.hits_addend) for r, _, _ in calls]
    # where: packed index of every non-nil descriptor, in arrival order
    flat = [j for w in where for j in w if j >= 0]
    assert flat == list(range(n))
    assert [j < 0 for w in where for j in w] == [l is None for _, ls, _ in calls for l in ls]
    return pb


def test_go_rules_random_and_c4_streams_stand_for_the_packed_arrays():
    for seed in range(3):
        _same_arrays(streams.random_stream(seed, n_calls=500, p_nil=0.3, p_override=0.2), prefix="pfx:")
    _same_arrays(streams.c4_stream(3, n_calls=700))


def _req_words(pb):
    return pb.section("req", np.uint32, pb.n_requests)


def test_go_rules_prefix_is_cut_at_entries_then_capped_at_255():
    rl = lambda k: O.RateLimit(k, O.RateLimitStats(k), O.Limit(3, O.SECOND), False, False)
    # the two stems share "d_a_xy" byte-wise, but only the domain entry-wise
    c1 = (O.RateLimitRequest("d", [O.Descriptor([("a", "xy1")]), O.Descriptor([("a", "xy2")])], 1),
          [rl("d.a"), rl("d.a")], 100)
    # a shared leading entry: domain + the first entry
    c2 = (O.RateLimitRequest("d", [O.Descriptor([("a", "v"), ("b", "1")]), O.Descriptor([("a", "v"), ("c", "2")])], 1),
          [rl("d.a.b"), rl("d.a.c")], 100)
    # a 400-byte shared entry: capped at 255 bytes
    big = "x" * 400
    c3 = (O.RateLimitRequest("d", [O.Descriptor([("k", big), ("b", "1")]), O.Descriptor([("k", big), ("c", "2")])], 1),
          [rl("d.k.b"), rl("d.k.c")], 100)
    # a nil limit does not take part in the prefix
    c4 = (O.RateLimitRequest("d", [O.Descriptor([("a", "v"), ("b", "1")]), O.Descriptor([("z", "q")]),
                                   O.Descriptor([("a", "v"), ("c", "2")])], 1), [rl("d.a.b"), None, rl("d.a.c")], 100)
    pb = _same_arrays([c1, c2, c3, c4], prefix="p:")
    plen = [int(w >> 16) for w in _req_words(pb)]
    assert plen == [len("p:d_"), len("p:d_a_v_"), 255, len("p:d_a_v_")]


def test_go_rules_limit_table_dedup_first_seen_and_layout_order():
    calls = streams.random_stream(9, n_calls=300, p_override=0.3)
    it = RuleInterner()
    pb, _ = go_prefixed_batch(calls, "", it)
    seen = []
    for req, lims, _ in calls:
        for l in lims:
            if l is None:
                continue
            k = (int(l.limit.requests_per_unit), it.ids[l.stats.key], int(l.limit.unit), bool(l.shadow_mode))
            if k not in seen:
                seen.append(k)
    tab = pb.section("limits", abi.LIMIT_DTYPE, pb.n_limits)
    assert [(int(t["requests_per_unit"]), int(t["rule_id"]), int(t["unit"]), bool(t["flags"])) for t in tab] == seen
    order = ["index", "req", "now", "hits", "desc", "prefix_bytes", "suffix_bytes", "limits"]
    offs = [pb.offsets[k] for k in order]
    assert offs == sorted(offs) and offs[0] == 0
    assert pb.buf.size == pb.offsets["limits"] + 12 * pb.n_limits  # Seal: buf_bytes ends at the used entries
