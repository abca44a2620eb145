"""Host packer: DoLimit calls -> one struct-of-arrays rl_batch (numpy, host memory).

This is the Python twin of the Go adapter's packer: for every
in-flight ``DoLimit(request, limits)`` call it
  * drops nil-limit descriptors (they answer {OK, nil, 0} host-side,
    base_limiter.go:78-81 / cache_key.go:51-56),
  * rejects UNKNOWN units up front (utils.UnitToDivider panics, utilities.go:29),
  * builds the key stem prefix ‖ domain ‖ '_' ‖ Σ(key ‖ '_' ‖ value ‖ '_')
    (cache_key.go:62-71) — the window suffix is added on the GPU,
  * interns limit.Stats.Key into a dense rule id (stats.RateLimitStats identity).
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi


class RuleInterner:
    """limit.Stats.Key -> dense rule id (stable across batches)."""

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.keys: List[str] = []

    def intern(self, key: str) -> int:
        i = self.ids.get(key)
        if i is None:
            i = len(self.keys)
            self.ids[key] = i
            self.keys.append(key)
        return i


def stem_of(prefix: str, domain: str, entries: Sequence[Tuple[str, str]]) -> bytes:
    parts = [prefix, domain, "_"]
    for k, v in entries:
        parts += [k, "_", v, "_"]
    return "".join(parts).encode("utf-8")


@dataclass
class PackedBatch:
    arrays: Dict[str, np.ndarray]
    n: int
    n_requests: int
    n_rules: int
    # (call index, descriptor index) for each packed descriptor
    origin: List[Tuple[int, int]] = field(default_factory=list)

    def batch_struct(self):
        return abi.make_batch_struct(self.arrays, self.n, self.n_requests, self.n_rules)

    def alloc_result(self, isolate: bool = False, reset: bool = True):
        """reset False: no reset_s array (host-buffer entry points then leave
        DurationUntilReset to the caller, as utils.CalculateReset computes it)."""
        out = {"code": np.zeros(max(self.n, 1), np.uint8),
               "limit_remaining": np.zeros(max(self.n, 1), np.uint32),
               "stats": np.zeros(max(self.n_rules, 1) * abi.RL_NUM_STATS, np.uint64)}
        if reset:
            out["reset_s"] = np.zeros(max(self.n, 1), np.uint32)
        if isolate:
            out["status"] = np.zeros(max(self.n, 1), np.uint8)
        return out


def arrays_from_lists(stems: List[bytes], now: Sequence[int], req_idx, unit, flags, limit, hits,
                      rule_id) -> Dict[str, np.ndarray]:
    n = len(stems)
    off = np.zeros(n + 1, np.uint32)
    if n:
        off[1:] = np.cumsum([len(s) for s in stems], dtype=np.uint64).astype(np.uint32)
    blob = np.frombuffer(b"".join(stems), np.uint8).copy() if n else np.zeros(1, np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, np.uint8)
    return {"stem_bytes": blob, "stem_off": off,
            "now": np.asarray(now, np.int64).reshape(-1) if len(now) else np.zeros(1, np.int64),
            "req_idx": np.asarray(req_idx, np.uint32), "unit": np.asarray(unit, np.uint8),
            "flags": np.asarray(flags, np.uint8), "limit": np.asarray(limit, np.uint32),
            "hits": np.asarray(hits, np.uint32), "rule_id": np.asarray(rule_id, np.uint32)}


def pack_calls(calls, prefix: str, interner: RuleInterner, n_rules: Optional[int] = None) -> PackedBatch:
    """calls: sequence of (request, limits, now) in arrival order.

    ``request`` / ``limits`` follow the reference's data model (RateLimitRequest with
    .domain/.descriptors[.entries]/.hits_addend, RateLimit with .limit/.stats/.shadow_mode).
    """
    stems, req_idx, unit, flags, limit, hits, rule_id, origin = [], [], [], [], [], [], [], []
    now_list = []
    for c, (request, limits, now) in enumerate(calls):
        if len(request.descriptors) != len(limits):
            raise AssertionError("len(descriptors) != len(limits)")  # base_limiter.go:47
        q = len(now_list)
        now_list.append(int(now))
        h = int(request.hits_addend)
        for i, (d, lim) in enumerate(zip(request.descriptors, limits)):
            if lim is None:
                continue
            u = int(lim.limit.unit)
            if u not in (1, 2, 3, 4):
                raise RuntimeError("should not get here")  # utils.UnitToDivider panic
            stems.append(stem_of(prefix, request.domain, d.entries))
            req_idx.append(q)
            unit.append(u)
            flags.append(abi.RL_FLAG_SHADOW if lim.shadow_mode else 0)
            limit.append(int(lim.limit.requests_per_unit))
            hits.append(h)
            rule_id.append(interner.intern(lim.stats.key))
            origin.append((c, i))
    arrays = arrays_from_lists(stems, now_list, req_idx, unit, flags, limit, hits, rule_id)
    nr = len(interner.keys) if n_rules is None else n_rules
    return PackedBatch(arrays, len(stems), len(now_list), nr, origin)


def slice_requests(arrays: Dict[str, np.ndarray], n: int, n_requests: int, r0: int, r1: int):
    """Requests [r0, r1) of a packed batch as a packed batch of its own (request
    indices and stem offsets rebased): how a node batcher hands each GPU rank a
    contiguous slice of the arrival order (ratelimit_amd/sharded.py)."""
    req = arrays["req_idx"][:n]
    d0, d1 = (int(x) for x in np.searchsorted(req, [r0, r1], side="left"))
    off = arrays["stem_off"]
    s0, s1 = int(off[d0]), int(off[d1])
    out = {"stem_bytes": np.ascontiguousarray(arrays["stem_bytes"][s0:s1]) if s1 > s0 else np.zeros(4, np.uint8),
           "stem_off": (off[d0:d1 + 1].astype(np.int64) - s0).astype(np.uint32),
           "now": np.ascontiguousarray(arrays["now"][r0:r1]) if r1 > r0 else np.zeros(1, np.int64),
           "req_idx": (req[d0:d1].astype(np.int64) - r0).astype(np.uint32)}
    for k in ("unit", "flags", "limit", "hits", "rule_id"):
        out[k] = np.ascontiguousarray(arrays[k][d0:d1])
    return out, d1 - d0, r1 - r0


@dataclass
class CompactBatch:
    """An rl_batch_compact: one contiguous buffer (``buf``, uint8) and the byte
    offsets of its sections (include/ratelimit_hip.h)."""
    buf: np.ndarray
    n: int
    n_requests: int
    n_rules: int
    n_limits: int
    offsets: Dict[str, int]

    def struct(self):
        s = abi.RlBatchCompact()
        s.n, s.n_requests, s.n_rules, s.n_limits = self.n, self.n_requests, self.n_rules, self.n_limits
        s.buf = abi.ptr(self.buf)
        s.buf_bytes = int(self.buf.size)
        for k, v in self.offsets.items():
            setattr(s, k, int(v))
        return s

    def alloc_result(self, isolate: bool = False, reset: bool = True):
        return PackedBatch({}, self.n, self.n_requests, self.n_rules).alloc_result(isolate, reset)


def compact_batch(arrays: Dict[str, np.ndarray], n: int, n_requests: int, n_rules: int, alloc=None) -> CompactBatch:
    """The compact (PCIe) layout of a packed batch: per request its clock (u32),
    HitsAddend and first descriptor, per descriptor its stem and an index into
    the table of the batch's distinct (limit, rule, unit, flags). `hits` must be
    one value per request (HitsAddend is a request field). alloc(nbytes) -> a
    uint8 array for the buffer (default numpy; PinnedArena.array for pinned)."""
    req = np.asarray(arrays["req_idx"][:n], np.int64)
    hits_d = np.asarray(arrays["hits"][:n], np.uint32)
    first = np.searchsorted(req, np.arange(n_requests + 1), side="left").astype(np.uint32)
    if n and np.any(hits_d != np.asarray(arrays["hits"], np.uint32)[np.minimum(first[req], n - 1)]):
        raise ValueError("hits differ inside a request (HitsAddend is per request)")
    hits_q = np.zeros(n_requests, np.uint32)
    has = first[1:] > first[:-1]
    hits_q[has] = hits_d[first[:-1][has]]
    key = np.zeros(n, abi.LIMIT_DTYPE)
    key["requests_per_unit"] = arrays["limit"][:n]
    key["rule_id"] = arrays["rule_id"][:n]
    key["unit"] = arrays["unit"][:n]
    key["flags"] = arrays["flags"][:n]
    table, idx = np.unique(key, return_inverse=True)
    if table.size > 65536:
        raise ValueError("more than 65536 distinct limits in one batch")
    stem_off = np.asarray(arrays["stem_off"][:n + 1], np.uint32)
    nb = int(stem_off[n]) if n else 0
    now = np.asarray(arrays["now"][:n_requests], np.int64)
    sections = [("stem_off", stem_off), ("req_first", first), ("now", now.astype(np.uint32)), ("hits", hits_q),
                ("limits", table), ("limit_idx", idx.astype(np.uint16)),
                ("stem_bytes", np.asarray(arrays["stem_bytes"][:nb], np.uint8))]
    offsets, pos = {}, 0
    for k, a in sections:
        offsets[k] = pos
        pos += (a.nbytes + 3) & ~3
    buf = np.zeros(max(pos, 4), np.uint8) if alloc is None else alloc(max(pos, 4))
    for k, a in sections:
        buf[offsets[k]:offsets[k] + a.nbytes] = np.frombuffer(a.tobytes(), np.uint8)
    return CompactBatch(buf[:max(pos, 4)], n, n_requests, n_rules, int(table.size), offsets)


@dataclass
class PrefixedBatch:
    """An rl_batch_prefixed: one contiguous buffer (``buf``, uint8) and the byte
    offsets of its sections (include/ratelimit_hip.h)."""
    buf: np.ndarray
    n: int
    n_requests: int
    n_rules: int
    n_limits: int
    offsets: Dict[str, int]

    def struct(self):
        s = abi.RlBatchPrefixed()
        s.n, s.n_requests, s.n_rules, s.n_limits = self.n, self.n_requests, self.n_rules, self.n_limits
        s.buf = abi.ptr(self.buf)
        s.buf_bytes = int(self.buf.size)
        for k, v in self.offsets.items():
            setattr(s, k, int(v))
        return s

    def alloc_result(self, isolate: bool = False, reset: bool = True):
        return PackedBatch({}, self.n, self.n_requests, self.n_rules).alloc_result(isolate, reset)

    def section(self, name: str, dtype, count: int) -> np.ndarray:
        o = self.offsets[name]
        return np.frombuffer(self.buf[o:o + count * np.dtype(dtype).itemsize].tobytes(), dtype)

    def tiles(self) -> int:
        return (self.n_requests + abi.RL_PREFIXED_TILE - 1) // abi.RL_PREFIXED_TILE


def _request_lcp(stems2d: np.ndarray, lens: np.ndarray, first: np.ndarray, req: np.ndarray, n_requests: int,
                 cap: int) -> np.ndarray:
    """Per request: the longest prefix every one of its descriptors' stems
    starts with (at most ``cap`` bytes; 0 for a request without descriptors)."""
    n = lens.size
    plen = np.zeros(n_requests, np.int64)
    if n == 0:
        return plen
    head = first[req]                                  # first descriptor of each descriptor's request
    L = stems2d.shape[1]
    diff = stems2d != stems2d[head]
    col = np.arange(L)[None, :]
    diff |= col >= np.minimum(lens, lens[head])[:, None]
    lcp = np.where(diff.any(axis=1), diff.argmax(axis=1), L)
    has = first[1:] > first[:-1]
    starts = first[:-1][has]
    plen[has] = np.minimum.reduceat(lcp, starts)
    return np.minimum(plen, cap)


def prefixed_batch(arrays: Dict[str, np.ndarray], n: int, n_requests: int, n_rules: int, alloc=None,
                   max_prefix: int = 255) -> PrefixedBatch:
    """The prefix-shared (PCIe) layout of a packed batch: per request the bytes
    all its descriptors' stems start with (at most ``max_prefix``), stored once,
    with the request's clock and HitsAddend; per descriptor its remaining
    suffix and an index into the table of the batch's distinct (limit, rule,
    unit, flags); the tile index of starting offsets. ``hits`` must be one value
    per request (HitsAddend is a request field). alloc(nbytes) -> a uint8 array
    for the buffer (default numpy; PinnedArena.array for pinned)."""
    if not 0 <= max_prefix <= 255:
        raise ValueError("max_prefix must be 0..255")
    req = np.asarray(arrays["req_idx"][:n], np.int64)
    first = np.searchsorted(req, np.arange(n_requests + 1), side="left").astype(np.int64)
    hits_d = np.asarray(arrays["hits"][:n], np.uint32)
    if n and np.any(hits_d != hits_d[first[req]]):
        raise ValueError("hits differ inside a request (HitsAddend is per request)")
    nd = np.diff(first)
    if nd.size and nd.max() > 0xFFFF:
        raise ValueError("more than 65535 descriptors in one request")
    hits_q = np.zeros(n_requests, np.uint32)
    has = nd > 0
    hits_q[has] = hits_d[first[:-1][has]]
    key = np.zeros(n, abi.LIMIT_DTYPE)
    key["requests_per_unit"] = arrays["limit"][:n]
    key["rule_id"] = arrays["rule_id"][:n]
    key["unit"] = arrays["unit"][:n]
    key["flags"] = arrays["flags"][:n]
    table, idx = np.unique(key, return_inverse=True)
    if table.size > 65536:
        raise ValueError("more than 65536 distinct limits in one batch")
    off = np.asarray(arrays["stem_off"][:n + 1], np.int64)
    lens = np.diff(off) if n else np.zeros(0, np.int64)
    blob = np.asarray(arrays["stem_bytes"], np.uint8)
    Lmax = int(lens.max()) if n else 0
    # stems as zero-padded rows (one row per descriptor)
    stems2d = np.zeros((n, max(Lmax, 1)), np.uint8)
    if n:
        cols = np.arange(max(Lmax, 1))[None, :]
        m = cols < lens[:, None]
        stems2d[m] = blob[(off[:-1, None] + cols)[m]]
    plen = _request_lcp(stems2d, lens, first, req, n_requests, max_prefix)
    pl_d = plen[req] if n else np.zeros(0, np.int64)
    slen = lens - pl_d
    if n and slen.max() > 0xFFFF:
        raise ValueError("a suffix longer than 65535 bytes")
    cols = np.arange(max(Lmax, 1))[None, :]
    prefix_bytes = stems2d[first[:-1][has]][cols < plen[has][:, None]] if n else np.zeros(0, np.uint8)
    suffix_bytes = stems2d[(cols >= pl_d[:, None]) & (cols < lens[:, None])] if n else np.zeros(0, np.uint8)
    reqw = (nd.astype(np.uint32) | (plen.astype(np.uint32) << 16)).astype(np.uint32)
    descw = (idx.astype(np.uint32) | (slen.astype(np.uint32) << 16)).astype(np.uint32)
    # tile index: {first descriptor, prefix byte, suffix byte, stem byte} per tile of requests
    T = (n_requests + abi.RL_PREFIXED_TILE - 1) // abi.RL_PREFIXED_TILE
    cut = np.minimum(np.arange(T + 1, dtype=np.int64) * abi.RL_PREFIXED_TILE, n_requests)
    cum_p = np.concatenate([[0], np.cumsum(plen)])
    cum_s = np.concatenate([[0], np.cumsum(slen)])
    index = np.stack([first[cut], cum_p[cut], cum_s[first[cut]], off[first[cut]] - off[0] if n else first[cut] * 0],
                     axis=1).astype(np.uint32).reshape(-1)
    now = np.asarray(arrays["now"][:n_requests], np.int64).astype(np.uint32)
    sections = [("index", index), ("req", reqw), ("now", now), ("hits", hits_q), ("limits", table),
                ("desc", descw), ("prefix_bytes", prefix_bytes.astype(np.uint8)),
                ("suffix_bytes", suffix_bytes.astype(np.uint8))]
    offsets, pos = {}, 0
    for k, a in sections:
        offsets[k] = pos
        pos += (a.nbytes + 3) & ~3
    buf = np.zeros(max(pos, 4), np.uint8) if alloc is None else alloc(max(pos, 4))
    for k, a in sections:
        buf[offsets[k]:offsets[k] + a.nbytes] = np.frombuffer(a.tobytes(), np.uint8)
    return PrefixedBatch(buf[:max(pos, 4)], n, n_requests, n_rules, int(table.size), offsets)


def unprefix(pb: PrefixedBatch) -> Dict[str, np.ndarray]:
    """The rl_batch arrays a prefix-shared batch stands for (the format's
    definition, restated on the host for the CPU tests; k_unpack_prefixed does
    this on the GPU). Raises ValueError on an index that does not match."""
    n, nq = pb.n, pb.n_requests
    T = pb.tiles()
    index = pb.section("index", np.uint32, 4 * (T + 1)).reshape(T + 1, 4).astype(np.int64)
    reqw = pb.section("req", np.uint32, nq)
    descw = pb.section("desc", np.uint32, n)
    nd = (reqw & 0xFFFF).astype(np.int64)
    plen = ((reqw >> 16) & 0xFF).astype(np.int64)
    if np.any(reqw >> 24):
        raise ValueError("reserved request bits set")
    tot = index[T]
    if nd.sum() != n or tot[0] != n or index[0].any():
        raise ValueError("index does not match the descriptors")
    pre = pb.section("prefix_bytes", np.uint8, int(tot[1])).tobytes()
    suf = pb.section("suffix_bytes", np.uint8, int(tot[2])).tobytes()
    table = pb.section("limits", abi.LIMIT_DTYPE, pb.n_limits)
    stems, req_idx = [], []
    p = s = d = 0
    for q in range(nq):
        if q % abi.RL_PREFIXED_TILE == 0:
            t = q // abi.RL_PREFIXED_TILE
            if tuple(index[t][:3]) != (d, p, s) or index[t][3] != sum(len(x) for x in stems):
                raise ValueError("index entry %d does not match" % t)
        P = pre[p:p + plen[q]]
        p += plen[q]
        for _ in range(nd[q]):
            sl = int(descw[d] >> 16)
            stems.append(P + suf[s:s + sl])
            s += sl
            req_idx.append(q)
            d += 1
    if (p, s) != (tot[1], tot[2]) or tot[3] != sum(len(x) for x in stems):
        raise ValueError("index totals do not match")
    k = (descw & 0xFFFF).astype(np.int64)
    ok = k < pb.n_limits
    kk = np.where(ok, k, 0)
    lim = table[kk] if pb.n_limits else np.zeros(n, abi.LIMIT_DTYPE)
    hits_q = pb.section("hits", np.uint32, nq)
    out = arrays_from_lists(stems, pb.section("now", np.uint32, nq).astype(np.int64), req_idx,
                            np.where(ok, lim["unit"], 0), np.where(ok, lim["flags"], 0),
                            np.where(ok, lim["requests_per_unit"], 0), hits_q[np.asarray(req_idx, np.int64)],
                            np.where(ok, lim["rule_id"], 0))
    return out


# ---------------------------------------------------------------------------
# The Go batcher's own packing rules (go/src/gpu/cache_impl.go shared / pack,
# go/src/gpu/gpu.go PrefixedBatch.Begin / Add / Seal), restated so that the
# exact layout the Go adapter builds runs through the C ABI in the GPU tests:
#  * nil limits are not packed (their status is {OK, nil, 0} host-side,
#    base_limiter.go:78-81); UNKNOWN units panic (utilities.go:29);
#  * a request's shared prefix is cut at ENTRY granularity: prefix ‖ domain ‖
#    '_' plus the leading entries every packed descriptor of the request
#    carries (cache_impl.go:231-265), then capped at 255 bytes;
#  * the limit table is deduplicated on (RequestsPerUnit, rule id, Unit,
#    ShadowMode) in first-seen order (gpu.go:308-323), at most max_limits;
#  * the buffer's sections are index, req, now, hits, desc, prefix, suffix,
#    limits, abutting at 4-byte alignment (gpu.go Begin), and buf_bytes ends
#    at the used limit entries (Seal);
#  * HitsAddend goes as the request carries it (the library applies
#    utils.Max(1, h)); `now` as uint32.
# go_statuses is cache_impl.go's finish: DurationUntilReset from the
# request's clock (utils.CalculateReset) and one failed descriptor failing its
# whole call.
# ---------------------------------------------------------------------------
GO_MAX_PREFIX = 255


def _go_shared(prefix: str, request, limits) -> Tuple[int, int, int]:
    """cache_impl.go shared(): (packed descriptors, shared prefix bytes, packed stems' bytes)."""
    head = len(prefix.encode()) + len(request.domain.encode()) + 1
    n = common = total = 0
    ref = None
    for d, lim in zip(request.descriptors, limits):
        if lim is None:
            continue
        total += head + sum(len(k.encode()) + len(v.encode()) + 2 for k, v in d.entries)
        if n == 0:
            ref, common = list(d.entries), len(d.entries)
        else:
            k = 0
            while k < common and k < len(d.entries) and tuple(d.entries[k]) == tuple(ref[k]):
                k += 1
            common = k
        n += 1
    if n == 0:
        return 0, 0, 0
    shared = head + sum(len(k.encode()) + len(v.encode()) + 2 for k, v in ref[:common])
    return n, min(shared, GO_MAX_PREFIX), total


def go_prefixed_batch(calls, prefix: str, interner: RuleInterner, n_rules: Optional[int] = None,
                      max_limits: int = 65536, alloc=None):
    """calls: (request, limits, now) in arrival order -> (PrefixedBatch, where),
    where[c][i] = the packed index of descriptor i of call c, -1 for a nil limit."""
    sizes = [_go_shared(prefix, req, lims) for req, lims, _ in calls]
    nq = len(calls)
    n = sum(s[0] for s in sizes)
    p_bytes = sum(s[1] for s in sizes)
    s_bytes = sum(s[2] - s[0] * s[1] for s in sizes)
    tiles = (nq + abi.RL_PREFIXED_TILE - 1) // abi.RL_PREFIXED_TILE
    a4 = lambda x: (x + 3) & ~3
    offsets, pos = {}, 0
    for name, nb in (("index", 16 * (tiles + 1)), ("req", 4 * nq), ("now", 4 * nq), ("hits", 4 * nq),
                     ("desc", 4 * n), ("prefix_bytes", p_bytes), ("suffix_bytes", s_bytes)):
        offsets[name] = pos
        pos += a4(nb)
    offsets["limits"] = pos
    cap = pos + 12 * max_limits
    buf = np.zeros(max(cap, 4), np.uint8) if alloc is None else alloc(max(cap, 4))
    buf[:] = 0
    index = np.zeros(4 * (tiles + 1), np.uint32)
    reqw = np.zeros(nq, np.uint32)
    nows = np.zeros(nq, np.uint32)
    hitw = np.zeros(nq, np.uint32)
    descw = np.zeros(n, np.uint32)
    pre, suf = bytearray(), bytearray()
    table = {}  # Limit -> index, first-seen order
    where = []
    d = n_stem = 0
    for q, ((req, lims, now), (_nd, p_len, _tot)) in enumerate(zip(calls, sizes)):
        if len(req.descriptors) != len(lims):
            raise AssertionError("len(descriptors) != len(limits)")  # base_limiter.go:47
        if q % abi.RL_PREFIXED_TILE == 0:
            t = 4 * (q // abi.RL_PREFIXED_TILE)
            index[t:t + 4] = (d, len(pre), len(suf), n_stem)
        idx, suffixes = [], []
        stem_head = None
        for i, (desc, lim) in enumerate(zip(req.descriptors, lims)):
            if lim is None:
                idx.append(-1)
                continue
            u = int(lim.limit.unit)
            if u not in (1, 2, 3, 4):
                raise RuntimeError("should not get here")  # utils.UnitToDivider panic
            stem = stem_of(prefix, req.domain, desc.entries)
            if stem_head is None:
                stem_head = stem[:p_len]
            key = (int(lim.limit.requests_per_unit), interner.intern(lim.stats.key), u, bool(lim.shadow_mode))
            k = table.get(key)
            if k is None:
                if len(table) == max_limits:
                    raise ValueError("gpu: more distinct limits than the batch's table holds")
                k = table[key] = len(table)
            sfx = stem[p_len:]
            if len(sfx) > 0xFFFF:
                raise ValueError("gpu: descriptor suffix longer than 65535 bytes")
            idx.append(d + len(suffixes))
            suffixes.append((k, sfx, len(stem)))
        if len(suffixes) > 0xFFFF or p_len > GO_MAX_PREFIX:
            raise ValueError("gpu: request does not fit the prefixed layout")
        reqw[q] = len(suffixes) | (p_len << 16)
        nows[q] = int(now) & 0xFFFFFFFF
        hitw[q] = int(req.hits_addend)
        if suffixes:
            pre += stem_head
        for k, sfx, sl in suffixes:
            descw[d] = k | (len(sfx) << 16)
            suf += sfx
            n_stem += sl
            d += 1
        where.append(idx)
    t = 4 * tiles
    index[t:t + 4] = (d, len(pre), len(suf), n_stem)
    keys = sorted(table, key=table.get)
    lim_arr = np.zeros(len(keys), abi.LIMIT_DTYPE)
    lim_arr["requests_per_unit"] = [k[0] for k in keys]
    lim_arr["rule_id"] = [k[1] for k in keys]
    lim_arr["unit"] = [k[2] for k in keys]
    lim_arr["flags"] = [abi.RL_FLAG_SHADOW if k[3] else 0 for k in keys]
    for name, a in (("index", index), ("req", reqw), ("now", nows), ("hits", hitw), ("desc", descw),
                     ("prefix_bytes", np.frombuffer(bytes(pre), np.uint8)),
                     ("suffix_bytes", np.frombuffer(bytes(suf), np.uint8)), ("limits", lim_arr)):
        raw = np.frombuffer(a.tobytes(), np.uint8)
        buf[offsets[name]:offsets[name] + raw.size] = raw
    used = offsets["limits"] + 12 * len(table)
    nr = len(interner.keys) if n_rules is None else n_rules
    pb = PrefixedBatch(buf[:max(used, 4)], d, nq, nr, len(table), offsets)
    return pb, where


def go_statuses(calls, where, out) -> list:
    """cache_impl.go finish(): per call either its statuses as (code, limit
    remaining, DurationUntilReset seconds or None) per descriptor, or the
    string of the RedisError it panics with (a failed descriptor fails the
    call)."""
    res = []
    for (req, lims, now), idx in zip(calls, where):
        st, failed = [], None
        for i, j in enumerate(idx):
            if j < 0:
                st.append((1, 0, None))  # {OK, nil, 0} (base_limiter.go:78-81)
                continue
            if out.get("status") is not None and out["status"][j] != 0:
                failed = "gpu: descriptor failed (rl_status %d)" % out["status"][j]
                continue
            div = {1: 1, 2: 60, 3: 3600, 4: 86400}[int(lims[i].limit.unit)]
            st.append((int(out["code"][j]), int(out["limit_remaining"][j]), div - int(now) % div))
        res.append(failed if failed else st)
    return res
