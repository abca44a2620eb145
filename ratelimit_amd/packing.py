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
