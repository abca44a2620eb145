// rl_kernels.hip — gfx950 kernels of the fixed-window rate-limit backend.
//
// Pipeline for one batch (inputs already in HBM); stage A (table-free):
//   k_prepare     validate the packed batch; hash every stem (LDS-staged
//                 bytes); pack each descriptor into a 32-B Rec (arrival order)
//   k_part        stable partition of (hash[63:32], index, hits) by the top
//                 10 bits, tile by tile (no look-back; tiles leave via LDS)
//   k_bucket      one workgroup per bucket: gather it, stable LDS sort by the
//                 remaining 22 bits (hot keys of a large bucket: k_big_*,
//                 k_bucket_big), run ids, run bounds and in-run prefix sums of
//                 hits: each stem's descriptors together, in arrival order
//   k_run_check   one stem and one unit per run (else RUN_MULTI); marks the
//                 descriptors of runs (BatchDev::dup)
//   k_split       RUN_MULTI runs of a few single-unit stems -> per-stem runs
//   ---- stage B (the table; batch order) ----
//   k_table       keys seen once (arrival order) and runs of two or more (one
//                 lane per run): probe/insert the (stem, unit) slot of the HBM
//                 table; replay short runs in registers, set up long uniform
//                 runs for the parallel path
//   k_late        the exact path (RUN_MULTI runs k_split left, k_table's
//                 deferrals) + long runs decided in parallel (k_fast_over
//                 first with the local cache on)
//   k_finish      packed results -> code / limit_remaining / reset_s, and the
//                 striped per-block stats -> rl_result.stats
// plus k_sweep (epoch sweep = Redis EXPIRE), k_table_info, debug kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "rl_device.h"
#include "rl_kernels.h"

// Ablation switches for profiling builds only (RL_ABL bits; 0 in the product):
// 1 = no table probe (slot = tag & mask), 2 = no replay body, 4 = no stats flush.
#ifndef RL_ABL
#define RL_ABL 0
#endif

namespace rl {

// ===========================================================================
// k_prepare: validation, stem hashing, record packing (arrival order).
// Each 256-thread block stages the contiguous byte range of its 256 stems in
// LDS with coalesced dword loads, then every lane hashes its own stem from LDS.
// ===========================================================================
constexpr uint32_t HASH_LDS_BYTES = 16384;

__global__ __launch_bounds__(256) void k_prepare(BatchDev b, Rec* __restrict__ rec, uint32_t* __restrict__ keys,
                                                 uint32_t* err, uint32_t* errs, int isolate,
                                                 const int64_t* time_floor, uint32_t* defer_n,
                                                 uint32_t* big_n, uint32_t* work_n, uint32_t* __restrict__ run_flags,
                                                 unsigned long long* num_runs, uint32_t* __restrict__ hit_a,
                                                 unsigned long long* __restrict__ res, uint32_t* sorted_n,
                                                 uint32_t* uniq_n) {
  __shared__ uint32_t lds[HASH_LDS_BYTES / 4 + 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t i = blockIdx.x * 256 + tid;
  uint32_t bad = 0;
  if (i < b.n) run_flags[i] = 0;  // k_run_check ORs run flags in from any block
  if (blockIdx.x == 0 && tid == 0) {  // per-batch counters: RUN_MULTI queue, run ids, large buckets, sorted positions
    *defer_n = 0;
    *num_runs = 0;
    *big_n = 0;
    *work_n = 0;
    *sorted_n = 0;
    *uniq_n = 0;
  }
  const int64_t floor = *time_floor;
  auto time_bad = [&](int64_t t) { return t < 0 || t > (int64_t)NOW_MAX || t < floor; };

  // ---- the descriptor: packed arrays, or (routed owner batch) its wire
  // record, whose stem starts at woff[i] (the lengths of the records before
  // it, summed); chunks arrive in source order, so the stem must lie inside
  // its source's chunk (a malformed exchange fails the batch, never a wrong
  // key). rule_stride > 0 attributes stats per source (rule' = source x
  // rule_stride + rule).
  uint32_t s0 = 0, s1 = 0, u = 0, q = 0, fl = 0, rule = 0, hits = 0, limit = 0, dstat = 0, len = 0;
  int64_t tnow = 0;
  unsigned long long whash = 0;
  bool layout_bad = false;
  const bool own = b.wire && i - b.own.lo < b.own.n;  // (unsigned: lo <= i < lo + n)
  uint32_t cap = b.stem_cap;
  if (i < b.n) {
    if (own) {
      // this rank's own descriptor, read in place from its source batch (whose
      // partition validated the request layout and computed the hash)
      const uint32_t si = b.own.idx[i - b.own.lo];
      const uint32_t sq = b.own.req[si];
      s0 = b.own.off[si];
      s1 = b.own.off[si + 1];
      cap = b.own.stem_total;
      u = b.own.unit[si];
      fl = b.own.flags[si];
      q = (b.own.rank << ROUTE_REQ_BITS) | sq;
      tnow = b.own.now[sq];
      const uint32_t r0 = b.own.rule[si] < b.own.n_rules ? b.own.rule[si] : 0xFFFFFFFFu;
      rule = !b.rule_stride ? r0 : r0 >= b.rule_stride ? 0xFFFFFFFFu : b.own.rank * b.rule_stride + r0;
      hits = b.own.hits[si];
      limit = b.own.limit[si];
      whash = b.own.hash[si];
    } else if (b.wire) {
      const Wire w = b.wire[i];
      const uint32_t src = w.label >> ROUTE_REQ_BITS;
      const uint32_t wl = w.lu & 0xFFFFu;
      layout_bad = src >= b.n_src;
      s0 = b.woff[i];
      const unsigned long long e0 = (unsigned long long)s0 + wl;
      s1 = (uint32_t)e0;
      if (!layout_bad) {
        const unsigned long long c0 = b.wbase[src], c1 = src + 1 < b.n_src ? b.wbase[src + 1] : b.stem_total;
        layout_bad = s0 < c0 || e0 > c1;
      }
      if (i + 1 < b.n && !(i + 1 - b.own.lo < b.own.n))  // (the own chunk's records carry no wire label)
        layout_bad = layout_bad || b.wire[i + 1].label < w.label;
      layout_bad = layout_bad || *b.wbad != 0;  // (a chunk whose lengths do not add up: every offset after it is shifted)
      layout_bad = layout_bad || e0 > b.stem_total;
      u = (w.lu >> 16) & 0xFFu;
      fl = w.lu >> 24;
      q = w.label;
      tnow = w.now;
      rule = !b.rule_stride ? w.rule : w.rule >= b.rule_stride ? 0xFFFFFFFFu : src * b.rule_stride + w.rule;
      hits = w.hits;
      limit = w.limit;
      whash = w.hash;
    } else {
      s0 = b.off[i];
      s1 = b.off[i + 1];
      u = b.unit[i];
      q = b.req[i];
      fl = b.flags[i];
      rule = b.rule[i];
      hits = b.hits[i];
      limit = b.limit[i];
      layout_bad = (!b.now_desc && q >= b.n_req) || (i && b.req[i - 1] > q);
      tnow = b.now_desc ? b.now[i] : (q < b.n_req ? b.now[q] : 0);
    }
    layout_bad = layout_bad || s1 < s0 || s1 > cap;
  }
  // ---- per-request clock checks (whole-batch mode): now in [0, NOW_MAX], not before the last sweep
  if (!isolate) {
    if (b.wire) {
      if (i < b.n && time_bad(tnow)) bad |= ERR_TIME;
    } else if (i < (b.now_desc ? b.n : b.n_req) && time_bad(b.now[i])) {
      bad |= ERR_TIME;
    }
  }

  // ---- per-descriptor checks. The batch layout (request order, offsets) is
  // fatal; a bad unit / rule / stem length or clock is the descriptor's own
  // error: with isolate it becomes its status (FLAG_SKIP), else it fails the batch.
  if (i < b.n) {
    if (layout_bad) {
      bad |= ERR_INVALID;
    } else {
      len = s1 - s0;
      if (u < 1 || u > 4 || rule >= b.n_rules || len == 0 || len > 65535) dstat = RL_E_INVALID;
      else if (isolate && time_bad(tnow)) dstat = RL_E_TIME;
      if (len > 65535) len = 0;
    }
    if (dstat && !isolate) bad |= ERR_INVALID;
  }
  if (bad) atomicOr(err, bad);

  auto emit_rec = [&](uint64_t h) {
    keys[i] = (uint32_t)(h >> 32) == KEY_DUP ? KEY_DUP - 1u : (uint32_t)(h >> 32);  // (KEY_DUP: k_run_check's mark)
    Rec r;
    r.hlo = (uint32_t)h;
    r.off = s0;
    r.lu = len | (u << 16) | ((uint32_t)((fl & RL_FLAG_SHADOW) | (dstat ? FLAG_SKIP : 0u) | (own ? FLAG_SRC : 0u)) << 24);
    r.rule = rule;
    r.req = q;
    r.now = (uint32_t)tnow;
    r.hits = hits;
    r.limit = limit;
    rec[i] = r;
    if (b.wire) hit_a[i] = r.hits;  // (a routed owner batch; else k_part reads the batch's own hits array)
    if (dstat && isolate) {  // answered here: the table kernels skip it
      res[i] = pack_fail(dstat);
      atomicOr(errs, dstat == RL_E_TIME ? ERR_TIME : ERR_INVALID);
    }
  };
  // ---- a routed owner batch carries the sources' stem hashes: no stem read
  if (b.wire) {
    if (i < b.n) emit_rec(len ? whash : 0ull);
    return;
  }

  // ---- stage this block's stem bytes in LDS (uniform decision per block)
  const uint32_t b0 = blockIdx.x * 256;
  if (b0 >= b.n) return;  // whole block past the descriptors (request checks done)
  const uint32_t b1 = min(b0 + 256u, b.n);
  const uint32_t lo = b.off[b0], hi = b.off[b1], total = b.off[b.n];
  const bool range_ok = hi >= lo && hi <= b.stem_cap && total <= b.stem_cap;
  const uint32_t* words = reinterpret_cast<const uint32_t*>(b.stem);  // 4-byte aligned base
  const uint32_t lead = lo & 3u;
  const uint32_t nbytes = range_ok ? hi - lo + lead : 0;
  const bool use_lds = range_ok && nbytes + 8 <= HASH_LDS_BYTES;
  if (use_lds) {
    const uint32_t* src = words + (lo >> 2);
    const uint32_t nw = (nbytes + 3) / 4;
    for (uint32_t w = tid; w < nw; w += 256) lds[w] = src[w];
    if (tid < 4) lds[nw + tid] = 0;
  }
  __syncthreads();
  if (i >= b.n) return;
  uint64_t h = 0;
  if (len && range_ok && s0 + len <= total) {
    if (use_lds) {
      h = hash_stem(b.hk, DwordReader{lds, HASH_LDS_BYTES / 4 + 4}, s0 - lo + lead, len);
    } else {
      const uint32_t nw = ((total + 3u) >> 2) - (s0 >> 2);
      h = hash_stem(b.hk, DwordReader{words + (s0 >> 2), nw}, s0 & 3u, len);
    }
  }
  emit_rec(h);
}

// ---- k_unpack: a compact host batch (rl_batch_compact: per request clock,
// hits and first descriptor; per descriptor a 16-bit index into the batch's
// limit table) -> the rl_batch arrays the pipeline reads. One lane per
// descriptor (its limit) and per request (its descriptors' request index and
// hits, its 64-bit clock), over descriptors [d0, n) and requests [q0, nq) (a
// multi-shard ctx's slice; indices stay absolute). A request layout that is
// not a partition of [d0, n) into non-decreasing ranges fails the batch
// (ERR_INVALID): a descriptor left out would keep a stale request index.
__global__ __launch_bounds__(256) void k_unpack(uint32_t d0, uint32_t n, uint32_t q0, uint32_t nq, uint32_t n_limits,
                                                const uint16_t* __restrict__ lidx, const rl_limit* __restrict__ lim,
                                                const uint32_t* __restrict__ first, const uint32_t* __restrict__ now32,
                                                const uint32_t* __restrict__ hits_q, uint32_t* __restrict__ req,
                                                uint8_t* __restrict__ unit, uint8_t* __restrict__ flags,
                                                uint32_t* __restrict__ limit, uint32_t* __restrict__ hits,
                                                uint32_t* __restrict__ rule, int64_t* __restrict__ now,
                                                uint32_t* err) {
  const uint32_t i = d0 + blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const uint32_t k = lidx[i];
    const rl_limit L = k < n_limits ? lim[k] : rl_limit{0, 0, 0, 0, 0};  // unit 0: the descriptor's RL_E_INVALID
    unit[i] = L.unit;
    flags[i] = L.flags;
    limit[i] = L.requests_per_unit;
    rule[i] = L.rule_id;
  }
  const uint32_t iq = q0 + blockIdx.x * 256 + threadIdx.x;
  if (iq < nq) {
    const uint32_t i = iq;
    const uint32_t a = first[i], z = first[i + 1];
    if (z < a || z > n || a < d0 || (i == q0 && a != d0) || (i + 1 == nq && z != n)) {
      atomicOr(err, ERR_INVALID);
    } else {
      const uint32_t h = hits_q[i];
      for (uint32_t d = a; d < z; d++) {
        req[d] = i;
        hits[d] = h;
      }
    }
    now[i] = now32[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && nq == q0 && n > d0) atomicOr(err, ERR_INVALID);  // descriptors without a request
}

void launch_unpack(const rl_batch_compact& cb, const uint8_t* buf, uint32_t* req, uint8_t* unit, uint8_t* flags,
                   uint32_t* limit, uint32_t* hits, uint32_t* rule, int64_t* now, uint32_t* err, hipStream_t st) {
  launch_unpack_range(cb, buf, 0, cb.n, 0, cb.n_requests, req, unit, flags, limit, hits, rule, now, err, st);
}

void launch_unpack_range(const rl_batch_compact& cb, const uint8_t* buf, uint32_t d0, uint32_t d1, uint32_t q0,
                         uint32_t q1, uint32_t* req, uint8_t* unit, uint8_t* flags, uint32_t* limit, uint32_t* hits,
                         uint32_t* rule, int64_t* now, uint32_t* err, hipStream_t st) {
  const uint32_t m = d1 - d0 > q1 - q0 ? d1 - d0 : q1 - q0;
  if (!m) return;
  k_unpack<<<(m + 255) / 256, 256, 0, st>>>(
      d0, d1, q0, q1, cb.n_limits, reinterpret_cast<const uint16_t*>(buf + cb.limit_idx),
      reinterpret_cast<const rl_limit*>(buf + cb.limits), reinterpret_cast<const uint32_t*>(buf + cb.req_first),
      reinterpret_cast<const uint32_t*>(buf + cb.now), reinterpret_cast<const uint32_t*>(buf + cb.hits), req, unit,
      flags, limit, hits, rule, now, err);
}

// ---- k_unpack_prefixed: a prefix-shared host batch (rl_batch_prefixed) ->
// the rl_batch arrays, stems rebuilt as prefix[q] ‖ suffix[d]. One workgroup
// per tile of PFX_TILE requests, one lane per request; the tile's index entry
// gives its starting descriptor, prefix, suffix and stem offsets, so tiles are
// independent (a multi-shard slice is a tile range). The tile's own sums are
// checked against the next entry before anything is written, and every read
// and write stays below the index's totals (host-checked against the sections
// and the staging capacity): a malformed index fails the batch (ERR_INVALID)
// and never writes outside it. The tile's stems are assembled in LDS and
// leave as whole dwords when they fit (C1: ~17 KB per tile).
constexpr uint32_t PFX_TILE = RL_PREFIXED_TILE;
constexpr uint32_t PFX_LDS = 24576;  // stem bytes assembled in LDS per tile

__device__ inline uint32_t block_excl_scan_u32(uint32_t v, uint32_t* tmp, uint32_t* total) {
  // 256 lanes: wave-level inclusive scans by shuffles, then across the 4 waves
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) tmp[wv] = x;
  __syncthreads();
  uint32_t base = 0;
  for (uint32_t k = 0; k < wv; k++) base += tmp[k];
  *total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  __syncthreads();
  return base + x - v;
}

__global__ __launch_bounds__(256) void k_unpack_prefixed(
    uint32_t t0, uint32_t nq, uint32_t n_limits, uint4 tot, const uint32_t* __restrict__ reqw,
    const uint32_t* __restrict__ now32, const uint32_t* __restrict__ hits_q, const uint32_t* __restrict__ descw,
    const uint8_t* __restrict__ pfx, const uint8_t* __restrict__ sfx, const rl_limit* __restrict__ lim,
    const uint4* __restrict__ index, uint8_t* __restrict__ stem, uint32_t* __restrict__ off,
    uint32_t* __restrict__ req, uint8_t* __restrict__ unit, uint8_t* __restrict__ flags,
    uint32_t* __restrict__ limit, uint32_t* __restrict__ hits, uint32_t* __restrict__ rule,
    int64_t* __restrict__ now, uint32_t* err) {
  __shared__ uint32_t s_tmp[4][4];
  __shared__ uint32_t s_first[PFX_TILE + 1], s_pl[PFX_TILE], s_pin[PFX_TILE];
  __shared__ uint32_t s_out[PFX_LDS / 4 + 2];
  const uint32_t tid = threadIdx.x, t = t0 + blockIdx.x;
  const uint32_t q0 = t * PFX_TILE, q = q0 + tid;
  const uint4 I0 = index[t], I1 = index[t + 1];
  const uint32_t rw = q < nq ? reqw[q] : 0u;
  const uint32_t nd = rw & 0xFFFFu, pl = (rw >> 16) & 0xFFu;
  uint32_t T_nd, T_pl;
  const uint32_t e_nd = block_excl_scan_u32(nd, s_tmp[0], &T_nd);
  const uint32_t e_pl = block_excl_scan_u32(pl, s_tmp[1], &T_pl);
  // the tile's entry against its own sums and the totals (uniform per block)
  const bool ok = I0.x <= I1.x && I0.y <= I1.y && I0.z <= I1.z && I0.w <= I1.w && I1.x <= tot.x && I1.y <= tot.y &&
                  I1.z <= tot.z && I1.w <= tot.w && I1.x - I0.x == T_nd && I1.y - I0.y == T_pl;
  s_first[tid] = I0.x + e_nd;
  s_pl[tid] = pl;
  s_pin[tid] = I0.y + e_pl;
  if (tid == 0) s_first[PFX_TILE] = I1.x;
  const int reserved_bits = __syncthreads_or((rw >> 24) != 0u);
  if (!ok || reserved_bits) {
    if (tid == 0) atomicOr(err, ERR_INVALID);
    return;
  }
  if (q < nq) {
    now[q] = now32[q];
    const uint32_t h = hits_q[q];
    for (uint32_t d = I0.x + e_nd, z = d + nd; d < z; d++) {
      req[d] = q;
      hits[d] = h;
    }
  }
  // descriptors of the tile, 256 at a time: stem offsets by a block scan
  const uint32_t D = T_nd;
  const uint32_t span = I1.w - I0.w;
  const bool in_lds = span <= PFX_LDS;
  uint32_t carry_s = 0, carry_o = 0, bad = 0;
  for (uint32_t c = 0; c < D; c += 256) {
    const uint32_t j = c + tid, d = I0.x + j;
    uint32_t w = 0, r = 0;
    if (j < D) {
      w = descw[d];
      // request of descriptor d: the last tile request whose first descriptor <= d
      uint32_t lo = 0, hi = PFX_TILE;  // s_first[lo] <= d < s_first[hi]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_first[mid] <= d) lo = mid;
        else hi = mid;
      }
      r = lo;
    }
    const uint32_t sl = w >> 16, p = j < D ? s_pl[r] : 0u;
    uint32_t T_s, T_o;
    const uint32_t e_s = block_excl_scan_u32(sl, s_tmp[2], &T_s);
    const uint32_t e_o = block_excl_scan_u32(p + sl, s_tmp[3], &T_o);
    if (j < D) {
      const uint32_t si = I0.z + carry_s + e_s;   // suffix bytes in
      const uint32_t lo = carry_o + e_o;          // stem bytes out (tile-relative)
      const uint32_t pi = s_pin[r];
      if (si + sl > I1.z || pi + p > I1.y || lo + p + sl > span) {
        bad = 1;
      } else {
        off[d] = I0.w + lo;
        if (in_lds) {
          uint8_t* o8 = reinterpret_cast<uint8_t*>(s_out) + (I0.w & 3u) + lo;
          for (uint32_t k = 0; k < p; k++) o8[k] = pfx[pi + k];
          for (uint32_t k = 0; k < sl; k++) o8[p + k] = sfx[si + k];
        } else {
          uint8_t* o8 = stem + I0.w + lo;
          for (uint32_t k = 0; k < p; k++) o8[k] = pfx[pi + k];
          for (uint32_t k = 0; k < sl; k++) o8[p + k] = sfx[si + k];
        }
      }
      const uint32_t k = w & 0xFFFFu;
      const rl_limit L = k < n_limits ? lim[k] : rl_limit{0, 0, 0, 0, 0};  // unit 0: RL_E_INVALID
      unit[d] = L.unit;
      flags[d] = L.flags;
      limit[d] = L.requests_per_unit;
      rule[d] = L.rule_id;
    }
    carry_s += T_s;
    carry_o += T_o;
  }
  if (tid == 0) {
    if (carry_s != I1.z - I0.z || carry_o != span) bad = 1;
    off[I1.x] = I1.w;  // (the next tile writes the same value as its first offset)
  }
  if (bad) atomicOr(err, ERR_INVALID);
  if (in_lds) {  // the tile's stems [I0.w, I1.w) as whole dwords, bytes at the ragged ends
    __syncthreads();
    const uint32_t a = I0.w, z = I1.w, sh = a & 3u;
    const uint8_t* s8 = reinterpret_cast<const uint8_t*>(s_out);
    const uint32_t a4 = (a + 3u) & ~3u, z4 = z & ~3u;
    if (a4 < z4) {
      // global byte g sits at byte g - a + sh of s_out: global dword w4 is s_out[w4 - a / 4]
      uint32_t* o32 = reinterpret_cast<uint32_t*>(stem);
      for (uint32_t w4 = a4 / 4 + tid; w4 < z4 / 4; w4 += 256) o32[w4] = s_out[w4 - a / 4];
      if (tid < a4 - a) stem[a + tid] = s8[sh + tid];
      if (tid < z - z4) stem[z4 + tid] = s8[z4 - a + sh + tid];
    } else if (tid < z - a) {
      stem[a + tid] = s8[sh + tid];
    }
  }
}

// ---- k_to_host: launch_to_host's copies. Copy k's 16-B-aligned middle in
// dwordx4 stores, grid-stride; its ragged head and tail bytes by the first
// workgroup (host arrays from rl_alloc_host are aligned: the head is empty).
__global__ __launch_bounds__(256) void k_to_host(ToHost c) {
  const uint64_t tid = blockIdx.x * 256ull + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  for (uint32_t k = 0; k < c.n; k++) {
    const uint8_t* s = c.src[k];
    uint8_t* d = c.dst[k];
    const uint64_t B = c.bytes[k];
    const uint64_t head = ((16u - ((uintptr_t)d & 15u)) & 15u) < B ? ((16u - ((uintptr_t)d & 15u)) & 15u) : B;
    if ((((uintptr_t)s + head) & 15u) == 0) {
      const uint64_t n16 = (B - head) / 16;
      const uint4* s4 = reinterpret_cast<const uint4*>(s + head);
      uint4* d4 = reinterpret_cast<uint4*>(d + head);
      for (uint64_t j = tid; j < n16; j += stride) d4[j] = s4[j];
      if (blockIdx.x == 0) {
        if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
        const uint64_t t0 = head + n16 * 16;
        if (t0 + threadIdx.x < B) d[t0 + threadIdx.x] = s[t0 + threadIdx.x];
      }
    } else {  // (source and destination misaligned against each other: bytes)
      for (uint64_t j = tid; j < B; j += stride) d[j] = s[j];
    }
  }
}

hipError_t copy_to_host(ToHost c, hipStream_t st) {
  static const bool dma = getenv("RL_D2H_MEMCPY") != nullptr;  // (A/B knob)
  bool mapped = !dma;
  ToHost m = c;
  for (uint32_t k = 0; k < c.n && mapped; k++) {
    void* dp = nullptr;
    void* de = nullptr;
    // both ends inside one page-locked allocation (an array running past its
    // allocation's end would have the kernel store to unmapped device VA)
    mapped = c.bytes[k] == 0 ||
             (hipHostGetDevicePointer(&dp, c.dst[k], 0) == hipSuccess && dp &&
              hipHostGetDevicePointer(&de, c.dst[k] + c.bytes[k] - 1, 0) == hipSuccess &&
              (uint8_t*)de == (uint8_t*)dp + c.bytes[k] - 1);
    m.dst[k] = (uint8_t*)dp;
  }
  if (mapped) {
    launch_to_host(m, st);
    return hipGetLastError();
  }
  (void)hipGetLastError();  // (the failed lookup's sticky error: pageable memory)
  for (uint32_t k = 0; k < c.n; k++)
    if (c.bytes[k]) {
      const hipError_t e = hipMemcpyAsync(c.dst[k], c.src[k], c.bytes[k], hipMemcpyDeviceToHost, st);
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}

void launch_to_host(const ToHost& c, hipStream_t st) {
  uint64_t most = 0;
  for (uint32_t k = 0; k < c.n; k++) most = c.bytes[k] > most ? c.bytes[k] : most;
  if (!most) return;
  static const uint32_t cap = getenv("RL_D2H_BLOCKS") ? (uint32_t)atoi(getenv("RL_D2H_BLOCKS")) : 1024u;  // (A/B knob)
  const uint64_t g = (most / 16 + 255) / 256;
  const uint32_t gmax = cap ? cap : 1u;
  k_to_host<<<(uint32_t)(g < gmax ? (g ? g : 1) : gmax), 256, 0, st>>>(c);
}

void launch_unpack_prefixed(const rl_batch_prefixed& pb, const uint8_t* buf, uint32_t t0, uint32_t t1, uint8_t* stem,
                            uint32_t* off, uint32_t* req, uint8_t* unit, uint8_t* flags, uint32_t* limit,
                            uint32_t* hits, uint32_t* rule, int64_t* now, uint32_t* err, hipStream_t st) {
  if (t1 <= t0) return;
  const uint32_t tiles = (pb.n_requests + PFX_TILE - 1) / PFX_TILE;
  const uint32_t* host_tot = reinterpret_cast<const uint32_t*>(pb.buf + pb.index) + 4ull * tiles;
  const uint4 tot = make_uint4(host_tot[0], host_tot[1], host_tot[2], host_tot[3]);
  k_unpack_prefixed<<<t1 - t0, 256, 0, st>>>(
      t0, pb.n_requests, pb.n_limits, tot, reinterpret_cast<const uint32_t*>(buf + pb.req),
      reinterpret_cast<const uint32_t*>(buf + pb.now), reinterpret_cast<const uint32_t*>(buf + pb.hits),
      reinterpret_cast<const uint32_t*>(buf + pb.desc), buf + pb.prefix_bytes, buf + pb.suffix_bytes,
      reinterpret_cast<const rl_limit*>(buf + pb.limits), reinterpret_cast<const uint4*>(buf + pb.index), stem, off,
      req, unit, flags, limit, hits, rule, now, err);
}

// The zero-padded first KEY_HEAD bytes of the stem at byte `off` of the packed
// stems, as 4 x uint4: five aligned 16-B loads, then dword selects and funnel
// shifts. Only chunks holding a byte of the head are loaded, so no load leaves
// the 16-B blocks (hence the pages) the stem occupies.
__device__ inline void load_head(const uint8_t* stem, uint32_t off, uint32_t len, uint4 out[KEY_HV]) {
  const uint32_t hl = len < KEY_HEAD ? len : KEY_HEAD;
  const uint32_t mis = (uint32_t)((uintptr_t)stem & 15u);
  const uint4* c16 = reinterpret_cast<const uint4*>(stem - mis);
  const uint32_t a = off + mis;
  const uint32_t c0 = a >> 4, last = (a + (hl ? hl : 1u) - 1u) >> 4;
  uint32_t w[4 * (KEY_HV + 1)];
#pragma unroll
  for (uint32_t j = 0; j < KEY_HV + 1; j++) {
    const uint4 v = c0 + j <= last ? c16[c0 + j] : make_uint4(0u, 0u, 0u, 0u);
    w[4 * j] = v.x;
    w[4 * j + 1] = v.y;
    w[4 * j + 2] = v.z;
    w[4 * j + 3] = v.w;
  }
  const uint32_t q = (a >> 2) & 3u, sb = a & 3u;
  uint32_t x[4 * KEY_HV + 1];
#pragma unroll
  for (uint32_t k = 0; k < 4 * KEY_HV + 1; k++) x[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
  uint32_t o[4 * KEY_HV];
#pragma unroll
  for (uint32_t k = 0; k < 4 * KEY_HV; k++) {
    uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sb);
    if (4 * k >= hl) v = 0;
    else if (4 * k + 4 > hl) v &= (1u << ((hl - 4 * k) * 8)) - 1u;
    o[k] = v;
  }
#pragma unroll
  for (uint32_t v = 0; v < KEY_HV; v++) out[v] = make_uint4(o[4 * v], o[4 * v + 1], o[4 * v + 2], o[4 * v + 3]);
}

// ===========================================================================
// Stem bytes as dwords. Stems sit at arbitrary byte offsets of the packed
// buffer; a StemRef reads them as aligned dwords and funnel-shifts
// (v_alignbyte) so compares move 4 bytes per load. Dwords past the end of the
// packed stems read as 0 (no access past the buffer).
// ===========================================================================
struct StemRef {
  const uint32_t* p;  // dword-aligned base
  uint32_t sh;        // byte offset of the stem's first byte in p[0]
  uint32_t nw;        // readable dwords from p
  __device__ inline uint32_t at(uint32_t i) const { return i < nw ? p[i] : 0u; }
  __device__ inline uint32_t word(uint32_t k) const { return __builtin_amdgcn_alignbyte(at(k + 1), at(k), sh); }
};

// b.stem is 4-byte aligned (checked on the host). Pointers are derived from the
// kernel argument by arithmetic only, so loads stay global_* (an integer
// round trip would make them flat_*).
__device__ inline StemRef stem_ref(const BatchDev& b, uint32_t o) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(b.stem);
  return StemRef{w + (o >> 2), o & 3u, ((b.stem_total + 3u) >> 2) - (o >> 2)};
}

__device__ inline uint32_t tail_mask(uint32_t len) { return (len & 3) ? ((1u << ((len & 3) * 8)) - 1u) : 0u; }

__device__ inline bool stem_words_equal(const StemRef& x, const StemRef& y, uint32_t len) {
  uint32_t diff = 0;
  const uint32_t nw = len >> 2;
#pragma unroll 4
  for (uint32_t k = 0; k < nw; k++) diff |= x.word(k) ^ y.word(k);
  if (len & 3) diff |= (x.word(nw) ^ y.word(nw)) & tail_mask(len);
  return diff == 0;
}

// A stem as the run kernels see it: its zero-padded 64-B head in registers
// (read from the packed stems with aligned 16-B loads) and, for stems longer
// than 64 B only, the rest through a StemRef.
struct Key {
  uint4 h[KEY_HV];
  StemRef st;  // full stem (bytes >= KEY_HEAD read from here)
  uint32_t len;
};

// The packed stems' byte counts, from the offsets (kernel-argument copies;
// the host sets the capacity): a received batch's is set by the host, an own
// chunk's comes from its source batch's offsets.
__device__ inline void refine_totals(BatchDev& b) {
  if (b.off) b.stem_total = b.off[b.n];
  if (b.own.n) b.own.stem_total = b.own.off[b.own.src_n];
}

__device__ inline Key key_of(const BatchDev& b, const Rec& r) {
  Key k;
  k.len = rec_len(r);
  if ((rec_flags(r) & FLAG_SRC) && b.own.stem) {  // (a routed owner's own chunk: the source batch's stems)
    const uint32_t* w = reinterpret_cast<const uint32_t*>(b.own.stem);
    k.st = StemRef{w + (r.off >> 2), r.off & 3u, ((b.own.stem_total + 3u) >> 2) - (r.off >> 2)};
    load_head(b.own.stem, r.off, k.len, k.h);
  } else {
    k.st = stem_ref(b, r.off);
    load_head(b.stem, r.off, k.len, k.h);
  }
  return k;
}

__device__ inline Key key_at(const BatchDev& b, SRec rec_s, uint32_t q) { return key_of(b, rec_s[q]); }

__device__ inline uint32_t head_diff(const uint4* x, const uint4* y) {
  uint32_t d = 0;
#pragma unroll
  for (uint32_t v = 0; v < KEY_HV; v++) {
    const uint4 a = x[v], c = y[v];
    d |= (a.x ^ c.x) | (a.y ^ c.y) | (a.z ^ c.z) | (a.w ^ c.w);
  }
  return d;
}

// bytes [KEY_HEAD, len) of two stems (words KEY_HEAD / 4.. of their StemRefs)
__device__ inline uint32_t tail_diff(const StemRef& x, const StemRef& y, uint32_t len) {
  uint32_t d = 0;
  const uint32_t nw = len >> 2;
  for (uint32_t k = KEY_HEAD / 4; k < nw; k++) d |= x.word(k) ^ y.word(k);
  if (len & 3) d |= (x.word(nw) ^ y.word(nw)) & tail_mask(len);
  return d;
}

// Same stem bytes (callers have compared hash and length).
__device__ inline bool key_equal(const Key& x, const Key& y) {
  uint32_t d = head_diff(x.h, y.h);
  if (x.len > KEY_HEAD) d |= tail_diff(x.st, y.st, x.len);
  return d == 0;
}

// ===========================================================================
// HBM table probing.
// ===========================================================================
__device__ inline uint32_t u4w(const uint4& a, uint32_t j) { return j == 0 ? a.x : j == 1 ? a.y : j == 2 ? a.z : a.w; }

// Stem dword k (static in unrolled loops): the zero-padded head, then the packed stems.
__device__ inline uint32_t key_dw(const Key& key, uint32_t k) {
  return k < KEY_HEAD / 4 ? u4w(key.h[k >> 2], k & 3) : key.st.word(k);
}

// Stem bytes [KEY_SPLIT, len) of `key` against the arena copy at ext_off.
__device__ inline uint32_t arena_diff(const uint8_t* arena, uint32_t ext_off, const Key& key) {
  const uint32_t* ek = reinterpret_cast<const uint32_t*>(arena + (size_t)ext_off * 16);
  const uint32_t rest = key.len - KEY_SPLIT, rw = rest >> 2;
  uint32_t d = 0;
  for (uint32_t k = 0; k < rw; k++) d |= ek[k] ^ key.st.word(KEY_SPLIT / 4 + k);
  if (rest & 3) d |= (ek[rw] ^ key.st.word(KEY_SPLIT / 4 + rw)) & tail_mask(rest);
  return d;
}

__device__ inline uint32_t slot_ext(const Slot* s) { return reinterpret_cast<const uint32_t*>(s)[SLOT_EXT_DW]; }

// Slot stem == `key`? Only the stem's own dwords are read (the last one masked).
__device__ inline bool slot_key_equal(const Slot* s, const Key& key, const uint8_t* arena) {
  if (s->key_len != key.len) return false;
  const uint32_t* sd = reinterpret_cast<const uint32_t*>(s);
  const uint32_t len = key.len, il = slot_inline(len), nw = il >> 2;
  uint32_t diff = 0;
#pragma unroll
  for (uint32_t k = 0; k < KEY_IN / 4; k++) {
    if (k < nw) diff |= sd[slot_key_dw(k)] ^ key_dw(key, k);
    else if (k == nw && (il & 3)) diff |= (sd[slot_key_dw(k)] ^ key_dw(key, k)) & tail_mask(il);
  }
  if (len > KEY_IN) diff |= arena_diff(arena, sd[SLOT_EXT_DW], key);
  return diff == 0;
}

// Claim n16 16-B units of the long-stem arena; the cursor never moves past the
// cap (a failed claim leaves it alone). rl_sweep compacts the arena.
__device__ __attribute__((always_inline)) inline bool arena_claim(const TableDev& t, uint32_t n16, unsigned long long* off) {
  unsigned long long cur = __hip_atomic_load(t.arena_used16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (cur + n16 > t.arena_cap16) return false;
    const unsigned long long prev = atomicCAS(t.arena_used16, cur, cur + n16);
    if (prev == cur) {
      *off = cur;
      return true;
    }
    cur = prev;
  }
}

// Fill a freshly claimed slot (no history yet). False when
// the arena cannot take the stem's tail: the caller returns the slot to the
// table as a tombstone.
__device__ __attribute__((always_inline)) inline bool slot_init(const TableDev& t, Slot* s, const Key& key, uint32_t unit) {
  const uint32_t len = key.len, il = slot_inline(len), nw = il >> 2;
  uint32_t* sd = reinterpret_cast<uint32_t*>(s);
  if (len > KEY_IN) {
    const uint32_t n16 = (len - KEY_SPLIT + 15) / 16;
    unsigned long long off;
    if (!arena_claim(t, n16, &off)) return false;
    sd[SLOT_EXT_DW] = (uint32_t)off;
    uint32_t* ek = reinterpret_cast<uint32_t*>(t.arena + off * 16);
    for (uint32_t k = 0; k < (len - KEY_SPLIT + 3) / 4; k++) ek[k] = key.st.word(KEY_SPLIT / 4 + k);
  }
  s->key_len = (uint16_t)len;
  s->unit = (uint8_t)unit;
  s->flags = 0;
#pragma unroll
  for (uint32_t k = 0; k < KEY_IN / 4; k++) {
    if (k < nw) sd[slot_key_dw(k)] = key_dw(key, k);
    else if (k == nw && (il & 3)) sd[slot_key_dw(k)] = key_dw(key, k) & tail_mask(il);
  }
  s->cur = Win{WS_INVALID, 0, 0, 0};
  s->ring = LOG_NONE;
  return true;
}

// find_slot* results below 0.
constexpr int64_t SLOT_ABSENT = -1, SLOT_TABLE_FULL = -2, SLOT_ARENA_FULL = -3;
__device__ inline uint32_t slot_fail_status(int64_t r) {
  return r == SLOT_ARENA_FULL ? (uint32_t)RL_E_ARENA_FULL : (uint32_t)RL_E_TABLE_FULL;
}

// Claim slot i (expected tag `from`) for (stem, unit) and initialise it.
// 1: claimed, 0: lost the race, -1: the arena is full (the slot is a tombstone again).
__device__ __attribute__((always_inline)) inline int slot_claim(const TableDev& t, uint64_t i, uint32_t from, uint32_t tag, const Key& key,
                                 uint32_t unit) {
  Slot* s = &t.slots[i];
  if (atomicCAS(&s->tag, from, tag) != from) return 0;
  if (slot_init(t, s, key, unit)) return 1;
  __hip_atomic_store(&s->tag, TAG_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return -1;
}

// Find (and optionally insert) the slot of (stem, unit). Returns SLOT_ABSENT
// when absent and insert == false, SLOT_TABLE_FULL / SLOT_ARENA_FULL (error
// bit set in *err) when it cannot be inserted. Linear probing over 64-B slots
// from the home slot = top bits of the stem hash, i.e. of the sort key:
// consecutive runs probe increasing slots (page and TLB locality). A tag
// match is confirmed by the full stem (collision-exact). Inserts claim the
// slot with a CAS on its tag; only one lane ever handles a given
// (stem, unit) per batch (runs are grouped by stem).
__device__ __attribute__((always_inline)) inline int64_t find_slot(const TableDev& t, uint64_t hstem, uint32_t tag, const Key& key, uint32_t unit,
                             bool insert, bool* inserted, uint32_t* err) {
  uint64_t i = hstem >> t.shift;
  int64_t tomb = -1;
  *inserted = false;
  for (uint32_t p = 0; p < t.max_probe; p++, i = (i + 1) & t.mask) {
    Slot* s = &t.slots[i];
    const uint32_t st = __hip_atomic_load(&s->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (st == tag) {  // (a 32-bit tag is a filter: the unit and the stem bytes decide)
      if (s->unit == unit && slot_key_equal(s, key, t.arena)) return (int64_t)i;
      continue;
    }
    if (st == TAG_TOMB) {
      if (tomb < 0) tomb = (int64_t)i;
      continue;
    }
    if (st != TAG_EMPTY) continue;
    // (stem, unit) is absent: claim the first tombstone on the path, else this slot.
    if (!insert) return SLOT_ABSENT;
    int c = tomb >= 0 ? slot_claim(t, (uint64_t)tomb, TAG_TOMB, tag, key, unit) : 0;
    if (c > 0) {
      *inserted = true;
      return tomb;
    }
    if (c == 0) c = slot_claim(t, i, TAG_EMPTY, tag, key, unit);
    if (c > 0) {
      *inserted = true;
      return (int64_t)i;
    }
    if (c < 0) {
      atomicOr(err, ERR_ARENA_FULL);
      return SLOT_ARENA_FULL;
    }
    // another stem claimed this slot concurrently: keep probing
  }
  atomicOr(err, ERR_TABLE_FULL);
  return SLOT_TABLE_FULL;
}

// A slot image for probing: the whole 64-B slot (tag, length, flags, cur,
// history chain head, stem bytes 0..35). Plain loads are enough: within a launch only
// CAS inserts change tags, and a lane only ever looks for its own stem, which
// no other lane inserts.
struct SlotImg {
  uint4 v[4];
  __device__ inline uint32_t dw(uint32_t k) const { return u4w(v[k >> 2], k & 3); }
  __device__ inline uint32_t tag() const { return v[0].x; }
  __device__ inline uint32_t key_len() const { return v[0].y & 0xFFFFu; }
  __device__ inline uint32_t unit() const { return (v[0].y >> 16) & 0xFFu; }
  __device__ inline uint32_t flags() const { return v[0].y >> 24; }
  __device__ inline Win cur() const { return Win{v[0].z, v[0].w, v[1].x, v[1].y}; }
  __device__ inline uint32_t ring() const { return v[1].z; }
};

__device__ inline void load_img_lo(const Slot* s, SlotImg& im) {
  const uint4* p = reinterpret_cast<const uint4*>(s);
#pragma unroll
  for (int j = 0; j < 4; j++) im.v[j] = p[j];
}

// Stem of `key` == the slot's stem? A stem longer than KEY_IN compares its
// tail with the arena.
__device__ inline bool img_key_equal(const SlotImg& im, const Key& key, const uint8_t* arena) {
  if (im.key_len() != key.len) return false;
  const uint32_t len = key.len, il = slot_inline(len), nw = il >> 2;
  uint32_t d = 0;
#pragma unroll
  for (uint32_t k = 0; k < KEY_IN / 4; k++) {
    if (k < nw) d |= im.dw(slot_key_dw(k)) ^ key_dw(key, k);
    else if (k == nw && (il & 3)) d |= (im.dw(slot_key_dw(k)) ^ key_dw(key, k)) & tail_mask(il);
  }
  if (len > KEY_IN) d |= arena_diff(arena, im.dw(SLOT_EXT_DW), key);
  return d == 0;
}

// ---- the history log (rl_device.h). A record of a slot with divider d is
// kept while a request could still ask for it: its window within HIST_W
// windows of the key's newest (ws_new), or its EXPIRE / local-cache TTL plus
// J + d not before ws_new (J = the horizon, rl_config's jitter bound). A
// request whose window has no record on the chain was never written — unless
// both bounds have passed, where a dropped record could have been: then
// RL_E_TIME. Sound: a dropped record r has max(r.expire, r.lc) + J + d <
// ws_new <= cur, so a request with now + J + d >= cur finds it dead (now >
// r.expire, now >= r.lc), i.e. equal to no record. Exact therefore for every
// request whose clock is within div + J of the key's newest window, and for
// any within HIST_W windows of it.
__device__ inline bool hist_keep(const TableDev& t, const Win& r, uint32_t ws_new, uint32_t d) {
  return r.ws != WS_INVALID &&
         (hist_reach(r.ws, ws_new, d) || (uint64_t)max(r.expire, r.lc) + t.horizon + d >= (uint64_t)ws_new);
}
// Or w is 2 div back: a record of w holds EXPIRE and the local-cache TTL of
// requests inside w (now + div), dead from w + 2 div on. An alias write (a
// multi-unit stem's key written through another unit's request) can move a
// record's EXPIRE further, but the writing unit's own record of w carries the
// same value and is checked too (every unit slot of the stem is), under its
// own div: a live key never goes unnoticed.
__device__ inline bool hist_dead(uint32_t now, uint32_t w, uint32_t d) { return (uint64_t)now >= (uint64_t)w + 2ull * d; }
__device__ inline bool hist_absent_ok(const TableDev& t, uint32_t now, uint32_t w, uint32_t cur_ws, uint32_t d) {
  return hist_reach(w, cur_ws, d) || (uint64_t)now + t.horizon + d >= (uint64_t)cur_ws || hist_dead(now, w, d);
}

// ---- Publishing an entry while others may read it. A lookup can reach an
// entry that is being overwritten: its chain was appended in an earlier batch
// and the partition has wrapped onto it since. Each entry is two 16-B halves
// (a dwordx4 is written and read whole); the writer and the reader follow a
// seqlock so a lookup never pairs one write's header with another's record:
//  - writer: the header with its tag BUSY, then the record, then the header
//    (LOG_WRITE_STEPS stores, in program order: the compiler barriers keep
//    them in order, and the hardware applies one wave's stores to one 128-B
//    line in order, in this CU's path and in the L2 channel that owns the line;
//    another XCD sees the line only as whole write-backs of that L2's state,
//    i.e. after some prefix of the three stores);
//  - reader: the header, the record, the header again past this CU's L1; the
//    record is used (even only to rule the entry out) when both headers are
//    equal and carry the owner's tag. A record changed between the two header
//    loads was written after an invalidation the second load sees (BUSY, or a
//    newer header).
// This holds when at most one writer writes an entry in a batch's table stage:
// log_append refuses an append that would overwrite an entry the same batch
// appended (the partition's counter at the batch's start, or earlier: k_b_begin), and
// the only other write, k_late's alias write-back, goes to an entry appended
// earlier in the same batch, which is therefore never overwritten under it.
// RL_LOG_TEAR builds (tests/test_gpu_log_tear.py) replay a concurrent writer's
// steps between the reader's loads in every interleaving.
#ifndef RL_LOG_ORDER
#define RL_LOG_ORDER 1  // (A/B builds: 0 = no compiler barriers between the entry's stores and loads)
#endif
#ifndef RL_LOG_BUSY
#define RL_LOG_BUSY 1  // (A/B builds: 0 = round 5's 2-step writer)
#endif
#ifndef RL_LOG_GUARD
#define RL_LOG_GUARD 1  // (A/B builds: 0 = no per-batch wrap guard)
#endif
__device__ __forceinline__ void log_order() {
#if RL_LOG_ORDER
  __asm__ __volatile__("" ::: "memory");
#endif
}
constexpr uint32_t LOG_WRITE_STEPS = RL_LOG_BUSY ? 3 : 2;

// Step s of writing entry e (header h, record r). legacy: round 5's order
// (header, record; 2 steps), kept for the tear tests only.
__device__ __forceinline__ void log_write_step(uint4* e, uint32_t s, const uint4& h, const uint4& r, bool legacy) {
  if (legacy) {
    if (s == 0) e[0] = h;
    else e[1] = r;
  } else if (s == 0) {
    e[0] = make_uint4(h.x, LOG_TAG_BUSY, h.z, h.w);
  } else if (s == 1) {
    e[1] = r;
  } else {
    e[0] = h;
  }
  log_order();
}

// Append r to the chain whose head is prev (slot si, tag, newest window
// t_app); returns the new head, or LOG_LOST when the partition has taken
// log_cap appends in this batch already (one batch's appends never wrap a
// partition onto its own entries; counted in rl_table_info.history_refused).
// The active lanes of a wave take consecutive entries of one partition with
// one atomic (partitions spread by workgroup and wave), so appends are
// coalesced stores.
__device__ inline uint32_t log_append(const TableDev& t, uint32_t si, uint32_t tag, uint32_t prev, uint32_t t_app,
                                      const Win& r) {
  const uint32_t lane = __lane_id();
  const uint32_t p = (blockIdx.x * 4u + (threadIdx.x >> 6)) & (LOG_PARTS - 1u);
  const uint64_t act = __ballot(1);
  const uint32_t leader = (uint32_t)__ffsll((unsigned long long)act) - 1u;
  unsigned long long* line = &t.log_ctr[(size_t)p * LOG_CTR_STRIDE];
  unsigned long long k = 0;
  if (lane == leader) k = atomicAdd(line, (unsigned long long)__popcll(act));
  k = __shfl(k, leader, 64) + (unsigned long long)__popcll(act & ((1ull << lane) - 1ull));
  if (RL_LOG_GUARD && k - t.log_epoch[p] >= t.log_cap) {
#ifdef RL_LOG_DEBUG  // (diagnostic builds: who was refused)
    if (atomicAdd(t.hist_lost + 2, 1ull) < 40)
      printf("refused: grid %u block %u thread %u part %u k %llu epoch %llu cap %u active %d si %u t_app %u ws %u\n",
             gridDim.x, blockIdx.x, threadIdx.x, p, k, t.log_epoch[p], t.log_cap, __popcll(act), si, t_app, r.ws);
#endif
    atomicAdd(t.hist_lost + 1, 1ull);
    return LOG_LOST;
  }
  const uint32_t pos = (uint32_t)k & (t.log_cap - 1u);
  uint4* e = reinterpret_cast<uint4*>(&t.log[(size_t)p * t.log_cap + pos]);
  const uint4 h = make_uint4(si, tag, prev, t_app), rv = make_uint4(r.ws, r.count, r.expire, r.lc);
#pragma unroll
  for (uint32_t s = 0; s < LOG_WRITE_STEPS; s++) log_write_step(e, s, h, rv, !RL_LOG_BUSY);
  return (p << LOG_POS_BITS) | pos;
}

#ifndef RL_LOG_REREAD
#define RL_LOG_REREAD 1  // (diagnostic builds: 0 = re-read only a found record's header (round 5), 2 = a plain re-read)
#endif
// The header of e re-read past this CU's L1 (agent scope).
__device__ __forceinline__ uint4 log_hdr_reread(const uint4* e) {
#if RL_LOG_REREAD == 2
  log_order();
  return *e;
#else
  const uint32_t* hd = reinterpret_cast<const uint32_t*>(e);
  return make_uint4(__hip_atomic_load(hd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                    __hip_atomic_load(hd + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                    __hip_atomic_load(hd + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                    __hip_atomic_load(hd + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#endif
}

#ifndef RL_LOG_TEAR
#define RL_LOG_TEAR 0
#endif
#if RL_LOG_TEAR
// Test builds: the armed rl_log_tear (include/ratelimit_hip.h, u32 words)
// fires at the first entry the next lookup reads. Its writer's steps are
// applied by the reading lane itself between its loads, per the schedule.
enum : uint32_t { TR_ARMED = 0, TR_PROTO = 1, TR_SCHED = 2, TR_ENTRY = 5, TR_BEFORE = 13, TR_SEEN = 21,
                  TR_VERDICT = 33 };
struct LogTear {
  uint32_t* p = nullptr;
  uint4 h, r;
  uint32_t done = 0, n = 0;
  bool legacy = false;
  __device__ inline void fire(const TableDev& t, uint4* e, uint32_t si, uint32_t tag) {
    if (!t.tear || atomicCAS(&t.tear[TR_ARMED], 1u, 2u) != 1u) return;
    p = t.tear;
    const uint4 a = e[0], b = e[1];
    const uint32_t o[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}, own[4] = {si, tag, a.z, a.w};
    uint32_t v[8];
    for (uint32_t k = 0; k < 8; k++) {
      p[TR_BEFORE + k] = o[k];
      v[k] = p[TR_ENTRY + k];
      if (k < 4 && v[k] == 0xFFFFFFFFu) v[k] = own[k];  // (the entry's own slot / tag / prev / t_app)
    }
    h = make_uint4(v[0], v[1], v[2], v[3]);
    r = make_uint4(v[4], v[5], v[6], v[7]);
    legacy = p[TR_PROTO] != 0;
    n = legacy ? 2u : LOG_WRITE_STEPS;
  }
  __device__ inline void to(uint4* e, uint32_t upto) {  // the writer's steps before the reader's next load
    for (; p && done < upto && done < n; done++) log_write_step(e, done, h, r, legacy);
  }
  __device__ inline void before_load(uint4* e, uint32_t i) {
    if (p) to(e, p[TR_SCHED + i]);
  }
  __device__ inline void seen(uint32_t i, const uint4& v) {
    if (!p) return;
    p[TR_SEEN + 4 * i] = v.x;
    p[TR_SEEN + 4 * i + 1] = v.y;
    p[TR_SEEN + 4 * i + 2] = v.z;
    p[TR_SEEN + 4 * i + 3] = v.w;
  }
  __device__ inline void verdict(uint4* e, int v) {
    if (!p) return;
    to(e, n);  // (the writer finishes)
    p[TR_VERDICT] = (uint32_t)v;
    p = nullptr;
  }
};
#else
struct LogTear {  // (product builds: no hook)
  __device__ __forceinline__ void fire(const TableDev&, uint4*, uint32_t, uint32_t) {}
  __device__ __forceinline__ void before_load(uint4*, uint32_t) {}
  __device__ __forceinline__ void seen(uint32_t, const uint4&) {}
  __device__ __forceinline__ void verdict(uint4*, int) {}
};
#endif

// The newest logged record of window w on slot si's chain from head (cur_ws:
// the slot's newest window): 1 found (*out), 0 none on the chain, -1 an
// entry on the way was overwritten (the log wrapped) before w could be ruled
// out. An entry overwritten by a newer one of the same slot (the owner check
// passes) lies on the chain already: the walk comes back to it, a cycle that
// Brent's check finds within twice its length.
__device__ inline int log_find(const TableDev& t, uint32_t head, uint32_t si, uint32_t tag, uint32_t cur_ws,
                               uint32_t w, Win* out) {
  uint32_t ptr = head, tprev = cur_ws, saved = LOG_NONE, power = 1, lam = 0;
  for (uint32_t hops = 0; ptr != LOG_NONE; hops++) {
    const uint32_t pos = ptr & LOG_POS_MASK;
    if (hops == LOG_MAX_HOPS || pos >= t.log_cap || ptr == saved) break;
    if (++lam == power) {
      saved = ptr;
      power <<= 1;
      lam = 0;
    }
    uint4* e = reinterpret_cast<uint4*>(&t.log[(size_t)(ptr >> LOG_POS_BITS) * t.log_cap + pos]);
    LogTear tr;
    tr.fire(t, e, si, tag);
    tr.before_load(e, 0);
    const uint4 a = e[0];
    tr.seen(0, a);
    log_order();
    tr.before_load(e, 1);
    const uint4 b = e[1];
    tr.seen(1, b);
    log_order();
    tr.before_load(e, 2);
#if RL_LOG_REREAD == 0
    const uint4 a2 = b.x == w ? log_hdr_reread(e) : a;
#else
    const uint4 a2 = log_hdr_reread(e);
#endif
    tr.seen(2, a2);
    // overwritten (owner, order), being written (BUSY), or rewritten between the loads
    if (a.x != si || a.y != tag || a.w > tprev || a2.x != a.x || a2.y != a.y || a2.z != a.z || a2.w != a.w) {
      tr.verdict(e, -1);
      break;
    }
    if (b.x == w) {
      tr.verdict(e, 1);
      *out = Win{b.x, b.y, b.z, b.w};
      return 1;
    }
    tr.verdict(e, 0);
    if (a.w <= w) return 0;  // every older entry holds a window below its t_app <= w
    tprev = a.w;
    ptr = a.z;
  }
  if (ptr == LOG_NONE) return 0;
  atomicAdd(t.hist_lost, 1ull);
  return -1;
}

// find_slot with insert, returning the slot's image (a fresh slot's image for
// an insert: no window, no flags). `im` holds the
// home slot's first sector on entry (the caller issues that load early,
// beside the stem's).
__device__ __attribute__((always_inline)) inline int64_t find_slot_img(const TableDev& t, uint64_t hstem, uint32_t tag, const Key& key, uint32_t unit,
                                 bool* inserted, SlotImg& im, uint32_t* err) {
  uint64_t i = hstem >> t.shift;
  int64_t tomb = -1;
  *inserted = false;
  for (uint32_t p = 0; p < t.max_probe; p++, i = (i + 1) & t.mask) {
    if (p) load_img_lo(&t.slots[i], im);
    const uint32_t st = im.tag();
    if (st == tag) {  // (a 32-bit tag is a filter: the unit and the stem bytes decide)
      if (im.unit() == unit && img_key_equal(im, key, t.arena)) return (int64_t)i;
      continue;
    }
    if (st == TAG_TOMB) {
      if (tomb < 0) tomb = (int64_t)i;
      continue;
    }
    if (st != TAG_EMPTY) continue;
    int64_t at = -1;
    int c = tomb >= 0 ? slot_claim(t, (uint64_t)tomb, TAG_TOMB, tag, key, unit) : 0;
    if (c > 0) at = tomb;
    if (c == 0) c = slot_claim(t, i, TAG_EMPTY, tag, key, unit);
    if (c > 0 && at < 0) at = (int64_t)i;
    if (c < 0) {
      atomicOr(err, ERR_ARENA_FULL);
      return SLOT_ARENA_FULL;
    }
    if (at >= 0) {
      im.v[0] = make_uint4(tag, key.len | (unit << 16), WS_INVALID, 0u);
      im.v[1] = make_uint4(0u, 0u, RING_NONE, 0u);
      *inserted = true;
      return at;
    }
    // another stem claimed this slot concurrently: keep probing
  }
  atomicOr(err, ERR_TABLE_FULL);
  return SLOT_TABLE_FULL;
}

// ===========================================================================
// Per-rule stats. Each lane sums its run's deltas in registers (u64); at the
// end the wave reduces lane sums rule by rule (butterfly shuffles) and one lane
// adds them to the block's LDS table, which is flushed once per block into one
// of STAT_STRIPES global partial tables (spreads same-address atomics), folded
// into rl_result.stats by k_finish. With more than LDS_RULES rules the
// wave sums go straight to rl_result.stats.
// ===========================================================================
constexpr uint32_t LDS_RULES = STAT_LDS_RULES;

// Block stats table in dynamic LDS (n_rules x RL_NUM_STATS u64, n_rules <= LDS_RULES).
extern __shared__ unsigned long long rl_sacc[];

struct StatAcc {
  bool use_lds;
  unsigned long long* glob;  // rl_result.stats (no LDS)
  __device__ inline void add(uint32_t rule, uint32_t which, unsigned long long v) {
    if (!v) return;
    if (use_lds) atomicAdd(&rl_sacc[rule * RL_NUM_STATS + which], v);
    else atomicAdd(&glob[(size_t)rule * RL_NUM_STATS + which], v);
  }
};

struct LaneStats {
  uint32_t rule;
  bool has;
  unsigned long long v[RL_NUM_STATS];
  __device__ inline void reset() {
    has = false;
#pragma unroll
    for (int i = 0; i < RL_NUM_STATS; i++) v[i] = 0;
  }
  __device__ inline void add(StatAcc& acc, uint32_t r, const uint32_t d[RL_NUM_STATS]) {
    if (has && rule != r) {  // rule changed inside this lane's run: flush directly
#pragma unroll
      for (int i = 0; i < RL_NUM_STATS; i++) acc.add(rule, i, v[i]);
      reset();
    }
    rule = r;
    has = true;
#pragma unroll
    for (int i = 0; i < RL_NUM_STATS; i++) v[i] += d[i];
  }
};

__device__ inline unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

// All lanes of the wave must call this (converged).
__device__ __attribute__((always_inline)) inline void wave_flush(LaneStats& L, StatAcc& acc) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t pending = __ballot(L.has);
  while (pending) {
    const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)pending) - 1);
    const uint32_t r = __shfl(L.rule, leader);
    const bool mine = L.has && L.rule == r;
#pragma unroll
    for (int i = 0; i < RL_NUM_STATS; i++) {
      const unsigned long long s = wave_sum(mine ? L.v[i] : 0ull);
      if (lane == leader) acc.add(r, i, s);
    }
    if (mine) L.has = false;
    pending = __ballot(L.has);
  }
}

__device__ inline void stats_block_begin(bool use_lds, uint32_t n_rules) {
  if (use_lds)
    for (uint32_t j = threadIdx.x; j < n_rules * RL_NUM_STATS; j += blockDim.x) rl_sacc[j] = 0;
  __syncthreads();
}

__device__ inline void stats_block_end(bool use_lds, uint32_t n_rules, unsigned long long* stripes) {
  __syncthreads();
  if (use_lds) {
    unsigned long long* dst = stripes + (size_t)(blockIdx.x % STAT_STRIPES) * n_rules * RL_NUM_STATS;
    for (uint32_t j = threadIdx.x; j < n_rules * RL_NUM_STATS; j += blockDim.x) {
      const unsigned long long v = rl_sacc[j];
      if (v) atomicAdd(&dst[j], v);
    }
  }
}

// ===========================================================================
// Replaying a stem's descriptors in arrival order.
//
// Per descriptor (fixed_cache_impl.go:33-113, base_limiter.go:45-197):
//   h = max(1, HitsAddend); TotalHits += h
//   local-cache check against the state BEFORE this request's statuses
//   (all of a request's checks precede its INCRBYs; its Sets follow them)
//   hit & !shadow -> OVER via local cache, no INCRBY
//   hit &  shadow -> no INCRBY, after = 0 (quirk: OK with the full limit)
//   else          -> INCRBY (a key past its EXPIRE reads 0), EXPIRE = now+div
//   status + stats (decide), localCache.Set(key, div) when over.
// ===========================================================================
struct Elem {
  uint32_t e, req, now, unit, d, w, h, thr, rule;
  bool shadow;
  uint8_t flags;
};

__device__ inline Elem load_elem(const Rec& r, uint32_t e, bool restore) {
  Elem x;
  x.e = e;
  x.req = r.req;
  x.now = r.now;
  x.unit = rec_unit(r);
  x.d = div_of(x.unit);
  x.w = x.now - x.now % x.d;
  x.h = restore ? r.hits : (r.hits > 1 ? r.hits : 1u);  // utils.Max(1, HitsAddend)
  x.thr = r.limit;
  x.rule = r.rule;
  x.flags = (uint8_t)(rec_flags(r) & RL_FLAG_SHADOW);  // (restore records: the local-cache bit)
  x.shadow = (x.flags & RL_FLAG_SHADOW) != 0;
  return x;
}

// One 8-B store per descriptor (pack_res): remaining, reset, code and the
// local-cache Get hit (k_finish counts them for the hitCount gauge).
__device__ __attribute__((always_inline)) inline void emit(unsigned long long* res, LaneStats& L, StatAcc& acc,
                                                           const Elem& x, const Decision& r, bool lc_get) {
  const uint32_t reset = x.d - x.now % x.d;  // utils.CalculateReset
  res[x.e] = pack_res(r.remaining, reset, r.code, lc_get);
  const uint32_t d[RL_NUM_STATS] = {x.h, r.d_over, r.d_near, r.d_lc, r.d_within, r.d_shadow};
  L.add(acc, x.rule, d);
}

// ---- single (stem, unit) slot, stem never seen with another unit: registers
// only. cur is the slot's newest window; `old` caches one older record (that
// of the last older window touched: the old cur after a roll, or one found on
// the slot's history chain), appended to the log when another one is needed
// or at the end, if it changed and a request could still ask for it.
struct SimpleState {
  Win cur, old;
  uint32_t si, tag;  // the slot and its tag (owner of its log entries)
  uint32_t chain;    // head of the slot's history chain (Slot::ring)
  bool cur_dirty, old_dirty, chain_dirty;
  uint32_t cur_req;
  bool pend;
  uint32_t pend_w, pend_e;
  __device__ inline void apply_pending() {
    if (pend) {
      if (cur.ws == pend_w) {
        cur.lc = pend_e;
        cur_dirty = true;
      } else if (old.ws == pend_w) {
        old.lc = pend_e;
        old_dirty = true;
      }
      pend = false;
    }
  }
};

// S.old to the log (a new version on the slot's chain: lookups take the newest)
__device__ __attribute__((always_inline)) inline void simple_put(const TableDev& t, SimpleState& S) {
  S.chain = log_append(t, S.si, S.tag, S.chain, S.cur.ws, S.old);
  S.chain_dirty = true;
  S.old_dirty = false;
}

// The record of window w: 0 = cur (rolled forward when w is newer: the old cur
// becomes S.old while a request could still ask for it), 1 = S.old, the
// record of an older w (found on the chain, or started afresh when w never
// had one), -1 = w's record may have been dropped or overwritten (RL_E_TIME,
// never a silently wrong count).
__device__ __attribute__((always_inline)) inline int simple_pick(const TableDev& t, SimpleState& S, uint32_t w, uint32_t d,
                                                                 uint32_t now) {
  if (S.cur.ws == w) return 0;
  if (S.cur.ws == WS_INVALID || w > S.cur.ws) {
    if (S.cur.ws != WS_INVALID) {
      if (S.old_dirty) simple_put(t, S);
      // a key revisited after more than HIST_W windows with the horizon past
      // (C1's SECOND keys at J = 0): nothing written
      if (hist_keep(t, S.cur, w, d)) {
        S.old = S.cur;
        S.old_dirty = true;
      }
    }
    S.cur = Win{w, 0, 0, 0};
    return 0;
  }
  if (S.old.ws != w) {
    if (S.old_dirty) simple_put(t, S);
    Win r;
    const int f = S.chain == LOG_NONE ? 0 : log_find(t, S.chain, S.si, S.tag, S.cur.ws, w, &r);
    // (an overwritten entry on the way: w's record may be gone, fine once dead)
    if (f < 0 ? !hist_dead(now, w, d) : (f == 0 && !hist_absent_ok(t, now, w, S.cur.ws, d))) return -1;
    S.old = f > 0 ? r : Win{w, 0, 0, 0};
    S.old_dirty = false;
  }
  return 1;
}

__device__ __attribute__((always_inline)) inline void simple_step(const TableDev& t, const Params& P, unsigned long long* res,
                                                                  LaneStats& L, StatAcc& acc, SimpleState& S,
                                                                  const Elem& x, bool restore, uint32_t* err) {
  if (x.req != S.cur_req) {
    S.apply_pending();
    S.cur_req = x.req;
  }
  const int which = simple_pick(t, S, x.w, x.d, x.now);
  if (which < 0) {  // its window's record may be gone: this descriptor's RL_E_TIME
    if (P.isolate) res[x.e] = pack_fail(RL_E_TIME);
    if (!(RL_ABL & 1)) atomicOr(err, ERR_HISTORY);  // (ablation builds probe garbage slots)
    return;
  }
  Win R = which ? S.old : S.cur;  // values, not pointers: the state stays in VGPRs
  uint32_t after = 0;
  bool lc_hit = false;
  if (restore) {
    R.count = x.h;
    R.expire = x.now + x.d;
    if (x.flags) R.lc = x.now + x.d;  // restore records: flags = local-cache bit
  } else {
    lc_hit = P.lc_en && x.now < R.lc;  // freecache Get (hit while now < expireAt)
    if (!lc_hit) {
      const uint32_t v = x.now <= R.expire ? R.count : 0u;  // a key past its EXPIRE reads as missing
      R.count = v + x.h;                                     // INCRBY
      R.expire = x.now + x.d;                                // EXPIRE div (jitter draw 0)
      after = R.count;
    }
  }
  if (which) {
    S.old = R;
    S.old_dirty = true;
  } else {
    S.cur = R;
    S.cur_dirty = true;
  }
  if (restore) return;
  const Decision r = decide(after - x.h, after, lc_hit && !x.shadow, x.h, x.thr, P.ratio, x.shadow, P.lc_en);
  if (r.set_lc) {
    S.pend = true;
    S.pend_w = x.w;
    S.pend_e = x.now + x.d;
  }
  emit(res, L, acc, x, r, lc_hit);
}

// ---- general: every unit slot of the stem, Redis keys shared across units.
// Each unit's cur lives in registers, with two older records per unit cached
// beside it (old, and vic: the one old held before), each appended to the
// unit slot's chain when a third one is needed, or at the end, if it changed.
// Two, because a multi-unit stem's replay alternates between two older windows
// of one slot: a SECOND request's own window and the minute's first second,
// which is also the key of every MINUTE request of that minute
// (cache_key.go:73-74); with one, every switch appended a version (one per
// descriptor of a hot stem: thousands into one partition per batch). The exact
// path is rare.
struct GeneralState {
  int64_t sidx[4];
  Win cur[4];
  Win old[4];         // per unit: an older record (WS_INVALID: none cached)
  Win vic[4];         // per unit: the older record old held before (WS_INVALID: none)
  uint32_t tag[4];    // each unit slot's tag (owner of its log entries)
  uint32_t chain[4];  // each unit slot's history chain head
  uint32_t odirty;    // bit u-1: old[u-1] changed
  uint32_t vdirty;    // bit u-1: vic[u-1] changed
  uint32_t cdirty;    // bit u-1: chain[u-1] changed
  uint32_t present;   // bit u-1
  uint32_t cur_req;
  uint32_t npend;
  uint32_t pend_w[4], pend_e[4];
};

__device__ inline bool ps_class(const Params& P, uint32_t k) { return P.per_second && k == 0; }

// old[k] (vic: vic[k]) to the log
__device__ inline void gen_put(const TableDev& t, GeneralState& G, uint32_t k, bool vic = false) {
  G.chain[k] = log_append(t, (uint32_t)G.sidx[k], G.tag[k], G.chain[k], G.cur[k].ws, vic ? G.vic[k] : G.old[k]);
  G.cdirty |= 1u << k;
  if (vic) G.vdirty &= ~(1u << k);
  else G.odirty &= ~(1u << k);
}

// old[k] becomes r; the one it held becomes vic[k] (whose record goes to the
// log first if it changed)
__device__ inline void gen_set_old(const TableDev& t, GeneralState& G, uint32_t k, const Win& r, bool dirty) {
  if ((G.vdirty >> k) & 1) gen_put(t, G, k, true);
  G.vic[k] = G.old[k];
  G.vdirty = (G.vdirty & ~(1u << k)) | (G.odirty & (1u << k));
  G.old[k] = r;
  G.odirty = (G.odirty & ~(1u << k)) | (dirty ? 1u << k : 0u);
}

// The record of window w in unit slot k (present): its cur, its cached older
// record (from the chain), or null when unit k has none. *lost: unit k may have
// had one, still live, that the history no longer holds.
__device__ inline Win* gen_rec(const TableDev& t, GeneralState& G, uint32_t k, uint32_t w, uint32_t now, bool* lost) {
  const uint32_t d = div_of(k + 1);
  Win& c = G.cur[k];
  if (c.ws == w) return &c;
  if (c.ws == WS_INVALID || w > c.ws || w % d) return nullptr;  // (unit k's keys are multiples of its div)
  if (G.old[k].ws == w) return &G.old[k];
  if (G.vic[k].ws == w) {  // the two cached older records trade places
    const Win v = G.vic[k];
    G.vic[k] = G.old[k];
    G.old[k] = v;
    const uint32_t b = 1u << k, od = G.odirty & b;
    G.odirty = (G.odirty & ~b) | (G.vdirty & b);
    G.vdirty = (G.vdirty & ~b) | od;
    return &G.old[k];
  }
  Win r;
  const int f = G.chain[k] == LOG_NONE ? 0 : log_find(t, G.chain[k], (uint32_t)G.sidx[k], G.tag[k], c.ws, w, &r);
  if (f > 0) {
    gen_set_old(t, G, k, r, false);
    return &G.old[k];
  }
  if (lost && (f < 0 ? !hist_dead(now, w, d) : !hist_absent_ok(t, now, w, c.ws, d))) *lost = true;
  return nullptr;
}

__device__ inline void gen_touch(GeneralState& G, uint32_t k, const Win* R) {
  if (R == &G.old[k]) G.odirty |= 1u << k;
}

__device__ inline void general_apply_pending(const TableDev& t, GeneralState& G) {
  for (uint32_t j = 0; j < G.npend; j++) {
    for (uint32_t k = 0; k < 4; k++) {
      if (!(G.present >> k & 1)) continue;
      Win* R = gen_rec(t, G, k, G.pend_w[j], 0u, nullptr);
      if (R) {
        R->lc = G.pend_e[j];
        gen_touch(G, k, R);
      }
    }
  }
  G.npend = 0;
}

__device__ inline void general_step(const TableDev& t, const Params& P, unsigned long long* res, LaneStats& L,
                                    StatAcc& acc, GeneralState& G, const Elem& x, bool restore, uint32_t* err) {
  if (x.req != G.cur_req) {
    general_apply_pending(t, G);
    G.cur_req = x.req;
  }
  const uint32_t ui = x.unit - 1;
  const bool ps_e = ps_class(P, ui);
  bool lc_hit = false, lost = false;
  uint32_t v = 0, lcw = 0;
  bool vfound = false;
  for (uint32_t k = 0; k < 4; k++) {
    if (!(G.present >> k & 1)) continue;
    const Win* R = gen_rec(t, G, k, x.w, x.now, &lost);
    if (!R) continue;
    if (x.now < R->lc) lc_hit = true;
    lcw = R->lc > lcw ? R->lc : lcw;
    if (ps_class(P, k) == ps_e && !vfound && x.now <= R->expire) {
      v = R->count;
      vfound = true;
    }
  }
  if (lost) {  // a record of w the history may have dropped while it could be live: RL_E_TIME
    if (P.isolate) res[x.e] = pack_fail(RL_E_TIME);
    atomicOr(err, ERR_HISTORY);
    return;
  }
  lc_hit = lc_hit && P.lc_en && !restore;
  uint32_t after = 0;
  if (!lc_hit) {
    const uint32_t nv = restore ? x.h : v + x.h;
    const uint32_t ex = x.now + x.d;
    Win& c = G.cur[ui];  // this unit's record of w: cur, a roll, its cached older record or a new one
    if (c.ws != x.w) {
      if (c.ws == WS_INVALID || x.w > c.ws) {
        if (c.ws != WS_INVALID && hist_keep(t, c, x.w, x.d)) gen_set_old(t, G, ui, c, true);  // the old cur
        c = Win{x.w, 0, 0, lcw};
      } else if (G.old[ui].ws != x.w) {  // (none found above, and none lost)
        gen_set_old(t, G, ui, Win{x.w, 0, 0, lcw}, true);
      }
    }
    for (uint32_t k = 0; k < 4; k++) {  // Redis key stem‖w in this store: every alias record
      if (!(G.present >> k & 1) || ps_class(P, k) != ps_e) continue;
      Win* R = gen_rec(t, G, k, x.w, x.now, nullptr);
      if (R) {
        R->count = nv;
        R->expire = ex;
        gen_touch(G, k, R);
      }
    }
    after = nv;
  }
  if (restore) {
    if (x.flags) {
      for (uint32_t k = 0; k < 4; k++) {
        if (!(G.present >> k & 1)) continue;
        Win* R = gen_rec(t, G, k, x.w, x.now, nullptr);
        if (R) {
          R->lc = x.now + x.d;
          gen_touch(G, k, R);
        }
      }
    }
    return;
  }
  const Decision r = decide(after - x.h, after, lc_hit && !x.shadow, x.h, x.thr, P.ratio, x.shadow, P.lc_en);
  if (r.set_lc) {  // freecache Set: last write wins, applied after this request
    uint32_t j = 0;
    while (j < G.npend && G.pend_w[j] != x.w) j++;
    if (j == G.npend) G.npend++;
    G.pend_w[j] = x.w;
    G.pend_e[j] = x.now + x.d;
  }
  emit(res, L, acc, x, r, lc_hit);
}

// Replay elements [p, end) (those of group k when grp is given) through the
// single-unit slot s0, in registers.
__device__ __attribute__((always_inline)) inline void replay_simple(SRec rec_s, const uint32_t* svals,
                                                                    unsigned long long* res, const TableDev& t,
                                                                    const Params& P, const uint32_t* grp,
                                                                    uint32_t p, uint32_t end, uint32_t k, int64_t s0,
                                                                    Win cur0, uint32_t ring0, uint32_t tag0,
                                                                    const Rec& x0, uint32_t e0, LaneStats& L,
                                                                    StatAcc& acc, uint32_t* err, bool restore) {
  Slot* s = &t.slots[s0];
  SimpleState S;
  S.cur = cur0;
  S.old = Win{WS_INVALID, 0, 0, 0};  // (never matches a pending window)
  S.si = (uint32_t)s0;
  S.tag = tag0;
  S.chain = ring0;
  S.cur_dirty = S.old_dirty = S.chain_dirty = false;
  S.cur_req = 0xFFFFFFFFu;
  S.pend = false;
  simple_step(t, P, res, L, acc, S, load_elem(x0, e0, restore), restore, err);  // element p (always stem k)
  for (uint32_t q = p + 1; q < end; q++) {
    if (grp && grp[q] != k) continue;
    simple_step(t, P, res, L, acc, S, load_elem(rec_s[q], svals[q], restore), restore, err);
  }
  S.apply_pending();
  // random writes are the costly part of the probe: store only what changed
  if (S.old_dirty) simple_put(t, S);
  if (S.cur_dirty) s->cur = S.cur;
  if (S.chain_dirty) s->ring = S.chain;
}

// ===========================================================================
// Run segmentation of the sorted order (3 phases over tiles of SEG_TILE):
// a run starts where the sort key changes. Produces, per sorted position q,
// the run id and the inclusive in-run sum of max(1, hits) (u32, wrapping like
// the sequential INCRBYs), and per run its start. Segmented-sum operator on
// (head, sum): (f1,s1)+(f2,s2) = (f1|f2, f2 ? s2 : s1+s2).
// Layout: each wave owns a strip of SEG_TILE/4 consecutive positions and walks
// it in SEG_ITEMS chunks of 64 (one position per lane), so every load and
// store is a coalesced 256-B wave access; scans are wave shuffles.
// ===========================================================================
__device__ __attribute__((always_inline)) inline uint32_t wave_incl_add(uint32_t x);
struct SegPair {
  uint32_t f, s;
};
__device__ inline SegPair seg_op(SegPair a, SegPair b) { return SegPair{a.f | b.f, b.f ? b.s : a.s + b.s}; }

struct SegChunk {
  uint64_t heads;  // ballot of run heads in the chunk
  uint32_t h;      // this lane's max(1, hits) (0 past n)
};

__device__ inline SegPair seg_chunk_scan(const SegChunk& c, uint32_t lane) {
  const uint32_t P = wave_incl_add(c.h);  // (all 64 lanes active: the callers' chunk loops are wave-uniform)
  const uint64_t le = c.heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
  const uint32_t lh = le ? 63u - (uint32_t)__clzll((long long)le) : 0u;
  const uint32_t Plh = __shfl(P, lh, 64), hlh = __shfl(c.h, lh, 64);
  return le ? SegPair{1u, P - (Plh - hlh)} : SegPair{0u, P};
}

// Block-level combine of the 4 wave aggregates: returns this wave's exclusive
// prefix within the tile (and the tile aggregate through *tot for lane 0 of
// wave 0 callers).
// ===========================================================================
// Grouping by MSD partition + per-bucket LDS sort (stage A).
//
// k_part: every PART_TILE tile of (sort key, index, hits), in arrival order,
// is stably partitioned by the key's top PART_BITS bits into its own tile
// region (one wave-ballot multisplit rank, digit segments), and records per
// digit its (offset, count) in the tile. No look-back and no atomics: bucket d
// is the concatenation, in tile (= arrival) order, of every tile's digit-d
// segment; its size is the sum of the counts and its place in the sorted batch
// the sum of the offsets (each offset counts the tile's smaller digits).
// k_bucket: one 4-wave workgroup per bucket (several per CU, so one group's
// barriers overlap another's work). It gathers the bucket, stably sorts it by
// the remaining 22 key bits (three multisplit passes in LDS), so the batch ends
// up sorted by the full key with arrival order kept within equal keys, and
// segments it in place (runs never cross buckets): in-run inclusive sums of
// max(1, hits), run ids and [run_start, run_end). Run ids are allocated per
// bucket from one atomic counter, contiguous and in sorted order within a
// bucket. Buckets larger than its LDS capacity are queued for k_bucket_big.
// k_bucket_big: 8-wave workgroups (register budget for 16 items per lane)
// over the queued buckets: the hot keys of a large bucket are peeled off
// (sampled, then moved as whole blocks in arrival order) and the rest sorted
// in LDS; failing that, the three passes run chunk by chunk through HBM.
// ===========================================================================
constexpr uint32_t BK_HEAVY = BIG_HEAVY;  // heavy keys peeled off a large bucket
constexpr uint32_t BK_HEAVY_MIN = 3;  // ... seen at least this often among the samples (sample_heavy)

template <uint32_t W, uint32_t IT>
struct BkShape {
  static constexpr uint32_t WAVES = W, ITEMS = IT, THREADS = 64 * W, CAP = 64 * W * IT, STRIP = 64 * IT;
};
using BkSmall = BkShape<4, 8>;   // k_bucket: 2048 elements in LDS
using BkBig = BkShape<8, 8>;     // k_bucket_big: 4096 elements per chunk (~62 KB of LDS: 2 workgroups per CU)

#ifdef RL_BK_PROF  // bucketbench only: per-bucket phase stamps
__device__ unsigned long long g_bk_prof[PART_DIGITS * 16];
__device__ uint32_t g_bk_peel[PART_DIGITS * 16];  // peel state per bucket
#define BK_STAMP(d, k) \
  if (threadIdx.x == 0) g_bk_prof[(d) * 16 + (k)] = wall_clock64()
#else
#define BK_STAMP(d, k)
#endif

// Wave-ballot multisplit on the BITS-bit digit at `shift`: rank of each item
// among the wave's earlier items with the same digit, against a wave-private
// running count row in LDS (item-major order: item i of lane l precedes item i
// of lane l+1 and item i+1 of lane 0). The digit group leaders add to the row
// with returning LDS atomics, issued back to back for all items (LDS applies
// them in order), then every lane fetches its leader's old count.
template <uint32_t IT, uint32_t BITS>
__device__ inline void wave_multisplit(const uint32_t (&kk)[IT], uint32_t nvalid_base, uint32_t limit, uint32_t shift,
                                       uint32_t* row, uint32_t (&pos)[IT]) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lt_mask = (1ull << lane) - 1;
  uint32_t leader[IT];
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) {
    leader[i] = lane;
    pos[i] = 0;
    if (nvalid_base + i * 64 >= limit) continue;  // wave-uniform: no item of the wave left
    const bool valid = nvalid_base + i * 64 + lane < limit;
    const uint32_t d = (kk[i] >> shift) & ((1u << BITS) - 1u);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (uint32_t bit = 0; bit < BITS; bit++) {
      const bool sb = (d >> bit) & 1u;
      const uint64_t bal = __ballot(sb);
      peers &= sb ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lt_mask);
    leader[i] = valid ? (uint32_t)(__ffsll((unsigned long long)peers) - 1) : lane;
    pos[i] = (valid && rank == 0) ? atomicAdd(&row[d], (uint32_t)__popcll(peers)) : 0u;
    pos[i] |= rank << 16;  // rank < 64; old counts < 2^16 (at most a chunk / a tile)
  }
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) pos[i] = __shfl(pos[i] & 0xFFFFu, leader[i]) + (pos[i] >> 16);
}

// Exclusive scan of one value per thread over threads [0, 256) (waves 0..3);
// every thread of the block must call it. *total = sum of the 256 values.
__device__ inline uint32_t scan256(uint32_t v, uint32_t* wsum4, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(inc, off, 64);
    if (lane >= off) inc += y;
  }
  if (wave < 4 && lane == 63) wsum4[wave] = inc;
  __syncthreads();
  uint32_t pre = 0;
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) pre += w < wave ? wsum4[w] : 0u;
  if (total) *total = wsum4[0] + wsum4[1] + wsum4[2] + wsum4[3];
  __syncthreads();
  return pre + inc - v;
}

__global__ __launch_bounds__(256) void k_part(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ hin,
                                              uint4* __restrict__ out, uint32_t n, uint32_t ntiles,
                                              uint32_t* __restrict__ info, const uint32_t* err) {
  constexpr uint32_t DPT = PART_DIGITS / 256;  // digits per thread
  __shared__ uint32_t wcnt[4][PART_DIGITS];
  __shared__ uint32_t wsum[4];
  // the tile in partitioned order (key, index, hits), written out as whole lines
  __shared__ uint32_t sk[PART_TILE], sv[PART_TILE], sh[PART_TILE];
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, tile = blockIdx.x;
  for (uint32_t j = tid; j < 4 * PART_DIGITS; j += 256) (&wcnt[0][0])[j] = 0;
  __syncthreads();
  const uint32_t wbase = tile * PART_TILE + wave * 64 * PART_ITEMS;
  uint32_t kk[PART_ITEMS], vv[PART_ITEMS], hh[PART_ITEMS], pos[PART_ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < PART_ITEMS; i++) {
    const uint32_t j = min(wbase + i * 64 + lane, n - 1);  // unconditional loads, all in flight
    kk[i] = kin[j];
    vv[i] = j;  // the descriptor index
    hh[i] = hin[j];
  }
  wave_multisplit<PART_ITEMS, PART_BITS>(kk, wbase, n, 32 - PART_BITS, wcnt[wave], pos);
  __syncthreads();
  // digits tid*DPT .. tid*DPT+DPT-1: per-wave exclusive offsets and counts,
  // then the tile's exclusive digit offsets (scan over threads)
  uint32_t c[DPT], tsum = 0;
#pragma unroll
  for (uint32_t j = 0; j < DPT; j++) {
    const uint32_t d = tid * DPT + j;
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
      const uint32_t t = wcnt[w][d];
      wcnt[w][d] = acc;
      acc += t;
    }
    c[j] = acc;
    tsum += acc;
  }
  uint32_t excl = scan256(tsum, wsum, nullptr);
#pragma unroll
  for (uint32_t j = 0; j < DPT; j++) {
    const uint32_t d = tid * DPT + j;
    info[(size_t)d * ntiles + tile] = (excl << 16) | c[j];
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) wcnt[w][d] += excl;  // rows now hold tile-relative bases
    excl += c[j];
  }
  __syncthreads();
  // Scatter into LDS, then stream the tile out with consecutive 16-B stores:
  // scattering straight to HBM left ~4 records per digit segment, i.e. partial
  // 64-B lines (3.8x write amplification, profiles/r02/traffic_c1.json).
#pragma unroll
  for (uint32_t i = 0; i < PART_ITEMS; i++) {
    if (wbase + i * 64 + lane < n) {
      const uint32_t d = kk[i] >> (32 - PART_BITS);
      const uint32_t q = wcnt[wave][d] + pos[i];
      sk[q] = kk[i];
      sv[q] = vv[i];
      sh[q] = hh[i];
    }
  }
  __syncthreads();
  const uint32_t cnt = min(PART_TILE, n - tile * PART_TILE);
  uint4* o = out + (size_t)tile * PART_TILE;
#pragma unroll
  for (uint32_t i = 0; i < PART_ITEMS; i++) {
    const uint32_t q = i * 256 + tid;
    if (q < cnt) o[q] = make_uint4(sk[q], sv[q], sh[q], 0u);  // one 16-B record
  }
}

// LDS of one bucket workgroup (the tile segment table is in dynamic LDS).
template <typename B>
struct BucketLds {
  uint32_t k[B::CAP], v[B::CAP], h[B::CAP];  // a bucket / chunk in sorted order: key, index, hits
  uint32_t wcnt[B::WAVES][256];             // multisplit rows
  uint32_t gsum[B::WAVES / 4][256];         // digit counts per group of 4 waves
  uint32_t base[256];                       // digit offsets: chunk-local / running in the bucket
  uint32_t roff[3][256];                    // large buckets: running digit offsets per pass
  uint32_t dtot[256];
  uint32_t wsum[B::WAVES];
  SegPair sp[B::WAVES];
  uint32_t sh[B::WAVES];
  SegPair carry;
  uint32_t hcarry, rb, nruns, S, base_pos, db, dcnt;
  // large buckets: heavy keys peeled off (bucket_peel)
  uint32_t heavy[BK_HEAVY];           // sampled heavy keys (class c)
  uint32_t hcnt[BK_HEAVY];            // elements per class
  uint32_t hstart[BK_HEAVY];          // first bucket position of each class's block
  uint32_t hrun[BK_HEAVY];            // elements of the class placed so far
  uint32_t hw[B::WAVES][BK_HEAVY];    // per-wave class counts of a chunk
  uint32_t hsw[B::WAVES][BK_HEAVY];   // per-wave class sums of max(1, hits) of a chunk
  uint32_t acc[1 + 2 * BK_HEAVY];     // k_big_place: sums over the bucket's earlier chunks
  uint32_t lw[B::WAVES];              // per-wave light counts of a chunk
  uint32_t nheavy, nlight;
  uint32_t ub;                        // k_bucket: this bucket's first entry in the keys-seen-once list
};

extern __shared__ uint32_t bk_seg[];  // [ntiles + 1] segment starts, then [ntiles] sources

// Bucket positions -> indices in the tile layout: for each item the last tile
// t with seg[t] <= p (a segment holding p), by a fixed-depth search whose
// levels visit all items together (independent LDS reads in flight).
template <uint32_t IT>
__device__ inline void bucket_src(uint32_t ntiles, const uint32_t (&p)[IT], uint32_t (&j)[IT]) {
  const uint32_t* seg = bk_seg;
  const uint32_t* src = bk_seg + ntiles + 1;
  uint32_t lo[IT];
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) lo[i] = 0;
#pragma unroll
  for (uint32_t step = MAX_PART_TILES / 2; step; step >>= 1) {
    if (step >= ntiles) continue;  // uniform
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint32_t m = lo[i] + step;
      if (m < ntiles && seg[m] <= p[i]) lo[i] = m;
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) j[i] = src[lo[i]] + p[i];
}

// Wave-sum of v over the block (all threads call); result in every thread.
template <typename B>
__device__ inline uint32_t block_sum(BucketLds<B>& L, uint32_t v) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (uint32_t off = 32; off; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) L.wsum[wave] = v;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (uint32_t w = 0; w < B::WAVES; w++) s += L.wsum[w];
  __syncthreads();
  return s;
}

// Bucket d's size, its first position in the sorted batch and its tile
// segment table (starts = exclusive scan of the tile counts) in bk_seg.
template <typename B>
__device__ inline void bucket_setup(BucketLds<B>& L, const uint32_t* __restrict__ info, uint32_t ntiles, uint32_t d) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t* seg = bk_seg;
  uint32_t* src = bk_seg + ntiles + 1;
  uint32_t carry = 0, offs = 0;
  for (uint32_t t0 = 0; t0 < ntiles; t0 += B::THREADS) {
    const uint32_t t = t0 + tid;
    const uint32_t e = t < ntiles ? info[(size_t)d * ntiles + t] : 0u;
    const uint32_t cnt = e & 0xFFFFu;
    offs += e >> 16;
    uint32_t inc = cnt;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(inc, off, 64);
      if (lane >= off) inc += y;
    }
    if (lane == 63) L.wsum[wave] = inc;
    __syncthreads();
    uint32_t pre = carry, all = carry;
    for (uint32_t w = 0; w < B::WAVES; w++) {
      pre += w < wave ? L.wsum[w] : 0u;
      all += L.wsum[w];
    }
    if (t < ntiles) {
      const uint32_t st = pre + inc - cnt;
      seg[t] = st;
      src[t] = t * PART_TILE + (e >> 16) - st;
    }
    carry = all;
    __syncthreads();
  }
  const uint32_t bp = block_sum(L, offs);
  if (tid == 0) {
    seg[ntiles] = carry;
    L.S = carry;
    L.base_pos = bp;
  }
  __syncthreads();
}

// Rank one chunk (IT items per lane, wave-strip layout) by the BITS-bit digit
// at `shift`: pos = L.base[d] + (earlier waves' count of d) + rank in the
// wave. With chunk_scan, L.base becomes the chunk's own exclusive digit
// offsets first. L.dtot = the chunk's digit counts. Ends with a barrier.
template <typename B, uint32_t BITS>
__device__ inline void bucket_rank(BucketLds<B>& L, const uint32_t (&kk)[B::ITEMS], uint32_t strip0, uint32_t limit,
                                   uint32_t shift, bool chunk_scan, uint32_t (&pos)[B::ITEMS]) {
  const uint32_t tid = threadIdx.x, wave = tid >> 6;
  for (uint32_t j = tid; j < B::WAVES * 256; j += B::THREADS) (&L.wcnt[0][0])[j] = 0;
  __syncthreads();
  uint32_t local[B::ITEMS];
  wave_multisplit<B::ITEMS, BITS>(kk, strip0, limit, shift, L.wcnt[wave], local);
  __syncthreads();
  // per digit, exclusive offsets over the wave rows: thread (g, d) scans rows
  // 4g..4g+3 of digit d, then adds the totals of the groups before g
  constexpr uint32_t NG = B::WAVES / 4;
  const uint32_t dg = tid & 255u, g = tid >> 8;
  uint32_t r[4], c = 0;
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) r[w] = L.wcnt[g * 4 + w][dg];
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) {
    const uint32_t t = r[w];
    r[w] = c;
    c += t;
  }
  L.gsum[g][dg] = c;
  __syncthreads();
  uint32_t pre = 0, all = 0;
#pragma unroll
  for (uint32_t q = 0; q < NG; q++) {
    const uint32_t t = L.gsum[q][dg];
    pre += q < g ? t : 0u;
    all += t;
  }
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) L.wcnt[g * 4 + w][dg] = r[w] + pre;
  if (tid < 256) L.dtot[tid] = all;
  const uint32_t excl = scan256(tid < 256 ? all : 0u, L.wsum, nullptr);
  if (chunk_scan && tid < 256) L.base[tid] = excl;
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    const uint32_t d = (kk[i] >> shift) & ((1u << BITS) - 1u);
    pos[i] = L.base[d] + L.wcnt[wave][d] + local[i];
  }
  __syncthreads();
}

// Stable sort of n <= CAP (key, value, hits) triples held in wave-strip
// order in registers by key bits [0, 32 - PART_BITS): passes of 8, 8 and 6
// bits, each ranked in LDS and scattered through L.k / L.v / L.h. On return
// L.k / L.v / L.h and kk / vv / hh hold the sorted triples.
template <typename B>
__device__ inline void lds_sort3(BucketLds<B>& L, uint32_t (&kk)[B::ITEMS], uint32_t (&vv)[B::ITEMS],
                                 uint32_t (&hh)[B::ITEMS], uint32_t n) {
  static_assert(32 - PART_BITS == 22, "passes of 8 + 8 + 6 bits");
  const uint32_t lane = threadIdx.x & 63, strip0 = (threadIdx.x >> 6) * B::STRIP;
  uint32_t pos[B::ITEMS];
#pragma unroll 1
  for (uint32_t pass = 0; pass < 3; pass++) {
    if (pass < 2) bucket_rank<B, 8>(L, kk, strip0, n, 8 * pass, true, pos);
    else bucket_rank<B, 6>(L, kk, strip0, n, 16, true, pos);
#pragma unroll
    for (uint32_t i = 0; i < B::ITEMS; i++) {
      if (strip0 + i * 64 + lane < n) {
        L.k[pos[i]] = kk[i];
        L.v[pos[i]] = vv[i];
        L.h[pos[i]] = hh[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < B::ITEMS; i++) {
      const uint32_t p = strip0 + i * 64 + lane;
      if (p < n) {
        kk[i] = L.k[p];
        vv[i] = L.v[p];
        hh[i] = L.h[p];
      }
    }
  }
}

// Segment the sorted bucket [0, S) (keys / hits from LDS or from the sorted
// global arrays at base): in-run sums, run ids and run bounds. Chunks of CAP
// positions; each wave walks its strip of the chunk in 64-position pieces, and
// the wave aggregates plus the carry of the earlier chunks give every wave its
// exclusive prefix. Every gather is an unconditional load at a clamped
// position, issued in a straight-line loop before any use, so all of a lane's
// loads are in flight together (a load under a branch is waited for on the spot).
template <typename B, bool FROM_LDS>
__device__ inline void bucket_segment(BucketLds<B>& L, uint32_t d, uint32_t S, uint32_t base,
                                      const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sh,
                                      uint32_t* __restrict__ segsum, uint32_t* __restrict__ rid,
                                      uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_end,
                                      unsigned long long* num_runs, uint32_t* __restrict__ drun) {
  constexpr uint32_t IT = B::ITEMS;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto key = [&](uint32_t p) -> uint32_t { return FROM_LDS ? L.k[p] : sk[base + p]; };
  auto hit = [&](uint32_t p) -> uint32_t { return FROM_LDS ? L.h[p] : sh[base + p]; };
  // runs of the bucket -> run id base; runs of two or more (counted at their
  // second element) -> their place in the dup-run list k_table works through
  uint32_t nh = 0, nd = 0;
  for (uint32_t c0 = 0; c0 < S; c0 += B::CAP) {
    uint32_t a[IT], b[IT], c[IT];
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint32_t p = min(c0 + i * B::THREADS + tid, S - 1);
      a[i] = key(p ? p - 1 : 0);
      b[i] = key(p);
      c[i] = key(p > 1 ? p - 2 : 0);
    }
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint32_t p = c0 + i * B::THREADS + tid;
      nh += (p < S && (p == 0 || a[i] != b[i])) ? 1u : 0u;
      nd += (p < S && p >= 1 && a[i] == b[i] && (p == 1 || c[i] != a[i])) ? 1u : 0u;
    }
  }
  nh = block_sum(L, nh);
  nd = block_sum(L, nd);
  BK_STAMP(d, 4);
  if (tid == 0) {
    const unsigned long long old = atomicAdd(num_runs, ((unsigned long long)nd << 32) | nh);
    L.rb = (uint32_t)old;
    L.db = (uint32_t)(old >> 32);
    L.dcnt = 0;
    L.nruns = nh;
    L.carry = SegPair{0, 0};
    L.hcarry = 0;
  }
  __syncthreads();
  const uint32_t rb = L.rb;
  for (uint32_t c0 = 0; c0 < S; c0 += B::CAP) {
    const uint32_t s0 = c0 + wave * B::STRIP;
    const uint32_t ni = s0 >= S ? 0u : min(IT, (S - s0 + 63) / 64);  // items of this wave in the bucket
    SegChunk ch[IT];
    SegPair agg{0, 0};
    uint32_t hc = 0;
    uint32_t kp[IT], kq[IT], hq[IT], kpp[IT];
#pragma unroll
    for (uint32_t j = 0; j < IT; j++) {
      const uint32_t q = min(s0 + 64 * j + lane, S - 1);
      kp[j] = key(q ? q - 1 : 0);
      kq[j] = key(q);
      hq[j] = hit(q);
      kpp[j] = key(q > 1 ? q - 2 : 0);
    }
    uint32_t hd = 0, sd = 0;  // head flags / second-element flags, bit j
#pragma unroll
    for (uint32_t j = 0; j < IT; j++) {
      const uint32_t q = s0 + 64 * j + lane;
      hd |= (q < S && (q == 0 || kp[j] != kq[j])) ? 1u << j : 0u;
      sd |= (q < S && q >= 1 && kp[j] == kq[j] && (q == 1 || kpp[j] != kp[j])) ? 1u << j : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < IT; j++) {
      ch[j] = SegChunk{0, 0};
      if (j >= ni) continue;  // wave-uniform
      // max(1, HitsAddend) (utils.Max, fixed_cache_impl.go:41); 0 past the bucket
      const uint32_t hv = s0 + 64 * j + lane < S ? (hq[j] > 1 ? hq[j] : 1u) : 0u;
      ch[j] = SegChunk{(uint64_t)__ballot((hd >> j) & 1u), hv};
      uint32_t t = hv;  // piece total, segmented: sum after the last head
      const uint32_t lh = ch[j].heads ? 63u - (uint32_t)__clzll((long long)ch[j].heads) : 0u;
      if (ch[j].heads && lane < lh) t = 0;
#pragma unroll
      for (uint32_t off = 32; off; off >>= 1) t += __shfl_xor(t, off, 64);
      agg = seg_op(agg, SegPair{ch[j].heads ? 1u : 0u, t});
      hc += (uint32_t)__popcll(ch[j].heads);
    }
    if (lane == 0) {
      L.sp[wave] = agg;
      L.sh[wave] = hc;
    }
    __syncthreads();
    SegPair run = L.carry;
    uint32_t hrun = L.hcarry;
    SegPair tot = run;
    uint32_t htot = hrun;
    for (uint32_t w = 0; w < B::WAVES; w++) {
      if (w == wave) {
        run = tot;
        hrun = htot;
      }
      tot = seg_op(tot, L.sp[w]);
      htot += L.sh[w];
    }
    __syncthreads();
    if (tid == 0) {
      L.carry = tot;
      L.hcarry = htot;
    }
#pragma unroll
    for (uint32_t j = 0; j < IT; j++) {
      if (j >= ni) continue;  // wave-uniform
      const uint32_t q = s0 + 64 * j + lane;
      const SegPair v = seg_chunk_scan(ch[j], lane);
      const SegPair in = seg_op(run, v);
      const uint64_t heads = ch[j].heads;
      const uint32_t r = hrun + (uint32_t)__popcll(heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1))) - 1;
      if (q < S) {
        segsum[base + q] = in.s;
        rid[base + q] = rb + r;
        if ((heads >> lane) & 1) {
          run_start[rb + r] = base + q;
          if (r) run_end[rb + r - 1] = base + q;
        }
        if ((sd >> j) & 1) drun[L.db + atomicAdd(&L.dcnt, 1u)] = rb + r;  // (any order)
      }
      run = seg_op(run, SegPair{__shfl(v.f, 63, 64), __shfl(v.s, 63, 64)});
      hrun += (uint32_t)__popcll(heads);
    }
    __syncthreads();  // carry
  }
  if (tid == 0 && S) run_end[rb + L.nruns - 1] = base + S;
}

constexpr uint32_t BIG_CHUNK = BkSmall::CAP;
constexpr uint32_t BIG_LIGHT_CAP = BkBig::CAP;
constexpr uint32_t BIG_CNT = 1 + 2 * BK_HEAVY;  // per work item: light count, class counts, class hit sums

// Hot keys of a large bucket: 256 evenly spaced positions are sampled by wave
// 0 (4 per lane); keys seen at least BK_HEAVY_MIN times become
// L.heavy[0..L.nheavy). (64 samples missed a second hot key of ~8 % of the
// bucket now and then: its elements then overflowed the light part's LDS
// capacity and the whole bucket took the one-workgroup radix path, ~0.8 ms.)
constexpr uint32_t BK_SAMPLES_PER_LANE = 4;
template <typename B>
__device__ inline void sample_heavy(BucketLds<B>& L, uint32_t S, uint32_t ntiles, const uint4* __restrict__ pt) {
  constexpr uint32_t R = BK_SAMPLES_PER_LANE, NS = 64 * R;
  const uint32_t lane = threadIdx.x & 63;
  if ((threadIdx.x >> 6) == 0) {
    uint32_t p[R], j[R], ks[R], cnt[R];
    bool first[R];
#pragma unroll
    for (uint32_t i = 0; i < R; i++) p[i] = (uint32_t)(((uint64_t)(2 * (lane * R + i) + 1) * S) / (2 * NS));
    bucket_src(ntiles, p, j);
#pragma unroll
    for (uint32_t i = 0; i < R; i++) {
      ks[i] = pt[j[i]].x;
      cnt[i] = 0;
      first[i] = true;
    }
    for (uint32_t q = 0; q < 64; q++) {
#pragma unroll
      for (uint32_t r = 0; r < R; r++) {
        const uint32_t kq = __shfl(ks[r], q, 64), g = q * R + r;
#pragma unroll
        for (uint32_t i = 0; i < R; i++) {
          cnt[i] += kq == ks[i] ? 1u : 0u;
          if (g < lane * R + i && kq == ks[i]) first[i] = false;
        }
      }
    }
    uint32_t nc = 0;  // this lane's candidates, ranked across the wave
#pragma unroll
    for (uint32_t i = 0; i < R; i++) nc += (first[i] && cnt[i] >= BK_HEAVY_MIN) ? 1u : 0u;
    uint32_t incl = nc;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    uint32_t rank = incl - nc;
#pragma unroll
    for (uint32_t i = 0; i < R; i++)
      if (first[i] && cnt[i] >= BK_HEAVY_MIN) {
        if (rank < BK_HEAVY) L.heavy[rank] = ks[i];
        rank++;
      }
    if (lane == 63) L.nheavy = min(incl, BK_HEAVY);
  }
  __syncthreads();
}

__global__ __launch_bounds__(BkSmall::THREADS, 4) void k_bucket(
    const uint4* __restrict__ pt,
    const uint32_t* __restrict__ info, uint32_t ntiles, uint32_t* __restrict__ sk, uint32_t* __restrict__ sv,
    uint32_t* __restrict__ sh, uint32_t* __restrict__ segsum, uint32_t* __restrict__ rid,
    uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_end, unsigned long long* num_runs,
    uint32_t* __restrict__ drun, BigMeta* __restrict__ meta, uint32_t* big_n, uint32_t* __restrict__ work,
    uint32_t* work_n, uint32_t* sorted_n, uint2* __restrict__ uniq, uint32_t* uniq_n, const uint32_t* err,
    uint32_t* big_hint) {
  using B = BkSmall;
  __shared__ BucketLds<B> L;
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, d = blockIdx.x;
  BK_STAMP(d, 0);
  bucket_setup(L, info, ntiles, d);
  const uint32_t S = L.S;
  if (!S) return;
  if (S > B::CAP) {  // queued: hot keys sampled, their run ids and the chunk work items allocated
    sample_heavy(L, S, ntiles, pt);
    if (tid == 0) {
      BigMeta M;
      M.d = d;
      M.S = S;
      M.base = atomicAdd(sorted_n, S);  // (every element: the hot keys' bucket is mostly runs)
      M.r = L.nheavy;
      M.nchunks = M.r ? (S + BIG_CHUNK - 1) / BIG_CHUNK : 0u;
      M.item0 = M.nchunks ? atomicAdd(work_n, M.nchunks) : 0u;
      const unsigned long long old =
          M.r ? atomicAdd(num_runs, ((unsigned long long)M.r << 32) | M.r) : 0ull;  // hot keys: runs of >= 3
      M.rb_heavy = (uint32_t)old;
      M.db_heavy = (uint32_t)(old >> 32);
      for (uint32_t c = 0; c < BK_HEAVY; c++) M.heavy[c] = c < M.r ? L.heavy[c] : 0u;
      const uint32_t b = atomicAdd(big_n, 1u);
      meta[b] = M;
      if (big_hint) *big_hint = 1u;  // (the host's cue: full large-bucket grids for the next batches)
      L.rb = b;
      L.nruns = M.item0;
      L.hcarry = M.nchunks;
    }
    __syncthreads();
    for (uint32_t t = tid; t < L.hcarry; t += B::THREADS) work[L.nruns + t] = (L.rb << 16) | t;
    return;
  }
  BK_STAMP(d, 1);
  uint32_t kk[B::ITEMS], vv[B::ITEMS], hh[B::ITEMS];
  const uint32_t strip0 = wave * B::STRIP;
  uint32_t pp[B::ITEMS], jj[B::ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) pp[i] = min(strip0 + i * 64 + lane, S - 1);
  bucket_src(ntiles, pp, jj);
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    const uint4 e = pt[jj[i]];
    kk[i] = e.x;
    vv[i] = e.y;
    hh[i] = e.z;
  }
  BK_STAMP(d, 2);
  // Keys seen once in the batch never enter the sorted order: every
  // descriptor of a key falls in its bucket, so an LDS hash of the bucket's
  // keys finds the duplicated ones (~5% at C1), and only those are sorted,
  // segmented and written. Their sorted positions are one block per bucket,
  // allocated from sorted_n (runs never cross buckets, so no order between
  // buckets is needed). The keys seen once are listed, bucket by bucket, for
  // k_table's singleton part: their home slots share the bucket's top 10
  // bits, so a workgroup walking the list probes 1/1024 of the table.
  uint32_t* ht = L.v;                                   // [2 CAP]: L.v and L.h (values are in registers)
  uint8_t* df = reinterpret_cast<uint8_t*>(&L.wcnt[0][0]);  // [CAP] duplicated-key flag per position
  static_assert(sizeof(L.wcnt) >= B::CAP, "dup flags fit the multisplit rows");
  constexpr uint32_t HT = 2 * B::CAP, HT_SHIFT = 32 - 12;
  static_assert(HT == 1u << 12, "hash index bits");
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    const uint32_t p = strip0 + i * 64 + lane;
    if (p < S) L.k[p] = kk[i];
  }
  for (uint32_t j = tid; j < HT; j += B::THREADS) ht[j] = 0xFFFFFFFFu;
  for (uint32_t j = tid; j < B::CAP / 4; j += B::THREADS) reinterpret_cast<uint32_t*>(df)[j] = 0u;
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    const uint32_t p = strip0 + i * 64 + lane;
    if (p >= S) continue;
    uint32_t h = (kk[i] * 0x9E3779B1u) >> HT_SHIFT;
    for (;;) {  // (S <= CAP = HT / 2: a free entry is always found)
      const uint32_t o = atomicCAS(&ht[h], 0xFFFFFFFFu, p);
      if (o == 0xFFFFFFFFu) break;  // first of its key in the bucket
      if (L.k[o] == kk[i]) {        // seen before: both are duplicated
        df[p] = 1;
        df[o] = 1;
        break;
      }
      h = (h + 1) & (HT - 1);
    }
  }
  __syncthreads();
  // compact the duplicated elements, keeping the bucket (= arrival) order,
  // and rank the keys seen once for the list
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t cidx[B::ITEMS], sidx[B::ITEMS], wc = 0, ws = 0, dmask = 0, smask = 0;
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    const uint32_t p = strip0 + i * 64 + lane;
    const bool dup = p < S && df[p], one = p < S && !df[p];
    const uint64_t bl = __ballot(dup), bs = __ballot(one);
    cidx[i] = wc + (uint32_t)__popcll(bl & lt);
    sidx[i] = ws + (uint32_t)__popcll(bs & lt);
    wc += (uint32_t)__popcll(bl);
    ws += (uint32_t)__popcll(bs);
    dmask |= dup ? 1u << i : 0u;
    smask |= one ? 1u << i : 0u;
  }
  if (lane == 0) {
    L.wsum[wave] = wc;
    L.lw[wave] = ws;
  }
  __syncthreads();
  uint32_t wpre = 0, M = 0, spre = 0;
#pragma unroll
  for (uint32_t w = 0; w < B::WAVES; w++) {
    wpre += w < wave ? L.wsum[w] : 0u;
    spre += w < wave ? L.lw[w] : 0u;
    M += L.wsum[w];
  }
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    if (!((dmask >> i) & 1u)) continue;
    const uint32_t c = wpre + cidx[i];
    L.k[c] = kk[i];
    L.v[c] = vv[i];
    L.h[c] = hh[i];
  }
  if (tid == 0) {
    if (M) L.base_pos = atomicAdd(sorted_n, M);
    L.ub = M < S ? atomicAdd(uniq_n, S - M) : 0u;
  }
  __syncthreads();
  const uint32_t ub = L.ub + spre;
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++)
    if ((smask >> i) & 1u) uniq[ub + sidx[i]] = make_uint2(vv[i], kk[i]);
  if (!M) return;  // (uniform) every key of the bucket is seen once
  const uint32_t base = L.base_pos;
  if (M <= 64) {
    // one wave: stable rank of (key, compact index) by comparisons
    if (wave == 0) {
      const bool v = lane < M;
      const uint32_t k = v ? L.k[lane] : 0xFFFFFFFFu, x = v ? L.v[lane] : 0u, y = v ? L.h[lane] : 0u;
      uint32_t r = 0;
      for (uint32_t j = 0; j < M; j++) {
        const uint32_t kj = __shfl(k, j, 64);
        r += (kj < k || (kj == k && j < lane)) ? 1u : 0u;
      }
      if (v) {
        L.k[r] = k;
        L.v[r] = x;
        L.h[r] = y;
      }
    }
    __syncthreads();
  } else {
#pragma unroll
    for (uint32_t i = 0; i < B::ITEMS; i++) {
      const uint32_t p = strip0 + i * 64 + lane;
      kk[i] = p < M ? L.k[p] : 0xFFFFFFFFu;
      vv[i] = p < M ? L.v[p] : 0u;
      hh[i] = p < M ? L.h[p] : 0u;
    }
    __syncthreads();
    lds_sort3(L, kk, vv, hh, M);
  }
  for (uint32_t p = tid; p < M; p += B::THREADS) {
    sk[base + p] = L.k[p];
    sv[base + p] = L.v[p];
  }
  BK_STAMP(d, 3);
  bucket_segment<B, true>(L, d, M, base, sk, sh, segsum, rid, run_start, run_end, num_runs, drun);
  BK_STAMP(d, 5);
}

// Large bucket dominated by a few keys (hot tenants): sample 64 positions;
// keys seen at least BK_HEAVY_MIN times are "heavy". Pass A compacts the light
// elements (arrival order) into LDS and counts each heavy key; the light ones
// are sorted in LDS; each heavy key's elements then form one block, placed
// between the light keys by key order, filled in arrival order by pass B.
// Returns false (nothing written) when no key is heavy or the light elements
// do not fit in LDS.
template <typename B>
__device__ inline bool bucket_peel(BucketLds<B>& L, uint32_t d, uint32_t S, uint32_t base, uint32_t ntiles,
                                   const uint4* __restrict__ pt,
                                   uint32_t* __restrict__ sk,
                                   uint32_t* __restrict__ sv, uint32_t* __restrict__ sh) {
  constexpr uint32_t IT = B::ITEMS;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt_mask = (1ull << lane) - 1;
  if (wave == 0) {
    uint32_t p[1] = {(uint32_t)(((uint64_t)(2 * lane + 1) * S) >> 7)}, j[1];
    bucket_src(ntiles, p, j);
    const uint32_t ks = pt[j[0]].x;
    uint32_t cnt = 0;
    bool first = true;
    for (uint32_t q = 0; q < 64; q++) {
      const uint32_t kq = __shfl(ks, q, 64);
      cnt += kq == ks ? 1u : 0u;
      if (q < lane && kq == ks) first = false;
    }
    const bool cand = first && cnt >= BK_HEAVY_MIN;
    const uint64_t b = __ballot(cand);
    const uint32_t rank = __popcll(b & lt_mask);
    if (cand && rank < BK_HEAVY) L.heavy[rank] = ks;
    if (lane < BK_HEAVY) {
      L.hcnt[lane] = 0;
      L.hrun[lane] = 0;
    }
    if (lane == 0) {
      L.nheavy = min((uint32_t)__popcll(b), BK_HEAVY);
      L.nlight = 0;
    }
  }
  __syncthreads();
  const uint32_t r = L.nheavy;
  if (!r) return false;
  uint32_t hk[BK_HEAVY];
#pragma unroll
  for (uint32_t c = 0; c < BK_HEAVY; c++) hk[c] = __builtin_amdgcn_readfirstlane(c < r ? L.heavy[c] : 0u);
  uint32_t kk[IT], vv[IT], hh[IT], cls[IT];
  // ---- pass A: light elements -> L.k / L.v / L.h (arrival order), class counts
  for (uint32_t c0 = 0; c0 < S; c0 += B::CAP) {
    const uint32_t strip0 = c0 + wave * B::STRIP;
    uint32_t pp[IT], jj[IT];
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) pp[i] = min(strip0 + i * 64 + lane, S - 1);
    bucket_src(ntiles, pp, jj);
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint4 e = pt[jj[i]];
      kk[i] = e.x;
      vv[i] = e.y;
      hh[i] = e.z;
    }
    uint32_t wl = 0, lr[IT];
    uint32_t wc[BK_HEAVY];
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++) wc[c] = 0;
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const bool in = strip0 + i * 64 + lane < S;
      cls[i] = in ? r : 0xFFu;  // light: class r (<= BK_HEAVY); past the bucket: 0xFF
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++)
        if (in && c < r && kk[i] == hk[c]) cls[i] = c;
      const uint64_t bl = __ballot(cls[i] == r);
      lr[i] = wl + __popcll(bl & lt_mask);
      wl += __popcll(bl);
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) wc[c] += c < r ? __popcll(__ballot(cls[i] == c)) : 0u;
    }
    if (lane == 0) {
      L.lw[wave] = wl;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) L.hw[wave][c] = wc[c];
    }
    __syncthreads();
    uint32_t pre = L.nlight, tl = 0;
    for (uint32_t w = 0; w < B::WAVES; w++) {
      pre += w < wave ? L.lw[w] : 0u;
      tl += L.lw[w];
    }
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint32_t at = pre + lr[i];
      if (cls[i] == r && at < B::CAP) {
        L.k[at] = kk[i];
        L.v[at] = vv[i];
        L.h[at] = hh[i];
      }
    }
    __syncthreads();
    if (tid < BK_HEAVY) {
      uint32_t t = 0;
      for (uint32_t w = 0; w < B::WAVES; w++) t += L.hw[w][tid];
      L.hcnt[tid] += t;
    }
    if (tid == 0) L.nlight += tl;
    __syncthreads();
  }
  const uint32_t nl = L.nlight;
  if (nl > B::CAP) return false;
  BK_STAMP(d, 13);
  // ---- sort the light elements in LDS
  const uint32_t strip0 = wave * B::STRIP;
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) {
    const uint32_t p = strip0 + i * 64 + lane;
    kk[i] = p < nl ? L.k[p] : 0xFFFFFFFFu;
    vv[i] = p < nl ? L.v[p] : 0u;
    hh[i] = p < nl ? L.h[p] : 0u;
  }
  if (nl) lds_sort3(L, kk, vv, hh, nl);
  // ---- block starts: light keys below the heavy key + heavy blocks of smaller keys
  if (tid < r) {
    const uint32_t K = hk[tid];
    uint32_t lo = 0, hi = nl;  // first light index with key >= K
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (L.k[mid] < K) lo = mid + 1;
      else hi = mid;
    }
    uint32_t st = lo;
    for (uint32_t c = 0; c < r; c++) st += hk[c] < K ? L.hcnt[c] : 0u;
    L.hstart[tid] = st;
  }
#ifdef RL_BK_PROF
  __syncthreads();
  if (tid == 0) {
    uint32_t* g = g_bk_peel + d * 16;
    g[0] = r;
    g[1] = nl;
    for (uint32_t c = 0; c < BK_HEAVY; c++) {
      g[2 + c] = hk[c];
      g[6 + c] = L.hcnt[c];
      g[10 + c] = L.hstart[c];
    }
    g[14] = S;
  }
#endif
  // light elements to their final positions (shifted past smaller heavy blocks)
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) {
    const uint32_t p = strip0 + i * 64 + lane;
    if (p < nl) {
      uint32_t at = p;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) at += (c < r && hk[c] < kk[i]) ? L.hcnt[c] : 0u;
      sk[base + at] = kk[i];
      sv[base + at] = vv[i];
      sh[base + at] = hh[i];
    }
  }
  __syncthreads();
  BK_STAMP(d, 14);
  // ---- pass B: heavy elements, in arrival order within each block
  for (uint32_t c0 = 0; c0 < S; c0 += B::CAP) {
    const uint32_t s0 = c0 + wave * B::STRIP;
    uint32_t pp[IT], jj[IT];
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) pp[i] = min(s0 + i * 64 + lane, S - 1);
    bucket_src(ntiles, pp, jj);
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint4 e = pt[jj[i]];
      kk[i] = e.x;
      vv[i] = e.y;
      hh[i] = e.z;
    }
    uint32_t hr[IT], wc[BK_HEAVY];
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++) wc[c] = 0;
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const bool in = s0 + i * 64 + lane < S;
      cls[i] = BK_HEAVY;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++)
        if (in && c < r && kk[i] == hk[c]) cls[i] = c;
      hr[i] = 0;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) {
        if (c >= r) continue;
        const uint64_t b = __ballot(cls[i] == c);
        if (cls[i] == c) hr[i] = wc[c] + __popcll(b & lt_mask);
        wc[c] += __popcll(b);
      }
    }
    if (lane == 0) {
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) L.hw[wave][c] = wc[c];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint32_t c = cls[i];
      if (c < BK_HEAVY) {
        uint32_t at = L.hstart[c] + L.hrun[c] + hr[i];
        for (uint32_t w = 0; w < wave; w++) at += L.hw[w][c];
        sk[base + at] = kk[i];
        sv[base + at] = vv[i];
        sh[base + at] = hh[i];
      }
    }
    __syncthreads();
    if (tid < r) {
      uint32_t t = 0;
      for (uint32_t w = 0; w < B::WAVES; w++) t += L.hw[w][tid];
      L.hrun[tid] += t;
    }
    __syncthreads();
  }
  __threadfence_block();
  __syncthreads();
  BK_STAMP(d, 15);
  return true;
}

// Large bucket without (enough) hot keys: the three stable passes chunk by
// chunk through HBM (tile layout -> sk -> temp -> sk; temp = this bucket's rid
// / segsum / ht ranges, which the segmentation overwrites or ignores
// afterwards). Running digit offsets per pass come from one histogram sweep.
template <typename B>
__device__ inline void bucket_lsd(BucketLds<B>& L, uint32_t S, uint32_t base, uint32_t ntiles,
                                  const uint4* __restrict__ pt,
                                  uint32_t* __restrict__ sk,
                                  uint32_t* __restrict__ sv, uint32_t* __restrict__ sh, uint32_t* __restrict__ ht,
                                  uint32_t* __restrict__ segsum, uint32_t* __restrict__ rid) {
  constexpr uint32_t IT = B::ITEMS;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t kk[IT], vv[IT], hh[IT], pos[IT];
  for (uint32_t j = tid; j < 3 * 256; j += B::THREADS) (&L.roff[0][0])[j] = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < S; c0 += B::CAP) {
    uint32_t pp[IT], jj[IT];
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) pp[i] = min(c0 + i * B::THREADS + tid, S - 1);
    bucket_src(ntiles, pp, jj);
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) kk[i] = pt[jj[i]].x;  // loads first, all in flight
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      if (c0 + i * B::THREADS + tid < S) {
        atomicAdd(&L.roff[0][kk[i] & 255u], 1u);
        atomicAdd(&L.roff[1][(kk[i] >> 8) & 255u], 1u);
        atomicAdd(&L.roff[2][(kk[i] >> 16) & 63u], 1u);
      }
    }
  }
  __syncthreads();
  for (uint32_t pass = 0; pass < 3; pass++) {
    const uint32_t v = tid < 256 ? L.roff[pass][tid] : 0u;
    const uint32_t excl = scan256(v, L.wsum, nullptr);
    if (tid < 256) L.roff[pass][tid] = excl;
  }
  __syncthreads();
  for (uint32_t pass = 0; pass < 3; pass++) {
    const uint32_t* ik = pass == 1 ? sk + base : rid + base;  // passes 1, 2 (pass 0 reads the tile layout)
    const uint32_t* iv = pass == 1 ? sv + base : segsum + base;
    const uint32_t* ih = pass == 1 ? sh + base : ht + base;
    uint32_t* ok = pass == 1 ? rid + base : sk + base;
    uint32_t* ov = pass == 1 ? segsum + base : sv + base;
    uint32_t* oh = pass == 1 ? ht + base : sh + base;
    for (uint32_t c0 = 0; c0 < S; c0 += B::CAP) {
      const uint32_t strip0 = c0 + wave * B::STRIP;
      uint32_t pp[IT], jj[IT];
#pragma unroll
      for (uint32_t i = 0; i < IT; i++) pp[i] = min(strip0 + i * 64 + lane, S - 1);
      if (pass == 0) {
        bucket_src(ntiles, pp, jj);
      } else {
#pragma unroll
        for (uint32_t i = 0; i < IT; i++) jj[i] = pp[i];
      }
      if (pass == 0) {
#pragma unroll
        for (uint32_t i = 0; i < IT; i++) {
          const uint4 e = pt[jj[i]];
          kk[i] = e.x;
          vv[i] = e.y;
          hh[i] = e.z;
        }
      } else {
#pragma unroll
        for (uint32_t i = 0; i < IT; i++) {
          kk[i] = ik[jj[i]];
          vv[i] = iv[jj[i]];
          hh[i] = ih[jj[i]];
        }
      }
#pragma unroll
      for (uint32_t i = 0; i < IT; i++)
        if (strip0 + i * 64 + lane >= S) kk[i] = 0xFFFFFFFFu;
      if (tid < 256) L.base[tid] = L.roff[pass][tid];
      if (pass < 2) bucket_rank<B, 8>(L, kk, strip0, S, 8 * pass, false, pos);
      else bucket_rank<B, 6>(L, kk, strip0, S, 16, false, pos);
      if (tid < 256) L.roff[pass][tid] += L.dtot[tid];
#pragma unroll
      for (uint32_t i = 0; i < IT; i++) {
        if (strip0 + i * 64 + lane < S) {
          ok[pos[i]] = kk[i];
          ov[pos[i]] = vv[i];
          oh[pos[i]] = hh[i];
        }
      }
    }
    __threadfence_block();
    __syncthreads();
  }
}

// ---- Large buckets, chunk-parallel. k_bucket samples a queued bucket's hot
// keys, allocates their run ids and one work item per BIG_CHUNK positions.
// k_big_count classifies every chunk (light / hot key c) and counts;
// k_big_place writes each hot key's elements straight to its block (after the
// bucket's light part, in arrival order: positions, in-run hit sums, run id)
// and compacts the light elements, in arrival order, into the front of the
// bucket; k_bucket_big then sorts and segments the light part in LDS (or, for
// a bucket without hot keys or with too many light elements, runs the whole
// single-workgroup path).
__device__ inline uint32_t wave_sum32(uint32_t x) {
#pragma unroll
  for (uint32_t m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
  return x;
}

// Inclusive sum over the wave's lanes (all 64 active) by DPP: row_shr 1, 2, 4,
// 8 inside each row of 16, then row_bcast 15 / 31 carry each row's total into
// the rows above. Twelve VALU operations; __shfl_up's six levels are six
// ds_bpermute round trips through the LDS crossbar plus their address math.
#ifndef RL_DPP_SCAN
#define RL_DPP_SCAN 1
#endif
__device__ __attribute__((always_inline)) inline uint32_t wave_incl_add(uint32_t x) {
#if RL_DPP_SCAN
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
#else
  const uint32_t lane = __lane_id();
#pragma unroll
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
#endif
  return x;
}

// Load one chunk of a queued bucket (BkSmall shape) and classify it: cls =
// hot key index c < r, r for a light element, 0xFF past the bucket.
__device__ inline void big_chunk_load(const BigMeta& M, uint32_t j, uint32_t ntiles, const uint4* __restrict__ pt,
                                      uint32_t (&kk)[BkSmall::ITEMS], uint32_t (&vv)[BkSmall::ITEMS],
                                      uint32_t (&hh)[BkSmall::ITEMS], uint32_t (&cls)[BkSmall::ITEMS], bool values) {
  using B = BkSmall;
  const uint32_t lane = threadIdx.x & 63, s0 = j * BIG_CHUNK + (threadIdx.x >> 6) * B::STRIP;
  uint32_t pp[B::ITEMS], jj[B::ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) pp[i] = min(s0 + i * 64 + lane, M.S - 1);
  bucket_src(ntiles, pp, jj);
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    const uint4 e = pt[jj[i]];
    kk[i] = e.x;
    hh[i] = e.z;
    vv[i] = values ? e.y : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < B::ITEMS; i++) {
    cls[i] = s0 + i * 64 + lane < M.S ? M.r : 0xFFu;
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++)
      if (cls[i] != 0xFFu && c < M.r && kk[i] == M.heavy[c]) cls[i] = c;
  }
}

__global__ __launch_bounds__(BkSmall::THREADS) void k_big_count(const uint4* __restrict__ pt,
                                                                const uint32_t* __restrict__ info, uint32_t ntiles,
                                                                const BigMeta* __restrict__ meta,
                                                                const uint32_t* __restrict__ work,
                                                                const uint32_t* work_n, uint32_t* __restrict__ cnt,
                                                                const uint32_t* err) {
  using B = BkSmall;
  __shared__ BucketLds<B> L;
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = *work_n;
  for (uint32_t it = blockIdx.x; it < nw; it += gridDim.x) {
    const uint32_t w = work[it];
    const BigMeta M = meta[w >> 16];
    bucket_setup(L, info, ntiles, M.d);
    uint32_t kk[B::ITEMS], vv[B::ITEMS], hh[B::ITEMS], cls[B::ITEMS];
    big_chunk_load(M, w & 0xFFFFu, ntiles, pt, kk, vv, hh, cls, false);
    uint32_t nl = 0, nc[BK_HEAVY], hs[BK_HEAVY];
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++) nc[c] = hs[c] = 0;
#pragma unroll
    for (uint32_t i = 0; i < B::ITEMS; i++) {
      const uint32_t hv = hh[i] > 1 ? hh[i] : 1u;
      nl += cls[i] == M.r ? 1u : 0u;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) {
        nc[c] += cls[i] == c ? 1u : 0u;
        hs[c] += cls[i] == c ? hv : 0u;
      }
    }
    nl = wave_sum32(nl);
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++) {
      nc[c] = wave_sum32(nc[c]);
      hs[c] = wave_sum32(hs[c]);
    }
    if (lane == 0) {
      L.lw[wave] = nl;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) {
        L.hw[wave][c] = nc[c];
        L.hsw[wave][c] = hs[c];
      }
    }
    __syncthreads();
    if (tid < BIG_CNT) {
      uint32_t t = 0;
      for (uint32_t v = 0; v < B::WAVES; v++)
        t += tid == 0 ? L.lw[v] : tid <= BK_HEAVY ? L.hw[v][tid - 1] : L.hsw[v][tid - 1 - BK_HEAVY];
      cnt[(size_t)it * BIG_CNT + tid] = t;
    }
    __syncthreads();  // L is reused by the next item
  }
}

__global__ __launch_bounds__(BkSmall::THREADS) void k_big_place(
    const uint4* __restrict__ pt,
    const uint32_t* __restrict__ info, uint32_t ntiles, const BigMeta* __restrict__ meta,
    const uint32_t* __restrict__ work, const uint32_t* work_n, const uint32_t* __restrict__ cnt,
    uint32_t* __restrict__ sk, uint32_t* __restrict__ sv, uint32_t* __restrict__ sh, uint32_t* __restrict__ segsum,
    uint32_t* __restrict__ rid, uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_end,
    uint32_t* __restrict__ drun, const uint32_t* err) {
  using B = BkSmall;
  __shared__ BucketLds<B> L;
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = *work_n;
  const uint64_t lt_mask = (1ull << lane) - 1;
  for (uint32_t it = blockIdx.x; it < nw; it += gridDim.x) {
    const uint32_t w = work[it], j = w & 0xFFFFu;
    const BigMeta M = meta[w >> 16];
    // sums over the bucket's earlier chunks (prefix) and all chunks (totals)
    if (tid < BIG_CNT) L.acc[tid] = 0;
    uint32_t tot[BIG_CNT];
#pragma unroll
    for (uint32_t k = 0; k < BIG_CNT; k++) tot[k] = 0;
    __syncthreads();
    for (uint32_t t = tid; t < M.nchunks; t += B::THREADS) {
      const uint32_t* ct = cnt + (size_t)(M.item0 + t) * BIG_CNT;
#pragma unroll
      for (uint32_t k = 0; k < BIG_CNT; k++) {
        const uint32_t v = ct[k];
        tot[k] += v;
        if (t < j) atomicAdd(&L.acc[k], v);
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < 1 + BK_HEAVY; k++) tot[k] = block_sum(L, tot[k]);  // light and class totals
    bucket_setup(L, info, ntiles, M.d);  // (barriers: L.acc complete)
    const uint32_t NL = tot[0];
    if (NL > BIG_LIGHT_CAP) continue;  // k_bucket_big runs the whole bucket
    uint32_t hstart[BK_HEAVY];  // hot key blocks after the light part, in class order
    uint32_t st = NL;
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++) {
      hstart[c] = st;
      st += c < M.r ? tot[1 + c] : 0u;
    }
    if (j == 0 && tid < M.r) {
      run_start[M.rb_heavy + tid] = M.base + hstart[tid];
      run_end[M.rb_heavy + tid] = M.base + hstart[tid] + tot[1 + tid];
      drun[M.db_heavy + tid] = M.rb_heavy + tid;
    }
    uint32_t kk[B::ITEMS], vv[B::ITEMS], hh[B::ITEMS], cls[B::ITEMS];
    big_chunk_load(M, j, ntiles, pt, kk, vv, hh, cls, true);
    // ranks in the chunk (item-major within the wave strip = arrival order):
    // light rank, and per hot key: rank and inclusive sum of max(1, hits)
    uint32_t rk[B::ITEMS], hp[B::ITEMS], wl = 0, wc[BK_HEAVY], wh[BK_HEAVY];
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++) wc[c] = wh[c] = 0;
#pragma unroll
    for (uint32_t i = 0; i < B::ITEMS; i++) {
      const uint64_t bl = __ballot(cls[i] == M.r);
      rk[i] = wl + __popcll(bl & lt_mask);
      wl += __popcll(bl);
      hp[i] = 0;
      const uint32_t hv = hh[i] > 1 ? hh[i] : 1u;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) {
        if (c >= M.r) continue;  // uniform
        const bool mine = cls[i] == c;
        const uint64_t b = __ballot(mine);
        const uint32_t x = wave_incl_add(mine ? hv : 0u);  // inclusive scan of the class's hits over the lanes
        if (mine) {
          rk[i] = wc[c] + __popcll(b & lt_mask);
          hp[i] = wh[c] + x;
        }
        wc[c] += __popcll(b);
        wh[c] += (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
      }
    }
    if (lane == 0) {
      L.lw[wave] = wl;
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) {
        L.hw[wave][c] = wc[c];
        L.hsw[wave][c] = wh[c];
      }
    }
    __syncthreads();
    uint32_t lpre = L.acc[0], cpre[BK_HEAVY], hpre[BK_HEAVY];
#pragma unroll
    for (uint32_t c = 0; c < BK_HEAVY; c++) {
      cpre[c] = L.acc[1 + c];
      hpre[c] = L.acc[1 + BK_HEAVY + c];
    }
    for (uint32_t v = 0; v < wave; v++) {
      lpre += L.lw[v];
#pragma unroll
      for (uint32_t c = 0; c < BK_HEAVY; c++) {
        cpre[c] += L.hw[v][c];
        hpre[c] += L.hsw[v][c];
      }
    }
#pragma unroll
    for (uint32_t i = 0; i < B::ITEMS; i++) {
      const uint32_t c = cls[i];
      if (c == M.r) {  // light: compacted in arrival order into [0, NL)
        const uint32_t at = M.base + lpre + rk[i];
        sk[at] = kk[i];
        sv[at] = vv[i];
        sh[at] = hh[i];
      } else if (c < BK_HEAVY) {  // hot key c: final position, run sums, run id
        uint32_t cp = 0, hq = 0, hs0 = 0;
#pragma unroll
        for (uint32_t q = 0; q < BK_HEAVY; q++)
          if (q == c) {
            cp = cpre[q];
            hq = hpre[q];
            hs0 = hstart[q];
          }
        const uint32_t at = M.base + hs0 + cp + rk[i];
        sk[at] = kk[i];
        sv[at] = vv[i];
        segsum[at] = hq + hp[i];
        rid[at] = M.rb_heavy + c;
      }
    }
    __syncthreads();  // L is reused by the next item
  }
}

__global__ __launch_bounds__(BkBig::THREADS) void k_bucket_big(
    const uint4* __restrict__ pt,
    const uint32_t* __restrict__ info, uint32_t ntiles, uint32_t* __restrict__ sk, uint32_t* __restrict__ sv,
    uint32_t* __restrict__ sh, uint32_t* __restrict__ ht, uint32_t* __restrict__ segsum, uint32_t* __restrict__ rid,
    uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_end, unsigned long long* num_runs,
    uint32_t* __restrict__ drun, const BigMeta* __restrict__ meta, const uint32_t* big_n,
    const uint32_t* __restrict__ cnt, const uint32_t* err) {
  using B = BkBig;
  __shared__ BucketLds<B> L;
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nb = *big_n;
  for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const BigMeta M = meta[bi];
    const uint32_t d = M.d, S = M.S, base = M.base;
    BK_STAMP(d, 0);
    uint32_t nl = 0;
    for (uint32_t t = tid; t < M.nchunks; t += B::THREADS) nl += cnt[(size_t)(M.item0 + t) * BIG_CNT];
    nl = block_sum(L, nl);
    if (M.r && nl <= BIG_LIGHT_CAP) {
      // hot keys placed by k_big_place; the light part [0, nl), compacted in
      // arrival order, is sorted and segmented here
      uint32_t kk[B::ITEMS], vv[B::ITEMS], hh[B::ITEMS];
      const uint32_t strip0 = wave * B::STRIP;
#pragma unroll
      for (uint32_t i = 0; i < B::ITEMS; i++) {
        const uint32_t p = min(strip0 + i * 64 + lane, nl ? nl - 1 : 0u);
        kk[i] = sk[base + p];
        vv[i] = sv[base + p];
        hh[i] = sh[base + p];
      }
#pragma unroll
      for (uint32_t i = 0; i < B::ITEMS; i++)
        if (strip0 + i * 64 + lane >= nl) kk[i] = 0xFFFFFFFFu;
      if (nl) {
        lds_sort3(L, kk, vv, hh, nl);
#pragma unroll
        for (uint32_t i = 0; i < B::ITEMS; i++) {
          const uint32_t p = strip0 + i * 64 + lane;
          if (p < nl) {
            sk[base + p] = kk[i];
            sv[base + p] = vv[i];
          }
        }
        __syncthreads();
        bucket_segment<B, true>(L, d, nl, base, sk, sh, segsum, rid, run_start, run_end, num_runs, drun);
      }
    } else {
      if (tid < M.r) run_start[M.rb_heavy + tid] = run_end[M.rb_heavy + tid] = 0;  // hot-key runs left empty
      bucket_setup(L, info, ntiles, d);
      BK_STAMP(d, 1);
      if (!bucket_peel(L, d, S, base, ntiles, pt, sk, sv, sh))
        bucket_lsd(L, S, base, ntiles, pt, sk, sv, sh, ht, segsum, rid);
      bucket_segment<B, false>(L, d, S, base, sk, sh, segsum, rid, run_start, run_end, num_runs, drun);
    }
    BK_STAMP(d, 7);
    __syncthreads();  // L is reused by the next bucket
  }
}

// Run checks against the predecessor (equality chains): a run must hold one
// stem under one unit, else it is flagged RUN_MULTI and queued once (by run
// id) for k_runs_general; a window change within a run makes a long run
// RUN_SLOW (serial replay). Run heads only compare two sort keys.
// ---------------------------------------------------------------------------
// Sparse work, densely. Where only some positions of a range need the random
// table / record accesses (the runs of two or more at C1, the keys seen once at
// C2), spreading them one per lane over the whole grid makes nearly every wave
// pay a full chain of dependent random loads for one or two active lanes. A
// block instead scans a range of positions with coalesced reads, compacts the
// active ones into LDS (any order: the items are independent) and works
// through them with all its lanes.
// ---------------------------------------------------------------------------
// k_run_check's positions per block: the sorted order holds only the runs
// (dedup-first buckets), about half of them non-heads, so a block of 256
// positions gives each lane about one chain of random reads (1024-position
// blocks left ~50 busy workgroups at C1, each lane walking several chains:
// 22 us isolated for ~53k positions).
#ifndef RL_RC_CHUNK
#define RL_RC_CHUNK 256
#endif
constexpr uint32_t RC_CHUNK = RL_RC_CHUNK;

template <typename Pred>
__device__ __attribute__((always_inline)) inline uint32_t block_compact(uint32_t lo, uint32_t hi, uint32_t* list,
                                                                        uint32_t* count, Pred pred) {
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x == 0) *count = 0;
  __syncthreads();
  for (uint32_t i0 = lo; i0 < hi; i0 += blockDim.x) {
    const uint32_t i = i0 + threadIdx.x;
    const bool take = i < hi && pred(i);
    const uint64_t m = __ballot(take);
    uint32_t base = 0;
    if (lane == 0 && m) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, 0);
    if (take) list[base + __popcll(m & ((1ull << lane) - 1))] = i;
  }
  __syncthreads();
  return *count;
}

// k_run_check's per-position word for split_long_body (grp): unit << 8 | low
// byte (0 = the head's stem, family 0; SPLIT_POS_OTHER = another stem;
// SPLIT_POS_SKIP = a failed descriptor) | bit 16: `now` differs from the head's
constexpr uint32_t SPLIT_POS_OTHER = 0xFFu, SPLIT_POS_SKIP = 0xFEu, SPLIT_POS_NOWVAR = 1u << 16;
constexpr uint32_t SPLIT_ULIST = 1024;  // split_long_body: other stems' positions listed in LDS

// k_run_check marks every descriptor whose sort key occurs twice or more in the
// batch (BatchDev::dup, one byte store per descriptor: the thread of
// sorted position q marks q, and the run's head when q is its second element).
// k_table answers the unmarked ones in arrival order and the runs in sorted
// order. A run must hold one stem under one unit and one window: every
// non-head element is compared with the run's HEAD (equivalent to comparing
// neighbours, and the head's record and stem are shared by the whole run, so
// they stay in cache: one random record and stem read per element instead of
// two, which matters for the hot keys' long runs).
__global__ __launch_bounds__(256) void k_run_check(BatchDev b, SRec rec_s,
                                                   const uint32_t* __restrict__ skeys,
                                                   const uint32_t* __restrict__ rid,
                                                   const uint32_t* __restrict__ run_start,
                                                   uint32_t* __restrict__ run_end,
                                                   uint32_t* __restrict__ run_flags, uint32_t* __restrict__ defer,
                                                   uint32_t* defer_n, const uint32_t* err,
                                                   const unsigned long long* num_runs, unsigned long long* split,
                                                   const uint32_t* sorted_n, uint32_t* __restrict__ pos_unit,
                                                   uint32_t* __restrict__ pos_hits, uint2* __restrict__ uniq,
                                                   uint32_t* uniq_n, uint32_t* long_runs, uint32_t* __restrict__ keys0) {
  __shared__ uint32_t s_list[RC_CHUNK], s_cnt;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // k_split's reservations start from the bucket kernels' count
    split[0] = 0;
    split[1] = *num_runs;
    long_runs[0] = 0;
  }
  if (*err) return;
  const uint32_t sn = *sorted_n;
  // a run of one (a large bucket sorts every element, light keys included) is
  // a key seen once: onto the list of k_table's singleton part
  for (uint32_t q0 = blockIdx.x * RC_CHUNK; q0 < min(blockIdx.x * RC_CHUNK + RC_CHUNK, sn); q0 += blockDim.x) {
    const uint32_t q = q0 + threadIdx.x;
    const uint32_t k = q < sn ? skeys[q] : 0u;
    const bool one = q < sn && (q == 0 || skeys[q - 1] != k) && (q + 1 >= sn || skeys[q + 1] != k);
    const uint64_t m = __ballot(one);
    if (!m) continue;  // (wave-uniform)
    const uint32_t lane = threadIdx.x & 63, leader = (uint32_t)__ffsll((unsigned long long)m) - 1;
    uint32_t at = 0;
    if (lane == leader) at = atomicAdd(uniq_n, (uint32_t)__popcll(m));
    at = __shfl(at, leader, 64) + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    if (one) uniq[at] = make_uint2(rec_s.sv[q], k);
  }
  const uint32_t lo = max(blockIdx.x * RC_CHUNK, 1u), hi = min(blockIdx.x * RC_CHUNK + RC_CHUNK, sn);
  if (lo >= hi) return;
  // non-head positions (the second and later descriptors of a run)
  const uint32_t cnt = block_compact(lo, hi, s_list, &s_cnt, [&](uint32_t q) { return skeys[q - 1] == skeys[q]; });
  refine_totals(b);
  Rec* rec = const_cast<Rec*>(rec_s.rec);
#pragma unroll 1
  for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) {
    const uint32_t q = s_list[j];
    const uint32_t r = rid[q];
    const uint32_t p = run_start[r];
    const uint32_t eq = rec_s.sv[q], ep = rec_s.sv[p];
    const Rec x = rec[eq], y = rec[ep];
    // a failed descriptor (FLAG_SKIP) makes its run exact-path: general_body leaves it out
    const bool skip = (rec_flags(x) | rec_flags(y)) & FLAG_SKIP;
    const bool same_stem = !skip && x.hlo == y.hlo && (x.lu & 0xFFFFu) == (y.lu & 0xFFFFu) &&  // hash, length
                           key_equal(key_of(b, x), key_of(b, y));
    if (!same_stem && !skip && q == p + 1 && run_end[r] == q + 1) {
      // two unrelated stems sharing the 32-bit sort key (~100 runs per 1M
      // batch at C1): each is a key seen once in the batch. Neither gets
      // a dup mark (k_table's singleton part answers both) and the run is
      // emptied (its sorted path skips it); no k_split pass.
      run_end[r] = p;
      const uint32_t at = atomicAdd(uniq_n, 2u);
      uniq[at] = make_uint2(ep, skeys[q]);
      uniq[at + 1] = make_uint2(eq, skeys[q]);
      continue;
    }
    keys0[eq] = KEY_DUP;  // (the arrival-order key, not the record: KEY_DUP)
    if (q == p + 1) keys0[ep] = KEY_DUP;  // the run's head
    const bool same = same_stem && rec_unit(x) == rec_unit(y);
    // per position, for k_split's long runs (coalesced there instead of a
    // random record read per element): the unit and max(1, hits), and how the
    // element compares with the head (SPLIT_POS_*: family 0 = the head's stem
    // is known without another pass over the run's records and stems)
    pos_unit[q] = (rec_unit(x) << 8) | (skip ? SPLIT_POS_SKIP : !same_stem ? SPLIT_POS_OTHER : 0u) |
                  (x.now != y.now ? SPLIT_POS_NOWVAR : 0u);
    pos_hits[q] = x.hits > 1 ? x.hits : 1u;
    uint32_t f = 0;
    if (!same)  // (+ the units seen, for k_split; a failed descriptor's unit may be out of range)
      f = RUN_MULTI | (same_stem ? RUN_UNITS | ((1u << (rec_unit(x) - 1)) << RUN_UMASK_SHIFT) : RUN_STEMS);
    if (x.now != y.now) {
      const uint32_t d = div_of(rec_unit(x));
      f |= (same && x.now / d != y.now / d) ? RUN_SLOW | RUN_NOWVAR : RUN_NOWVAR;
    }
    // a hot run fills whole waves with the same verdict: one lane per (wave,
    // run) reads the word and ORs in what its wave found, so a run of tens of
    // thousands does not serialise on one word (nor on one L2 line)
    uint64_t pend = __ballot(f != 0);
    while (pend) {  // (wave-uniform)
      const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)pend) - 1);
      const uint32_t rr = __shfl(r, leader, 64);
      const bool mine = f != 0 && r == rr;
      const uint64_t mm = __ballot(mine);
      constexpr uint32_t kBits[] = {RUN_MULTI, RUN_UNITS, RUN_STEMS, RUN_SLOW, RUN_NOWVAR,
                                    1u << RUN_UMASK_SHIFT, 2u << RUN_UMASK_SHIFT, 4u << RUN_UMASK_SHIFT,
                                    8u << RUN_UMASK_SHIFT};
      uint32_t fo = 0;
#pragma unroll
      for (uint32_t bi = 0; bi < sizeof(kBits) / sizeof(kBits[0]); bi++)
        if (__ballot(mine && (f & kBits[bi]))) fo |= kBits[bi];
      if ((threadIdx.x & 63u) == leader &&
          (__hip_atomic_load(&run_flags[rr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & fo) != fo) {
        const uint32_t old = atomicOr(&run_flags[rr], fo);
        if ((fo & RUN_MULTI) && !(old & RUN_MULTI)) defer[atomicAdd(defer_n, 1u)] = rr;
      }
      pend &= ~mm;
    }
  }
}

// ---- k_split: hash-prefix collisions and multi-unit stems. A run is defined
// by the 32-bit sort key; k_run_check flags it RUN_MULTI when its elements do
// not all share the head's stem and unit. Its distinct stems ("families") are
// found by the full bytes; each becomes one or more groups:
//  * a stem under one unit is one group (the usual case: unrelated keys whose
//    hashes agree in 32 bits, ~100 runs per 1M batch at C1);
//  * a stem under several units (per-request overrides, config_impl.go:254-265)
//    is one group per Redis key: the key is stem ‖ windowStart
//    (cache_key.go:73-74), so two units whose windows coincide (SECOND and
//    MINUTE at t % 60 == 0) share a counter and form one group in arrival
//    order, and units whose windows differ are independent keys.
// The run is reordered stably into consecutive sub-runs, one per group, with
// their own run ids, in-run sums and flags, and k_table answers them like any
// other run (a lone group of one element becomes a key seen once) instead of
// the one-lane exact path, whose chain of dependent table accesses outlasted
// k_table. A multi-unit stem's groups carry RUN_ALIAS (its first one
// RUN_AHEAD and the group count): k_table's lane for the head sets all of them
// up at once (alias_setup). Anything else stays on the exact path: a 64-bit
// hash collision, a failed descriptor, more than SPLIT_MAXG groups, a
// multi-unit stem whose descriptors do not share one `now`, one window of a
// stem in both stores of the per-second split (their local-cache entry is
// shared), or no room left in the dup-run list. Runs over SPLIT_CAP elements
// take split_long_body (global-memory scratch instead of LDS).
#ifndef RL_SPLIT_BLOCKS
#define RL_SPLIT_BLOCKS 128  // k_split's workgroups (a grid-stride loop over the deferred runs)
#endif
constexpr uint32_t SPLIT_CAP = 1024, SPLIT_MAXG = 8, SPLIT_BLOCKS = RL_SPLIT_BLOCKS;
constexpr uint32_t DEFER_DONE = 0xFFFFFFFFu;  // a deferral k_split resolved
constexpr uint32_t SPLIT_BAD = 0xFFu;

// Families -> groups (one thread). fmask: units seen per family (bit u-1);
// fnow / fnv: the family leader's `now` / whether another one was seen.
struct SplitPlan {
  uint8_t ug[SPLIT_MAXG][4];  // group of (family, unit - 1)
  uint8_t head[SPLIT_MAXG];   // family -> its first group
  uint8_t ng[SPLIT_MAXG];     // family -> its group count
  uint8_t fam[SPLIT_MAXG];    // group -> family
  uint8_t alias[SPLIT_MAXG];  // group of a multi-unit family
  uint8_t gmask[SPLIT_MAXG];  // group -> its units
  uint32_t G, any_alias;
};

__device__ inline uint32_t split_plan(SplitPlan& S, uint32_t NF, const uint32_t* fmask, const uint32_t* fnow,
                                      const uint32_t* fnv, int per_second) {
  uint32_t G = 0;
  S.any_alias = 0;
  for (uint32_t f = 0; f < NF; f++) {
    const uint32_t m = fmask[f];
    S.head[f] = (uint8_t)G;
    if (__popc(m) == 1) {
      if (G >= SPLIT_MAXG) return SPLIT_BAD;
      for (uint32_t u = 0; u < 4; u++) S.ug[f][u] = (uint8_t)G;
      S.fam[G] = (uint8_t)f;
      S.alias[G] = 0;
      S.gmask[G] = (uint8_t)m;
      S.ng[f] = 1;
      G++;
      continue;
    }
    if (fnv[f]) return SPLIT_BAD;  // one window per unit needs one `now`
    const uint32_t now = fnow[f], first = G;
    uint32_t w[4];
    for (uint32_t u = 0; u < 4; u++) {
      S.ug[f][u] = SPLIT_BAD;
      if (!((m >> u) & 1)) continue;
      w[u] = now - now % div_of(u + 1);
      const bool cls = per_second && u == 0;
      uint32_t g = SPLIT_BAD;
      for (uint32_t v = 0; v < u; v++) {
        if (!((m >> v) & 1) || w[v] != w[u]) continue;
        if ((per_second && v == 0) != cls) return SPLIT_BAD;  // one window in both stores
        g = S.ug[f][v];
      }
      if (g == SPLIT_BAD) {
        if (G >= SPLIT_MAXG) return SPLIT_BAD;
        g = G++;
        S.fam[g] = (uint8_t)f;
        S.alias[g] = 1;
        S.gmask[g] = 0;
      }
      S.ug[f][u] = (uint8_t)g;
      S.gmask[g] |= (uint8_t)(1u << u);
    }
    S.ng[f] = (uint8_t)(G - first);
    S.any_alias = 1;
  }
  S.G = G;
  return G;
}

// run_flags of group g once split (s_fl: RUN_SLOW / RUN_NOWVAR of a one-unit group)
__device__ inline uint32_t split_group_flags(const SplitPlan& S, uint32_t g, uint32_t fl) {
  if (!S.alias[g]) return fl;
  const uint32_t f = S.fam[g];
  uint32_t x = RUN_ALIAS | ((uint32_t)S.gmask[g] << RUN_UMASK_SHIFT);
  if (S.head[f] == g) x |= RUN_AHEAD | ((uint32_t)S.ng[f] << RUN_G_SHIFT);
  return x;
}

// ---- split_long (k_split's blocks, for RUN_MULTI runs over SPLIT_CAP
// elements): the same reordering. Under an unlucky hash key a hot stem (tens
// of thousands of descriptors per batch at C2) shares its sort key with
// another stem, and the one-lane exact path replayed the whole run: 1.3 ms per
// batch on average at C2 under seed 5 (profiles/r02/seed_sweep/); a hot stem
// under two units (an override) is such a run in every batch. Split, each
// group is an ordinary long run for the parallel path. The per-element state
// lives in global scratch owned by the run's range: grp (family | unit << 8,
// then the group) and lead (the rank inside the group) are the exact path's
// per-position scratch, which it rewrites for any run it sees; segsum (the
// run's in-run sums) is touched only once the split is committed: it then
// holds the permutation's source until the new sums overwrite it. (A kernel
// of its own with 1024-lane blocks cost every batch 4-6 us of launch on the
// critical path, 1-3 %, profiles/r02/ab/long_*.)
constexpr uint32_t SPLIT_UNROLL = 8;
#ifndef RL_SPLIT_ST
#define RL_SPLIT_ST 16  // (8: C2U 3.33-3.42 G, 16: 3.52-3.53 G; 4: 2.2-3.2 G; 32 in round 4: C2 -2 %, C2U flat)
#endif
constexpr uint32_t SPLIT_ST = RL_SPLIT_ST;  // 64-element steps in flight per wave in split_long_body's walks
// k_split's workgroup (a long run is reordered by its waves, each walking a
// chunk of it: more waves, shorter walks, but slower short runs)
// k_split_long's workgroup (0: k_split's own workgroups walk the long runs)
// and its steps in flight per wave (<= 128 VGPRs at 1024 lanes)
#ifndef RL_SPLIT_LONG_THREADS
#define RL_SPLIT_LONG_THREADS 1024
#endif
#ifndef RL_SPLIT_LONG_ST
#define RL_SPLIT_LONG_ST 8
#endif
#ifndef RL_SPLIT_LONG_OCC
#define RL_SPLIT_LONG_OCC 4  // k_split_long's minimum waves per SIMD (8: <= 64 VGPRs)
#endif
#ifndef RL_SPLIT_LONG_BLOCKS
#define RL_SPLIT_LONG_BLOCKS 8
#endif
#ifndef RL_SPLIT_THREADS
#define RL_SPLIT_THREADS 256  // (1024: C2U's 58k-element runs 481 -> 377 us, but C1's k_split 18 -> 26 us;
                              //  512 in round 4: C2U +2.4 %, C2 -4 %, C1 -1.5 %)
#endif
constexpr uint32_t SPLIT_THREADS = RL_SPLIT_THREADS;

// The keys-seen-once list (Scratch::uniq) as k_split appends to it: a lone
// one-element group is a key seen once (rare: one atomic each).
struct UniqList {
  uint2* list;
  uint32_t* n;
  const uint32_t* skeys;  // sorted keys: a run shares its sort key
  uint32_t* keys0;        // arrival-order keys (KEY_DUP marks)
  // descriptor e (its run starts at sorted position p) is a key seen once
  // after all: its arrival-order key back, and onto k_table's list
  __device__ inline void single(uint32_t e, uint32_t p) const {
    const uint32_t k = skeys[p];
    keys0[e] = k;
    list[atomicAdd(n, 1u)] = make_uint2(e, k);
  }
};

template <uint32_t NT, uint32_t ST>
__device__ __attribute__((always_inline)) inline void split_long_body(uint32_t j, uint32_t r, uint32_t p, uint32_t L, BatchDev b,
                                                          SRec rec_s, uint32_t* svals, uint32_t* segsum,
                                                          uint32_t* __restrict__ rid, uint32_t* __restrict__ run_start,
                                                          uint32_t* __restrict__ run_end,
                                                          uint32_t* __restrict__ run_flags, uint32_t* __restrict__ defer,
                                                          unsigned long long* num_runs, unsigned long long* split,
                                                          uint32_t* __restrict__ drun, uint32_t drun_cap, uint32_t* grp,
                                                          uint32_t* rank, uint32_t* __restrict__ pos_hits,
                                                          uint32_t* __restrict__ hnew, int per_second, uint32_t rfl,
                                                          const UniqList& uq) {
  constexpr uint32_t NW = NT / 64;
  __shared__ uint32_t s_wc[NW][SPLIT_MAXG], s_wh[NW][SPLIT_MAXG], s_wp[NW][SPLIT_MAXG], s_ws[NW];
  __shared__ uint32_t s_cnt[SPLIT_MAXG], s_base[SPLIT_MAXG], s_id[SPLIT_MAXG], s_fl[SPLIT_MAXG], s_off[SPLIT_MAXG];
  __shared__ uint32_t s_lnow[SPLIT_MAXG], s_lunit[SPLIT_MAXG], s_fmask[SPLIT_MAXG], s_fnv[SPLIT_MAXG];
  __shared__ uint32_t s_bad, s_lead, s_nu, s_ul[SPLIT_ULIST];
  __shared__ SplitPlan s_plan;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  Rec* rec = const_cast<Rec*>(rec_s.rec);
  const uint32_t* sv = rec_s.sv;  // (= svals: unchanged until the scatter)
  {
#ifdef RL_SPLIT_PROF  // (measurement builds: phase stamps of long runs, printed by one lane)
    uint64_t ts[8];
    ts[0] = wall_clock64();
#define SPLIT_STAMP(i) ts[i] = wall_clock64()
#else
#define SPLIT_STAMP(i)
#endif
    __syncthreads();  // the previous run's shared state has been read
    if (tid == 0) {
      s_bad = 0;
      s_nu = 0;
    }
    if (tid < SPLIT_MAXG) {
      s_fmask[tid] = 0;
      s_fnv[tid] = 0;
    }
    __syncthreads();
    uint32_t NF = 0;
    // k_run_check left each non-head position's unit << 8 in grp and its
    // max(1, hits) in pos_hits; the head's are set here
    if (tid == 0) {
      const Rec y = rec[sv[p]];
      pos_hits[p] = y.hits > 1 ? y.hits : 1u;
      if ((rfl & (RUN_UNITS | RUN_STEMS)) == RUN_UNITS) {
        // one stem under several units (k_run_check compared every element
        // with the head, bytes included): one family, units known
        grp[p] = rec_unit(y) << 8;  // family 0
        s_lnow[0] = y.now;
        s_lunit[0] = rec_unit(y);
        s_fnv[0] = (rfl & RUN_NOWVAR) ? 1u : 0u;
        s_fmask[0] = ((rfl >> RUN_UMASK_SHIFT) & 0xFu) | (1u << (rec_unit(y) - 1));
      }
    }
    if ((rfl & (RUN_UNITS | RUN_STEMS)) == RUN_UNITS) {
      NF = 1;
    } else {
      // family 0, the head's stem: from k_run_check's comparison of every
      // element with the head (one coalesced pass; the records and stems of
      // a hot stem's tens of thousands of descriptors are not read again)
      // The other stems' positions (few: stems that share the hot stem's sort
      // key by chance) are listed in LDS, so the family passes below visit
      // only them (past SPLIT_ULIST of them: the whole run)
      uint32_t fm0 = 0, nv0 = 0;
      for (uint32_t k = tid + 1; k < L; k += NT) {
        const uint32_t v = grp[p + k], lo = v & 0xFFu;
        if (lo == SPLIT_POS_SKIP) {
          s_bad = 1;
        } else if (lo == 0) {
          fm0 |= 1u << (((v >> 8) & 0xFFu) - 1);
          nv0 |= (v & SPLIT_POS_NOWVAR) ? 1u : 0u;
        } else {
          const uint32_t j = atomicAdd(&s_nu, 1u);
          if (j < SPLIT_ULIST) s_ul[j] = k;
        }
      }
      if (tid == 0) {
        const Rec y = rec[sv[p]];
        if ((y.lu >> 24) & FLAG_SKIP) s_bad = 1;
        grp[p] = rec_unit(y) << 8;  // family 0
        s_lnow[0] = y.now;
        s_lunit[0] = rec_unit(y);
        fm0 |= 1u << (rec_unit(y) - 1);
      }
      if (fm0) atomicOr(&s_fmask[0], fm0);
      if (nv0) s_fnv[0] = 1;
      NF = 1;
      __syncthreads();
      const uint32_t nu = s_nu;
      // families, as in k_split: the first unassigned element leads, and every
      // element with its stem joins
      for (; nu <= SPLIT_ULIST;) {  // (the listed positions only)
        if (tid == 0) s_lead = 0xFFFFFFFFu;
        __syncthreads();
        for (uint32_t j = tid; j < nu; j += NT)
          if ((grp[p + s_ul[j]] & 0xFFu) == 0xFFu) atomicMin(&s_lead, s_ul[j]);
        __syncthreads();
        const uint32_t ld = s_lead;
        if (ld == 0xFFFFFFFFu || s_bad || NF == SPLIT_MAXG) break;  // (uniform)
        const Rec y = rec[sv[p + ld]];
        const Key ky = key_of(b, y);
        if (tid == 0) {
          s_lnow[NF] = y.now;
          s_lunit[NF] = rec_unit(y);
        }
        uint32_t fm = 0, nv = 0;
        for (uint32_t j = tid; j < nu; j += NT) {
          const uint32_t k = s_ul[j];
          if ((grp[p + k] & 0xFFu) != 0xFFu) continue;
          const Rec x = rec[sv[p + k]];
          if (x.hlo != y.hlo || (x.lu & 0xFFFFu) != (y.lu & 0xFFFFu)) continue;
          if (!key_equal(key_of(b, x), ky)) {
            s_bad = 1;  // equal 64-bit hash, different stem
          } else {
            grp[p + k] = NF | (rec_unit(x) << 8);
            fm |= 1u << (rec_unit(x) - 1);
            nv |= x.now != y.now;
          }
        }
        if (fm) atomicOr(&s_fmask[NF], fm);
        if (nv) s_fnv[NF] = 1;
        NF++;
        __syncthreads();
      }
      // (records read SPLIT_UNROLL at a time: the scan is a chain of random reads)
      for (; nu > SPLIT_ULIST;) {
        if (tid == 0) s_lead = 0xFFFFFFFFu;
        __syncthreads();
        for (uint32_t k = tid; k < L; k += NT)
          if ((grp[p + k] & 0xFFu) == 0xFFu) {
            atomicMin(&s_lead, k);  // this lane's first is its smallest
            break;
          }
        __syncthreads();
        const uint32_t ld = s_lead;
        if (ld == 0xFFFFFFFFu || s_bad || NF == SPLIT_MAXG) break;  // (uniform)
        const Rec y = rec[sv[p + ld]];
        const Key ky = key_of(b, y);
        if (tid == 0) {
          s_lnow[NF] = y.now;
          s_lunit[NF] = rec_unit(y);
        }
        uint32_t fm = 0, nv = 0;
        for (uint32_t k0 = tid; k0 < L; k0 += NT * SPLIT_UNROLL) {
          Rec x[SPLIT_UNROLL];
          bool act[SPLIT_UNROLL];
#pragma unroll
          for (uint32_t u = 0; u < SPLIT_UNROLL; u++) {
            const uint32_t k = k0 + u * NT;
            act[u] = k < L && (grp[p + k] & 0xFFu) == 0xFFu;
            if (act[u]) x[u] = rec[sv[p + k]];
          }
#pragma unroll
          for (uint32_t u = 0; u < SPLIT_UNROLL; u++) {
            if (!act[u] || x[u].hlo != y.hlo || (x[u].lu & 0xFFFFu) != (y.lu & 0xFFFFu)) continue;
            if (!key_equal(key_of(b, x[u]), ky)) {
              s_bad = 1;  // equal 64-bit hash, different stem
            } else {
              grp[p + k0 + u * NT] = NF | (rec_unit(x[u]) << 8);
              fm |= 1u << (rec_unit(x[u]) - 1);
              nv |= x[u].now != y.now;
            }
          }
        }
        if (fm) atomicOr(&s_fmask[NF], fm);
        if (nv) s_fnv[NF] = 1;
        NF++;
        __syncthreads();
      }
      if (tid == 0 && s_lead != 0xFFFFFFFFu) s_bad = 1;  // more than SPLIT_MAXG stems
    }
    __syncthreads();
    if (s_bad) return;  // (uniform) the exact path keeps it
    if (tid == 0 && split_plan(s_plan, NF, s_fmask, s_lnow, s_fnv, per_second) == SPLIT_BAD) s_bad = 1;
    __syncthreads();
    const uint32_t G = s_plan.G;
    if (s_bad || (G < 2 && !s_plan.any_alias)) return;  // (uniform) the exact path keeps it
    SPLIT_STAMP(1);
    // The reordering as wave walks (no block barrier inside a walk; ST steps
    // of 64 elements in flight per wave): wave w owns the positions
    // [w CH, (w+1) CH). Walk 1 counts each group's elements and sums its
    // max(1, hits) in the wave's chunk; the chunks' starting ranks and each
    // group's hits before it follow from the NW x G totals.
    const uint32_t CH = ((L + NT - 1) / NT) * 64;
    const uint32_t a0 = min(L, wv * CH), a1 = min(L, a0 + CH);
    {
      uint32_t cl[SPLIT_MAXG], hl[SPLIT_MAXG];
#pragma unroll
      for (uint32_t g = 0; g < SPLIT_MAXG; g++) cl[g] = hl[g] = 0;
      for (uint32_t c = a0; c < a1; c += 64 * ST) {
        uint32_t fu[ST], h[ST];
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          const uint32_t k = c + st * 64 + lane;
          fu[st] = k < a1 ? grp[p + k] : 0xFFFFFFFFu;
          h[st] = k < a1 ? pos_hits[p + k] : 0u;
        }
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          if (fu[st] == 0xFFFFFFFFu) continue;
          const uint32_t gk = s_plan.ug[fu[st] & 0xFFu][((fu[st] >> 8) & 0xFFu) - 1];
#pragma unroll
          for (uint32_t g = 0; g < SPLIT_MAXG; g++)
            if (gk == g) {
              cl[g]++;
              hl[g] += h[st];
            }
        }
      }
#pragma unroll
      for (uint32_t g = 0; g < SPLIT_MAXG; g++) {
        if (g >= G) break;  // (uniform)
        const uint32_t cg = wave_sum32(cl[g]), hg = wave_sum32(hl[g]);
        if (lane == 0) {
          s_wc[wv][g] = cg;
          s_wh[wv][g] = hg;
        }
      }
    }
    __syncthreads();
    if (tid < SPLIT_MAXG) {
      uint32_t cn = 0;
      for (uint32_t w = 0; w < NW; w++) cn += tid < G ? s_wc[w][tid] : 0u;
      s_cnt[tid] = cn;
    }
    __syncthreads();
    SPLIT_STAMP(2);
    if (tid == 0) {  // run ids and room, exactly as k_split
      uint32_t acc = 0, nd2 = 0;
      for (uint32_t g = 0; g < SPLIT_MAXG; g++) {
        s_base[g] = acc;
        s_fl[g] = 0;
        acc += s_cnt[g];
        if (g >= 1 && g < G && (s_cnt[g] >= 2 || s_plan.alias[g])) nd2++;
      }
      const unsigned long long add = ((unsigned long long)nd2 << 32) | (unsigned long long)(G - 1);
      const unsigned long long rs = atomicAdd(&split[0], add), base = split[1];
      const bool room = (uint32_t)(base >> 32) + (uint32_t)(rs >> 32) + nd2 <= drun_cap &&
                        (uint32_t)base + (uint32_t)rs + (G - 1) <= b.n;
      if (!room) {
        s_bad = 1;  // (the reservation stays: it only makes later checks stricter)
      } else {
        const unsigned long long old = atomicAdd(num_runs, add);
        s_id[0] = r;
        uint32_t di = (uint32_t)(old >> 32);
        for (uint32_t g = 1; g < G; g++) {
          s_id[g] = (uint32_t)old + g - 1;
          if (s_cnt[g] >= 2 || s_plan.alias[g]) drun[di++] = s_id[g];
        }
      }
    }
    __syncthreads();
    if (s_bad) return;  // (uniform) no room in the dup-run list: the exact path keeps it
    // each wave's starting rank per group, and each group's hits before it
    // (groups are consecutive in the new order: the in-run sums subtract it)
    if (tid < G) {
      uint32_t a = s_base[tid], o = 0;
      for (uint32_t w = 0; w < NW; w++) {
        s_wp[w][tid] = a;
        a += s_wc[w][tid];
      }
      for (uint32_t g = 0; g < (uint32_t)tid; g++)
        for (uint32_t w = 0; w < NW; w++) o += s_wh[w][g];
      s_off[tid] = o;
    }
    if (tid < NW) s_ws[tid] = 0;
    __syncthreads();
    SPLIT_STAMP(3);
    // walk 2, the scatter: a stable rank per group from wave ballots and the
    // wave's running counts; the element id lands in `rank` (a temporary: svals
    // is still being read), hits in hnew, the run id in rid; only a one-unit
    // group's records are read (its clock, its lone-element flag)
    {
      uint32_t run[SPLIT_MAXG], acc[NW];  // acc: hits landing in each wave's chunk of the new order
#pragma unroll
      for (uint32_t g = 0; g < SPLIT_MAXG; g++) run[g] = g < G ? s_wp[wv][g] : 0u;
#pragma unroll
      for (uint32_t w = 0; w < NW; w++) acc[w] = 0;
      // (software-pipelined: the next ST steps' loads are issued before this
      // step's stores, so waiting for them never waits for the stores)
      uint32_t fu[ST], e[ST], h[ST];
#pragma unroll
      for (uint32_t st = 0; st < ST; st++) {
        const uint32_t k = a0 + st * 64 + lane;
        fu[st] = k < a1 ? grp[p + k] : 0xFFFFFFFFu;
        e[st] = k < a1 ? sv[p + k] : 0u;
        h[st] = k < a1 ? pos_hits[p + k] : 0u;
      }
      for (uint32_t c = a0; c < a1; c += 64 * ST) {
        uint32_t fn[ST], en[ST], hn[ST];
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          const uint32_t k = c + (ST + st) * 64 + lane;
          fn[st] = k < a1 ? grp[p + k] : 0xFFFFFFFFu;
          en[st] = k < a1 ? sv[p + k] : 0u;
          hn[st] = k < a1 ? pos_hits[p + k] : 0u;
        }
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          const uint32_t gk =
              fu[st] == 0xFFFFFFFFu ? 0xFFu : s_plan.ug[fu[st] & 0xFFu][((fu[st] >> 8) & 0xFFu) - 1];
          uint32_t np = 0;
#pragma unroll
          for (uint32_t g = 0; g < SPLIT_MAXG; g++) {
            if (g >= G) break;  // (uniform)
            const uint64_t m = __ballot(gk == g);
            if (gk == g) np = run[g] + __popcll(m & lt);
            run[g] += __popcll(m);
          }
          if (gk >= SPLIT_MAXG) continue;
          rank[p + np] = e[st];
          rid[p + np] = s_id[gk];
          hnew[p + np] = h[st];
          if constexpr (NW <= 4) {  // (more waves: walk 3 sums its chunks in a pass of its own)
            uint32_t dw = 0;  // the wave whose chunk of the new order np is in
#pragma unroll
            for (uint32_t w = 1; w < NW; w++) dw += np >= w * CH ? 1u : 0u;
#pragma unroll
            for (uint32_t w = 0; w < NW; w++)
              if (dw == w) acc[w] += h[st];
          }
          if (!s_plan.alias[gk]) {  // (a multi-unit stem's groups share one `now`)
            const uint32_t f = s_plan.fam[gk];
            // (the head's family: k_run_check compared `now` with the head's,
            // s_lnow[0]; only an element whose clock differs is read again)
            const bool known = f == 0 && s_cnt[gk] != 1 && !(fu[st] & SPLIT_POS_NOWVAR);
            if (!known) {
              const Rec x = rec[e[st]];
              const uint32_t d = div_of(s_lunit[f]);
              if (x.now != s_lnow[f])
                atomicOr(&s_fl[gk], x.now / d != s_lnow[f] / d ? RUN_SLOW | RUN_NOWVAR : RUN_NOWVAR);
              // a lone group of one element is a key seen once (k_table's singleton part)
              if (s_cnt[gk] == 1) {
                uq.single(e[st], p);
              }
            }
          }
        }
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          fu[st] = fn[st];
          e[st] = en[st];
          h[st] = hn[st];
        }
      }
      if constexpr (NW <= 4) {
#pragma unroll
        for (uint32_t w = 0; w < NW; w++) {
          const uint32_t t = wave_sum32(acc[w]);
          if (lane == 0 && t) atomicAdd(&s_ws[w], t);
        }
      }
    }
    __syncthreads();
    if constexpr (NW > 4) {  // each wave's chunk of the new order: its hits, summed
      uint32_t t = 0;
      for (uint32_t k = a0 + lane; k < a1; k += 64) t += hnew[p + k];
      t = wave_sum32(t);
      if (lane == 0) s_ws[wv] = t;
      __syncthreads();
    }
    SPLIT_STAMP(4);
    SPLIT_STAMP(5);
    // walk 3: inclusive sums in the new order (mod 2^32, like the bucket
    // kernels'; each wave starts from the hits of the chunks before its own,
    // summed by the scatter) with the group's offset taken off, and the new
    // permutation from `rank` into svals
    {
      uint32_t carry = 0, g = 0;
      for (uint32_t w = 0; w < wv; w++) carry += s_ws[w];
      uint32_t h[ST], e[ST];
#pragma unroll
      for (uint32_t st = 0; st < ST; st++) {
        const uint32_t k = a0 + st * 64 + lane;
        h[st] = k < a1 ? hnew[p + k] : 0u;
        e[st] = k < a1 ? rank[p + k] : 0u;
      }
      for (uint32_t c = a0; c < a1; c += 64 * ST) {
        uint32_t hn[ST], en[ST];  // (software-pipelined, as the scatter)
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          const uint32_t k = c + (ST + st) * 64 + lane;
          hn[st] = k < a1 ? hnew[p + k] : 0u;
          en[st] = k < a1 ? rank[p + k] : 0u;
        }
        // the ST wave scans (DPP: ST independent chains of VALU operations)
        uint32_t inc[ST];
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) inc[st] = wave_incl_add(h[st]);
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          const uint32_t k = c + st * 64 + lane;
          const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc[st], 63);
          if (k < a1) {
            while (g + 1 < G && k >= s_base[g + 1]) g++;  // (k grows along the walk)
            segsum[p + k] = carry + inc[st] - s_off[g];
            svals[p + k] = e[st];
          }
          carry += tot;
        }
#pragma unroll
        for (uint32_t st = 0; st < ST; st++) {
          h[st] = hn[st];
          e[st] = en[st];
        }
      }
    }
    if (tid < G) {
      const uint32_t id = s_id[tid];
      run_start[id] = p + s_base[tid];
      run_end[id] = p + s_base[tid] + s_cnt[tid];
      run_flags[id] = split_group_flags(s_plan, tid, s_fl[tid]);
    }
    if (tid == 0) defer[j] = DEFER_DONE;
#ifdef RL_SPLIT_PROF
    if (tid == 0 && L > 20000) {
      ts[6] = wall_clock64();
      printf("split_long L=%u G=%u rfl=%x: fam %lu walk1 %lu ids %lu walk2 %lu walk3a %lu walk3b %lu (x10ns)\n", L, G, rfl,
             (unsigned long)(ts[1] - ts[0]), (unsigned long)(ts[2] - ts[1]), (unsigned long)(ts[3] - ts[2]),
             (unsigned long)(ts[4] - ts[3]), (unsigned long)(ts[5] - ts[4]), (unsigned long)(ts[6] - ts[5]));
    }
#endif
  }
}


// k_split_long: the runs over SPLIT_CAP elements k_split listed (long_runs[0]
// of them, defer indices from long_runs[1]), one per workgroup of
// RL_SPLIT_LONG_THREADS lanes. split_long_body's walks are a wave's chain of
// steps (one wave per SIMD at 256 lanes: each step's LDS lookup, ballots and
// stores wait on one another), so four times the waves walk a four times
// shorter chunk each; k_split itself keeps 256-lane workgroups for the many
// short runs (C1's k_split at 1024 lanes: 18 -> 26 us).
#if RL_SPLIT_LONG_THREADS
__global__ __launch_bounds__(RL_SPLIT_LONG_THREADS, RL_SPLIT_LONG_OCC) void k_split_long(
    BatchDev b, SRec rec_s, uint32_t* __restrict__ svals, uint32_t* __restrict__ segsum, uint32_t* __restrict__ rid,
    uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_end, uint32_t* __restrict__ run_flags,
    uint32_t* __restrict__ defer, unsigned long long* num_runs, unsigned long long* split, uint32_t* __restrict__ drun,
    uint32_t drun_cap, uint32_t* grp, uint32_t* rank, uint32_t* __restrict__ pos_hits, uint32_t* __restrict__ hnew,
    const uint32_t* err, int per_second, UniqList uq, const uint32_t* __restrict__ long_runs) {
  if (*err) return;
  refine_totals(b);
  const uint32_t nl = long_runs[0];
  for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const uint32_t j = long_runs[1 + i], r = defer[j];
    const uint32_t p = run_start[r], L = run_end[r] - p;
    split_long_body<RL_SPLIT_LONG_THREADS, RL_SPLIT_LONG_ST>(j, r, p, L, b, rec_s, svals, segsum, rid, run_start,
                                                             run_end, run_flags, defer, num_runs, split, drun,
                                                             drun_cap, grp, rank, pos_hits, hnew, per_second,
                                                             run_flags[r], uq);
  }
}
#endif

// k_split's minimum waves per SIMD (1: what the inline long walk asks for,
// 221 VGPRs; 4: 128, the long walk spills — it runs here only until the host
// switches to k_split_long —: C1, C2, C2U flat, profiles/r05/split_long/)
#ifndef RL_SPLIT_OCC
#define RL_SPLIT_OCC 1
#endif
__global__ __launch_bounds__(SPLIT_THREADS, RL_SPLIT_OCC) void k_split(BatchDev b, SRec rec_s, uint32_t* __restrict__ svals,
                                               uint32_t* __restrict__ segsum, uint32_t* __restrict__ rid,
                                               uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_end,
                                               uint32_t* __restrict__ run_flags, uint32_t* __restrict__ defer,
                                               const uint32_t* defer_n, unsigned long long* num_runs,
                                               unsigned long long* split, uint32_t* __restrict__ drun,
                                               uint32_t drun_cap, uint32_t* grp, uint32_t* rank,
                                               uint32_t* __restrict__ pos_hits, uint32_t* __restrict__ hnew,
                                               const uint32_t* err, int per_second, UniqList uq,
                                               uint32_t* __restrict__ long_runs, uint32_t* long_hint, int delegate) {
  __shared__ uint32_t s_e[SPLIT_CAP], s_hlo[SPLIT_CAP], s_lu[SPLIT_CAP], s_now[SPLIT_CAP], s_h[SPLIT_CAP];
  __shared__ uint32_t s_nh[SPLIT_CAP];           // max(1, hits) in the new order
  __shared__ uint16_t s_pos[SPLIT_CAP];          // rank inside the element's group
  __shared__ uint8_t s_g[SPLIT_CAP], s_ng[SPLIT_CAP];  // family, then group, of each element / group of each new position
  __shared__ uint32_t s_cnt[SPLIT_MAXG], s_base[SPLIT_MAXG], s_id[SPLIT_MAXG], s_fl[SPLIT_MAXG];
  __shared__ uint32_t s_lnow[SPLIT_MAXG], s_lunit[SPLIT_MAXG], s_fmask[SPLIT_MAXG], s_fnv[SPLIT_MAXG];
  __shared__ uint32_t s_bad, s_lead;
  __shared__ SplitPlan s_plan;
  if (*err) return;
  refine_totals(b);
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t nd = *defer_n;
  Rec* rec = const_cast<Rec*>(rec_s.rec);
  for (uint32_t j = blockIdx.x; j < nd; j += gridDim.x) {
    const uint32_t r = defer[j];
    const uint32_t p = run_start[r], L = run_end[r] - p;
    if (L > SPLIT_CAP) {  // (uniform)
      if (tid == 0 && long_hint) *long_hint = 1u;  // (the host's cue to launch k_split_long for the next batches)
#if RL_SPLIT_LONG_THREADS
      if (delegate) {
        if (tid == 0) long_runs[1 + atomicAdd(&long_runs[0], 1u)] = j;  // k_split_long's
        continue;
      }
#endif
      split_long_body<SPLIT_THREADS, SPLIT_ST>(j, r, p, L, b, rec_s, svals, segsum, rid, run_start, run_end, run_flags,
                                               defer, num_runs, split, drun, drun_cap, grp, rank, pos_hits, hnew,
                                               per_second, run_flags[r], uq);
      continue;
    }
    __syncthreads();  // the previous run's shared state has been read
    if (tid == 0) s_bad = 0;
    if (tid < SPLIT_MAXG) {
      s_fmask[tid] = 0;
      s_fnv[tid] = 0;
    }
    for (uint32_t k = tid; k < L; k += SPLIT_THREADS) {
      const uint32_t e = rec_s.sv[p + k];
      const Rec x = rec[e];
      s_e[k] = e;
      s_hlo[k] = x.hlo;
      s_lu[k] = x.lu;
      s_now[k] = x.now;
      s_h[k] = x.hits > 1 ? x.hits : 1u;
      s_g[k] = 0xFF;
    }
    __syncthreads();
    for (uint32_t k = tid; k < L; k += SPLIT_THREADS)
      if ((s_lu[k] >> 24) & FLAG_SKIP) s_bad = 1;
    // families: repeatedly the first unassigned element leads, and every
    // element with its stem (hash, length, then bytes) joins
    uint32_t NF = 0;
    for (;;) {
      if (tid == 0) s_lead = 0xFFFFFFFFu;
      __syncthreads();
      for (uint32_t k = tid; k < L; k += SPLIT_THREADS)
        if (s_g[k] == 0xFF) atomicMin(&s_lead, k);
      __syncthreads();
      const uint32_t ld = s_lead;
      if (ld == 0xFFFFFFFFu || s_bad || NF == SPLIT_MAXG) break;  // (uniform)
      const Rec y = rec[s_e[ld]];
      const Key ky = key_of(b, y);
      if (tid == 0) {
        s_lnow[NF] = y.now;
        s_lunit[NF] = rec_unit(y);
      }
      for (uint32_t k = tid; k < L; k += SPLIT_THREADS) {
        if (s_g[k] != 0xFF || s_hlo[k] != y.hlo || (s_lu[k] & 0xFFFFu) != (y.lu & 0xFFFFu)) continue;
        if (!key_equal(key_of(b, rec[s_e[k]]), ky)) {
          s_bad = 1;  // equal 64-bit hash, different stem
        } else {
          atomicOr(&s_fmask[NF], 1u << (((s_lu[k] >> 16) & 0xFFu) - 1));
          if (s_now[k] != y.now) s_fnv[NF] = 1;
          s_g[k] = (uint8_t)NF;
        }
      }
      NF++;
      __syncthreads();
    }
    if (s_lead != 0xFFFFFFFFu) s_bad = 1;  // more than SPLIT_MAXG stems (or stopped early)
    __syncthreads();
    if (s_bad) continue;  // (uniform) the exact path keeps it
    if (tid == 0 && split_plan(s_plan, NF, s_fmask, s_lnow, s_fnv, per_second) == SPLIT_BAD) s_bad = 1;
    __syncthreads();
    const uint32_t G = s_plan.G;
    if (s_bad || (G < 2 && !s_plan.any_alias)) continue;  // (uniform) the exact path keeps it
    for (uint32_t k = tid; k < L; k += SPLIT_THREADS) s_g[k] = s_plan.ug[s_g[k]][((s_lu[k] >> 16) & 0xFFu) - 1];
    __syncthreads();
    // stable ranks inside the groups (wave 0 walks the run in arrival order)
    if (tid < 64) {
      uint32_t cnt[SPLIT_MAXG];
#pragma unroll
      for (uint32_t g = 0; g < SPLIT_MAXG; g++) cnt[g] = 0;
      const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
      for (uint32_t c0 = 0; c0 < L; c0 += 64) {
        const uint32_t k = c0 + lane;
        const uint32_t gk = k < L ? s_g[k] : 0xFFu;
#pragma unroll
        for (uint32_t g = 0; g < SPLIT_MAXG; g++) {
          const uint64_t m = __ballot(gk == g);
          if (gk == g) s_pos[k] = (uint16_t)(cnt[g] + __popcll(m & lt));
          cnt[g] += __popcll(m);
        }
      }
      if (lane == 0) {
        uint32_t acc = 0;
#pragma unroll
        for (uint32_t g = 0; g < SPLIT_MAXG; g++) {
          s_cnt[g] = cnt[g];
          s_base[g] = acc;
          s_fl[g] = 0;
          acc += cnt[g];
        }
        // run ids: group 0 keeps r, the others are new; the dup-run list
        // (k_table's runs part) takes the new ones of two or more elements and
        // every group of a multi-unit stem
        uint32_t nd2 = 0;
        for (uint32_t g = 1; g < G; g++) nd2 += (cnt[g] >= 2 || s_plan.alias[g]) ? 1u : 0u;
        // room: a reservation (one fetch-add; a CAS loop on the shared
        // counter serialised ~100 blocks) is checked against the bucket
        // kernels' count plus every reservation before it, so the successful
        // ones, the only ones added to num_runs, always fit
        const unsigned long long add = ((unsigned long long)nd2 << 32) | (unsigned long long)(G - 1);
        const unsigned long long rs = atomicAdd(&split[0], add), base = split[1];
        const bool room = (uint32_t)(base >> 32) + (uint32_t)(rs >> 32) + nd2 <= drun_cap &&
                          (uint32_t)base + (uint32_t)rs + (G - 1) <= b.n;
        unsigned long long old = 0;
        if (!room) s_bad = 1;
        else old = atomicAdd(num_runs, add);
        if (!s_bad) {
          s_id[0] = r;
          uint32_t di = (uint32_t)(old >> 32);
          for (uint32_t g = 1; g < G; g++) {
            s_id[g] = (uint32_t)old + g - 1;
            if (cnt[g] >= 2 || s_plan.alias[g]) drun[di++] = s_id[g];
          }
        }
      }
    }
    __syncthreads();
    if (s_bad) continue;  // (uniform) no room in the dup-run list: the exact path keeps it
    for (uint32_t k = tid; k < L; k += SPLIT_THREADS) {
      const uint32_t g = s_g[k], np = s_base[g] + s_pos[k];
      svals[p + np] = s_e[k];
      rid[p + np] = s_id[g];
      s_nh[np] = s_h[k];
      s_ng[np] = (uint8_t)g;
      if (!s_plan.alias[g]) {  // (a multi-unit stem's groups share one `now`)
        const uint32_t f = s_plan.fam[g], d = div_of(s_lunit[f]);
        if (s_now[k] != s_lnow[f])
          atomicOr(&s_fl[g], s_now[k] / d != s_lnow[f] / d ? RUN_SLOW | RUN_NOWVAR : RUN_NOWVAR);
        // a lone group of one element is a key seen once (k_table's singleton part)
        if (s_cnt[g] == 1) {
          uq.single(s_e[k], p);
        }
      }
    }
    __syncthreads();
    // inclusive sums of max(1, hits) inside each group, in the new order
    // (wave 0; the groups are consecutive): segmented wave scans + carry
    if (tid < 64) {
      uint32_t carry = 0;
      for (uint32_t c0 = 0; c0 < L; c0 += 64) {
        const uint32_t k = c0 + lane;
        const bool in = k < L;
        uint32_t v = in ? s_nh[k] : 0u;
        bool f = in && (k == 0 || s_ng[k - 1] != s_ng[k]);  // a group starts here
#pragma unroll
        for (uint32_t off = 1; off < 64; off <<= 1) {
          const uint32_t y = __shfl_up(v, off, 64);
          const bool yf = __shfl_up(f ? 1 : 0, off, 64) != 0;
          if (lane >= off) {
            if (!f) v += y;
            f = f || yf;
          }
        }
        if (!f) v += carry;  // no group start since the chunk began
        if (in) segsum[p + k] = v;
        carry = __shfl(v, 63, 64);
      }
    }
    if (tid < G) {
      const uint32_t id = s_id[tid];
      run_start[id] = p + s_base[tid];
      run_end[id] = p + s_base[tid] + s_cnt[tid];
      run_flags[id] = split_group_flags(s_plan, tid, s_fl[tid]);
    }
    if (tid == 0) defer[j] = DEFER_DONE;
  }
}

// ---- k_table, keys seen once (unique_body): sort key once in the batch (no
// dup mark), one lane each. Such a stem has no other descriptor in the batch,
// so the lanes are independent and this part commutes with the sorted path
// (runs_body). A stem that lives in the table under another unit too is left
// to k_runs_general (defer1). Two orders, chosen per batch on the device:
//  * a batch made mostly of keys seen once (C1, C3) is answered in ARRIVAL
//    order: the record, the sort key and the stem are coalesced wave reads
//    (consecutive descriptors sit side by side in the packed batch), the
//    result a coalesced store; only the slot's first sector (and the changed
//    window record) is a random access. A block with >= 75% of them answers in
//    place, a sparser one compacts them onto its first lanes;
//  * a sparser batch (hot keys, C2) walks the list the stage-A kernels leave
//    (Scratch::uniq, bucket by bucket): every workgroup is full, and the
//    record, stem and result are gathers. C2 4.83 -> 5.29 G (profiles/r05/).
//    At C1 the gathers cost more than the list order saves on the table
//    probes (a workgroup's probes inside 1/1024 of the table): 5.35 vs 5.99 G
//    with the list for every batch; tools/orderprobe.hip prices the whole
//    access pattern per order and layout (profiles/r05/orderprobe.txt).
#ifndef RL_UNIQ_DENSE
#define RL_UNIQ_DENSE 3  // (A/B builds: quarters of the batch below which the list is walked; 5 = always, 0 = never)
#endif
__device__ __attribute__((always_inline)) inline void unique_body(uint32_t blk, BatchDev b, TableDev t, Params P, const Rec* __restrict__ rec,
                                                const uint32_t* __restrict__ keys0,
                                                const uint2* __restrict__ uniq, const uint32_t* uniq_n,
                                                unsigned long long* __restrict__ res,
                                                uint32_t* __restrict__ defer1, uint32_t* defer1_n,
                                                unsigned long long* stats, unsigned long long* stripes, uint32_t* err,
                                                uint32_t* errs, int restore, const uint32_t* errb_prev) {
  __shared__ uint32_t s_err, s_nu, s_cnt, s_list[256];
  if (threadIdx.x == 0) {
    s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (errb_prev ? *errb_prev : 0u);
    s_nu = *uniq_n;
  }
  __syncthreads();
  const uint32_t nu = s_nu;
  const bool by_list = (uint64_t)nu * 4 < (uint64_t)b.n * RL_UNIQ_DENSE;  // (uniform) fewer than 75% keys seen once
  const uint32_t lo = blk * 256, hi = min(lo + 256, by_list ? nu : b.n);
  if (s_err || lo >= hi) return;
  refine_totals(b);
  uint32_t* ferr = P.isolate ? errs : err;
  const bool use_lds = !restore && b.n_rules <= LDS_RULES;
  stats_block_begin(use_lds, b.n_rules);
  StatAcc acc{use_lds, stats};
  LaneStats L;
  L.reset();
  // not a duplicated key (the sorted path's), not failed (answered already)
  auto single = [&](uint32_t i) { return keys0[i] != KEY_DUP && !((rec[i].lu >> 24) & FLAG_SKIP); };
  bool act;
  uint32_t i, key = 0;
  if (by_list) {
    const uint32_t pos = lo + threadIdx.x;
    const uint2 ent = pos < hi ? uniq[pos] : make_uint2(0u, 0u);
    i = ent.x;
    key = ent.y;
    act = pos < hi && single(i);
  } else {
    const uint32_t i0 = lo + threadIdx.x;
    const bool own = i0 < hi && single(i0);
    if (__syncthreads_count(own) >= 192) {
      act = own;
      i = i0;
    } else {
      const uint32_t cnt = block_compact(lo, hi, s_list, &s_cnt, single);
      act = threadIdx.x < cnt;
      i = act ? s_list[threadIdx.x] : 0u;
    }
    if (act) key = keys0[i];
  }
  if (act) {
    const Rec x = rec[i];
    {
      const uint64_t h0 = ((uint64_t)key << 32) | x.hlo;
      const uint32_t u0 = rec_unit(x);
      SlotImg im;
      load_img_lo(&t.slots[h0 >> t.shift], im);  // home slot's first sector, in flight beside the stem
      const Key k0 = key_of(b, x);
      bool ins = false, ok = true;
      const uint32_t tg0 = slot_tag(h0, u0);
      const int64_t s0 = find_slot_img(t, h0, tg0, k0, u0, &ins, im, ferr);
      if (s0 < 0) {
        ok = false;
      } else if (im.flags() & SLOT_EXACT) {
        ok = false;
      } else if (ins) {  // new (stem, unit): the stem must not exist under another unit
        for (uint32_t u = 1; u <= 4; u++) {
          bool dummy;
          const int64_t so = u == u0 ? -1 : find_slot(t, h0, slot_tag(h0, u), k0, u, false, &dummy, ferr);
          if (so >= 0) {
            t.slots[so].flags |= SLOT_EXACT;
            ok = false;
          }
        }
        if (!ok) t.slots[s0].flags |= SLOT_EXACT;
      }
      if (ok) {
        replay_simple(SRec{rec, nullptr}, nullptr, res, t, P, nullptr, 0, 1, 0, s0, im.cur(), im.ring(), tg0, x, i,
                      L, acc, ferr,
                      restore);
      } else if (s0 == SLOT_TABLE_FULL || s0 == SLOT_ARENA_FULL) {
        if (P.isolate) res[i] = pack_fail(slot_fail_status(s0));  // else the batch fails
      } else {
        defer1[atomicAdd(defer1_n, 1u)] = i;
      }
    }
  }
  if (!restore) wave_flush(L, acc);
  stats_block_end(use_lds, b.n_rules, stripes);
}

// ---- k_table, runs (runs_body): one lane per run of one stem and one unit. Short
// runs whose slot is not flagged multi-unit are replayed here in registers;
// long uniform runs are set up for the parallel path (k_fast_*); a stem that
// turns out to live in the table under another unit too is queued for the
// exact path (defer2, k_runs_general after this kernel).
// Every element of sorted positions [p, end) gets status st (isolate mode).
__device__ inline void fail_range(unsigned long long* res, const uint32_t* svals, uint32_t p, uint32_t end,
                                  uint32_t st) {
  for (uint32_t q = p; q < end; q++) res[svals[q]] = pack_fail(st);
}

// ---- alias_setup (k_table's runs part, one lane): the groups of a stem that
// lives in the table under several units, or is seen under several in this
// batch (k_split: one group per Redis key stem ‖ windowStart, consecutive,
// sharing one `now`). general_step's semantics, set up for the parallel path
// (k_fast_over / fast_emit_body) instead of replayed by one lane:
//  * a Redis key's count and EXPIRE live in every unit slot that holds a
//    record of its window (the same store under the per-second split); its
//    local-cache entry in every one of them;
//  * the count a group starts from is the first such record, in unit order,
//    still live at `now`; its local-cache hit (F) is any record's entry live
//    at `now` — one `now` per group, so both hold for the whole group;
//  * each unit of a group that increments gets its record of the window
//    (rolled into cur; a new one takes the live local-cache expiry of the
//    others), and the group's last INCRBY writes its count and EXPIRE to every
//    record of the key, its local-cache Set to all of them.
// The parallel path writes curs only. A group that would need a record below
// a unit's cur (a new one, or one held in the history log, or a cur that
// another group rolls away), or whose record the history may have dropped, is
// left — rare by construction — to the exact path untouched (returns true).
struct AliasGroup {
  uint32_t id, p, end, mask, w;
};

// A stem's unit slots in one walk of its probe sequence (they share the home
// slot: the unit is in the tag, not in the hash): per unit, the first slot of
// its tag, unit and stem before the first empty slot, with its cur and
// history head from the same 64-B image. Returns the units found, and
// UNIT_WALK_ENDED when the walk reached an empty slot (a unit not found is
// then absent). find_slot takes the rest (inserts; a probe window without an
// empty slot). Four walks, one per unit, of a few dependent loads each took
// ~20 us per hot stem under k_table's load (RL_ALIAS_PROF builds).
#ifndef RL_ALIAS_ONE_WALK
#define RL_ALIAS_ONE_WALK 1
#endif
constexpr uint32_t UNIT_WALK_ENDED = 0x10u;
__device__ inline uint32_t find_unit_slots(const TableDev& t, uint64_t hs, const Key& stem, int64_t sidx[4], Win c[4],
                                           uint32_t chain[4]) {
  uint64_t i = hs >> t.shift;
  uint32_t found = 0;
  SlotImg im;
  for (uint32_t p = 0; p < t.max_probe && found != 0xFu; p++, i = (i + 1) & t.mask) {
    load_img_lo(&t.slots[i], im);
    const uint32_t st = im.tag();
    if (st == TAG_EMPTY) return found | UNIT_WALK_ENDED;
    const uint32_t u = im.unit();
    if (u < 1 || u > 4 || ((found >> (u - 1)) & 1) || st != slot_tag(hs, u) || !img_key_equal(im, stem, t.arena))
      continue;
    sidx[u - 1] = (int64_t)i;
    c[u - 1] = im.cur();
    chain[u - 1] = im.ring();
    found |= 1u << (u - 1);
  }
  return found;
}

#ifndef RL_ALIAS_NOINLINE
#define RL_ALIAS_NOINLINE 0  // (noinline: k_table gets a 448-B scratch frame; C1 -1.5 %, profiles/r03/ab_alias_variants/)
#endif
#if RL_ALIAS_NOINLINE
#define RL_ALIAS_ATTR __attribute__((noinline))
#else
#define RL_ALIAS_ATTR inline
#endif
__device__ RL_ALIAS_ATTR bool alias_setup(const TableDev& t, const Params& P, SRec rec_s, const uint32_t* __restrict__ rid,
                                   const uint32_t* __restrict__ run_start, const uint32_t* __restrict__ run_end,
                                   uint32_t* __restrict__ run_flags, uint4* __restrict__ run_state,
                                   uint4* __restrict__ run_alias, uint32_t* __restrict__ run_f,
                                   uint32_t* __restrict__ fast_blk, unsigned long long* __restrict__ res,
                                   const uint32_t* __restrict__ svals, uint32_t* ferr, uint32_t r, uint32_t fl,
                                   uint32_t u0, uint64_t hs, const Key& stem, uint32_t now) {
#ifdef RL_NO_ALIAS  // (measurement builds: what the alias path costs the common case)
  return true;
#endif
#ifdef RL_ALIAS_PROF  // (measurement builds: phase stamps of the setup of long alias groups)
  uint64_t ta[4];
  ta[0] = wall_clock64();
#define ALIAS_STAMP(i) ta[i] = wall_clock64()
#else
#define ALIAS_STAMP(i)
#endif
  AliasGroup A[4];
  uint32_t G = 1, M;
  A[0].id = r;
  A[0].p = run_start[r];
  A[0].end = run_end[r];
  if (fl & RUN_AHEAD) {
    G = (fl >> RUN_G_SHIFT) & 0xFFu;
    A[0].mask = (fl >> RUN_UMASK_SHIFT) & 0xFu;
    for (uint32_t g = 1; g < G && g < 4; g++) {
      const uint32_t id = rid[A[g - 1].end];
      A[g].id = id;
      A[g].p = run_start[id];
      A[g].end = run_end[id];
      A[g].mask = (run_flags[id] >> RUN_UMASK_SHIFT) & 0xFu;
    }
    if (G > 4) return true;  // (cannot happen: one group per unit at most)
  } else {
    A[0].mask = 1u << (u0 - 1);
  }
  M = 0;
  for (uint32_t g = 0; g < G; g++) {
    const uint32_t d = div_of(__ffs(A[g].mask));
    A[g].w = now - now % d;
    M |= A[g].mask;
  }
  // every unit slot of the stem (created for the units seen here)
  int64_t sidx[4];
  Win c[4];
  uint32_t chain[4];
  uint32_t present = 0;
  int64_t fail = 0;
#if RL_ALIAS_ONE_WALK
  const uint32_t fr = find_unit_slots(t, hs, stem, sidx, c, chain);
#else
  const uint32_t fr = 0;
#endif
  for (uint32_t k = 0; k < 4; k++) {
    if ((fr >> k) & 1) {  // (found by the one walk: image read there)
      present |= 1u << k;
      continue;
    }
    chain[k] = LOG_NONE;
    if ((fr & UNIT_WALK_ENDED) && !((M >> k) & 1)) {  // absent: the walk reached an empty slot first
      sidx[k] = SLOT_ABSENT;
      continue;
    }
    bool ins;
    sidx[k] = find_slot(t, hs, slot_tag(hs, k + 1), stem, k + 1, (M >> k) & 1, &ins, ferr);
    if (sidx[k] >= 0) {
      const Slot& su = t.slots[sidx[k]];
      present |= 1u << k;
      c[k] = su.cur;
      chain[k] = su.ring;
    } else if ((M >> k) & 1) {
      fail = sidx[k];
    }
  }
  if (fail) {
    if (P.isolate)
      for (uint32_t g = 0; g < G; g++) fail_range(res, svals, A[g].p, A[g].end, slot_fail_status(fail));
    return false;  // (else find_slot set the batch's error)
  }
  ALIAS_STAMP(1);
  // the units that roll their cur forward (a group that may increment: the
  // local-cache hit F is not known yet) and so move it to the history log
  uint32_t rolls = 0;
  for (uint32_t g = 0; g < G; g++)
    for (uint32_t k = 0; k < 4; k++)
      if (((A[g].mask >> k) & 1) && c[k].ws != A[g].w) {
        if (c[k].ws != WS_INVALID && A[g].w < c[k].ws) return true;  // a new record below cur: the exact path
        rolls |= 1u << k;
      }
  // The groups' starting state from the curs and the logged records. A
  // group's key held in a unit's history log (below that unit's cur: e.g. a
  // SECOND slot's record of the minute's first second, which is the MINUTE
  // key too) is read there and written back to a new version of that record
  // appended below (lgm: bit 4g + k). A group whose record is in a cur that
  // rolls away, or may have been dropped, goes to the exact path.
  // A group whose record is a cur that another group rolls away (the SECOND
  // slot's cur of the minute's first second, one second later) finds it in
  // the roll's log entry instead (lgr: bit 4g + k), provided the roll keeps it.
  uint32_t v0[4], lcm[4], F[4], lgm = 0, lgr = 0;
  for (uint32_t g = 0; g < G; g++) {
    const uint32_t w = A[g].w;
    const bool cls = P.per_second && (A[g].mask & 1u);
    bool vf = false;
    v0[g] = 0;
    lcm[g] = 0;
    for (uint32_t k = 0; k < 4; k++) {
      if (!((present >> k) & 1)) continue;
      const uint32_t d = div_of(k + 1);
      Win R;
      if (c[k].ws == w) {
        if ((rolls >> k) & 1) {
          uint32_t wn = w;  // the window unit k rolls to: the newest of its groups'
          for (uint32_t h = 0; h < G; h++)
            if (((A[h].mask >> k) & 1) && A[h].w > wn) wn = A[h].w;
          if (!hist_keep(t, c[k], wn, d)) return true;
          lgr |= 1u << (4 * g + k);
        }
        R = c[k];
      } else if (c[k].ws == WS_INVALID || w > c[k].ws || w % d) {
        continue;  // (unit k's keys are multiples of its div)
      } else {
        const int f = chain[k] == LOG_NONE ? 0 : log_find(t, chain[k], (uint32_t)sidx[k], slot_tag(hs, k + 1), c[k].ws, w, &R);
        if (f < 0 || (f == 0 && !hist_absent_ok(t, now, w, c[k].ws, d))) return true;
        if (f == 0) continue;
        lgm |= 1u << (4 * g + k);
      }
      const bool live = (P.per_second && k == 0) == cls && now <= R.expire;
      lcm[g] = R.lc > lcm[g] ? R.lc : lcm[g];
      if (!vf && live) {
        v0[g] = R.count;
        vf = true;
      }
    }
    F[g] = (P.lc_en && now < lcm[g]) ? 1u : 0u;
  }
  ALIAS_STAMP(2);
  // the new cur of each unit that rolls (groups that increment)
  Win cn[4];
  for (uint32_t k = 0; k < 4; k++) cn[k] = c[k];
  for (uint32_t g = 0; g < G; g++)
    for (uint32_t k = 0; k < 4; k++)
      if (!F[g] && ((A[g].mask >> k) & 1) && (c[k].ws == WS_INVALID || A[g].w > c[k].ws))
        cn[k] = Win{A[g].w, 0, 0, lcm[g]};
  // commit: rolls (the old cur to the history log while a request could still ask for it)
  uint32_t rolled[4] = {LOG_NONE, LOG_NONE, LOG_NONE, LOG_NONE};  // the roll's log entry per unit
  for (uint32_t k = 0; k < 4; k++) {
    if (cn[k].ws == c[k].ws) continue;
    Slot* su = &t.slots[sidx[k]];
    if (c[k].ws != WS_INVALID && hist_keep(t, c[k], cn[k].ws, div_of(k + 1))) {
      su->ring = log_append(t, (uint32_t)sidx[k], slot_tag(hs, k + 1), chain[k], cn[k].ws, c[k]);
      rolled[k] = su->ring;
    }
    su->cur = cn[k];
  }
  if (__popc(present) >= 2)
    for (uint32_t k = 0; k < 4; k++)
      if ((present >> k) & 1) t.slots[sidx[k]].flags |= SLOT_EXACT;
  // write-back targets (per unit: bit 0 its cur holds w, bit 1 its history
  // log does — the record's new version appended here, whose entry pointer
  // takes the unit's place in run_alias —, bit 2 same store)
  for (uint32_t g = 0; g < G; g++) {
    const uint32_t w = A[g].w;
    const bool cls = P.per_second && (A[g].mask & 1u);
    uint32_t tm = 0;
    uint32_t sl[4];
    for (uint32_t k = 0; k < 4; k++) sl[k] = (present >> k) & 1 ? (uint32_t)sidx[k] : 0xFFFFFFFFu;
    if (!F[g]) {
      for (uint32_t k = 0; k < 4; k++) {
        if (!((present >> k) & 1)) continue;
        uint32_t bits = cn[k].ws == w ? 1u : 0u;
        if (!bits && ((lgr >> (4 * g + k)) & 1) && rolled[k] != LOG_NONE) {  // (its record rolled into the log)
          sl[k] = rolled[k];
          bits = 2u;
        } else if ((lgm >> (4 * g + k)) & 1) {  // (rare: the hot key's group in another unit's log, once per batch)
          Win R;
          if (log_find(t, chain[k], (uint32_t)sidx[k], slot_tag(hs, k + 1), c[k].ws, w, &R) == 1) {
            Slot* su = &t.slots[sidx[k]];
            su->ring = log_append(t, (uint32_t)sidx[k], slot_tag(hs, k + 1), su->ring, cn[k].ws, R);
            sl[k] = su->ring;
            bits = 2u;
          }
        }
        if (bits && (P.per_second && k == 0) == cls) bits |= 4;
        tm |= bits << (3 * k);
      }
    }
    const uint32_t id = A[g].id;
    run_state[id] = make_uint4(tm, v0[g], lcm[g], F[g]);
    run_alias[id] = make_uint4(sl[0], sl[1], sl[2], sl[3]);
    run_f[id] = 0xFFFFFFFFu;
    run_flags[id] = (g == 0 ? fl : run_flags[id]) | RUN_FAST | RUN_ALIAS;
    const uint32_t b0 = A[g].p >> 8, b1 = (A[g].end - 1) >> 8;
    for (uint32_t x = b0 >> 5; x <= b1 >> 5; x++) {
      const uint32_t lo = x == (b0 >> 5) ? (b0 & 31) : 0u, hi = x == (b1 >> 5) ? (b1 & 31) : 31u;
      atomicOr(&fast_blk[x], (0xFFFFFFFFu >> (31 - hi)) & (0xFFFFFFFFu << lo));
    }
  }
#ifdef RL_ALIAS_PROF
  ta[3] = wall_clock64();
  if (A[0].end - A[0].p > 4000)
    printf("alias_setup G=%u L=%u: slots %lu reads %lu commit %lu (x10ns)\n", G, A[0].end - A[0].p,
           (unsigned long)(ta[1] - ta[0]), (unsigned long)(ta[2] - ta[1]), (unsigned long)(ta[3] - ta[2]));
#endif
  return false;
}


__device__ __attribute__((always_inline)) inline void runs_body(uint32_t blk, BatchDev b, TableDev t, Params P, SRec rec_s,
                                              const uint32_t* __restrict__ skeys,
                                              const uint32_t* __restrict__ svals, unsigned long long* __restrict__ res,
                                              const uint32_t* __restrict__ run_start,
                                              const uint32_t* __restrict__ run_end,
                                              uint32_t* __restrict__ run_flags, uint4* __restrict__ run_state,
                                              uint4* __restrict__ run_alias, const uint32_t* __restrict__ rid,
                                              uint32_t* __restrict__ run_f, const unsigned long long* num_runs,
                                              const uint32_t* __restrict__ drun,
                                              uint32_t* __restrict__ defer, uint32_t* defer_n,
                                              unsigned long long* stats, unsigned long long* stripes, uint32_t* err,
                                              uint32_t* errs, int restore, uint32_t* __restrict__ fast_blk,
                                              const uint32_t* errb_prev) {
  __shared__ uint32_t s_err, s_nr, s_cnt, s_list[256];
  // err may change while this kernel runs (other blocks): read it once per block
  if (threadIdx.x == 0) {
    s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (errb_prev ? *errb_prev : 0u);
    s_nr = (uint32_t)(*num_runs >> 32);  // runs of two or more (drun)
  }
  __syncthreads();
  const uint32_t lo = blk * 256, hi = min(lo + 256, s_nr);
  if (s_err || lo >= hi) return;
  refine_totals(b);
  uint32_t* ferr = P.isolate ? errs : err;  // descriptor-level failures: soft word with statuses
  // the dup-run list, compacted once more (a large bucket's hot-key run left
  // to its fallback path is empty)
  const uint32_t cnt =
      block_compact(lo, hi, s_list, &s_cnt, [&](uint32_t j) {
        const uint32_t r = drun[j];
        return run_end[r] - run_start[r] >= 2 || (run_flags[r] & RUN_ALIAS);  // (a multi-unit stem's groups: any size)
      });
  // Waves without a run leave at once (no block barrier after this point):
  // stats go wave by wave to this block's stripe (or straight to the output
  // past LDS_RULES rules), not through a block-wide LDS table.
  if ((threadIdx.x & ~63u) >= cnt) return;
  StatAcc acc{false, b.n_rules <= LDS_RULES && !restore
                         ? stripes + (size_t)(blk % STAT_STRIPES) * b.n_rules * RL_NUM_STATS : stats};
  LaneStats L;
  L.reset();
  if (threadIdx.x < cnt) {
    const uint32_t j = threadIdx.x;
    const uint32_t r = drun[s_list[j]];
    const uint32_t p = run_start[r], end = run_end[r];
    const uint32_t fl = run_flags[r];
    const Rec x0 = rec_s[p];
    const uint32_t e0 = svals[p];
    const uint64_t h0 = ((uint64_t)skeys[p] << 32) | x0.hlo;
    const uint32_t u0 = rec_unit(x0);
    SlotImg im;
    load_img_lo(&t.slots[h0 >> t.shift], im);  // home slot's first sector, in flight beside the stem
    const Key k0 = key_of(b, x0);
    if (fl & RUN_AHEAD) {
      // the groups of a stem seen under several units (k_split): set up together
      if (restore || alias_setup(t, P, rec_s, rid, run_start, run_end, run_flags, run_state, run_alias, run_f, fast_blk,
                                 res, svals, ferr, r, fl, u0, h0, k0, x0.now)) {
        if (((fl >> RUN_G_SHIFT) & 0xFFu) > 1) run_flags[r] = fl | RUN_MERGE;  // exact path: every group, merged
        defer[atomicAdd(defer_n, 1u)] = r;
      }
    } else if (fl & RUN_ALIAS) {
      // a later group of such a stem: its head's lane set it up
    } else if (!(fl & RUN_MULTI) && !(rec_flags(x0) & FLAG_SKIP)) {
      // (RUN_MULTI runs belong to the exact path (k_late); a run of one failed descriptor is done)
      const bool long_run = !restore && end - p >= LONG_RUN && !(fl & RUN_SLOW);
      bool ok = true;
      int64_t s0 = -1;
      bool ins = false;
      if (RL_ABL & 1) {
        s0 = (int64_t)(h0 >> t.shift);
      } else {
        s0 = find_slot_img(t, h0, slot_tag(h0, u0), k0, u0, &ins, im, ferr);
        if (s0 < 0) {
          ok = false;
        } else if (im.flags() & SLOT_EXACT) {
          ok = false;
        } else if (ins) {  // new (stem, unit): the stem must not exist under another unit
          for (uint32_t u = 1; u <= 4; u++) {
            bool dummy;
            const int64_t so = u == u0 ? -1 : find_slot(t, h0, slot_tag(h0, u), k0, u, false, &dummy, ferr);
            if (so >= 0) {  // multi-unit stem from now on: flag both before deferring
              t.slots[so].flags |= SLOT_EXACT;
              ok = false;
            }
          }
          if (!ok) t.slots[s0].flags |= SLOT_EXACT;
        }
      }
      const Elem el0 = load_elem(x0, e0, false);
      const Win cur = im.cur();
      // (a long run of a window older than the key's newest: replayed here, its
      // record lives in the history log)
      if (ok && long_run && (cur.ws == WS_INVALID || el0.w >= cur.ws)) {
        // Parallel path: pick the window record once; k_fast_* decide every element.
        Slot* s = &t.slots[s0];
        // the record of el0.w: cur, or a roll (the old cur to the history log
        // while a request could still ask for it: simple_pick)
        Win R = cur;
        if (cur.ws != el0.w) {
          R = Win{el0.w, 0, 0, 0};
          if (cur.ws != WS_INVALID && hist_keep(t, cur, el0.w, el0.d)) {
            const uint32_t head = log_append(t, (uint32_t)s0, slot_tag(h0, u0), im.ring(), el0.w, cur);
            s->cur = R;
            s->ring = head;
          } else {
            s->cur = R;
          }
        }
        // A record of window w was written inside w: its EXPIRE and local-cache
        // TTL both end at or after w + div, so they hold for the whole run.
        const uint32_t c0 = el0.now <= R.expire ? R.count : 0u;
        const uint32_t F = (P.lc_en && el0.now < R.lc) ? 1u : 0u;
        run_state[r] = make_uint4((uint32_t)s0, c0, R.lc, F);
        run_f[r] = 0xFFFFFFFFu;
        run_flags[r] = fl | RUN_FAST;
        // mark the 256-descriptor blocks of k_fast_emit this run spans
        const uint32_t b0 = p >> 8, b1 = (end - 1) >> 8;
        for (uint32_t w = b0 >> 5; w <= b1 >> 5; w++) {
          const uint32_t lo = w == (b0 >> 5) ? (b0 & 31) : 0u, hi = w == (b1 >> 5) ? (b1 & 31) : 31u;
          atomicOr(&fast_blk[w], (0xFFFFFFFFu >> (31 - hi)) & (0xFFFFFFFFu << lo));
        }
      } else if (ok) {
        if (RL_ABL & 2) {
          Slot* sl = &t.slots[s0];
          Win c = im.cur();
          c.count += end - p;
          sl->cur = c;
        } else {
          replay_simple(rec_s, svals, res, t, P, nullptr, p, end, 0, s0, im.cur(), im.ring(), slot_tag(h0, u0), x0, e0, L,
                        acc, ferr, restore);
        }
      } else if (s0 == SLOT_TABLE_FULL || s0 == SLOT_ARENA_FULL) {
        if (P.isolate) fail_range(res, svals, p, end, slot_fail_status(s0));  // else the batch fails
      } else if (s0 >= 0 && !restore && !(fl & (RUN_SLOW | RUN_NOWVAR)) && !(RL_ABL & 1)) {
        // a stem that lives under several units: the parallel path over every unit slot
        if (alias_setup(t, P, rec_s, rid, run_start, run_end, run_flags, run_state, run_alias, run_f, fast_blk, res,
                        svals, ferr, r, fl, u0, h0, k0, x0.now))
          defer[atomicAdd(defer_n, 1u)] = r;
      } else {
        defer[atomicAdd(defer_n, 1u)] = r;
      }
    }
  }
  if (!(RL_ABL & 4) && !restore) wave_flush(L, acc);
}

// ---- parallel path for long uniform runs (one stem, one unit, one window).
// Sequential replay of such a run is: count a_j = c0 + Σ_{k<=j} h_k; with the
// local cache on, the first element f with a_f > limit_f makes every element of
// a LATER request a local-cache hit (Set happens after request q_f's statuses),
// i.e. a suffix of the run, which therefore never increments.
__global__ __launch_bounds__(256) void k_fast_over(const uint32_t* sorted_n, SRec rec_s,
                                                   const uint32_t* __restrict__ segsum,
                                                   const uint32_t* __restrict__ rid,
                                                   const uint32_t* __restrict__ run_flags,
                                                   const uint4* __restrict__ run_state, uint32_t* __restrict__ run_f,
                                                   const uint32_t* err) {
  if (*err) return;
  const uint32_t n = *sorted_n;
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  bool cand = false;
  uint32_t r = 0;
  if (q < n) {
    r = rid[q];
    if (run_flags[r] & RUN_FAST) {
      const uint4 st = run_state[r];
      if (!(st.w & 5u)) cand = st.y + segsum[q] > rec_s[q].limit;  // (not for a local-cache hit or failed run)
    }
  }
  uint64_t pending = __ballot(cand);
  while (pending) {  // lowest candidate position per run in this wave
    const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)pending) - 1);
    const uint32_t rr = __shfl(r, leader);
    if (lane == leader) atomicMin(&run_f[rr], q);
    pending &= ~__ballot(cand && r == rr);
  }
}

__device__ __attribute__((always_inline)) inline void fast_emit_body(uint32_t blk, const uint32_t* sorted_n, uint32_t n_rules, TableDev t, Params P,
                                                   SRec rec_s, const uint32_t* __restrict__ svals,
                                                   unsigned long long* __restrict__ res,
                                                   const uint32_t* __restrict__ segsum,
                                                   const uint32_t* __restrict__ rid,
                                                   const uint32_t* __restrict__ run_start,
                                                   const uint32_t* __restrict__ run_end,
                                                   const uint32_t* __restrict__ run_flags,
                                                   const uint4* __restrict__ run_state,
                                                   const uint4* __restrict__ run_alias,
                                                   const uint32_t* __restrict__ run_f, unsigned long long* stats,
                                                   unsigned long long* stripes, const uint32_t* err,
                                                   const uint32_t* __restrict__ fast_blk, uint32_t* hint) {
  __shared__ uint32_t s_err, s_fast, s_n;
  __syncthreads();  // (grid-stride callers: the previous block's shared state has been read)
  if (threadIdx.x == 0) {
    s_err = *err;
    const uint32_t word = fast_blk[blk >> 5];
    s_fast = (word >> (blk & 31)) & 1u;
    s_n = *sorted_n;
    // the host's cue (one store per bitmap word): this batch had long runs
    if (hint && s_fast && (uint32_t)(__ffs(word) - 1) == (blk & 31)) *hint = 1u;
  }
  __syncthreads();
  if (s_err || !s_fast) return;  // no RUN_FAST descriptor in this block (k_table's bitmap)
  const uint32_t n = s_n;  // sorted positions of this batch
  const bool use_lds = n_rules <= LDS_RULES;
  stats_block_begin(use_lds, n_rules);
  StatAcc acc{use_lds, stats};
  LaneStats L;
  L.reset();
  const uint32_t q = blk * 256 + threadIdx.x;
  const uint32_t r = q < n ? rid[q] : 0u;
  const uint32_t fl = q < n ? run_flags[r] : 0u;
  if (fl & RUN_FAST) {
    const uint4 st = run_state[r];
    {
      const uint32_t f = run_f[r];
      const bool F = st.w & 1u;
      const Elem x = load_elem(rec_s[q], svals[q], false);
      uint32_t req_f = 0xFFFFFFFFu, lc_f = 0;
      if (P.lc_en && f != 0xFFFFFFFFu) {
        const Rec xf = rec_s[f];
        req_f = xf.req;
        lc_f = xf.now + div_of(rec_unit(xf));  // freecache Set with the over-limit descriptor's ttl
      }
      const bool masked = F || x.req > req_f;  // local-cache hit
      const uint32_t after = masked ? 0u : st.y + segsum[q];
      const Decision d = decide(after - x.h, after, masked && !x.shadow, x.h, x.thr, P.ratio, x.shadow, P.lc_en);
      emit(res, L, acc, x, d, masked);
      if (!masked) {
        const uint32_t nq = q + 1;
        // (the next element's request only matters below an over-limit one:
        // no gather of its record otherwise, e.g. every element with the local
        // cache off)
        const bool last = nq == run_end[r] || (req_f != 0xFFFFFFFFu && rec_s[nq].req > req_f);
        if (last && (fl & RUN_ALIAS)) {  // the key's records in every unit slot (alias_setup's targets)
          const uint4 sl = run_alias[r];
#pragma unroll
          for (uint32_t k = 0; k < 4; k++) {
            const uint32_t bits = (st.x >> (3 * k)) & 7u;
            if (!(bits & 3u)) continue;
            const uint32_t idx = k == 0 ? sl.x : k == 1 ? sl.y : k == 2 ? sl.z : sl.w;
            // a cur, or the new version alias_setup appended to the unit's history
            // log in this batch (no append of the batch overwrites it: log_append;
            // LOG_LOST when the log refused it: the window's later lookups fail)
            if ((bits & 2u) && (idx & LOG_POS_MASK) >= t.log_cap) continue;
            Win* R = (bits & 2u) ? &t.log[(size_t)(idx >> LOG_POS_BITS) * t.log_cap + (idx & LOG_POS_MASK)].w
                                 : &t.slots[idx].cur;
            if (bits & 4u) {  // same store: INCRBY + EXPIRE
              R->count = after;
              R->expire = x.now + x.d;
            }
            if (req_f != 0xFFFFFFFFu) R->lc = lc_f;
          }
        } else if (last) {  // the last INCRBY of the run leaves the key's state
          Win R;
          R.ws = x.w;
          R.count = after;
          R.expire = x.now + x.d;
          R.lc = (req_f != 0xFFFFFFFFu) ? lc_f : st.z;
          t.slots[st.x].cur = R;
        }
      }
    }
  }
  wave_flush(L, acc);
  stats_block_end(use_lds, n_rules, stripes);
}

// ---- k_runs_general: deferred runs (hash-prefix collisions, multi-unit
// stems, failed descriptors). Splits the run into its distinct stems by the
// full bytes (any number of them: correctness never depends on the hash; a
// secret hash key keeps the count small), then replays each stem exactly.
// Group g of run [p, end) is recorded in grp[q] for its positions; its first
// position in lead[p + g] and its units in gmask[p + g] (a run owns its range
// of these arrays).
constexpr uint32_t GRP_NONE = 0xFFFFFFFFu;

__device__ inline void fail_group(unsigned long long* res, const uint32_t* svals, const uint32_t* grp, uint32_t p,
                                  uint32_t end, uint32_t g, uint32_t st) {
  for (uint32_t q = p; q < end; q++)
    if (grp[q] == g) res[svals[q]] = pack_fail(st);
}

// Exact replay of one stem's descriptors over every unit slot it has (Redis
// keys shared across units: general_step). visit(f) calls f(Elem) for each of
// the stem's descriptors in arrival order.
template <typename Visit>
__device__ inline void stem_exact(const TableDev& t, const Params& P, unsigned long long* res, LaneStats& L,
                                  StatAcc& acc, uint32_t* ferr, int restore, uint64_t hs, const Key& stem, uint32_t um,
                                  Visit visit) {
  GeneralState G;
  G.present = 0;
  G.odirty = G.vdirty = G.cdirty = 0;
  G.cur_req = 0xFFFFFFFFu;
  G.npend = 0;
  int64_t fail = 0;
  for (uint32_t u = 1; u <= 4; u++) {
    bool ins;
    G.tag[u - 1] = slot_tag(hs, u);
    G.sidx[u - 1] = find_slot(t, hs, G.tag[u - 1], stem, u, (um >> (u - 1)) & 1, &ins, ferr);
    G.chain[u - 1] = LOG_NONE;
    G.old[u - 1] = G.vic[u - 1] = Win{WS_INVALID, 0, 0, 0};
    if (G.sidx[u - 1] >= 0) {
      const Slot& su = t.slots[G.sidx[u - 1]];
      G.present |= 1u << (u - 1);
      G.cur[u - 1] = su.cur;
      G.chain[u - 1] = su.ring;
    } else if ((um >> (u - 1)) & 1) {
      fail = G.sidx[u - 1];
    }
  }
  if (fail) {
    if (P.isolate) visit([&](const Elem& x) { res[x.e] = pack_fail(slot_fail_status(fail)); });
    return;
  }
  visit([&](const Elem& x) { general_step(t, P, res, L, acc, G, x, restore, ferr); });
  general_apply_pending(t, G);
  const uint8_t fl = __popc(G.present) >= 2 ? SLOT_EXACT : 0;
  for (uint32_t u = 0; u < 4; u++) {
    if (!(G.present >> u & 1)) continue;
    if ((G.vdirty >> u) & 1) gen_put(t, G, u, true);
    if ((G.odirty >> u) & 1) gen_put(t, G, u);
    Slot* s = &t.slots[G.sidx[u]];
    s->cur = G.cur[u];
    if ((G.cdirty >> u) & 1) s->ring = G.chain[u];
    s->flags |= fl;
  }
}

__device__ __attribute__((always_inline)) inline void general_body(uint32_t blk, uint32_t nblk, BatchDev b, TableDev t, Params P, SRec rec_s,
                                                      const uint32_t* __restrict__ skeys,
                                                      const uint32_t* __restrict__ svals,
                                                      unsigned long long* __restrict__ res,
                                                      const uint32_t* __restrict__ run_start,
                                                      const uint32_t* __restrict__ run_end,
                                                      const uint32_t* __restrict__ defer_a, const uint32_t* defer_a_n,
                                                      const uint32_t* __restrict__ defer_b, const uint32_t* defer_b_n,
                                                      uint32_t* __restrict__ grp, uint32_t* __restrict__ lead,
                                                      uint8_t* __restrict__ gmask, const uint32_t* __restrict__ keys0,
                                                      const uint32_t* __restrict__ defer1, const uint32_t* defer1_n,
                                                      const uint32_t* __restrict__ run_flags,
                                                      const uint32_t* __restrict__ rid,
                                                      unsigned long long* stats, unsigned long long* stripes,
                                                      uint32_t* err, uint32_t* errs, int restore) {
  __shared__ uint32_t s_err, s_na, s_n, s_n1;
  if (threadIdx.x == 0) {
    s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_na = *defer_a_n;
    s_n = s_na + *defer_b_n;
    s_n1 = defer1_n ? *defer1_n : 0u;
  }
  __syncthreads();
  if (s_err || (blk * 256 >= s_n && blk * 256 >= s_n1)) return;
  refine_totals(b);
  uint32_t* ferr = P.isolate ? errs : err;
  const bool use_lds = !restore && b.n_rules <= LDS_RULES;
  stats_block_begin(use_lds, b.n_rules);
  StatAcc acc{use_lds, stats};
  LaneStats L;
  L.reset();
  // Grid-stride over the deferred runs: the grid is small and fixed (deferrals
  // are rare), so an empty deferral list costs one short launch.
  for (uint32_t di = blk * 256 + threadIdx.x; di < s_n; di += nblk * 256) {
    const uint32_t rr = di < s_na ? defer_a[di] : defer_b[di - s_na];  // run id
    if (rr == DEFER_DONE) continue;  // split into ordinary runs (k_split)
    const uint32_t p = run_start[rr], end = run_end[rr];
    const uint32_t key = skeys[p];
    const uint32_t rfl = di < s_na ? 0u : run_flags[rr];  // (defer_a: RUN_MULTI runs as the bucket kernels left them)
    if (rfl & RUN_MERGE) {
      // the groups of one stem seen under several units (k_split ordered them
      // by Redis key): replayed exactly, merged back into arrival order
      constexpr uint32_t MG = 4;
      uint32_t cq[MG], ce[MG], um = (rfl >> RUN_UMASK_SHIFT) & 0xFu;
      const uint32_t G = min((rfl >> RUN_G_SHIFT) & 0xFFu, MG);
      cq[0] = p;
      ce[0] = end;
      for (uint32_t g = 1; g < G; g++) {
        const uint32_t id = rid[ce[g - 1]];
        cq[g] = run_start[id];
        ce[g] = run_end[id];
        um |= (run_flags[id] >> RUN_UMASK_SHIFT) & 0xFu;
      }
      const Rec y = rec_s[p];
      stem_exact(t, P, res, L, acc, ferr, restore, ((uint64_t)key << 32) | y.hlo, key_at(b, rec_s, p), um,
                 [&](auto&& f) {
                   for (;;) {
                     uint32_t bg = MG, be = 0xFFFFFFFFu;
                     for (uint32_t g = 0; g < G; g++)
                       if (cq[g] < ce[g] && svals[cq[g]] < be) {
                         be = svals[cq[g]];
                         bg = g;
                       }
                     if (bg == MG) break;
                     f(load_elem(rec_s[cq[bg]], be, restore));
                     cq[bg]++;
                   }
                 });
      continue;
    }
    // ---- split the run into distinct stems (hash, length, then bytes)
    uint32_t ng = 0;
    for (uint32_t q = p; q < end; q++) {
      const Rec x = rec_s[q];
      if (rec_flags(x) & FLAG_SKIP) {  // failed in validation: answered already
        grp[q] = GRP_NONE;
        continue;
      }
      const Key kx = key_of(b, x);
      uint32_t g = 0;
      for (; g < ng; g++) {
        const Rec y = rec_s[lead[p + g]];
        if (y.hlo == x.hlo && rec_len(y) == rec_len(x) && key_equal(key_of(b, y), kx)) break;
      }
      if (g == ng) {
        lead[p + ng] = q;
        gmask[p + ng] = 0;
        ng++;
      }
      grp[q] = g;
      gmask[p + g] |= (uint8_t)(1u << (rec_unit(x) - 1));
    }
    for (uint32_t g = 0; g < ng; g++) {
      const uint32_t q0 = lead[p + g], um = gmask[p + g];
      const Rec y = rec_s[q0];
      const Key stem = key_at(b, rec_s, q0);
      const uint64_t hs = ((uint64_t)key << 32) | y.hlo;
      // ---- resolve the slot(s)
      bool simple = false;
      int64_t s0 = -1;
      if (__popc(um) == 1) {
        const uint32_t u0 = __ffs(um);
        bool ins;
        s0 = find_slot(t, hs, slot_tag(hs, u0), stem, u0, true, &ins, ferr);
        if (s0 < 0) {
          if (P.isolate) fail_group(res, svals, grp, q0, end, g, slot_fail_status(s0));
          continue;
        }
        if (!(t.slots[s0].flags & SLOT_EXACT)) {
          simple = true;
          if (ins) {  // new (stem, unit): the stem must not exist under another unit
            for (uint32_t u = 1; u <= 4 && simple; u++) {
              bool dummy;
              if (u != u0 && find_slot(t, hs, slot_tag(hs, u), stem, u, false, &dummy, ferr) >= 0) simple = false;
            }
          }
        }
      }
      if (simple) {
        replay_simple(rec_s, svals, res, t, P, grp, q0, end, g, s0, t.slots[s0].cur, t.slots[s0].ring, slot_tag(hs, __ffs(um)), y,
                      svals[q0], L, acc, ferr,
                      restore);
        continue;
      }
      stem_exact(t, P, res, L, acc, ferr, restore, hs, stem, um, [&](auto&& f) {
        for (uint32_t q = q0; q < end; q++)
          if (grp[q] == g) f(load_elem(rec_s[q], svals[q], restore));
      });
    }
  }
  // keys seen once that k_table found under several units (arrival indices)
  for (uint32_t di = blk * 256 + threadIdx.x; di < s_n1; di += nblk * 256) {
    const uint32_t e = defer1[di];
    const Rec x = rec_s.rec[e];
    const uint64_t hs = ((uint64_t)keys0[e] << 32) | x.hlo;
    stem_exact(t, P, res, L, acc, ferr, restore, hs, key_of(b, x), 1u << (rec_unit(x) - 1),
               [&](auto&& f) { f(load_elem(x, e, restore)); });
  }
  if (!restore) wave_flush(L, acc);
  stats_block_end(use_lds, b.n_rules, stripes);
}

// ---- stage B grids. Each combines parts that touch disjoint stems, so they
// share the GPU instead of queueing one behind the other on the table stage's
// critical path.
//
// k_table: the runs of two or more (runs_body, blocks [0, g_runs)) and the keys
// seen once (unique_body, the rest).
// k_late's long-run part on a few workgroups (recent batches had no long
// runs): workgroup k of F reads 256 words of k_table's bitmap at once and walks
// only the marked blocks, so an empty bitmap costs one load per lane; a long
// run that does appear is still answered (and cues full grids for the next
// batches).
__device__ __attribute__((always_inline)) inline void late_scan(uint32_t k, uint32_t F, BatchDev b, TableDev t, Params P,
                                                   SRec rec_s, const uint32_t* __restrict__ svals,
                                                   unsigned long long* __restrict__ res,
                                                   const uint32_t* __restrict__ segsum, const uint32_t* __restrict__ rid,
                                                   const uint32_t* __restrict__ run_start,
                                                   const uint32_t* __restrict__ run_end,
                                                   const uint32_t* __restrict__ run_flags,
                                                   const uint4* __restrict__ run_state,
                                                   const uint4* __restrict__ run_alias, const uint32_t* __restrict__ run_f,
                                                   unsigned long long* stats, unsigned long long* stripes,
                                                   const uint32_t* err, const uint32_t* __restrict__ fast_blk,
                                                   const uint32_t* sorted_n, uint32_t* hint) {
  __shared__ uint32_t s_w[256], s_word[256], s_cnt;
  const uint32_t nw = (b.n + 256u * 32u - 1) / (256u * 32u);
  for (uint32_t w0 = k * 256; w0 < nw; w0 += F * 256) {
    __syncthreads();
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const uint32_t w = w0 + threadIdx.x;
    const uint32_t word = w < nw ? fast_blk[w] : 0u;
    if (word) {
      const uint32_t at = atomicAdd(&s_cnt, 1u);
      s_w[at] = w;
      s_word[at] = word;
    }
    __syncthreads();
    const uint32_t cnt = s_cnt;
    for (uint32_t j = 0; j < cnt; j++) {
      uint32_t bits = s_word[j];
      while (bits) {
        const uint32_t blk = s_w[j] * 32 + (uint32_t)(__ffs(bits) - 1);
        bits &= bits - 1;
        fast_emit_body(blk, sorted_n, b.n_rules, t, P, rec_s, svals, res, segsum, rid, run_start, run_end, run_flags,
                       run_state, run_alias, run_f, stats, stripes, err, fast_blk, hint);
      }
    }
  }
}

#ifndef RL_KT_UNIQ_FIRST
#define RL_KT_UNIQ_FIRST 0
#endif
#ifndef RL_KTABLE_WAVES
#define RL_KTABLE_WAVES 5  // waves per SIMD: <= 96 VGPRs (110 uncapped: 4 waves); 5 vs 1: C1 +1.2 %, C2 +0.8 %, C2U -0.3 %; 6 / 8 spill in the hot path: C1 -6 / -12 % (profiles/r05/ktable_waves)
#endif
__global__ __launch_bounds__(256, RL_KTABLE_WAVES) void k_table(uint32_t g_runs, BatchDev b, TableDev t, Params P, SRec rec_s,
                                               const uint32_t* __restrict__ skeys,
                                               const uint32_t* __restrict__ svals,
                                               unsigned long long* __restrict__ res,
                                               const uint32_t* __restrict__ run_start,
                                               const uint32_t* __restrict__ run_end, uint32_t* __restrict__ run_flags,
                                               uint4* __restrict__ run_state, uint4* __restrict__ run_alias,
                                               const uint32_t* __restrict__ rid, uint32_t* __restrict__ run_f,
                                               const unsigned long long* num_runs, const uint32_t* __restrict__ drun,
                                               uint32_t* __restrict__ defer2, uint32_t* defer2_n,
                                               const uint32_t* __restrict__ keys0, uint32_t* __restrict__ defer1,
                                               uint32_t* defer1_n, unsigned long long* stats,
                                               unsigned long long* stripes, uint32_t* err, uint32_t* errs, int restore,
                                               uint32_t* __restrict__ fast_blk, const uint2* __restrict__ uniq,
                                               const uint32_t* uniq_n, unsigned long long* __restrict__ kt,
                                               const uint32_t* errb_prev) {
  // kt (rl_profile on): each workgroup's start and end on the device's

  // constant clock, plain stores (one address for all of them serialised the
  // launch: +40 %); k_finish folds them into the launch's duration
  if (kt && threadIdx.x == 0) kt[2 * blockIdx.x] = wall_clock64();
  // early table-stage begin (errb_prev set): this batch's word holds its own
  // validation only; the previous batch's (final: the table order) is folded
  // in here, and every block checks both
  if (errb_prev && blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t p = *errb_prev;
    if (p) atomicOr(err, p);
  }
#if RL_KT_UNIQ_FIRST  // (A/B builds: the keys seen once take the grid's first workgroups, the runs part the last)
  const uint32_t g_uniq = gridDim.x - g_runs;
  if (blockIdx.x >= g_uniq)
    runs_body(blockIdx.x - g_uniq, b, t, P, rec_s, skeys, svals, res, run_start, run_end, run_flags, run_state,
              run_alias, rid, run_f, num_runs, drun, defer2, defer2_n, stats, stripes, err, errs, restore, fast_blk,
              errb_prev);
  else
    unique_body(blockIdx.x, b, t, P, rec_s.rec, keys0, uniq, uniq_n, res, defer1, defer1_n, stats, stripes, err, errs,
                restore, errb_prev);
#else
  if (blockIdx.x < g_runs)
    runs_body(blockIdx.x, b, t, P, rec_s, skeys, svals, res, run_start, run_end, run_flags, run_state, run_alias, rid,
              run_f, num_runs, drun, defer2, defer2_n, stats, stripes, err, errs, restore, fast_blk, errb_prev);
  else
    unique_body(blockIdx.x - g_runs, b, t, P, rec_s.rec, keys0, uniq, uniq_n, res, defer1, defer1_n, stats, stripes,
                err, errs, restore, errb_prev);
#endif
  if (kt && threadIdx.x == 0) kt[2 * blockIdx.x + 1] = wall_clock64();
}

// k_late (after k_table, and k_fast_over with the local cache on): the exact
// path (general_body, blocks [0, RUNS_GENERAL_LATE_BLOCKS): the RUN_MULTI runs
// k_split left (defer), the stems k_table found under several units in the
// table (defer2: its runs, defer1: keys seen once)) and the long runs'
// elements (fast_emit_body, the rest). They touch disjoint stems, and none of
// k_table's. (Until round 3 the RUN_MULTI runs had a launch of their own on a
// side stream beside k_table: 64 workgroups that k_finish waited for, 12% of
// kernel time at C1 for an all-but-empty list once k_split resolves it.) At least 8 waves per SIMD caps the grid at 64 VGPRs: the
// rare exact path spills to scratch instead of lowering the streaming part's
// occupancy (uncapped, the exact path's 88 VGPRs slowed the long-run part
// 55 -> 85 us at C2).
#ifndef RL_LATE_OCC
#define RL_LATE_OCC 8  // k_late's waves per SIMD (8: <= 64 VGPRs, the rare exact path spills; 6: the same, 4: C2 -7 %)
#endif
__global__ __launch_bounds__(256, RL_LATE_OCC) void k_late(BatchDev b, TableDev t, Params P, SRec rec_s,
                                                 const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ svals,
                                                 unsigned long long* __restrict__ res,
                                                 const uint32_t* __restrict__ run_start,
                                                 const uint32_t* __restrict__ run_end,
                                                 const uint32_t* __restrict__ defer, const uint32_t* defer_n,
                                                 const uint32_t* __restrict__ defer2, const uint32_t* defer2_n,
                                                 uint32_t* __restrict__ grp, uint32_t* __restrict__ lead,
                                                 uint8_t* __restrict__ gmask, const uint32_t* __restrict__ keys0,
                                                 const uint32_t* __restrict__ defer1, const uint32_t* defer1_n,
                                                 const uint32_t* __restrict__ segsum, const uint32_t* __restrict__ rid,
                                                 const uint32_t* __restrict__ run_flags,
                                                 const uint4* __restrict__ run_state,
                                                 const uint4* __restrict__ run_alias, const uint32_t* __restrict__ run_f,
                                                 unsigned long long* stats, unsigned long long* stripes, uint32_t* err,
                                                 uint32_t* errs, int restore, const uint32_t* __restrict__ fast_blk,
                                                 const uint32_t* sorted_n, uint32_t* hint, int scan) {
  if (blockIdx.x < RUNS_GENERAL_LATE_BLOCKS) {
    general_body(blockIdx.x, RUNS_GENERAL_LATE_BLOCKS, b, t, P, rec_s, skeys, svals, res, run_start, run_end, defer,
                 defer_n, defer2, defer2_n, grp, lead, gmask, keys0, defer1, defer1_n, run_flags, rid, stats, stripes,
                 err, errs, restore);
  } else if (restore) {
  } else if (!scan) {  // one workgroup per 256 sorted positions (grid-stride when the launch caps them)
    for (uint32_t blk = blockIdx.x - RUNS_GENERAL_LATE_BLOCKS; blk * 256 < b.n;
         blk += gridDim.x - RUNS_GENERAL_LATE_BLOCKS)
      fast_emit_body(blk, sorted_n, b.n_rules, t, P, rec_s, svals, res, segsum, rid, run_start, run_end, run_flags,
                     run_state, run_alias, run_f, stats, stripes, err, fast_blk, hint);
  } else {
    late_scan(blockIdx.x - RUNS_GENERAL_LATE_BLOCKS, gridDim.x - RUNS_GENERAL_LATE_BLOCKS, b, t, P, rec_s, svals, res,
              segsum, rid, run_start, run_end, run_flags, run_state, run_alias, run_f, stats, stripes, err, fast_blk,
              sorted_n, hint);
  }
}

// First kernel of the table stage: merge this batch's validation errors into
// the sticky table-stage word, clear k_table's deferral counters and this call's
// output stats (n_rules x RL_NUM_STATS).
__global__ __launch_bounds__(256) void k_b_begin(const uint32_t* __restrict__ erra, uint32_t* errb,
                                                 const uint32_t* errb_prev,
                                                 uint32_t* __restrict__ defer_n, uint32_t* __restrict__ defer1_n,
                                                 unsigned long long* __restrict__ stats, uint32_t m,
                                                 uint32_t* __restrict__ fast_blk, uint32_t nw,
                                                 const unsigned long long* log_ctr,
                                                 unsigned long long* __restrict__ log_epoch) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  // the history log's append counters now: at most their values when this
  // batch's table stage starts (early: at the end of its stage A, while
  // earlier batches may still append), so log_append's bound is the same or
  // stricter (one batch's appends never wrap a partition onto its own entries)
  if (log_ctr && i < LOG_PARTS)
    log_epoch[i] = __hip_atomic_load(log_ctr + (size_t)i * LOG_CTR_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (i == 0) {
    // this batch's table-stage word: the previous batch's (sticky: a failed
    // batch fails every later one) | this batch's validation result
    *errb = (errb_prev ? *errb_prev : 0u) | *erra;
    *defer_n = 0;
    *defer1_n = 0;
  }
  for (uint32_t j = i; j < m; j += gridDim.x * 256) stats[j] = 0;
  for (uint32_t j = i; j < nw; j += gridDim.x * 256) fast_blk[j] = 0;
}

// Last kernel of a batch: packed results -> the three rl_result arrays
// (arrival order, coalesced), and the first n_fold x RL_NUM_STATS threads fold
// the striped per-block stats into rl_result.stats (clearing the stripes even
// when the batch failed, so nothing leaks into the next one).
__global__ __launch_bounds__(256) void k_finish(const unsigned long long* __restrict__ res, uint32_t n, OutDev o,
                                                unsigned long long* __restrict__ stripes, uint32_t n_fold,
                                                const uint32_t* err, unsigned long long* lc_ctr,
                                                const unsigned long long* __restrict__ kt, uint32_t kt_n,
                                                unsigned long long* kt_acc, const OwnChunk own) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (kt && blockIdx.x == 0) {  // (rl_profile) k_table's duration: first workgroup start to last end
    __shared__ unsigned long long s_lo[256], s_hi[256];
    unsigned long long lo = ~0ull, hi = 0;
    for (uint32_t j = threadIdx.x; j < kt_n; j += 256) {
      lo = min(lo, kt[2 * j]);
      hi = max(hi, kt[2 * j + 1]);
    }
    s_lo[threadIdx.x] = lo;
    s_hi[threadIdx.x] = hi;
    __syncthreads();
    for (uint32_t w = 128; w; w >>= 1) {
      if (threadIdx.x < w) {
        s_lo[threadIdx.x] = min(s_lo[threadIdx.x], s_lo[threadIdx.x + w]);
        s_hi[threadIdx.x] = max(s_hi[threadIdx.x], s_hi[threadIdx.x + w]);
      }
      __syncthreads();
    }
    if (threadIdx.x == 0 && s_hi[0] > s_lo[0]) {
      atomicAdd(&kt_acc[0], s_hi[0] - s_lo[0]);
      atomicAdd(&kt_acc[1], 1ull);
    }
  }
  const bool ok = *err == 0;
  const uint32_t m = n_fold * RL_NUM_STATS;
  if (i < m) {
    unsigned long long s = 0;
    for (uint32_t k = 0; k < STAT_STRIPES; k++) {
      s += stripes[(size_t)k * m + i];
      stripes[(size_t)k * m + i] = 0;
    }
    if (ok) o.stats[i] += s;
  }
  bool hit = false;
  if (ok && i < n) {
    const unsigned long long v = res[i];
    if (o.code) {  // (routed owner batches keep the packed results only)
      o.code[i] = (uint8_t)res_code(v);
      o.rem[i] = res_rem(v);
      o.reset[i] = res_reset(v);
      if (o.status) o.status[i] = (uint8_t)res_status(v);
    }
    hit = res_lc_hit(v);
  }
  // a routed owner's own chunk: answered in place in the source batch's
  // outputs (k_route_scatter's work for these positions; a failed batch
  // answers its status for each)
  if (own.code && i < n && i - own.lo < own.n) {
    const unsigned long long v = ok ? res[i] : pack_fail(err_status(*err));
    const uint32_t e = own.idx[i - own.lo];
    own.code[e] = (uint8_t)res_code(v);
    own.rem[e] = res_rem(v);
    if (own.reset) own.reset[e] = res_reset(v);
    if (own.status) own.status[e] = (uint8_t)res_status(v);
    else if (own.src_err && res_status(v)) atomicOr(own.src_err, status_err(res_status(v)));
  }
  if (lc_ctr && ok) {  // freecache LookupCount / HitCount (local_cache_stats.go:36-43)
    const unsigned long long w = __ballot(hit);
    if ((threadIdx.x & 63u) == 0 && w) atomicAdd(&lc_ctr[1], (unsigned long long)__popcll(w));
    if (i == 0) atomicAdd(&lc_ctr[0], (unsigned long long)n);
  }
}

// Walk slot s's history chain: f(entry record, hop index) for each entry the
// log still holds, newest first (stops where one was overwritten, or when f says so).
template <typename F>
__device__ inline void chain_walk(const TableDev& t, uint32_t si, const Slot& s, F f) {
  uint32_t ptr = s.ring, tprev = s.cur.ws, saved = LOG_NONE, power = 1, lam = 0;
  for (uint32_t hops = 0; ptr != LOG_NONE && hops < LOG_MAX_HOPS && ptr != saved; hops++) {  // (log_find's checks)
    const uint32_t pos = ptr & LOG_POS_MASK;
    if (pos >= t.log_cap) return;
    if (++lam == power) {
      saved = ptr;
      power <<= 1;
      lam = 0;
    }
    const LogEnt& e = t.log[(size_t)(ptr >> LOG_POS_BITS) * t.log_cap + pos];
    if (e.slot != si || e.tag != s.tag || e.t_app > tprev) return;
    if (!f(e.w, hops)) return;
    tprev = e.t_app;
    ptr = e.prev;
  }
}

// Keys in the local over-limit cache at `now` (freecache EntryCount of live
// entries): window records whose local-cache TTL has not passed (the newest
// version of each window on a chain).
__global__ __launch_bounds__(256) void k_lc_count(const TableDev t, uint64_t nslots, uint32_t now,
                                                  unsigned long long* out) {
  uint32_t live = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * 256) {
    const Slot& s = t.slots[i];
    if (s.tag < 2) continue;
    live += s.cur.ws != WS_INVALID && now < s.cur.lc;
    chain_walk(t, (uint32_t)i, s, [&](const Win& w, uint32_t at) {
      if (w.ws == WS_INVALID || !(now < w.lc)) return true;
      bool newest = true;  // no newer entry of the same window before this one
      chain_walk(t, (uint32_t)i, s, [&](const Win& v, uint32_t at2) {
        if (at2 >= at) return false;
        if (v.ws == w.ws) newest = false;
        return newest;
      });
      live += newest;
      return true;
    });
  }
  if (live) atomicAdd(out, (unsigned long long)live);
}

// ===========================================================================
// Epoch sweep: a slot whose window records are all dead (Redis key past its
// EXPIRE and local-cache entry past its TTL) becomes a tombstone; its chain's
// log entries are left to be overwritten.
// ===========================================================================
__device__ inline bool win_alive(const Win& w, uint32_t now) {
  return w.ws != WS_INVALID && (now <= w.expire || now < w.lc);
}

__global__ __launch_bounds__(256) void k_sweep(TableDev t, uint64_t nslots, uint32_t now, unsigned long long* evicted) {
  uint32_t local = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * 256) {
    Slot* s = &t.slots[i];
    if (s->tag < 2) continue;
    bool alive = win_alive(s->cur, now);
    if (!alive)
      chain_walk(t, (uint32_t)i, *s, [&](const Win& w, uint32_t) {
        alive = win_alive(w, now);
        return !alive;
      });
    if (alive) continue;
    s->tag = TAG_TOMB;
    s->ring = LOG_NONE;
    local++;
  }
  if (local) atomicAdd(evicted, (unsigned long long)local);
}

// Long-stem arena compaction (rl_sweep, after k_sweep): every live slot's
// overflow bytes move to a fresh arena, packed from offset 0, so the space of
// swept slots is reclaimed. Order inside the new arena does not matter (a slot
// keeps its own offset), so a bump counter replaces a scan.
__global__ __launch_bounds__(256) void k_arena_compact(Slot* slots, uint64_t nslots, const uint8_t* __restrict__ from,
                                                       uint8_t* __restrict__ to, unsigned long long* used16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * 256) {
    Slot* s = &slots[i];
    if (s->tag < 2 || s->key_len <= KEY_IN) continue;
    uint32_t* sd = reinterpret_cast<uint32_t*>(s);
    const uint32_t n16 = (s->key_len - KEY_SPLIT + 15) / 16;
    const unsigned long long off = atomicAdd(used16, (unsigned long long)n16);
    const uint4* src = reinterpret_cast<const uint4*>(from + (size_t)sd[SLOT_EXT_DW] * 16);
    uint4* dst = reinterpret_cast<uint4*>(to + off * 16);
    for (uint32_t k = 0; k < n16; k++) dst[k] = src[k];
    sd[SLOT_EXT_DW] = (uint32_t)off;
  }
}

__global__ __launch_bounds__(256) void k_table_info(const Slot* slots, uint64_t nslots, unsigned long long* out) {
  uint32_t live = 0, tomb = 0, exact = 0, hist = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * 256) {
    const uint32_t tg = slots[i].tag;
    if (tg == TAG_TOMB) tomb++;
    else if (tg >= 2) {
      live++;
      exact += (slots[i].flags & SLOT_EXACT) != 0;
      hist += slots[i].ring != LOG_NONE;
    }
  }
  if (live) atomicAdd(&out[0], (unsigned long long)live);
  if (tomb) atomicAdd(&out[1], (unsigned long long)tomb);
  if (exact) atomicAdd(&out[2], (unsigned long long)exact);
  if (hist) atomicAdd(&out[3], (unsigned long long)hist);
}

// ===========================================================================
// Diagnostics
// ===========================================================================
// Full Redis key stem ‖ strconv.FormatInt((now/div)*div, 10) into a padded
// buffer: descriptor i writes at off[i] + 24*i, its length in klen[i].
__global__ __launch_bounds__(256) void k_debug_keys(BatchDev b, uint8_t* out, uint32_t* klen) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n) return;
  const uint32_t s0 = b.off[i], len = b.off[i + 1] - s0;
  uint8_t* dst = out + s0 + 24ull * i;
  for (uint32_t j = 0; j < len; j++) dst[j] = b.stem[s0 + j];
  const uint32_t now = (uint32_t)b.now[b.req[i]];
  const uint32_t d = div_of(b.unit[i]);
  uint32_t ws = now / d * d;
  uint8_t tmp[12];
  uint32_t nd = 0;
  do { tmp[nd++] = (uint8_t)('0' + ws % 10); ws /= 10; } while (ws);
  for (uint32_t j = 0; j < nd; j++) dst[len + j] = tmp[nd - 1 - j];
  klen[i] = len + nd;
}

__global__ __launch_bounds__(256) void k_debug_decide(uint32_t n, const uint32_t* before, const uint32_t* after,
                                                      const uint8_t* lc_hit, const uint32_t* hits,
                                                      const uint32_t* limit, const uint8_t* unit,
                                                      const uint8_t* flags, const int64_t* now, float ratio,
                                                      int lc_en, uint8_t* code, uint32_t* rem, uint32_t* reset,
                                                      unsigned long long* deltas, uint8_t* lc_set) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const bool shadow = flags[i] & RL_FLAG_SHADOW;
  const Decision r = decide(before[i], after[i], lc_hit[i] != 0, hits[i], limit[i], ratio, shadow, lc_en != 0);
  code[i] = r.code;
  rem[i] = r.remaining;
  const uint32_t d = div_of(unit[i]);
  reset[i] = d - (uint32_t)(now[i] % d);
  unsigned long long* s = deltas + (size_t)i * RL_NUM_STATS;
  s[RL_STAT_TOTAL_HITS] = 0;  // TotalHits is counted in GenerateCacheKeys, not here
  s[RL_STAT_OVER_LIMIT] = r.d_over;
  s[RL_STAT_NEAR_LIMIT] = r.d_near;
  s[RL_STAT_OVER_LIMIT_WITH_LOCAL_CACHE] = r.d_lc;
  s[RL_STAT_WITHIN_LIMIT] = r.d_within;
  s[RL_STAT_SHADOW_MODE] = r.d_shadow;
  lc_set[i] = r.set_lc;
}

// ===========================================================================
// Launch wrappers
// ===========================================================================
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Stage A (table-free): validate, hash, sort, segment, and mark the descriptors
// whose sort key occurs more than once. Uses only this buffer's scratch and its
// validation word s.err. Sorted keys go to keys[1] (keys[0] keeps the arrival
// order for k_table's keys seen once), the sort permutation to vals[0].
void launch_stage_a(const BatchDev& b, const Scratch& s, int isolate, int per_second, hipStream_t st,
                    hipEvent_t* ev, uint32_t* long_hint, bool long_kernel, uint32_t* big_hint, bool big_full) {
  const uint32_t g0 = cdiv(b.n > b.n_req ? b.n : b.n_req, 256);
  if (ev) (void)hipEventRecord(ev[0], st);
  if (g0)
    k_prepare<<<g0, 256, 0, st>>>(b, s.rec, s.keys[0], s.err, s.errs, isolate, s.time_floor, s.defer_n, s.big_n,
                                  s.work_n, s.run_flags, s.runs64, s.hit_a, s.res, s.sorted_n, s.uniq_n);
  if (ev) (void)hipEventRecord(ev[1], st);
  const uint32_t ptiles = cdiv(b.n, PART_TILE);
  if (b.n)
    k_part<<<ptiles, 256, 0, st>>>(s.keys[0], b.wire ? s.hit_a : b.hits, s.tile, b.n, ptiles, s.part_info, s.err);
  if (ev) (void)hipEventRecord(ev[2], st);
  if (b.n) {
    const size_t seg_lds = (2ull * ptiles + 1) * 4;
    k_bucket<<<PART_DIGITS, BkSmall::THREADS, seg_lds, st>>>(s.tile, s.part_info, ptiles,
                                                             s.keys[1], s.vals[0], s.hits_s, s.segsum, s.rid,
                                                             s.run_start, s.run_end, s.runs64, s.drun, s.big_meta, s.big_n,
                                                             s.big_work, s.work_n, s.sorted_n, s.uniq, s.uniq_n,
                                                             s.err, big_hint);
#ifndef RL_EXP_NO_BIG  // (measurement builds only: without the large-bucket kernels, C1 has none)
    const uint32_t gi = big_full ? BIG_ITEM_BLOCKS : 1u, gb = big_full ? BIG_BLOCKS : 1u;
    k_big_count<<<gi, BkSmall::THREADS, seg_lds, st>>>(s.tile, s.part_info, ptiles,
                                                                    s.big_meta, s.big_work, s.work_n, s.big_cnt,
                                                                    s.err);
    k_big_place<<<gi, BkSmall::THREADS, seg_lds, st>>>(
        s.tile, s.part_info, ptiles, s.big_meta, s.big_work, s.work_n, s.big_cnt, s.keys[1],
        s.vals[0], s.hits_s, s.segsum, s.rid, s.run_start, s.run_end, s.drun, s.err);
    k_bucket_big<<<gb, BkBig::THREADS, seg_lds, st>>>(s.tile, s.part_info, ptiles,
                                                              s.keys[1], s.vals[0], s.hits_s, s.hit_t, s.segsum,
                                                              s.rid, s.run_start, s.run_end, s.runs64, s.drun, s.big_meta,
                                                              s.big_n, s.big_cnt, s.err);
#endif
    k_run_check<<<cdiv(b.n, RC_CHUNK), 256, 0, st>>>(b, SRec{s.rec, s.vals[0]}, s.keys[1], s.rid, s.run_start,
                                                s.run_end, s.run_flags, s.defer, s.defer_n, s.err, s.runs64, s.split,
                                                s.sorted_n, s.grp, s.hit_t, s.uniq, s.uniq_n, s.long_runs, s.keys[0]);
#ifndef RL_EXP_NO_SPLIT  // (measurement builds only: C1 defers no run to k_split)
    k_split<<<SPLIT_BLOCKS, SPLIT_THREADS, 0, st>>>(b, SRec{s.rec, s.vals[0]}, s.vals[0], s.segsum, s.rid, s.run_start,
                                          s.run_end, s.run_flags, s.defer, s.defer_n, s.runs64, s.split, s.drun,
                                          b.n / 2 + BIG_HEAVY * PART_DIGITS, s.grp, s.lead, s.hit_t, s.vals[1], s.err,
                                          per_second, UniqList{s.uniq, s.uniq_n, s.keys[1], s.keys[0]}, s.long_runs, long_hint,
                                          long_kernel ? 1 : 0);
#endif
#if RL_SPLIT_LONG_THREADS
    if (long_kernel)
      k_split_long<<<RL_SPLIT_LONG_BLOCKS, RL_SPLIT_LONG_THREADS, 0, st>>>(
          b, SRec{s.rec, s.vals[0]}, s.vals[0], s.segsum, s.rid, s.run_start, s.run_end, s.run_flags, s.defer,
          s.runs64, s.split, s.drun, b.n / 2 + BIG_HEAVY * PART_DIGITS, s.grp, s.lead, s.hit_t, s.vals[1], s.err,
          per_second, UniqList{s.uniq, s.uniq_n, s.keys[1], s.keys[0]}, s.long_runs);
#endif
  }
}

// Stage B (the table): runs strictly in batch order. Every kernel reads the
// sticky table-stage word s.errb; k_b_begin folds this batch's validation
// result into it first. The keys seen once and the sorted path (runs
// and its exact / parallel companions) touch disjoint stems.
#ifndef RL_LATE_FAST_BLOCKS
#define RL_LATE_FAST_BLOCKS 0  // cap on k_late's long-run workgroups (0: one per 256 descriptors)
#endif
constexpr uint32_t LATE_SCAN_BLOCKS = 4;  // k_late's long-run workgroups while recent batches had none
// The table stage's first kernel, early (before the table-order wait, at the
// end of stage A): this batch's table-stage word = its own validation, its
// deferral counters, block bitmap and output stats cleared. k_table folds the
// previous batch's word in (launch_stage_b with early set).
void launch_b_begin_early(const BatchDev& b, const OutDev& o, const Scratch& s, int restore, hipStream_t st,
                          const unsigned long long* log_ctr) {
  const uint32_t m = restore ? 0u : b.n_rules * RL_NUM_STATS;
  const uint32_t gb = m ? (cdiv(m, 256) < 64 ? cdiv(m, 256) : 64) : 1;
  k_b_begin<<<gb, 256, 0, st>>>(s.err, s.errb, nullptr, s.defer2_n, s.defer1_n, o.stats, m, s.fast_blk,
                                cdiv(b.n, 256 * 32), log_ctr, s.log_epoch);
}

void launch_stage_b(const BatchDev& b, const OutDev& o, const TableDev& t, const Params& P, const Scratch& s,
                    int restore, hipStream_t st, hipEvent_t* ev, const uint32_t* errb_prev, hipEvent_t table_done,
                    unsigned long long* kt_acc, bool early, uint32_t* late_hint, bool late_full) {
  const uint32_t m = restore ? 0u : b.n_rules * RL_NUM_STATS;
  const uint32_t gb = m ? (cdiv(m, 256) < 64 ? cdiv(m, 256) : 64) : 1;
  if (!early)
    k_b_begin<<<gb, 256, 0, st>>>(s.err, s.errb, errb_prev, s.defer2_n, s.defer1_n, o.stats, m, s.fast_blk,
                                  cdiv(b.n, 256 * 32), t.log_ctr, s.log_epoch);
  else if (!b.n)  // (no k_table to fold the previous batch's word in)
    k_b_begin<<<1, 256, 0, st>>>(s.errb, s.errb, errb_prev, s.defer2_n, s.defer1_n, o.stats, 0, s.fast_blk, 0,
                                 nullptr, nullptr);
  if (b.n) {
    const uint32_t g = cdiv(b.n, 256);
    const size_t lds = (!restore && b.n_rules <= LDS_RULES) ? (size_t)b.n_rules * RL_NUM_STATS * 8 : 0;
    const SRec rs{s.rec, s.vals[0]};
    // k_table (the runs of two or more and the keys seen once), then k_late
    // (the exact path and the long runs' elements): grids whose parts touch
    // disjoint stems.
    if (ev) (void)hipEventRecord(ev[3], st);
    const uint32_t g_runs = cdiv(b.n / 2 + BIG_HEAVY * PART_DIGITS, 256);
    k_table<<<g_runs + g, 256, lds, st>>>(g_runs, b, t, P, rs, s.keys[1], s.vals[0], s.res, s.run_start, s.run_end,
                                         s.run_flags, s.run_state, s.run_alias, s.rid, s.run_f, s.runs64, s.drun,
                                         s.defer2, s.defer2_n,
                                         s.keys[0], s.defer1, s.defer1_n, o.stats, s.stripes, s.errb, s.errs, restore,
                                         s.fast_blk, s.uniq, s.uniq_n, kt_acc ? s.kt_blk : nullptr,
                                         early ? errb_prev : nullptr);
    if (ev) (void)hipEventRecord(ev[4], st);
    if (!restore && P.lc_en)
      k_fast_over<<<g, 256, 0, st>>>(s.sorted_n, rs, s.segsum, s.rid, s.run_flags, s.run_state, s.run_f, s.errb);
#ifndef RL_EXP_NO_LATE  // (measurement builds only: C1 leaves k_late nothing to do)
    // its long-run part: one workgroup per 256 sorted positions while recent
    // batches had long runs (C2, C2U), else LATE_SCAN_BLOCKS walking the bitmap
    const uint32_t gl = restore ? 0u : !late_full ? LATE_SCAN_BLOCKS
                                     : (RL_LATE_FAST_BLOCKS && g > RL_LATE_FAST_BLOCKS ? RL_LATE_FAST_BLOCKS : g);
    k_late<<<RUNS_GENERAL_LATE_BLOCKS + gl, 256, lds, st>>>(
        b, t, P, rs, s.keys[1], s.vals[0], s.res, s.run_start, s.run_end, s.defer, s.defer_n, s.defer2, s.defer2_n,
        s.grp, s.lead, s.gmask,
        s.keys[0], s.defer1, s.defer1_n, s.segsum, s.rid, s.run_flags, s.run_state, s.run_alias, s.run_f, o.stats,
        s.stripes, s.errb,
        s.errs, restore, s.fast_blk, s.sorted_n, late_hint, late_full ? 0 : 1);
#endif
    if (table_done) (void)hipEventRecord(table_done, st);
    if (!restore) {
      const uint32_t nf = b.n_rules <= LDS_RULES ? b.n_rules : 0u;
      const uint32_t gf = cdiv(nf * RL_NUM_STATS > b.n ? nf * RL_NUM_STATS : b.n, 256);
      k_finish<<<gf, 256, 0, st>>>(s.res, b.n, o, s.stripes, nf, s.errb, P.lc_en ? s.counters + 5 : nullptr,
                                   kt_acc ? s.kt_blk : nullptr, g_runs + g, kt_acc, b.own);
    }
  } else {
    if (ev) {
      (void)hipEventRecord(ev[3], st);
      (void)hipEventRecord(ev[4], st);
    }
    if (table_done) (void)hipEventRecord(table_done, st);
  }
  if (ev) (void)hipEventRecord(ev[5], st);
}


void launch_sweep(const TableDev& t, uint64_t nslots, uint32_t now, unsigned long long* evicted, hipStream_t st) {
  k_sweep<<<2048, 256, 0, st>>>(t, nslots, now, evicted);
}

void launch_arena_compact(Slot* slots, uint64_t nslots, const uint8_t* from, uint8_t* to, unsigned long long* used16,
                          hipStream_t st) {
  k_arena_compact<<<2048, 256, 0, st>>>(slots, nslots, from, to, used16);
}

void launch_lc_count(const TableDev& t, uint64_t nslots, uint32_t now, unsigned long long* out, hipStream_t st) {
  k_lc_count<<<2048, 256, 0, st>>>(t, nslots, now, out);
}

void launch_table_info(const Slot* slots, uint64_t nslots, unsigned long long* out, hipStream_t st) {
  k_table_info<<<2048, 256, 0, st>>>(slots, nslots, out);
}

bool log_tear_hook() { return RL_LOG_TEAR != 0; }

void launch_debug_keys(const BatchDev& b, uint8_t* out, uint32_t* klen, hipStream_t st) {
  if (b.n) k_debug_keys<<<cdiv(b.n, 256), 256, 0, st>>>(b, out, klen);
}

void launch_debug_decide(uint32_t n, const uint32_t* before, const uint32_t* after, const uint8_t* lc_hit,
                         const uint32_t* hits, const uint32_t* limit, const uint8_t* unit, const uint8_t* flags,
                         const int64_t* now, float ratio, int lc_en, uint8_t* code, uint32_t* rem, uint32_t* reset,
                         unsigned long long* deltas, uint8_t* lc_set, hipStream_t st) {
  if (n)
    k_debug_decide<<<cdiv(n, 256), 256, 0, st>>>(n, before, after, lc_hit, hits, limit, unit, flags, now, ratio,
                                                 lc_en, code, rem, reset, deltas, lc_set);
}

}  // namespace rl
