// rl_route.hip — multi-GPU routing of a batch to the GPUs that own its keys
// (hash-sharded table). The exchange itself is driven by
// rl_comm.hip (RCCL send/recv inside the library), rl_api.hip (shards of one
// ctx: peer copies) or ratelimit_amd/sharded.py (collectives from Python);
// these kernels are the device-side halves around it:
//
//   source: hash -> owner, stable partition by owner, 32-B wire records +
//           stem bytes in owner order (k_rp_count / k_rp_scan / k_rp_pack);
//   owner:  the received chunks (concatenated in source-rank order = global
//           arrival order) feed the normal DoLimit pipeline directly: its
//           k_prepare reads the wire records (BatchDev.wire);
//           k_route_ret hands the packed results (or the batch's failure) back;
//   source: scatter the returned packed results to arrival order.
//
// Owner of a stem = (low 32 bits of its 64-bit hash x n_shards) >> 32: the
// table's home slot uses the top bits, so the two are independent.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_device.h"
#include "rl_kernels.h"

namespace rl {

namespace {

inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

__device__ inline uint32_t owner_of(uint64_t h, uint32_t n_shards) {
  return (uint32_t)(((uint64_t)(uint32_t)h * n_shards) >> 32);
}

// ---- source side ----------------------------------------------------------
// Partition of a slice by owner, in three launches over tiles of RP_TILE
// descriptors (all HBM-streaming; the byte moves go through LDS):
//   k_rp_count  keyed stem hash (kept for the wire record: owners never
//               rehash; no stem offset: owners scan the lengths) -> owner per descriptor (dest, u8), per-tile record
//               and stem-byte counts per owner;
//   k_rp_scan   per owner: exclusive scan of the tile counts, the totals
//               (= the exchange counts);
//   k_rp_pack   stable rank of each descriptor inside its tile and owner
//               (wave ballots), its 32-B wire record and perm entry, and its
//               stem bytes staged in LDS so that each owner's run of stems
//               leaves the tile as whole dwords.
#ifndef RL_RP_ABL
#define RL_RP_ABL 0  // measurement builds: 1 = no stem moves, 2 = no record stores
#endif
constexpr uint32_t RP_ITEMS = 2;
constexpr uint32_t RP_TILE = 256 * RP_ITEMS;
static_assert(RP_TILE == ROUTE_TILE, "scratch sizing");
constexpr uint32_t RP_WAVE = RP_TILE / 4;       // consecutive descriptors per wave
constexpr uint32_t RP_STAGE = 24 * 1024;        // LDS bytes for a tile's stems (else direct byte copies)

__device__ inline uint32_t lane_id() { return threadIdx.x & 63u; }

// Inclusive prefix sum over the 64 lanes of a wave.
__device__ inline uint32_t wave_incl(uint32_t v) {
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o, 64);
    if (lane_id() >= o) v += y;
  }
  return v;
}

// Exclusive prefix over the NW x 64 threads of a block of (a, b); returns the
// block totals. tmp: 2 x NW shared words.
template <uint32_t NW>
__device__ inline void block_excl2(uint32_t& a, uint32_t& b, uint32_t& ta, uint32_t& tb, uint32_t* tmp) {
  const uint32_t ia = wave_incl(a), ib = wave_incl(b), w = threadIdx.x >> 6;
  if (lane_id() == 63) {
    tmp[w] = ia;
    tmp[NW + w] = ib;
  }
  __syncthreads();
  uint32_t pa = 0, pb = 0;
  ta = tb = 0;
#pragma unroll
  for (uint32_t k = 0; k < NW; k++) {
    const uint32_t xa = tmp[k], xb = tmp[NW + k];
    if (k < w) {
      pa += xa;
      pb += xb;
    }
    ta += xa;
    tb += xb;
  }
  a = pa + ia - a;
  b = pb + ib - b;
  __syncthreads();
}

// A descriptor the partition cannot route: malformed layout only (a bad
// unit, rule id or clock is the owner's to judge).
__device__ inline bool rp_bad(const BatchDev& b, uint32_t i, uint32_t total) {
  const uint32_t s0 = b.off[i], s1 = b.off[i + 1], q = b.req[i];
  return q >= ROUTE_MAX_REQ || (i && b.req[i - 1] > q) || s1 <= s0 || s1 - s0 > 65535 || total > b.stem_cap ||
         s1 > total || q >= b.n_req;
}

__global__ __launch_bounds__(256) void k_rp_count(BatchDev b, uint32_t n_shards, uint32_t ntiles, uint32_t own_rank,
                                                  uint8_t* __restrict__ dest, unsigned long long* __restrict__ hash,
                                                  uint32_t* __restrict__ hist, uint32_t* err) {
  __shared__ uint32_t cr[RL_MAX_SHARDS], cb[RL_MAX_SHARDS];
  for (uint32_t d = threadIdx.x; d < n_shards; d += 256) cr[d] = cb[d] = 0;
  __syncthreads();
  const uint32_t total = b.off[b.n];
  const uint32_t* words = reinterpret_cast<const uint32_t*>(b.stem);
  const uint32_t nw = (total + 3u) >> 2;
  bool bad = false;
#pragma unroll
  for (uint32_t t = 0; t < RP_ITEMS; t++) {
    const uint32_t i = blockIdx.x * RP_TILE + t * 256 + threadIdx.x;
    const bool valid = i < b.n;
    uint32_t d = 0, len = 0;
    if (valid) {
      if (rp_bad(b, i, total)) {
        bad = true;
      } else {
        const uint32_t s0 = b.off[i];
        len = b.off[i + 1] - s0;
        const uint64_t h = hash_stem(b.hk, DwordReader{words + (s0 >> 2), nw - (s0 >> 2)}, s0 & 3u, len);
        d = owner_of(h, n_shards);
        hash[i] = h;
        if (d == own_rank) len = 0;  // (the own chunk's stems stay in place: no bytes sent)
      }
      dest[i] = (uint8_t)d;
    }
    // one LDS add per owner present in the wave (few owners: few adds)
    uint64_t todo = __ballot(valid);
    while (todo) {
      const uint32_t leader = __ffsll((unsigned long long)todo) - 1;
      const uint32_t dl = __shfl(d, leader, 64);
      const bool mine = valid && d == dl;
      const uint64_t mask = __ballot(mine);
      const uint32_t bytes = wave_incl(mine ? len : 0u);
      if (lane_id() == 63) {
        atomicAdd(&cr[dl], (uint32_t)__popcll(mask));
        atomicAdd(&cb[dl], bytes);
      }
      todo &= ~mask;
    }
  }
  if (bad) atomicOr(err, ERR_INVALID);
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < n_shards; d += 256) {
    hist[(size_t)d * ntiles + blockIdx.x] = cr[d];
    hist[((size_t)n_shards + d) * ntiles + blockIdx.x] = cb[d];
  }
}

// One block per owner d: exclusive scans of its row of tile counts (records,
// bytes); counts[cstride d], [cstride d + 1] = the totals (zero when the slice
// is malformed, so the exchange stays well-formed); tot[d], tot[n_shards + d]
// too.
// (256 lanes: a workgroup of 1024 waits longer for a whole CU beside the
// owner pipeline's kernels: 19 us in flight per batch at N = 1)
__global__ __launch_bounds__(256) void k_rp_scan(uint32_t* __restrict__ hist, uint32_t n_shards, uint32_t ntiles,
                                                  unsigned long long* __restrict__ counts, uint32_t cstride,
                                                  unsigned long long meta0, unsigned long long meta1,
                                                  uint32_t* __restrict__ tot, const uint32_t* err,
                                                  unsigned long long* counts_host) {
  __shared__ uint32_t tmp[32];
  const uint32_t d = blockIdx.x;
  uint32_t* rr = hist + (size_t)d * ntiles;
  uint32_t* rb = hist + ((size_t)n_shards + d) * ntiles;
  uint32_t ca = 0, cb = 0;
  for (uint32_t base = 0; base < ntiles; base += 256) {
    const uint32_t j = base + threadIdx.x;
    uint32_t a = j < ntiles ? rr[j] : 0u, bb = j < ntiles ? rb[j] : 0u, ta, tb;
    block_excl2<4>(a, bb, ta, tb, tmp);
    if (j < ntiles) {
      rr[j] = ca + a;
      rb[j] = cb + bb;
    }
    ca += ta;
    cb += tb;
  }
  if (threadIdx.x == 0) {
    const bool ok = *err == 0;
    for (unsigned long long* c : {counts, counts_host}) {  // (the host's copy: stores to page-locked memory)
      if (!c) continue;
      c[(size_t)cstride * d] = ok ? ca : 0u;
      c[(size_t)cstride * d + 1] = ok ? cb : 0u;
      if (cstride >= 4) {  // (the in-library router's counts message: n_rules, flags)
        c[(size_t)cstride * d + 2] = meta0;
        c[(size_t)cstride * d + 3] = meta1;
      }
    }
    tot[d] = ca;
    tot[n_shards + d] = cb;
  }
}

__global__ __launch_bounds__(256) void k_rp_pack(BatchDev b, uint32_t n_shards, uint32_t ntiles, uint32_t src_rank,
                                                 uint32_t own_rank,
                                                 const uint8_t* __restrict__ dest,
                                                 const unsigned long long* __restrict__ hash,
                                                 const uint32_t* __restrict__ hist,
                                                 const uint32_t* __restrict__ tot, Wire* __restrict__ out,
                                                 uint8_t* __restrict__ out_stem, uint32_t* __restrict__ perm,
                                                 const uint32_t* err) {
  __shared__ uint32_t wr[4][RL_MAX_SHARDS], wb[4][RL_MAX_SHARDS];  // per wave, then wave bases
  __shared__ uint32_t gr[RL_MAX_SHARDS], gb[RL_MAX_SHARDS];        // tile's first record / chunk byte per owner
  __shared__ uint32_t sb[RL_MAX_SHARDS], lo[RL_MAX_SHARDS], tb[RL_MAX_SHARDS];
  __shared__ uint32_t tmp[8];
  __shared__ uint32_t stage32[RP_STAGE / 4];
  uint8_t* stage = reinterpret_cast<uint8_t*>(stage32);
  if (*err) return;
  const uint32_t tile = blockIdx.x, w = threadIdx.x >> 6, lane = lane_id();
  for (uint32_t d = threadIdx.x; d < n_shards; d += 256) {
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) wr[k][d] = wb[k][d] = 0;
  }
  // owners' first record (global) and stem byte (send buffer): exclusive
  // scans of the totals over owners
  {
    uint32_t ra = 0, rb = 0, sa = 0, sbb = 0;
    const uint32_t d = threadIdx.x;  // (n_shards <= 256)
    if (d < n_shards) {
      ra = tot[d];
      rb = tot[n_shards + d];
    }
    sa = ra;
    sbb = rb;
    uint32_t ta, tbb;
    block_excl2<4>(sa, sbb, ta, tbb, tmp);
    if (d < n_shards) {
      gr[d] = sa + hist[(size_t)d * ntiles + tile];
      sb[d] = sbb;
      gb[d] = hist[((size_t)n_shards + d) * ntiles + tile];
    }
  }
  __syncthreads();
  // stable rank inside (tile, owner): wave w takes RP_WAVE consecutive
  // descriptors, 64 per round, grouping lanes by owner with ballots
  const uint32_t i0 = tile * RP_TILE + w * RP_WAVE;
  uint32_t my_d[RP_ITEMS], my_r[RP_ITEMS], my_b[RP_ITEMS], my_len[RP_ITEMS];
  const uint64_t lt = (lane ? ~0ull >> (64 - lane) : 0ull);
#pragma unroll
  for (uint32_t t = 0; t < RP_ITEMS; t++) {
    const uint32_t i = i0 + t * 64 + lane;
    const bool valid = i < b.n;
    const uint32_t d = valid ? dest[i] : 0xFFFFu;
    const uint32_t len = valid && d != own_rank ? b.off[i + 1] - b.off[i] : 0u;
    uint64_t todo = __ballot(valid);
    uint32_t r = 0, bp = 0;
    while (todo) {
      const uint32_t leader = __ffsll((unsigned long long)todo) - 1;
      const uint32_t dl = __shfl(d, leader, 64);
      const bool mine = valid && d == dl;
      const uint64_t mask = __ballot(mine);
      const uint32_t incl = wave_incl(mine ? len : 0u);
      const uint32_t gbytes = __shfl(incl, 63, 64);
      const uint32_t br = wr[w][dl], bb = wb[w][dl];  // (one wave: read before the leader's update)
      if (mine) {
        r = br + (uint32_t)__popcll(mask & lt);
        bp = bb + incl - len;
      }
      if (lane == leader) {
        wr[w][dl] = br + (uint32_t)__popcll(mask);
        wb[w][dl] = bb + gbytes;
      }
      todo &= ~mask;
    }
    my_d[t] = d;
    my_r[t] = r;
    my_b[t] = bp;
    my_len[t] = len;
  }
  __syncthreads();
  // wave bases inside the tile, the tile's bytes per owner, LDS segments
  {
    const uint32_t d = threadIdx.x;
    uint32_t byt = 0;
    if (d < n_shards) {
      uint32_t ar = 0, ab = 0;
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t xr = wr[k][d], xb = wb[k][d];
        wr[k][d] = ar;
        wb[k][d] = ab;
        ar += xr;
        ab += xb;
      }
      tb[d] = ab;
      byt = ab ? ab + 3u : 0u;  // (room to align the segment, below)
    }
    uint32_t dummy = 0, t1, t2;
    block_excl2<4>(byt, dummy, t1, t2, tmp);
    // owner d's LDS segment starts at the same offset mod 4 as its bytes in
    // the send buffer (sb + gb), so the segment leaves as aligned dwords
    if (d < n_shards) lo[d] = byt + ((sb[d] + gb[d] - byt) & 3u);
    if (d == 0) tmp[0] = t1;  // the tile's stem bytes (+ alignment room)
  }
  __syncthreads();
  const bool staged = tmp[0] <= RP_STAGE;
  const uint32_t* words = reinterpret_cast<const uint32_t*>(b.stem);
  const uint32_t nw = (b.off[b.n] + 3u) >> 2;
#pragma unroll
  for (uint32_t t = 0; t < RP_ITEMS; t++) {
    const uint32_t i = i0 + t * 64 + lane;
    if (i >= b.n) continue;
    const uint32_t d = my_d[t], len = my_len[t];
    const uint32_t j = gr[d] + wr[w][d] + my_r[t];      // record index in the send buffer
    if (d == own_rank) {  // read in place by this rank's owner batch (BatchDev::own): its position only
      perm[j] = i;
      continue;
    }
    const uint32_t local = gb[d] + wb[w][d] + my_b[t];  // byte offset inside owner d's chunk (not sent: the owner scans lengths)
    const uint32_t q = b.req[i];
    const int64_t tq = b.now[q];
    Wire x;
    x.label = (src_rank << ROUTE_REQ_BITS) | q;
    x.lu = len | ((uint32_t)b.unit[i] << 16) | ((uint32_t)b.flags[i] << 24);
    x.limit = b.limit[i];
    x.hits = b.hits[i];
    x.rule = b.rule[i] < b.n_rules ? b.rule[i] : 0xFFFFFFFFu;  // (the owner fails it alone, any rule stride)
    x.now = tq < 0 || tq > (int64_t)NOW_MAX ? WIRE_NOW_BAD : (uint32_t)tq;  // (the owner fails it: RL_E_TIME)
    x.hash = hash[i];
#if !(RL_RP_ABL & 2)
    out[j] = x;
    perm[j] = i;
#endif
    const uint32_t s0 = b.off[i];
#if RL_RP_ABL & 1
    continue;
#endif
    if (staged) {
      // whole LDS dwords of the destination from funnel-shifted source dwords;
      // single bytes only at the two ends (shared with the neighbours' stems)
      const uint32_t D = lo[d] + wb[w][d] + my_b[t];
      auto src4 = [&](uint32_t a) {  // stem bytes a..a+3 of the packed batch
        const uint32_t wi = a >> 2, sh = (a & 3u) * 8;
        const uint32_t v = words[wi];
        return sh ? (v >> sh) | ((wi + 1 < nw ? words[wi + 1] : 0u) << (32 - sh)) : v;
      };
      const uint32_t A0 = (D + 3u) & ~3u, A1 = (D + len) & ~3u;
      if (A0 >= A1) {
        for (uint32_t k = 0; k < len; k++) stage[D + k] = b.stem[s0 + k];
      } else {
        for (uint32_t a = D; a < A0; a++) stage[a] = b.stem[s0 + (a - D)];
        for (uint32_t a = A0; a < A1; a += 4) reinterpret_cast<uint32_t*>(stage)[a >> 2] = src4(s0 + (a - D));
        for (uint32_t a = A1; a < D + len; a++) stage[a] = b.stem[s0 + (a - D)];
      }
    } else {
      uint8_t* dst = out_stem + sb[d] + local;
      for (uint32_t k = 0; k < len; k++) dst[k] = b.stem[s0 + k];
    }
  }
  if (!staged) return;
  __syncthreads();
  // each owner's run of stems leaves the tile as dwords (bytes at its ends:
  // the neighbouring tiles own the rest of those dwords)
  for (uint32_t d = 0; d < n_shards; d++) {
    const uint32_t T = tb[d];
    if (!T) continue;
    const uint32_t G = sb[d] + gb[d], L = lo[d];
    const uint32_t A0 = G & ~3u, nd = (((G + T + 3u) & ~3u) - A0) >> 2;
    for (uint32_t k = threadIdx.x; k < nd; k += 256) {
      const uint32_t A = A0 + 4 * k;
      if (A >= G && A + 4 <= G + T) {
        *reinterpret_cast<uint32_t*>(out_stem + A) = reinterpret_cast<const uint32_t*>(stage)[(L + (A - G)) >> 2];
      } else {
        for (uint32_t z = 0; z < 4; z++) {
          const uint32_t a = A + z;
          if (a >= G && a < G + T) out_stem[a] = stage[L + (a - G)];
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_route_scatter(const uint32_t* __restrict__ perm,
                                                       const unsigned long long* __restrict__ ret, uint32_t n,
                                                       OutDev o, uint32_t* src_err, const uint32_t* errb,
                                                       uint32_t own_lo, uint32_t own_hi) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n || (j >= own_lo && j < own_hi)) return;  // (the own chunk: answered in place by its owner batch)
  const uint32_t e = perm[j];
  const uint32_t fail = errb ? *errb : 0u;  // (results straight from an owner batch: k_route_ret's check)
  const unsigned long long v = fail ? pack_fail(err_status(fail)) : ret[j];
  o.code[e] = (uint8_t)res_code(v);
  o.rem[e] = res_rem(v);
  o.reset[e] = res_reset(v);
  if (o.status) o.status[e] = (uint8_t)res_status(v);
  else if (src_err && res_status(v)) atomicOr(src_err, status_err(res_status(v)));
}

__global__ __launch_bounds__(256) void k_route_ret(const unsigned long long* __restrict__ res, uint32_t n,
                                                   const uint32_t* errb, unsigned long long* __restrict__ ret) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = *errb;
  ret[i] = e ? pack_fail(err_status(e)) : res[i];
}

// Per-rule stats deltas of several owners (blocks of `stride` counters, the
// first m of each) summed into out[0, m).
__global__ __launch_bounds__(256) void k_stats_sum(const unsigned long long* __restrict__ stage, uint32_t n_blocks,
                                                   uint32_t m, uint32_t stride, unsigned long long* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  unsigned long long s = 0;
  for (uint32_t b = 0; b < n_blocks; b++) s += stage[(size_t)b * stride + i];
  out[i] = s;
}

// An owner batch that cannot run: every received record answers `status`.
__global__ __launch_bounds__(256) void k_route_fail(unsigned long long* __restrict__ ret, uint32_t n, uint32_t status) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) ret[i] = pack_fail(status);
}

// The counts message of a slice that failed on the host: no records, no
// bytes, and the sender's meta words.
__global__ void k_cnt_fill(unsigned long long* cnt, uint32_t n_peers, uint32_t cstride, unsigned long long meta0,
                           unsigned long long meta1, unsigned long long* cnt_host) {
  for (uint32_t p = threadIdx.x; p < n_peers; p += blockDim.x) {
    for (unsigned long long* base : {cnt, cnt_host}) {
      if (!base) continue;
      unsigned long long* c = base + (size_t)cstride * p;
      c[0] = c[1] = 0;
      if (cstride >= 4) {
        c[2] = meta0;
        c[3] = meta1;
      }
    }
  }
}

// ---- owner side: the received records' stem offsets ----------------------
// Two passes over tiles of WIRE_SCAN_TILE records (8 per thread): k_ws_tiles
// stores each record's stem length (0 in the own chunk [olo, ohi), whose stems
// are read in place) into woff and the tile's sum into tsum; k_ws_offsets adds
// the sums of the tiles before its own and turns woff's lengths into
// exclusive offsets in place (each thread reads its 8 lengths before writing).
constexpr uint32_t WS_ITEMS = WIRE_SCAN_TILE / 256;

__device__ inline unsigned long long block_sum64(unsigned long long v, unsigned long long* tmp) {
#pragma unroll
  for (uint32_t o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane_id() == 0) tmp[threadIdx.x >> 6] = v;
  __syncthreads();
  v = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  __syncthreads();
  return v;
}

__global__ __launch_bounds__(256) void k_ws_tiles(const Wire* __restrict__ w, uint32_t n, uint32_t olo, uint32_t ohi,
                                                  uint32_t* __restrict__ woff, unsigned long long* __restrict__ tsum) {
  __shared__ unsigned long long tmp[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) tsum[gridDim.x] = 0;  // (the verdict: k_ws_offsets sets it)
  const uint32_t j0 = blockIdx.x * WIRE_SCAN_TILE + threadIdx.x * WS_ITEMS;
  unsigned long long acc = 0;
#pragma unroll
  for (uint32_t t = 0; t < WS_ITEMS; t++) {
    const uint32_t j = j0 + t;
    const uint32_t len = j < n && !(j - olo < ohi - olo) ? (w[j].lu & 0xFFFFu) : 0u;
    if (j < n) woff[j] = len;
    acc += len;
  }
  acc = block_sum64(acc, tmp);
  if (threadIdx.x == 0) tsum[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_ws_offsets(const Wire* __restrict__ w, uint32_t n, uint32_t olo,
                                                    uint32_t ohi, const unsigned long long* __restrict__ wbase,
                                                    uint32_t n_src, unsigned long long total,
                                                    unsigned long long* __restrict__ tsum,
                                                    uint32_t* __restrict__ woff) {
  __shared__ unsigned long long tmp[4], wtot[4];
  unsigned long long base = 0;  // the tiles before this one
  for (uint32_t k = threadIdx.x; k < blockIdx.x; k += 256) base += tsum[k];
  base = block_sum64(base, tmp);
  const uint32_t j0 = blockIdx.x * WIRE_SCAN_TILE + threadIdx.x * WS_ITEMS;
  uint32_t len[WS_ITEMS];
  unsigned long long mine = 0;
#pragma unroll
  for (uint32_t t = 0; t < WS_ITEMS; t++) {
    len[t] = j0 + t < n ? woff[j0 + t] : 0u;
    mine += len[t];
  }
  // exclusive prefix of `mine` over the block's threads (wave scan, then waves)
  unsigned long long inc = mine;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o, 64);
    if (lane_id() >= o) inc += y;
  }
  const uint32_t wv = threadIdx.x >> 6;
  if (lane_id() == 63) wtot[wv] = inc;
  __syncthreads();
  unsigned long long at = base + inc - mine;
  for (uint32_t k = 0; k < wv; k++) at += wtot[k];
  bool bad = false;
  auto own = [&](uint32_t j) { return j - olo < ohi - olo; };
#pragma unroll
  for (uint32_t t = 0; t < WS_ITEMS; t++) {
    const uint32_t j = j0 + t;
    if (j <= n) woff[j] = at < (1ull << 32) ? (uint32_t)at : 0xFFFFFFFFu;  // (woff[n]: the total)
    if (j < n && !own(j)) {  // a source's chunk starts at its base and ends at the next one's
      const uint32_t src = w[j].label >> ROUTE_REQ_BITS;
      if (src >= n_src) {
        bad = true;
      } else {
        if (j == 0 || own(j - 1) || (w[j - 1].label >> ROUTE_REQ_BITS) != src) bad = bad || at != wbase[src];
        if (j + 1 == n || own(j + 1) || (w[j + 1].label >> ROUTE_REQ_BITS) != src)
          bad = bad || at + len[t] != (src + 1 < n_src ? wbase[src + 1] : total);
      }
    }
    at += len[t];
  }
  if (__any(bad) && (threadIdx.x & 63u) == 0) atomicOr(tsum + gridDim.x, 1ull);
}

}  // namespace

void launch_wire_offsets(const Wire* w, uint32_t n, uint32_t olo, uint32_t ohi, const unsigned long long* wbase,
                         uint32_t n_src, unsigned long long stem_total, uint32_t* woff, unsigned long long* tsum,
                         hipStream_t st) {
  const uint32_t tiles = WIRE_SCAN_TILES(n);  // (n + 1 entries: a tile more when n is a multiple of the tile)
  k_ws_tiles<<<tiles, 256, 0, st>>>(w, n, olo, ohi, woff, tsum);
  k_ws_offsets<<<tiles, 256, 0, st>>>(w, n, olo, ohi, wbase, n_src, stem_total, tsum, woff);
}

void launch_stats_sum(const unsigned long long* stage, uint32_t n_blocks, uint32_t m, unsigned long long* out,
                      hipStream_t st, uint32_t stride) {
  if (m) k_stats_sum<<<cdiv(m, 256), 256, 0, st>>>(stage, n_blocks, m, stride ? stride : m, out);
}

void launch_route_fail(unsigned long long* ret, uint32_t n, uint32_t status, hipStream_t st) {
  if (n) k_route_fail<<<cdiv(n, 256), 256, 0, st>>>(ret, n, status);
}

void launch_cnt_fill(unsigned long long* cnt, uint32_t n_peers, uint32_t cstride, unsigned long long meta0,
                     unsigned long long meta1, hipStream_t st, unsigned long long* cnt_host) {
  k_cnt_fill<<<1, 256, 0, st>>>(cnt, n_peers, cstride, meta0, meta1, cnt_host);
}

void launch_route_pack(const BatchDev& b, uint32_t n_shards, uint32_t src_rank, Wire* out, uint8_t* out_stem,
                       uint32_t* perm, unsigned long long* counts, const Scratch& s, hipStream_t st, uint32_t cstride,
                       unsigned long long meta0, unsigned long long meta1, uint32_t own_rank,
                       unsigned long long* hash_out, unsigned long long* counts_host) {
  const uint32_t ntiles = b.n ? cdiv(b.n, RP_TILE) : 0u;
  unsigned long long* hash = hash_out ? hash_out : s.route_hash;
  if (b.n) k_rp_count<<<ntiles, 256, 0, st>>>(b, n_shards, ntiles, own_rank, s.route_dest, hash, s.route_hist, s.err);
  k_rp_scan<<<n_shards, 256, 0, st>>>(s.route_hist, n_shards, ntiles, counts, cstride, meta0, meta1, s.route_start,
                                       s.err, counts_host);
  if (b.n)
    k_rp_pack<<<ntiles, 256, 0, st>>>(b, n_shards, ntiles, src_rank, own_rank, s.route_dest, hash, s.route_hist,
                                      s.route_start, out,
                                      out_stem, perm, s.err);
}

void launch_route_scatter(const uint32_t* perm, const unsigned long long* ret, uint32_t n, const OutDev& o,
                          hipStream_t st, uint32_t* src_err, const uint32_t* errb, uint32_t own_lo, uint32_t own_hi) {
  if (n && !(own_lo == 0 && own_hi >= n))
    k_route_scatter<<<cdiv(n, 256), 256, 0, st>>>(perm, ret, n, o, src_err, errb, own_lo, own_hi);
}

void launch_route_ret(const unsigned long long* res, uint32_t n, const uint32_t* errb, unsigned long long* ret,
                      hipStream_t st) {
  if (n) k_route_ret<<<cdiv(n, 256), 256, 0, st>>>(res, n, errb, ret);
}

}  // namespace rl
