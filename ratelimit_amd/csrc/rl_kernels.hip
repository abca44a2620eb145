// rl_kernels.hip — gfx950 kernels of the fixed-window rate-limit backend.
//
// Pipeline for one batch (inputs already in HBM); stage A (table-free):
//   k_prepare     validate the packed batch; hash every stem (LDS-staged
//                 bytes); pack each descriptor into a 32-B Rec
//   k_os_*        onesweep stable LSD sort of (hash[63:32], index): groups each
//                 stem's descriptors together, in arrival (sequence) order
//   k_segment     Recs into sorted order, run ids, in-run prefix sums of hits
//                 (single pass, decoupled look-back), and the run checks: one
//                 stem and one unit per run (else k_runs_general)
//   ---- stage B (the table; batch order) ----
//   k_runs        one lane per run: probe/insert the (stem, unit) slot of the
//                 HBM table (one 128-B line per probe); replay short runs in
//                 registers, set up long uniform runs for k_fast_*
//   k_runs_general multi-stem / multi-unit runs, exact (beside k_runs)
//   k_fast_*      long uniform runs decided in parallel (scan + first-over)
//   k_finish      packed results -> code / limit_remaining / reset_s, and the
//                 striped per-block stats -> rl_result.stats
// plus k_sweep (epoch sweep = Redis EXPIRE), k_table_info, debug kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

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
                                                 uint32_t* __restrict__ vals, uint32_t* err,
                                                 const int64_t* time_floor, uint32_t* defer_n,
                                                 uint32_t* __restrict__ os_ghist, uint32_t* __restrict__ os_ctr,
                                                 uint32_t* __restrict__ run_flags, uint32_t* num_runs) {
  __shared__ uint32_t lds[HASH_LDS_BYTES / 4 + 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t i = blockIdx.x * 256 + tid;
  uint32_t bad = 0;
  if (i < b.n) run_flags[i] = 0;  // k_run_check ORs run flags in from any block
  if (blockIdx.x == 0) {  // per-batch counters: RUN_MULTI queue, run ids, digit totals and tile tickets
    if (tid == 0) {
      *defer_n = 0;
      *num_runs = 0;
    }
    if (tid < 5) os_ctr[tid] = 0;  // [0..3] sort passes, [4] k_segment
#pragma unroll
    for (uint32_t p = 0; p < 4; p++) os_ghist[p * 256 + tid] = 0;
  }

  // ---- per-request clock checks: now in [0, NOW_MAX] and not before the last sweep
  if (i < (b.now_desc ? b.n : b.n_req)) {
    const int64_t t = b.now[i];
    if (t < 0 || t > (int64_t)NOW_MAX || t < *time_floor) bad |= ERR_TIME;
  }

  // ---- per-descriptor checks
  uint32_t s0 = 0, len = 0, u = 0, q = 0;
  if (i < b.n) {
    s0 = b.off[i];
    const uint32_t s1 = b.off[i + 1];
    u = b.unit[i];
    q = b.req[i];
    if (u < 1 || u > 4 || b.rule[i] >= b.n_rules || (!b.now_desc && q >= b.n_req) || (i && b.req[i - 1] > q) || s1 < s0 ||
        s1 > b.stem_cap || s1 - s0 == 0 || s1 - s0 > 65535)
      bad |= ERR_INVALID;
    else
      len = s1 - s0;
  }
  if (bad) atomicOr(err, bad);

  // ---- stage this block's stem bytes in LDS (uniform decision per block)
  const uint32_t b0 = blockIdx.x * 256;
  if (b0 >= b.n) return;  // whole block past the descriptors (request checks done)
  const uint32_t b1 = min(b0 + 256u, b.n);
  const uint32_t lo = b.off[b0], hi = b.off[b1];
  const uint32_t total = b.off[b.n];
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
  if (len && range_ok) {
    if (use_lds) {
      h = hash_stem(DwordReader{lds, HASH_LDS_BYTES / 4 + 4}, s0 - lo + lead, len);
    } else {
      const uint32_t nw = ((total + 3u) >> 2) - (s0 >> 2);
      h = hash_stem(DwordReader{words + (s0 >> 2), nw}, s0 & 3u, len);
    }
  }
  keys[i] = (uint32_t)(h >> 32);
  vals[i] = i;
  Rec r;
  r.hlo = (uint32_t)h;
  r.off = s0;
  r.lu = len | (u << 16) | ((uint32_t)b.flags[i] << 24);
  r.rule = b.rule[i];
  r.req = q;
  r.now = b.now_desc ? (uint32_t)b.now[i] : (q < b.n_req) ? (uint32_t)b.now[q] : 0u;
  r.hits = b.hits[i];
  r.limit = b.limit[i];
  rec[i] = r;
}

// ===========================================================================
// Stable LSD radix sort of (u32 key, u32 value), 8-bit digits, 256-thread
// tiles of RS_ITEMS x 256 elements. Per pass: tile histograms (digit-major) ->
// per-digit row scans -> stable scatter.
// ===========================================================================
__global__ __launch_bounds__(256) void k_rs_hist(const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift,
                                                 uint32_t ntiles, uint32_t* __restrict__ hist, const uint32_t* err) {
  __shared__ uint32_t h[256];
  if (*err) return;
  const uint32_t tid = threadIdx.x;
  h[tid] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RS_TILE;
#pragma unroll 4
  for (uint32_t c = 0; c < RS_ITEMS; c++) {
    uint32_t j = base + c * 256 + tid;
    if (j < n) atomicAdd(&h[(keys[j] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[tid * ntiles + blockIdx.x] = h[tid];
}

// Row scan of the digit-major histogram: block d turns row d (ntiles tile
// counts) into exclusive prefixes in place and writes the row total.
__global__ __launch_bounds__(256) void k_rs_rowscan(uint32_t* __restrict__ hist, uint32_t ntiles,
                                                    uint32_t* __restrict__ totals, const uint32_t* err) {
  __shared__ uint32_t part[256];
  if (*err) return;
  const uint32_t tid = threadIdx.x;
  uint32_t* row = hist + (size_t)blockIdx.x * ntiles;
  const uint32_t per = (ntiles + 255) / 256;
  const uint32_t s0 = tid * per, s1 = min(s0 + per, ntiles);
  uint32_t sum = 0;
  for (uint32_t j = s0; j < s1; j++) sum += row[j];
  part[tid] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < 256; off <<= 1) {
    const uint32_t v = tid >= off ? part[tid - off] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = part[tid] - sum;
  for (uint32_t j = s0; j < s1; j++) {
    const uint32_t v = row[j];
    row[j] = run;
    run += v;
  }
  if (tid == 255) totals[blockIdx.x] = part[255];
}

// Stable scatter. Wave w of a tile owns elements [w*64*RS_ITEMS, (w+1)*64*RS_ITEMS)
// of it, item-major: it ranks them with a ballot multisplit (8 ballots -> the
// lanes sharing a digit) against a wave-private running count in LDS, keeps
// keys/values/ranks in registers, and only then (one barrier) learns the
// other waves' counts and the digit's global base.
__global__ __launch_bounds__(256) void k_rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                    uint32_t n, uint32_t shift, uint32_t ntiles,
                                                    const uint32_t* __restrict__ hist,
                                                    const uint32_t* __restrict__ totals, const uint32_t* err) {
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t dsum[256];
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  wcnt[0][tid] = 0; wcnt[1][tid] = 0; wcnt[2][tid] = 0; wcnt[3][tid] = 0;
  dsum[tid] = totals[tid];
  __syncthreads();
  const uint64_t lt_mask = (1ull << lane) - 1;
  const uint32_t wbase = blockIdx.x * RS_TILE + wave * 64 * RS_ITEMS;
  uint32_t kk[RS_ITEMS], vv[RS_ITEMS], pos[RS_ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < RS_ITEMS; i++) {
    const uint32_t j = wbase + i * 64 + lane;
    const bool valid = j < n;
    kk[i] = valid ? kin[j] : 0xFFFFFFFFu;
    vv[i] = valid ? vin[j] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < RS_ITEMS; i++) {
    const bool valid = wbase + i * 64 + lane < n;
    const uint32_t d = (kk[i] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (uint32_t bit = 0; bit < 8; bit++) {
      const bool sb = (d >> bit) & 1u;
      const uint64_t bal = __ballot(sb);
      peers &= sb ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lt_mask);
    const uint32_t leader = valid ? (uint32_t)(__ffsll((unsigned long long)peers) - 1) : lane;
    uint32_t old = 0;
    if (valid && rank == 0) {
      old = wcnt[wave][d];
      wcnt[wave][d] = old + __popcll(peers);
    }
    old = __shfl(old, leader);
    pos[i] = old + rank;
  }
  __syncthreads();
  {  // digit base for this tile = exclusive scan of the digit totals + row prefix
    uint32_t x = dsum[tid];
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {
      const uint32_t v = tid >= off ? dsum[tid - off] : 0u;
      __syncthreads();
      dsum[tid] += v;
      __syncthreads();
    }
    uint32_t run = dsum[tid] - x + hist[(size_t)tid * ntiles + blockIdx.x];
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
      const uint32_t t = wcnt[w][tid];
      wcnt[w][tid] = run;
      run += t;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < RS_ITEMS; i++) {
    if (wbase + i * 64 + lane < n) {
      const uint32_t p = wcnt[wave][(kk[i] >> shift) & 255u] + pos[i];
      kout[p] = kk[i];
      vout[p] = vv[i];
    }
  }
}

// ===========================================================================
// Onesweep LSD radix sort of (u32 key, u32 value), 8-bit digits: one kernel
// reads the keys once for all four digit histograms, then one kernel per pass.
// A pass block takes the next tile ticket (so every earlier tile belongs to a
// block that is already running), ranks its RS_TILE elements in LDS with the
// wave ballot multisplit, publishes its per-digit counts and learns the counts
// of all earlier tiles by decoupled look-back over 8-byte {count, tag} granules
// (one agent-scope store / load each: untorn, no separate flag). The tag holds
// the batch epoch and pass, so granules are never cleared.
// ===========================================================================
constexpr uint32_t OS_AGG = 1u, OS_INC = 2u;

__host__ __device__ inline uint32_t os_tag(uint32_t epoch, uint32_t pass) { return (epoch << 4) | (pass << 2); }

__global__ __launch_bounds__(256) void k_os_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                 uint32_t* __restrict__ ghist, const uint32_t* err) {
  __shared__ uint32_t h[4][256];
  if (*err) return;
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (uint32_t p = 0; p < 4; p++) h[p][tid] = 0;
  __syncthreads();
  for (uint32_t j = blockIdx.x * 256 + tid; j < n; j += gridDim.x * 256) {
    const uint32_t k = keys[j];
    atomicAdd(&h[0][k & 255u], 1u);
    atomicAdd(&h[1][(k >> 8) & 255u], 1u);
    atomicAdd(&h[2][(k >> 16) & 255u], 1u);
    atomicAdd(&h[3][k >> 24], 1u);
  }
  __syncthreads();
#pragma unroll
  for (uint32_t p = 0; p < 4; p++) {
    const uint32_t v = h[p][tid];
    if (v) atomicAdd(&ghist[p * 256 + tid], v);
  }
}

#ifdef RL_OS_PROF  // sortbench only: per-tile phase stamps of the last pass launched
__device__ unsigned long long g_os_prof[8192 * 8];
#define OS_STAMP(k) \
  if (threadIdx.x == 0) g_os_prof[tile * 8 + (k)] = wall_clock64()
#else
#define OS_STAMP(k)
#endif

__global__ __launch_bounds__(OS_THREADS) void k_os_pass(const uint32_t* __restrict__ kin,
                                                        const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
                                                        uint32_t* __restrict__ vout, uint32_t n, uint32_t pass,
                                                        const uint32_t* __restrict__ ghist, uint32_t* __restrict__ ctr,
                                                        unsigned long long* status, uint32_t tag, const uint32_t* err) {
  __shared__ uint32_t wcnt[OS_WAVES][256];
  __shared__ uint32_t dbase[256];
  __shared__ uint32_t gsum[4];
  __shared__ uint32_t s_tile;
  if (*err) return;  // the same for every block: no tile is left half-published
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(&ctr[pass], 1u);
  for (uint32_t j = tid; j < OS_WAVES * 256; j += OS_THREADS) (&wcnt[0][0])[j] = 0;
  __syncthreads();
  const uint32_t tile = s_tile, shift = 8 * pass;
  OS_STAMP(0);
  const uint64_t lt_mask = (1ull << lane) - 1;
  const uint32_t wbase = tile * OS_TILE + wave * 64 * OS_ITEMS;
  uint32_t kk[OS_ITEMS], vv[OS_ITEMS], pos[OS_ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < OS_ITEMS; i++) {
    const uint32_t j = wbase + i * 64 + lane;
    const bool valid = j < n;
    kk[i] = valid ? kin[j] : 0xFFFFFFFFu;
    vv[i] = valid ? vin[j] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < OS_ITEMS; i++) {
    const bool valid = wbase + i * 64 + lane < n;
    const uint32_t d = (kk[i] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (uint32_t bit = 0; bit < 8; bit++) {
      const bool sb = (d >> bit) & 1u;
      const uint64_t bal = __ballot(sb);
      peers &= sb ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lt_mask);
    const uint32_t leader = valid ? (uint32_t)(__ffsll((unsigned long long)peers) - 1) : lane;
    uint32_t old = 0;
    if (valid && rank == 0) {
      old = wcnt[wave][d];
      wcnt[wave][d] = old + __popcll(peers);
    }
    old = __shfl(old, leader);
    pos[i] = old + rank;
  }
  __syncthreads();
  OS_STAMP(1);
  if (tid < 256) {
    // digit tid: this tile's count and the per-wave exclusive offsets
    uint32_t c = 0;
#pragma unroll
    for (uint32_t w = 0; w < OS_WAVES; w++) {
      const uint32_t t = wcnt[w][tid];
      wcnt[w][tid] = c;
      c += t;
    }
    unsigned long long* mine = status + (size_t)tile * 256 + tid;
    __hip_atomic_store(mine, (unsigned long long)c | ((unsigned long long)(tag | (tile ? OS_AGG : OS_INC)) << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // global exclusive base of digit tid: wave scans of the pass's digit totals
    const uint32_t g = ghist[pass * 256 + tid];
    uint32_t inc = g;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(inc, off, 64);
      if (lane >= off) inc += y;
    }
    if (lane == 63) gsum[wave] = inc;
    // decoupled look-back: add earlier tiles' counts until an inclusive prefix.
    // OS_LB granules (tiles j, j-1, ...) are loaded together per round trip;
    // the ready prefix of them is consumed (an aggregate is a final tile count,
    // so a partial window is exact) and the walk resumes below it.
    uint32_t excl = 0;
    if (tile) {
      int32_t j = (int32_t)tile - 1;
      for (;;) {
        unsigned long long v[OS_LB];
#pragma unroll
        for (uint32_t k = 0; k < OS_LB; k++)
          v[k] = j - (int32_t)k >= 0 ? __hip_atomic_load(status + (size_t)(j - (int32_t)k) * 256 + tid,
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : 0ull;
        uint32_t add = 0, used = 0;
        bool stop = false, done = false;
#pragma unroll
        for (uint32_t k = 0; k < OS_LB; k++) {
          const uint32_t tg = (uint32_t)(v[k] >> 32);
          if (stop || (tg & ~3u) != tag) {  // not yet published for this pass
            stop = true;
            continue;
          }
          add += (uint32_t)v[k];
          used++;
          if (tg & OS_INC) stop = done = true;  // tile 0 is inclusive, so j never passes it
        }
        excl += add;
        if (done) break;
        j -= (int32_t)used;
        if (!used) __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(mine, (unsigned long long)(excl + c) | ((unsigned long long)(tag | OS_INC) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    dbase[tid] = inc - g + excl;  // + earlier waves' digit totals, below
  }
  __syncthreads();  // gsum, dbase
  if (tid < 256) {
    uint32_t wpre = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) wpre += w < wave ? gsum[w] : 0u;
    dbase[tid] += wpre;
  }
  __syncthreads();
  OS_STAMP(2);
#pragma unroll
  for (uint32_t i = 0; i < OS_ITEMS; i++) {
    if (wbase + i * 64 + lane < n) {
      const uint32_t d = (kk[i] >> shift) & 255u;
      const uint32_t p = dbase[d] + wcnt[wave][d] + pos[i];
      kout[p] = kk[i];
      vout[p] = vv[i];
    }
  }
  OS_STAMP(3);
}

// The zero-padded first KEY_HEAD bytes of the stem at byte `off` of the packed
// stems, as 4 x uint4: five aligned 16-B loads, then dword selects and funnel
// shifts. Only chunks holding a byte of the head are loaded, so no load leaves
// the 16-B blocks (hence the pages) the stem occupies.
__device__ inline void load_head(const uint8_t* stem, uint32_t off, uint32_t len, uint4 out[4]) {
  const uint32_t hl = len < KEY_HEAD ? len : KEY_HEAD;
  const uint32_t mis = (uint32_t)((uintptr_t)stem & 15u);
  const uint4* c16 = reinterpret_cast<const uint4*>(stem - mis);
  const uint32_t a = off + mis;
  const uint32_t c0 = a >> 4, last = (a + (hl ? hl : 1u) - 1u) >> 4;
  uint32_t w[20];
#pragma unroll
  for (uint32_t j = 0; j < 5; j++) {
    const uint4 v = c0 + j <= last ? c16[c0 + j] : make_uint4(0u, 0u, 0u, 0u);
    w[4 * j] = v.x;
    w[4 * j + 1] = v.y;
    w[4 * j + 2] = v.z;
    w[4 * j + 3] = v.w;
  }
  const uint32_t q = (a >> 2) & 3u, sb = a & 3u;
  uint32_t x[17];
#pragma unroll
  for (uint32_t k = 0; k < 17; k++) x[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
  uint32_t o[16];
#pragma unroll
  for (uint32_t k = 0; k < 16; k++) {
    uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sb);
    if (4 * k >= hl) v = 0;
    else if (4 * k + 4 > hl) v &= (1u << ((hl - 4 * k) * 8)) - 1u;
    o[k] = v;
  }
#pragma unroll
  for (uint32_t v = 0; v < 4; v++) out[v] = make_uint4(o[4 * v], o[4 * v + 1], o[4 * v + 2], o[4 * v + 3]);
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
  uint4 h[4];
  StemRef st;  // full stem (bytes >= KEY_HEAD read from here)
  uint32_t len;
};

__device__ inline Key key_of(const BatchDev& b, const Rec& r) {
  Key k;
  k.len = rec_len(r);
  k.st = stem_ref(b, r.off);
  load_head(b.stem, r.off, k.len, k.h);
  return k;
}

__device__ inline Key key_at(const BatchDev& b, const Rec* rec_s, uint32_t q) { return key_of(b, rec_s[q]); }

__device__ inline uint32_t head_diff(const uint4* x, const uint4* y) {
  uint32_t d = 0;
#pragma unroll
  for (uint32_t v = 0; v < 4; v++) {
    const uint4 a = x[v], c = y[v];
    d |= (a.x ^ c.x) | (a.y ^ c.y) | (a.z ^ c.z) | (a.w ^ c.w);
  }
  return d;
}

// bytes [64, len) of two stems (words 16.. of their StemRefs)
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
// Slot key bytes 0..63 were written from a zero-padded key head, so they
// compare as whole uint4s; bytes 64..79 inline and the arena cover the rest.
__device__ inline bool slot_key_equal(const Slot* s, const Key& key, const uint8_t* arena) {
  if (s->key_len != key.len) return false;
  const uint4* sk4 = reinterpret_cast<const uint4*>(s->key);
  uint32_t diff = head_diff(sk4, key.h);
  const uint32_t len = key.len;
  if (len > KEY_HEAD) {
    const uint32_t* sk = reinterpret_cast<const uint32_t*>(s->key);
    const uint32_t il = len < INLINE_KEY ? len : INLINE_KEY;
    const uint32_t nw = il >> 2;
    for (uint32_t k = KEY_HEAD / 4; k < nw; k++) diff |= sk[k] ^ key.st.word(k);
    if (il & 3) diff |= (sk[nw] ^ key.st.word(nw)) & tail_mask(il);
    if (len > INLINE_KEY) {
      const uint32_t* ek = reinterpret_cast<const uint32_t*>(arena + (size_t)s->ext_off * 16);
      const uint32_t rest = len - INLINE_KEY, rw = rest >> 2;
      for (uint32_t k = 0; k < rw; k++) diff |= ek[k] ^ key.st.word(INLINE_KEY / 4 + k);
      if (rest & 3) diff |= (ek[rw] ^ key.st.word(INLINE_KEY / 4 + rw)) & tail_mask(rest);
    }
  }
  return diff == 0;
}

__device__ inline void slot_init(const TableDev& t, Slot* s, const Key& key, uint32_t unit, uint32_t* err) {
  const uint32_t len = key.len;
  s->key_len = (uint16_t)len;
  s->unit = (uint8_t)unit;
  s->flags = 0;
  s->ext_off = 0;
  uint4* sk4 = reinterpret_cast<uint4*>(s->key);
#pragma unroll
  for (uint32_t v = 0; v < 4; v++) sk4[v] = key.h[v];
  if (len > KEY_HEAD) {
    uint32_t* sk = reinterpret_cast<uint32_t*>(s->key);
    const uint32_t il = len < INLINE_KEY ? len : INLINE_KEY;
    for (uint32_t k = KEY_HEAD / 4; k < (il + 3) / 4; k++) sk[k] = key.st.word(k);
  }
  if (len > INLINE_KEY) {
    const uint32_t n16 = (len - INLINE_KEY + 15) / 16;
    unsigned long long off = atomicAdd(t.arena_used16, (unsigned long long)n16);
    if (off + n16 > t.arena_cap16) {
      atomicOr(err, ERR_ARENA_FULL);
    } else {
      s->ext_off = (uint32_t)off;
      uint32_t* ek = reinterpret_cast<uint32_t*>(t.arena + off * 16);
      for (uint32_t k = 0; k < (len - INLINE_KEY + 3) / 4; k++) ek[k] = key.st.word(INLINE_KEY / 4 + k);
    }
  }
  s->cur = Win{WS_INVALID, 0, 0, 0};
  s->prev = Win{WS_INVALID, 0, 0, 0};
}

// Find (and optionally insert) the slot of (stem, unit). Returns -1 when absent
// and insert == false, or on a full table (error bit set). Linear probing over
// 128-B slots from the home slot = top bits of the stem hash, i.e. of the sort
// key: consecutive runs probe increasing slots (page and TLB locality). A tag
// match is confirmed by the full stem (collision-exact). Inserts claim the slot
// with a 64-bit CAS on its tag; only one lane ever handles a given (stem, unit)
// per batch (runs are grouped by stem).
__device__ int64_t find_slot(const TableDev& t, uint64_t hstem, uint64_t tag, const Key& key, uint32_t unit,
                             bool insert, bool* inserted, uint32_t* err) {
  uint64_t i = hstem >> t.shift;
  int64_t tomb = -1;
  *inserted = false;
  for (uint32_t p = 0; p < t.max_probe; p++, i = (i + 1) & t.mask) {
    Slot* s = &t.slots[i];
    const uint64_t st = __hip_atomic_load(&s->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (st == tag) {
      if (slot_key_equal(s, key, t.arena)) return (int64_t)i;
      continue;
    }
    if (st == TAG_TOMB) {
      if (tomb < 0) tomb = (int64_t)i;
      continue;
    }
    if (st != TAG_EMPTY) continue;
    // (stem, unit) is absent: claim the first tombstone on the path, else this slot.
    if (!insert) return -1;
    if (tomb >= 0) {
      Slot* ts = &t.slots[tomb];
      if (atomicCAS((unsigned long long*)&ts->tag, (unsigned long long)TAG_TOMB, (unsigned long long)tag) ==
          TAG_TOMB) {
        slot_init(t, ts, key, unit, err);
        *inserted = true;
        return tomb;
      }
    }
    const unsigned long long prev =
        atomicCAS((unsigned long long*)&s->tag, (unsigned long long)TAG_EMPTY, (unsigned long long)tag);
    if (prev == TAG_EMPTY) {
      slot_init(t, s, key, unit, err);
      *inserted = true;
      return (int64_t)i;
    }
    // another stem claimed this slot concurrently: keep probing
  }
  atomicOr(err, ERR_TABLE_FULL);
  return -1;
}

// A slot's whole 128-B line, loaded in one round trip (8 x dwordx4): [0] tag |
// key_len, unit, flags | ext_off, [1] cur, [2] prev, [3..7] stem bytes 0..79.
// The run kernel probes with it: tag, stem and both window records arrive
// together instead of three dependent loads. Plain loads are enough: within a
// launch only CAS inserts change tags, and a lane only ever looks for its own
// stem, which no other lane inserts.
struct SlotImg {
  uint4 v[8];
  __device__ inline uint64_t tag() const { return ((uint64_t)v[0].y << 32) | v[0].x; }
  __device__ inline uint32_t key_len() const { return v[0].z & 0xFFFFu; }
  __device__ inline uint32_t flags() const { return v[0].z >> 24; }
  __device__ inline uint32_t ext_off() const { return v[0].w; }
  __device__ inline Win cur() const { return Win{v[1].x, v[1].y, v[1].z, v[1].w}; }
  __device__ inline Win prev() const { return Win{v[2].x, v[2].y, v[2].z, v[2].w}; }
};

__device__ inline void load_img(const Slot* s, SlotImg& im) {
  const uint4* p = reinterpret_cast<const uint4*>(s);
#pragma unroll
  for (int j = 0; j < 8; j++) im.v[j] = p[j];
}

__device__ inline uint32_t u4w(const uint4& a, uint32_t j) { return j == 0 ? a.x : j == 1 ? a.y : j == 2 ? a.z : a.w; }

// Stem of `key` == the slot's stem?
__device__ inline bool img_key_equal(const SlotImg& im, const Key& key, const uint8_t* arena) {
  const uint4* kh = key.h;
  if (im.key_len() != key.len) return false;
  uint32_t d = 0;
#pragma unroll
  for (uint32_t v = 0; v < 4; v++) {
    const uint4 a = im.v[3 + v], c = kh[v];
    d |= (a.x ^ c.x) | (a.y ^ c.y) | (a.z ^ c.z) | (a.w ^ c.w);
  }
  const uint32_t len = key.len;
  if (len > KEY_HEAD) {
    const uint32_t il = len < INLINE_KEY ? len : INLINE_KEY, nw = il >> 2;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t k = KEY_HEAD / 4 + j;
      const uint32_t x = u4w(im.v[7], j) ^ key.st.word(k);
      if (k < nw) d |= x;
      else if (k == nw && (il & 3)) d |= x & tail_mask(il);
    }
    if (len > INLINE_KEY) {
      const uint32_t* ek = reinterpret_cast<const uint32_t*>(arena + (size_t)im.ext_off() * 16);
      const uint32_t rest = len - INLINE_KEY, rw = rest >> 2;
      for (uint32_t k = 0; k < rw; k++) d |= ek[k] ^ key.st.word(INLINE_KEY / 4 + k);
      if (rest & 3) d |= (ek[rw] ^ key.st.word(INLINE_KEY / 4 + rw)) & tail_mask(rest);
    }
  }
  return d == 0;
}

// find_slot with insert, returning the slot's image (a fresh slot's image for
// an insert: empty windows, no flags). `im` holds the home slot's image on
// entry (the caller issues that load early, beside the stem's).
__device__ int64_t find_slot_img(const TableDev& t, uint64_t hstem, uint64_t tag, const Key& key, uint32_t unit,
                                 bool* inserted, SlotImg& im, uint32_t* err) {
  uint64_t i = hstem >> t.shift;
  int64_t tomb = -1;
  *inserted = false;
  for (uint32_t p = 0; p < t.max_probe; p++, i = (i + 1) & t.mask) {
    if (p) load_img(&t.slots[i], im);
    const uint64_t st = im.tag();
    if (st == tag) {
      if (img_key_equal(im, key, t.arena)) return (int64_t)i;
      continue;
    }
    if (st == TAG_TOMB) {
      if (tomb < 0) tomb = (int64_t)i;
      continue;
    }
    if (st != TAG_EMPTY) continue;
    int64_t at = -1;
    if (tomb >= 0 && atomicCAS((unsigned long long*)&t.slots[tomb].tag, (unsigned long long)TAG_TOMB,
                               (unsigned long long)tag) == TAG_TOMB)
      at = tomb;
    else if (atomicCAS((unsigned long long*)&t.slots[i].tag, (unsigned long long)TAG_EMPTY,
                       (unsigned long long)tag) == TAG_EMPTY)
      at = (int64_t)i;
    if (at >= 0) {
      slot_init(t, &t.slots[at], key, unit, err);
      im.v[0] = make_uint4((uint32_t)tag, (uint32_t)(tag >> 32), key.len | (unit << 16), 0u);
      im.v[1] = make_uint4(WS_INVALID, 0u, 0u, 0u);
      im.v[2] = im.v[1];
      *inserted = true;
      return at;
    }
    // another stem claimed this slot concurrently: keep probing
  }
  atomicOr(err, ERR_TABLE_FULL);
  return -1;
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
constexpr uint32_t MAX_REPS = 8;

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
  x.flags = (uint8_t)rec_flags(r);
  x.shadow = (x.flags & RL_FLAG_SHADOW) != 0;
  return x;
}

// One 8-B store per descriptor: remaining | reset << 32 | code << 56 (k_finish).
__device__ __attribute__((always_inline)) inline void emit(unsigned long long* res, LaneStats& L, StatAcc& acc,
                                                           const Elem& x, const Decision& r) {
  const uint32_t reset = x.d - x.now % x.d;  // utils.CalculateReset
  res[x.e] = (unsigned long long)r.remaining | ((unsigned long long)reset << 32) |
             ((unsigned long long)r.code << 56);
  const uint32_t d[RL_NUM_STATS] = {x.h, r.d_over, r.d_near, r.d_lc, r.d_within, r.d_shadow};
  L.add(acc, x.rule, d);
}

// The record of window w in a slot's (cur, prev) pair: 0 (cur), 1 (prev) or
// -1. cur is the newest window ever written for this (stem, unit), prev the
// newest before it, so a window strictly between them was never written (a
// fresh key): it takes prev's place. A newer window rolls cur into prev. A
// window older than prev is outside the table's history: -1 -> RL_E_TIME,
// never silently wrong. With allow_back false (multi-unit stems, where other
// units may alias the key) only the current or a newer window is accepted.
__device__ __attribute__((always_inline)) inline int window_pick(Win& cur, Win& prev, uint32_t w, uint32_t lc_init,
                                                                bool allow_back) {
  if (cur.ws == w) return 0;
  if (cur.ws == WS_INVALID || w > cur.ws) {
    prev = cur;
    cur = Win{w, 0, 0, lc_init};
    return 0;
  }
  if (!allow_back) return -1;
  if (prev.ws == w) return 1;
  if (prev.ws == WS_INVALID || w > prev.ws) {
    prev = Win{w, 0, 0, lc_init};
    return 1;
  }
  return -1;
}

// ---- single (stem, unit) slot, stem never seen with another unit: registers only
struct SimpleState {
  Win cur, prev;
  uint32_t cur_req;
  bool pend;
  uint32_t pend_w, pend_e;
  __device__ inline void apply_pending() {
    if (pend) {
      if (cur.ws == pend_w) cur.lc = pend_e;
      else if (prev.ws == pend_w) prev.lc = pend_e;
      pend = false;
    }
  }
};

__device__ __attribute__((always_inline)) inline void simple_step(const Params& P, unsigned long long* res,
                                                                  LaneStats& L, StatAcc& acc, SimpleState& S,
                                                                  const Elem& x, bool restore, uint32_t* err) {
  if (x.req != S.cur_req) {
    S.apply_pending();
    S.cur_req = x.req;
  }
  const int which = window_pick(S.cur, S.prev, x.w, 0, true);
  if (which < 0) {
    if (!(RL_ABL & 1)) atomicOr(err, ERR_HISTORY);  // (ablation builds probe garbage slots)
    return;
  }
  Win R = which ? S.prev : S.cur;  // values, not pointers: the state stays in VGPRs
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
  if (which) S.prev = R;
  else S.cur = R;
  if (restore) return;
  const Decision r = decide(after - x.h, after, lc_hit && !x.shadow, x.h, x.thr, P.ratio, x.shadow, P.lc_en);
  if (r.set_lc) {
    S.pend = true;
    S.pend_w = x.w;
    S.pend_e = x.now + x.d;
  }
  emit(res, L, acc, x, r);
}

// ---- general: every unit slot of the stem, Redis keys shared across units
struct GeneralState {
  int64_t sidx[4];
  Win cur[4], prev[4];
  uint32_t present;  // bit u-1
  uint32_t cur_req;
  uint32_t npend;
  uint32_t pend_w[4], pend_e[4];
};

__device__ inline bool ps_class(const Params& P, uint32_t k) { return P.per_second && k == 0; }

__device__ inline void general_apply_pending(GeneralState& G) {
  for (uint32_t j = 0; j < G.npend; j++) {
    for (uint32_t k = 0; k < 4; k++) {
      if (!(G.present >> k & 1)) continue;
      if (G.cur[k].ws == G.pend_w[j]) G.cur[k].lc = G.pend_e[j];
      if (G.prev[k].ws == G.pend_w[j]) G.prev[k].lc = G.pend_e[j];
    }
  }
  G.npend = 0;
}

__device__ inline void general_step(const Params& P, unsigned long long* res, LaneStats& L, StatAcc& acc,
                                    GeneralState& G, const Elem& x, bool restore, uint32_t* err) {
  if (x.req != G.cur_req) {
    general_apply_pending(G);
    G.cur_req = x.req;
  }
  const uint32_t ui = x.unit - 1;
  const bool ps_e = ps_class(P, ui);
  bool lc_hit = false;
  uint32_t v = 0, lcw = 0;
  bool vfound = false;
  for (uint32_t k = 0; k < 4; k++) {
    if (!(G.present >> k & 1)) continue;
    const Win* recs[2] = {&G.cur[k], &G.prev[k]};
    for (uint32_t r = 0; r < 2; r++) {
      const Win& R = *recs[r];
      if (R.ws != x.w) continue;
      if (x.now < R.lc) lc_hit = true;
      lcw = R.lc > lcw ? R.lc : lcw;
      if (ps_class(P, k) == ps_e && !vfound && x.now <= R.expire) {
        v = R.count;
        vfound = true;
      }
    }
  }
  lc_hit = lc_hit && P.lc_en && !restore;
  uint32_t after = 0;
  if (!lc_hit) {
    const uint32_t nv = restore ? x.h : v + x.h;
    const uint32_t ex = x.now + x.d;
    if (window_pick(G.cur[ui], G.prev[ui], x.w, lcw, false) < 0) {
      if (!(RL_ABL & 1)) atomicOr(err, ERR_HISTORY);  // (ablation builds probe garbage slots)
      return;
    }
    for (uint32_t k = 0; k < 4; k++) {  // Redis key stem‖w in this store: every alias record
      if (!(G.present >> k & 1) || ps_class(P, k) != ps_e) continue;
      if (G.cur[k].ws == x.w) { G.cur[k].count = nv; G.cur[k].expire = ex; }
      if (G.prev[k].ws == x.w) { G.prev[k].count = nv; G.prev[k].expire = ex; }
    }
    after = nv;
  }
  if (restore) {
    if (x.flags) {
      for (uint32_t k = 0; k < 4; k++) {
        if (!(G.present >> k & 1)) continue;
        if (G.cur[k].ws == x.w) G.cur[k].lc = x.now + x.d;
        if (G.prev[k].ws == x.w) G.prev[k].lc = x.now + x.d;
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
  emit(res, L, acc, x, r);
}

// Replay elements [p, end) (those of stem k when repid is given) through the
// single-unit slot s0, in registers.
__device__ __attribute__((always_inline)) inline void replay_simple(const Rec* rec_s, const uint32_t* svals,
                                                                    unsigned long long* res, const TableDev& t,
                                                                    const Params& P, const uint8_t* repid,
                                                                    uint32_t p, uint32_t end, uint32_t k, int64_t s0,
                                                                    Win cur0, Win prev0, const Rec& x0, uint32_t e0,
                                                                    LaneStats& L, StatAcc& acc, uint32_t* err,
                                                                    bool restore, const SlotImg* img = nullptr) {
  Slot* s = &t.slots[s0];
  SimpleState S;
  S.cur = cur0;
  S.prev = prev0;
  S.cur_req = 0xFFFFFFFFu;
  S.pend = false;
  simple_step(P, res, L, acc, S, load_elem(x0, e0, restore), restore, err);  // element p (always stem k)
  for (uint32_t q = p + 1; q < end; q++) {
    if (repid && repid[q] != k) continue;
    simple_step(P, res, L, acc, S, load_elem(rec_s[q], svals[q], restore), restore, err);
  }
  S.apply_pending();
  if (img) {  // random writes are the costly part of the probe: store only records that changed
    const uint4 c = img->v[1], q = img->v[2];
    if (S.cur.ws != c.x || S.cur.count != c.y || S.cur.expire != c.z || S.cur.lc != c.w) s->cur = S.cur;
    if (S.prev.ws != q.x || S.prev.count != q.y || S.prev.expire != q.z || S.prev.lc != q.w) s->prev = S.prev;
  } else {
    s->cur = S.cur;
    s->prev = S.prev;
  }
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
struct SegPair {
  uint32_t f, s;
};
__device__ inline SegPair seg_op(SegPair a, SegPair b) { return SegPair{a.f | b.f, b.f ? b.s : a.s + b.s}; }

constexpr uint32_t SEG_STRIP = SEG_TILE / 4;  // positions per wave
static_assert(SEG_STRIP == SEG_ITEMS * 64, "4 waves x SEG_ITEMS chunks of 64");

struct SegChunk {
  uint64_t heads;  // ballot of run heads in the chunk
  uint32_t h;      // this lane's max(1, hits) (0 past n)
};

__device__ inline SegChunk seg_chunk(const uint32_t* skeys, const uint32_t* hits_s, uint32_t n, uint32_t q) {
  const bool valid = q < n;
  const bool head = valid && (q == 0 || skeys[q - 1] != skeys[q]);
  const uint32_t hv = valid ? hits_s[q] : 0u;
  return SegChunk{(uint64_t)__ballot(head), valid ? (hv > 1 ? hv : 1u) : 0u};
}

// Inclusive segmented scan of a chunk (lane order). Plain prefix sum P, then
// subtract the prefix before the lane's last head.
__device__ inline SegPair seg_chunk_scan(const SegChunk& c, uint32_t lane) {
  uint32_t P = c.h;
#pragma unroll
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(P, off, 64);
    if (lane >= off) P += y;
  }
  const uint64_t le = c.heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
  const uint32_t lh = le ? 63u - (uint32_t)__clzll((long long)le) : 0u;
  const uint32_t Plh = __shfl(P, lh, 64), hlh = __shfl(c.h, lh, 64);
  return le ? SegPair{1u, P - (Plh - hlh)} : SegPair{0u, P};
}

// Block-level combine of the 4 wave aggregates: returns this wave's exclusive
// prefix within the tile (and the tile aggregate through *tot for lane 0 of
// wave 0 callers).
__device__ inline void seg_waves(SegPair agg, uint32_t hc, SegPair* sp, uint32_t* sh, SegPair& excl, uint32_t& hexcl,
                                 SegPair& tot, uint32_t& htot) {
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sp[w] = agg;
    sh[w] = hc;
  }
  __syncthreads();
  excl = SegPair{0, 0};
  hexcl = 0;
  tot = SegPair{0, 0};
  htot = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    if (k == w) {
      excl = tot;
      hexcl = htot;
    }
    tot = seg_op(tot, sp[k]);
    htot += sh[k];
  }
}

__global__ __launch_bounds__(256) void k_seg_reduce(const uint32_t* __restrict__ skeys,
                                                    const uint32_t* __restrict__ hits_s, uint32_t n,
                                                    uint32_t* __restrict__ tile_f, uint32_t* __restrict__ tile_s,
                                                    uint32_t* __restrict__ tile_h, const uint32_t* err) {
  __shared__ SegPair sp[4];
  __shared__ uint32_t sh[4];
  if (*err) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * SEG_TILE + (threadIdx.x >> 6) * SEG_STRIP + lane;
  SegPair agg{0, 0};
  uint32_t hc = 0;
#pragma unroll 4
  for (uint32_t c = 0; c < SEG_ITEMS; c++) {
    const SegChunk ch = seg_chunk(skeys, hits_s, n, base + 64 * c);
    const SegPair v = seg_chunk_scan(ch, lane);
    agg = seg_op(agg, SegPair{__shfl(v.f, 63, 64), __shfl(v.s, 63, 64)});
    hc += (uint32_t)__popcll(ch.heads);
  }
  SegPair excl, tot;
  uint32_t hexcl, htot;
  seg_waves(agg, hc, sp, sh, excl, hexcl, tot, htot);
  if (threadIdx.x == 0) {
    tile_f[blockIdx.x] = tot.f;
    tile_s[blockIdx.x] = tot.s;
    tile_h[blockIdx.x] = htot;
  }
}

// Exclusive scan over the tile aggregates (one block), in place.
__global__ __launch_bounds__(1024) void k_seg_tiles(uint32_t* __restrict__ tile_f, uint32_t* __restrict__ tile_s,
                                                    uint32_t* __restrict__ tile_h, uint32_t ntiles, const uint32_t* err) {
  __shared__ SegPair sp[1024];
  __shared__ uint32_t sh[1024];
  if (*err) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (ntiles + 1023) / 1024;
  const uint32_t s0 = tid * per, s1 = min(s0 + per, ntiles);
  SegPair v{0, 0};
  uint32_t hc = 0;
  for (uint32_t j = s0; j < s1; j++) {
    v = seg_op(v, SegPair{tile_f[j], tile_s[j]});
    hc += tile_h[j];
  }
  sp[tid] = v;
  sh[tid] = hc;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    SegPair a = v;
    uint32_t c = hc;
    if (tid >= off) {
      a = seg_op(sp[tid - off], v);
      c = sh[tid - off] + hc;
    }
    __syncthreads();
    v = a;
    hc = c;
    sp[tid] = v;
    sh[tid] = hc;
    __syncthreads();
  }
  SegPair run = tid ? sp[tid - 1] : SegPair{0, 0};
  uint32_t hrun = tid ? sh[tid - 1] : 0u;
  for (uint32_t j = s0; j < s1; j++) {
    const SegPair x{tile_f[j], tile_s[j]};
    const uint32_t xh = tile_h[j];
    tile_f[j] = run.f;
    tile_s[j] = run.s;
    tile_h[j] = hrun;
    run = seg_op(run, x);
    hrun += xh;
  }
}

__global__ __launch_bounds__(256) void k_seg_apply(const uint32_t* __restrict__ skeys,
                                                   const uint32_t* __restrict__ hits_s, uint32_t n,
                                                   const uint32_t* __restrict__ tile_f,
                                                   const uint32_t* __restrict__ tile_s,
                                                   const uint32_t* __restrict__ tile_h, uint32_t* __restrict__ segsum,
                                                   uint32_t* __restrict__ rid, uint32_t* __restrict__ run_start,
                                                   uint32_t* __restrict__ run_flags, uint32_t* num_runs,
                                                   const uint32_t* err) {
  __shared__ SegPair sp[4];
  __shared__ uint32_t sh[4];
  if (*err) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * SEG_TILE + (threadIdx.x >> 6) * SEG_STRIP + lane;
  // pass 1 (chunks kept in registers): this wave's aggregate
  SegChunk ch[SEG_ITEMS];
  SegPair agg{0, 0};
  uint32_t hc = 0;
#pragma unroll
  for (uint32_t c = 0; c < SEG_ITEMS; c++) {
    ch[c] = seg_chunk(skeys, hits_s, n, base + 64 * c);
    uint32_t t = ch[c].h;  // chunk total, segmented: sum after the last head
    const uint32_t lh = ch[c].heads ? 63u - (uint32_t)__clzll((long long)ch[c].heads) : 0u;
    if (ch[c].heads && lane < lh) t = 0;
#pragma unroll
    for (uint32_t off = 32; off; off >>= 1) t += __shfl_xor(t, off, 64);
    agg = seg_op(agg, SegPair{ch[c].heads ? 1u : 0u, t});
    hc += (uint32_t)__popcll(ch[c].heads);
  }
  SegPair excl, tot;
  uint32_t hexcl, htot;
  seg_waves(agg, hc, sp, sh, excl, hexcl, tot, htot);
  // pass 2: exclusive prefix of the wave = tile carry + earlier waves
  SegPair run = seg_op(SegPair{tile_f[blockIdx.x], tile_s[blockIdx.x]}, excl);
  uint32_t hrun = tile_h[blockIdx.x] + hexcl;
#pragma unroll
  for (uint32_t c = 0; c < SEG_ITEMS; c++) {
    const uint32_t q = base + 64 * c;
    const SegPair v = seg_chunk_scan(ch[c], lane);
    const SegPair in = seg_op(run, v);
    const uint64_t heads = ch[c].heads;
    const uint32_t r = hrun + (uint32_t)__popcll(heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1))) - 1;
    if (q < n) {
      segsum[q] = in.s;
      rid[q] = r;
      if ((heads >> lane) & 1) {
        run_start[r] = q;
        run_flags[r] = 0;
      }
      if (q == n - 1) {
        run_start[r + 1] = n;
        *num_runs = r + 1;
      }
    }
    run = seg_op(run, SegPair{__shfl(v.f, 63, 64), __shfl(v.s, 63, 64)});
    hrun += (uint32_t)__popcll(heads);
  }
}

// ---- k_segment: gather + run segmentation in one pass over the sorted order,
// tiles of SEG_TILE positions taken by ticket, decoupled look-back across
// tiles. Per sorted position q: rec_s[q] = rec[svals[q]] (one random 32-B
// read), head = q == 0 || skeys[q-1] != skeys[q], rid[q] = heads in [0, q] - 1,
// segsum[q] = inclusive in-run sum of max(1, hits) (u32, wrapping like the
// sequential INCRBYs); per run its start (flags cleared), and num_runs. A
// tile's look-back state is (heads, segmented sum): two 8-B {value, tag}
// granules that a reader accepts only when both carry the same tag and flag.
__device__ inline SegPair seg_read(const unsigned long long* st, uint32_t j, uint32_t tag, bool& ready, bool& inc,
                                   uint32_t& h) {
  const unsigned long long g0 = __hip_atomic_load(st + 2 * j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long g1 = __hip_atomic_load(st + 2 * j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t t0 = (uint32_t)(g0 >> 32), t1 = (uint32_t)(g1 >> 32);
  ready = (t0 & ~3u) == tag && t0 == t1;
  inc = ready && (t0 & OS_INC);
  h = (uint32_t)g1;
  return SegPair{h ? 1u : 0u, (uint32_t)g0};
}

__device__ inline void seg_publish(unsigned long long* st, uint32_t j, uint32_t tag, SegPair v, uint32_t h) {
  __hip_atomic_store(st + 2 * j, (unsigned long long)v.s | ((unsigned long long)tag << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(st + 2 * j + 1, (unsigned long long)h | ((unsigned long long)tag << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_segment(const Rec* __restrict__ rec, const uint32_t* __restrict__ skeys,
                                                 const uint32_t* __restrict__ svals, uint32_t n,
                                                 Rec* __restrict__ rec_s, uint32_t* __restrict__ segsum,
                                                 uint32_t* __restrict__ rid, uint32_t* __restrict__ run_start,
                                                 uint32_t* num_runs, uint32_t* __restrict__ ctr,
                                                 unsigned long long* status, uint32_t tag, const uint32_t* err) {
  __shared__ SegPair sp[4];
  __shared__ uint32_t sh[4];
  __shared__ SegPair s_pre;
  __shared__ uint32_t s_tile, s_preh;
  if (*err) return;  // the same for every block
  if (threadIdx.x == 0) s_tile = atomicAdd(ctr, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t base = tile * SEG_TILE + wave * SEG_STRIP + lane;
  // pass 1: records into sorted order; head flags and hits kept per chunk
  SegChunk ch[SEG_ITEMS];
  SegPair agg{0, 0};
  uint32_t hc = 0;
#pragma unroll
  for (uint32_t c = 0; c < SEG_ITEMS; c++) {
    const uint32_t q = base + 64 * c;
    const bool valid = q < n;
    bool head = false;
    uint32_t hv = 0;
    if (valid) {
      head = q == 0 || skeys[q - 1] != skeys[q];
      const Rec r = rec[svals[q]];
      rec_s[q] = r;
      hv = r.hits > 1 ? r.hits : 1u;
    }
    ch[c] = SegChunk{(uint64_t)__ballot(head), hv};
    uint32_t t = hv;  // chunk total, segmented: sum after the last head
    const uint32_t lh = ch[c].heads ? 63u - (uint32_t)__clzll((long long)ch[c].heads) : 0u;
    if (ch[c].heads && lane < lh) t = 0;
#pragma unroll
    for (uint32_t off = 32; off; off >>= 1) t += __shfl_xor(t, off, 64);
    agg = seg_op(agg, SegPair{ch[c].heads ? 1u : 0u, t});
    hc += (uint32_t)__popcll(ch[c].heads);
  }
  SegPair excl, tot;
  uint32_t hexcl, htot;
  seg_waves(agg, hc, sp, sh, excl, hexcl, tot, htot);
  // publish this tile's aggregate, look back for the prefix, publish the inclusive value
  if (wave == 0) {
    if (lane == 0) seg_publish(status, tile, tag | (tile ? OS_AGG : OS_INC), tot, htot);
    SegPair acc{0, 0};
    uint32_t acch = 0;
    int32_t top = (int32_t)tile - 1;
    while (top >= 0) {
      const int32_t j = top - (int32_t)lane;
      bool ready = true, inc = false;
      uint32_t h = 0;
      SegPair v{0, 0};
      if (j >= 0) v = seg_read(status, (uint32_t)j, tag, ready, inc, h);
      const uint64_t mi = __ballot(inc), mnr = __ballot(!ready);
      const uint32_t fi = mi ? (uint32_t)(__ffsll((unsigned long long)mi) - 1) : 64u;
      const uint64_t need = fi >= 63 ? ~0ull : ((2ull << fi) - 1);  // lanes 0..fi
      if (mnr & need) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      // older tiles sit in higher lanes: x = x_63 (+) ... (+) x_0 over lanes 0..fi
      SegPair x = lane <= fi ? v : SegPair{0, 0};
      uint32_t xh = lane <= fi ? h : 0u;
#pragma unroll
      for (uint32_t off = 1; off < 64; off <<= 1) {
        const SegPair y{__shfl_down(x.f, off, 64), __shfl_down(x.s, off, 64)};
        const uint32_t yh = __shfl_down(xh, off, 64);
        if (lane + off < 64) {
          x = seg_op(y, x);
          xh += yh;
        }
      }
      acc = seg_op(SegPair{__shfl(x.f, 0, 64), __shfl(x.s, 0, 64)}, acc);
      acch += __shfl(xh, 0, 64);
      if (fi < 64) break;
      top -= 64;
    }
    if (lane == 0) {
      if (tile) seg_publish(status, tile, tag | OS_INC, seg_op(acc, tot), acch + htot);
      s_pre = acc;
      s_preh = acch;
    }
  }
  __syncthreads();
  // pass 2: exclusive prefix of the wave = tiles before + earlier waves
  SegPair run = seg_op(s_pre, excl);
  uint32_t hrun = s_preh + hexcl;
#pragma unroll
  for (uint32_t c = 0; c < SEG_ITEMS; c++) {
    const uint32_t q = base + 64 * c;
    const SegPair v = seg_chunk_scan(ch[c], lane);
    const SegPair in = seg_op(run, v);
    const uint64_t heads = ch[c].heads;
    const uint32_t r = hrun + (uint32_t)__popcll(heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1))) - 1;
    if (q < n) {
      segsum[q] = in.s;
      rid[q] = r;
      if ((heads >> lane) & 1) {
        run_start[r] = q;
      }
      if (q == n - 1) {
        run_start[r + 1] = n;
        *num_runs = r + 1;
      }
    }
    run = seg_op(run, SegPair{__shfl(v.f, 63, 64), __shfl(v.s, 63, 64)});
    hrun += (uint32_t)__popcll(heads);
  }
}

// ===========================================================================
// Grouping by MSD partition + per-bucket LDS sort (stage A).
//
// k_part: every PART_TILE tile of (sort key, index) pairs, in arrival order, is
// stably partitioned by the key's top byte into its own tile region (one
// wave-ballot multisplit rank, coalesced digit segments), and publishes per
// digit its (offset, count) in the tile and the digit total. No look-back:
// bucket d is the concatenation, in tile (= arrival) order, of every tile's
// digit-d segment.
// k_bucket: one 1024-thread workgroup per top byte. It gathers its bucket,
// stably sorts it by key bits [0, 24) (three 8-bit multisplit passes in LDS;
// buckets larger than BK_CAP run the same passes chunk by chunk through HBM),
// so the batch ends up sorted by the full key with arrival order kept within
// equal keys. It then segments the bucket in place (runs never cross buckets):
// records into sorted order, in-run inclusive sums of max(1, hits), run ids
// and [run_start, run_end). Run ids are allocated per bucket from one atomic
// counter, contiguous and in sorted order within a bucket.
// ===========================================================================
constexpr uint32_t BK_WAVES = 16, BK_THREADS = 64 * BK_WAVES, BK_ITEMS = 8, BK_CAP = BK_THREADS * BK_ITEMS;
constexpr uint32_t BK_STRIP = 64 * BK_ITEMS;  // positions per wave in a chunk

// Wave-ballot multisplit: rank of each item among the wave's earlier items with
// the same digit, against a wave-private running count row in LDS (item-major
// order: item i of lane l precedes item i of lane l+1 and item i+1 of lane 0).
template <uint32_t IT>
__device__ inline void wave_multisplit(const uint32_t (&kk)[IT], uint32_t nvalid_base, uint32_t limit, uint32_t shift,
                                       uint32_t* row, uint32_t (&pos)[IT]) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lt_mask = (1ull << lane) - 1;
  uint32_t leader[IT];
  // The digit group leaders add to the row with returning LDS atomics, issued
  // back to back for all items (LDS applies them in order), then every lane
  // fetches its leader's old count.
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) {
    const bool valid = nvalid_base + i * 64 + lane < limit;
    const uint32_t d = (kk[i] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (uint32_t bit = 0; bit < 8; bit++) {
      const bool sb = (d >> bit) & 1u;
      const uint64_t bal = __ballot(sb);
      peers &= sb ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lt_mask);
    leader[i] = valid ? (uint32_t)(__ffsll((unsigned long long)peers) - 1) : lane;
    pos[i] = (valid && rank == 0) ? atomicAdd(&row[d], (uint32_t)__popcll(peers)) : 0u;
    pos[i] |= rank << 16;  // rank < 64; old counts < 2^16 (at most BK_CAP / PART_TILE)
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

__global__ __launch_bounds__(256) void k_part(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                              uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, uint32_t n,
                                              uint32_t ntiles, uint32_t* __restrict__ info, uint32_t* __restrict__ tot,
                                              const uint32_t* err) {
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t dbase[256];
  __shared__ uint32_t wsum[4];
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, tile = blockIdx.x;
  wcnt[0][tid] = 0; wcnt[1][tid] = 0; wcnt[2][tid] = 0; wcnt[3][tid] = 0;
  __syncthreads();
  const uint32_t wbase = tile * PART_TILE + wave * 64 * PART_ITEMS;
  uint32_t kk[PART_ITEMS], vv[PART_ITEMS], pos[PART_ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < PART_ITEMS; i++) {
    const uint32_t j = wbase + i * 64 + lane;
    kk[i] = j < n ? kin[j] : 0xFFFFFFFFu;
    vv[i] = j < n ? vin[j] : 0u;
  }
  wave_multisplit(kk, wbase, n, 24, wcnt[wave], pos);
  __syncthreads();
  uint32_t c = 0;
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) {
    const uint32_t t = wcnt[w][tid];
    wcnt[w][tid] = c;
    c += t;
  }
  const uint32_t excl = scan256(c, wsum, nullptr);
  dbase[tid] = excl;
  info[(size_t)tid * ntiles + tile] = (excl << 16) | c;
  if (c) atomicAdd(&tot[tid], c);
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < PART_ITEMS; i++) {
    if (wbase + i * 64 + lane < n) {
      const uint32_t d = kk[i] >> 24;
      const uint32_t p = tile * PART_TILE + dbase[d] + wcnt[wave][d] + pos[i];
      kout[p] = kk[i];
      vout[p] = vv[i];
    }
  }
}

#ifdef RL_BK_PROF  // bucketbench only: per-bucket phase stamps
__device__ unsigned long long g_bk_prof[256 * 16];
#define BK_STAMP(k) \
  if (threadIdx.x == 0) g_bk_prof[blockIdx.x * 16 + (k)] = wall_clock64()
#else
#define BK_STAMP(k)
#endif

// LDS of one k_bucket workgroup.
struct BucketLds {
  uint32_t k[BK_CAP], v[BK_CAP];      // the bucket (fast path) in sorted order
  uint32_t wcnt[BK_WAVES][256];       // multisplit rows
  uint32_t seg[MAX_PART_TILES + 1];   // bucket position where each tile's segment starts
  uint32_t src[MAX_PART_TILES];       // tile-layout index of a segment's element = src[t] + position
  uint32_t base[256];                 // digit offsets: chunk-local (fast) / running in the bucket (slow)
  uint32_t roff[3][256];              // slow path: running digit offsets per pass
  uint32_t dtot[256];
  uint32_t gsum[4][256];              // bucket_rank: digit counts per group of 4 waves
  uint32_t wsum[BK_WAVES];
  SegPair sp[BK_WAVES];
  uint32_t sh[BK_WAVES];
  SegPair carry;
  uint32_t hcarry, rb, nruns;
};

// Bucket positions -> indices in the tile layout: for each item the last tile
// t with seg[t] <= p (a segment holding p), by a fixed-depth search whose
// levels visit all items together (independent LDS reads in flight).
template <uint32_t IT>
__device__ inline void bucket_src(const BucketLds& L, uint32_t ntiles, const uint32_t (&p)[IT], uint32_t (&j)[IT]) {
  uint32_t lo[IT];
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) lo[i] = 0;
#pragma unroll
  for (uint32_t step = MAX_PART_TILES / 2; step; step >>= 1) {
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) {
      const uint32_t m = lo[i] + step;
      if (m < ntiles && L.seg[m] <= p[i]) lo[i] = m;
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) j[i] = L.src[lo[i]] + p[i];
}

// Rank one chunk (BK_ITEMS per lane, wave-strip layout) by digit [shift, shift+8):
// pos = L.base[d] + (earlier waves' count of d) + rank in the wave. With
// chunk_scan, L.base becomes the chunk's own exclusive digit offsets first.
// L.dtot = the chunk's digit counts. Ends with a barrier.
__device__ inline void bucket_rank(BucketLds& L, const uint32_t (&kk)[BK_ITEMS], uint32_t strip0, uint32_t limit,
                                   uint32_t shift, bool chunk_scan, uint32_t (&pos)[BK_ITEMS]) {
  const uint32_t tid = threadIdx.x, wave = tid >> 6;
  for (uint32_t j = tid; j < BK_WAVES * 256; j += BK_THREADS) (&L.wcnt[0][0])[j] = 0;
  __syncthreads();
  if (shift == 0 && chunk_scan) BK_STAMP(8);
  uint32_t local[BK_ITEMS];
  wave_multisplit(kk, strip0, limit, shift, L.wcnt[wave], local);
  __syncthreads();
  if (shift == 0 && chunk_scan) BK_STAMP(9);
  // per digit, exclusive offsets over the 16 wave rows: thread (g, d) scans rows
  // 4g..4g+3 of digit d, then adds the totals of the groups before g
  constexpr uint32_t G = BK_WAVES / 4;
  const uint32_t dg = tid & 255u, g = tid >> 8;
  uint32_t r[G], c = 0;
#pragma unroll
  for (uint32_t w = 0; w < G; w++) r[w] = L.wcnt[g * G + w][dg];
#pragma unroll
  for (uint32_t w = 0; w < G; w++) {
    const uint32_t t = r[w];
    r[w] = c;
    c += t;
  }
  L.gsum[g][dg] = c;
  __syncthreads();
  uint32_t pre = 0, all = 0;
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    const uint32_t t = L.gsum[q][dg];
    pre += q < g ? t : 0u;
    all += t;
  }
#pragma unroll
  for (uint32_t w = 0; w < G; w++) L.wcnt[g * G + w][dg] = r[w] + pre;
  if (tid < 256) L.dtot[tid] = all;
  const uint32_t excl = scan256(tid < 256 ? all : 0u, L.wsum, nullptr);
  if (chunk_scan && tid < 256) L.base[tid] = excl;
  __syncthreads();
  if (shift == 0 && chunk_scan) BK_STAMP(10);
#pragma unroll
  for (uint32_t i = 0; i < BK_ITEMS; i++) {
    const uint32_t d = (kk[i] >> shift) & 255u;
    pos[i] = L.base[d] + L.wcnt[wave][d] + local[i];
  }
  __syncthreads();
  if (shift == 0 && chunk_scan) BK_STAMP(11);
}

// Wave-sum of v over the block (all threads call); result in every thread.
__device__ inline uint32_t block_sum(BucketLds& L, uint32_t v) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (uint32_t off = 32; off; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) L.wsum[wave] = v;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (uint32_t w = 0; w < BK_WAVES; w++) s += L.wsum[w];
  __syncthreads();
  return s;
}

// Segment the sorted bucket [0, S) (keys/values from LDS or from the sorted
// global arrays at base): records into sorted order, in-run sums, run ids and
// run bounds. Chunks of BK_CAP positions; each wave walks its strip of the
// chunk in 64-position pieces, and the 16 wave aggregates plus the carry of
// the earlier chunks give every wave its exclusive prefix.
template <bool FROM_LDS>
__device__ inline void bucket_segment(BucketLds& L, uint32_t S, uint32_t base, const uint32_t* __restrict__ sk,
                                      const uint32_t* __restrict__ sv, const Rec* __restrict__ rec,
                                      Rec* __restrict__ rec_s, uint32_t* __restrict__ segsum,
                                      uint32_t* __restrict__ rid, uint32_t* __restrict__ run_start,
                                      uint32_t* __restrict__ run_end, uint32_t* num_runs) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto key = [&](uint32_t p) -> uint32_t { return FROM_LDS ? L.k[p] : sk[base + p]; };
  auto val = [&](uint32_t p) -> uint32_t { return FROM_LDS ? L.v[p] : sv[base + p]; };
  // runs of the bucket -> run id base
  uint32_t nh = 0;
  for (uint32_t c0 = 0; c0 < S; c0 += BK_CAP) {
    uint32_t a[BK_ITEMS], b[BK_ITEMS];
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) {  // loads first, BK_ITEMS pairs in flight
      const uint32_t p = c0 + i * BK_THREADS + tid;
      a[i] = p < S && p ? key(p - 1) : 0u;
      b[i] = p < S && p ? key(p) : 1u;
    }
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) nh += (c0 + i * BK_THREADS + tid < S && a[i] != b[i]) ? 1u : 0u;
  }
  nh = block_sum(L, nh);
  BK_STAMP(4);
  if (tid == 0) {
    L.rb = atomicAdd(num_runs, nh);
    L.nruns = nh;
    L.carry = SegPair{0, 0};
    L.hcarry = 0;
  }
  __syncthreads();
  const uint32_t rb = L.rb;
  for (uint32_t c0 = 0; c0 < S; c0 += BK_CAP) {
    const uint32_t s0 = c0 + wave * BK_STRIP;
    SegChunk ch[BK_ITEMS];
    SegPair agg{0, 0};
    uint32_t hc = 0;
    bool hd[BK_ITEMS];
    uint32_t hvs[BK_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < BK_ITEMS; j++) {  // gathers first (all in flight), scans after
      const uint32_t q = s0 + 64 * j + lane;
      hd[j] = false;
      hvs[j] = 0;
      if (q < S) {
        const uint32_t kq = key(q);
        hd[j] = q == 0 || key(q - 1) != kq;
        const Rec r = rec[val(q)];
        rec_s[base + q] = r;
        hvs[j] = r.hits > 1 ? r.hits : 1u;
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < BK_ITEMS; j++) {
      const bool head = hd[j];
      const uint32_t hv = hvs[j];
      ch[j] = SegChunk{(uint64_t)__ballot(head), hv};
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
    for (uint32_t w = 0; w < BK_WAVES; w++) {
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
    for (uint32_t j = 0; j < BK_ITEMS; j++) {
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
      }
      run = seg_op(run, SegPair{__shfl(v.f, 63, 64), __shfl(v.s, 63, 64)});
      hrun += (uint32_t)__popcll(heads);
    }
    __syncthreads();  // carry
  }
  if (tid == 0 && S) run_end[rb + L.nruns - 1] = base + S;
}

__global__ __launch_bounds__(BK_THREADS) void k_bucket(const uint32_t* __restrict__ pk, const uint32_t* __restrict__ pv,
                                                       const uint32_t* __restrict__ info,
                                                       const uint32_t* __restrict__ tot, uint32_t ntiles,
                                                       const Rec* __restrict__ rec, uint32_t* __restrict__ sk,
                                                       uint32_t* __restrict__ sv, Rec* __restrict__ rec_s,
                                                       uint32_t* __restrict__ segsum, uint32_t* __restrict__ rid,
                                                       uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_end,
                                                       uint32_t* num_runs, const uint32_t* err) {
  __shared__ BucketLds L;
  __shared__ uint32_t s_base, s_S;
  if (*err) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, d = blockIdx.x;
  BK_STAMP(0);
  {  // bucket position in the sorted batch
    const uint32_t v = tid < 256 ? tot[tid] : 0u;
    const uint32_t excl = scan256(v, L.wsum, nullptr);
    if (tid == d) {
      s_base = excl;
      s_S = v;
    }
    __syncthreads();
  }
  const uint32_t base = s_base, S = s_S;
  if (!S) return;
  // tile segments of the bucket: starts (exclusive scan of the counts) and sources
  for (uint32_t t0 = 0; t0 < ntiles; t0 += BK_THREADS) {
    const uint32_t t = t0 + tid;
    const uint32_t e = t < ntiles ? info[(size_t)d * ntiles + t] : 0u;
    const uint32_t cnt = e & 0xFFFFu;
    uint32_t inc = cnt;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(inc, off, 64);
      if (lane >= off) inc += y;
    }
    if (lane == 63) L.wsum[wave] = inc;
    __syncthreads();
    uint32_t pre = t0 ? L.seg[t0] : 0u;  // carried from the previous round
    for (uint32_t w = 0; w < wave; w++) pre += L.wsum[w];
    if (t < ntiles) {
      const uint32_t st = pre + inc - cnt;
      L.seg[t] = st;
      L.src[t] = t * PART_TILE + (e >> 16) - st;
    }
    __syncthreads();
    if (tid == BK_THREADS - 1 && t0 + BK_THREADS < ntiles) L.seg[t0 + BK_THREADS] = pre + inc;  // next round's carry
    __syncthreads();
  }
  if (tid == 0) L.seg[ntiles] = S;
  __syncthreads();
  BK_STAMP(1);
  uint32_t kk[BK_ITEMS], vv[BK_ITEMS], pos[BK_ITEMS];
  if (S <= BK_CAP) {
    // ---- fast path: the bucket lives in registers / LDS for all three passes
    const uint32_t strip0 = wave * BK_STRIP;
    uint32_t pp[BK_ITEMS], jj[BK_ITEMS];
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) pp[i] = min(strip0 + i * 64 + lane, S - 1);
    bucket_src(L, ntiles, pp, jj);
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) {
      const bool in = strip0 + i * 64 + lane < S;
      kk[i] = in ? pk[jj[i]] : 0xFFFFFFFFu;
      vv[i] = in ? pv[jj[i]] : 0u;
    }
    BK_STAMP(2);
    for (uint32_t pass = 0; pass < 3; pass++) {
      bucket_rank(L, kk, strip0, S, 8 * pass, true, pos);
#pragma unroll
      for (uint32_t i = 0; i < BK_ITEMS; i++) {
        if (strip0 + i * 64 + lane < S) {
          L.k[pos[i]] = kk[i];
          L.v[pos[i]] = vv[i];
        }
      }
      __syncthreads();
#pragma unroll
      for (uint32_t i = 0; i < BK_ITEMS; i++) {
        const uint32_t p = strip0 + i * 64 + lane;
        if (p < S) {
          kk[i] = L.k[p];
          vv[i] = L.v[p];
        }
      }
      if (pass == 0) BK_STAMP(12);
    }
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) {
      const uint32_t p = strip0 + i * 64 + lane;
      if (p < S) {
        sk[base + p] = kk[i];
        sv[base + p] = vv[i];
      }
    }
    __syncthreads();
    BK_STAMP(3);
    bucket_segment<true>(L, S, base, sk, sv, rec, rec_s, segsum, rid, run_start, run_end, num_runs);
    BK_STAMP(5);
    return;
  }
  // ---- large bucket: the same three stable passes, chunk by chunk through HBM
  // (tile layout -> sk -> temp -> sk; temp = this bucket's rid / segsum ranges,
  // which the segmentation overwrites afterwards). Running digit offsets per
  // pass come from one histogram sweep.
  for (uint32_t j = tid; j < 3 * 256; j += BK_THREADS) (&L.roff[0][0])[j] = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < S; c0 += BK_CAP) {
    uint32_t pp[BK_ITEMS], jj[BK_ITEMS];
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) pp[i] = min(c0 + i * BK_THREADS + tid, S - 1);
    bucket_src(L, ntiles, pp, jj);
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) kk[i] = pk[jj[i]];  // loads first, BK_ITEMS in flight
#pragma unroll
    for (uint32_t i = 0; i < BK_ITEMS; i++) {
      if (c0 + i * BK_THREADS + tid < S) {
        atomicAdd(&L.roff[0][kk[i] & 255u], 1u);
        atomicAdd(&L.roff[1][(kk[i] >> 8) & 255u], 1u);
        atomicAdd(&L.roff[2][(kk[i] >> 16) & 255u], 1u);
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
    const uint32_t* ik = pass == 0 ? pk : pass == 1 ? sk + base : rid + base;
    const uint32_t* iv = pass == 0 ? pv : pass == 1 ? sv + base : segsum + base;
    uint32_t* ok = pass == 1 ? rid + base : sk + base;
    uint32_t* ov = pass == 1 ? segsum + base : sv + base;
    for (uint32_t c0 = 0; c0 < S; c0 += BK_CAP) {
      const uint32_t strip0 = c0 + wave * BK_STRIP;
      uint32_t pp[BK_ITEMS], jj[BK_ITEMS];
#pragma unroll
      for (uint32_t i = 0; i < BK_ITEMS; i++) pp[i] = min(strip0 + i * 64 + lane, S - 1);
      if (pass == 0) {
        bucket_src(L, ntiles, pp, jj);
      } else {
#pragma unroll
        for (uint32_t i = 0; i < BK_ITEMS; i++) jj[i] = pp[i];
      }
#pragma unroll
      for (uint32_t i = 0; i < BK_ITEMS; i++) {
        const bool in = strip0 + i * 64 + lane < S;
        kk[i] = in ? ik[jj[i]] : 0xFFFFFFFFu;
        vv[i] = in ? iv[jj[i]] : 0u;
      }
      if (tid < 256) L.base[tid] = L.roff[pass][tid];
      bucket_rank(L, kk, strip0, S, 8 * pass, false, pos);
      if (tid < 256) L.roff[pass][tid] += L.dtot[tid];
#pragma unroll
      for (uint32_t i = 0; i < BK_ITEMS; i++) {
        if (strip0 + i * 64 + lane < S) {
          ok[pos[i]] = kk[i];
          ov[pos[i]] = vv[i];
        }
      }
    }
    __threadfence_block();
    __syncthreads();
  }
  bucket_segment<false>(L, S, base, sk, sv, rec, rec_s, segsum, rid, run_start, run_end, num_runs);
}

// Run checks against the predecessor (equality chains): a run must hold one
// stem under one unit, else it is flagged RUN_MULTI and queued once (by run
// id) for k_runs_general; a window change within a run makes a long run
// RUN_SLOW (serial replay). Run heads only compare two sort keys.
__global__ __launch_bounds__(256) void k_run_check(BatchDev b, const Rec* __restrict__ rec_s,
                                                   const uint32_t* __restrict__ skeys,
                                                   const uint32_t* __restrict__ rid,
                                                   uint32_t* __restrict__ run_flags, uint32_t* __restrict__ defer,
                                                   uint32_t* defer_n, const uint32_t* err) {
  if (*err) return;
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q == 0 || q >= b.n || skeys[q - 1] != skeys[q]) return;
  b.stem_total = b.off[b.n];
  const Rec x = rec_s[q], y = rec_s[q - 1];
  const uint32_t r = rid[q];
  const bool same = x.hlo == y.hlo && (x.lu & 0xFFFFFFu) == (y.lu & 0xFFFFFFu) &&  // hash, length, unit
                    key_equal(key_of(b, x), key_of(b, y));
  if (!same) {
    if (!(atomicOr(&run_flags[r], RUN_MULTI) & RUN_MULTI)) defer[atomicAdd(defer_n, 1u)] = r;
  } else {
    const uint32_t d = div_of(rec_unit(x));
    if (x.now / d != y.now / d) atomicOr(&run_flags[r], RUN_SLOW);
  }
}

// ---- k_runs: one lane per run of one stem and one unit (k_run_check). Short
// runs whose slot is not flagged multi-unit are replayed here in registers;
// long uniform runs are set up for the parallel path (k_fast_*); a stem that
// turns out to live in the table under another unit too is queued for the
// exact path (defer2, k_runs_general after this kernel).
__global__ __launch_bounds__(256) void k_runs(BatchDev b, TableDev t, Params P, const Rec* __restrict__ rec_s,
                                              const uint32_t* __restrict__ skeys,
                                              const uint32_t* __restrict__ svals, unsigned long long* __restrict__ res,
                                              const uint32_t* __restrict__ run_start,
                                              const uint32_t* __restrict__ run_end,
                                              uint32_t* __restrict__ run_flags, uint4* __restrict__ run_state,
                                              uint32_t* __restrict__ run_f, const uint32_t* num_runs,
                                              uint32_t* __restrict__ defer, uint32_t* defer_n,
                                              unsigned long long* stats, unsigned long long* stripes, uint32_t* err,
                                              int restore) {
  __shared__ uint32_t s_err, s_nr;
  // err may change while this kernel runs (other blocks): read it once per block
  if (threadIdx.x == 0) {
    s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_nr = *num_runs;
  }
  __syncthreads();
  if (s_err || blockIdx.x * 256 >= s_nr) return;
  b.stem_total = b.off[b.n];
  const bool use_lds = !restore && b.n_rules <= LDS_RULES;
  stats_block_begin(use_lds, b.n_rules);
  StatAcc acc{use_lds, stats};
  LaneStats L;
  L.reset();
  const uint32_t r = blockIdx.x * 256 + threadIdx.x;
  if (r < s_nr) {
    const uint32_t p = run_start[r], end = run_end[r];
    const uint32_t fl = run_flags[r];
    const Rec x0 = rec_s[p];
    const uint32_t e0 = svals[p];
    const uint64_t h0 = ((uint64_t)skeys[p] << 32) | x0.hlo;
    const uint32_t u0 = rec_unit(x0);
    SlotImg im;
    load_img(&t.slots[h0 >> t.shift], im);  // home slot, in flight beside the stem
    const Key k0 = key_of(b, x0);
    if (!(fl & RUN_MULTI)) {  // RUN_MULTI runs belong to k_runs_general
      const bool long_run = !restore && end - p >= LONG_RUN && !(fl & RUN_SLOW);
      bool ok = true;
      int64_t s0 = -1;
      bool ins = false;
      if (RL_ABL & 1) {
        s0 = (int64_t)(h0 >> t.shift);
      } else {
        s0 = find_slot_img(t, h0, slot_tag(h0, u0), k0, u0, &ins, im, err);
        if (s0 < 0) {
          ok = false;
        } else if (im.flags() & SLOT_EXACT) {
          ok = false;
        } else if (ins) {  // new (stem, unit): the stem must not exist under another unit
          for (uint32_t u = 1; u <= 4; u++) {
            bool dummy;
            const int64_t so = u == u0 ? -1 : find_slot(t, h0, slot_tag(h0, u), k0, u, false, &dummy, err);
            if (so >= 0) {  // multi-unit stem from now on: flag both before deferring
              t.slots[so].flags |= SLOT_EXACT;
              ok = false;
            }
          }
          if (!ok) t.slots[s0].flags |= SLOT_EXACT;
        }
      }
      if (ok && long_run) {
        // Parallel path: pick the window record once; k_fast_* decide every element.
        Slot* s = &t.slots[s0];
        Win cur = im.cur(), prev = im.prev();
        const Elem el0 = load_elem(x0, e0, false);
        const int which = window_pick(cur, prev, el0.w, 0, true);
        if (which < 0) {
          if (!(RL_ABL & 1)) atomicOr(err, ERR_HISTORY);  // (ablation builds probe garbage slots)
        } else {
          const Win R = which ? prev : cur;
          // A record of window w was written inside w: its EXPIRE and local-cache
          // TTL both end at or after w + div, so they hold for the whole run.
          const uint32_t c0 = el0.now <= R.expire ? R.count : 0u;
          const uint32_t F = (P.lc_en && el0.now < R.lc) ? 1u : 0u;
          s->cur = cur;
          s->prev = prev;
          run_state[r] = make_uint4((uint32_t)s0, c0, R.lc, F | ((uint32_t)which << 1));
          run_f[r] = 0xFFFFFFFFu;
          run_flags[r] = fl | RUN_FAST;
        }
      } else if (ok) {
        if (RL_ABL & 2) {
          Slot* sl = &t.slots[s0];
          Win c = im.cur();
          c.count += end - p;
          sl->cur = c;
        } else {
          replay_simple(rec_s, svals, res, t, P, nullptr, p, end, 0, s0, im.cur(), im.prev(), x0, e0, L, acc, err,
                        restore, ins ? nullptr : &im);
        }
      } else if (!(s0 < 0 && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ERR_TABLE_FULL))) {
        defer[atomicAdd(defer_n, 1u)] = r;
      }
    }
  }
  if (!(RL_ABL & 4)) {
    if (!restore) wave_flush(L, acc);
    stats_block_end(use_lds, b.n_rules, stripes);
  }
}

// ---- parallel path for long uniform runs (one stem, one unit, one window).
// Sequential replay of such a run is: count a_j = c0 + Σ_{k<=j} h_k; with the
// local cache on, the first element f with a_f > limit_f makes every element of
// a LATER request a local-cache hit (Set happens after request q_f's statuses),
// i.e. a suffix of the run, which therefore never increments.
__global__ __launch_bounds__(256) void k_fast_over(uint32_t n, const Rec* __restrict__ rec_s,
                                                   const uint32_t* __restrict__ segsum,
                                                   const uint32_t* __restrict__ rid,
                                                   const uint32_t* __restrict__ run_flags,
                                                   const uint4* __restrict__ run_state, uint32_t* __restrict__ run_f,
                                                   const uint32_t* err) {
  if (*err) return;
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  bool cand = false;
  uint32_t r = 0;
  if (q < n) {
    r = rid[q];
    if (run_flags[r] & RUN_FAST) {
      const uint4 st = run_state[r];
      if (!(st.w & 1u)) cand = st.y + segsum[q] > rec_s[q].limit;
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

__global__ __launch_bounds__(256) void k_fast_emit(uint32_t n, uint32_t n_rules, TableDev t, Params P,
                                                   const Rec* __restrict__ rec_s, const uint32_t* __restrict__ svals,
                                                   unsigned long long* __restrict__ res,
                                                   const uint32_t* __restrict__ segsum,
                                                   const uint32_t* __restrict__ rid,
                                                   const uint32_t* __restrict__ run_start,
                                                   const uint32_t* __restrict__ run_end,
                                                   const uint32_t* __restrict__ run_flags,
                                                   const uint4* __restrict__ run_state,
                                                   const uint32_t* __restrict__ run_f, unsigned long long* stats,
                                                   unsigned long long* stripes, const uint32_t* err) {
  __shared__ uint32_t s_err;
  if (threadIdx.x == 0) s_err = *err;
  __syncthreads();
  if (s_err) return;
  const bool use_lds = n_rules <= LDS_RULES;
  stats_block_begin(use_lds, n_rules);
  StatAcc acc{use_lds, stats};
  LaneStats L;
  L.reset();
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q < n) {
    const uint32_t r = rid[q];
    if (run_flags[r] & RUN_FAST) {
      const uint4 st = run_state[r];
      const uint32_t f = run_f[r];
      const bool F = st.w & 1u;
      const Elem x = load_elem(rec_s[q], svals[q], false);
      uint32_t req_f = 0xFFFFFFFFu, now_f = 0;
      if (P.lc_en && f != 0xFFFFFFFFu) {
        const Rec xf = rec_s[f];
        req_f = xf.req;
        now_f = xf.now;
      }
      const bool masked = F || x.req > req_f;  // local-cache hit
      const uint32_t after = masked ? 0u : st.y + segsum[q];
      const Decision d = decide(after - x.h, after, masked && !x.shadow, x.h, x.thr, P.ratio, x.shadow, P.lc_en);
      emit(res, L, acc, x, d);
      if (!masked) {
        const uint32_t nq = q + 1;
        const bool last = nq == run_end[r] || rec_s[nq].req > req_f;
        if (last) {  // the last INCRBY of the run leaves the key's state
          Win R;
          R.ws = x.w;
          R.count = after;
          R.expire = x.now + x.d;
          R.lc = (req_f != 0xFFFFFFFFu) ? now_f + x.d : st.z;
          Slot* s = &t.slots[st.x];
          if (st.w & 2u) s->prev = R;
          else s->cur = R;
        }
      }
    }
  }
  wave_flush(L, acc);
  stats_block_end(use_lds, n_rules, stripes);
}

// ---- k_runs_general: deferred runs (hash-prefix collisions, multi-unit
// stems). Splits the run into distinct stems, then replays each exactly.
__global__ __launch_bounds__(256) void k_runs_general(BatchDev b, TableDev t, Params P, const Rec* __restrict__ rec_s,
                                                      const uint32_t* __restrict__ skeys,
                                                      const uint32_t* __restrict__ svals,
                                                      unsigned long long* __restrict__ res,
                                                      const uint32_t* __restrict__ run_start,
                                                      const uint32_t* __restrict__ run_end,
                                                      const uint32_t* __restrict__ defer, const uint32_t* defer_n,
                                                      uint8_t* __restrict__ repid, unsigned long long* stats,
                                                      unsigned long long* stripes, uint32_t* err, int restore) {
  __shared__ uint32_t s_err, s_n;
  if (threadIdx.x == 0) {
    s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_n = *defer_n;
  }
  __syncthreads();
  if (s_err || blockIdx.x * 256 >= s_n) return;
  b.stem_total = b.off[b.n];
  const bool use_lds = !restore && b.n_rules <= LDS_RULES;
  stats_block_begin(use_lds, b.n_rules);
  StatAcc acc{use_lds, stats};
  LaneStats L;
  L.reset();
  // Grid-stride over the deferred runs: the grid is small and fixed (deferrals
  // are rare), so an empty deferral list costs one short launch.
  for (uint32_t di = blockIdx.x * 256 + threadIdx.x; di < s_n; di += gridDim.x * 256) {
    const uint32_t rr = defer[di];  // run id
    const uint32_t p = run_start[rr], end = run_end[rr];
    const uint32_t key = skeys[p];
    // ---- split the run into distinct stems (hash, then bytes)
    uint32_t rep[MAX_REPS];
    uint32_t umask[MAX_REPS];
    uint32_t nrep = 1;
    rep[0] = p;
    umask[0] = 1u << (rec_unit(rec_s[p]) - 1);
    for (uint32_t q = p + 1; q < end; q++) {
      const Rec x = rec_s[q];
      const Key kx = key_of(b, x);
      uint32_t k = 0;
      for (; k < nrep; k++) {
        const Rec y = rec_s[rep[k]];
        if (y.hlo == x.hlo && rec_len(y) == rec_len(x) && key_equal(key_of(b, y), kx)) break;
      }
      if (k == nrep) {
        if (nrep == MAX_REPS) { atomicOr(err, ERR_COLLISIONS); k = 0; }
        else { rep[nrep] = q; umask[nrep] = 0; nrep++; }
      }
      repid[q] = (uint8_t)k;
      umask[k] |= 1u << (rec_unit(x) - 1);
    }
    for (uint32_t k = 0; k < nrep; k++) {
      const Rec y = rec_s[rep[k]];
      const Key stem = key_at(b, rec_s, rep[k]);
      const uint64_t hs = ((uint64_t)key << 32) | y.hlo;
      // ---- resolve the slot(s)
      bool simple = false;
      int64_t s0 = -1;
      if (__popc(umask[k]) == 1) {
        const uint32_t u0 = __ffs(umask[k]);
        bool ins;
        s0 = find_slot(t, hs, slot_tag(hs, u0), stem, u0, true, &ins, err);
        if (s0 < 0) break;
        if (!(t.slots[s0].flags & SLOT_EXACT)) {
          simple = true;
          if (ins) {  // new (stem, unit): the stem must not exist under another unit
            for (uint32_t u = 1; u <= 4 && simple; u++) {
              bool dummy;
              if (u != u0 && find_slot(t, hs, slot_tag(hs, u), stem, u, false, &dummy, err) >= 0) simple = false;
            }
          }
        }
      }
      if (simple) {
        // (the run's stem k starts at rep[k], not necessarily at p)
        replay_simple(rec_s, svals, res, t, P, repid, rep[k], end, k, s0, t.slots[s0].cur, t.slots[s0].prev,
                      rec_s[rep[k]], svals[rep[k]], L, acc, err, restore);
      } else {
        GeneralState G;
        G.present = 0;
        G.cur_req = 0xFFFFFFFFu;
        G.npend = 0;
        bool fail = false;
        for (uint32_t u = 1; u <= 4; u++) {
          bool ins;
          G.sidx[u - 1] = find_slot(t, hs, slot_tag(hs, u), stem, u, (umask[k] >> (u - 1)) & 1, &ins, err);
          if (G.sidx[u - 1] >= 0) {
            G.present |= 1u << (u - 1);
            G.cur[u - 1] = t.slots[G.sidx[u - 1]].cur;
            G.prev[u - 1] = t.slots[G.sidx[u - 1]].prev;
          } else if ((umask[k] >> (u - 1)) & 1) {
            fail = true;
          }
        }
        if (fail) break;
        for (uint32_t q = p; q < end; q++) {
          if (((q == p) ? 0u : repid[q]) != k) continue;
          general_step(P, res, L, acc, G, load_elem(rec_s[q], svals[q], restore), restore, err);
        }
        general_apply_pending(G);
        const uint8_t fl = __popc(G.present) >= 2 ? SLOT_EXACT : 0;
        for (uint32_t u = 0; u < 4; u++) {
          if (!(G.present >> u & 1)) continue;
          Slot* s = &t.slots[G.sidx[u]];
          s->cur = G.cur[u];
          s->prev = G.prev[u];
          s->flags |= fl;
        }
      }
    }
  }
  if (!restore) wave_flush(L, acc);
  stats_block_end(use_lds, b.n_rules, stripes);
}

// First kernel of the table stage: merge this batch's validation errors into
// the sticky table-stage word, clear k_runs' deferral counter and this call's
// output stats (n_rules x RL_NUM_STATS).
__global__ __launch_bounds__(256) void k_b_begin(const uint32_t* __restrict__ erra, uint32_t* errb,
                                                 uint32_t* __restrict__ defer_n,
                                                 unsigned long long* __restrict__ stats, uint32_t m) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) {
    const uint32_t e = *erra;
    if (e) atomicOr(errb, e);
    *defer_n = 0;
  }
  for (uint32_t j = i; j < m; j += gridDim.x * 256) stats[j] = 0;
}

// Last kernel of a batch: packed results -> the three rl_result arrays
// (arrival order, coalesced), and the first n_fold x RL_NUM_STATS threads fold
// the striped per-block stats into rl_result.stats (clearing the stripes even
// when the batch failed, so nothing leaks into the next one).
__global__ __launch_bounds__(256) void k_finish(const unsigned long long* __restrict__ res, uint32_t n, OutDev o,
                                                unsigned long long* __restrict__ stripes, uint32_t n_fold,
                                                const uint32_t* err) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
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
  if (!ok || i >= n) return;
  const unsigned long long v = res[i];
  o.code[i] = (uint8_t)(v >> 56);
  o.rem[i] = (uint32_t)v;
  o.reset[i] = (uint32_t)(v >> 32) & 0xFFFFFFu;
}

// ===========================================================================
// Epoch sweep: a slot whose window records are all dead (Redis key past its
// EXPIRE and local-cache entry past its TTL) becomes a tombstone.
// ===========================================================================
__device__ inline bool win_alive(const Win& w, uint32_t now) {
  return w.ws != WS_INVALID && (now <= w.expire || now < w.lc);
}

__global__ __launch_bounds__(256) void k_sweep(Slot* slots, uint64_t nslots, uint32_t now,
                                               unsigned long long* evicted) {
  uint32_t local = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * 256) {
    Slot* s = &slots[i];
    if (s->tag < 2) continue;
    if (!win_alive(s->cur, now) && !win_alive(s->prev, now)) {
      s->tag = TAG_TOMB;
      local++;
    }
  }
  if (local) atomicAdd(evicted, (unsigned long long)local);
}

__global__ __launch_bounds__(256) void k_table_info(const Slot* slots, uint64_t nslots, unsigned long long* out) {
  uint32_t live = 0, tomb = 0, exact = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * 256) {
    const uint64_t tg = slots[i].tag;
    if (tg == TAG_TOMB) tomb++;
    else if (tg >= 2) { live++; if (slots[i].flags & SLOT_EXACT) exact++; }
  }
  if (live) atomicAdd(&out[0], (unsigned long long)live);
  if (tomb) atomicAdd(&out[1], (unsigned long long)tomb);
  if (exact) atomicAdd(&out[2], (unsigned long long)exact);
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

// Stage A (table-free): validate, hash, sort, gather, segment. Uses only this
// buffer's scratch and its validation word s.err.
void launch_stage_a(const BatchDev& b, const Scratch& s, uint32_t epoch, hipStream_t st, hipEvent_t* ev) {
  const uint32_t g0 = cdiv(b.n > b.n_req ? b.n : b.n_req, 256);
  if (ev) (void)hipEventRecord(ev[0], st);
  if (g0)
    k_prepare<<<g0, 256, 0, st>>>(b, s.rec, s.keys[0], s.vals[0], s.err, s.time_floor, s.defer_n, s.os_ghist,
                                  s.os_ctr, s.run_flags, s.num_runs);
  if (ev) (void)hipEventRecord(ev[1], st);
  const uint32_t ptiles = cdiv(b.n, PART_TILE);
  if (b.n) k_part<<<ptiles, 256, 0, st>>>(s.keys[0], s.vals[0], s.keys[1], s.vals[1], b.n, ptiles, s.part_info,
                                         s.os_ghist, s.err);
  if (ev) (void)hipEventRecord(ev[2], st);
  if (b.n) {
    k_bucket<<<256, BK_THREADS, 0, st>>>(s.keys[1], s.vals[1], s.part_info, s.os_ghist, ptiles, s.rec, s.keys[0],
                                         s.vals[0], s.rec_s, s.segsum, s.rid, s.run_start, s.run_end, s.num_runs,
                                         s.err);
    k_run_check<<<cdiv(b.n, 256), 256, 0, st>>>(b, s.rec_s, s.keys[0], s.rid, s.run_flags, s.defer, s.defer_n,
                                                s.err);
  }
}

// Stage B (the table): runs strictly in batch order. Every kernel reads the
// sticky table-stage word s.errb; k_b_begin folds this batch's validation
// result into it first.
void launch_stage_b(const BatchDev& b, const OutDev& o, const TableDev& t, const Params& P, const Scratch& s,
                    int restore, hipStream_t st, hipStream_t side, hipEvent_t go, hipEvent_t side_done,
                    hipEvent_t* ev) {
  const uint32_t m = restore ? 0u : b.n_rules * RL_NUM_STATS;
  const uint32_t gb = m ? (cdiv(m, 256) < 64 ? cdiv(m, 256) : 64) : 1;
  k_b_begin<<<gb, 256, 0, st>>>(s.err, s.errb, s.defer2_n, o.stats, m);
  if (b.n) {
    const uint32_t g = cdiv(b.n, 256);
    const size_t lds = (!restore && b.n_rules <= LDS_RULES) ? (size_t)b.n_rules * RL_NUM_STATS * 8 : 0;
    // RUN_MULTI runs (known since k_run_check) on the side stream, beside k_runs
    (void)hipEventRecord(go, st);
    (void)hipStreamWaitEvent(side, go, 0);
    k_runs_general<<<g < RUNS_GENERAL_BLOCKS ? g : RUNS_GENERAL_BLOCKS, 256, lds, side>>>(
        b, t, P, s.rec_s, s.keys[0], s.vals[0], s.res, s.run_start, s.run_end, s.defer, s.defer_n, s.repid, o.stats, s.stripes,
        s.errb, restore);
    (void)hipEventRecord(side_done, side);
    if (ev) (void)hipEventRecord(ev[3], st);
    k_runs<<<g, 256, lds, st>>>(b, t, P, s.rec_s, s.keys[0], s.vals[0], s.res, s.run_start, s.run_end, s.run_flags,
                                s.run_state, s.run_f, s.num_runs, s.defer2, s.defer2_n, o.stats, s.stripes, s.errb,
                                restore);
    if (ev) (void)hipEventRecord(ev[4], st);
    // stems k_runs found under several units in the table (rare)
    k_runs_general<<<RUNS_GENERAL_LATE_BLOCKS, 256, lds, st>>>(b, t, P, s.rec_s, s.keys[0], s.vals[0],
                                                                s.res, s.run_start, s.run_end, s.defer2, s.defer2_n, s.repid, o.stats,
                                                                s.stripes, s.errb, restore);
    (void)hipStreamWaitEvent(st, side_done, 0);
    if (!restore) {
      if (P.lc_en)
        k_fast_over<<<g, 256, 0, st>>>(b.n, s.rec_s, s.segsum, s.rid, s.run_flags, s.run_state, s.run_f, s.errb);
      k_fast_emit<<<g, 256, lds, st>>>(b.n, b.n_rules, t, P, s.rec_s, s.vals[0], s.res, s.segsum, s.rid,
                                       s.run_start, s.run_end, s.run_flags, s.run_state, s.run_f, o.stats, s.stripes, s.errb);
      const uint32_t nf = b.n_rules <= LDS_RULES ? b.n_rules : 0u;
      const uint32_t gf = cdiv(nf * RL_NUM_STATS > b.n ? nf * RL_NUM_STATS : b.n, 256);
      k_finish<<<gf, 256, 0, st>>>(s.res, b.n, o, s.stripes, nf, s.errb);
    }
  } else if (ev) {
    (void)hipEventRecord(ev[3], st);
    (void)hipEventRecord(ev[4], st);
  }
  if (ev) (void)hipEventRecord(ev[5], st);
}

void launch_partition(const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout, uint32_t n,
                      const Scratch& s, hipStream_t st) {
  if (!n) return;
  const uint32_t ntiles = cdiv(n, RS_TILE);
  k_rs_hist<<<ntiles, 256, 0, st>>>(kin, n, 0, ntiles, s.hist, s.err);
  k_rs_rowscan<<<256, 256, 0, st>>>(s.hist, ntiles, s.hist_tot, s.err);
  k_rs_scatter<<<ntiles, 256, 0, st>>>(kin, vin, kout, vout, n, 0, ntiles, s.hist, s.hist_tot, s.err);
}

void launch_run_sums(const uint32_t* skeys, const uint32_t* w, uint32_t n, const Scratch& s, hipStream_t st) {
  if (!n) return;
  const uint32_t nt = cdiv(n, SEG_TILE);
  k_seg_reduce<<<nt, 256, 0, st>>>(skeys, w, n, s.tile_f, s.tile_s, s.tile_h, s.err);
  k_seg_tiles<<<1, 1024, 0, st>>>(s.tile_f, s.tile_s, s.tile_h, nt, s.err);
  k_seg_apply<<<nt, 256, 0, st>>>(skeys, w, n, s.tile_f, s.tile_s, s.tile_h, s.segsum, s.rid, s.run_start,
                                  s.run_flags, s.num_runs, s.err);
}

void launch_sweep(Slot* slots, uint64_t nslots, uint32_t now, unsigned long long* evicted, hipStream_t st) {
  k_sweep<<<2048, 256, 0, st>>>(slots, nslots, now, evicted);
}

void launch_table_info(const Slot* slots, uint64_t nslots, unsigned long long* out, hipStream_t st) {
  k_table_info<<<2048, 256, 0, st>>>(slots, nslots, out);
}

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
