// rl_route.hip — multi-GPU routing of a batch to the GPUs that own its keys
// (hash-sharded table). The exchange itself is two RCCL
// all_to_all calls issued by the host (ratelimit_amd/sharded.py); these
// kernels do the device-side halves around it:
//
//   source: hash -> owner, stable partition by owner (one 8-bit counting
//           pass), per-owner stem offsets (segmented sums), pack 32-B wire
//           records + stem bytes in owner order;
//   owner:  unpack the received chunks (concatenated in source-rank order =
//           global arrival order) into a batch with per-descriptor `now` and
//           request labels, run the normal DoLimit pipeline;
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
__global__ __launch_bounds__(256) void k_route_prep(BatchDev b, uint32_t n_shards, uint32_t* __restrict__ dest,
                                                    uint32_t* __restrict__ idx, uint32_t* err) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n) return;
  const uint32_t s0 = b.off[i], s1 = b.off[i + 1], total = b.off[b.n];
  // Only a malformed layout fails the partition; a bad unit, rule id or clock
  // is the owner's to judge (per-descriptor status, or the batch's error).
  const uint32_t q = b.req[i];
  const bool bad = q >= ROUTE_MAX_REQ || (i && b.req[i - 1] > q) || s1 <= s0 ||
                   s1 - s0 > 65535 || total > b.stem_cap || s1 > total || q >= b.n_req;
  uint64_t h = 0;
  if (bad) {
    atomicOr(err, ERR_INVALID);
  } else {
    const uint32_t* words = reinterpret_cast<const uint32_t*>(b.stem);
    h = hash_stem(b.hk, DwordReader{words + (s0 >> 2), ((total + 3u) >> 2) - (s0 >> 2)}, s0 & 3u, s1 - s0);
  }
  dest[i] = bad ? 0u : owner_of(h, n_shards);
  idx[i] = i;
}

__global__ __launch_bounds__(256) void k_route_lens(const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ perm, uint32_t n,
                                                    uint32_t* __restrict__ lens_s, const uint32_t* err) {
  if (*err) return;
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const uint32_t e = perm[j];
  lens_s[j] = off[e + 1] - off[e];
}

// Per owner: record count (partition digit totals) and stem bytes (the in-run
// sum at the owner's last record); stem_start = exclusive prefix of the bytes.
// All zero when the batch failed validation, so the exchange stays well-formed.
__global__ void k_route_counts(const uint32_t* __restrict__ digit_tot, const uint32_t* __restrict__ segsum,
                               uint32_t n_shards, uint32_t* __restrict__ stem_start,
                               unsigned long long* __restrict__ counts, const uint32_t* err) {
  if (threadIdx.x != 0) return;
  const bool ok = *err == 0;
  uint32_t rec = 0, sb = 0;
  for (uint32_t d = 0; d < n_shards; d++) {
    const uint32_t c = ok ? digit_tot[d] : 0u;
    const uint32_t bytes = c ? segsum[rec + c - 1] : 0u;
    counts[2 * d] = c;
    counts[2 * d + 1] = bytes;
    stem_start[d] = sb;
    rec += c;
    sb += bytes;
  }
  stem_start[n_shards] = sb;
}

__global__ __launch_bounds__(256) void k_route_pack(BatchDev b, const uint32_t* __restrict__ perm,
                                                    const uint32_t* __restrict__ sdest,
                                                    const uint32_t* __restrict__ segsum,
                                                    const uint32_t* __restrict__ lens_s,
                                                    const uint32_t* __restrict__ stem_start, uint32_t src_rank,
                                                    Wire* __restrict__ out, uint8_t* __restrict__ out_stem,
                                                    const uint32_t* err) {
  if (*err) return;
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= b.n) return;
  const uint32_t e = perm[j], len = lens_s[j];
  const uint32_t local = segsum[j] - len;  // byte offset inside the owner's chunk
  const uint32_t q = b.req[e];
  Wire w;
  w.label = (src_rank << ROUTE_REQ_BITS) | q;
  w.off = local;
  w.lu = len | ((uint32_t)b.unit[e] << 16) | ((uint32_t)b.flags[e] << 24);
  w.limit = b.limit[e];
  w.hits = b.hits[e];
  w.rule = b.rule[e];
  w.now = b.now[q];
  out[j] = w;
  const uint8_t* src = b.stem + b.off[e];
  uint8_t* dst = out_stem + stem_start[sdest[j]] + local;
  for (uint32_t k = 0; k < len; k++) dst[k] = src[k];
}

__global__ __launch_bounds__(256) void k_route_scatter(const uint32_t* __restrict__ perm,
                                                       const unsigned long long* __restrict__ ret, uint32_t n,
                                                       OutDev o, uint32_t* src_err) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const uint32_t e = perm[j];
  const unsigned long long v = ret[j];
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

// ---- owner side -----------------------------------------------------------
// Received records -> batch arrays. Chunks arrive in source-rank order, each
// with its stems contiguous in record order, so consecutive records' stems
// must abut (checked: a malformed exchange is RL_E_INVALID, never a wrong key).
// rule_stride > 0: per-source stats, rule' = source x rule_stride + rule.
__global__ __launch_bounds__(256) void k_route_unpack(const Wire* __restrict__ rec, uint32_t n,
                                                      const unsigned long long* __restrict__ base,
                                                      uint32_t n_shards, uint64_t stem_bytes, uint32_t rule_stride,
                                                      BatchOut bo, uint32_t* err) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const Wire w = rec[j];
  const uint32_t src = w.label >> ROUTE_REQ_BITS, len = w.lu & 0xFFFFu;
  bool bad = src >= n_shards;
  const uint64_t o = (bad ? 0ull : base[src]) + w.off;
  if (j + 1 < n) {
    const Wire x = rec[j + 1];
    const uint32_t s2 = x.label >> ROUTE_REQ_BITS;
    bad = bad || s2 >= n_shards || (s2 >= n_shards ? true : base[s2] + x.off != o + len) || x.label < w.label;
  } else {
    bad = bad || o + len > stem_bytes;
    bo.off[n] = (uint32_t)(o + len);
  }
  if (bad) atomicOr(err, ERR_INVALID);
  bo.off[j] = (uint32_t)o;
  bo.now[j] = w.now;
  bo.req[j] = w.label;
  bo.unit[j] = (uint8_t)(w.lu >> 16);
  bo.flags[j] = (uint8_t)(w.lu >> 24);
  bo.limit[j] = w.limit;
  bo.hits[j] = w.hits;
  // (a rule id past the stride stays out of range for the owner's validation)
  bo.rule[j] = !rule_stride ? w.rule : w.rule >= rule_stride ? 0xFFFFFFFFu : (bad ? 0u : src) * rule_stride + w.rule;
}

// Per-rule stats deltas of several owners (blocks of m counters) summed into out.
__global__ __launch_bounds__(256) void k_stats_sum(const unsigned long long* __restrict__ stage, uint32_t n_blocks,
                                                   uint32_t m, unsigned long long* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  unsigned long long s = 0;
  for (uint32_t b = 0; b < n_blocks; b++) s += stage[(size_t)b * m + i];
  out[i] = s;
}

}  // namespace

void launch_stats_sum(const unsigned long long* stage, uint32_t n_blocks, uint32_t m, unsigned long long* out,
                      hipStream_t st) {
  if (m) k_stats_sum<<<cdiv(m, 256), 256, 0, st>>>(stage, n_blocks, m, out);
}

void launch_route_pack(const BatchDev& b, uint32_t n_shards, uint32_t src_rank, Wire* out, uint8_t* out_stem,
                       uint32_t* perm, unsigned long long* counts, const Scratch& s, hipStream_t st) {
  const uint32_t g = cdiv(b.n, 256);
  if (b.n) {
    k_route_prep<<<g, 256, 0, st>>>(b, n_shards, s.keys[0], s.vals[0], s.err);
    launch_partition(s.keys[0], s.vals[0], s.keys[1], perm, b.n, s, st);
    k_route_lens<<<g, 256, 0, st>>>(b.off, perm, b.n, s.hits_s, s.err);
    launch_run_sums(s.keys[1], s.hits_s, b.n, s, st);
  } else {
    (void)hipMemsetAsync(s.hist_tot, 0, 256 * sizeof(uint32_t), st);
  }
  k_route_counts<<<1, 64, 0, st>>>(s.hist_tot, s.segsum, n_shards, s.route_start, counts, s.err);
  if (b.n)
    k_route_pack<<<g, 256, 0, st>>>(b, perm, s.keys[1], s.segsum, s.hits_s, s.route_start, src_rank, out, out_stem,
                                    s.err);
}

void launch_route_unpack(const Wire* rec, uint32_t n, const unsigned long long* base, uint32_t n_shards,
                         uint64_t stem_bytes, uint32_t rule_stride, const BatchOut& bo, uint32_t* err, hipStream_t st) {
  if (n) k_route_unpack<<<cdiv(n, 256), 256, 0, st>>>(rec, n, base, n_shards, stem_bytes, rule_stride, bo, err);
}

void launch_route_scatter(const uint32_t* perm, const unsigned long long* ret, uint32_t n, const OutDev& o,
                          hipStream_t st, uint32_t* src_err) {
  if (n) k_route_scatter<<<cdiv(n, 256), 256, 0, st>>>(perm, ret, n, o, src_err);
}

void launch_route_ret(const unsigned long long* res, uint32_t n, const uint32_t* errb, unsigned long long* ret,
                      hipStream_t st) {
  if (n) k_route_ret<<<cdiv(n, 256), 256, 0, st>>>(res, n, errb, ret);
}

}  // namespace rl
