// rl_match.hip — the request path on the device: the service's GetLimit per
// descriptor (src/config/config_impl.go:243-298, called from
// constructLimitsToCheck, src/service/ratelimit.go:104-143), compaction of
// the matched descriptors into the DoLimit batch (the nil / unlimited ones
// never reach DoLimit, ratelimit.go:140-143 and base_limiter.go:78-81), and
// the per-descriptor answer of shouldRateLimitWorker (ratelimit.go:176-190).
//
// k_match: one lane per descriptor. The config trie is an open-addressing
// index of (parent node, key bytes) -> node, a few KB that stays in L2; the
// walk is GetLimit's loop: look up "key_value", else "key"; a node with a
// limit answers only at the descriptor's last entry; descend while the node
// has children. Matched descriptors get a stem length; a device-wide scan of
// (matched << 40 | stem bytes) gives each its slot in the compacted batch and
// k_match_emit writes the DoLimit arrays and the stem
//   prefix ‖ domain ‖ '_' ‖ Σ(key ‖ '_' ‖ value ‖ '_')   (cache_key.go:62-71)
// (the descriptor's entry bytes already are the tail). k_match_expand maps the
// DoLimit results back to every descriptor.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "../../include/ratelimit_hip.h"
#include "rl_match.h"

namespace rl {

namespace {

constexpr uint32_t MT = 256;                // descriptors per workgroup
constexpr uint32_t IN_WORDS = 8192 / 4;     // entry bytes staged per workgroup (LDS; 32 B per descriptor)
constexpr uint32_t OUT_WORDS = 12288 / 4;   // stem bytes assembled per workgroup (LDS; 48 B per descriptor)
constexpr unsigned long long M40 = (1ull << 40) - 1;

// Byte sources for the walk: the workgroup's entry bytes staged in LDS
// (coalesced dword loads), or global memory when a workgroup's bytes do not fit.
struct LdsBytes {
  const uint8_t* p;  // LDS copy of [base & ~3, ...)
  uint32_t base;
  __device__ __forceinline__ uint8_t operator[](uint32_t i) const { return p[i - base]; }
};
struct GlobalBytes {
  const uint8_t* p;
  __device__ __forceinline__ uint8_t operator[](uint32_t i) const { return p[i]; }
};

// Stage bytes [a, b) of a 4-byte aligned buffer into LDS words (word 0 = byte a & ~3).
// Reads may run up to 3 bytes past b (the buffers are padded).
__device__ __forceinline__ void stage_words(const uint8_t* src, uint32_t a, uint32_t b, uint32_t* lds) {
  const uint32_t w0 = a >> 2, nw = ((b + 3) >> 2) - w0;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src) + w0;
  for (uint32_t i = threadIdx.x; i < nw; i += MT) lds[i] = s32[i];
}

template <class R>
__device__ __forceinline__ uint64_t hash_r(int32_t parent, const R& rd, uint32_t a, uint32_t len) {
  uint64_t h = 0xcbf29ce484222325ull ^ ((uint64_t)(uint32_t)(parent + 1) * 0x9E3779B97F4A7C15ull);
  for (uint32_t i = 0; i < len; i++) {
    h ^= rd[a + i];
    h *= 0x100000001b3ull;
  }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h;  // == cfg_hash over the same bytes
}

// rateLimitDescriptor.descriptors[key] lookup (a Go map of finalKey) at `parent`
// (-1: the domains map, config_impl.go:247). Collision-exact.
template <class R>
__device__ __forceinline__ int32_t cfg_find(const CfgDev& c, int32_t parent, const R& rd, uint32_t a, uint32_t len) {
  const uint64_t h = hash_r(parent, rd, a, len);
  const uint32_t tag = (uint32_t)(h >> 32);
  uint32_t pos = (uint32_t)h & c.mask;
  for (uint32_t i = 0; i <= c.mask; i++) {
    const unsigned long long e = c.index[pos];
    if (!e) return -1;
    if ((uint32_t)e == tag) {
      const uint32_t nd = (uint32_t)(e >> 32) - 1u;
      const CfgNode& N = c.nodes[nd];
      if (N.parent == parent && N.key_len == len) {
        uint32_t k = 0;
        while (k < len && c.keys[N.key_off + k] == rd[a + k]) k++;
        if (k == len) return (int32_t)nd;
      }
    }
    pos = (pos + 1) & c.mask;
  }
  return -1;
}

// GetLimit's walk (config_impl.go:268-295) over the entries [e0, e1) whose
// bytes start at b0: look up "key_value", else "key"; a node with a limit
// answers only at the last entry; descend while the node has children.
template <class R>
__device__ __forceinline__ int32_t walk(const CfgDev& c, const ReqDev& r, int32_t root, const R& rd, uint32_t b0,
                                        uint32_t e0, uint32_t e1) {
  int32_t node = root, hit = -1;
  uint32_t p = b0;
  for (uint32_t e = e0; e < e1; e++) {
    const uint32_t kl = r.klen[e], vl = r.vlen[e];
    int32_t nx = cfg_find(c, node, rd, p, kl + 1u + vl);  // key_value
    if (nx < 0) nx = cfg_find(c, node, rd, p, kl);        // key
    if (nx >= 0 && c.nodes[nx].has_limit && e == e1 - 1) hit = nx;
    if (nx >= 0 && c.nodes[nx].n_children) node = nx;
    else break;
    p += kl + vl + 2u;
  }
  return hit;
}

// Whether a workgroup's byte range [a, b) is well formed and fits `cap` LDS words.
__device__ __forceinline__ bool fits(uint32_t a, uint32_t b, uint32_t total, uint32_t cap) {
  return a <= b && b <= total && ((b + 3) >> 2) - (a >> 2) <= cap;
}

__global__ __launch_bounds__(MT) void k_match(CfgDev cg, ReqDev r, MatchBuf m) {
  __shared__ uint32_t s_in[IN_WORDS];
  extern __shared__ __attribute__((aligned(16))) uint32_t s_cfg[];  // cg.blob_words (dynamic: only what the config needs)
  const uint32_t d0 = blockIdx.x * MT, d1 = min(d0 + MT, r.n_desc);
  const uint32_t ba = r.desc_off[d0], bb = r.desc_off[d1];
  const bool staged = fits(ba, bb, r.desc_total, IN_WORDS);
  if (staged) stage_words(r.desc, ba, bb, s_in);
  // a small config (the usual case: a few KB) is walked from LDS
  CfgDev c = cg;
  if (cg.blob_words) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(cg.blob);
    for (uint32_t i = threadIdx.x; i < cg.blob_words; i += MT) s_cfg[i] = src[i];
    c.nodes = reinterpret_cast<const CfgNode*>(s_cfg);
    c.index = reinterpret_cast<const unsigned long long*>(s_cfg + cg.idx_word);
    c.prefix = reinterpret_cast<const uint8_t*>(s_cfg + cg.key_word);
    c.keys = c.prefix + cg.prefix_len;
  }
  __syncthreads();
  const uint32_t d = d0 + threadIdx.x;
  if (d >= d1) return;
  const uint32_t q = r.req[d];
  uint32_t kind = RL_MATCH_NONE, rpu = 0, rule = 0, unit = 0, shadow = 0;
  unsigned long long v = 0;
  const uint32_t e0 = r.ent_first[d], e1 = r.ent_first[d + 1];
  const uint32_t b0 = r.desc_off[d], b1 = r.desc_off[d + 1];
  bool bad = q >= r.n_req || e1 < e0 || e1 > r.n_ent || b1 < b0 || b1 > r.desc_total ||
             (staged && (b0 < ba || b1 > bb));
  if (!bad) bad = r.dom_off[q + 1] < r.dom_off[q] || r.dom_off[q + 1] > r.dom_total;
  if (!bad) {
    // entry byte layout: Σ(key ‖ '_' ‖ value ‖ '_') must fill [b0, b1)
    uint64_t tot = 0;
    for (uint32_t e = e0; e < e1; e++) tot += (uint64_t)r.klen[e] + r.vlen[e] + 2u;
    bad = tot != (uint64_t)(b1 - b0);
  }
  if (bad) {
    atomicOr(m.count + 2, MATCH_ERR_REQ);
  } else {
    const uint32_t da = r.dom_off[q], dl = r.dom_off[q + 1] - da;
    const int32_t root = cfg_find(c, -1, GlobalBytes{r.dom}, da, dl);  // this.domains[domain] (:247)
    if (root >= 0) {
      if (r.ovf && (r.ovf[d] & 1u)) {  // descriptor.GetLimit() != nil (:254-266): never shadow
        kind = RL_MATCH_LIMIT;
        rpu = r.ov_rpu[d];
        unit = r.ov_unit[d];
        rule = r.ov_rule[d];
      } else {
        const int32_t hit = staged ? walk(c, r, root, LdsBytes{(const uint8_t*)s_in, ba & ~3u}, b0, e0, e1)
                                   : walk(c, r, root, GlobalBytes{r.desc}, b0, e0, e1);
        if (hit >= 0) {
          const CfgNode& N = c.nodes[hit];
          kind = N.unlimited ? RL_MATCH_UNLIMITED : RL_MATCH_LIMIT;
          rpu = N.rpu;
          unit = N.unit;
          rule = N.rule;
          shadow = N.shadow;
        }
      }
      if (kind == RL_MATCH_LIMIT) v = (1ull << 40) | (uint64_t)(c.prefix_len + dl + 1u + (b1 - b0));
    }
  }
  m.v[d] = v;
  m.kind[d] = kind | unit << 8 | shadow << 16;
  m.rpu[d] = rpu;
  m.rule[d] = rule;
}

// s = inclusive scan of m.v. Matched descriptor d goes to position
// (s[d] >> 40) - 1 with its stem at byte (s[d] - v[d]) & (2^40 - 1). A
// workgroup's stems are contiguous in the output: they are assembled in LDS
// and written with coalesced dword stores (byte stores at the two ends, which
// neighbouring workgroups share).
__global__ __launch_bounds__(MT) void k_match_emit(CfgDev c, ReqDev r, MatchBuf m,
                                                   const unsigned long long* __restrict__ s, PackOut o) {
  __shared__ uint32_t s_in[IN_WORDS];
  __shared__ uint32_t s_out[OUT_WORDS];
  const uint32_t d0 = blockIdx.x * MT, d1 = min(d0 + MT, r.n_desc);
  const uint32_t ba = r.desc_off[d0], bb = r.desc_off[d1];
  const bool staged = fits(ba, bb, r.desc_total, IN_WORDS);
  const unsigned long long oa = (s[d0] - m.v[d0]) & M40, ob = s[d1 - 1] & M40;
  const bool assembled = ob <= o.stem_cap && ((ob + 3) >> 2) - (oa >> 2) <= OUT_WORDS;
  if (staged) stage_words(r.desc, ba, bb, s_in);
  __syncthreads();
  const uint32_t d = d0 + threadIdx.x;
  if (d < d1) {
    const unsigned long long incl = s[d], v = m.v[d];
    if (d == r.n_desc - 1) {
      const uint32_t cnt = (uint32_t)(incl >> 40);
      const unsigned long long tot = incl & M40;
      m.count[0] = cnt;
      m.count[1] = (uint32_t)(tot < 0xFFFFFFFFull ? tot : 0xFFFFFFFFull);
      if (tot > o.stem_cap) atomicOr(m.count + 2, MATCH_ERR_CAP);
      else o.off[cnt] = (uint32_t)tot;
    }
    const unsigned long long b = (incl - v) & M40, len = v & M40;
    if (v && b + len <= o.stem_cap) {  // (else MATCH_ERR_CAP, set by the last lane)
      const uint32_t j = (uint32_t)(incl >> 40) - 1u;
      const uint32_t q = r.req[d], k = m.kind[d];
      o.off[j] = (uint32_t)b;
      o.req[j] = q;
      o.unit[j] = (uint8_t)(k >> 8);
      o.flags[j] = (uint8_t)(k >> 16);  // RL_FLAG_SHADOW
      o.limit[j] = m.rpu[d];
      o.hits[j] = r.hits[q];
      o.rule[j] = m.rule[d];
      // prefix ‖ domain ‖ '_' ‖ entry bytes
      const uint32_t da = r.dom_off[q], dl = r.dom_off[q + 1] - da;
      const uint32_t b0 = r.desc_off[d], bl = r.desc_off[d + 1] - b0;
      uint8_t* dst = assembled ? (uint8_t*)s_out + (uint32_t)(b - (oa & ~3ull)) : o.stem + b;
      for (uint32_t i = 0; i < c.prefix_len; i++) dst[i] = c.prefix[i];
      dst += c.prefix_len;
      for (uint32_t i = 0; i < dl; i++) dst[i] = r.dom[da + i];
      dst[dl] = '_';
      dst += dl + 1;
      if (staged) {
        const uint8_t* src = (const uint8_t*)s_in + (b0 - (ba & ~3u));
        for (uint32_t i = 0; i < bl; i++) dst[i] = src[i];
      } else {
        for (uint32_t i = 0; i < bl; i++) dst[i] = r.desc[b0 + i];
      }
    }
  }
  if (!assembled) return;
  __syncthreads();
  const uint32_t w0 = (uint32_t)(oa >> 2), nw = (uint32_t)(((ob + 3) >> 2) - w0);
  uint32_t* out32 = reinterpret_cast<uint32_t*>(o.stem);
  for (uint32_t i = threadIdx.x; i < nw; i += MT) {
    const uint64_t lo = (uint64_t)(w0 + i) * 4;
    if (lo >= oa && lo + 4 <= ob) {
      out32[w0 + i] = s_out[i];
    } else {
      for (uint32_t k = 0; k < 4; k++)
        if (lo + k >= oa && lo + k < ob) o.stem[lo + k] = ((const uint8_t*)s_out)[i * 4 + k];
    }
  }
}

// shouldRateLimitWorker's statuses (ratelimit.go:176-190): nil limit ->
// {OK, nil, 0} (base_limiter.go:78-81); unlimited -> {OK, MaxUint32}; matched
// -> DoLimit's status.
__global__ __launch_bounds__(256) void k_match_expand(ReqDev r, MatchBuf m, const unsigned long long* __restrict__ s,
                                                      const uint8_t* __restrict__ code,
                                                      const uint32_t* __restrict__ rem,
                                                      const uint32_t* __restrict__ reset, ReqOutDev out) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d >= r.n_desc) return;
  const uint32_t k = m.kind[d], kind = k & 0xFFu;
  uint8_t cd = RL_CODE_OK;
  uint32_t rm = 0, rs = 0;
  if (kind == RL_MATCH_LIMIT) {
    const uint32_t j = (uint32_t)(s[d] >> 40) - 1u;
    cd = code[j];
    rm = rem[j];
    rs = reset[j];
  } else if (kind == RL_MATCH_UNLIMITED) {
    rm = 0xFFFFFFFFu;
  }
  out.code[d] = cd;
  out.rem[d] = rm;
  out.reset[d] = rs;
  out.match[d] = (uint8_t)kind;
  out.rule[d] = m.rule[d];
  out.rpu[d] = m.rpu[d];
  out.unit[d] = (uint8_t)(k >> 8);
}

}  // namespace

size_t match_scan_bytes(uint32_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const unsigned long long*)nullptr,
                                         (unsigned long long*)nullptr, (int)n, (hipStream_t)0);
  return bytes;
}

void launch_match(const CfgDev& cfg, const ReqDev& r, const MatchBuf& m, const PackOut& o, void* tmp,
                  size_t tmp_bytes, hipStream_t st) {
  if (!r.n_desc) return;
  const uint32_t g = (r.n_desc + 255) / 256;
  k_match<<<g, MT, (size_t)cfg.blob_words * 4, st>>>(cfg, r, m);
  (void)hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, m.v, m.v + r.n_desc, (int)r.n_desc, st);
  k_match_emit<<<g, MT, 0, st>>>(cfg, r, m, m.v + r.n_desc, o);
}

void launch_match_expand(const ReqDev& r, const MatchBuf& m, const uint8_t* code, const uint32_t* rem,
                         const uint32_t* reset, const ReqOutDev& out, hipStream_t st) {
  if (!r.n_desc) return;
  k_match_expand<<<(r.n_desc + 255) / 256, 256, 0, st>>>(r, m, m.v + r.n_desc, code, rem, reset, out);
}

}  // namespace rl
