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

__device__ inline bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

// rateLimitDescriptor.descriptors[key] lookup (a Go map of finalKey) at `parent`
// (-1: the domains map, config_impl.go:247).
__device__ int32_t cfg_find(const CfgDev& c, int32_t parent, const uint8_t* p, uint32_t len) {
  const uint64_t h = cfg_hash(parent, p, len);
  const uint32_t tag = (uint32_t)(h >> 32);
  uint32_t pos = (uint32_t)h & c.mask;
  for (uint32_t i = 0; i <= c.mask; i++) {
    const unsigned long long e = c.index[pos];
    if (!e) return -1;
    if ((uint32_t)e == tag) {
      const uint32_t nd = (uint32_t)(e >> 32) - 1u;
      const CfgNode& N = c.nodes[nd];
      if (N.parent == parent && N.key_len == len && bytes_eq(c.keys + N.key_off, p, len)) return (int32_t)nd;
    }
    pos = (pos + 1) & c.mask;
  }
  return -1;
}

__global__ __launch_bounds__(256) void k_match(CfgDev c, ReqDev r, MatchBuf m) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d >= r.n_desc) return;
  const uint32_t q = r.req[d];
  uint32_t kind = RL_MATCH_NONE, rpu = 0, rule = 0, unit = 0, shadow = 0;
  unsigned long long v = 0;
  const uint32_t e0 = r.ent_first[d], e1 = r.ent_first[d + 1];
  const uint32_t b0 = r.desc_off[d], b1 = r.desc_off[d + 1];
  bool bad = q >= r.n_req || e1 < e0 || e1 > r.n_ent || b1 < b0 || b1 > r.desc_total;
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
    const int32_t root = cfg_find(c, -1, r.dom + da, dl);  // this.domains[domain] (:247)
    if (root >= 0) {
      if (r.ovf && (r.ovf[d] & 1u)) {  // descriptor.GetLimit() != nil (:254-266): never shadow
        kind = RL_MATCH_LIMIT;
        rpu = r.ov_rpu[d];
        unit = r.ov_unit[d];
        rule = r.ov_rule[d];
      } else {  // the trie walk (:268-295)
        int32_t node = root, hit = -1;
        uint32_t p = b0;
        for (uint32_t e = e0; e < e1; e++) {
          const uint32_t kl = r.klen[e], vl = r.vlen[e];
          int32_t nx = cfg_find(c, node, r.desc + p, kl + 1u + vl);  // key_value
          if (nx < 0) nx = cfg_find(c, node, r.desc + p, kl);          // key
          if (nx >= 0 && c.nodes[nx].has_limit && e == e1 - 1) hit = nx;
          if (nx >= 0 && c.nodes[nx].n_children) node = nx;
          else break;
          p += kl + vl + 2u;
        }
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

__device__ inline void copy_bytes(uint8_t* dst, const uint8_t* src, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) dst[i] = src[i];
}

// s = inclusive scan of m.v. Matched descriptor d goes to position
// (s[d] >> 40) - 1 with its stem at byte (s[d] - v[d]) & (2^40 - 1).
__global__ __launch_bounds__(256) void k_match_emit(CfgDev c, ReqDev r, MatchBuf m,
                                                    const unsigned long long* __restrict__ s, PackOut o) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d >= r.n_desc) return;
  constexpr unsigned long long M40 = (1ull << 40) - 1;
  const unsigned long long incl = s[d], v = m.v[d];
  if (d == r.n_desc - 1) {
    const uint32_t cnt = (uint32_t)(incl >> 40);
    const unsigned long long tot = incl & M40;
    m.count[0] = cnt;
    m.count[1] = (uint32_t)(tot < 0xFFFFFFFFull ? tot : 0xFFFFFFFFull);
    if (tot > o.stem_cap) atomicOr(m.count + 2, MATCH_ERR_CAP);
    else o.off[cnt] = (uint32_t)tot;
  }
  if (!v) return;
  const uint32_t j = (uint32_t)(incl >> 40) - 1u;
  const unsigned long long b = (incl - v) & M40, len = v & M40;
  if (b + len > o.stem_cap) return;  // MATCH_ERR_CAP (set by the last lane)
  const uint32_t q = r.req[d], k = m.kind[d];
  o.off[j] = (uint32_t)b;
  o.req[j] = q;
  o.unit[j] = (uint8_t)(k >> 8);
  o.flags[j] = (uint8_t)(k >> 16);  // RL_FLAG_SHADOW
  o.limit[j] = m.rpu[d];
  o.hits[j] = r.hits[q];
  o.rule[j] = m.rule[d];
  uint8_t* dst = o.stem + b;
  const uint32_t da = r.dom_off[q], dl = r.dom_off[q + 1] - da;
  const uint32_t b0 = r.desc_off[d], bl = r.desc_off[d + 1] - b0;
  copy_bytes(dst, c.prefix, c.prefix_len);
  dst += c.prefix_len;
  copy_bytes(dst, r.dom + da, dl);
  dst[dl] = '_';
  copy_bytes(dst + dl + 1, r.desc + b0, bl);
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
  uint8_t c = RL_CODE_OK;
  uint32_t rm = 0, rs = 0;
  if (kind == RL_MATCH_LIMIT) {
    const uint32_t j = (uint32_t)(s[d] >> 40) - 1u;
    c = code[j];
    rm = rem[j];
    rs = reset[j];
  } else if (kind == RL_MATCH_UNLIMITED) {
    rm = 0xFFFFFFFFu;
  }
  out.code[d] = c;
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
  k_match<<<g, 256, 0, st>>>(cfg, r, m);
  (void)hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, m.v, m.v + r.n_desc, (int)r.n_desc, st);
  k_match_emit<<<g, 256, 0, st>>>(cfg, r, m, m.v + r.n_desc, o);
}

void launch_match_expand(const ReqDev& r, const MatchBuf& m, const uint8_t* code, const uint32_t* rem,
                         const uint32_t* reset, const ReqOutDev& out, hipStream_t st) {
  if (!r.n_desc) return;
  k_match_expand<<<(r.n_desc + 255) / 256, 256, 0, st>>>(r, m, m.v + r.n_desc, code, rem, reset, out);
}

}  // namespace rl
