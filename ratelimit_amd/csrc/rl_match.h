// rl_match.h — the config trie on the device and the kernels of the request
// path (rl_match.hip): GetLimit per descriptor, compaction of the matched
// descriptors into the DoLimit batch, and the service's status mapping.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rl {

// One config node on the device (rl_config_node plus its child count).
struct CfgNode {
  int32_t parent;
  uint32_t key_off, key_len;
  uint32_t rpu, rule;
  uint32_t n_children;
  uint8_t unit, has_limit, unlimited, shadow;
  uint32_t pad;
};

// The loaded config: nodes, their key bytes and an open-addressing index of
// (parent, key) -> node. Index entries: tag (high hash bits) | (node + 1) << 32;
// 0 = empty. Collision-exact: a tag match is confirmed with the key bytes.
struct CfgDev {
  const CfgNode* nodes;
  const uint8_t* keys;
  const unsigned long long* index;
  uint32_t mask;      // index size - 1
  uint32_t n_nodes;
  const uint8_t* prefix;
  uint32_t prefix_len;
  // the whole config as one blob [nodes | index | prefix ‖ keys]; staged into
  // LDS by k_match when blob_words != 0 (it fits CFG_LDS_WORDS)
  const uint8_t* blob;
  uint32_t blob_words, idx_word, key_word;
};
constexpr uint32_t CFG_LDS_WORDS = 12288 / 4;

// Raw request batch on the device (rl_request_batch).
struct ReqDev {
  uint32_t n_req, n_desc, n_ent;
  uint32_t dom_total, desc_total;  // bytes behind dom / desc (offsets are checked against them)
  const uint8_t* dom;
  const uint32_t* dom_off;
  const uint32_t* hits;
  const uint32_t* req;
  const uint32_t* ent_first;
  const uint32_t* desc_off;
  const uint8_t* desc;
  const uint16_t* klen;
  const uint16_t* vlen;
  const uint8_t* ovf;
  const uint32_t* ov_rpu;
  const uint8_t* ov_unit;
  const uint32_t* ov_rule;
};

// The compacted DoLimit batch the matched descriptors are written into.
struct PackOut {
  uint8_t* stem;
  uint32_t* off;
  uint32_t* req;
  uint8_t* unit;
  uint8_t* flags;
  uint32_t* limit;
  uint32_t* hits;
  uint32_t* rule;
  uint32_t stem_cap;
};

// Per-descriptor match results.
struct MatchBuf {
  unsigned long long* v;     // [2n]: (matched << 40) | stem bytes, then its inclusive scan
  uint32_t* kind;            // rl_match | unit << 8 | shadow << 16
  uint32_t* rpu;
  uint32_t* rule;
  uint32_t* count;           // [0] matched descriptors, [1] stem bytes, [2] error bits
};

// The service's per-descriptor answer (rl_request_result, device arrays).
struct ReqOutDev {
  uint8_t* code;
  uint32_t* rem;
  uint32_t* reset;
  uint8_t* match;
  uint32_t* rule;
  uint32_t* rpu;
  uint8_t* unit;
};

constexpr uint32_t MATCH_ERR_REQ = 1, MATCH_ERR_CAP = 2;

__host__ __device__ inline uint64_t cfg_hash(int32_t parent, const uint8_t* p, uint32_t len) {
  uint64_t h = 0xcbf29ce484222325ull ^ ((uint64_t)(uint32_t)(parent + 1) * 0x9E3779B97F4A7C15ull);
  for (uint32_t i = 0; i < len; i++) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h;
}

// Enqueue: match every descriptor, scan, compact. Scan temp storage is
// `tmp` (tmp_bytes from match_scan_bytes).
size_t match_scan_bytes(uint32_t n);
void launch_match(const CfgDev& cfg, const ReqDev& r, const MatchBuf& m, const PackOut& o, void* tmp,
                  size_t tmp_bytes, hipStream_t st);
void launch_match_expand(const ReqDev& r, const MatchBuf& m, const uint8_t* code, const uint32_t* rem,
                         const uint32_t* reset, const ReqOutDev& out, hipStream_t st);

}  // namespace rl
