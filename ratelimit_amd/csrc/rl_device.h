// rl_device.h — HBM table layout, hashing and the per-descriptor decision
// function shared by every kernel of libratelimit_hip.so (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/ratelimit_hip.h"

namespace rl {

// ---------------------------------------------------------------------------
// HBM counter table.
//
// One 64-B slot per (stem, unit). The Redis key of the reference is
// stem ‖ decimal(windowStart) (cache_key.go:62-74); a slot holds the state of
// the newest window key of its (stem, unit), `cur`. For a stem used with a
// single unit the current window is the only live key while time moves
// forward, so the slot is recycled in place when the window advances (no
// insert per window, no EXPIRE traffic).
//
// Older windows live in the HISTORY LOG: when a key's cur moves to a newer
// window, the old record is appended to the log (a 32-B entry in one of
// LOG_PARTS append-only ring buffers) while a request could still ask for it,
// and the slot's `ring` word becomes the head of the key's chain of entries,
// newest first. Redis keeps a key div + jitter seconds after its last hit
// (fixed_cache_impl.go:71-74), so a request that waited in a batcher, or whose
// clock is behind, finds its window's count: a record is kept while its
// window is within HIST_W windows of the key's newest one, or its EXPIRE (or
// local-cache TTL) plus the horizon J (rl_config.expiration_jitter_max_seconds)
// has not passed the newest window's start. A request older than both bounds
// whose record is not on the chain is RL_E_TIME; any other request is answered
// exactly (no record on the chain: the key had none, count 0). An entry the
// log overwrote before its time (the log too small for the horizon) makes a
// lookup that reaches it RL_E_TIME, counted in rl_table_info, never a wrong
// count. The log replaces round 4's pool of 128-B ring lines: appends are
// wave-aggregated and coalesced, where a line took a random write per move.
// ---------------------------------------------------------------------------
constexpr uint32_t WS_INVALID = 0xFFFFFFFFu;  // record never written
constexpr uint32_t TAG_EMPTY = 0;
constexpr uint32_t TAG_TOMB = 1;
constexpr uint32_t KEY_IN = 36;               // a stem of at most KEY_IN bytes is stored whole in its slot
constexpr uint32_t KEY_SPLIT = 32;            // a longer one: bytes [0, KEY_SPLIT) here, the rest in the arena
constexpr uint32_t RING_NONE = 0xFFFFFFFFu;   // Slot::ring of a key without logged history (= LOG_NONE)
constexpr uint8_t SLOT_EXACT = 0x1;           // stem has >1 unit slot: exact (serial) path
constexpr uint32_t HIST_W = 8;                // windows 1..HIST_W back from cur are always kept

struct Win {
  uint32_t ws;      // window start (Redis key suffix); WS_INVALID = no record
  uint32_t count;   // INCRBY value (u32, radix decodes into *uint32)
  uint32_t expire;  // Redis key live while now <= expire (EXPIRE = now + div)
  uint32_t lc;      // freecache entry live while now < lc (Set ttl = div)
};

// One 64-B sector: a probe reads exactly one sector, and only changed window
// records are written back. A stem longer than KEY_IN keeps its first
// KEY_SPLIT bytes here and the rest in the long-stem arena, whose offset (in
// 16-B units) takes the slot's last stem dword.
struct __attribute__((aligned(64))) Slot {
  uint32_t tag;       // TAG_EMPTY / TAG_TOMB / mix(hash(stem), unit) >= 2
  uint16_t key_len;   // stem length
  uint8_t unit;       // rl_unit
  uint8_t flags;      // SLOT_EXACT
  Win cur;            // bytes 8..23
  uint32_t ring;      // 24..27: head of the slot's history chain in the log (RING_NONE: none)
  uint8_t key[KEY_IN];  // 28..63: stem bytes (key_len > KEY_IN: bytes 0..31, then the arena offset)
};
static_assert(offsetof(Slot, cur) == 8 && offsetof(Slot, ring) == 24 && offsetof(Slot, key) == 28, "slot layout");
static_assert(sizeof(Slot) == 64, "slot must be one 64-B sector");
// dword of the slot holding stem dword k (k < KEY_IN / 4)
__host__ __device__ constexpr uint32_t slot_key_dw(uint32_t k) { return 7 + k; }
constexpr uint32_t SLOT_EXT_DW = 15;          // arena offset of a stem longer than KEY_IN
// stem bytes kept in the slot for a stem of len bytes
__host__ __device__ constexpr uint32_t slot_inline(uint32_t len) { return len <= KEY_IN ? len : KEY_SPLIT; }

// One entry of the history log: an older window record of slot `slot` (whose
// tag was `tag` when it was written), the previous entry of the slot's chain,
// and t_app = the slot's newest window when it was appended (never decreases
// along a chain; an entry the log overwrote breaks that, or the owner check).
struct __attribute__((aligned(32))) LogEnt {
  uint32_t slot, tag, prev, t_app;
  Win w;
};
static_assert(sizeof(LogEnt) == 32, "log entry is two dwordx4");
constexpr uint32_t LOG_NONE = RING_NONE;
#ifndef RL_LOG_PARTS_LOG2
#define RL_LOG_PARTS_LOG2 6  // (A/B builds: 8 = 256 partitions)
#endif
constexpr uint32_t LOG_PARTS = 1u << RL_LOG_PARTS_LOG2;   // partitions (each its own append counter)
constexpr uint32_t LOG_POS_BITS = 32 - RL_LOG_PARTS_LOG2; // entry pointer = part << LOG_POS_BITS | position
constexpr uint32_t LOG_POS_MASK = (1u << LOG_POS_BITS) - 1u;
constexpr uint32_t LOG_PART_MAX = 1u << (LOG_POS_BITS - 1);  // entries per partition (2^31 in all)
static_assert(LOG_PARTS <= 256, "k_b_begin copies the counters with one workgroup");
constexpr uint32_t LOG_CTR_STRIDE = 16;                   // counters on 128-B lines of their own
// Word 0 of partition p's line: the append counter. Line LOG_PARTS: [0]
// lookups that met an overwritten entry, [1] appends refused (below). Each
// batch's k_b_begin copies the counters to the batch's own array
// (Scratch::log_epoch, lines of their own: the counters' lines take every
// append's atomic).
// Chain pointer standing for a record the log could not keep (its partition
// had taken log_cap appends in this batch already): its position is past any
// partition, so a walk that reaches it fails like one that meets an
// overwritten entry (RL_E_TIME unless the window is dead).
constexpr uint32_t LOG_LOST = LOG_POS_MASK;
static_assert(LOG_LOST != LOG_NONE && (LOG_LOST & LOG_POS_MASK) >= LOG_PART_MAX, "LOG_LOST is no position");
// An entry's header tag while the entry is being written (tags are >= 2).
constexpr uint32_t LOG_TAG_BUSY = 0;
constexpr uint32_t LOG_MAX_HOPS = 1u << 16;               // a chain walk gives up (RL_E_TIME) past this
// Window w < cur_ws is within HIST_W windows of the key's newest one.
__host__ __device__ inline bool hist_reach(uint32_t w, uint32_t cur_ws, uint32_t d) { return cur_ws - w <= HIST_W * d; }

__host__ __device__ inline uint32_t div_of(uint32_t unit) {  // utils.UnitToDivider
  return unit == RL_UNIT_SECOND ? 1u : unit == RL_UNIT_MINUTE ? 60u : unit == RL_UNIT_HOUR ? 3600u : 86400u;
}

__host__ __device__ inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

__host__ __device__ inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// Keyed 64-bit stem hash: SipHash-1-3 (one compression round per 8-byte
// little-endian word, three finalisation rounds) under a 128-bit key drawn per
// rl_ctx (rl_config.hash_seed; random when 0). Descriptor values are
// client-controlled; with a secret key an attacker cannot aim stems at one
// sort key or one home slot. Correctness never depends on the hash: every
// match is confirmed on the full stem bytes, and any number of stems sharing a
// sort key takes the exact path.
struct HashKey {
  uint64_t k0, k1;
  uint32_t hi_bits;  // test knob: keep only the top hi_bits of the high word (32 = all)
};

__host__ __device__ inline HashKey hash_key_of(uint64_t seed, uint32_t hi_bits) {
  return HashKey{fmix64(seed ^ 0x243F6A8885A308D3ull), fmix64(seed + 0x13198A2E03707344ull),
                 hi_bits == 0 || hi_bits > 63 ? 32u : hi_bits};
}

struct StemHasher {
  uint64_t v0, v1, v2, v3, b;
  __host__ __device__ inline StemHasher(const HashKey& k, uint32_t len)
      : v0(k.k0 ^ 0x736f6d6570736575ull), v1(k.k1 ^ 0x646f72616e646f6dull), v2(k.k0 ^ 0x6c7967656e657261ull),
        v3(k.k1 ^ 0x7465646279746573ull), b(uint64_t(len) << 56) {}
  __host__ __device__ inline void round() {
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);
  }
  __host__ __device__ inline void word(uint64_t m) {
    v3 ^= m;
    round();
    v0 ^= m;
  }
  // tail = the last len % 8 bytes (little-endian, zero above them)
  __host__ __device__ inline uint64_t finish(uint64_t tail, uint32_t hi_bits) {
    word(b | tail);
    v2 ^= 0xff;
    round(); round(); round();
    uint64_t x = v0 ^ v1 ^ v2 ^ v3;
    if (hi_bits < 32) x &= ~(((1ull << (32 - hi_bits)) - 1) << 32);
    else if (hi_bits > 32) x |= ((1ull << (64 - hi_bits)) - 1) << 32;  // (33..63: the dropped bits set)
    return x ? x : 1;
  }
};

// 64-bit hash of the stem bytes [a, a+len) read through rd (8 bytes per call).
template <typename Rd>
__device__ inline uint64_t hash_stem(const HashKey& key, Rd rd, uint32_t a, uint32_t len) {
  StemHasher hs(key, len);
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) hs.word(rd(a + i));
  uint64_t tail = 0;
  if (i < len) tail = rd(a + i) & ((1ull << ((len - i) * 8)) - 1);
  return hs.finish(tail, key.hi_bits);
}

// Host reference of the same hash (tests, tools).
__host__ inline uint64_t hash_stem_host(const HashKey& key, const uint8_t* s, uint32_t len) {
  StemHasher hs(key, len);
  uint32_t i = 0;
  auto rd = [&](uint32_t at, uint32_t nb) {
    uint64_t w = 0;
    for (uint32_t j = 0; j < nb; j++) w |= uint64_t(s[at + j]) << (8 * j);
    return w;
  };
  for (; i + 8 <= len; i += 8) hs.word(rd(i, 8));
  return hs.finish(i < len ? rd(i, len - i) : 0, key.hi_bits);
}

// 8 bytes starting at byte address a of a dword array (little-endian); dwords
// at index >= nw read as 0 (no access past the stem buffer).
struct DwordReader {
  const uint32_t* p;
  uint32_t nw;
  __device__ inline uint32_t at(uint32_t i) const { return i < nw ? p[i] : 0u; }
  __device__ inline uint64_t operator()(uint32_t a) const {
    uint32_t idx = a >> 2, sh = (a & 3) * 8;
    uint64_t lo = at(idx), mid = at(idx + 1);
    uint64_t x = lo | (mid << 32);
    if (sh) x = (x >> sh) | (uint64_t(at(idx + 2)) << (64 - sh));
    return x;
  }
};

__host__ __device__ inline uint32_t slot_tag(uint64_t hstem, uint32_t unit) {
  const uint32_t t = (uint32_t)fmix64(hstem + uint64_t(unit) * 0x9E3779B97F4A7C15ull);
  return t < 2 ? t + 2 : t;
}

// ---------------------------------------------------------------------------
// GetResponseDescriptorStatus (base_limiter.go:76-135) for a non-empty key,
// including checkOverLimitThreshold / checkNearLimitThreshold (:150-179).
// All arithmetic in uint32 like the Go code, widened to u64 for the counters.
// ---------------------------------------------------------------------------
struct Decision {
  uint8_t code;
  uint8_t set_lc;
  uint32_t remaining;
  uint32_t d_over, d_near, d_lc, d_within, d_shadow;
};

// uint32(math.Floor(float64(float32(limit) * ratio))): a single IEEE fp32
// multiply (no FMA contraction), then Go's uint32(float64) = low 32 bits of a
// truncating int64 conversion (0x8000000000000000 when out of range).
__host__ __device__ inline uint32_t near_threshold(uint32_t limit, float ratio) {
#if defined(__HIP_DEVICE_COMPILE__)
  float prod = __fmul_rn((float)limit, ratio);
#else
  volatile float prod = (float)limit * ratio;
#endif
  double f = floor((double)prod);
  int64_t v = (f >= -9223372036854775808.0 && f < 9223372036854775808.0) ? (int64_t)f : INT64_MIN;
  return (uint32_t)v;
}

__host__ __device__ inline Decision decide(uint32_t before, uint32_t after, bool lc_hit, uint32_t h,
                                           uint32_t thr, float ratio, bool shadow, bool lc_enabled) {
  Decision r = {RL_CODE_OK, 0, 0, 0, 0, 0, 0, 0};
  bool over = false;
  if (lc_hit) {
    over = true;
    r.d_over = h; r.d_lc = h; r.code = RL_CODE_OVER_LIMIT;
  } else {
    uint32_t near = near_threshold(thr, ratio);
    if (after > thr) {
      over = true;
      r.code = RL_CODE_OVER_LIMIT;
      if (before >= thr) {
        r.d_over = h;
      } else {
        r.d_over = after - thr;
        r.d_near = thr - (near > before ? near : before);
      }
      r.set_lc = lc_enabled ? 1 : 0;
    } else {
      r.remaining = thr - after;
      if (after > near) r.d_near = (before >= near) ? h : after - near;
      r.d_within = h;
    }
  }
  if (over && shadow) {
    r.code = RL_CODE_OK;
    r.d_shadow = h;
  }
  return r;
}

// Device error word bits (mapped to rl_status by the host). Without per-descriptor
// statuses every bit fails the batch; with them (rl_result.status) only
// ERR_INVALID from a malformed batch layout does, and the others become the
// statuses of the descriptors they concern, collected in a soft word.
enum : uint32_t {
  ERR_INVALID = 1u << 0,
  ERR_TABLE_FULL = 1u << 1,
  ERR_ARENA_FULL = 1u << 2,
  ERR_TIME = 1u << 3,
  ERR_HISTORY = 1u << 5,     // a key's window is older than its ring reaches (HIST_W windows)
};

// rl_status of a batch that failed with device error bits e (the host's
// map_err order), and the error bit that reports a descriptor status.
__host__ __device__ inline uint32_t err_status(uint32_t e) {
  return (e & (ERR_TIME | ERR_HISTORY)) ? (uint32_t)RL_E_TIME
         : (e & ERR_INVALID)            ? (uint32_t)RL_E_INVALID
         : (e & ERR_TABLE_FULL)         ? (uint32_t)RL_E_TABLE_FULL
         : (e & ERR_ARENA_FULL)         ? (uint32_t)RL_E_ARENA_FULL
                                        : (uint32_t)RL_E_INTERNAL;
}
__host__ __device__ inline uint32_t status_err(uint32_t st) {
  return st == RL_E_TIME ? ERR_TIME : st == RL_E_TABLE_FULL ? ERR_TABLE_FULL : st == RL_E_ARENA_FULL ? ERR_ARENA_FULL
                                                                                                       : ERR_INVALID;
}

// Packed 8-B result of one descriptor (k_finish / the route exchange unpack it):
//   bits  0..31 LimitRemaining, 32..51 DurationUntilReset (<= 86400),
//   52..55 rl_status of the descriptor (0 = answered), 56..61 code,
//   62 the local-cache Get hit (localCacheStats hitCount).
__host__ __device__ inline unsigned long long pack_res(uint32_t rem, uint32_t reset, uint32_t code, bool lc_hit) {
  return (unsigned long long)rem | ((unsigned long long)(reset & 0xFFFFFu) << 32) |
         ((unsigned long long)code << 56) | ((unsigned long long)lc_hit << 62);
}
__host__ __device__ inline unsigned long long pack_fail(uint32_t status) {
  return (unsigned long long)(status & 0xFu) << 52;
}
__host__ __device__ inline uint32_t res_rem(unsigned long long v) { return (uint32_t)v; }
__host__ __device__ inline uint32_t res_reset(unsigned long long v) { return (uint32_t)(v >> 32) & 0xFFFFFu; }
__host__ __device__ inline uint32_t res_status(unsigned long long v) { return (uint32_t)(v >> 52) & 0xFu; }
__host__ __device__ inline uint32_t res_code(unsigned long long v) { return (uint32_t)(v >> 56) & 0x3Fu; }
__host__ __device__ inline bool res_lc_hit(unsigned long long v) { return (v >> 62) & 1u; }

// Rec / wire flags byte: bit 0 = RL_FLAG_SHADOW (ABI); bit 7 = the descriptor
// failed (its status is already in its packed result): every table kernel
// leaves it alone.
constexpr uint32_t FLAG_SKIP = 0x80;
// k_run_check marks a descriptor whose sort key occurs more than once in the
// batch by overwriting its arrival-order key (Scratch::keys[0], read after the
// partition only by the keys-seen-once part) with KEY_DUP: a random 4-B store
// into a 4-B-per-descriptor array instead of into its 32-B record, and no
// extra read where the keys are read anyway. k_prepare keeps KEY_DUP out of
// the real keys (a stem whose hash starts with it sorts as KEY_DUP - 1, its
// slot tags and home slot likewise: collisions are resolved by the stems).
constexpr uint32_t KEY_DUP = 0xFFFFFFFFu;
// (bit 6, free: until round 6 the mark of a sort key that occurs more than
// once in the batch; now KEY_DUP in the arrival-order keys)
// bit 5 = a routed owner batch's own-chunk record: its stem lies in the
// source batch (BatchDev::own), not in the received stems.
constexpr uint32_t FLAG_SRC = 0x20;

constexpr uint32_t NOW_MAX = 0xFFFFFFFFu - 2u * 86400u;  // now + 2*div must fit u32

}  // namespace rl
