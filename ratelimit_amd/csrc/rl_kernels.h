// rl_kernels.h — device-side views of a batch / the table and the kernel entry
// points of rl_kernels.hip (launched from rl_api.hip through the wrappers).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_device.h"

namespace rl {

#ifndef RL_PART_ITEMS
#define RL_PART_ITEMS 16  // (8: 82 instead of 144 VGPRs, twice the tiles: C1 -3 %, C2 -8 %)
#endif
constexpr uint32_t PART_ITEMS = RL_PART_ITEMS, PART_TILE = 256 * PART_ITEMS;  // k_part: 256 threads x PART_ITEMS
constexpr uint32_t PART_BITS = 10, PART_DIGITS = 1u << PART_BITS;   // buckets = top key bits
#ifndef RL_BIG_BLOCKS
#define RL_BIG_BLOCKS 64
#endif
constexpr uint32_t BIG_BLOCKS = RL_BIG_BLOCKS;                      // k_bucket_big workgroups
constexpr uint32_t BIG_ITEM_BLOCKS = 256;                           // k_big_count / k_big_place workgroups
constexpr uint32_t BIG_HEAVY = 4;                                   // hot keys peeled off a large bucket

// A bucket too large for k_bucket's LDS, queued with its sampled hot keys.
struct BigMeta {
  uint32_t d, S, base, nchunks, item0, r, rb_heavy, db_heavy;
  uint32_t heavy[BIG_HEAVY];
};
constexpr uint32_t MAX_PART_TILES = 2048 * 16 / PART_ITEMS;  // k_part tiles per batch (max_batch <= 8388608)
constexpr uint32_t LONG_RUN = 32;        // runs at least this long take the parallel path
constexpr uint32_t RUN_SLOW = 1, RUN_FAST = 2, RUN_MULTI = 4;
// A stem under several units (per-request overrides, config_impl.go:254-265)
// shares Redis keys across its unit slots whenever two windows coincide
// (SECOND and MINUTE at t % 60 == 0, cache_key.go:73-74). k_split orders such
// a stem's descriptors into one sub-run per Redis key (stem, window[, store])
// — its "groups", consecutive, the first one the head — and the head's
// k_table lane sets every group up for the parallel path with the key's
// records in all unit slots as write-back targets (alias_setup).
constexpr uint32_t RUN_NOWVAR = 8;    // the run's descriptors do not share one `now`
constexpr uint32_t RUN_ALIAS = 16;    // a group of a multi-unit stem (or a lone run of a SLOT_EXACT stem)
constexpr uint32_t RUN_AHEAD = 32;    // ... its first group: bits 8..15 = the stem's group count
constexpr uint32_t RUN_MERGE = 64;    // a deferred head: the exact path replays all groups in arrival order
constexpr uint32_t RUN_G_SHIFT = 8, RUN_UMASK_SHIFT = 16;  // group count (head), units of the group (bit u-1)
// k_run_check's verdict on a RUN_MULTI run (k_split reads it): some element has
// the head's stem under another unit / some element has another stem or failed
constexpr uint32_t RUN_UNITS = 128, RUN_STEMS = 1u << 24;
#ifndef RL_KEY_HEAD
#define RL_KEY_HEAD 64
#endif
constexpr uint32_t KEY_HEAD = RL_KEY_HEAD;  // stem bytes carried inline (zero-padded) per descriptor (a multiple of 16)
constexpr uint32_t KEY_HV = KEY_HEAD / 16;  // ... as uint4s
static_assert(KEY_HEAD % 16 == 0 && KEY_HEAD >= 48 && KEY_HEAD <= 64, "key head: 48 or 64 bytes (>= KEY_IN)");
constexpr uint32_t STAT_STRIPES = 64;     // global partial stats tables
constexpr uint32_t STAT_LDS_RULES = 512;  // rules aggregated in LDS (== LDS_RULES)
constexpr uint32_t RUNS_GENERAL_LATE_BLOCKS = 8;  // k_late's exact-path workgroups (grid-stride over deferrals)

struct Wire;
// A routed owner batch's own chunk (the descriptors this rank owns of its own
// slice), read in place from the source batch instead of as wire records and
// copied stems: received positions [lo, lo + n) are the source's descriptors
// idx[j - lo] (arrival order), with the stem hashes its partition computed.
// Their records carry FLAG_SRC: their stem offsets index `stem`.
struct OwnChunk {
  uint32_t lo, n, rank, stem_total;  // (stem_total: the capacity; kernels refine it from off[src_n])
  uint32_t src_n;    // the source batch's descriptors
  uint32_t n_rules;  // the source batch's n_rules (a rule id at or above it fails alone)
  const uint32_t* idx;
  const unsigned long long* hash;
  const uint8_t* stem;
  const uint32_t* off;
  const int64_t* now;
  const uint32_t* req;
  const uint8_t* unit;
  const uint8_t* flags;
  const uint32_t* limit;
  const uint32_t* hits;
  const uint32_t* rule;
  // the source batch's outputs (arrival order; null code: none): k_finish
  // answers the own chunk in place, no packed results go back for it. Without
  // a status array a failed descriptor ORs its error bit into src_err.
  uint8_t* code;
  uint32_t* rem;
  uint32_t* reset;
  uint8_t* status;
  uint32_t* src_err;
};
struct BatchDev {
  uint32_t n, n_req, n_rules, stem_cap;
  uint32_t stem_total;  // bytes of packed stems (off[n]); reads stay below it
  uint32_t now_desc;    // 1: now[] per descriptor and req[] an opaque non-decreasing label (routed batches)
  HashKey hk;           // the ctx's stem-hash key
  const uint8_t* stem;  // 4-byte aligned
  const uint32_t* off;
  const int64_t* now;
  const uint32_t* req;
  const uint8_t* unit;
  const uint8_t* flags;
  const uint32_t* limit;
  const uint32_t* hits;
  const uint32_t* rule;
  // routed owner batch (eng_route_owner): the received wire records replace
  // the arrays above (off, now, req, unit, flags, limit, hits, rule = null);
  // the stem of record j starts at woff[j] and must lie inside its source's
  // chunk [wbase[src], wbase[src + 1]) (the last source's ends at stem_total)
  const Wire* wire;
  const uint32_t* woff;             // [n] stem offset of each record (launch_wire_offsets)
  const unsigned long long* wbad;   // the offset scan's verdict (non-zero: a chunk's lengths do not add up)
  const unsigned long long* wbase;  // [n_src] chunk offset of each source in stem
  uint32_t n_src, rule_stride;
  OwnChunk own;  // (n = 0: none)
};

// One descriptor, packed by k_prepare (arrival order) and gathered once into
// sorted order, so the run kernels read one 32-B record per descriptor,
// contiguously per run, instead of ~10 scattered fields.
struct __attribute__((aligned(16))) Rec {
  uint32_t hlo;    // low 32 bits of the stem hash (high 32 bits = sort key)
  uint32_t off;    // stem byte offset
  uint32_t lu;     // stem length (16) | unit << 16 | flags << 24
  uint32_t rule;
  uint32_t req;
  uint32_t now;    // now[req] (validated to fit 32 bits)
  uint32_t hits;   // raw HitsAddend (restore records: the count)
  uint32_t limit;
};
static_assert(sizeof(Rec) == 32, "Rec is two dwordx4");

// A descriptor's record by sorted position: records stay in arrival order
// (k_prepare) and the sorted order is the permutation svals (one gather per
// access, no sorted copy of the records).
struct SRec {
  const Rec* rec;
  const uint32_t* sv;
  __device__ inline Rec operator[](uint32_t q) const { return rec[sv[q]]; }
};

__host__ __device__ inline uint32_t rec_len(const Rec& r) { return r.lu & 0xFFFFu; }
__host__ __device__ inline uint32_t rec_unit(const Rec& r) { return (r.lu >> 16) & 0xFFu; }
__host__ __device__ inline uint32_t rec_flags(const Rec& r) { return r.lu >> 24; }

// Multi-GPU routing wire record (rl_route.hip): one per routed descriptor.
constexpr uint32_t ROUTE_REQ_BITS = 24;  // label = source rank << 24 | request index
constexpr uint32_t ROUTE_MAX_REQ = 1u << ROUTE_REQ_BITS;
constexpr uint32_t ROUTE_TILE = 512;  // descriptors per partition tile (rl_route.hip RP_TILE)
// No stem offset: the stems of the records follow each other in record order
// (each source's chunk, sources in rank order), so the owner derives every
// offset from the lengths (launch_wire_offsets, one scan per exchange).
struct __attribute__((aligned(8))) Wire {
  uint32_t label;  // global request label (non-decreasing in global arrival order); first field (rl_comm reads it strided)
  uint32_t lu;     // stem length (16) | unit << 16 | flags << 24
  uint32_t limit;
  uint32_t hits;
  uint32_t rule;
  uint32_t now;    // the request's clock as the table keeps it (WIRE_NOW_BAD: outside [0, NOW_MAX] at the source)
  unsigned long long hash;  // keyed stem hash (source side): the owner's sort key and slot tag
};
constexpr uint32_t WIRE_NOW_BAD = 0xFFFFFFFFu;  // (> NOW_MAX: the owner's clock check fails it)
static_assert(sizeof(Wire) == RL_WIRE_BYTES, "wire record size is part of the ABI");

struct OutDev {
  uint8_t* code;
  uint32_t* rem;
  uint32_t* reset;
  unsigned long long* stats;
  uint8_t* status;  // per-descriptor rl_status (isolate mode), or null
};

struct TableDev {
  Slot* slots;
  // the history log (rl_device.h): LOG_PARTS append-only ring buffers of
  // log_cap entries each, one append counter per partition (LOG_CTR_STRIDE
  // apart); horizon = J seconds (rl_config.expiration_jitter_max_seconds)
  LogEnt* log;
  unsigned long long* log_ctr;
  uint32_t log_cap;  // entries per partition (power of 2)
  uint32_t horizon;
  unsigned long long* hist_lost;  // lookups that met an entry the log had overwritten ([1]: appends refused)
  const unsigned long long* log_epoch;  // this batch's [LOG_PARTS] append-counter floor (Scratch::log_epoch)
  uint32_t* tear;  // RL_LOG_TEAR builds only (tests): an armed rl_log_tear, or null
  uint64_t mask;
  uint8_t* arena;
  unsigned long long* arena_used16;
  uint64_t arena_cap16;
  uint32_t max_probe;
  uint32_t shift;  // home slot = stem hash >> shift (64 - log2 slots)
};

struct Params {
  float ratio;
  int lc_en;
  int per_second;
  int isolate;  // per-descriptor statuses (rl_result.status): descriptor errors do not fail the batch
};

// Per-batch scratch (device), sized for max_batch.
struct Scratch {
  Rec* rec;                  // [n] arrival order
  unsigned long long* res;   // [n] packed result per descriptor (arrival order)
  uint32_t* keys[2];
  uint32_t* vals[2];
  BigMeta* big_meta;                 // [PART_DIGITS] buckets queued for the large-bucket kernels
  uint32_t* big_n;
  uint32_t* big_work;                // [n / BIG_CHUNK + PART_DIGITS] chunk work items (bucket << 16 | chunk)
  uint32_t* work_n;
  uint32_t* sorted_n;                // sorted positions of the batch: the descriptors whose sort key repeats
                                     // (plus every element of a large bucket), one block per bucket
  uint32_t* big_cnt;                 // [work items x (1 + 2 x BIG_HEAVY)] k_big_count per chunk
  uint32_t* grp;                  // exact path: stem group of each position of a deferred run
  uint32_t* lead;                 //   first position of each group (stored from the run's start)
  uint8_t* gmask;                 //   units seen per group
  uint32_t* defer;                // RUN_MULTI runs (k_run_check); k_split marks the ones it resolves
  uint32_t* defer_n;
  uint32_t* defer2;               // runs k_table found to need the exact path (k_late)
  uint32_t* defer2_n;
  uint32_t* defer1;               // keys seen once k_table found to need the exact path (arrival indices)
  uint32_t* defer1_n;
  uint32_t* fast_blk;             // bit per 256-descriptor block holding a RUN_FAST run (k_table -> k_late)
  unsigned long long* log_epoch;  // [LOG_PARTS] the history log's append counters as k_b_begin saw them (log_append)
  // the keys seen once, listed bucket by bucket ({arrival index, sort key}):
  // k_table's singleton part walks them in this order, so a workgroup's
  // table probes stay inside the 1/1024 of the table its bucket's home slots
  // fall in (address-translation reach, tools/tlbprobe.hip)
  uint2* uniq;
  uint32_t* uniq_n;
  uint32_t* long_runs;  // [1 + n / 1024 + 1] runs over SPLIT_CAP elements: count, then defer indices (k_split_long)
  unsigned long long* kt_blk;  // [2 x k_table workgroups] start / end stamps (rl_profile)
  unsigned long long* stripes;    // STAT_STRIPES x STAT_LDS_RULES x RL_NUM_STATS
  // run segmentation (sorted order)
  uint32_t* hits_s;                    // [n] raw hits, sorted order
  uint32_t* hit_a;                     // [n] raw hits, arrival order (k_prepare)
  uint4* tile;                         // [n] k_part tile layout: {sort key, index, hits, 0}
  uint32_t* hit_t;                     // [n] k_bucket large-bucket temp
  uint32_t* segsum;                    // [n] inclusive in-run sum of hits
  uint32_t* rid;                       // [n] run id
  uint32_t* run_start;                 // [n] first sorted position of run r
  uint32_t* run_end;                   // [n] one past its last
  uint32_t* part_info;                 // [256 x part tiles] k_part: offset << 16 | count per digit and tile
  uint32_t* run_flags;                 // [n] RUN_*
  uint4* run_state;                    // [n] {slot, c0, old lc, F | which<<1}; alias groups: {targets, c0, lc, F}
  uint4* run_alias;                    // [n] alias groups: the stem's slot per unit (0xFFFFFFFF: none)
  uint32_t* run_f;                     // [n] first over-limit position
  unsigned long long* runs64;          // bucket path: runs | runs of two or more << 32
  unsigned long long* split;           // k_split: [0] reservations (ids | dup-run entries << 32), [1] runs64 before it
  uint32_t* drun;                      // [n/2 + BIG_HEAVY x PART_DIGITS] ids of the runs of two or more
  uint32_t* err;   // validation word of this buffer's batch (stage A)
  uint32_t* errb;  // sticky table-stage word (stage B), shared by both buffers
  uint32_t* errs;  // soft word: descriptor errors answered by statuses (isolate mode)
  int64_t* time_floor;  // requests earlier than the last sweep are rejected
  unsigned long long* counters;  // [0..3] sweep / info outputs
  // multi-GPU routing
  uint32_t* route_start;             // [2 x RL_MAX_SHARDS + 1] records / stem bytes per owner (partition)
  uint8_t* route_dest;               // [n] owner of each descriptor (routing scratch only)
  unsigned long long* route_hash;    // [n] its stem hash (routing scratch only)
  uint32_t* route_hist;              // [2 x RL_MAX_SHARDS x tiles] per-tile counts (routing scratch only)
  // routed owner batches (eng_route_owner)
  unsigned long long* r_base;        // [RL_MAX_SHARDS] received stem chunk starts per source
  uint32_t* woff;                    // [max_batch + 1] received records' stem offsets (rl_route_do_limit)
  unsigned long long* wtsum;         // [WIRE_SCAN_WORDS(max_batch)] its scan's tile sums and verdict
};

// The two stages of one batch. Stage A (validate, hash, sort, segment) touches
// only the batch and this buffer's scratch, so it may overlap the previous
// batch's stage B; stage B (table probe, replay, decisions, stats, results)
// must run in batch order.
// long_hint: a host word k_split sets when it meets a run over 1024 elements;
// long_kernel: such runs go to k_split_long's 1024-lane workgroups (else
// k_split's own 256-lane ones walk them). big_hint: a host word k_bucket sets
// when it queues a bucket too large for its LDS (hot keys); big_full: the
// large-bucket kernels get their full grids (else one workgroup each: they are
// grid-stride, so a batch with a large bucket the host did not expect is
// still answered, more slowly; C1 never has one)
void launch_stage_a(const BatchDev& b, const Scratch& s, int isolate, int per_second, hipStream_t st,
                    hipEvent_t* ev = nullptr, uint32_t* long_hint = nullptr, bool long_kernel = false,
                    uint32_t* big_hint = nullptr, bool big_full = true);
// errb_prev: the previous batch's table-stage word (this batch's starts from
// it); table_done (optional) is recorded once the table kernels are done, before
// k_finish: the next batch's stage B waits for it, not for k_finish.
// kt_acc (optional, rl_profile on): k_table's duration on the device clock
// (first workgroup start to last workgroup end) added to kt_acc[0], and 1 to
// kt_acc[1], by k_finish.
// early: k_b_begin already ran (launch_b_begin_early, end of stage A); k_table
// folds errb_prev into this batch's word.
void launch_stage_b(const BatchDev& b, const OutDev& o, const TableDev& t, const Params& P, const Scratch& s,
                    int restore, hipStream_t st, hipEvent_t* ev, const uint32_t* errb_prev, hipEvent_t table_done,
                    unsigned long long* kt_acc = nullptr, bool early = false, uint32_t* late_hint = nullptr,
                    bool late_full = true);
void launch_b_begin_early(const BatchDev& b, const OutDev& o, const Scratch& s, int restore, hipStream_t st,
                          const unsigned long long* log_ctr);
// ev (optional, RL_NUM_STAGES + 1 events on stream st): recorded before
// k_prepare, after it, after the sort, just before and just after k_table, and
// at the end (per-stage timing, rl_profile).
// A compact host batch (rl_batch_compact, device copy of its buffer at buf)
// -> the rl_batch arrays req / unit / flags / limit / hits / rule / now. A
// malformed request layout sets ERR_INVALID in *err (the batch fails); a limit
// index past the table gives the descriptor unit 0 (k_prepare: RL_E_INVALID).
void launch_unpack(const rl_batch_compact& cb, const uint8_t* buf, uint32_t* req, uint8_t* unit, uint8_t* flags,
                   uint32_t* limit, uint32_t* hits, uint32_t* rule, int64_t* now, uint32_t* err, hipStream_t st);
// The same over descriptors [d0, d1) and requests [q0, q1) of the batch (a
// multi-shard ctx's slice: buf mirrors the host buffer's layout, only the
// slice's parts present; the outputs at the same absolute indices).
void launch_unpack_range(const rl_batch_compact& cb, const uint8_t* buf, uint32_t d0, uint32_t d1, uint32_t q0,
                         uint32_t q1, uint32_t* req, uint8_t* unit, uint8_t* flags, uint32_t* limit, uint32_t* hits,
                         uint32_t* rule, int64_t* now, uint32_t* err, hipStream_t st);
// A prefix-shared host batch (rl_batch_prefixed; buf = the device copy of its
// buffer, or of a slice's parts at the host buffer's offsets): tiles [t0, t1)
// -> the rl_batch arrays at their absolute indices, stems rebuilt into `stem`
// at the index's stem offsets, off[] the stem offsets (off[n] included). The
// totals come from the host buffer's last index entry (already checked). A
// tile whose entry does not match its sections sets ERR_INVALID in *err.
// Device -> page-locked host copies done by a kernel's vector stores over
// PCIe (posted writes), not by the DMA engine: the host-fed paths' outputs
// then cross back while the next batch's input copy holds the engine
// (an SDMA D2H copy queues behind it). dst[k] are device-visible host
// addresses (hipHostGetDevicePointer).
constexpr uint32_t TO_HOST_MAX = 6;
struct ToHost {
  const uint8_t* src[TO_HOST_MAX];
  uint8_t* dst[TO_HOST_MAX];
  uint64_t bytes[TO_HOST_MAX];
  uint32_t n;
};
void launch_to_host(const ToHost& c, hipStream_t st);
// The copies of c (dst: host addresses as the caller holds them) by k_to_host
// when every dst is page-locked, else by hipMemcpyAsync.
hipError_t copy_to_host(ToHost c, hipStream_t st);

void launch_unpack_prefixed(const rl_batch_prefixed& pb, const uint8_t* buf, uint32_t t0, uint32_t t1, uint8_t* stem,
                            uint32_t* off, uint32_t* req, uint8_t* unit, uint8_t* flags, uint32_t* limit,
                            uint32_t* hits, uint32_t* rule, int64_t* now, uint32_t* err, hipStream_t st);
// counts: cstride u64 per owner (records, stem bytes[, meta0, meta1]).
// own_rank < n_shards: that owner's descriptors get a perm entry only (no
// wire record, no stem bytes: its owner batch reads them in place,
// BatchDev::own). hash_out: where the stem hashes go (null: the scratch's).
constexpr uint32_t ROUTE_OWN_NONE = 0xFFFFFFFFu;
// Stem offsets of n received wire records: woff[j] = the lengths of records
// [0, j) summed, the records [olo, ohi) (the own chunk, stems read in place)
// counted as 0; woff[n] = the total. A sum past 32 bits saturates (the owner's
// bounds check then fails the record). Every source's chunk must start at its
// base (wbase[src], device) and end at the next one's (the last at
// stem_total): else tsum[WIRE_SCAN_TILES(n)] (the scan's verdict word,
// BatchDev::wbad) is set and the owner batches reading these offsets fail
// (RL_E_INVALID) instead of reading shifted keys. tsum: WIRE_SCAN_WORDS(n).
constexpr uint32_t WIRE_SCAN_TILE = 2048;
inline uint32_t WIRE_SCAN_TILES(uint64_t n) { return (uint32_t)((n + WIRE_SCAN_TILE) / WIRE_SCAN_TILE); }
inline uint32_t WIRE_SCAN_WORDS(uint64_t n) { return WIRE_SCAN_TILES(n) + 1; }
void launch_wire_offsets(const Wire* w, uint32_t n, uint32_t olo, uint32_t ohi, const unsigned long long* wbase,
                         uint32_t n_src, unsigned long long stem_total, uint32_t* woff, unsigned long long* tsum,
                         hipStream_t st);
void launch_route_pack(const BatchDev& b, uint32_t n_shards, uint32_t src_rank, Wire* out, uint8_t* out_stem,
                       uint32_t* perm, unsigned long long* counts, const Scratch& s, hipStream_t st,
                       uint32_t cstride = 2, unsigned long long meta0 = 0, unsigned long long meta1 = 0,
                       uint32_t own_rank = ROUTE_OWN_NONE, unsigned long long* hash_out = nullptr,
                       unsigned long long* counts_host = nullptr);
// The counts of a slice that failed on the host (zero records and bytes, meta words set).
void launch_cnt_fill(unsigned long long* cnt, uint32_t n_peers, uint32_t cstride, unsigned long long meta0,
                     unsigned long long meta1, hipStream_t st, unsigned long long* cnt_host = nullptr);
// ret[0, n) = a failed record's packed result with rl_status `status`.
void launch_route_fail(unsigned long long* ret, uint32_t n, uint32_t status, hipStream_t st);
// src_err (optional): without o.status, a returned failure status sets its
// error bit there (the source's batch then fails at rl_synchronize). errb
// (optional): ret is an owner batch's own results; a failed batch (*errb)
// answers every record with its status, as k_route_ret does. Records
// [own_lo, own_hi) are the own chunk, answered in place by the owner batch's
// k_finish (OwnChunk outputs): skipped (all of them: no launch).
void launch_route_scatter(const uint32_t* perm, const unsigned long long* ret, uint32_t n, const OutDev& o,
                          hipStream_t st, uint32_t* src_err = nullptr, const uint32_t* errb = nullptr,
                          uint32_t own_lo = 0, uint32_t own_hi = 0);
// Owner side: ret[i] = res[i], or every record failed with the status of
// *errb when the batch's table stage failed.
void launch_route_ret(const unsigned long long* res, uint32_t n, const uint32_t* errb, unsigned long long* ret,
                      hipStream_t st);
// out[i] = sum over blocks b of stage[b * stride + i], i < m (stride 0: m).
void launch_stats_sum(const unsigned long long* stage, uint32_t n_blocks, uint32_t m, unsigned long long* out,
                      hipStream_t st, uint32_t stride = 0);
// The epoch sweep: evict the slots whose records (cur and logged) are all dead.
void launch_sweep(const TableDev& t, uint64_t nslots, uint32_t now, unsigned long long* evicted, hipStream_t st);
void launch_arena_compact(Slot* slots, uint64_t nslots, const uint8_t* from, uint8_t* to, unsigned long long* used16,
                          hipStream_t st);
void launch_lc_count(const TableDev& t, uint64_t nslots, uint32_t now, unsigned long long* out, hipStream_t st);
void launch_table_info(const Slot* slots, uint64_t nslots, unsigned long long* out, hipStream_t st);
// Built with RL_LOG_TEAR (rl_debug_log_tear's hook in the history log's lookups)?
bool log_tear_hook();
void launch_debug_keys(const BatchDev& b, uint8_t* out, uint32_t* klen, hipStream_t st);
void launch_debug_decide(uint32_t n, const uint32_t* before, const uint32_t* after, const uint8_t* lc_hit,
                         const uint32_t* hits, const uint32_t* limit, const uint8_t* unit, const uint8_t* flags,
                         const int64_t* now, float ratio, int lc_en, uint8_t* code, uint32_t* rem, uint32_t* reset,
                         unsigned long long* deltas, uint8_t* lc_set, hipStream_t st);

}  // namespace rl
