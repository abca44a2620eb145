// rl_engine.h — one table shard on one GPU: the HBM table, the per-batch
// scratch of the pipeline buffers, and the HIP streams and events that order
// them (rl_engine.hip). The C ABI (rl_api.hip) drives one engine per shard; a
// ctx with one shard is one engine.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ratelimit_hip.h"
#include "rl_device.h"
#include "rl_kernels.h"
#include "rl_match.h"

namespace rl {

// Pipeline depth: scratch buffers (and streams) in flight. Stage A of up to
// NBUF - 1 later batches may run while one batch's stage B holds the table.
#ifndef RL_NBUF
#define RL_NBUF 4
#endif
constexpr uint32_t NBUF = RL_NBUF;
// errw words: [0, NBUF) stage A of each buffer, [NBUF] (unused), [NBUF + 1]
// the soft word (per-descriptor statuses), [NBUF + 2] the routing partition,
// [ERRW_B0 + j] the table-stage words, one per batch in a ring of ERRB_RING
// (a batch's word is set at the end of its stage A, while up to NBUF - 1
// earlier batches may still read theirs and their predecessors')
constexpr uint32_t ERRB_RING = 2 * NBUF;
constexpr uint32_t ERRW_B0 = NBUF + 3, ERRW_WORDS = ERRW_B0 + ERRB_RING;
constexpr uint32_t PROF_RING = 8;  // timed batches in flight (> NBUF)
constexpr uint32_t PROGRESS_RING = 64;  // batches rl_batch_progress tracks in flight

// Device staging of one host-fed batch in flight (eng_do_limit_host_async).
struct HostSlot {
  uint8_t* stem = nullptr;
  uint32_t *off = nullptr, *req = nullptr, *limit = nullptr, *hits = nullptr, *rule = nullptr;
  int64_t* now = nullptr;
  uint8_t *unit = nullptr, *flags = nullptr;
  uint8_t *code = nullptr, *status = nullptr;
  uint32_t *rem = nullptr, *reset = nullptr;
  unsigned long long* stats = nullptr;
  uint8_t* cbuf = nullptr;        // a compact batch's buffer (rl_do_limit_compact_async), allocated on first use
  uint64_t cbuf_cap = 0;
  hipEvent_t in_done = nullptr;   // its inputs are on the device
  hipEvent_t out_done = nullptr;  // its outputs are back on the host (the slot is free)
};

struct Engine {
  rl_config cfg;
  hipStream_t stream = nullptr;   // serial work (== pipe[0])
  hipStream_t pipe[NBUF] = {};    // one per scratch buffer
  hipEvent_t b_done[NBUF] = {};   // stage B of the last batch on each buffer is done
  hipEvent_t b_table[NBUF] = {};  // ... its table kernels are (the next batch's stage B waits for this)
  hipEvent_t consumed[NBUF] = {}; // a routed owner batch's packed results (s[k].res) have been read
  hipEvent_t route_ready = nullptr;  // eng_route_do_limit: the caller's received buffers are ready
  hipEvent_t caller_ready = nullptr; // eng_do_limit_async: the caller stream's work so far (the inputs)
  bool serial_debug = false;         // RL_DEBUG_SERIAL: async batches run serially on the caller's stream
  uint32_t next = 0, last = NBUF - 1;  // buffer of the next / of the latest batch
  uint32_t errb_seq = NBUF;            // table-stage word of the next batch (ring position)
  bool b_early = true;                 // k_b_begin at the end of stage A (RL_B_BEGIN_EARLY=0: in the table chain)
  uint64_t hash_seed = 0;
  HashKey hk{};
  // table
  Slot* slots = nullptr;
  uint64_t nslots = 0;
  // the history log (window records below the slots' cur, rl_device.h):
  // LOG_PARTS partitions of log_cap entries, their append counters (one
  // 128-B line each; the line after them: the lookups that found an entry
  // overwritten), and the horizon J in seconds
  LogEnt* log = nullptr;
  uint32_t log_cap = 0;
  unsigned long long* log_ctr = nullptr;
  uint32_t horizon = 0;
  uint32_t* tear = nullptr;  // rl_debug_log_tear's armed state (device; RL_LOG_TEAR builds)
  // RL_DEBUG_COPYTIME: host-fed input copies timed with events (stderr at destroy)
  bool copy_time = false;
  // RL_DEBUG_HOSTTIME: host seconds per section of the host-fed prefixed path (stderr at destroy)
  bool host_time = false;
  double ht[8] = {};
  uint64_t ht_n = 0;
  hipEvent_t ct_ev[3][64] = {};  // copy start, copy end, before the slot wait
  uint32_t ct_n = 0;
  double ct_ms = 0, ct_wait_ms = 0, ct_gap_ms = 0;
  uint64_t ct_count = 0;
  uint8_t* arena = nullptr;
  uint8_t* arena2 = nullptr;  // compaction target (rl_sweep), swapped with arena
  uint64_t arena_cap16 = 0;
  // scratch: s[k] per buffer; stripes, counters, time floor, routing and the
  // table-stage error word are shared
  Scratch s[NBUF]{};
  Scratch rs{};                 // routing partition (eng_route_pack), allocated on first use
  bool rs_ready = false;
  unsigned long long* h_base = nullptr;  // pinned [NBUF][RL_MAX_SHARDS] routed chunk bases
  uint32_t* errw = nullptr;  // [0, NBUF) stage-A words of the buffers, [NBUF] stage-B word, [NBUF+1] soft word
  // device staging for the host-buffer entry points
  uint8_t* d_stem = nullptr;
  uint32_t *d_off = nullptr, *d_req = nullptr, *d_limit = nullptr, *d_hits = nullptr, *d_rule = nullptr;
  int64_t* d_now = nullptr;
  uint8_t *d_unit = nullptr, *d_flags = nullptr, *d_code = nullptr, *d_status = nullptr;
  uint32_t *d_rem = nullptr, *d_reset = nullptr;
  unsigned long long* d_stats = nullptr;
  uint32_t* h_err = nullptr;  // pinned [4]
  // k_split_long (the runs over 1024 elements on 1024-lane workgroups) is
  // launched only while recent batches had such runs: k_split writes a
  // buffer's word when it meets one; an empty launch of 1024-lane workgroups
  // costs C1 / C2 about 1-2.5 % (profiles/r05/split_long/)
  uint32_t* h_long = nullptr;  // pinned [NBUF]
  uint32_t long_recent = 0;    // batches left in long-run mode
  int long_mode = 1;           // RL_SPLIT_LONG: 0 never, 1 while recent batches had long runs, 2 always
  uint32_t* h_big = nullptr;   // pinned [NBUF]: k_bucket queued a large bucket (hot keys)
  uint32_t big_recent = 0;     // batches left with full large-bucket grids
  int big_mode = 1;            // RL_BIG_CUE: 0 full grids always, 1 while recent batches had large buckets
  uint32_t* h_late = nullptr;  // pinned [NBUF]: k_late met a long run (RUN_FAST) in this buffer's batch
  uint32_t late_recent = 0;    // batches left with k_late's full long-run grid
  int late_mode = 1;           // RL_LATE_CUE: 0 full grid always, 1 while recent batches had long runs
  unsigned long long* h_counters = nullptr;
  std::string last_error;
  uint64_t batches = 0, decisions = 0;
  // rl_profile: a ring of per-batch event sets (stage boundaries, recorded on
  // the batch's own stream, so pipelined batches are timed as they run),
  // folded into the stage sums when a set is reused or read
  bool prof = false;
  uint32_t prof_every = 1, prof_skip = 0;  // time every prof_every-th batch
  bool prof_pending[PROF_RING] = {};
  uint32_t prof_next = 0;
  hipEvent_t ev[PROF_RING][RL_NUM_STAGES + 1] = {};
  double stage_ms[RL_NUM_STAGES] = {};
  uint64_t prof_batches = 0;
  // ... and k_table's own run time on those batches (device
  // clock): {sum of durations in ticks, batches}, and the clock's rate (kHz)
  unsigned long long* d_kt_acc = nullptr;
  double wclk_khz = 0;
  // config match (rl_config_load / rl_do_limit_requests): the device trie and
  // one growable device buffer carved per call for the raw requests
  uint8_t* cfg_blob = nullptr;  // [nodes | index | prefix ‖ keys]
  CfgDev cfg_dev{};
  bool cfg_loaded = false;
  uint8_t* mbuf = nullptr;
  size_t mbuf_cap = 0;
  uint32_t* h_match = nullptr;  // pinned [4]: matched count, stem bytes, error bits
  // host-fed async batches: NBUF staging slots and two copy streams, so that
  // batch t+1's inputs cross PCIe and batch t-1's outputs come back while
  // batch t's kernels run (allocated on first use)
  HostSlot hs[NBUF]{};
  hipStream_t h2d = nullptr, d2h = nullptr;
  uint32_t hnext = 0;
  bool hs_ready = false;
  // rl_batch_progress: batches submitted through the batch entry points and
  // the ones whose outputs are complete, from a ring of completion events
  uint64_t seq_sub = 0, seq_done = 0;
  hipEvent_t done_ring[PROGRESS_RING] = {};
};

// Engine entry points (rl_engine.hip): the single-shard implementations of
// the C ABI functions of the same name (rl_x -> eng_x).
// A non-blocking stream of one of the library's roles. A stream created the
// usual way shares one of the process's GPU_MAX_HW_QUEUES hardware queues with
// other streams, and a marker or kernel queued on it waits behind whatever the
// other stream queued first; RL_DEDICATED_QUEUES (bits: 1 router streams, 2
// host copy streams, 4 pipeline streams) gives a role's streams queues of
// their own (a CU-masked queue with every CU enabled).
enum StreamRole : uint32_t { SR_ROUTER = 1, SR_HOSTCOPY = 2, SR_PIPE = 4 };
hipError_t rl_stream_create(hipStream_t* st, uint32_t role);
Engine* eng_create(const rl_config* cfg, char* err, size_t errlen);
void eng_destroy(Engine* c);
const char* eng_last_error(const Engine* c);
int eng_do_limit(Engine* c, const rl_batch* in, rl_result* out);
int eng_do_limit_async(Engine* c, const rl_batch* in, rl_result* out, void* stream);
int eng_do_limit_host_async(Engine* c, const rl_batch* in, rl_result* out);
int eng_do_limit_compact_async(Engine* c, const rl_batch_compact* in, rl_result* out);
// The compact batch's sizes and sections against the ctx's limits (no GPU work).
int eng_compact_check(Engine* c, const rl_batch_compact* in, const rl_result* out);
int eng_do_limit_prefixed_async(Engine* c, const rl_batch_prefixed* in, rl_result* out);
// The prefix-shared batch's sizes, sections and index ends against the ctx's
// limits (no GPU work); *tiles = its request tiles.
int eng_prefixed_check(Engine* c, const rl_batch_prefixed* in, const rl_result* out, uint32_t* tiles);
int eng_synchronize(Engine* c);
int eng_batch_progress(Engine* c, uint64_t* submitted, uint64_t* completed);
int eng_sweep(Engine* c, int64_t now, uint64_t* n_evicted);
int eng_restore(Engine* c, const rl_restore_batch* in);
int eng_table_info_get(Engine* c, rl_table_info* info);
int eng_debug_keys(Engine* c, const rl_batch* in, uint8_t* out_bytes, uint32_t* out_off, uint32_t out_cap);
int eng_debug_log_tear(Engine* c, const rl_log_tear* arm, rl_log_tear* out);
int eng_debug_decide(Engine* c, uint32_t n, const uint32_t* before, const uint32_t* after, const uint8_t* lc_hit,
                     const uint32_t* hits, const uint32_t* limit, const uint8_t* unit, const uint8_t* flags,
                     const int64_t* now, uint8_t* code, uint32_t* remaining, uint32_t* reset_s, uint64_t* stat_deltas,
                     uint8_t* lc_set);
// counts: cstride u64 per owner (records, stem bytes[, meta0, meta1]: the
// in-library router's counts message).
// A partition's own scratch (the router's slots: partitions of consecutive
// batches run on different pipeline streams, concurrently): owner per
// descriptor [max_batch], per-tile counts [2 x n_shards x tiles], totals
// [2 x n_shards + 1]. Null: the engine's single routing scratch (c->rs).
struct RouteBufs {
  uint8_t* dest;
  uint32_t* hist;
  uint32_t* start;
};
int eng_route_pack(Engine* c, const rl_batch* in, uint32_t n_shards, uint32_t src_rank, void* send_rec,
                   uint8_t* send_stem, uint32_t* perm, uint64_t* counts, void* stream, uint32_t cstride = 2,
                   uint64_t meta0 = 0, uint64_t meta1 = 0, uint32_t own_rank = ROUTE_OWN_NONE,
                   unsigned long long* hash_out = nullptr, unsigned long long* counts_host = nullptr,
                   const RouteBufs* bufs = nullptr);
int eng_route_do_limit(Engine* c, uint32_t n, const void* recv_rec, const uint8_t* recv_stem, uint64_t recv_stem_bytes,
                       const uint64_t* src_stem_base, uint32_t n_shards, uint32_t n_rules, uint32_t rule_stride,
                       uint64_t* ret, uint64_t* stats, int isolate, void* stream);
int eng_route_scatter(Engine* c, uint32_t n, const uint32_t* perm, const uint64_t* ret, rl_result* out, void* stream);
int eng_profile(Engine* c, int enable);
int eng_profile_read(Engine* c, double* ms, uint32_t n, uint64_t* batches);
int eng_config_load(Engine* c, const rl_config_tree* tree);
// The DoLimit step of eng_do_limit_requests done elsewhere (a multi-shard
// ctx's shards): the matched batch and the result arrays in device memory of
// c's GPU, inputs ready on `st`; returns once the results are complete.
using RequestsDoLimit = int (*)(void* user, const rl_batch* dev_in, rl_result* dev_out, hipStream_t st);
int eng_do_limit_requests(Engine* c, const rl_request_batch* in, rl_request_result* out, RequestsDoLimit run = nullptr,
                          void* user = nullptr);
int eng_local_cache_info_get(Engine* c, int64_t now, rl_local_cache_info* info);
int eng_snapshot_size(Engine* c, uint64_t* bytes);
int eng_snapshot_save(Engine* c, void* host, uint64_t bytes);
int eng_snapshot_load(Engine* c, const void* host, uint64_t bytes);

// Owner side of a routed batch, pipelined on the engine's streams like
// eng_do_limit_async: unpack the n received wire records (chunks of n_src
// sources, concatenated in source order, stems in recv_stem) and enqueue the
// DoLimit pipeline once `ready` (an event of any device, or null) has fired.
// rule_stride > 0 attributes stats per source: rule' = source x rule_stride +
// rule (stats then holds n_src blocks of rule_stride x RL_NUM_STATS). The
// packed results land in s[*slot].res (record order); b_done[*slot] marks
// them complete and the reader must record consumed[*slot] once it has copied
// them (the buffer is not reused before). own (optional, own->n > 0): records
// [own->lo, own->lo + own->n) are read in place from the source batch
// (BatchDev::own; recv_rec holds nothing there). woff, wbad (optional): the
// records' stem offsets and the scan's verdict word (launch_wire_offsets over
// the whole exchange, when it runs in parts); null: scanned here.
int eng_route_owner(Engine* c, uint32_t n, const Wire* recv_rec, const uint8_t* recv_stem, uint64_t recv_stem_bytes,
                    const uint64_t* src_stem_base, uint32_t n_src, uint32_t n_rules, uint32_t rule_stride,
                    unsigned long long* stats, int isolate, hipEvent_t ready, uint32_t* slot,
                    const OwnChunk* own = nullptr, const uint32_t* woff = nullptr,
                    const unsigned long long* wbad = nullptr);

// Record an error on the engine (its rl_last_error) and return code.
int eng_fail(Engine* c, int code, const std::string& msg);

// Per-batch scratch arrays (rl_engine.hip), for the router's own partition.
bool scratch_alloc(Scratch& s, uint32_t n);
void scratch_free(Scratch& s);

}  // namespace rl
