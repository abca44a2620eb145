// rl_api.hip — the extern "C" boundary of libratelimit_hip.so
// (include/ratelimit_hip.h). Owns the HBM table, two sets of per-batch scratch
// and the HIP streams; every entry point maps the device error words to an
// rl_status.
//
// Batches submitted with eng_do_limit_async(stream = NULL) are pipelined: batch
// t's table-free stage A (validate, hash, sort, segment) runs on scratch buffer
// t % NBUF and that buffer's stream while batch t-1's stage B (the table) still
// runs. Stage B of every batch waits for the previous batch's stage B (an
// event chain), so the table sees batches in submission order and every key
// sees the reference's sequential INCRBY order. Every other call is serial and
// ordered after all submitted batches.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ratelimit_hip.h"
#include "rl_device.h"
#include "rl_kernels.h"
#include "rl_match.h"
#include "rl_engine.h"

using namespace rl;



namespace {

thread_local std::string g_err;

int set_err(Engine* c, int code, const std::string& msg);

// Fold event set k (a timed batch) into the stage sums; waits for the batch.
void prof_fold(Engine* c, uint32_t k) {
  if (!c->prof_pending[k]) return;
  c->prof_pending[k] = false;
  if (hipEventSynchronize(c->ev[k][RL_NUM_STAGES]) != hipSuccess) return;
  for (int i = 0; i < RL_NUM_STAGES; i++) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->ev[k][i], c->ev[k][i + 1]) == hipSuccess) c->stage_ms[i] += ms;
  }
  c->prof_batches++;
}

void prof_fold_all(Engine* c) {
  for (uint32_t k = 0; k < PROF_RING; k++) prof_fold(c, (c->prof_next + k) % PROF_RING);
}

hipEvent_t* prof_events(Engine* c) {
  if (!c->prof) return nullptr;
  if (c->prof_skip) {
    c->prof_skip--;
    return nullptr;
  }
  c->prof_skip = c->prof_every - 1;
  const uint32_t k = c->prof_next;
  c->prof_next = (k + 1) % PROF_RING;
  prof_fold(c, k);  // the batch that used this set PROF_RING batches ago
  c->prof_pending[k] = true;
  return c->ev[k];
}

int set_err(Engine* c, int code, const std::string& msg) {
  if (c) c->last_error = msg;
  else g_err = msg;
  return code;
}

#define HIPCHK(c, expr)                                                                        \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return set_err((c), RL_E_HIP, std::string("gpu: ") + #expr + ": " + hipGetErrorString(_e)); \
  } while (0)

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

inline double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int map_err(Engine* c, uint32_t e) {
  if (!e) return RL_OK;
  if (e & ERR_TIME) return set_err(c, RL_E_TIME, "gpu: now outside [0, 2^32-172800] or before the last sweep");
  if (e & ERR_HISTORY)
    return set_err(c, RL_E_TIME,
                   "gpu: a request's window is older than its key's history holds (more than 8 windows and "
                   "div + expiration_jitter_max_seconds behind the key's newest, or the history log overwrote it: "
                   "raise history_entries)");
  if (e & ERR_INVALID) return set_err(c, RL_E_INVALID, "gpu: malformed batch (unit, rule id, request index or stem offsets)");
  if (e & ERR_TABLE_FULL) return set_err(c, RL_E_TABLE_FULL, "gpu: counter table full (raise table_slots or sweep)");
  if (e & ERR_ARENA_FULL) return set_err(c, RL_E_ARENA_FULL, "gpu: long-stem arena full (raise arena_bytes)");
  return set_err(c, RL_E_INTERNAL, "gpu: unknown device error");
}

// Order stream st after every batch submitted so far: each buffer's last
// batch to its end (a batch's k_finish may still run after the next batch's
// stage B has started: that waits for b_table only).
hipError_t after_batches(Engine* c, hipStream_t st) {
  for (uint32_t k = 0; k < NBUF; k++) {
    const hipError_t e = hipStreamWaitEvent(st, c->b_done[k], 0);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Read (and clear) the sticky device error words; synchronises the stream,
// which must already be ordered after all submitted work.
// The soft word (descriptor errors answered by statuses) is cleared, not reported.
int collect(Engine* c, hipStream_t st = nullptr) {
  if (!st) st = c->stream;
  HIPCHK(c, hipMemcpyAsync(c->h_err, c->errw, ERRW_WORDS * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  uint32_t e = c->h_err[NBUF + 2];  // the routing partition's word
  for (uint32_t j = 0; j < NBUF; j++) e |= c->h_err[j];
  for (uint32_t j = 0; j < ERRB_RING; j++) e |= c->h_err[ERRW_B0 + j];
  if (e || c->h_err[NBUF + 1]) {
    HIPCHK(c, hipMemsetAsync(c->errw, 0, ERRW_WORDS * sizeof(uint32_t), st));
    HIPCHK(c, hipStreamSynchronize(st));
  }
  return map_err(c, e);
}

TableDev table_view(Engine* c);
Params params(Engine* c, int isolate = 0);

// Enqueue one batch. Pipelined (ctx streams): stage A on the buffer's own
// stream as soon as the buffer is free, stage B after the previous batch's
// stage B. Serial: both stages on `st` after all earlier work. With rl_profile
// on, the stage boundaries are recorded on the batch's stream either way.
uint32_t enqueue(Engine* c, const BatchDev& b_in, const OutDev& o, int restore, hipStream_t st, bool pipelined) {
  const uint32_t k = c->next;
  const BatchDev& b = b_in;
  c->next = (k + 1) % NBUF;
  TableDev t = table_view(c);
  t.log_epoch = c->s[k].log_epoch;  // (k_b_begin sets it for this batch)
  const int isolate = (!restore && o.status) ? 1 : 0;
  const Params P = params(c, isolate);
  const uint32_t* errb_prev = c->s[c->last].errb;  // the previous batch's table-stage word
  c->s[k].errb = c->errw + ERRW_B0 + (c->errb_seq++ % ERRB_RING);
  const bool early = c->b_early;
  bool lng = c->long_mode == 2;  // k_split_long for this batch: a recent batch had a run over 1024 elements
  if (c->long_mode == 1) {
    for (uint32_t j = 0; j < NBUF; j++)
      if (__atomic_load_n(&c->h_long[j], __ATOMIC_RELAXED)) {
        __atomic_store_n(&c->h_long[j], 0u, __ATOMIC_RELAXED);
        c->long_recent = 4 * NBUF;
      }
    lng = c->long_recent > 0;
    if (c->long_recent) c->long_recent--;
  }
  uint32_t* hint = c->long_mode ? c->h_long + k : nullptr;
  // the large-bucket kernels' grids: full while recent batches had a bucket
  // too large for k_bucket (hot keys: C2, C2U), one workgroup each otherwise
  // (C1, C3): they are grid-stride, so an unexpected one is still sorted
  bool big_full = c->big_mode == 0;
  if (c->big_mode == 1) {
    for (uint32_t j = 0; j < NBUF; j++)
      if (__atomic_load_n(&c->h_big[j], __ATOMIC_RELAXED)) {
        __atomic_store_n(&c->h_big[j], 0u, __ATOMIC_RELAXED);
        c->big_recent = 4 * NBUF;
      }
    big_full = c->big_recent > 0;
    if (c->big_recent) c->big_recent--;
  }
  uint32_t* bhint = c->big_mode == 1 ? c->h_big + k : nullptr;
  // k_late's long-run part likewise: one workgroup per 256 sorted positions
  // while recent batches had long runs, else a few that walk the bitmap
  bool late_full = c->late_mode == 0;
  if (c->late_mode == 1) {
    for (uint32_t j = 0; j < NBUF; j++)
      if (__atomic_load_n(&c->h_late[j], __ATOMIC_RELAXED)) {
        __atomic_store_n(&c->h_late[j], 0u, __ATOMIC_RELAXED);
        c->late_recent = 4 * NBUF;
      }
    late_full = c->late_recent > 0;
    if (c->late_recent) c->late_recent--;
  }
  uint32_t* lhint = c->late_mode == 1 ? c->h_late + k : nullptr;
  if (pipelined) {
    hipStream_t a = c->pipe[k];
    hipEvent_t* ev = prof_events(c);
    (void)hipStreamWaitEvent(a, c->b_done[k], 0);    // buffer k's previous batch is done
    (void)hipStreamWaitEvent(a, c->consumed[k], 0);  // ... and its routed results were read
    launch_stage_a(b, c->s[k], isolate, P.per_second, a, ev, hint, lng, bhint, big_full);
    if (early) launch_b_begin_early(b, o, c->s[k], restore, a, c->log_ctr);  // (off the table-order chain)
    (void)hipStreamWaitEvent(a, c->b_table[c->last], 0);  // table order (not the previous k_finish)
    launch_stage_b(b, o, t, P, c->s[k], restore, a, ev, errb_prev, c->b_table[k], ev ? c->d_kt_acc : nullptr,
                   early, lhint, late_full);
    (void)hipEventRecord(c->b_done[k], a);
  } else {
    if (!st) st = c->stream;
    (void)after_batches(c, st);
    hipEvent_t* ev = prof_events(c);
    launch_stage_a(b, c->s[k], isolate, P.per_second, st, ev, hint, lng, bhint, big_full);
    if (early) launch_b_begin_early(b, o, c->s[k], restore, st, c->log_ctr);
    launch_stage_b(b, o, t, P, c->s[k], restore, st, ev, errb_prev, c->b_table[k], ev ? c->d_kt_acc : nullptr,
                   early, lhint, late_full);
    (void)hipEventRecord(c->b_done[k], st);
  }
  c->last = k;
  return k;
}

// A batch submitted through a batch entry point is complete once the work now
// on `st` is (its outputs written; host-fed: copied back). Keeps at most
// PROGRESS_RING batches tracked: a caller that runs further ahead waits here
// for the oldest one (never in a paced server).
hipError_t track(Engine* c, hipStream_t st) {
  if (c->seq_sub - c->seq_done >= PROGRESS_RING) {
    const hipError_t e = hipEventSynchronize(c->done_ring[c->seq_done % PROGRESS_RING]);
    if (e != hipSuccess) return e;
    c->seq_done++;
  }
  const hipError_t e = hipEventRecord(c->done_ring[c->seq_sub % PROGRESS_RING], st);
  c->seq_sub++;
  return e;
}

int check_sizes(Engine* c, const rl_batch* in, uint64_t stem_bytes) {
  if (!in) return set_err(c, RL_E_INVALID, "gpu: null batch");
  if (in->n > c->cfg.max_batch || in->n_requests > c->cfg.max_requests || in->n_rules > c->cfg.max_rules ||
      stem_bytes > c->cfg.max_stem_bytes)
    return set_err(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_rules/max_stem_bytes");
  if (in->n && in->n_requests == 0) return set_err(c, RL_E_INVALID, "gpu: descriptors without requests");
  return RL_OK;
}

BatchDev dev_view(const Engine* c, const rl_batch* in, uint32_t stem_cap) {
  BatchDev b{};
  b.hk = c->hk;
  b.n = in->n;
  b.n_req = in->n_requests;
  b.n_rules = in->n_rules;
  b.stem_cap = stem_cap;
  b.stem_total = stem_cap;  // refined on the device from off[n]
  b.now_desc = 0;
  b.stem = in->stem_bytes;
  b.off = in->stem_off;
  b.now = in->now;
  b.req = in->req_idx;
  b.unit = in->unit;
  b.flags = in->flags;
  b.limit = in->limit;
  b.hits = in->hits;
  b.rule = in->rule_id;
  return b;
}

// The history log's append counters (LOG_PARTS) and its lost-lookup count.
hipError_t log_ctr_get(Engine* c, std::vector<unsigned long long>& ctr, unsigned long long* lost,
                       unsigned long long* refused = nullptr) {
  std::vector<unsigned long long> h((size_t)(LOG_PARTS + 1) * LOG_CTR_STRIDE);
  hipError_t e = hipMemcpyAsync(h.data(), c->log_ctr, h.size() * 8, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return e;
  ctr.resize(LOG_PARTS);
  for (uint32_t k = 0; k < LOG_PARTS; k++) ctr[k] = h[(size_t)k * LOG_CTR_STRIDE];
  if (lost) *lost = h[(size_t)LOG_PARTS * LOG_CTR_STRIDE];
  if (refused) *refused = h[(size_t)LOG_PARTS * LOG_CTR_STRIDE + 1];
  return hipSuccess;
}

TableDev table_view(Engine* c) {
  TableDev t;
  t.slots = c->slots;
  t.log = c->log;
  t.log_ctr = c->log_ctr;
  t.log_cap = c->log_cap;
  t.horizon = c->horizon;
  t.hist_lost = c->log_ctr + (size_t)LOG_PARTS * LOG_CTR_STRIDE;
  t.tear = c->tear;
  t.log_epoch = nullptr;  // (a batch's: enqueue)
  t.mask = c->nslots - 1;
  t.arena = c->arena;
  t.arena_used16 = c->s[0].counters + 4;
  t.arena_cap16 = c->arena_cap16;
  t.max_probe = (uint32_t)std::min<uint64_t>(c->nslots, 1u << 16);
  t.shift = 64u - (uint32_t)__builtin_ctzll(c->nslots);
  return t;
}

Params params(Engine* c, int isolate) {
  Params P;
  P.ratio = c->cfg.near_limit_ratio;
  P.lc_en = c->cfg.local_cache_enabled != 0;
  P.per_second = c->cfg.per_second_split != 0;
  P.isolate = isolate;
  return P;
}

// Per-batch scratch of one pipeline buffer (sized for max_batch descriptors).
bool alloc_buffer(Scratch& s, uint32_t n) {
  const size_t items = (size_t)n / (64 * 4 * 8) + 1 + PART_DIGITS;  // BIG_CHUNK-position work items
  bool ok = dalloc(&s.big_meta, PART_DIGITS) == hipSuccess && dalloc(&s.big_n, 1) == hipSuccess &&
            dalloc(&s.big_work, items) == hipSuccess && dalloc(&s.work_n, 1) == hipSuccess &&
            dalloc(&s.sorted_n, 1) == hipSuccess &&
            dalloc(&s.big_cnt, items * (1 + 2 * BIG_HEAVY)) == hipSuccess;
  ok = ok && dalloc(&s.rec, n) == hipSuccess && dalloc(&s.res, n) == hipSuccess;
  for (int i = 0; i < 2; i++) ok = ok && dalloc(&s.keys[i], n) == hipSuccess && dalloc(&s.vals[i], n) == hipSuccess;
  ok = ok && dalloc(&s.grp, n) == hipSuccess && dalloc(&s.lead, n) == hipSuccess && dalloc(&s.gmask, n) == hipSuccess &&
       dalloc(&s.defer, n) == hipSuccess &&
       dalloc(&s.defer_n, 1) == hipSuccess && dalloc(&s.defer2, n) == hipSuccess &&
       dalloc(&s.defer1, n) == hipSuccess && dalloc(&s.defer1_n, 1) == hipSuccess &&
       dalloc(&s.defer2_n, 1) == hipSuccess && dalloc(&s.fast_blk, (size_t)n / (256 * 32) + 1) == hipSuccess &&
       dalloc(&s.log_epoch, LOG_PARTS) == hipSuccess &&
       dalloc(&s.uniq, n) == hipSuccess && dalloc(&s.uniq_n, 1) == hipSuccess &&
       dalloc(&s.long_runs, (size_t)n / 1024 + 2) == hipSuccess &&
       dalloc(&s.kt_blk, 2 * ((size_t)n / 2 + BIG_HEAVY * PART_DIGITS + 2 * (size_t)n + 512) / 256) == hipSuccess;
  ok = ok && dalloc(&s.hits_s, n) == hipSuccess && dalloc(&s.segsum, n) == hipSuccess &&
       dalloc(&s.rid, n) == hipSuccess && dalloc(&s.run_start, (size_t)n + 1) == hipSuccess &&
       dalloc(&s.run_flags, n) == hipSuccess && dalloc(&s.run_state, n) == hipSuccess && dalloc(&s.run_alias, n) == hipSuccess &&
       dalloc(&s.run_f, n) == hipSuccess &&
       dalloc(&s.runs64, 1) == hipSuccess && dalloc(&s.split, 2) == hipSuccess && dalloc(&s.drun, (size_t)n / 2 + BIG_HEAVY * PART_DIGITS) == hipSuccess;
  ok = ok && dalloc(&s.hit_a, n) == hipSuccess && dalloc(&s.tile, n) == hipSuccess &&
       dalloc(&s.hit_t, n) == hipSuccess;
  ok = ok && dalloc(&s.run_end, n) == hipSuccess &&
       dalloc(&s.part_info, (size_t)PART_DIGITS * std::max((n + PART_TILE - 1) / PART_TILE, 1u)) == hipSuccess;
  ok = ok && dalloc(&s.r_base, RL_MAX_SHARDS) == hipSuccess && dalloc(&s.woff, (size_t)n + 1) == hipSuccess &&
       dalloc(&s.wtsum, WIRE_SCAN_WORDS(n)) == hipSuccess;
  return ok;
}

void free_buffer(Scratch& s) {
  void* bufs[] = {s.rec, s.res, s.big_meta, s.big_n, s.big_work, s.work_n, s.sorted_n, s.big_cnt, s.keys[0], s.keys[1],
                  s.vals[0], s.vals[1], s.grp, s.lead, s.gmask, s.defer, s.defer_n, s.defer2, s.defer2_n, s.defer1,
                  s.defer1_n, s.fast_blk, s.hits_s, s.segsum, s.rid, s.run_start, s.run_flags, s.run_state, s.run_alias,
                  s.run_f, s.runs64, s.split, s.drun, s.run_end, s.part_info, s.hit_a, s.tile, s.hit_t, s.r_base,
                  s.uniq, s.uniq_n, s.long_runs, s.kt_blk, s.log_epoch, s.woff, s.wtsum};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
}

// Copy a host batch into the staging buffers; returns the device view.
int stage(Engine* c, const rl_batch* in, BatchDev* out) {
  const uint32_t n = in->n, nq = in->n_requests;
  const uint64_t nb = n ? in->stem_off[n] : 0;
  int rc = check_sizes(c, in, nb);
  if (rc) return rc;
  hipStream_t st = c->stream;
  HIPCHK(c, after_batches(c, st));  // staging may still feed a routed batch
  if (nb) HIPCHK(c, hipMemcpyAsync(c->d_stem, in->stem_bytes, nb, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->d_off, in->stem_off, (n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  if (nq) HIPCHK(c, hipMemcpyAsync(c->d_now, in->now, nq * sizeof(int64_t), hipMemcpyHostToDevice, st));
  if (n) {
    HIPCHK(c, hipMemcpyAsync(c->d_req, in->req_idx, n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->d_unit, in->unit, n, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->d_flags, in->flags, n, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->d_limit, in->limit, n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->d_hits, in->hits, n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->d_rule, in->rule_id, n * 4, hipMemcpyHostToDevice, st));
  }
  rl_batch d = *in;
  d.stem_bytes = c->d_stem;
  d.stem_off = c->d_off;
  d.now = c->d_now;
  d.req_idx = c->d_req;
  d.unit = c->d_unit;
  d.flags = c->d_flags;
  d.limit = c->d_limit;
  d.hits = c->d_hits;
  d.rule_id = c->d_rule;
  *out = dev_view(c, &d, c->cfg.max_stem_bytes);
  return RL_OK;
}

}  // namespace

namespace rl {

const char* eng_last_error(const Engine* c) { return c ? c->last_error.c_str() : g_err.c_str(); }

hipError_t rl_stream_create(hipStream_t* st, uint32_t role) {
  static const uint32_t dedicated =
      getenv("RL_DEDICATED_QUEUES") ? (uint32_t)strtoul(getenv("RL_DEDICATED_QUEUES"), nullptr, 0) : 0u;
  if (!(dedicated & role)) return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  std::vector<uint32_t> mask(((uint32_t)cus + 31) / 32, 0xFFFFFFFFu);
  return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data());
}

Engine* eng_create(const rl_config* cfg_in, char* err, size_t errlen) {
  auto fail = [&](const std::string& m, Engine* c) -> Engine* {
    if (err && errlen) snprintf(err, errlen, "%s", m.c_str());
    g_err = m;
    if (c) eng_destroy(c);
    return nullptr;
  };
  if (!cfg_in) return fail("gpu: null config", nullptr);
  rl_config cfg = *cfg_in;
  if (!cfg.table_slots) cfg.table_slots = 1ull << 24;
  if (cfg.table_slots & (cfg.table_slots - 1)) return fail("gpu: table_slots must be a power of two", nullptr);
  if (!cfg.arena_bytes) cfg.arena_bytes = 64ull << 20;
  if (!cfg.history_entries) cfg.history_entries = cfg.table_slots;
  if (cfg.history_entries > (uint64_t)LOG_PARTS * LOG_PART_MAX)
    return fail("gpu: history_entries must be at most 2^31", nullptr);
  if (cfg.expiration_jitter_max_seconds < 0) return fail("gpu: expiration_jitter_max_seconds must be >= 0", nullptr);
  if (!cfg.max_batch) cfg.max_batch = 1u << 20;
  if (cfg.max_batch > MAX_PART_TILES * PART_TILE)
    return fail("gpu: max_batch must be at most 8388608 descriptors", nullptr);
  if (!cfg.max_requests) cfg.max_requests = cfg.max_batch;
  if (!cfg.max_rules) cfg.max_rules = 65536;
  if (!cfg.max_stem_bytes) cfg.max_stem_bytes = 128u * cfg.max_batch;
  if (hipSetDevice(cfg.device) != hipSuccess) return fail("gpu: hipSetDevice failed", nullptr);

  Engine* c = new Engine();
  c->cfg = cfg;
  c->hash_seed = cfg.hash_seed;
  while (!c->hash_seed) {  // a secret per-ctx key unless the caller shares one (multi-shard tables)
    std::random_device rd;
    c->hash_seed = ((uint64_t)rd() << 32) ^ rd();
  }
  c->cfg.hash_seed = c->hash_seed;
  c->hk = hash_key_of(c->hash_seed, cfg.debug_hash_bits);
  c->nslots = cfg.table_slots;
  {
    // per partition a power of two, and at least 1/16 of a batch. A batch's
    // appends are spread over the partitions by workgroup and wave, but a
    // skewed one (a hot key replayed serially, the exact path's 8 workgroups)
    // can send more than that to one partition: log_append then refuses the
    // excess (rl_table_info.history_refused; those windows' later lookups are
    // RL_E_TIME) rather than wrap onto entries of the same batch
    const uint64_t want = std::max<uint64_t>(cfg.history_entries / LOG_PARTS, std::max<uint64_t>(cfg.max_batch / 16, 1024));
    uint64_t cap = 1;
    while (cap * 2 <= want && cap * 2 <= LOG_PART_MAX) cap *= 2;
    if (cap < want && cap < LOG_PART_MAX) cap *= 2;
    c->log_cap = (uint32_t)cap;
    c->cfg.history_entries = (uint64_t)LOG_PARTS * cap;
    c->horizon = (uint32_t)std::min<int64_t>(cfg.expiration_jitter_max_seconds, 1ll << 30);
  }
  c->arena_cap16 = cfg.arena_bytes / 16;
  const uint32_t n = cfg.max_batch;
  bool ok = true;
  for (uint32_t k = 0; k < NBUF; k++) ok = ok && rl_stream_create(&c->pipe[k], SR_PIPE) == hipSuccess;
  if (const char* be = getenv("RL_B_BEGIN_EARLY")) c->b_early = atoi(be) != 0;  // (A/B knob)
  c->stream = c->pipe[0];
  for (uint32_t k = 0; k < NBUF; k++)
    ok = ok && hipEventCreateWithFlags(&c->b_done[k], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->b_table[k], hipEventDisableTiming) == hipSuccess;
  for (uint32_t k = 0; k < PROGRESS_RING; k++)
    ok = ok && hipEventCreateWithFlags(&c->done_ring[k], hipEventDisableTiming) == hipSuccess;
  ok = ok && dalloc(&c->slots, c->nslots) == hipSuccess &&
       dalloc(&c->log, (size_t)LOG_PARTS * c->log_cap) == hipSuccess &&
       dalloc(&c->log_ctr, (size_t)(LOG_PARTS + 1) * LOG_CTR_STRIDE) == hipSuccess;
  ok = ok && dalloc(&c->arena, cfg.arena_bytes) == hipSuccess && dalloc(&c->arena2, cfg.arena_bytes) == hipSuccess;
  for (uint32_t k = 0; k < NBUF; k++) ok = ok && alloc_buffer(c->s[k], n);
  Scratch& s0 = c->s[0];
  ok = ok && dalloc(&c->errw, ERRW_WORDS) == hipSuccess;
  for (uint32_t k = 0; k < NBUF; k++)
    ok = ok && hipEventCreateWithFlags(&c->consumed[k], hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&c->route_ready, hipEventDisableTiming) == hipSuccess &&
       hipEventCreateWithFlags(&c->caller_ready, hipEventDisableTiming) == hipSuccess;
  c->serial_debug = getenv("RL_DEBUG_SERIAL") != nullptr;
  c->copy_time = getenv("RL_DEBUG_COPYTIME") != nullptr;
  c->host_time = getenv("RL_DEBUG_HOSTTIME") != nullptr;
  for (uint32_t k = 0; c->copy_time && k < 64; k++)
    ok = ok && hipEventCreate(&c->ct_ev[0][k]) == hipSuccess && hipEventCreate(&c->ct_ev[1][k]) == hipSuccess &&
         hipEventCreate(&c->ct_ev[2][k]) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_base, (size_t)NBUF * RL_MAX_SHARDS * 8) == hipSuccess;
  for (uint32_t k = 0; k < NBUF; k++)  // per buffer: a batch's k_finish overlaps the next batch's table kernels
    ok = ok && dalloc(&c->s[k].stripes, (size_t)STAT_STRIPES * STAT_LDS_RULES * RL_NUM_STATS) == hipSuccess;
  ok = ok && dalloc(&s0.time_floor, 1) == hipSuccess;
  ok = ok && dalloc(&s0.counters, 8) == hipSuccess;
  for (uint32_t k = 0; k < NBUF; k++) {  // shared members
    Scratch& sk = c->s[k];
    sk.err = c->errw ? c->errw + k : nullptr;
    sk.errb = c->errw ? c->errw + ERRW_B0 + k : nullptr;
    sk.errs = c->errw ? c->errw + NBUF + 1 : nullptr;
    sk.time_floor = s0.time_floor;
    sk.counters = s0.counters;
  }
  ok = ok && dalloc(&c->d_stem, (size_t)cfg.max_stem_bytes + 64) == hipSuccess;
  ok = ok && dalloc(&c->d_off, (size_t)n + 1) == hipSuccess;
  ok = ok && dalloc(&c->d_now, cfg.max_requests) == hipSuccess;
  ok = ok && dalloc(&c->d_req, n) == hipSuccess && dalloc(&c->d_unit, n) == hipSuccess &&
       dalloc(&c->d_flags, n) == hipSuccess && dalloc(&c->d_limit, n) == hipSuccess &&
       dalloc(&c->d_hits, n) == hipSuccess && dalloc(&c->d_rule, n) == hipSuccess;
  ok = ok && dalloc(&c->d_code, n) == hipSuccess && dalloc(&c->d_status, n) == hipSuccess &&
       dalloc(&c->d_rem, n) == hipSuccess &&
       dalloc(&c->d_reset, n) == hipSuccess;
  ok = ok && dalloc(&c->d_stats, (size_t)cfg.max_rules * RL_NUM_STATS) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_err, ERRW_WORDS * sizeof(uint32_t)) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_counters, 8 * sizeof(unsigned long long)) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_long, NBUF * sizeof(uint32_t)) == hipSuccess;
  if (ok) memset(c->h_long, 0, NBUF * sizeof(uint32_t));
  if (const char* sl = getenv("RL_SPLIT_LONG")) c->long_mode = atoi(sl);  // (A/B knob)
  ok = ok && hipHostMalloc((void**)&c->h_big, NBUF * sizeof(uint32_t)) == hipSuccess;
  if (ok) memset(c->h_big, 0, NBUF * sizeof(uint32_t));
  if (const char* bc = getenv("RL_BIG_CUE")) c->big_mode = atoi(bc);  // (A/B knob)
  ok = ok && hipHostMalloc((void**)&c->h_late, NBUF * sizeof(uint32_t)) == hipSuccess;
  if (ok) memset(c->h_late, 0, NBUF * sizeof(uint32_t));
  if (const char* lc = getenv("RL_LATE_CUE")) c->late_mode = atoi(lc);  // (A/B knob)
  if (!ok) return fail("gpu: device allocation failed (table_slots/arena/max_batch too large?)", c);
  ok = hipMemsetAsync(c->slots, 0, c->nslots * sizeof(Slot), c->stream) == hipSuccess &&
       hipMemsetAsync(c->log_ctr, 0, (size_t)(LOG_PARTS + 1) * LOG_CTR_STRIDE * 8, c->stream) == hipSuccess &&
       // (entries are written before any chain points at them)
       hipMemsetAsync(c->errw, 0, ERRW_WORDS * 4, c->stream) == hipSuccess &&
       hipMemsetAsync(s0.time_floor, 0, 8, c->stream) == hipSuccess &&
       hipMemsetAsync(s0.counters, 0, 64, c->stream) == hipSuccess &&
       hipMemsetAsync(c->s[0].stripes, 0, (size_t)STAT_STRIPES * STAT_LDS_RULES * RL_NUM_STATS * 8, c->stream) ==
           hipSuccess &&
       hipMemsetAsync(c->d_stem, 0, (size_t)cfg.max_stem_bytes + 64, c->stream) == hipSuccess &&
       hipStreamSynchronize(c->stream) == hipSuccess;
  for (uint32_t k = 0; k < NBUF; k++)
    ok = ok && hipEventRecord(c->b_done[k], c->stream) == hipSuccess &&
         hipEventRecord(c->b_table[k], c->stream) == hipSuccess &&
         (k == 0 || hipMemsetAsync(c->s[k].stripes, 0, (size_t)STAT_STRIPES * STAT_LDS_RULES * RL_NUM_STATS * 8,
                                   c->stream) == hipSuccess) &&
         hipEventRecord(c->consumed[k], c->stream) == hipSuccess;
  if (!ok) return fail("gpu: device initialisation failed", c);
  return c;
}

void free_host_slots(Engine* c) {
  for (HostSlot& h : c->hs) {
    void* bufs[] = {h.stem, h.off, h.req, h.limit, h.hits, h.rule, h.now, h.unit, h.flags, h.code, h.status, h.rem,
                    h.reset, h.stats, h.cbuf};
    for (void* p : bufs)
      if (p) (void)hipFree(p);
    if (h.in_done) (void)hipEventDestroy(h.in_done);
    if (h.out_done) (void)hipEventDestroy(h.out_done);
    h = HostSlot{};
  }
  for (hipStream_t st : {c->h2d, c->d2h})
    if (st) (void)hipStreamDestroy(st);
  c->h2d = c->d2h = nullptr;
  c->hs_ready = false;
}

void copy_time_fold(Engine* c, bool all);

void eng_destroy(Engine* c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  if (c->host_time && c->ht_n)
    fprintf(stderr, "RL_DEBUG_HOSTTIME: %llu batches, ms each: check %.4f copy %.4f unpack %.4f enqueue %.4f to_host %.4f "
            "track %.4f\n", (unsigned long long)c->ht_n, c->ht[0] / c->ht_n * 1e3, c->ht[1] / c->ht_n * 1e3,
            c->ht[2] / c->ht_n * 1e3, c->ht[3] / c->ht_n * 1e3, c->ht[4] / c->ht_n * 1e3, c->ht[5] / c->ht_n * 1e3);
  if (c->copy_time) {
    (void)hipDeviceSynchronize();
    copy_time_fold(c, true);
    if (c->ct_count)
      fprintf(stderr, "RL_DEBUG_COPYTIME: %llu input copies, %.4f ms each, slot wait %.4f ms, gap after the previous "
              "copy %.4f ms\n", (unsigned long long)c->ct_count, c->ct_ms / c->ct_count, c->ct_wait_ms / c->ct_count,
              c->ct_gap_ms / c->ct_count);
    for (uint32_t k = 0; k < 64; k++)
      for (int j = 0; j < 3; j++)
        if (c->ct_ev[j][k]) (void)hipEventDestroy(c->ct_ev[j][k]);
  }
  if (c->hs_ready) {
    (void)hipDeviceSynchronize();
    free_host_slots(c);
  }
  for (uint32_t k = 0; k < NBUF; k++)
    if (c->pipe[k]) (void)hipStreamSynchronize(c->pipe[k]);
  for (uint32_t k = 0; k < PROF_RING; k++)
    for (int i = 0; i <= RL_NUM_STAGES; i++)
      if (c->ev[k][i]) (void)hipEventDestroy(c->ev[k][i]);
  if (c->d_kt_acc) (void)hipFree(c->d_kt_acc);
  for (uint32_t k = 0; k < NBUF; k++) {
    free_buffer(c->s[k]);
    if (c->b_done[k]) (void)hipEventDestroy(c->b_done[k]);
    if (c->b_table[k]) (void)hipEventDestroy(c->b_table[k]);
    if (c->consumed[k]) (void)hipEventDestroy(c->consumed[k]);
  }
  for (uint32_t k = 0; k < PROGRESS_RING; k++)
    if (c->done_ring[k]) (void)hipEventDestroy(c->done_ring[k]);
  if (c->rs_ready) {
    c->rs.err = nullptr;  // (a word of errw)
    scratch_free(c->rs);
  }
  if (c->route_ready) (void)hipEventDestroy(c->route_ready);
  if (c->caller_ready) (void)hipEventDestroy(c->caller_ready);
  if (c->h_base) (void)hipHostFree(c->h_base);
  const Scratch& s0 = c->s[0];
  void* bufs[] = {c->slots, c->log, c->log_ctr, c->tear, c->arena, c->arena2, c->errw, s0.stripes, s0.time_floor, s0.counters, c->d_stem, c->d_off,
                  c->d_now, c->d_req, c->d_unit, c->d_flags, c->d_limit, c->d_hits, c->d_rule, c->d_code, c->d_status,
                  c->d_rem,
                  c->d_reset, c->d_stats};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  for (uint32_t k = 1; k < NBUF; k++)
    if (c->s[k].stripes) (void)hipFree(c->s[k].stripes);
  if (c->h_err) (void)hipHostFree(c->h_err);
  if (c->h_counters) (void)hipHostFree(c->h_counters);
  if (c->h_long) (void)hipHostFree(c->h_long);
  if (c->h_big) (void)hipHostFree(c->h_big);
  if (c->h_late) (void)hipHostFree(c->h_late);
  for (void* p : {(void*)c->cfg_blob, (void*)c->mbuf})
    if (p) (void)hipFree(p);
  if (c->h_match) (void)hipHostFree(c->h_match);
  for (uint32_t k = 0; k < NBUF; k++)
    if (c->pipe[k]) (void)hipStreamDestroy(c->pipe[k]);
  delete c;
}

int eng_do_limit_async(Engine* c, const rl_batch* in, rl_result* out, void* stream) {
  if (!c || !in || !out) return set_err(c, RL_E_INVALID, "gpu: null argument");
  // device pointers: the total stem size is only known on the device; the
  // kernels bound-check offsets against max_stem_bytes (stem_cap)
  int rc = check_sizes(c, in, 0);
  if (rc) return rc;
  if ((uintptr_t)in->stem_bytes & 3u) return set_err(c, RL_E_INVALID, "gpu: stem_bytes must be 4-byte aligned");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  BatchDev b = dev_view(c, in, c->cfg.max_stem_bytes);
  OutDev o{out->code, out->limit_remaining, out->reset_s, (unsigned long long*)out->stats, out->status};
  // Pipelined on the ctx streams. With a caller stream, after the work already
  // on it (the inputs' producer); NULL: the caller completes the inputs first.
  // Either way *out is read after rl_synchronize: ordering the caller's stream
  // after each batch would chain the next batch's inputs behind this batch's
  // stage B and serialise the pipeline. RL_DEBUG_SERIAL: every stage on the
  // caller's stream, one batch at a time (isolated kernel timings).
  hipStream_t st = (hipStream_t)stream;
  if (st && c->serial_debug) {
    enqueue(c, b, o, 0, st, false);
    HIPCHK(c, track(c, st));
  } else {
    // (an idle caller stream needs no event: a cross-stream wait can stall
    // behind whatever shares the caller's hardware queue)
    if (st && hipStreamQuery(st) == hipErrorNotReady) {
      HIPCHK(c, hipEventRecord(c->caller_ready, st));
      HIPCHK(c, hipStreamWaitEvent(c->pipe[c->next], c->caller_ready, 0));
    }
    const uint32_t k = enqueue(c, b, o, 0, nullptr, true);
    HIPCHK(c, track(c, c->pipe[k]));
  }
  HIPCHK(c, hipGetLastError());
  c->batches++;
  c->decisions += in->n;
  return RL_OK;
}

bool scratch_alloc(Scratch& s, uint32_t n) {
  s = Scratch{};
  bool ok = alloc_buffer(s, n);
  ok = ok && dalloc(&s.err, 1) == hipSuccess && dalloc(&s.route_start, 2 * RL_MAX_SHARDS + 1) == hipSuccess &&
       dalloc(&s.route_dest, n) == hipSuccess && dalloc(&s.route_hash, n) == hipSuccess &&
       dalloc(&s.route_hist, 2ull * RL_MAX_SHARDS * ((n + ROUTE_TILE - 1) / ROUTE_TILE)) == hipSuccess;
  ok = ok && hipMemset(s.err, 0, 4) == hipSuccess;
  return ok;
}

void scratch_free(Scratch& s) {
  free_buffer(s);
  for (void* p : {(void*)s.err, (void*)s.route_start, (void*)s.route_dest, (void*)s.route_hash, (void*)s.route_hist})
    if (p) (void)hipFree(p);
  s = Scratch{};
}

// The routing partition runs on its own scratch (c->rs), so it never waits
// for, or disturbs, the pipeline buffers; its validation word is the ctx's
// errw[NBUF + 2] (reported at rl_synchronize). counts = device memory.
int eng_route_pack(Engine* c, const rl_batch* in, uint32_t n_shards, uint32_t src_rank, void* send_rec,
                   uint8_t* send_stem, uint32_t* perm, uint64_t* counts, void* stream, uint32_t cstride,
                   uint64_t meta0, uint64_t meta1, uint32_t own_rank, unsigned long long* hash_out,
                   unsigned long long* counts_host, const RouteBufs* bufs) {
  if (!c || !in || !counts || (in->n && (!send_rec || !send_stem || !perm)))
    return set_err(c, RL_E_INVALID, "gpu: null argument");
  if (n_shards < 1 || n_shards > RL_MAX_SHARDS || src_rank >= n_shards)
    return set_err(c, RL_E_INVALID, "gpu: n_shards must be 1..256 and src_rank < n_shards");
  int rc = check_sizes(c, in, 0);
  if (rc) return rc;
  if ((uintptr_t)in->stem_bytes & 3u) return set_err(c, RL_E_INVALID, "gpu: stem_bytes must be 4-byte aligned");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (!c->rs_ready) {
    HIPCHK(c, after_batches(c, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!scratch_alloc(c->rs, c->cfg.max_batch)) {
      scratch_free(c->rs);
      return set_err(c, RL_E_HIP, "gpu: routing scratch allocation failed");
    }
    (void)hipFree(c->rs.err);
    c->rs.err = c->errw + NBUF + 2;
    c->rs_ready = true;
  }
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  BatchDev b = dev_view(c, in, c->cfg.max_stem_bytes);
  Scratch rs = c->rs;
  if (bufs) {
    rs.route_dest = bufs->dest;
    rs.route_hist = bufs->hist;
    rs.route_start = bufs->start;
  }
  launch_route_pack(b, n_shards, src_rank, (Wire*)send_rec, send_stem, perm, (unsigned long long*)counts, rs, st,
                    cstride, meta0, meta1, own_rank, hash_out, counts_host);
  HIPCHK(c, hipGetLastError());
  return RL_OK;
}

int eng_route_owner(Engine* c, uint32_t n, const Wire* recv_rec, const uint8_t* recv_stem, uint64_t recv_stem_bytes,
                    const uint64_t* src_stem_base, uint32_t n_src, uint32_t n_rules, uint32_t rule_stride,
                    unsigned long long* stats, int isolate, hipEvent_t ready, uint32_t* slot,
                    const OwnChunk* own, const uint32_t* woff, const unsigned long long* wbad) {
  const uint32_t rules_eff = rule_stride ? n_src * rule_stride : n_rules;
  const bool has_own = own && own->n;
  // (recv_stem may be null with no received stem bytes: an own chunk alone)
  if (!c || !src_stem_base || (n && (!recv_rec || (!recv_stem && recv_stem_bytes))) || (rules_eff && !stats))
    return set_err(c, RL_E_INVALID, "gpu: null argument");
  if (n && !recv_stem && !(has_own && own->n == n)) return set_err(c, RL_E_INVALID, "gpu: null argument");
  if (has_own && ((uint64_t)own->lo + own->n > n || own->rank >= n_src || !own->idx || !own->hash || !own->stem ||
                  ((uintptr_t)own->stem & 3u)))
    return set_err(c, RL_E_INVALID, "gpu: bad own chunk");
  if (n_src < 1 || n_src > RL_MAX_SHARDS) return set_err(c, RL_E_INVALID, "gpu: n_shards must be 1..256");
  if (rule_stride && n_rules > rule_stride) return set_err(c, RL_E_INVALID, "gpu: n_rules exceeds the rule stride");
  // (the received stems are the caller's buffer: only 32-bit offsets bound them)
  if (n > c->cfg.max_batch || rules_eff > c->cfg.max_rules || recv_stem_bytes >= (1ull << 32))
    return set_err(c, RL_E_CAPACITY, "gpu: routed batch exceeds max_batch/max_rules or 4 GiB of stems");
  if ((uintptr_t)recv_stem & 3u) return set_err(c, RL_E_INVALID, "gpu: recv_stem must be 4-byte aligned");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  // the buffer this batch will take (enqueue advances c->next the same way)
  const uint32_t k = c->next;
  Scratch& sk = c->s[k];
  hipStream_t a = c->pipe[k];
  HIPCHK(c, hipStreamWaitEvent(a, c->b_done[k], 0));
  HIPCHK(c, hipStreamWaitEvent(a, c->consumed[k], 0));
  if (ready) HIPCHK(c, hipStreamWaitEvent(a, ready, 0));
  if (!(has_own && own->n == n)) {  // (an own chunk alone reads no received stems: no bases)
    unsigned long long* hb = c->h_base + (size_t)k * RL_MAX_SHARDS;
    HIPCHK(c, hipEventSynchronize(c->b_done[k]));  // (the pinned bases of buffer k's previous batch were read)
    for (uint32_t j = 0; j < n_src; j++) hb[j] = src_stem_base[j];
    HIPCHK(c, hipMemcpyAsync(sk.r_base, hb, (size_t)n_src * 8, hipMemcpyHostToDevice, a));
    if (!woff) {  // (the records' stem offsets: the lengths scanned here, unless the caller did it for every part)
      launch_wire_offsets(recv_rec, n, has_own ? own->lo : 0u, has_own ? own->lo + own->n : 0u, sk.r_base, n_src,
                          recv_stem_bytes, sk.woff, sk.wtsum, a);
      woff = sk.woff;
      wbad = sk.wtsum + WIRE_SCAN_TILES(n);
    }
  }
  // k_prepare reads the wire records in place (a malformed exchange fails
  // the batch's validation word)
  BatchDev b{};
  b.hk = c->hk;
  b.n = n;
  b.n_req = n;
  b.n_rules = rules_eff;
  b.stem_cap = (uint32_t)recv_stem_bytes;
  b.stem_total = (uint32_t)recv_stem_bytes;
  b.now_desc = 1;
  b.stem = recv_stem;
  b.wire = recv_rec;
  b.woff = woff;
  b.wbad = wbad;
  b.wbase = sk.r_base;
  b.n_src = n_src;
  b.rule_stride = rule_stride;
  if (has_own) b.own = *own;
  OutDev o{nullptr, nullptr, nullptr, stats, isolate ? c->d_status : nullptr};
  const uint32_t kk = enqueue(c, b, o, 0, nullptr, true);
  HIPCHK(c, hipGetLastError());
  c->batches++;
  c->decisions += n;
  *slot = kk;
  return RL_OK;
}

// The per-rank owner step of the multi-process exchange (sharded.py): the
// pipelined owner batch, then on `stream` its packed results copied to ret.
int eng_route_do_limit(Engine* c, uint32_t n, const void* recv_rec, const uint8_t* recv_stem, uint64_t recv_stem_bytes,
                       const uint64_t* src_stem_base, uint32_t n_shards, uint32_t n_rules, uint32_t rule_stride,
                       uint64_t* ret, uint64_t* stats, int isolate, void* stream) {
  if (!c || (n && !ret)) return set_err(c, RL_E_INVALID, "gpu: null argument");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  HIPCHK(c, hipEventRecord(c->route_ready, st));  // the received buffers are ordered on the caller's stream
  uint32_t k = 0;
  const int rc = eng_route_owner(c, n, (const Wire*)recv_rec, recv_stem, recv_stem_bytes, src_stem_base, n_shards,
                                 n_rules, rule_stride, (unsigned long long*)stats, isolate, c->route_ready, &k);
  if (rc) return rc;
  HIPCHK(c, hipStreamWaitEvent(st, c->b_done[k], 0));
  if (n) HIPCHK(c, hipMemcpyAsync(ret, c->s[k].res, (size_t)n * 8, hipMemcpyDeviceToDevice, st));
  HIPCHK(c, hipEventRecord(c->consumed[k], st));
  return RL_OK;
}

int eng_fail(Engine* c, int code, const std::string& msg) { return set_err(c, code, msg); }

int eng_route_scatter(Engine* c, uint32_t n, const uint32_t* perm, const uint64_t* ret, rl_result* out, void* stream) {
  if (!c || !out || (n && (!perm || !ret))) return set_err(c, RL_E_INVALID, "gpu: null argument");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  OutDev o{out->code, out->limit_remaining, out->reset_s, (unsigned long long*)out->stats, out->status};
  launch_route_scatter(perm, (const unsigned long long*)ret, n, o, st);
  HIPCHK(c, hipGetLastError());
  return RL_OK;
}

int eng_profile(Engine* c, int enable) {
  if (!c) return set_err(c, RL_E_INVALID, "gpu: null ctx");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (enable && !c->ev[0][0]) {
    for (uint32_t k = 0; k < PROF_RING; k++)
      for (int i = 0; i <= RL_NUM_STAGES; i++) HIPCHK(c, hipEventCreate(&c->ev[k][i]));
    HIPCHK(c, dalloc(&c->d_kt_acc, 2));
    HIPCHK(c, hipMemset(c->d_kt_acc, 0, 2 * sizeof(unsigned long long)));
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->cfg.device) == hipSuccess) c->wclk_khz = khz;
  }
  prof_fold_all(c);
  c->prof = enable > 0;
  c->prof_every = enable > 0 ? (uint32_t)enable : 1u;
  // (the first sampled batch is the k-th: a timed region's first batch, whose
  // stage A runs with nothing beside it, is not one of them)
  c->prof_skip = c->prof_every - 1;
  return RL_OK;
}

int eng_profile_read(Engine* c, double* ms, uint32_t n, uint64_t* batches) {
  if (!c) return set_err(c, RL_E_INVALID, "gpu: null ctx");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  prof_fold_all(c);
  for (uint32_t i = 0; i < n && i < RL_NUM_STAGES; i++) ms[i] = c->stage_ms[i];
  if (n > RL_NUM_STAGES) {
    ms[RL_NUM_STAGES] = 0;
    if (c->d_kt_acc) {  // every batch since the last read: their k_finish kernels are done
      unsigned long long acc[2] = {0, 0};
      HIPCHK(c, after_batches(c, c->stream));
      HIPCHK(c, hipMemcpyAsync(acc, c->d_kt_acc, sizeof(acc), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipMemsetAsync(c->d_kt_acc, 0, sizeof(acc), c->stream));
      if (acc[1] && c->wclk_khz > 0) ms[RL_NUM_STAGES] = (double)acc[0] / (double)acc[1] / c->wclk_khz;
    }
  }
  if (batches) *batches = c->prof_batches;
  for (int i = 0; i < RL_NUM_STAGES; i++) c->stage_ms[i] = 0;
  c->prof_batches = 0;
  return RL_OK;
}

// RL_DEBUG_COPYTIME: fold the timed copies (all when `all`, else the ring's
// oldest pair when it is about to be reused).
void copy_time_fold(Engine* c, bool all) {
  const uint32_t lo = c->ct_n > 64 ? c->ct_n - 64 : 0;
  for (uint32_t k = all ? lo : c->ct_n - (c->ct_n >= 64 ? 64 : c->ct_n); k < c->ct_n; k++) {
    if (!all && k + 64 != c->ct_n) continue;
    float ms = 0;
    if (hipEventSynchronize(c->ct_ev[1][k % 64]) == hipSuccess &&
        hipEventElapsedTime(&ms, c->ct_ev[0][k % 64], c->ct_ev[1][k % 64]) == hipSuccess) {
      c->ct_ms += ms;
      c->ct_count++;
      float w = 0, g = 0;
      if (hipEventElapsedTime(&w, c->ct_ev[2][k % 64], c->ct_ev[0][k % 64]) == hipSuccess) c->ct_wait_ms += w;
      if (k > lo && hipEventElapsedTime(&g, c->ct_ev[1][(k - 1) % 64], c->ct_ev[0][k % 64]) == hipSuccess)
        c->ct_gap_ms += g;
    }
  }
  if (all) c->ct_n = 0;
}

int eng_synchronize(Engine* c) {
  if (!c) return set_err(c, RL_E_INVALID, "gpu: null ctx");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, hipDeviceSynchronize());
  if (c->copy_time) copy_time_fold(c, true);
  c->seq_done = c->seq_sub;
  return collect(c);
}

int eng_batch_progress(Engine* c, uint64_t* submitted, uint64_t* completed) {
  if (!c || !submitted || !completed) return set_err(c, RL_E_INVALID, "gpu: null argument");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  while (c->seq_done < c->seq_sub) {
    const hipError_t e = hipEventQuery(c->done_ring[c->seq_done % PROGRESS_RING]);
    if (e == hipErrorNotReady) break;
    if (e != hipSuccess) return set_err(c, RL_E_HIP, std::string("gpu: hipEventQuery: ") + hipGetErrorString(e));
    c->seq_done++;
  }
  *submitted = c->seq_sub;
  *completed = c->seq_done;
  return RL_OK;
}

// Host buffers in and out, nothing waited for: the inputs cross PCIe on the
// h2d stream into a staging slot, the batch is pipelined on the ctx streams
// once they have landed, its outputs cross back on the d2h stream; the caller
// reads *out after rl_synchronize. Pinned host buffers (rl_alloc_host) make
// the copies truly asynchronous; the host buffers of a batch must stay
// untouched until then.
// The NBUF host-fed staging slots and their copy streams (first use).
int ensure_host_slots(Engine* c) {
  if (!c->hs_ready) {
    const rl_config& g = c->cfg;
    bool ok = rl_stream_create(&c->h2d, SR_HOSTCOPY) == hipSuccess && rl_stream_create(&c->d2h, SR_HOSTCOPY) == hipSuccess;
    for (HostSlot& h : c->hs) {
      ok = ok && dalloc(&h.stem, (size_t)g.max_stem_bytes + 64) == hipSuccess &&
           dalloc(&h.off, (size_t)g.max_batch + 1) == hipSuccess && dalloc(&h.req, g.max_batch) == hipSuccess &&
           dalloc(&h.limit, g.max_batch) == hipSuccess && dalloc(&h.hits, g.max_batch) == hipSuccess &&
           dalloc(&h.rule, g.max_batch) == hipSuccess && dalloc(&h.now, g.max_requests) == hipSuccess &&
           dalloc(&h.unit, g.max_batch) == hipSuccess && dalloc(&h.flags, g.max_batch) == hipSuccess &&
           dalloc(&h.code, g.max_batch) == hipSuccess && dalloc(&h.status, g.max_batch) == hipSuccess &&
           dalloc(&h.rem, g.max_batch) == hipSuccess && dalloc(&h.reset, g.max_batch) == hipSuccess &&
           dalloc(&h.stats, (size_t)g.max_rules * RL_NUM_STATS) == hipSuccess &&
           hipEventCreateWithFlags(&h.in_done, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&h.out_done, hipEventDisableTiming) == hipSuccess &&
           hipEventRecord(h.out_done, c->d2h) == hipSuccess;
    }
    if (!ok) {
      free_host_slots(c);
      return set_err(c, RL_E_HIP, "gpu: host-fed staging allocation failed");
    }
    c->hs_ready = true;
  }
  return RL_OK;
}

// The streams of a host-fed batch. By default its input copy goes on the
// pipeline stream the batch will take (c->pipe[c->next]) and its outputs'
// copy back on the pipeline stream it took (k): a separate copy stream shares
// a hardware queue with one of the pipeline streams, and its copies and
// markers then wait behind that stream's later batches (the routed step's
// measured stall, CommRouter::one_stream). RL_HOSTFED_STREAMS=2: the h2d / d2h
// streams (A/B).
hipStream_t hostfed_stream(Engine* c, bool input, uint32_t k = 0) {
  static const bool own = getenv("RL_HOSTFED_STREAMS") && atoi(getenv("RL_HOSTFED_STREAMS")) == 2;
  if (own) return input ? c->h2d : c->d2h;
  return input ? c->pipe[c->next] : c->pipe[k];
}

// The copy stream's order after the slot's previous batch (its outputs
// drained). A cross-queue wait in front of an SDMA copy made hipMemcpyAsync
// block the submitting thread for ~0.3 ms on some boxes, and the link idled
// while the host caught up (0.1 ms between 0.58-ms copies): the host checks
// the event instead (RL_COPY_STREAM_WAIT=1: the stream wait, for A/B). The
// slot is four batches back, so the host rarely waits at all.
hipError_t slot_drained(Engine* c, HostSlot& h, hipStream_t up) {
  static const bool stream_wait = getenv("RL_COPY_STREAM_WAIT") != nullptr;
  if (stream_wait) return hipStreamWaitEvent(up, h.out_done, 0);
  const hipError_t q = hipEventQuery(h.out_done);
  if (q == hipSuccess) return hipSuccess;
  if (q != hipErrorNotReady) return q;
  (void)c;
  return hipEventSynchronize(h.out_done);
}

// Enqueue the staged batch d (device pointers; its inputs complete at
// h.in_done) and its outputs' copies back into *out on the d2h stream.
int host_slot_run(Engine* c, HostSlot& h, const rl_batch& d, uint64_t nb, rl_result* out) {
  const uint32_t n = d.n;
  BatchDev b = dev_view(c, &d, c->cfg.max_stem_bytes);
  b.stem_total = (uint32_t)nb;
  OutDev o{h.code, h.rem, h.reset, d.n_rules ? h.stats : nullptr, out->status ? h.status : nullptr};
  const double w0 = c->host_time ? wall_s() : 0;
  HIPCHK(c, hipStreamWaitEvent(c->pipe[c->next], h.in_done, 0));
  const uint32_t k = enqueue(c, b, o, 0, nullptr, true);
  hipStream_t down = hostfed_stream(c, false, k);
  if (down != c->pipe[k]) HIPCHK(c, hipStreamWaitEvent(down, c->b_done[k], 0));
  const double w1 = c->host_time ? wall_s() : 0;
  // (stores by a kernel into page-locked outputs: not queued behind the next
  // batch's input copy on the DMA engine, rl_kernels.h ToHost)
  ToHost th{};
  auto add = [&](void* dst, const void* src, uint64_t bytes) {
    th.dst[th.n] = (uint8_t*)dst;
    th.src[th.n] = (const uint8_t*)src;
    th.bytes[th.n++] = bytes;
  };
  if (n) {
    add(out->code, h.code, n);
    add(out->limit_remaining, h.rem, n * 4ull);
    if (out->reset_s) add(out->reset_s, h.reset, n * 4ull);
    if (out->status) add(out->status, h.status, n);
  }
  if (d.n_rules && out->stats) add(out->stats, h.stats, (size_t)d.n_rules * RL_NUM_STATS * 8);
  if (th.n) HIPCHK(c, copy_to_host(th, down));
  HIPCHK(c, hipEventRecord(h.out_done, down));
  const double w2 = c->host_time ? wall_s() : 0;
  HIPCHK(c, track(c, down));
  if (c->host_time) {
    const double w3 = wall_s();
    c->ht[3] += w1 - w0;
    c->ht[4] += w2 - w1;
    c->ht[5] += w3 - w2;
  }
  HIPCHK(c, hipGetLastError());
  c->batches++;
  c->decisions += n;
  return RL_OK;
}

int eng_do_limit_host_async(Engine* c, const rl_batch* in, rl_result* out) {
  if (!c || !in || !out) return set_err(c, RL_E_INVALID, "gpu: null argument");
  const uint32_t n = in->n, nq = in->n_requests;
  if (n && (!in->stem_off || !out->code || !out->limit_remaining))
    return set_err(c, RL_E_INVALID, "gpu: null argument");
  const uint64_t nb = n ? in->stem_off[n] : 0;
  int rc = check_sizes(c, in, nb);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if ((rc = ensure_host_slots(c))) return rc;
  const uint32_t j = c->hnext;
  c->hnext = (j + 1) % NBUF;
  HostSlot& h = c->hs[j];
  hipStream_t up = hostfed_stream(c, true);
  HIPCHK(c, slot_drained(c, h, up));  // the slot's previous batch is drained
  if (nb) HIPCHK(c, hipMemcpyAsync(h.stem, in->stem_bytes, nb, hipMemcpyHostToDevice, up));
  HIPCHK(c, hipMemcpyAsync(h.off, in->stem_off, (n + 1) * 4ull, hipMemcpyHostToDevice, up));
  if (nq) HIPCHK(c, hipMemcpyAsync(h.now, in->now, nq * 8ull, hipMemcpyHostToDevice, up));
  if (n) {
    HIPCHK(c, hipMemcpyAsync(h.req, in->req_idx, n * 4ull, hipMemcpyHostToDevice, up));
    HIPCHK(c, hipMemcpyAsync(h.unit, in->unit, n, hipMemcpyHostToDevice, up));
    HIPCHK(c, hipMemcpyAsync(h.flags, in->flags, n, hipMemcpyHostToDevice, up));
    HIPCHK(c, hipMemcpyAsync(h.limit, in->limit, n * 4ull, hipMemcpyHostToDevice, up));
    HIPCHK(c, hipMemcpyAsync(h.hits, in->hits, n * 4ull, hipMemcpyHostToDevice, up));
    HIPCHK(c, hipMemcpyAsync(h.rule, in->rule_id, n * 4ull, hipMemcpyHostToDevice, up));
  }
  HIPCHK(c, hipEventRecord(h.in_done, up));
  rl_batch d = *in;
  d.stem_bytes = h.stem;
  d.stem_off = h.off;
  d.now = h.now;
  d.req_idx = h.req;
  d.unit = h.unit;
  d.flags = h.flags;
  d.limit = h.limit;
  d.hits = h.hits;
  d.rule_id = h.rule;
  return host_slot_run(c, h, d, nb, out);
}

// A compact batch: its one buffer crosses PCIe in one copy into the slot's
// cbuf, k_unpack rebuilds the rl_batch arrays in the slot, then as above. Section
// bounds are checked here; contents (offsets, request ranges, limit indices)
// on the device, like rl_batch's.
// The compact batch's sizes and sections (every entry point taking one).
int eng_compact_check(Engine* c, const rl_batch_compact* in, const rl_result* out) {
  if (!c || !in || !out) return set_err(c, RL_E_INVALID, "gpu: null argument");
  const rl_config& g = c->cfg;
  const uint32_t n = in->n, nq = in->n_requests;
  if (n && (!in->buf || !out->code || !out->limit_remaining))
    return set_err(c, RL_E_INVALID, "gpu: null argument");
  if (n > g.max_batch || nq > g.max_requests || in->n_rules > g.max_rules || in->n_limits > 65536)
    return set_err(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_rules (or > 65536 limits)");
  if (n && !nq) return set_err(c, RL_E_INVALID, "gpu: descriptors without requests");
  const uint64_t B = in->buf_bytes;
  auto sect = [&](uint64_t off, uint64_t bytes) { return off % 4 == 0 && off <= B && bytes <= B - off; };
  if (!sect(in->stem_off, (n + 1) * 4ull) || !sect(in->limit_idx, n * 2ull) || !sect(in->req_first, (nq + 1) * 4ull) ||
      !sect(in->now, nq * 4ull) || !sect(in->hits, nq * 4ull) || !sect(in->limits, in->n_limits * 12ull) ||
      !sect(in->stem_bytes, 0))
    return set_err(c, RL_E_INVALID, "gpu: compact batch section outside buf or not 4-byte aligned");
  const uint64_t nb = n ? reinterpret_cast<const uint32_t*>(in->buf + in->stem_off)[n] : 0;
  if (nb > g.max_stem_bytes) return set_err(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_stem_bytes");
  if (!sect(in->stem_bytes, nb)) return set_err(c, RL_E_INVALID, "gpu: compact batch stems outside buf");
  return RL_OK;
}

int eng_do_limit_compact_async(Engine* c, const rl_batch_compact* in, rl_result* out) {
  int rc = eng_compact_check(c, in, out);
  if (rc) return rc;
  const rl_config& g = c->cfg;
  const uint32_t n = in->n, nq = in->n_requests;
  const uint64_t B = in->buf_bytes;
  const uint64_t nb = n ? reinterpret_cast<const uint32_t*>(in->buf + in->stem_off)[n] : 0;
  HIPCHK(c, hipSetDevice(g.device));
  rc = ensure_host_slots(c);
  if (rc) return rc;
  const uint32_t j = c->hnext;
  HostSlot& h = c->hs[j];
  if (B > h.cbuf_cap) {  // grows to the largest buffer seen (the slot's previous batch drained first)
    HIPCHK(c, hipEventSynchronize(h.out_done));
    if (h.cbuf) HIPCHK(c, hipFree(h.cbuf));
    h.cbuf = nullptr;
    h.cbuf_cap = 0;
    HIPCHK(c, dalloc(&h.cbuf, B + 64));
    h.cbuf_cap = B;
  }
  c->hnext = (j + 1) % NBUF;
  hipStream_t up = hostfed_stream(c, true);
  HIPCHK(c, slot_drained(c, h, up));  // the slot's previous batch is drained
  if (B) HIPCHK(c, hipMemcpyAsync(h.cbuf, in->buf, B, hipMemcpyHostToDevice, up));
  HIPCHK(c, hipEventRecord(h.in_done, up));
  // unpacked on the batch's pipeline stream, so the copy stream runs the
  // next batch's copy back to back (on the copy stream it left a ~35 us gap
  // per batch: the kernel and its launch)
  HIPCHK(c, hipStreamWaitEvent(c->pipe[c->next], h.in_done, 0));
  launch_unpack(*in, h.cbuf, h.req, h.unit, h.flags, h.limit, h.hits, h.rule, h.now, c->s[c->next].err,
                c->pipe[c->next]);
  rl_batch d{};
  d.n = n;
  d.n_requests = nq;
  d.n_rules = in->n_rules;
  d.stem_bytes = h.cbuf + in->stem_bytes;
  d.stem_off = reinterpret_cast<const uint32_t*>(h.cbuf + in->stem_off);
  d.now = h.now;
  d.req_idx = h.req;
  d.unit = h.unit;
  d.flags = h.flags;
  d.limit = h.limit;
  d.hits = h.hits;
  d.rule_id = h.rule;
  return host_slot_run(c, h, d, nb, out);
}

// A prefix-shared batch (rl_batch_prefixed): the host checks only what the
// copies and the unpack's bounds rely on — sections inside buf, the index's
// first entry zero and its last the totals; every tile's own entry is checked
// on the device against its sections before the tile is unpacked.
int eng_prefixed_check(Engine* c, const rl_batch_prefixed* in, const rl_result* out, uint32_t* tiles) {
  if (!c || !in || !out) return set_err(c, RL_E_INVALID, "gpu: null argument");
  const rl_config& g = c->cfg;
  const uint32_t n = in->n, nq = in->n_requests;
  if (n && (!in->buf || !out->code || !out->limit_remaining))
    return set_err(c, RL_E_INVALID, "gpu: null argument");
  if (n > g.max_batch || nq > g.max_requests || in->n_rules > g.max_rules || in->n_limits > 65536)
    return set_err(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_rules (or > 65536 limits)");
  if (n && !nq) return set_err(c, RL_E_INVALID, "gpu: descriptors without requests");
  const uint32_t T = (nq + RL_PREFIXED_TILE - 1) / RL_PREFIXED_TILE;
  *tiles = T;
  const uint64_t B = in->buf_bytes;
  auto sect = [&](uint64_t off, uint64_t bytes) { return off % 4 == 0 && off <= B && bytes <= B - off; };
  if (!in->buf && B) return set_err(c, RL_E_INVALID, "gpu: null argument");
  if (!sect(in->index, 16ull * (T + 1)) || !sect(in->req, nq * 4ull) || !sect(in->now, nq * 4ull) ||
      !sect(in->hits, nq * 4ull) || !sect(in->desc, n * 4ull) || !sect(in->limits, in->n_limits * 12ull))
    return set_err(c, RL_E_INVALID, "gpu: prefixed batch section outside buf or not 4-byte aligned");
  const uint32_t* ix = reinterpret_cast<const uint32_t*>(in->buf + in->index);
  const uint32_t* tot = ix + 4ull * T;
  if (ix[0] || ix[1] || ix[2] || ix[3] || tot[0] != n)
    return set_err(c, RL_E_INVALID, "gpu: prefixed batch index does not start at zero or end at n");
  if (tot[3] > g.max_stem_bytes) return set_err(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_stem_bytes");
  if (!sect(in->prefix_bytes, tot[1]) || !sect(in->suffix_bytes, tot[2]))
    return set_err(c, RL_E_INVALID, "gpu: prefixed batch prefix or suffix bytes outside buf");
  return RL_OK;
}

int eng_do_limit_prefixed_async(Engine* c, const rl_batch_prefixed* in, rl_result* out) {
  uint32_t T = 0;
  const double w0 = c && c->host_time ? wall_s() : 0;
  int rc = eng_prefixed_check(c, in, out, &T);
  if (c->host_time) c->ht[0] += wall_s() - w0;
  if (rc) return rc;
  const rl_config& g = c->cfg;
  const uint32_t n = in->n, nq = in->n_requests;
  const uint64_t B = in->buf_bytes;
  const uint64_t nb = reinterpret_cast<const uint32_t*>(in->buf + in->index)[4ull * T + 3];
  HIPCHK(c, hipSetDevice(g.device));
  rc = ensure_host_slots(c);
  if (rc) return rc;
  const uint32_t j = c->hnext;
  HostSlot& h = c->hs[j];
  if (B > h.cbuf_cap) {  // grows to the largest buffer seen (the slot's previous batch drained first)
    HIPCHK(c, hipEventSynchronize(h.out_done));
    if (h.cbuf) HIPCHK(c, hipFree(h.cbuf));
    h.cbuf = nullptr;
    h.cbuf_cap = 0;
    HIPCHK(c, dalloc(&h.cbuf, B + 64));
    h.cbuf_cap = B;
  }
  c->hnext = (j + 1) % NBUF;
  hipStream_t up = hostfed_stream(c, true);
  const double w1 = c->host_time ? wall_s() : 0;
  if (c->copy_time) HIPCHK(c, hipEventRecord(c->ct_ev[2][c->ct_n % 64], up));
  HIPCHK(c, slot_drained(c, h, up));  // the slot's previous batch is drained
  if (c->copy_time) {
    copy_time_fold(c, false);
    HIPCHK(c, hipEventRecord(c->ct_ev[0][c->ct_n % 64], up));
  }
  if (B) HIPCHK(c, hipMemcpyAsync(h.cbuf, in->buf, B, hipMemcpyHostToDevice, up));
  if (c->copy_time) HIPCHK(c, hipEventRecord(c->ct_ev[1][c->ct_n++ % 64], up));
  HIPCHK(c, hipEventRecord(h.in_done, up));
  const double w2 = c->host_time ? wall_s() : 0;
  // unpacked on the batch's pipeline stream (as the compact batch)
  HIPCHK(c, hipStreamWaitEvent(c->pipe[c->next], h.in_done, 0));
  launch_unpack_prefixed(*in, h.cbuf, 0, T, h.stem, h.off, h.req, h.unit, h.flags, h.limit, h.hits, h.rule, h.now,
                         c->s[c->next].err, c->pipe[c->next]);
  if (c->host_time) {
    const double w3 = wall_s();
    c->ht[1] += w2 - w1;
    c->ht[2] += w3 - w2;
    c->ht_n++;
  }
  rl_batch d{};
  d.n = n;
  d.n_requests = nq;
  d.n_rules = in->n_rules;
  d.stem_bytes = h.stem;
  d.stem_off = h.off;
  d.now = h.now;
  d.req_idx = h.req;
  d.unit = h.unit;
  d.flags = h.flags;
  d.limit = h.limit;
  d.hits = h.hits;
  d.rule_id = h.rule;
  return host_slot_run(c, h, d, nb, out);
}

int eng_do_limit(Engine* c, const rl_batch* in, rl_result* out) {
  if (!c || !in || !out) return set_err(c, RL_E_INVALID, "gpu: null argument");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  BatchDev b{};
  int rc = stage(c, in, &b);
  if (rc) return rc;
  hipStream_t st = c->stream;
  OutDev o{c->d_code, c->d_rem, c->d_reset, c->d_stats, out->status ? c->d_status : nullptr};
  enqueue(c, b, o, 0, st, false);
  HIPCHK(c, hipGetLastError());
  const uint32_t n = in->n;
  if (n) {
    if (out->status) HIPCHK(c, hipMemcpyAsync(out->status, c->d_status, n, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(out->code, c->d_code, n, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(out->limit_remaining, c->d_rem, n * 4, hipMemcpyDeviceToHost, st));
    if (out->reset_s) HIPCHK(c, hipMemcpyAsync(out->reset_s, c->d_reset, n * 4, hipMemcpyDeviceToHost, st));
  }
  if (in->n_rules)
    HIPCHK(c, hipMemcpyAsync(out->stats, c->d_stats, (size_t)in->n_rules * RL_NUM_STATS * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, track(c, st));
  c->batches++;
  c->decisions += n;
  return collect(c);
}

int eng_restore(Engine* c, const rl_restore_batch* r) {
  if (!c || !r) return set_err(c, RL_E_INVALID, "gpu: null argument");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (!r->n) return RL_OK;
  // A restore batch is a batch of SET records: req = record index, hits = count,
  // flags = local-cache bit. It runs through the same grouping pipeline.
  std::string* e = &c->last_error;
  (void)e;
  const uint32_t n = r->n;
  uint32_t* req = new uint32_t[n];
  uint32_t* zero = new uint32_t[n]();
  uint8_t* lcf = new uint8_t[n]();
  for (uint32_t i = 0; i < n; i++) {
    req[i] = i;
    if (r->lc) lcf[i] = r->lc[i] ? 1 : 0;
  }
  rl_batch in{};
  in.n = n;
  in.n_requests = n;
  in.n_rules = 1;
  in.stem_bytes = r->stem_bytes;
  in.stem_off = r->stem_off;
  in.now = r->now;
  in.req_idx = req;
  in.unit = r->unit;
  in.flags = lcf;
  in.limit = zero;
  in.hits = r->count;
  in.rule_id = zero;
  BatchDev b{};
  int rc = stage(c, &in, &b);
  if (!rc) {
    OutDev o{c->d_code, c->d_rem, c->d_reset, c->d_stats, nullptr};
    enqueue(c, b, o, 1, c->stream, false);
    hipError_t he = hipGetLastError();
    rc = he != hipSuccess ? set_err(c, RL_E_HIP, std::string("gpu: ") + hipGetErrorString(he)) : collect(c);
  }
  delete[] req;
  delete[] zero;
  delete[] lcf;
  return rc;
}

int eng_sweep(Engine* c, int64_t now, uint64_t* n_evicted) {
  if (!c) return set_err(c, RL_E_INVALID, "gpu: null ctx");
  if (now < 0 || now > (int64_t)NOW_MAX) return set_err(c, RL_E_TIME, "gpu: sweep time out of range");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  // the sweep time becomes a floor: later requests may not be earlier
  int64_t last = 0;
  HIPCHK(c, after_batches(c, c->stream));
  HIPCHK(c, hipMemcpyAsync(&last, c->s[0].time_floor, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (now > last) HIPCHK(c, hipMemcpyAsync(c->s[0].time_floor, &now, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(c->s[0].counters, 0, 8, c->stream));
  {
    const TableDev t = table_view(c);
    launch_sweep(t, c->nslots, (uint32_t)now, c->s[0].counters, c->stream);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->h_counters, c->s[0].counters, 40, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (n_evicted) *n_evicted = c->h_counters[0];
  if (c->h_counters[0] && c->h_counters[4]) {
    // reclaim the long-stem arena: live slots' overflow bytes move to the spare
    // arena, packed from 0, and the two swap (counters[4] = the arena cursor)
    HIPCHK(c, hipMemsetAsync(c->s[0].counters + 4, 0, 8, c->stream));
    launch_arena_compact(c->slots, c->nslots, c->arena, c->arena2, c->s[0].counters + 4, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::swap(c->arena, c->arena2);
  }
  return RL_OK;
}

int eng_table_info_get(Engine* c, rl_table_info* info) {
  if (!c || !info) return set_err(c, RL_E_INVALID, "gpu: null argument");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, after_batches(c, c->stream));
  HIPCHK(c, hipMemsetAsync(c->s[0].counters, 0, 32, c->stream));
  launch_table_info(c->slots, c->nslots, c->s[0].counters, c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->h_counters, c->s[0].counters, 40, hipMemcpyDeviceToHost, c->stream));
  std::vector<unsigned long long> ctr;
  unsigned long long lost = 0, refused = 0;
  HIPCHK(c, log_ctr_get(c, ctr, &lost, &refused));  // (synchronises: h_counters is read below)
  info->history_entries = (uint64_t)LOG_PARTS * c->log_cap;
  info->history_appended = 0;
  for (unsigned long long k : ctr) info->history_appended += k;
  info->history_lost = lost;
  info->history_refused = refused;
  info->history_slots = c->h_counters[3];
  info->table_slots = c->nslots;
  info->live_slots = c->h_counters[0];
  info->tombstones = c->h_counters[1];
  info->exact_stems = c->h_counters[2];
  info->arena_bytes_used = c->h_counters[4] * 16;
  info->batches = c->batches;
  info->decisions = c->decisions;
  return RL_OK;
}

int eng_debug_keys(Engine* c, const rl_batch* in, uint8_t* out_bytes, uint32_t* out_off, uint32_t out_cap) {
  if (!c || !in || !out_off) return set_err(c, RL_E_INVALID, "gpu: null argument");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  BatchDev b{};
  int rc = stage(c, in, &b);
  if (rc) return rc;
  const uint32_t n = in->n;
  const size_t cap = (size_t)(n ? in->stem_off[n] : 0) + 24ull * n + 1;
  uint8_t* d_out = nullptr;
  uint32_t* d_len = nullptr;
  HIPCHK(c, dalloc(&d_out, cap));
  HIPCHK(c, dalloc(&d_len, (size_t)n + 1));
  launch_debug_keys(b, d_out, d_len, c->stream);
  uint8_t* h_out = new uint8_t[cap];
  uint32_t* h_len = new uint32_t[n + 1];
  hipError_t e1 = hipMemcpyAsync(h_out, d_out, cap, hipMemcpyDeviceToHost, c->stream);
  hipError_t e2 = hipMemcpyAsync(h_len, d_len, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream);
  hipError_t e3 = hipStreamSynchronize(c->stream);
  (void)hipFree(d_out);
  (void)hipFree(d_len);
  rc = (e1 || e2 || e3) ? set_err(c, RL_E_HIP, "gpu: debug_keys copy failed") : RL_OK;
  uint32_t pos = 0;
  out_off[0] = 0;
  for (uint32_t i = 0; i < n && rc == RL_OK; i++) {
    if (pos + h_len[i] > out_cap) {
      rc = set_err(c, RL_E_CAPACITY, "gpu: debug_keys output buffer too small");
      break;
    }
    memcpy(out_bytes + pos, h_out + in->stem_off[i] + 24ull * i, h_len[i]);
    pos += h_len[i];
    out_off[i + 1] = pos;
  }
  delete[] h_out;
  delete[] h_len;
  return rc;
}

int eng_debug_log_tear(Engine* c, const rl_log_tear* arm, rl_log_tear* out) {
  if (!c) return set_err(c, RL_E_INVALID, "gpu: null ctx");
  if (!log_tear_hook()) return set_err(c, RL_E_INVALID, "gpu: rl_debug_log_tear needs a library built with RL_LOG_TEAR");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, after_batches(c, c->stream));
  if (!c->tear) {
    HIPCHK(c, dalloc(&c->tear, sizeof(rl_log_tear) / 4));
    HIPCHK(c, hipMemsetAsync(c->tear, 0, sizeof(rl_log_tear), c->stream));
  }
  if (out) {
    HIPCHK(c, hipMemcpyAsync(out, c->tear, sizeof *out, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemsetAsync(c->tear, 0, 4, c->stream));  // disarmed
  }
  if (arm) {
    if (arm->protocol > 1 || arm->sched[0] > arm->sched[1] || arm->sched[1] > arm->sched[2])
      return set_err(c, RL_E_INVALID, "gpu: bad rl_log_tear");
    rl_log_tear a = *arm;
    a.armed = 1;
    a.verdict = 0;
    HIPCHK(c, hipMemcpyAsync(c->tear, &a, sizeof a, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RL_OK;
}

int eng_debug_decide(Engine* c, uint32_t n, const uint32_t* before, const uint32_t* after, const uint8_t* lc_hit,
                    const uint32_t* hits, const uint32_t* limit, const uint8_t* unit, const uint8_t* flags,
                    const int64_t* now, uint8_t* code, uint32_t* remaining, uint32_t* reset_s,
                    uint64_t* stat_deltas, uint8_t* lc_set) {
  if (!c) return set_err(c, RL_E_INVALID, "gpu: null ctx");
  if (!n) return RL_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  for (uint32_t i = 0; i < n; i++)
    if (unit[i] < 1 || unit[i] > 4) return set_err(c, RL_E_INVALID, "gpu: unit out of range");
  uint32_t *d_b, *d_a, *d_h, *d_l, *d_rem, *d_rs;
  uint8_t *d_lc, *d_u, *d_f, *d_code, *d_set;
  int64_t* d_now;
  unsigned long long* d_del;
  HIPCHK(c, dalloc(&d_b, n));
  HIPCHK(c, dalloc(&d_a, n));
  HIPCHK(c, dalloc(&d_h, n));
  HIPCHK(c, dalloc(&d_l, n));
  HIPCHK(c, dalloc(&d_rem, n));
  HIPCHK(c, dalloc(&d_rs, n));
  HIPCHK(c, dalloc(&d_lc, n));
  HIPCHK(c, dalloc(&d_u, n));
  HIPCHK(c, dalloc(&d_f, n));
  HIPCHK(c, dalloc(&d_code, n));
  HIPCHK(c, dalloc(&d_set, n));
  HIPCHK(c, dalloc(&d_now, n));
  HIPCHK(c, dalloc(&d_del, (size_t)n * RL_NUM_STATS));
  hipStream_t st = c->stream;
  HIPCHK(c, hipMemcpyAsync(d_b, before, n * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(d_a, after, n * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(d_h, hits, n * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(d_l, limit, n * 4, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(d_lc, lc_hit, n, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(d_u, unit, n, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(d_f, flags, n, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(d_now, now, n * 8, hipMemcpyHostToDevice, st));
  launch_debug_decide(n, d_b, d_a, d_lc, d_h, d_l, d_u, d_f, d_now, c->cfg.near_limit_ratio,
                      c->cfg.local_cache_enabled, d_code, d_rem, d_rs, d_del, d_set, st);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(code, d_code, n, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(remaining, d_rem, n * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(reset_s, d_rs, n * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(stat_deltas, d_del, (size_t)n * RL_NUM_STATS * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(lc_set, d_set, n, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  void* bufs[] = {d_b, d_a, d_h, d_l, d_rem, d_rs, d_lc, d_u, d_f, d_code, d_set, d_now, d_del};
  for (void* p : bufs) (void)hipFree(p);
  return RL_OK;
}

// ---- config match: GetLimit on the device (rl_match.hip) -------------------

int eng_config_load(Engine* c, const rl_config_tree* t) {
  if (!c || !t || (t->n_nodes && (!t->nodes || (t->key_bytes_len && !t->key_bytes))) ||
      (t->cache_key_prefix_len && !t->cache_key_prefix))
    return set_err(c, RL_E_INVALID, "gpu: null config tree");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const uint32_t n = t->n_nodes;
  std::vector<CfgNode> nodes(n);
  for (uint32_t i = 0; i < n; i++) {
    const rl_config_node& x = t->nodes[i];
    if (x.parent < -1 || x.parent >= (int32_t)i || (uint64_t)x.key_off + x.key_len > t->key_bytes_len)
      return set_err(c, RL_E_INVALID, "gpu: config node " + std::to_string(i) + ": bad parent or key range");
    if (x.has_limit && !x.unlimited && (x.unit < RL_UNIT_SECOND || x.unit > RL_UNIT_DAY))
      return set_err(c, RL_E_INVALID, "gpu: config node " + std::to_string(i) + ": invalid rate limit unit");
    if (x.has_limit && x.rule_id >= c->cfg.max_rules)
      return set_err(c, RL_E_INVALID, "gpu: config node " + std::to_string(i) + ": rule id >= max_rules");
    CfgNode& d = nodes[i];
    d = CfgNode{};
    d.parent = x.parent;
    d.key_off = x.key_off;
    d.key_len = x.key_len;
    d.rpu = x.requests_per_unit;
    d.rule = x.rule_id;
    d.unit = x.unit;
    d.has_limit = x.has_limit ? 1 : 0;
    d.unlimited = x.unlimited ? 1 : 0;
    d.shadow = x.shadow_mode ? 1 : 0;
    if (x.parent >= 0) nodes[x.parent].n_children++;
  }
  uint32_t size = 16;
  while (size < 2 * n) size <<= 1;
  std::vector<unsigned long long> index(size, 0);
  const uint8_t* kb = t->key_bytes;
  for (uint32_t i = 0; i < n; i++) {
    const rl_config_node& x = t->nodes[i];
    const uint64_t h = cfg_hash(x.parent, kb + x.key_off, x.key_len);
    uint32_t pos = (uint32_t)h & (size - 1);
    for (;; pos = (pos + 1) & (size - 1)) {
      const unsigned long long e = index[pos];
      if (!e) break;
      const rl_config_node& y = t->nodes[(uint32_t)(e >> 32) - 1];
      if (y.parent == x.parent && y.key_len == x.key_len && !memcmp(kb + y.key_off, kb + x.key_off, x.key_len))
        return set_err(c, RL_E_INVALID, "gpu: duplicate config key under one parent (node " + std::to_string(i) + ")");
    }
    index[pos] = (unsigned long long)(uint32_t)(h >> 32) | (unsigned long long)(i + 1) << 32;
  }
  // one blob [nodes | index | prefix ‖ keys], so a small config is staged into LDS in one copy
  const uint64_t nkeys = t->cache_key_prefix_len + t->key_bytes_len;
  const uint64_t idx_off = (uint64_t)n * sizeof(CfgNode), key_off = idx_off + size * 8ull;
  const uint64_t blob = (key_off + nkeys + 3) & ~3ull;
  std::vector<uint8_t> host(blob, 0);
  if (n) memcpy(host.data(), nodes.data(), n * sizeof(CfgNode));
  memcpy(host.data() + idx_off, index.data(), size * 8ull);
  if (t->cache_key_prefix_len) memcpy(host.data() + key_off, t->cache_key_prefix, t->cache_key_prefix_len);
  if (t->key_bytes_len) memcpy(host.data() + key_off + t->cache_key_prefix_len, kb, t->key_bytes_len);
  HIPCHK(c, after_batches(c, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->cfg_blob) (void)hipFree(c->cfg_blob);
  c->cfg_blob = nullptr;
  c->cfg_loaded = false;
  HIPCHK(c, dalloc(&c->cfg_blob, blob));
  if (!c->h_match) HIPCHK(c, hipHostMalloc((void**)&c->h_match, 16, hipHostMallocDefault));
  HIPCHK(c, hipMemcpy(c->cfg_blob, host.data(), blob, hipMemcpyHostToDevice));
  uint8_t* B = c->cfg_blob;
  CfgDev d{};
  d.nodes = (const CfgNode*)B;
  d.index = (const unsigned long long*)(B + idx_off);
  d.keys = B + key_off + t->cache_key_prefix_len;
  d.mask = size - 1;
  d.n_nodes = n;
  d.prefix = B + key_off;
  d.prefix_len = t->cache_key_prefix_len;
  d.blob = B;
  d.blob_words = blob / 4 <= CFG_LDS_WORDS ? (uint32_t)(blob / 4) : 0u;
  d.idx_word = (uint32_t)(idx_off / 4);
  d.key_word = (uint32_t)(key_off / 4);
  c->cfg_dev = d;
  c->cfg_loaded = true;
  return RL_OK;
}

int eng_do_limit_requests(Engine* c, const rl_request_batch* in, rl_request_result* out, RequestsDoLimit run,
                          void* user) {
  if (!c || !in || !out) return set_err(c, RL_E_INVALID, "gpu: null argument");
  // checkServiceErr(snappedConfig != nil, ...) (ratelimit.go:106)
  if (!c->cfg_loaded) return set_err(c, RL_E_INVALID, "gpu: no rate limit configuration loaded");
  const uint32_t n = in->n_descriptors, nq = in->n_requests, ne = in->n_entries;
  if (n > c->cfg.max_batch || nq > c->cfg.max_requests || in->n_rules > c->cfg.max_rules)
    return set_err(c, RL_E_CAPACITY, "gpu: request batch exceeds configured max_batch/max_requests/max_rules");
  if (n && !nq) return set_err(c, RL_E_INVALID, "gpu: descriptors without requests");
  if (!in->domain_off || !in->entry_first || !in->desc_off || (nq && (!in->now || !in->hits)) ||
      (n && !in->req_idx) || (ne && (!in->key_len || !in->value_len)))
    return set_err(c, RL_E_INVALID, "gpu: null request batch array");
  const bool ovr = in->override_flags != nullptr;
  if (ovr && (!in->override_rpu || !in->override_unit || !in->override_rule))
    return set_err(c, RL_E_INVALID, "gpu: override_flags without override_rpu/unit/rule");
  if (in->entry_first[0] != 0 || in->entry_first[n] != ne || in->desc_off[0] != 0 || in->domain_off[0] != 0)
    return set_err(c, RL_E_INVALID, "gpu: request batch offsets must start at 0 and end at n_entries");
  const uint64_t dom_bytes = in->domain_off[nq], desc_bytes = in->desc_off[n];
  if ((dom_bytes && !in->domain_bytes) || (desc_bytes && !in->desc_bytes))
    return set_err(c, RL_E_INVALID, "gpu: null request byte array");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  // one device buffer, carved (256-B aligned pieces)
  const size_t scan = n ? match_scan_bytes(n) : 0;
  size_t need = 0;
  auto piece = [&need](size_t bytes) {
    const size_t o = need;
    need += (std::max<size_t>(bytes, 1) + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_dom = piece(dom_bytes), o_domoff = piece((nq + 1) * 4ull), o_hits = piece(nq * 4ull),
               o_req = piece(n * 4ull), o_ent = piece((n + 1) * 4ull), o_doff = piece((n + 1) * 4ull),
               o_desc = piece(desc_bytes), o_kl = piece(ne * 2ull), o_vl = piece(ne * 2ull),
               o_ovf = piece(ovr ? n : 0), o_ovr = piece(ovr ? n * 4ull : 0), o_ovu = piece(ovr ? n : 0),
               o_ovrule = piece(ovr ? n * 4ull : 0), o_v = piece(n * 16ull), o_kind = piece(n * 4ull),
               o_rpu = piece(n * 4ull), o_rule = piece(n * 4ull), o_cnt = piece(16), o_code = piece(n),
               o_rem = piece(n * 4ull), o_reset = piece(n * 4ull), o_match = piece(n), o_orule = piece(n * 4ull),
               o_orpu = piece(n * 4ull), o_ounit = piece(n), o_tmp = piece(scan);
  hipStream_t st = c->stream;
  HIPCHK(c, after_batches(c, st));
  if (need > c->mbuf_cap) {
    HIPCHK(c, hipStreamSynchronize(st));
    if (c->mbuf) (void)hipFree(c->mbuf);
    c->mbuf = nullptr;
    c->mbuf_cap = 0;
    HIPCHK(c, hipMalloc((void**)&c->mbuf, need));
    c->mbuf_cap = need;
  }
  uint8_t* B = c->mbuf;
  auto h2d = [&](size_t off, const void* src, size_t bytes) {
    return bytes ? hipMemcpyAsync(B + off, src, bytes, hipMemcpyHostToDevice, st) : hipSuccess;
  };
  HIPCHK(c, h2d(o_dom, in->domain_bytes, dom_bytes));
  HIPCHK(c, h2d(o_domoff, in->domain_off, (nq + 1) * 4ull));
  HIPCHK(c, h2d(o_hits, in->hits, nq * 4ull));
  HIPCHK(c, h2d(o_req, in->req_idx, n * 4ull));
  HIPCHK(c, h2d(o_ent, in->entry_first, (n + 1) * 4ull));
  HIPCHK(c, h2d(o_doff, in->desc_off, (n + 1) * 4ull));
  HIPCHK(c, h2d(o_desc, in->desc_bytes, desc_bytes));
  HIPCHK(c, h2d(o_kl, in->key_len, ne * 2ull));
  HIPCHK(c, h2d(o_vl, in->value_len, ne * 2ull));
  if (ovr) {
    HIPCHK(c, h2d(o_ovf, in->override_flags, n));
    HIPCHK(c, h2d(o_ovr, in->override_rpu, n * 4ull));
    HIPCHK(c, h2d(o_ovu, in->override_unit, n));
    HIPCHK(c, h2d(o_ovrule, in->override_rule, n * 4ull));
  }
  if (nq) HIPCHK(c, hipMemcpyAsync(c->d_now, in->now, nq * 8ull, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemsetAsync(B + o_cnt, 0, 16, st));
  ReqDev r;
  r.n_req = nq;
  r.n_desc = n;
  r.n_ent = ne;
  r.dom_total = (uint32_t)dom_bytes;
  r.desc_total = (uint32_t)desc_bytes;
  r.dom = B + o_dom;
  r.dom_off = (const uint32_t*)(B + o_domoff);
  r.hits = (const uint32_t*)(B + o_hits);
  r.req = (const uint32_t*)(B + o_req);
  r.ent_first = (const uint32_t*)(B + o_ent);
  r.desc_off = (const uint32_t*)(B + o_doff);
  r.desc = B + o_desc;
  r.klen = (const uint16_t*)(B + o_kl);
  r.vlen = (const uint16_t*)(B + o_vl);
  r.ovf = ovr ? B + o_ovf : nullptr;
  r.ov_rpu = ovr ? (const uint32_t*)(B + o_ovr) : nullptr;
  r.ov_unit = ovr ? B + o_ovu : nullptr;
  r.ov_rule = ovr ? (const uint32_t*)(B + o_ovrule) : nullptr;
  MatchBuf m{(unsigned long long*)(B + o_v), (uint32_t*)(B + o_kind), (uint32_t*)(B + o_rpu),
             (uint32_t*)(B + o_rule), (uint32_t*)(B + o_cnt)};
  // the matched descriptors become an ordinary DoLimit batch in the staging buffers
  PackOut po{c->d_stem, c->d_off, c->d_req, c->d_unit, c->d_flags, c->d_limit, c->d_hits, c->d_rule,
             c->cfg.max_stem_bytes};
  launch_match(c->cfg_dev, r, m, po, B + o_tmp, scan, st);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->h_match, B + o_cnt, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if (c->h_match[2] & MATCH_ERR_REQ)
    return set_err(c, RL_E_INVALID, "gpu: malformed request batch (request index or entry byte layout)");
  if (c->h_match[2] & MATCH_ERR_CAP)
    return set_err(c, RL_E_CAPACITY, "gpu: matched stems exceed max_stem_bytes");
  const uint32_t nm = n ? c->h_match[0] : 0;
  if (!n) {  // off[0] of the empty batch
    HIPCHK(c, hipMemsetAsync(c->d_off, 0, 4, st));
  }
  rl_batch pb{};
  pb.n = nm;
  pb.n_requests = nq;
  pb.n_rules = in->n_rules;
  pb.stem_bytes = c->d_stem;
  pb.stem_off = c->d_off;
  pb.now = c->d_now;
  pb.req_idx = c->d_req;
  pb.unit = c->d_unit;
  pb.flags = c->d_flags;
  pb.limit = c->d_limit;
  pb.hits = c->d_hits;
  pb.rule_id = c->d_rule;
  if (run) {
    rl_result dout{};
    dout.code = c->d_code;
    dout.limit_remaining = c->d_rem;
    dout.reset_s = c->d_reset;
    dout.stats = reinterpret_cast<uint64_t*>(c->d_stats);
    const int rc = run(user, &pb, &dout, st);
    if (rc) return rc;  // (the runner's own error report)
    HIPCHK(c, hipSetDevice(c->cfg.device));
  } else {
    BatchDev b = dev_view(c, &pb, c->cfg.max_stem_bytes);
    OutDev o{c->d_code, c->d_rem, c->d_reset, c->d_stats, nullptr};
    enqueue(c, b, o, 0, st, false);
  }
  ReqOutDev ro{B + o_code, (uint32_t*)(B + o_rem), (uint32_t*)(B + o_reset), B + o_match,
               (uint32_t*)(B + o_orule), (uint32_t*)(B + o_orpu), B + o_ounit};
  launch_match_expand(r, m, c->d_code, c->d_rem, c->d_reset, ro, st);
  HIPCHK(c, hipGetLastError());
  auto d2h = [&](void* dst, size_t off, size_t bytes) {
    return (bytes && dst) ? hipMemcpyAsync(dst, B + off, bytes, hipMemcpyDeviceToHost, st) : hipSuccess;
  };
  HIPCHK(c, d2h(out->code, o_code, n));
  HIPCHK(c, d2h(out->limit_remaining, o_rem, n * 4ull));
  HIPCHK(c, d2h(out->reset_s, o_reset, n * 4ull));
  HIPCHK(c, d2h(out->match, o_match, n));
  HIPCHK(c, d2h(out->rule_id, o_orule, n * 4ull));
  HIPCHK(c, d2h(out->requests_per_unit, o_orpu, n * 4ull));
  HIPCHK(c, d2h(out->unit, o_ounit, n));
  if (in->n_rules && out->stats)
    HIPCHK(c, hipMemcpyAsync(out->stats, c->d_stats, (size_t)in->n_rules * RL_NUM_STATS * 8, hipMemcpyDeviceToHost, st));
  c->batches++;
  c->decisions += nm;
  return collect(c);
}

// ---- observability and restart ---------------------------------------------

int eng_local_cache_info_get(Engine* c, int64_t now, rl_local_cache_info* info) {
  if (!c || !info) return set_err(c, RL_E_INVALID, "gpu: null argument");
  if (now < 0 || now > (int64_t)NOW_MAX) return set_err(c, RL_E_TIME, "gpu: now out of range");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, after_batches(c, c->stream));
  unsigned long long* ctr = c->s[0].counters;
  HIPCHK(c, hipMemsetAsync(ctr + 7, 0, 8, c->stream));
  launch_lc_count(table_view(c), c->nslots, (uint32_t)now, ctr + 7, c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->h_counters, ctr, 64, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  info->entry_count = c->h_counters[7];
  info->lookup_count = c->h_counters[5];
  info->hit_count = c->h_counters[6];
  info->miss_count = c->h_counters[5] - c->h_counters[6];
  return RL_OK;
}

namespace {
// "LSNAPA06": 64-B slots, history log; since round 6 a stem whose hash's high
// word is KEY_DUP homes as KEY_DUP - 1 (rl_device.h), so a round-5 image ("05")
// is refused rather than loaded with such a stem where lookups no longer go
constexpr uint64_t SNAP_MAGIC = 0x36304150414e534cull;
struct SnapHeader {
  uint64_t magic, nslots, arena_used16, hash_seed;  // slots are placed by the keyed hash: restore adopts its key
  int64_t time_floor;
  uint32_t log_parts, log_cap;  // slots hold entry pointers, so restore needs the same log geometry
  uint64_t reserved[2];
};
static_assert(sizeof(SnapHeader) == 64, "snapshot header");
// then: the slots; the LOG_PARTS append counters; per partition its written
// entries [0, min(counter, log_cap)); the used arena

uint64_t part_entries(unsigned long long ctr, uint32_t cap) { return std::min<uint64_t>(ctr, cap); }

int snap_state(Engine* c, SnapHeader* h, std::vector<unsigned long long>& ctr) {
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, after_batches(c, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->h_counters, c->s[0].counters, 64, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(&h->time_floor, c->s[0].time_floor, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, log_ctr_get(c, ctr, nullptr));
  h->arena_used16 = std::min<uint64_t>(c->h_counters[4], c->arena_cap16);
  h->log_parts = LOG_PARTS;
  h->log_cap = c->log_cap;
  return RL_OK;
}

uint64_t snap_bytes(uint64_t nslots, const SnapHeader& h, const std::vector<unsigned long long>& ctr) {
  uint64_t b = sizeof(SnapHeader) + nslots * sizeof(Slot) + (uint64_t)h.log_parts * 8 + h.arena_used16 * 16;
  for (unsigned long long k : ctr) b += part_entries(k, h.log_cap) * sizeof(LogEnt);
  return b;
}

// A slot image the kernels can use without reading past the arena: a live
// slot's unit is a rate-limit unit and a long stem's tail lies in the used
// arena. (Chain pointers need no check: every one addresses the log, and a
// foreign or stale entry fails its owner check: RL_E_TIME, never a count.)
bool slots_valid(const Slot* s, uint64_t n, uint64_t arena_used16) {
  for (uint64_t i = 0; i < n; i++) {
    if (s[i].tag < 2) continue;
    if (s[i].unit < RL_UNIT_SECOND || s[i].unit > RL_UNIT_DAY) return false;
    if (s[i].key_len > KEY_IN) {
      const uint32_t off = reinterpret_cast<const uint32_t*>(&s[i])[SLOT_EXT_DW];
      if ((uint64_t)off + (s[i].key_len - KEY_SPLIT + 15) / 16 > arena_used16) return false;
    }
  }
  return true;
}
}  // namespace

int eng_snapshot_size(Engine* c, uint64_t* bytes) {
  if (!c || !bytes) return set_err(c, RL_E_INVALID, "gpu: null argument");
  SnapHeader h{};
  std::vector<unsigned long long> ctr;
  int rc = snap_state(c, &h, ctr);
  if (rc) return rc;
  *bytes = snap_bytes(c->nslots, h, ctr);
  return RL_OK;
}

int eng_snapshot_save(Engine* c, void* host, uint64_t bytes) {
  if (!c || !host) return set_err(c, RL_E_INVALID, "gpu: null argument");
  SnapHeader h{};
  std::vector<unsigned long long> ctr;
  int rc = snap_state(c, &h, ctr);
  if (rc) return rc;
  h.magic = SNAP_MAGIC;
  h.nslots = c->nslots;
  h.hash_seed = c->hash_seed;
  if (bytes < snap_bytes(c->nslots, h, ctr))
    return set_err(c, RL_E_CAPACITY, "gpu: snapshot buffer smaller than rl_snapshot_size");
  uint8_t* p = (uint8_t*)host;
  memcpy(p, &h, sizeof h);
  p += sizeof h;
  const uint64_t tb = c->nslots * sizeof(Slot);
  HIPCHK(c, hipMemcpy(p, c->slots, tb, hipMemcpyDeviceToHost));
  p += tb;
  memcpy(p, ctr.data(), ctr.size() * 8);
  p += ctr.size() * 8;
  for (uint32_t k = 0; k < LOG_PARTS; k++) {
    const uint64_t m = part_entries(ctr[k], c->log_cap);
    if (m) HIPCHK(c, hipMemcpy(p, c->log + (size_t)k * c->log_cap, m * sizeof(LogEnt), hipMemcpyDeviceToHost));
    p += m * sizeof(LogEnt);
  }
  if (h.arena_used16) HIPCHK(c, hipMemcpy(p, c->arena, h.arena_used16 * 16, hipMemcpyDeviceToHost));
  return RL_OK;
}

int eng_snapshot_load(Engine* c, const void* host, uint64_t bytes) {
  if (!c || !host) return set_err(c, RL_E_INVALID, "gpu: null argument");
  SnapHeader h;
  if (bytes < sizeof h) return set_err(c, RL_E_INVALID, "gpu: snapshot too short");
  memcpy(&h, host, sizeof h);
  if (h.magic != SNAP_MAGIC) return set_err(c, RL_E_INVALID, "gpu: not a table snapshot");
  if (h.nslots != c->nslots) return set_err(c, RL_E_INVALID, "gpu: snapshot table_slots differ from this ctx");
  if (h.arena_used16 > c->arena_cap16) return set_err(c, RL_E_INVALID, "gpu: snapshot arena larger than this ctx's");
  if (h.log_parts != LOG_PARTS || h.log_cap != c->log_cap)
    return set_err(c, RL_E_INVALID, "gpu: snapshot history_entries differ from this ctx");
  const uint8_t* p = (const uint8_t*)host + sizeof h;
  const uint64_t tb = h.nslots * sizeof(Slot);
  if (bytes < sizeof h + tb + LOG_PARTS * 8ull) return set_err(c, RL_E_INVALID, "gpu: snapshot truncated");
  std::vector<unsigned long long> ctr(LOG_PARTS);
  memcpy(ctr.data(), p + tb, LOG_PARTS * 8);
  if (bytes < snap_bytes(h.nslots, h, ctr)) return set_err(c, RL_E_INVALID, "gpu: snapshot truncated");
  if (!slots_valid(reinterpret_cast<const Slot*>(p), h.nslots, h.arena_used16))
    return set_err(c, RL_E_INVALID, "gpu: snapshot slots inconsistent (unit or long-stem arena offset)");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, after_batches(c, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->slots, p, tb, hipMemcpyHostToDevice));
  p += tb + LOG_PARTS * 8ull;
  for (uint32_t k = 0; k < LOG_PARTS; k++) {
    const uint64_t m = part_entries(ctr[k], c->log_cap);
    if (m) HIPCHK(c, hipMemcpy(c->log + (size_t)k * c->log_cap, p, m * sizeof(LogEnt), hipMemcpyHostToDevice));
    p += m * sizeof(LogEnt);
  }
  std::vector<unsigned long long> hc((size_t)(LOG_PARTS + 1) * LOG_CTR_STRIDE, 0ull);
  for (uint32_t k = 0; k < LOG_PARTS; k++) hc[(size_t)k * LOG_CTR_STRIDE] = ctr[k];
  HIPCHK(c, hipMemcpy(c->log_ctr, hc.data(), hc.size() * 8, hipMemcpyHostToDevice));
  if (h.arena_used16) HIPCHK(c, hipMemcpy(c->arena, p, h.arena_used16 * 16, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->s[0].counters + 4, &h.arena_used16, 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->s[0].time_floor, &h.time_floor, 8, hipMemcpyHostToDevice));
  c->hash_seed = h.hash_seed;
  c->cfg.hash_seed = h.hash_seed;
  c->hk = hash_key_of(h.hash_seed, c->cfg.debug_hash_bits);
  return RL_OK;
}

}  // namespace rl


