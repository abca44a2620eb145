// rl_api.hip — the extern "C" boundary of libratelimit_hip.so
// (include/ratelimit_hip.h).
//
// A ctx holds one engine per table shard (rl_engine.h: HBM table, pipeline
// buffers, streams). With one shard every entry point is the engine's own.
// With rl_config.n_shards > 1 the table is hash-sharded over the shards'
// devices inside this one process (the reference's single service process
// scaled out over a Redis cluster, src/redis/driver_impl.go:108-126; here the
// cgo adapter still drives one ctx). Each shard then also has a router
// (rl_comm.hip) and a worker thread; the routers form an in-process loopback
// world, so a multi-shard ctx runs exactly the protocol of one process per
// GPU (partition by owner, counts, records and stems, owner pipelines,
// results and stats, scatter), each shard on its own thread:
//
//   host batches (rl_do_limit, rl_do_limit_host_async): the batch is cut into
//     one request-aligned slice per shard; each shard's router copies its
//     slice over ITS device's PCIe link, partitions it and exchanges with the
//     others over xGMI (peer copies); the answers cross back per slice, and
//     the per-shard stats deltas are summed on the host;
//   device batches (rl_do_limit_async, memory of shard 0's GPU): shard 0's
//     router takes the whole batch and the others submit empty slices.
//
// The caller's thread only hands each batch to the workers and waits until
// they have ENQUEUED it (never for the GPU); rl_synchronize completes the
// in-flight batches (a collective step of the routers).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ratelimit_hip.h"
#include "rl_comm.h"
#include "rl_device.h"
#include "rl_engine.h"
#include "rl_kernels.h"

using namespace rl;

namespace {

constexpr uint32_t MAX_LOCAL_SHARDS = 16;

// One shard's worker: runs its router's collective steps on its own thread.
struct ShardWorker {
  enum Job { IDLE, BATCH, SYNC, EXIT };
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  Job job = IDLE;
  rl_batch in{};
  rl_result out{};
  CommIO io{};
  hipStream_t caller = nullptr;
  int rc = RL_OK;
};

// Stats of a host batch in flight: each shard's deltas land in a pinned ring
// entry (slot = the routers' slot of the batch); they are summed into the
// caller's out->stats once the batch is complete.
struct PendingStats {
  bool used = false;
  uint64_t* out = nullptr;
  uint32_t m = 0;
};

}  // namespace

struct rl_ctx {
  rl_config cfg;
  uint32_t n = 1;
  Engine* e[MAX_LOCAL_SHARDS] = {};
  CommRouter* comm = nullptr;  // rl_comm_init: multi-process routing (single-shard ctx)
  std::string last_error;
  // shards of this ctx (n > 1)
  CommRouter* r[MAX_LOCAL_SHARDS] = {};
  ShardWorker w[MAX_LOCAL_SHARDS];
  std::mutex done_mu;
  std::condition_variable done_cv;
  uint32_t busy = 0;
  uint32_t batch_no = 0;                      // batches submitted (router slot = batch_no % slots)
  std::vector<PendingStats> pend;             // [slots]
  unsigned long long* stats_ring = nullptr;   // pinned [slots][n][stats_cap]
  uint32_t stats_cap = 0;
};

namespace {

thread_local std::string g_api_err;

int fail(rl_ctx* c, int code, const std::string& msg) {
  if (c) c->last_error = msg;
  else g_api_err = msg;
  return code;
}

// An engine's failure, surfaced through the ctx.
int from_engine(rl_ctx* c, Engine* e, int rc) {
  if (rc && c->n > 1) c->last_error = eng_last_error(e);
  return rc;
}

#define API_HIP(c, expr)                                                                        \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess)                                                                       \
      return fail((c), RL_E_HIP, std::string("gpu: ") + #expr + ": " + hipGetErrorString(_e));  \
  } while (0)

uint32_t owner_of_host(uint64_t h, uint32_t n) { return (uint32_t)(((uint64_t)(uint32_t)h * n) >> 32); }

void worker_main(rl_ctx* c, uint32_t j) {
  (void)hipSetDevice(c->cfg.shard_device[j]);
  ShardWorker& w = c->w[j];
  for (;;) {
    ShardWorker::Job job;
    {
      std::unique_lock<std::mutex> l(w.mu);
      w.cv.wait(l, [&] { return w.job != ShardWorker::IDLE; });
      job = w.job;
    }
    if (job == ShardWorker::EXIT) return;
    int rc = RL_OK;
    if (job == ShardWorker::BATCH) {
      rc = comm_do_limit(c->r[j], c->e[j], &w.in, &w.out, w.caller, &w.io);
    } else {  // SYNC: the pending batch (collective), the router's streams, then the engine's error words
      rc = comm_synchronize(c->r[j], c->e[j]);
      const int re = eng_synchronize(c->e[j]);
      if (!rc) rc = re;
    }
    {
      std::lock_guard<std::mutex> l(w.mu);
      w.rc = rc;
      w.job = ShardWorker::IDLE;
    }
    {
      std::lock_guard<std::mutex> l(c->done_mu);
      c->busy--;
    }
    c->done_cv.notify_all();
  }
}

// Hand every shard its job (set up by the caller) and wait until all have
// returned from it; the first failing shard's status and message.
int run_shards(rl_ctx* c, ShardWorker::Job job) {
  {
    std::lock_guard<std::mutex> l(c->done_mu);
    c->busy = c->n;
  }
  for (uint32_t j = 0; j < c->n; j++) {
    {
      std::lock_guard<std::mutex> l(c->w[j].mu);
      c->w[j].job = job;
    }
    c->w[j].cv.notify_one();
  }
  {
    std::unique_lock<std::mutex> l(c->done_mu);
    c->done_cv.wait(l, [&] { return c->busy == 0; });
  }
  for (uint32_t j = 0; j < c->n; j++)
    if (c->w[j].rc) return fail(c, c->w[j].rc, eng_last_error(c->e[j]));
  return RL_OK;
}

void stop_shards(rl_ctx* c) {
  for (uint32_t j = 0; j < c->n; j++) {
    if (!c->w[j].th.joinable()) continue;
    {
      std::lock_guard<std::mutex> l(c->w[j].mu);
      c->w[j].job = ShardWorker::EXIT;
    }
    c->w[j].cv.notify_one();
    c->w[j].th.join();
  }
}

// The summed stats of the host batch that used ring entry s (its shards'
// slots are complete once their done events fired).
int finalize_stats(rl_ctx* c, uint32_t s, bool keep) {
  PendingStats& P = c->pend[s];
  if (!P.used) return RL_OK;
  P.used = false;
  for (uint32_t j = 0; j < c->n; j++) {
    const int rc = comm_wait_slot(c->r[j], c->e[j], s);
    if (rc) return from_engine(c, c->e[j], rc);
  }
  if (!keep || !P.out) return RL_OK;
  for (uint32_t i = 0; i < P.m; i++) {
    unsigned long long v = 0;
    for (uint32_t j = 0; j < c->n; j++) v += c->stats_ring[((size_t)s * c->n + j) * c->stats_cap + i];
    P.out[i] = v;
  }
  return RL_OK;
}

// keep_stats false (rl_destroy): the shards complete, but no caller memory is
// written (the caller may have freed a pending batch's outputs).
int synchronize_all(rl_ctx* c, bool keep_stats = true) {
  if (c->n > 1) {
    const int rc = run_shards(c, ShardWorker::SYNC);
    const std::string msg = c->last_error;
    for (uint32_t s = 0; s < c->pend.size(); s++) {
      const int fr = finalize_stats(c, s, keep_stats && rc == RL_OK);
      if (fr && !rc) return fr;
    }
    if (rc) c->last_error = msg;
    return rc;
  }
  int comm_rc = RL_OK;
  std::string comm_msg;
  if (c->comm) {  // (collective on a routed ctx: it completes the pending batch)
    comm_rc = comm_synchronize(c->comm, c->e[0]);
    if (comm_rc) comm_msg = eng_last_error(c->e[0]);
  }
  if (comm_rc) {
    // the engine's own words are collected (and cleared) too; the router's
    // failure is the one reported
    (void)eng_synchronize(c->e[0]);
    return eng_fail(c->e[0], comm_rc, comm_msg);
  }
  return eng_synchronize(c->e[0]);
}

// One batch through the shards: host (slices over every shard's link) or
// device (memory of shard 0's GPU: shard 0 takes it whole). cb: a compact host
// batch (in then carries only its sizes), cut at request boundaries.
int shards_submit(rl_ctx* c, const rl_batch* in, rl_result* out, bool host, hipStream_t caller,
                  const rl_batch_compact* cb = nullptr, const rl_batch_prefixed* pb = nullptr) {
  const uint32_t N = c->n, n = in->n, nq = in->n_requests;
  const uint32_t slots = (uint32_t)c->pend.size(), s = c->batch_no % slots;
  // the batch that used this slot of the routers is complete: its stats first
  int rc = finalize_stats(c, s, true);
  if (rc) return rc;
  const uint32_t m = in->n_rules * RL_NUM_STATS;
  if (host && m > c->stats_cap) {  // a larger stats ring: every pending batch completed and finalized first
    // (the last batch's second half runs only at the next call or a sync:
    // finalizing its ring entry before that read zeros)
    if ((rc = synchronize_all(c))) return rc;
    if (c->stats_ring) (void)hipHostFree(c->stats_ring);
    c->stats_ring = nullptr;
    c->stats_cap = 0;
    API_HIP(c, hipHostMalloc((void**)&c->stats_ring, (size_t)slots * N * m * 8));
    c->stats_cap = m;
  }
  if (host && c->stats_ring && c->stats_cap)  // (a slice that fails never writes its part: no stale deltas)
    memset(c->stats_ring + (size_t)s * N * c->stats_cap, 0, (size_t)N * c->stats_cap * 8);
  // request-aligned cuts of about n / N descriptors
  uint32_t d[MAX_LOCAL_SHARDS + 1], q[MAX_LOCAL_SHARDS + 1];
  d[0] = 0;
  q[0] = 0;
  d[N] = n;
  q[N] = nq;
  const uint32_t* first = cb ? reinterpret_cast<const uint32_t*>(cb->buf + cb->req_first) : nullptr;
  // a prefix-shared batch is cut at request tiles: the index holds each tile's first descriptor
  const uint32_t tiles = pb ? (nq + RL_PREFIXED_TILE - 1) / RL_PREFIXED_TILE : 0;
  const uint32_t* pix = pb ? reinterpret_cast<const uint32_t*>(pb->buf + pb->index) : nullptr;
  uint32_t t[MAX_LOCAL_SHARDS + 1];
  t[0] = 0;
  t[N] = tiles;
  for (uint32_t j = 1; j < N; j++) {
    if (pb) {  // (entries are checked against the sections on the device; clamp so slices stay ordered)
      t[j] = (uint32_t)((uint64_t)tiles * j / N);
      q[j] = std::min(t[j] * RL_PREFIXED_TILE, nq);
      d[j] = std::min(std::max(pix[4ull * t[j]], d[j - 1]), n);
      continue;
    }
    if (cb) {  // (about nq / N requests each; req_first was checked to lie in [0, n] by nobody yet: clamp)
      q[j] = std::max(q[j - 1], (uint32_t)((uint64_t)nq * j / N));
      d[j] = std::min(std::max(first[q[j]], d[j - 1]), n);
      continue;
    }
    uint32_t x = host ? (uint32_t)((uint64_t)n * j / N) : n;
    if (x < d[j - 1]) x = d[j - 1];
    while (x > 0 && x < n && in->req_idx[x] == in->req_idx[x - 1]) x++;
    d[j] = x;
    q[j] = x < n ? std::min(in->req_idx[x], nq) : nq;
    if (q[j] < q[j - 1]) q[j] = q[j - 1];
  }
  for (uint32_t j = 0; j < N; j++) {
    ShardWorker& w = c->w[j];
    w.caller = j == 0 ? caller : nullptr;
    w.io = CommIO{};
    w.in = *in;
    w.out = rl_result{};
    if (host && (cb || pb)) {
      const uint32_t a = d[j], b = d[j + 1];
      w.in = rl_batch{};
      w.in.n = b - a;
      w.in.n_requests = q[j + 1];  // (absolute: the slice's first request is q[j])
      w.in.n_rules = in->n_rules;
      w.out.code = out->code + a;
      w.out.limit_remaining = out->limit_remaining + a;
      w.out.reset_s = out->reset_s ? out->reset_s + a : nullptr;
      w.out.status = out->status ? out->status + a : nullptr;
      w.io.host = true;
      w.io.cb = cb;
      w.io.pb = pb;
      w.io.t0 = t[j];
      w.io.t1 = t[j + 1];
      w.io.da = a;
      w.io.qa = q[j];
      w.io.stats_host = m ? c->stats_ring + ((size_t)s * N + j) * c->stats_cap : nullptr;
    } else if (host) {
      const uint32_t a = d[j], b = d[j + 1];
      w.in.n = b - a;
      w.in.n_requests = q[j + 1];  // (absolute: the slice's first request is q[j])
      w.in.stem_off = in->stem_off + a;
      w.in.req_idx = in->req_idx + a;
      w.in.unit = in->unit + a;
      w.in.flags = in->flags + a;
      w.in.limit = in->limit + a;
      w.in.hits = in->hits + a;
      w.in.rule_id = in->rule_id + a;
      w.out.code = out->code ? out->code + a : nullptr;
      w.out.limit_remaining = out->limit_remaining ? out->limit_remaining + a : nullptr;
      w.out.reset_s = out->reset_s ? out->reset_s + a : nullptr;
      w.out.status = out->status ? out->status + a : nullptr;
      w.io.host = true;
      w.io.da = a;
      w.io.qa = q[j];
      w.io.stats_host = m ? c->stats_ring + ((size_t)s * N + j) * c->stats_cap : nullptr;
    } else if (j == 0) {
      w.out = *out;
    } else {  // an empty slice (the exchange is collective)
      w.in = rl_batch{};
      w.in.n_rules = in->n_rules;
    }
  }
  c->batch_no++;
  rc = run_shards(c, ShardWorker::BATCH);
  if (rc) return rc;
  if (host) {
    c->pend[s].used = true;
    c->pend[s].out = out->stats;
    c->pend[s].m = out->stats ? m : 0;
  }
  return RL_OK;
}

// Settle a multi-shard or routed ctx before a call that changes the table
// (on a routed ctx this makes the call collective, like rl_synchronize).
int settle(rl_ctx* c) { return (c->comm || c->n > 1) ? synchronize_all(c) : RL_OK; }
// Before a read-only getter: the shards of one ctx complete their batches
// (in-process, no peer to wait for); a routed ctx is not settled, since its
// pending batch's second half is a collective exchange and one rank polling
// its gauges would block on its peers. The engine getters order after every
// batch already enqueued on the engine, so a routed ctx's getters see all
// batches but the last one submitted.
int settle_local(rl_ctx* c) { return c->n > 1 ? synchronize_all(c) : RL_OK; }

constexpr uint64_t MSNAP_MAGIC = 0x31304853414e534cull;  // "LSNASH01": one image per shard

}  // namespace

extern "C" {

uint32_t rl_abi_version(void) { return RL_ABI_VERSION; }

const char* rl_last_error(const rl_ctx* c) {
  if (!c) return g_api_err.c_str();
  return c->n == 1 ? eng_last_error(c->e[0]) : c->last_error.c_str();
}

rl_ctx* rl_create(const rl_config* cfg_in, char* err, size_t errlen) {
  auto bad = [&](const std::string& m) -> rl_ctx* {
    if (err && errlen) snprintf(err, errlen, "%s", m.c_str());
    g_api_err = m;
    return nullptr;
  };
  if (!cfg_in) return bad("gpu: null config");
  rl_config cfg = *cfg_in;
  const uint32_t n = cfg.n_shards ? cfg.n_shards : 1;
  if (n > MAX_LOCAL_SHARDS) return bad("gpu: n_shards must be at most 16");
  rl_ctx* c = new rl_ctx();
  if (n == 1) {
    cfg.n_shards = 1;
    c->e[0] = eng_create(&cfg, err, errlen);
    if (!c->e[0]) {
      delete c;
      return nullptr;
    }
    c->cfg = c->e[0]->cfg;
    return c;
  }
  // one key for every shard: the owner of a stem is a function of its hash
  while (!cfg.hash_seed) {
    std::random_device rd;
    cfg.hash_seed = ((uint64_t)rd() << 32) ^ rd();
  }
  if (!cfg.max_batch) cfg.max_batch = 1u << 20;
  if (!cfg.max_requests) cfg.max_requests = cfg.max_batch;
  if (!cfg.max_rules) cfg.max_rules = 65536;
  if (!cfg.max_stem_bytes) cfg.max_stem_bytes = 128u * cfg.max_batch;
  c->n = n;
  c->cfg = cfg;
  for (uint32_t j = 0; j < n; j++) {
    rl_config ec = cfg;
    ec.n_shards = 1;
    ec.device = cfg.shard_device[j];
    // the shards' router keeps stats per source slice (rule' = source x n_rules + rule):
    // an owner needs n x max_rules rows for batches of max_rules rules
    ec.max_rules = cfg.max_rules * n;
    c->e[j] = eng_create(&ec, err, errlen);
    if (!c->e[j]) {
      const std::string m = g_api_err = (err && errlen) ? std::string(err) : std::string("gpu: shard creation failed");
      rl_destroy(c);
      return bad(m);
    }
  }
  c->cfg = c->e[0]->cfg;
  c->cfg.n_shards = n;
  c->cfg.max_rules = cfg.max_rules;  // (what a batch may carry; the shards hold n x as many rows)
  for (uint32_t j = 0; j < MAX_LOCAL_SHARDS; j++) c->cfg.shard_device[j] = cfg.shard_device[j];
  // every pair of distinct shard devices talks directly over xGMI
  for (uint32_t i = 0; i < n; i++)
    for (uint32_t j = 0; j < n; j++) {
      const int di = cfg.shard_device[i], dj = cfg.shard_device[j];
      int can = 0;
      if (di == dj || hipDeviceCanAccessPeer(&can, di, dj) != hipSuccess || !can) continue;
      (void)hipSetDevice(di);
      const hipError_t e = hipDeviceEnablePeerAccess(dj, 0);
      (void)hipGetLastError();
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        rl_destroy(c);
        return bad("gpu: peer access between shard devices failed");
      }
    }
  // the shards' routers: one in-process loopback world
  uint8_t id[RL_COMM_ID_BYTES];
  std::string cerr;
  if (comm_loopback_id(id, &cerr)) {
    rl_destroy(c);
    return bad(cerr);
  }
  for (uint32_t j = 0; j < n; j++) {
    c->r[j] = comm_create(c->e[j], n, j, id, &cerr);
    if (!c->r[j]) {
      rl_destroy(c);
      return bad(cerr);
    }
  }
  c->pend.assign(comm_slots(), PendingStats{});
  for (uint32_t j = 0; j < n; j++) c->w[j].th = std::thread(worker_main, c, j);
  return c;
}

void rl_destroy(rl_ctx* c) {
  if (!c) return;
  if (c->comm) comm_destroy(c->comm);
  if (c->n > 1) {
    bool live = true;
    for (uint32_t j = 0; j < c->n; j++) live = live && c->w[j].th.joinable();
    if (live) (void)synchronize_all(c, false);  // (the last batches complete on every shard together)
    stop_shards(c);
    for (uint32_t j = 0; j < c->n; j++)
      if (c->r[j]) comm_destroy(c->r[j]);
    if (c->stats_ring) (void)hipHostFree(c->stats_ring);
  }
  for (uint32_t j = 0; j < c->n; j++)
    if (c->e[j]) eng_destroy(c->e[j]);
  delete c;
}

int rl_do_limit_async(rl_ctx* c, const rl_batch* in, rl_result* out, void* stream) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n == 1) return eng_do_limit_async(c->e[0], in, out, stream);
  if ((uintptr_t)in->stem_bytes & 3u) return fail(c, RL_E_INVALID, "gpu: stem_bytes must be 4-byte aligned");
  return shards_submit(c, in, out, false, (hipStream_t)stream);
}

// A host batch for the shards: the checks of the single-table path, on the
// whole batch (a batch is taken by every shard or by none).
int check_host_batch(rl_ctx* c, const rl_batch* in, const rl_result* out) {
  const uint32_t n = in->n, nq = in->n_requests;
  if (n && (!in->stem_off || !in->req_idx || !out->code || !out->limit_remaining))
    return fail(c, RL_E_INVALID, "gpu: null argument");
  const uint64_t nb = n ? in->stem_off[n] : 0;
  if (n > c->cfg.max_batch || nq > c->cfg.max_requests || in->n_rules > c->cfg.max_rules ||
      nb > c->cfg.max_stem_bytes)
    return fail(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_rules/max_stem_bytes");
  if (n && !nq) return fail(c, RL_E_INVALID, "gpu: descriptors without requests");
  return RL_OK;
}

int rl_do_limit_host_async(rl_ctx* c, const rl_batch* in, rl_result* out) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n == 1) return eng_do_limit_host_async(c->e[0], in, out);
  if (const int rc = check_host_batch(c, in, out)) return rc;
  return shards_submit(c, in, out, true, nullptr);
}

int rl_do_limit_compact_async(rl_ctx* c, const rl_batch_compact* in, rl_result* out) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->comm) return eng_fail(c->e[0], RL_E_INVALID, "gpu: compact batches are not routed (rl_do_limit_routed_async)");
  if (c->n == 1) return eng_do_limit_compact_async(c->e[0], in, out);
  // a multi-shard ctx: one request-aligned slice per shard, each over its own
  // device's link (rl_comm's stage_host_compact: the slice's parts, unpacked
  // on the device), then the shards' exchange as for rl_batch host batches
  // (the shards hold n x max_rules rows: check the ctx's own limit first)
  if (in->n_rules > c->cfg.max_rules) return fail(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_rules");
  if (const int rc = eng_compact_check(c->e[0], in, out)) return from_engine(c, c->e[0], rc);
  const uint32_t* first = reinterpret_cast<const uint32_t*>(in->buf + in->req_first);
  if (in->n_requests && (first[0] != 0 || first[in->n_requests] != in->n))
    return fail(c, RL_E_INVALID, "gpu: compact batch request layout is not a partition of the descriptors");
  rl_batch sizes{};
  sizes.n = in->n;
  sizes.n_requests = in->n_requests;
  sizes.n_rules = in->n_rules;
  return shards_submit(c, &sizes, out, true, nullptr, in);
}

int rl_batch_progress(rl_ctx* c, uint64_t* submitted, uint64_t* completed) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n > 1 || c->comm) return fail(c, RL_E_INVALID, "gpu: rl_batch_progress is for single-shard ctxs");
  return eng_batch_progress(c->e[0], submitted, completed);
}

int rl_do_limit_prefixed_async(rl_ctx* c, const rl_batch_prefixed* in, rl_result* out) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->comm) {
    // a ctx that joined a communicator (one process per GPU): the whole
    // prefix-shared batch is this rank's slice of the node batch, staged over
    // this GPU's link and unpacked on it, then routed like a device slice
    // (collective, as rl_do_limit_routed_async; out->stats = this rank's
    // requests' deltas). The Go batcher of every rank submits one batch per
    // tick, empty when idle.
    uint32_t tiles = 0;
    if (const int rc = eng_prefixed_check(c->e[0], in, out, &tiles)) {
      // a rejected slice still takes part in the exchange (no records) and
      // fails at rl_synchronize: no peer waits for it
      rl_batch none{};
      rl_result nout = *out;
      return comm_do_limit(c->comm, c->e[0], &none, &nout, nullptr, nullptr, rc);  // (RL_OK unless the router broke)
    }
    rl_batch sizes{};
    sizes.n = in->n;
    sizes.n_requests = in->n_requests;
    sizes.n_rules = in->n_rules;
    CommIO io;
    io.host = true;
    io.pb = in;
    io.t0 = 0;
    io.t1 = tiles;
    io.stats_host = in->n_rules ? (unsigned long long*)out->stats : nullptr;
    return comm_do_limit(c->comm, c->e[0], &sizes, out, nullptr, &io);
  }
  if (c->n == 1) return eng_do_limit_prefixed_async(c->e[0], in, out);
  // a multi-shard ctx: one slice of request tiles per shard, each over its own
  // device's link (rl_comm's stage_host_prefixed), then the shards' exchange
  uint32_t tiles = 0;
  if (in->n_rules > c->cfg.max_rules) return fail(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_rules");
  if (const int rc = eng_prefixed_check(c->e[0], in, out, &tiles)) return from_engine(c, c->e[0], rc);
  rl_batch sizes{};
  sizes.n = in->n;
  sizes.n_requests = in->n_requests;
  sizes.n_rules = in->n_rules;
  return shards_submit(c, &sizes, out, true, nullptr, nullptr, in);
}

int rl_do_limit(rl_ctx* c, const rl_batch* in, rl_result* out) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n == 1) return eng_do_limit(c->e[0], in, out);
  if (const int rc = check_host_batch(c, in, out)) return rc;
  const int rc = shards_submit(c, in, out, true, nullptr);
  const int sr = synchronize_all(c);
  return rc ? rc : sr;
}

int rl_comm_unique_id(uint8_t* id) {
  if (!id) return fail(nullptr, RL_E_INVALID, "gpu: null argument");
  std::string err;
  const int rc = comm_unique_id(id, &err);
  if (rc) return fail(nullptr, rc, err);
  return RL_OK;
}

int rl_comm_loopback_id(uint8_t* id) {
  if (!id) return fail(nullptr, RL_E_INVALID, "gpu: null argument");
  std::string err;
  const int rc = comm_loopback_id(id, &err);
  if (rc) return fail(nullptr, rc, err);
  return RL_OK;
}

int rl_comm_init(rl_ctx* c, uint32_t world, uint32_t rank, const uint8_t* id) {
  if (!c || !id) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n > 1) return fail(c, RL_E_INVALID, "gpu: rl_comm_init needs a single-shard ctx (one per process and GPU)");
  if (c->comm) return eng_fail(c->e[0], RL_E_INVALID, "gpu: ctx already joined a communicator");
  if (!c->cfg.hash_seed)
    return eng_fail(c->e[0], RL_E_INVALID, "gpu: a routed table needs an explicit hash_seed shared by every rank");
  std::string err;
  c->comm = comm_create(c->e[0], world, rank, id, &err);
  if (!c->comm) return eng_fail(c->e[0], RL_E_COMM, err);
  return RL_OK;
}

int rl_do_limit_routed_async(rl_ctx* c, const rl_batch* in, rl_result* out, void* stream) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (!c->comm) return fail(c, RL_E_INVALID, "gpu: ctx has no communicator (rl_comm_init)");
  return comm_do_limit(c->comm, c->e[0], in, out, (hipStream_t)stream);
}

int rl_synchronize(rl_ctx* c) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  return synchronize_all(c);
}

int rl_sweep(rl_ctx* c, int64_t now, uint64_t* n_evicted) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  int rc = settle(c);
  if (rc) return rc;
  if (c->comm) {  // (routed: one floor for the world, the least of the ranks' now)
    rc = from_engine(c, c->e[0], comm_sweep_floor(c->comm, c->e[0], now, &now));
    if (rc) return rc;
  }
  uint64_t total = 0;
  for (uint32_t j = 0; j < c->n; j++) {
    uint64_t ev = 0;
    rc = from_engine(c, c->e[j], eng_sweep(c->e[j], now, &ev));
    if (rc) return rc;
    total += ev;
  }
  if (n_evicted) *n_evicted = total;
  return RL_OK;
}

int rl_restore(rl_ctx* c, const rl_restore_batch* r) {
  if (!c || !r) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (const int src = settle(c)) return src;
  if (c->n == 1) return eng_restore(c->e[0], r);
  // route the SET records by owner on the host (restores are rare)
  const uint32_t N = c->n;
  std::vector<std::vector<uint32_t>> idx(N);
  for (uint32_t i = 0; i < r->n; i++) {
    const uint32_t a = r->stem_off[i], b = r->stem_off[i + 1];
    if (b < a) return fail(c, RL_E_INVALID, "gpu: restore stem offsets");
    idx[owner_of_host(hash_stem_host(c->e[0]->hk, r->stem_bytes + a, b - a), N)].push_back(i);
  }
  for (uint32_t j = 0; j < N; j++) {
    if (idx[j].empty()) continue;
    std::vector<uint8_t> stems, unit, lc;
    std::vector<uint32_t> off{0}, count;
    std::vector<int64_t> now;
    for (uint32_t i : idx[j]) {
      stems.insert(stems.end(), r->stem_bytes + r->stem_off[i], r->stem_bytes + r->stem_off[i + 1]);
      off.push_back((uint32_t)stems.size());
      unit.push_back(r->unit[i]);
      now.push_back(r->now[i]);
      count.push_back(r->count[i]);
      lc.push_back(r->lc ? r->lc[i] : 0);
    }
    rl_restore_batch sub{};
    sub.n = (uint32_t)idx[j].size();
    sub.stem_bytes = stems.data();
    sub.stem_off = off.data();
    sub.unit = unit.data();
    sub.now = now.data();
    sub.count = count.data();
    sub.lc = lc.data();
    const int rc = from_engine(c, c->e[j], eng_restore(c->e[j], &sub));
    if (rc) return rc;
  }
  return RL_OK;
}

int rl_table_info_get(rl_ctx* c, rl_table_info* info) {
  if (!c || !info) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (const int src = settle_local(c)) return src;
  rl_table_info sum{};
  for (uint32_t j = 0; j < c->n; j++) {
    rl_table_info x{};
    const int rc = from_engine(c, c->e[j], eng_table_info_get(c->e[j], &x));
    if (rc) return rc;
    sum.table_slots += x.table_slots;
    sum.live_slots += x.live_slots;
    sum.tombstones += x.tombstones;
    sum.arena_bytes_used += x.arena_bytes_used;
    sum.exact_stems += x.exact_stems;
    sum.decisions += x.decisions;
    sum.history_entries += x.history_entries;
    sum.history_appended += x.history_appended;
    sum.history_lost += x.history_lost;
    sum.history_slots += x.history_slots;
    sum.history_refused += x.history_refused;
    sum.batches = std::max(sum.batches, x.batches);
  }
  *info = sum;
  return RL_OK;
}

int rl_local_cache_info_get(rl_ctx* c, int64_t now, rl_local_cache_info* info) {
  if (!c || !info) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (const int src = settle_local(c)) return src;
  rl_local_cache_info sum{};
  for (uint32_t j = 0; j < c->n; j++) {
    rl_local_cache_info x{};
    const int rc = from_engine(c, c->e[j], eng_local_cache_info_get(c->e[j], now, &x));
    if (rc) return rc;
    sum.entry_count += x.entry_count;
    sum.lookup_count += x.lookup_count;
    sum.hit_count += x.hit_count;
    sum.miss_count += x.miss_count;
  }
  *info = sum;
  return RL_OK;
}

int rl_snapshot_size(rl_ctx* c, uint64_t* bytes) {
  if (!c || !bytes) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n == 1) return eng_snapshot_size(c->e[0], bytes);
  uint64_t total = 8 * (2 + c->n);  // magic, n, per-shard sizes
  for (uint32_t j = 0; j < c->n; j++) {
    uint64_t b = 0;
    const int rc = from_engine(c, c->e[j], eng_snapshot_size(c->e[j], &b));
    if (rc) return rc;
    total += b;
  }
  *bytes = total;
  return RL_OK;
}

int rl_snapshot_save(rl_ctx* c, void* host, uint64_t bytes) {
  if (!c || !host) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (const int src = settle(c)) return src;
  if (c->n == 1) return eng_snapshot_save(c->e[0], host, bytes);
  uint64_t* h = (uint64_t*)host;
  const uint64_t head = 8 * (2 + c->n);
  if (bytes < head) return fail(c, RL_E_CAPACITY, "gpu: snapshot buffer smaller than rl_snapshot_size");
  h[0] = MSNAP_MAGIC;
  h[1] = c->n;
  uint64_t pos = head;
  for (uint32_t j = 0; j < c->n; j++) {
    uint64_t b = 0;
    int rc = from_engine(c, c->e[j], eng_snapshot_size(c->e[j], &b));
    if (rc) return rc;
    if (pos + b > bytes) return fail(c, RL_E_CAPACITY, "gpu: snapshot buffer smaller than rl_snapshot_size");
    rc = from_engine(c, c->e[j], eng_snapshot_save(c->e[j], (uint8_t*)host + pos, b));
    if (rc) return rc;
    h[2 + j] = b;
    pos += b;
  }
  return RL_OK;
}

int rl_snapshot_load(rl_ctx* c, const void* host, uint64_t bytes) {
  if (!c || !host) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (const int src = settle(c)) return src;
  if (c->n == 1) return eng_snapshot_load(c->e[0], host, bytes);
  const uint64_t* h = (const uint64_t*)host;
  if (bytes < 16 || h[0] != MSNAP_MAGIC || h[1] != c->n || bytes < 8 * (2 + c->n))
    return fail(c, RL_E_INVALID, "gpu: not a snapshot of a ctx with this many shards");
  uint64_t pos = 8 * (2 + c->n);
  for (uint32_t j = 0; j < c->n; j++) {
    if (pos + h[2 + j] > bytes) return fail(c, RL_E_INVALID, "gpu: snapshot truncated");
    const int rc = from_engine(c, c->e[j], eng_snapshot_load(c->e[j], (const uint8_t*)host + pos, h[2 + j]));
    if (rc) return rc;
    pos += h[2 + j];
  }
  return RL_OK;
}

int rl_config_load(rl_ctx* c, const rl_config_tree* t) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  if (c->n > 1 && t && t->nodes)  // (the shards' own check allows their n x max_rules rows)
    for (uint32_t i = 0; i < t->n_nodes; i++)
      if (t->nodes[i].rule_id >= c->cfg.max_rules)
        return fail(c, RL_E_INVALID, "gpu: config node " + std::to_string(i) + ": rule id >= max_rules");
  for (uint32_t j = 0; j < c->n; j++) {
    const int rc = from_engine(c, c->e[j], eng_config_load(c->e[j], t));
    if (rc) return rc;
  }
  return RL_OK;
}

int rl_do_limit_requests(rl_ctx* c, const rl_request_batch* in, rl_request_result* out) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  if (c->comm) return fail(c, RL_E_INVALID, "gpu: rl_do_limit_requests is not routed (rl_do_limit_routed_async)");
  if (c->n == 1) return eng_do_limit_requests(c->e[0], in, out);
  // a multi-shard ctx: the config match on shard 0's GPU, the matched batch
  // through the shards as a device batch (shard 0 partitions it, every owner
  // answers its keys), then the expansion to the request layout on shard 0
  int rc = synchronize_all(c);  // (earlier batches first: the call is synchronous)
  if (rc) return rc;
  struct Run {
    rl_ctx* c;
    bool failed;
  } u{c, false};
  auto run = [](void* p, const rl_batch* din, rl_result* dout, hipStream_t st) -> int {
    Run& r = *static_cast<Run*>(p);
    const int sr = shards_submit(r.c, din, dout, false, st);
    const int yr = synchronize_all(r.c);
    r.failed = sr || yr;
    return sr ? sr : yr;
  };
  rc = eng_do_limit_requests(c->e[0], in, out, run, &u);
  return u.failed ? rc : from_engine(c, c->e[0], rc);
}

// Diagnostics, profiling and the per-rank routing halves act on shard 0.
int rl_table_info_shard(rl_ctx* c, uint32_t shard, rl_table_info* info) {
  if (!c || !info || shard >= c->n) return fail(c, RL_E_INVALID, "gpu: bad shard");
  return from_engine(c, c->e[shard], eng_table_info_get(c->e[shard], info));
}

int rl_debug_keys(rl_ctx* c, const rl_batch* in, uint8_t* out_bytes, uint32_t* out_off, uint32_t out_cap) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  return from_engine(c, c->e[0], eng_debug_keys(c->e[0], in, out_bytes, out_off, out_cap));
}

int rl_debug_log_tear(rl_ctx* c, const rl_log_tear* arm, rl_log_tear* out) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  return from_engine(c, c->e[0], eng_debug_log_tear(c->e[0], arm, out));
}

int rl_debug_decide(rl_ctx* c, uint32_t n, const uint32_t* before, const uint32_t* after, const uint8_t* lc_hit,
                    const uint32_t* hits, const uint32_t* limit, const uint8_t* unit, const uint8_t* flags,
                    const int64_t* now, uint8_t* code, uint32_t* remaining, uint32_t* reset_s,
                    uint64_t* stat_deltas, uint8_t* lc_set) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  return from_engine(c, c->e[0], eng_debug_decide(c->e[0], n, before, after, lc_hit, hits, limit, unit, flags, now,
                                                   code, remaining, reset_s, stat_deltas, lc_set));
}

int rl_profile(rl_ctx* c, int enable) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  for (uint32_t j = 0; j < c->n; j++) {
    const int rc = from_engine(c, c->e[j], eng_profile(c->e[j], enable));
    if (rc) return rc;
  }
  return RL_OK;
}

int rl_profile_read(rl_ctx* c, double* ms, uint32_t n, uint64_t* batches) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  return from_engine(c, c->e[0], eng_profile_read(c->e[0], ms, n, batches));
}

int rl_route_pack(rl_ctx* c, const rl_batch* in, uint32_t n_shards, uint32_t src_rank, void* send_rec,
                  uint8_t* send_stem, uint32_t* perm, uint64_t* counts, void* stream) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  if (c->n > 1) return fail(c, RL_E_INVALID, "gpu: per-rank routing needs a single-shard ctx");
  return eng_route_pack(c->e[0], in, n_shards, src_rank, send_rec, send_stem, perm, counts, stream);
}

int rl_route_do_limit(rl_ctx* c, uint32_t n, const void* recv_rec, const uint8_t* recv_stem, uint64_t recv_stem_bytes,
                      const uint64_t* src_stem_base, uint32_t n_shards, uint32_t n_rules, uint32_t rule_stride,
                      uint64_t* ret, uint64_t* stats, int isolate, void* stream) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  if (c->n > 1) return fail(c, RL_E_INVALID, "gpu: per-rank routing needs a single-shard ctx");
  return eng_route_do_limit(c->e[0], n, recv_rec, recv_stem, recv_stem_bytes, src_stem_base, n_shards, n_rules,
                            rule_stride, ret, stats, isolate, stream);
}

int rl_route_scatter(rl_ctx* c, uint32_t n, const uint32_t* perm, const uint64_t* ret, rl_result* out, void* stream) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  if (c->n > 1) return fail(c, RL_E_INVALID, "gpu: per-rank routing needs a single-shard ctx");
  return eng_route_scatter(c->e[0], n, perm, ret, out, stream);
}

void* rl_alloc_host(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
  return p;
}

void rl_free_host(void* p) {
  if (p) (void)hipHostFree(p);
}

}  // extern "C"
