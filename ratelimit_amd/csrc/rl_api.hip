// rl_api.hip — the extern "C" boundary of libratelimit_hip.so
// (include/ratelimit_hip.h).
//
// A ctx holds one engine per table shard (rl_engine.h: HBM table, pipeline
// buffers, streams). With one shard every entry point is the engine's own.
// With rl_config.n_shards > 1 the table is hash-sharded over the shards'
// devices inside this one process (the reference's single service process
// scaled out over a Redis cluster, src/redis/driver_impl.go:108-126; here the
// cgo adapter still drives one ctx), and every batch is routed:
//
//   shard 0's device (the source): partition the batch by owner (stem hash)
//     into wire records + stem bytes, on the forward stream;
//   host: read the per-owner counts (the one wait per batch: the partition
//     only, never the owners' pipelines);
//   forward stream: copy each owner's chunk to its device (xGMI peer copies;
//     a plain device copy when shards share a device);
//   each owner: the normal pipelined DoLimit over its chunk (eng_route_owner);
//   return stream: copy the packed results and stats deltas back, scatter the
//     results to arrival order, sum the stats.
//
// Batch t's partition and copies run while earlier batches' owner pipelines
// still hold the tables; RSLOTS batches may be in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/ratelimit_hip.h"
#include "rl_comm.h"
#include "rl_device.h"
#include "rl_engine.h"
#include "rl_kernels.h"

using namespace rl;

namespace {

constexpr uint32_t MAX_LOCAL_SHARDS = 16;
constexpr uint32_t RSLOTS = 3;

struct RouteSlot {
  Wire* send_rec = nullptr;              // dev0: wire records in owner order
  uint8_t* send_stem = nullptr;          // dev0: their stems
  uint32_t* perm = nullptr;              // dev0: record -> batch index
  unsigned long long* counts = nullptr;  // dev0: [2 x n] records / stem bytes per owner
  unsigned long long* back = nullptr;    // dev0: packed results, record order
  unsigned long long* stats_stage = nullptr;  // dev0: [n][max_rules x RL_NUM_STATS] owners' deltas
  Wire* recv_rec[MAX_LOCAL_SHARDS] = {};      // owner devices: received records
  uint8_t* recv_stem[MAX_LOCAL_SHARDS] = {};
  unsigned long long* ostats[MAX_LOCAL_SHARDS] = {};
  uint32_t k[MAX_LOCAL_SHARDS] = {};     // owner engine buffer of this slot's batch
  hipEvent_t packed = nullptr;           // forward stream: partition + counts copy done
  hipEvent_t done = nullptr;             // return stream: results and stats complete
};

}  // namespace

struct rl_ctx {
  rl_config cfg;
  uint32_t n = 1;
  Engine* e[MAX_LOCAL_SHARDS] = {};
  CommRouter* comm = nullptr;  // rl_comm_init: multi-process routing (single-shard ctx)
  std::string last_error;
  // router (n > 1), on shard 0's device
  int dev0 = 0;
  hipStream_t fwd = nullptr, ret = nullptr;
  hipEvent_t fwd_ready = nullptr, in_ready = nullptr;
  RouteSlot slot[RSLOTS];
  uint32_t next_slot = 0;
  unsigned long long* h_counts = nullptr;  // pinned [RSLOTS][2 x MAX_LOCAL_SHARDS]
  // staging for the host-buffer entry point (dev0)
  uint8_t* d_stem = nullptr;
  uint32_t *d_off = nullptr, *d_req = nullptr, *d_limit = nullptr, *d_hits = nullptr, *d_rule = nullptr;
  int64_t* d_now = nullptr;
  uint8_t *d_unit = nullptr, *d_flags = nullptr, *d_code = nullptr, *d_status = nullptr;
  uint32_t *d_rem = nullptr, *d_reset = nullptr;
  unsigned long long* d_stats = nullptr;
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

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

uint32_t owner_of_host(uint64_t h, uint32_t n) { return (uint32_t)(((uint64_t)(uint32_t)h * n) >> 32); }

void free_router(rl_ctx* c) {
  for (uint32_t s = 0; s < RSLOTS; s++) {
    RouteSlot& S = c->slot[s];
    void* dev0_bufs[] = {S.send_rec, S.send_stem, S.perm, S.counts, S.back, S.stats_stage};
    (void)hipSetDevice(c->dev0);
    for (void* p : dev0_bufs)
      if (p) (void)hipFree(p);
    for (uint32_t j = 0; j < c->n; j++) {
      (void)hipSetDevice(c->cfg.shard_device[j]);
      for (void* p : {(void*)S.recv_rec[j], (void*)S.recv_stem[j], (void*)S.ostats[j]})
        if (p) (void)hipFree(p);
    }
    (void)hipSetDevice(c->dev0);
    if (S.packed) (void)hipEventDestroy(S.packed);
    if (S.done) (void)hipEventDestroy(S.done);
  }
  (void)hipSetDevice(c->dev0);
  void* bufs[] = {c->d_stem, c->d_off, c->d_req, c->d_limit, c->d_hits, c->d_rule, c->d_now, c->d_unit,
                  c->d_flags, c->d_code, c->d_status, c->d_rem, c->d_reset, c->d_stats};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  if (c->h_counts) (void)hipHostFree(c->h_counts);
  for (hipEvent_t ev : {c->fwd_ready, c->in_ready})
    if (ev) (void)hipEventDestroy(ev);
  for (hipStream_t st : {c->fwd, c->ret})
    if (st) (void)hipStreamDestroy(st);
}

bool alloc_router(rl_ctx* c) {
  const rl_config& g = c->cfg;
  const uint32_t n = g.max_batch, sb = g.max_stem_bytes, m = g.max_rules * RL_NUM_STATS;
  // every pair of distinct shard devices talks directly over xGMI
  for (uint32_t i = 0; i < c->n; i++)
    for (uint32_t j = 0; j < c->n; j++) {
      const int di = g.shard_device[i], dj = g.shard_device[j];
      if (di == dj) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, di, dj) == hipSuccess && can) {
        (void)hipSetDevice(di);
        const hipError_t e = hipDeviceEnablePeerAccess(dj, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return false;
        (void)hipGetLastError();
      }
    }
  if (hipSetDevice(c->dev0) != hipSuccess) return false;
  bool ok = hipStreamCreateWithFlags(&c->fwd, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->ret, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&c->fwd_ready, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->in_ready, hipEventDisableTiming) == hipSuccess &&
            hipHostMalloc((void**)&c->h_counts, RSLOTS * 2 * MAX_LOCAL_SHARDS * 8) == hipSuccess;
  for (uint32_t s = 0; s < RSLOTS && ok; s++) {
    RouteSlot& S = c->slot[s];
    ok = dalloc(&S.send_rec, n) == hipSuccess && dalloc(&S.send_stem, (size_t)sb + 64) == hipSuccess &&
         dalloc(&S.perm, n) == hipSuccess && dalloc(&S.counts, 2 * RL_MAX_SHARDS) == hipSuccess &&
         dalloc(&S.back, n) == hipSuccess && dalloc(&S.stats_stage, (size_t)c->n * m) == hipSuccess &&
         hipEventCreateWithFlags(&S.packed, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&S.done, hipEventDisableTiming) == hipSuccess &&
         hipEventRecord(S.done, c->ret) == hipSuccess;
    for (uint32_t j = 0; j < c->n && ok; j++) {
      ok = hipSetDevice(g.shard_device[j]) == hipSuccess && dalloc(&S.recv_rec[j], n) == hipSuccess &&
           dalloc(&S.recv_stem[j], (size_t)sb + 64) == hipSuccess && dalloc(&S.ostats[j], m) == hipSuccess;
    }
    ok = ok && hipSetDevice(c->dev0) == hipSuccess;
  }
  ok = ok && dalloc(&c->d_stem, (size_t)sb + 64) == hipSuccess && dalloc(&c->d_off, (size_t)n + 1) == hipSuccess &&
       dalloc(&c->d_req, n) == hipSuccess && dalloc(&c->d_limit, n) == hipSuccess &&
       dalloc(&c->d_hits, n) == hipSuccess && dalloc(&c->d_rule, n) == hipSuccess &&
       dalloc(&c->d_now, g.max_requests) == hipSuccess && dalloc(&c->d_unit, n) == hipSuccess &&
       dalloc(&c->d_flags, n) == hipSuccess && dalloc(&c->d_code, n) == hipSuccess &&
       dalloc(&c->d_status, n) == hipSuccess && dalloc(&c->d_rem, n) == hipSuccess &&
       dalloc(&c->d_reset, n) == hipSuccess && dalloc(&c->d_stats, m) == hipSuccess;
  ok = ok && hipStreamSynchronize(c->ret) == hipSuccess;
  return ok;
}

// One routed batch (device arrays on dev0; see the file comment).
int routed_async(rl_ctx* c, const rl_batch* in, rl_result* out, hipStream_t caller) {
  const uint32_t n = in->n, N = c->n;
  if (n > c->cfg.max_batch || in->n_requests > c->cfg.max_requests || in->n_rules > c->cfg.max_rules)
    return fail(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_rules");
  const uint32_t s = c->next_slot;
  c->next_slot = (s + 1) % RSLOTS;
  RouteSlot& S = c->slot[s];
  Engine* e0 = c->e[0];
  API_HIP(c, hipSetDevice(c->dev0));
  API_HIP(c, hipStreamWaitEvent(c->fwd, S.done, 0));  // the slot's previous batch is complete
  if (caller && hipStreamQuery(caller) == hipErrorNotReady) {  // the inputs' producer (still running)
    API_HIP(c, hipEventRecord(c->in_ready, caller));
    API_HIP(c, hipStreamWaitEvent(c->fwd, c->in_ready, 0));
  }
  int rc = eng_route_pack(e0, in, N, 0, S.send_rec, S.send_stem, S.perm, (uint64_t*)S.counts, c->fwd);
  if (rc) return from_engine(c, e0, rc);
  unsigned long long* hc = c->h_counts + (size_t)s * 2 * MAX_LOCAL_SHARDS;
  API_HIP(c, hipMemcpyAsync(hc, S.counts, 2ull * N * 8, hipMemcpyDeviceToHost, c->fwd));
  API_HIP(c, hipEventRecord(S.packed, c->fwd));
  API_HIP(c, hipEventSynchronize(S.packed));  // the one host wait: this batch's partition
  uint64_t roff[MAX_LOCAL_SHARDS], soff[MAX_LOCAL_SHARDS], acc_r = 0, acc_s = 0;
  for (uint32_t j = 0; j < N; j++) {
    roff[j] = acc_r;
    soff[j] = acc_s;
    acc_r += hc[2 * j];
    acc_s += hc[2 * j + 1];
  }
  if (acc_r != (n ? n : 0) && acc_r != 0) return fail(c, RL_E_INTERNAL, "gpu: routing counts do not add up");
  for (uint32_t j = 0; j < N; j++) {
    const int dj = c->cfg.shard_device[j];
    if (hc[2 * j])
      API_HIP(c, hipMemcpyPeerAsync(S.recv_rec[j], dj, S.send_rec + roff[j], c->dev0, hc[2 * j] * sizeof(Wire),
                                    c->fwd));
    if (hc[2 * j + 1])
      API_HIP(c, hipMemcpyPeerAsync(S.recv_stem[j], dj, S.send_stem + soff[j], c->dev0, hc[2 * j + 1], c->fwd));
  }
  API_HIP(c, hipEventRecord(c->fwd_ready, c->fwd));
  const int isolate = out->status ? 1 : 0;
  const uint64_t zero = 0;
  for (uint32_t j = 0; j < N; j++) {
    rc = eng_route_owner(c->e[j], (uint32_t)hc[2 * j], S.recv_rec[j], S.recv_stem[j], hc[2 * j + 1], &zero, 1,
                         in->n_rules, 0, S.ostats[j], isolate, c->fwd_ready, &S.k[j]);
    if (rc) return from_engine(c, c->e[j], rc);
  }
  API_HIP(c, hipSetDevice(c->dev0));
  const uint32_t m = in->n_rules * RL_NUM_STATS;
  for (uint32_t j = 0; j < N; j++) {
    Engine* ej = c->e[j];
    const uint32_t k = S.k[j];
    const int dj = c->cfg.shard_device[j];
    API_HIP(c, hipStreamWaitEvent(c->ret, ej->b_done[k], 0));
    if (hc[2 * j])
      API_HIP(c, hipMemcpyPeerAsync(S.back + roff[j], c->dev0, ej->s[k].res, dj, hc[2 * j] * 8, c->ret));
    if (m) API_HIP(c, hipMemcpyPeerAsync(S.stats_stage + (size_t)j * m, c->dev0, S.ostats[j], dj, (size_t)m * 8, c->ret));
    API_HIP(c, hipEventRecord(ej->consumed[k], c->ret));
  }
  OutDev o{out->code, out->limit_remaining, out->reset_s, (unsigned long long*)out->stats, out->status};
  launch_route_scatter(S.perm, S.back, n, o, c->ret);
  if (m && out->stats) launch_stats_sum(S.stats_stage, N, m, (unsigned long long*)out->stats, c->ret);
  API_HIP(c, hipGetLastError());
  API_HIP(c, hipEventRecord(S.done, c->ret));  // (outputs: read after rl_synchronize)
  return RL_OK;
}

int synchronize_all(rl_ctx* c) {
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
  if (c->n > 1) {
    API_HIP(c, hipSetDevice(c->dev0));
    API_HIP(c, hipStreamSynchronize(c->fwd));
    API_HIP(c, hipStreamSynchronize(c->ret));
  }
  int first = RL_OK;
  for (uint32_t j = 0; j < c->n; j++) {
    const int rc = from_engine(c, c->e[j], eng_synchronize(c->e[j]));
    if (rc && !first) first = rc;
  }
  if (first && c->n > 1) {  // keep the first failing shard's message
    for (uint32_t j = 0; j < c->n; j++)
      if (*eng_last_error(c->e[j])) {
        c->last_error = eng_last_error(c->e[j]);
        break;
      }
  }
  return first;
}

constexpr uint64_t MSNAP_MAGIC = 0x31304853414e534cull;  // "LSNASH01": one image per shard

// Calls that read or change the table order after every submitted batch: on a
// multi-shard or routed ctx the batches still in the router first complete
// (on a routed ctx this makes the call collective, like rl_synchronize).
int settle(rl_ctx* c) { return (c->comm || c->n > 1) ? synchronize_all(c) : RL_OK; }

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
  c->dev0 = cfg.shard_device[0];
  for (uint32_t j = 0; j < n; j++) {
    rl_config ec = cfg;
    ec.n_shards = 1;
    ec.device = cfg.shard_device[j];
    c->e[j] = eng_create(&ec, err, errlen);
    if (!c->e[j]) {
      const std::string m = g_api_err = (err && errlen) ? std::string(err) : std::string("gpu: shard creation failed");
      rl_destroy(c);
      return bad(m);
    }
  }
  c->cfg = c->e[0]->cfg;
  c->cfg.n_shards = n;
  for (uint32_t j = 0; j < MAX_LOCAL_SHARDS; j++) c->cfg.shard_device[j] = cfg.shard_device[j];
  if (!alloc_router(c)) {
    rl_destroy(c);
    return bad("gpu: router allocation failed (peer access or device memory)");
  }
  return c;
}

void rl_destroy(rl_ctx* c) {
  if (!c) return;
  if (c->comm) comm_destroy(c->comm);
  if (c->n > 1) {
    (void)hipSetDevice(c->dev0);
    if (c->fwd) (void)hipStreamSynchronize(c->fwd);
    if (c->ret) (void)hipStreamSynchronize(c->ret);
    free_router(c);
  }
  for (uint32_t j = 0; j < c->n; j++)
    if (c->e[j]) eng_destroy(c->e[j]);
  delete c;
}

int rl_do_limit_async(rl_ctx* c, const rl_batch* in, rl_result* out, void* stream) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n == 1) return eng_do_limit_async(c->e[0], in, out, stream);
  if ((uintptr_t)in->stem_bytes & 3u) return fail(c, RL_E_INVALID, "gpu: stem_bytes must be 4-byte aligned");
  return routed_async(c, in, out, (hipStream_t)stream);
}

int rl_do_limit_host_async(rl_ctx* c, const rl_batch* in, rl_result* out) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n > 1) return fail(c, RL_E_INVALID, "gpu: rl_do_limit_host_async runs on a single-shard ctx");
  return eng_do_limit_host_async(c->e[0], in, out);
}

int rl_do_limit(rl_ctx* c, const rl_batch* in, rl_result* out) {
  if (!c || !in || !out) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (c->n == 1) return eng_do_limit(c->e[0], in, out);
  const uint32_t n = in->n, nq = in->n_requests;
  const uint64_t nb = n ? in->stem_off[n] : 0;
  if (n > c->cfg.max_batch || nq > c->cfg.max_requests || in->n_rules > c->cfg.max_rules ||
      nb > c->cfg.max_stem_bytes)
    return fail(c, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_rules/max_stem_bytes");
  if (n && !nq) return fail(c, RL_E_INVALID, "gpu: descriptors without requests");
  API_HIP(c, hipSetDevice(c->dev0));
  hipStream_t st = c->fwd;
  API_HIP(c, hipStreamWaitEvent(st, c->slot[(c->next_slot + RSLOTS - 1) % RSLOTS].done, 0));  // staging is free
  if (nb) API_HIP(c, hipMemcpyAsync(c->d_stem, in->stem_bytes, nb, hipMemcpyHostToDevice, st));
  API_HIP(c, hipMemcpyAsync(c->d_off, in->stem_off, (n + 1) * 4ull, hipMemcpyHostToDevice, st));
  if (nq) API_HIP(c, hipMemcpyAsync(c->d_now, in->now, nq * 8ull, hipMemcpyHostToDevice, st));
  if (n) {
    API_HIP(c, hipMemcpyAsync(c->d_req, in->req_idx, n * 4ull, hipMemcpyHostToDevice, st));
    API_HIP(c, hipMemcpyAsync(c->d_unit, in->unit, n, hipMemcpyHostToDevice, st));
    API_HIP(c, hipMemcpyAsync(c->d_flags, in->flags, n, hipMemcpyHostToDevice, st));
    API_HIP(c, hipMemcpyAsync(c->d_limit, in->limit, n * 4ull, hipMemcpyHostToDevice, st));
    API_HIP(c, hipMemcpyAsync(c->d_hits, in->hits, n * 4ull, hipMemcpyHostToDevice, st));
    API_HIP(c, hipMemcpyAsync(c->d_rule, in->rule_id, n * 4ull, hipMemcpyHostToDevice, st));
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
  rl_result r{c->d_code, c->d_rem, c->d_reset, (uint64_t*)c->d_stats, out->status ? c->d_status : nullptr};
  int rc = routed_async(c, &d, &r, nullptr);
  if (rc) return rc;
  hipStream_t rs = c->ret;
  if (n) {
    API_HIP(c, hipMemcpyAsync(out->code, c->d_code, n, hipMemcpyDeviceToHost, rs));
    API_HIP(c, hipMemcpyAsync(out->limit_remaining, c->d_rem, n * 4ull, hipMemcpyDeviceToHost, rs));
    API_HIP(c, hipMemcpyAsync(out->reset_s, c->d_reset, n * 4ull, hipMemcpyDeviceToHost, rs));
    if (out->status) API_HIP(c, hipMemcpyAsync(out->status, c->d_status, n, hipMemcpyDeviceToHost, rs));
  }
  if (in->n_rules && out->stats)
    API_HIP(c, hipMemcpyAsync(out->stats, c->d_stats, (size_t)in->n_rules * RL_NUM_STATS * 8, hipMemcpyDeviceToHost,
                              rs));
  return synchronize_all(c);
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
  if (const int src = settle(c)) return src;
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
    sum.batches = std::max(sum.batches, x.batches);
  }
  *info = sum;
  return RL_OK;
}

int rl_local_cache_info_get(rl_ctx* c, int64_t now, rl_local_cache_info* info) {
  if (!c || !info) return fail(c, RL_E_INVALID, "gpu: null argument");
  if (const int src = settle(c)) return src;
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
  for (uint32_t j = 0; j < c->n; j++) {
    const int rc = from_engine(c, c->e[j], eng_config_load(c->e[j], t));
    if (rc) return rc;
  }
  return RL_OK;
}

int rl_do_limit_requests(rl_ctx* c, const rl_request_batch* in, rl_request_result* out) {
  if (!c) return fail(c, RL_E_INVALID, "gpu: null ctx");
  if (c->n > 1) return fail(c, RL_E_INVALID, "gpu: rl_do_limit_requests runs on a single-shard ctx");
  return eng_do_limit_requests(c->e[0], in, out);
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
