// rl_comm.hip — the multi-process routed DoLimit step over RCCL, driven
// entirely by the library.
//
// One process per GPU, one single-shard engine per process; every rank calls
// comm_do_limit once per node batch with its own slice. Per batch:
//
//   cnt stream:  rl_route_pack partition of the slice by owner (stem hash);
//                counts exchange (2 u64 per peer, grouped send/recv);
//   host:        read the counts (the one wait per batch, one call later);
//   fwd stream:  records + stem bytes exchange (one grouped send/recv over
//                xGMI: each peer pair uses its own link);
//   engine:      the owner pipeline over the received chunks, concatenated in
//                source-rank order (= global arrival order), in parts of at
//                most max_batch records; stats attributed per source rank;
//   ret stream:  packed results (a failed owner batch returns its status for
//                every record) and each source's stats block go back (grouped
//                send/recv); scatter to arrival order, sum the stats blocks.
//
// A call enqueues its batch's partition and counts exchange and then
// completes the PREVIOUS batch (whose counts have had a whole call to arrive):
// the host never waits for work it just issued, batch t's partition runs
// beside batch t-1's owner pipeline, and rl_synchronize completes the last
// one. Three communicators, one per direction of traffic (counts, records,
// results), each on its own stream, so that no exchange waits in RCCL's
// per-communicator order behind another kind. RSLOTS batches may be in
// flight. RCCL is loaded with dlopen, preferring an instance already in the
// process (torch's, which shares the HIP runtime this library binds to), so
// the library loads and runs single-GPU without RCCL present.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rl_comm.h"
#include "rl_kernels.h"

namespace rl {

namespace {

// batches a router keeps in flight: a slot's partition waits for the batch
// RSLOTS back to complete (its buffers are reused). 6 rather than 3 so that
// this wait never binds (routed N=1 3.33-3.36 vs 3.22-3.30 G); the host's
// remaining ~150 us wait per step for the counts is the partition waiting for
// GPU capacity beside the owner pipelines (RL_DEBUG_ROUTE_TIMING).
constexpr uint32_t RSLOTS = 6;

struct Rccl {
  bool ok = false;
  std::string err;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclCommSplit) split = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGroupStart) gstart = nullptr;
  decltype(&ncclGroupEnd) gend = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) estr = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, if loaded
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.err = std::string("gpu: RCCL not loadable: ") + (e ? e : "?");
      return;
    }
    r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
    r.init = (decltype(r.init))dlsym(h, "ncclCommInitRank");
    r.split = (decltype(r.split))dlsym(h, "ncclCommSplit");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.gstart = (decltype(r.gstart))dlsym(h, "ncclGroupStart");
    r.gend = (decltype(r.gend))dlsym(h, "ncclGroupEnd");
    r.send = (decltype(r.send))dlsym(h, "ncclSend");
    r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
    r.estr = (decltype(r.estr))dlsym(h, "ncclGetErrorString");
    r.ok = r.get_id && r.init && r.split && r.destroy && r.gstart && r.gend && r.send && r.recv && r.estr;
    if (!r.ok) r.err = "gpu: RCCL library lacks a required symbol";
  });
  return r;
}

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

}  // namespace

struct CommSlot {
  Wire* send_rec = nullptr;                // partition of this rank's slice, owner order
  uint8_t* send_stem = nullptr;
  uint32_t* perm = nullptr;                // record -> slice index
  unsigned long long* cnt = nullptr;       // [4 x world]: sent (records, bytes) per peer, then received
  Wire* recv_rec = nullptr;                // chunks of every source, rank order
  uint8_t* recv_stem = nullptr;
  unsigned long long* ret_send = nullptr;  // packed results of the received records
  uint64_t cap_rec = 0, cap_stem = 0;
  unsigned long long* back = nullptr;      // this rank's results, record order
  unsigned long long* ostats = nullptr;    // [cap_parts][world x m_max]: owner deltas per source
  uint32_t cap_parts = 0;
  unsigned long long* stats_stage = nullptr;  // [world x m_max]: the owners' blocks for this rank
  hipEvent_t packed = nullptr, sent = nullptr, done = nullptr;
  std::vector<uint32_t> k;                 // engine buffer of each owner part
  std::vector<uint64_t> cut;               // owner part boundaries (record indices)
  // the batch between its two halves
  rl_result out{};
  uint32_t n = 0, n_rules = 0;
};

struct CommRouter {
  ncclComm_t comm_c = nullptr, comm_f = nullptr, comm_r = nullptr;  // counts, records, results
  uint32_t world = 1, rank = 0;
  int dev = 0;
  uint32_t m_max = 0;
  uint32_t part_max = 0;  // owner part size: max_batch (test knob: RL_DEBUG_OWNER_PART)
  bool alias = false;     // world 1: the owner reads the partition in place, no exchange
  hipStream_t cs = nullptr, fwd = nullptr, ret = nullptr;
  hipEvent_t in_ready = nullptr;
  CommSlot slot[RSLOTS];
  uint32_t next = 0;
  int pending = -1;                     // slot whose second half is still to run
  unsigned long long* h_cnt = nullptr;  // pinned [RSLOTS][4 x world]
  std::vector<uint64_t> base;           // received chunk offsets in recv_stem (host)
  std::vector<uint64_t> so_r, so_b, ro_r;  // per-peer send / receive offsets (host)
  // host seconds per phase (printed at destroy when RL_DEBUG_ROUTE_TIMING is set)
  bool timing = false;
  double t_first = 0, t_wait_counts = 0, t_owner = 0, t_second = 0;
  uint64_t n_steps = 0;
};

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

namespace {

#define CHK_HIP(e, expr)                                                                         \
  do {                                                                                           \
    hipError_t _h = (expr);                                                                      \
    if (_h != hipSuccess) return eng_fail((e), RL_E_HIP, std::string("gpu: ") + #expr + ": " + hipGetErrorString(_h)); \
  } while (0)

#define CHK_NCCL(e, expr)                                                                        \
  do {                                                                                           \
    ncclResult_t _r = (expr);                                                                    \
    if (_r != ncclSuccess) return eng_fail((e), RL_E_COMM, std::string("gpu: ") + #expr + ": " + rccl().estr(_r)); \
  } while (0)

void free_slot(CommSlot& S) {
  void* bufs[] = {S.send_rec, S.send_stem, S.perm, S.cnt, S.recv_rec, S.recv_stem, S.ret_send, S.back, S.ostats,
                  S.stats_stage};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  for (hipEvent_t ev : {S.packed, S.sent, S.done})
    if (ev) (void)hipEventDestroy(ev);
  S = CommSlot{};
}

// Receive-side buffers of slot S hold at least n_rec records / n_stem bytes /
// parts x world x m_max stats (grown on demand: the slot's last batch is
// complete once S.done has fired).
hipError_t grow(CommRouter* r, CommSlot& S, uint64_t n_rec, uint64_t n_stem, uint32_t parts) {
  if (n_rec <= S.cap_rec && n_stem <= S.cap_stem && parts <= S.cap_parts) return hipSuccess;
  hipError_t e = hipEventSynchronize(S.done);
  if (e != hipSuccess) return e;
  if (n_rec > S.cap_rec) {
    const uint64_t c = std::max<uint64_t>(n_rec, S.cap_rec + S.cap_rec / 2);
    (void)hipFree(S.recv_rec);
    (void)hipFree(S.ret_send);
    S.recv_rec = nullptr;
    S.ret_send = nullptr;
    S.cap_rec = 0;
    if ((e = dalloc(&S.recv_rec, c)) != hipSuccess || (e = dalloc(&S.ret_send, c)) != hipSuccess) return e;
    S.cap_rec = c;
  }
  if (n_stem > S.cap_stem) {
    const uint64_t c = std::max<uint64_t>(n_stem, S.cap_stem + S.cap_stem / 2);
    (void)hipFree(S.recv_stem);
    S.recv_stem = nullptr;
    S.cap_stem = 0;
    if ((e = dalloc(&S.recv_stem, c + 64)) != hipSuccess) return e;
    S.cap_stem = c;
  }
  if (parts > S.cap_parts) {
    (void)hipFree(S.ostats);
    S.ostats = nullptr;
    S.cap_parts = 0;
    if ((e = dalloc(&S.ostats, (size_t)parts * r->world * r->m_max)) != hipSuccess) return e;
    S.cap_parts = parts;
  }
  return hipSuccess;
}

// First half of a batch (slot s): partition, counts exchange, counts to the
// host. (The next call's second half waits on the host for this partition:
// from then on the inputs may be reused.)
int first_half(CommRouter* r, Engine* e, CommSlot& S, uint32_t s, const rl_batch* in, hipStream_t caller) {
  Rccl& R = rccl();
  const uint32_t W = r->world, me = r->rank;
  CHK_HIP(e, hipStreamWaitEvent(r->cs, S.done, 0));  // the slot's previous batch is complete
  if (caller && hipStreamQuery(caller) == hipErrorNotReady) {  // the inputs' producer (still running)
    CHK_HIP(e, hipEventRecord(r->in_ready, caller));
    CHK_HIP(e, hipStreamWaitEvent(r->cs, r->in_ready, 0));
  }
  // a malformed slice sends nothing (zero counts) and fails this rank's batch
  // at rl_synchronize
  const int rc = eng_route_pack(e, in, W, me, S.send_rec, S.send_stem, S.perm, (uint64_t*)S.cnt, r->cs);
  if (rc) return rc;
  if (!r->alias) {
    CHK_NCCL(e, R.gstart());
    for (uint32_t p = 0; p < W; p++) {
      if (p == me) continue;
      CHK_NCCL(e, R.send(S.cnt + 2 * p, 2, ncclUint64, (int)p, r->comm_c, r->cs));
      CHK_NCCL(e, R.recv(S.cnt + 2 * W + 2 * p, 2, ncclUint64, (int)p, r->comm_c, r->cs));
    }
    CHK_NCCL(e, R.gend());
  }
  CHK_HIP(e, hipMemcpyAsync(r->h_cnt + (size_t)s * 4 * W, S.cnt, 4ull * W * 8, hipMemcpyDeviceToHost, r->cs));
  CHK_HIP(e, hipEventRecord(S.packed, r->cs));
  return RL_OK;
}

// Second half (slot s): records and stems to their owners, the owner
// pipeline, results and per-source stats back, scatter.
int second_half(CommRouter* r, Engine* e, CommSlot& S, uint32_t s) {
  Rccl& R = rccl();
  const uint32_t W = r->world, me = r->rank, n = S.n, nr = S.n_rules;
  const uint32_t m = nr * RL_NUM_STATS;
  unsigned long long* h = r->h_cnt + (size_t)s * 4 * W;
  const double t0 = now_s();
  CHK_HIP(e, hipEventSynchronize(S.packed));  // (issued one call ago)
  const double t1 = now_s();
  r->t_wait_counts += t1 - t0;
  h[2 * W + 2 * me] = h[2 * me];  // (own chunk)
  h[2 * W + 2 * me + 1] = h[2 * me + 1];
  uint64_t n_send = 0, n_recv = 0, b_recv = 0;
  for (uint32_t p = 0; p < W; p++) {
    n_send += h[2 * p];
    r->base[p] = b_recv;
    n_recv += h[2 * W + 2 * p];
    b_recv += h[2 * W + 2 * p + 1];
  }
  if (n_send != n && n_send != 0) return eng_fail(e, RL_E_INTERNAL, "gpu: routing counts do not add up");
  const uint32_t mb = r->part_max;
  if (b_recv >= (1ull << 32)) return eng_fail(e, RL_E_CAPACITY, "gpu: more than 4 GiB of stems routed to one owner");
  // per-peer offsets: so_* into the send buffers, ro_* into the receive ones
  r->so_r.assign(W + 1, 0);
  r->so_b.assign(W + 1, 0);
  r->ro_r.assign(W + 1, 0);
  for (uint32_t p = 0; p < W; p++) {
    r->so_r[p + 1] = r->so_r[p] + h[2 * p];
    r->so_b[p + 1] = r->so_b[p] + h[2 * p + 1];
    r->ro_r[p + 1] = r->ro_r[p] + h[2 * W + 2 * p];
  }
  CHK_HIP(e, hipStreamWaitEvent(r->fwd, S.packed, 0));
  if (!r->alias) CHK_HIP(e, grow(r, S, n_recv, b_recv, 1));
  // (world 1: the partition is the received batch)
  const Wire* recv_rec = r->alias ? S.send_rec : S.recv_rec;
  const uint8_t* recv_stem = r->alias ? S.send_stem : S.recv_stem;
  if (!r->alias) {
    // records and stems to their owners; this rank's own chunk by device copy
    CHK_NCCL(e, R.gstart());
    for (uint32_t p = 0; p < W; p++) {
      const uint64_t sn = h[2 * p], sb = h[2 * p + 1], rn = h[2 * W + 2 * p], rb = h[2 * W + 2 * p + 1];
      if (p == me) continue;
      if (sn) CHK_NCCL(e, R.send(S.send_rec + r->so_r[p], sn * sizeof(Wire), ncclUint8, (int)p, r->comm_f, r->fwd));
      if (sb) CHK_NCCL(e, R.send(S.send_stem + r->so_b[p], sb, ncclUint8, (int)p, r->comm_f, r->fwd));
      if (rn) CHK_NCCL(e, R.recv(S.recv_rec + r->ro_r[p], rn * sizeof(Wire), ncclUint8, (int)p, r->comm_f, r->fwd));
      if (rb) CHK_NCCL(e, R.recv(S.recv_stem + r->base[p], rb, ncclUint8, (int)p, r->comm_f, r->fwd));
    }
    CHK_NCCL(e, R.gend());
    if (h[2 * me])
      CHK_HIP(e, hipMemcpyAsync(S.recv_rec + r->ro_r[me], S.send_rec + r->so_r[me], h[2 * me] * sizeof(Wire),
                                hipMemcpyDeviceToDevice, r->fwd));
    if (h[2 * me + 1])
      CHK_HIP(e, hipMemcpyAsync(S.recv_stem + r->base[me], S.send_stem + r->so_b[me], h[2 * me + 1],
                                hipMemcpyDeviceToDevice, r->fwd));
  }
  CHK_HIP(e, hipEventRecord(S.sent, r->fwd));
  // the owner pipeline, in parts of at most max_batch records. A part ends on
  // a request boundary (a request's descriptors check the local cache before
  // any of them sets it, fixed_cache_impl.go:50-66 then :100-109), so more
  // than max_batch received records (hash skew; rare) cost one host read of
  // the received labels.
  std::vector<uint64_t>& cut = S.cut;
  cut.assign(1, 0);
  if (n_recv > mb) {
    std::vector<uint32_t> lab(n_recv);
    CHK_HIP(e, hipStreamSynchronize(r->fwd));
    CHK_HIP(e, hipMemcpy2D(lab.data(), 4, recv_rec, sizeof(Wire), 4, n_recv, hipMemcpyDeviceToHost));
    uint64_t a = 0;
    while (n_recv - a > mb) {
      uint64_t b = a + mb;
      while (b > a + 1 && lab[b - 1] == lab[b]) b--;  // (labels of one request are adjacent)
      cut.push_back(b);
      a = b;
    }
  }
  cut.push_back(n_recv);
  const uint32_t parts = (uint32_t)cut.size() - 1;
  if (parts > S.cap_parts) CHK_HIP(e, grow(r, S, 0, 0, parts));
  unsigned long long* ret_send = r->alias ? S.back : S.ret_send;  // (world 1: results land in place)
  // world 1, one part: the scatter reads the owner batch's results directly
  const bool direct = r->alias && parts == 1;
  const int isolate = S.out.status ? 1 : 0;
  S.k.assign(parts, 0);
  const size_t blk = (size_t)W * m;  // one part's per-source stats
  const double t2 = now_s();
  for (uint32_t q = 0; q < parts; q++) {
    const uint64_t a = cut[q], b = cut[q + 1];
    const int rc = eng_route_owner(e, (uint32_t)(b - a), recv_rec + a, recv_stem, b_recv, r->base.data(), W, nr,
                                   nr, S.ostats + q * blk, isolate, S.sent, &S.k[q]);
    if (rc) return rc;
    // its packed results, before a later part can take the same engine buffer
    const uint32_t k = S.k[q];
    CHK_HIP(e, hipSetDevice(r->dev));
    CHK_HIP(e, hipStreamWaitEvent(r->ret, e->b_done[k], 0));
    if (direct) break;
    launch_route_ret(e->s[k].res, (uint32_t)(b - a), e->s[k].errb, ret_send + a, r->ret);
    CHK_HIP(e, hipEventRecord(e->consumed[k], r->ret));
  }
  const double t3 = now_s();
  r->t_owner += t3 - t2;
  // results and per-source stats back to their sources
  if (parts > 1 && m) launch_stats_sum(S.ostats, parts, (uint32_t)blk, S.ostats, r->ret);
  const unsigned long long* stats_in = S.ostats;  // (world 1: this rank's block is the owner's)
  if (!r->alias) {
    CHK_NCCL(e, R.gstart());
    for (uint32_t p = 0; p < W; p++) {
      const uint64_t sn = h[2 * p], rn = h[2 * W + 2 * p];
      if (p == me) continue;
      if (rn) CHK_NCCL(e, R.send(S.ret_send + r->ro_r[p], rn, ncclUint64, (int)p, r->comm_r, r->ret));
      if (sn) CHK_NCCL(e, R.recv(S.back + r->so_r[p], sn, ncclUint64, (int)p, r->comm_r, r->ret));
      if (m) {
        CHK_NCCL(e, R.send(S.ostats + (size_t)p * m, m, ncclUint64, (int)p, r->comm_r, r->ret));
        CHK_NCCL(e, R.recv(S.stats_stage + (size_t)p * m, m, ncclUint64, (int)p, r->comm_r, r->ret));
      }
    }
    CHK_NCCL(e, R.gend());
    if (h[2 * me])
      CHK_HIP(e, hipMemcpyAsync(S.back + r->so_r[me], S.ret_send + r->ro_r[me], h[2 * me] * 8,
                                hipMemcpyDeviceToDevice, r->ret));
    if (m)
      CHK_HIP(e, hipMemcpyAsync(S.stats_stage + (size_t)me * m, S.ostats + (size_t)me * m, (size_t)m * 8,
                                hipMemcpyDeviceToDevice, r->ret));
    stats_in = S.stats_stage;
  }
  const rl_result& out = S.out;
  OutDev o{out.code, out.limit_remaining, out.reset_s, (unsigned long long*)out.stats, out.status};
  uint32_t* src_err = isolate ? nullptr : e->errw + NBUF + 2;
  if (direct) {
    const uint32_t k = S.k[0];
    launch_route_scatter(S.perm, e->s[k].res, n, o, r->ret, src_err, e->s[k].errb);
    CHK_HIP(e, hipEventRecord(e->consumed[k], r->ret));
  } else {
    launch_route_scatter(S.perm, S.back, n, o, r->ret, src_err);
  }
  if (m && out.stats) launch_stats_sum(stats_in, W, m, (unsigned long long*)out.stats, r->ret);
  CHK_HIP(e, hipGetLastError());
  CHK_HIP(e, hipEventRecord(S.done, r->ret));  // (outputs: read after rl_synchronize)
  r->t_second += now_s() - t1;
  r->n_steps++;
  return RL_OK;
}

}  // namespace

int comm_unique_id(uint8_t* id, std::string* err) {
  Rccl& R = rccl();
  if (!R.ok) {
    *err = R.err;
    return RL_E_COMM;
  }
  static_assert(sizeof(ncclUniqueId) == RL_COMM_ID_BYTES, "RL_COMM_ID_BYTES");
  ncclUniqueId u;
  const ncclResult_t rc = R.get_id(&u);
  if (rc != ncclSuccess) {
    *err = std::string("gpu: ncclGetUniqueId: ") + R.estr(rc);
    return RL_E_COMM;
  }
  memcpy(id, &u, sizeof(u));
  return RL_OK;
}

CommRouter* comm_create(Engine* e, uint32_t world, uint32_t rank, const uint8_t* id, std::string* err) {
  Rccl& R = rccl();
  if (!R.ok) {
    *err = R.err;
    return nullptr;
  }
  if (world < 1 || world > RL_MAX_SHARDS || rank >= world) {
    *err = "gpu: world must be 1..256 and rank < world";
    return nullptr;
  }
  CommRouter* r = new CommRouter();
  r->world = world;
  r->rank = rank;
  r->dev = e->cfg.device;
  r->m_max = e->cfg.max_rules * RL_NUM_STATS;
  const rl_config& g = e->cfg;
  r->part_max = g.max_batch;
  r->alias = world == 1 && !getenv("RL_DEBUG_ROUTE_NOALIAS");
  r->timing = getenv("RL_DEBUG_ROUTE_TIMING") != nullptr;
  if (const char* pm = getenv("RL_DEBUG_OWNER_PART"))
    r->part_max = std::max<uint32_t>(1, std::min<uint32_t>(g.max_batch, (uint32_t)atoi(pm)));
  bool ok = hipSetDevice(r->dev) == hipSuccess;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  // one communicator per direction of traffic (collective: every rank splits alike)
  ncclResult_t nr = ok ? R.init(&r->comm_c, (int)world, u, (int)rank) : ncclSuccess;
  if (nr == ncclSuccess && ok) nr = R.split(r->comm_c, 0, (int)rank, &r->comm_f, nullptr);
  if (nr == ncclSuccess && ok) nr = R.split(r->comm_c, 0, (int)rank, &r->comm_r, nullptr);
  if (nr != ncclSuccess) {
    *err = std::string("gpu: RCCL communicator setup: ") + R.estr(nr);
    comm_destroy(r);
    return nullptr;
  }
  ok = ok && hipStreamCreateWithFlags(&r->cs, hipStreamNonBlocking) == hipSuccess &&
       hipStreamCreateWithFlags(&r->fwd, hipStreamNonBlocking) == hipSuccess &&
       hipStreamCreateWithFlags(&r->ret, hipStreamNonBlocking) == hipSuccess &&
       hipEventCreateWithFlags(&r->in_ready, hipEventDisableTiming) == hipSuccess &&
       hipHostMalloc((void**)&r->h_cnt, (size_t)RSLOTS * 4 * world * 8) == hipSuccess;
  for (uint32_t s = 0; s < RSLOTS && ok; s++) {
    CommSlot& S = r->slot[s];
    ok = dalloc(&S.send_rec, g.max_batch) == hipSuccess && dalloc(&S.send_stem, (size_t)g.max_stem_bytes + 64) == hipSuccess &&
         dalloc(&S.perm, g.max_batch) == hipSuccess && dalloc(&S.cnt, 4 * (size_t)world) == hipSuccess &&
         dalloc(&S.back, g.max_batch) == hipSuccess &&
         dalloc(&S.stats_stage, (size_t)world * r->m_max) == hipSuccess &&
         hipEventCreateWithFlags(&S.packed, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&S.sent, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&S.done, hipEventDisableTiming) == hipSuccess &&
         hipEventRecord(S.done, r->ret) == hipSuccess &&
         grow(r, S, world == 1 ? 0 : g.max_batch, world == 1 ? 0 : g.max_stem_bytes, 1) == hipSuccess;
  }
  ok = ok && hipStreamSynchronize(r->ret) == hipSuccess;
  if (!ok) {
    *err = "gpu: routing buffer allocation failed";
    comm_destroy(r);
    return nullptr;
  }
  r->base.assign(world, 0);
  return r;
}

void comm_destroy(CommRouter* r) {
  if (!r) return;
  if (r->timing && r->n_steps)
    fprintf(stderr, "{\"route_host_us\": {\"first_half\": %.1f, \"wait_counts\": %.1f, \"owner_enqueue\": %.1f, "
                    "\"second_half\": %.1f, \"batches\": %llu}}\n",
            r->t_first / r->n_steps * 1e6, r->t_wait_counts / r->n_steps * 1e6, r->t_owner / r->n_steps * 1e6,
            r->t_second / r->n_steps * 1e6, (unsigned long long)r->n_steps);
  (void)hipSetDevice(r->dev);
  for (hipStream_t st : {r->cs, r->fwd, r->ret})
    if (st) (void)hipStreamSynchronize(st);
  for (ncclComm_t c : {r->comm_r, r->comm_f, r->comm_c})
    if (c) (void)rccl().destroy(c);
  for (CommSlot& S : r->slot) free_slot(S);
  if (r->h_cnt) (void)hipHostFree(r->h_cnt);
  if (r->in_ready) (void)hipEventDestroy(r->in_ready);
  for (hipStream_t st : {r->cs, r->fwd, r->ret})
    if (st) (void)hipStreamDestroy(st);
  delete r;
}

// Completes the pending batch (collective, like every routed step), then
// waits for the router's streams.
int comm_synchronize(CommRouter* r, Engine* e) {
  CHK_HIP(e, hipSetDevice(r->dev));
  if (r->pending >= 0) {
    const uint32_t p = (uint32_t)r->pending;
    r->pending = -1;
    const int rc = second_half(r, e, r->slot[p], p);
    if (rc) return rc;
  }
  for (hipStream_t st : {r->cs, r->fwd, r->ret}) CHK_HIP(e, hipStreamSynchronize(st));
  return RL_OK;
}

int comm_do_limit(CommRouter* r, Engine* e, const rl_batch* in, rl_result* out, hipStream_t caller) {
  const uint32_t W = r->world, n = in->n, nr = in->n_rules;
  if ((uint64_t)W * nr > e->cfg.max_rules)
    return eng_fail(e, RL_E_CAPACITY, "gpu: routed batches need max_rules >= world x n_rules (per-source stats)");
  if (n && (!out->code || !out->limit_remaining || !out->reset_s))
    return eng_fail(e, RL_E_INVALID, "gpu: null result array");
  CHK_HIP(e, hipSetDevice(r->dev));
  const uint32_t s = r->next;
  r->next = (s + 1) % RSLOTS;
  CommSlot& S = r->slot[s];
  S.out = *out;
  S.n = n;
  S.n_rules = nr;
  const double t0 = now_s();
  int rc = first_half(r, e, S, s, in, caller);
  r->t_first += now_s() - t0;
  if (rc) return rc;
  // the previous batch: its counts had a whole call to arrive
  if (r->pending >= 0) {
    const uint32_t p = (uint32_t)r->pending;
    r->pending = -1;
    rc = second_half(r, e, r->slot[p], p);
    if (rc) return rc;
  }
  r->pending = (int)s;
  return RL_OK;
}

}  // namespace rl
