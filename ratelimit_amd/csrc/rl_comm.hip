// rl_comm.hip — the multi-rank routed DoLimit step, driven entirely by the
// library.
//
// One single-shard engine per rank; every rank calls comm_do_limit once per
// node batch with its own slice. The exchanges go through a Transport
// (rl_transport.h): RCCL between processes (one per GPU, the 8-GPU node), or
// the in-process loopback (several ranks as host threads, e.g. on one GPU).
// Per batch:
//
//   cnt stream:  rl_route_pack partition of the slice by owner (stem hash);
//                counts exchange (channel 0): per peer {records, stem bytes,
//                n_rules, flags};
//   host:        read the counts (the one wait per batch, one call later);
//   fwd stream:  records + stem bytes to their owners (channel 1; each peer
//                pair uses its own xGMI link);
//   engine:      the owner pipeline over the received chunks, concatenated in
//                source-rank order (= global arrival order), in parts of at
//                most max_batch records; stats attributed per source rank
//                (rule stride = the largest n_rules any rank sent);
//   ret stream:  packed results (a failed owner batch answers its status for
//                every record) and each source's stats block go back (channel
//                2); scatter to arrival order, sum the stats blocks.
//
// A call enqueues its batch's partition and counts exchange and then
// completes the batch ROUTE_LAG calls back (whose counts have had that many
// calls to arrive): the host never waits for work it just issued, batch t's
// partition runs beside the owner pipelines of batches t-1 .. t-LAG, and
// rl_synchronize completes the pending ones. RSLOTS batches may be in flight.
//
// Failures never break the exchange. A slice the host rejects (sizes, null
// outputs, a bad n_rules) sends zero counts with the FAILED flag and still
// takes part in every group; its rank's batch fails at rl_synchronize. An
// owner that cannot run what it received (stats stride or stems beyond its
// capacity) answers every received record with the failure status, which
// each source reports per descriptor (rl_result.status) or at rl_synchronize.
// Only a runtime failure of HIP or the transport itself leaves the router
// broken (every later call fails; RCCL peers may then wait forever, loopback
// peers time out).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "rl_comm.h"
#include "rl_kernels.h"
#include "rl_transport.h"

namespace rl {

namespace {

// batches a router keeps in flight: a slot's partition waits for the batch
// RSLOTS back to complete (its buffers are reused). 6 rather than 3 so that
// this wait never binds (routed N=1 3.33-3.36 vs 3.22-3.30 G); the host's
// remaining ~150 us wait per step for the counts is the partition waiting for
// GPU capacity beside the owner pipelines (RL_DEBUG_ROUTE_TIMING).
constexpr uint32_t RSLOTS = RL_ROUTED_INFLIGHT;
// A call completes the batch LAG calls back (its counts have had LAG calls to
// arrive), so LAG owner pipelines are queued ahead of the one being set up and
// the GPU never drains while the host waits for a partition. LAG < RSLOTS (a
// slot is reused RSLOTS calls later). RL_DEBUG_ROUTE_LAG overrides it (A/B).
constexpr uint32_t ROUTE_LAG = RL_ROUTED_LAG;
static_assert(ROUTE_LAG >= 1 && ROUTE_LAG < RSLOTS, "lag within the slots in flight");

// The counts message: CNT_W u64 per peer.
constexpr uint32_t CNT_W = 4;                 // records, stem bytes, n_rules, flags
constexpr uint64_t CNT_ISOLATE = 1;           // the sender wants per-descriptor statuses
constexpr uint64_t CNT_FAILED = 2;            // the sender's slice failed on its host (nothing sent)

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

}  // namespace

struct CommSlot {
  Wire* send_rec = nullptr;                // partition of this rank's slice, owner order
  uint8_t* send_stem = nullptr;
  uint32_t* perm = nullptr;                // record -> slice index
  unsigned long long* hash = nullptr;      // [slice] stem hashes (the own chunk's owner batch reads them)
  RouteBufs pb{};                          // the partition's scratch (slots' partitions may run concurrently)
  rl_batch src{};                          // the slice as partitioned (device view): the own chunk's source
  unsigned long long* cnt = nullptr;       // [2 x CNT_W x world]: sent per peer, then received
  Wire* recv_rec = nullptr;                // chunks of every source, rank order
  uint8_t* recv_stem = nullptr;
  unsigned long long* ret_send = nullptr;  // packed results of the received records
  uint64_t cap_rec = 0, cap_stem = 0;
  uint32_t* woff = nullptr;                // an exchange run in several owner parts: the records' stem offsets
  unsigned long long* wtsum = nullptr;     // (and the scan's tile sums and verdict)
  unsigned long long* wbase = nullptr;     // [RL_MAX_SHARDS] the chunk bases the scan checks (device)
  unsigned long long* h_wbase = nullptr;   // (pinned staging)
  uint64_t cap_woff = 0;
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
  int err = RL_OK;                         // the slice failed on the host: it sent nothing
  std::string errmsg;
  CommIO io{};
  // host-fed slices (CommIO.host): device staging at the caller's absolute
  // offsets, allocated on first use; io slices' stats (device) for stats_host
  uint8_t* h_stem = nullptr;
  uint32_t *h_off = nullptr, *h_req = nullptr, *h_limit = nullptr, *h_hits = nullptr, *h_rule = nullptr;
  int64_t* h_now = nullptr;
  uint8_t *h_unit = nullptr, *h_flags = nullptr, *h_code = nullptr, *h_status = nullptr;
  uint32_t *h_rem = nullptr, *h_reset = nullptr;
  uint8_t* h_cbuf = nullptr;  // compact slices: the host buffer's layout, the slice's parts
  uint64_t h_cbuf_cap = 0;
  unsigned long long* io_stats = nullptr;
};

struct CommRouter {
  std::unique_ptr<Transport> tr;
  uint32_t world = 1, rank = 0;
  int dev = 0;
  uint32_t m_max = 0;
  uint32_t part_max = 0;  // owner part size: max_batch (test knob: RL_DEBUG_OWNER_PART)
  bool alias = false;     // world 1: the owner reads the partition in place, no exchange
  bool own = true;        // this rank's own chunk read in place from its slice (no wire records, no stem copy)
  hipStream_t cs = nullptr, fwd = nullptr, ret = nullptr;
  // one_stream (default): a batch's routed work runs on the engine pipeline
  // stream its owner part will take (partition and counts on the one its
  // owner batch is predicted to use, records out and results back on the
  // owner part's own), so no router marker or kernel waits behind another
  // stream's batches on a shared hardware queue. RL_DEBUG_ROUTE_STREAMS=3:
  // the router's own three streams (cs / fwd / ret), for A/B.
  bool one_stream = true;
  hipStream_t scs = nullptr;  // this call's partition stream
  hipEvent_t in_ready = nullptr;
  CommSlot slot[RSLOTS];
  uint32_t next = 0;
  uint32_t lag = ROUTE_LAG;             // second halves run this many calls after their first
  uint32_t pend[RSLOTS] = {};           // slots whose second half is still to run, oldest first
  uint32_t n_pend = 0;
  unsigned long long* h_cnt = nullptr;  // pinned [RSLOTS][2 x CNT_W x world]
  unsigned long long* d_hcnt = nullptr;  // h_cnt as the device sees it (world 1: the partition stores the counts there)
  long long* d_floor = nullptr;          // [1 + world]: this rank's sweep time, then each peer's (comm_sweep_floor)
  std::vector<uint64_t> base;           // received chunk offsets in recv_stem (host)
  std::vector<uint64_t> so_r, so_b, ro_r;  // per-peer send / receive offsets (host)
  std::vector<Xfer> ops;
  // the first batch failure since the last synchronize (reported there)
  int sticky = RL_OK;
  std::string sticky_msg;
  // a HIP / transport runtime failure: the router is unusable
  int broken = RL_OK;
  std::string broken_msg;
  // host seconds per phase (printed at destroy when RL_DEBUG_ROUTE_TIMING is set)
  bool timing = false;
  double t_first = 0, t_wait_counts = 0, t_owner = 0, t_second = 0, t_slot = 0, t_call = 0;
  uint64_t n_steps = 0, n_slot_busy = 0, n_lat = 0;
  double t_enq[RSLOTS] = {}, t_lat = 0;  // host time of each slot's owner enqueue; enqueue -> found done
};

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

namespace {

// A runtime failure: the router stops here.
int breaks(CommRouter* r, Engine* e, int code, const std::string& msg) {
  if (!r->broken) {
    r->broken = code;
    r->broken_msg = msg;
  }
  return eng_fail(e, code, msg);
}

#define CHK_HIP(e, expr)                                                                                  \
  do {                                                                                                    \
    hipError_t _h = (expr);                                                                               \
    if (_h != hipSuccess) return breaks(r, (e), RL_E_HIP, std::string("gpu: ") + #expr + ": " + hipGetErrorString(_h)); \
  } while (0)

int run_group(CommRouter* r, Engine* e, uint32_t ch, hipStream_t st) {
  std::string err;
  const int rc = r->tr->group(ch, r->ops, st, &err);
  if (rc) return breaks(r, e, rc, err);
  return RL_OK;
}

void free_slot(CommSlot& S) {
  void* bufs[] = {S.pb.dest, S.pb.hist, S.pb.start, S.send_rec, S.send_stem, S.perm, S.hash, S.cnt, S.recv_rec,
                  S.recv_stem, S.ret_send, S.back, S.ostats, S.woff, S.wtsum, S.wbase,
                  S.stats_stage, S.h_stem, S.h_off, S.h_req, S.h_limit, S.h_hits, S.h_rule, S.h_now, S.h_unit,
                  S.h_flags, S.h_code, S.h_status, S.h_rem, S.h_reset, S.io_stats, S.h_cbuf};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  if (S.h_wbase) (void)hipHostFree(S.h_wbase);
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

// Slot S's stem-offset scan buffers hold n records' offsets (+ the total).
hipError_t grow_woff(CommSlot& S, uint64_t n) {
  if (n <= S.cap_woff) return hipSuccess;
  hipError_t e = hipEventSynchronize(S.done);
  if (e != hipSuccess) return e;
  (void)hipFree(S.woff);
  (void)hipFree(S.wtsum);
  S.woff = nullptr;
  S.wtsum = nullptr;
  S.cap_woff = 0;
  if ((e = dalloc(&S.woff, n + 1)) != hipSuccess || (e = dalloc(&S.wtsum, WIRE_SCAN_WORDS(n))) != hipSuccess) return e;
  if (!S.wbase && (e = dalloc(&S.wbase, RL_MAX_SHARDS)) != hipSuccess) return e;
  if (!S.h_wbase && (e = hipHostMalloc((void**)&S.h_wbase, RL_MAX_SHARDS * 8)) != hipSuccess) return e;
  S.cap_woff = n;
  return hipSuccess;
}

// A host-fed slice (CommIO.host) into slot S's device staging, on the counts
// stream (after the slot's previous batch): the same absolute offsets, so the
// staged view *d indexes like the caller's batch. Checks the sizes the copies
// rely on first (a failure is the slice's own: zero counts).
// The slot's host-fed staging arrays (first use).
int ensure_stage(CommRouter* r, Engine* e, CommSlot& S) {
  const rl_config& g = e->cfg;
  if (!S.h_stem) {
    const bool ok = dalloc(&S.h_stem, (size_t)g.max_stem_bytes + 64) == hipSuccess &&
                    dalloc(&S.h_off, (size_t)g.max_batch + 1) == hipSuccess && dalloc(&S.h_req, g.max_batch) == hipSuccess &&
                    dalloc(&S.h_limit, g.max_batch) == hipSuccess && dalloc(&S.h_hits, g.max_batch) == hipSuccess &&
                    dalloc(&S.h_rule, g.max_batch) == hipSuccess && dalloc(&S.h_now, g.max_requests) == hipSuccess &&
                    dalloc(&S.h_unit, g.max_batch) == hipSuccess && dalloc(&S.h_flags, g.max_batch) == hipSuccess &&
                    dalloc(&S.h_code, g.max_batch) == hipSuccess && dalloc(&S.h_status, g.max_batch) == hipSuccess &&
                    dalloc(&S.h_rem, g.max_batch) == hipSuccess && dalloc(&S.h_reset, g.max_batch) == hipSuccess;
    if (!ok) return breaks(r, e, RL_E_HIP, "gpu: host-fed routing staging allocation failed");
  }
  return RL_OK;
}

int stage_host(CommRouter* r, Engine* e, CommSlot& S, const rl_batch* in, rl_batch* d) {
  const rl_config& g = e->cfg;
  if (const int rc = ensure_stage(r, e, S)) return rc;
  const uint32_t n = in->n, da = S.io.da, qa = S.io.qa, qb = in->n_requests;
  if (!n) {
    *d = *in;
    return RL_OK;
  }
  const uint64_t a0 = in->stem_off[0] & ~3u, a1 = in->stem_off[n];
  if ((uint64_t)da + n > g.max_batch || qb > g.max_requests || qa > qb || a1 > g.max_stem_bytes || a1 < a0)
    return eng_fail(e, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_stem_bytes");
  hipStream_t st = r->scs;
  CHK_HIP(e, hipMemcpyAsync(S.h_stem + a0, in->stem_bytes + a0, a1 - a0, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_off + da, in->stem_off, (n + 1) * 4ull, hipMemcpyHostToDevice, st));
  if (qb > qa) CHK_HIP(e, hipMemcpyAsync(S.h_now + qa, in->now + qa, (qb - qa) * 8ull, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_req + da, in->req_idx, n * 4ull, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_unit + da, in->unit, n, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_flags + da, in->flags, n, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_limit + da, in->limit, n * 4ull, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_hits + da, in->hits, n * 4ull, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_rule + da, in->rule_id, n * 4ull, hipMemcpyHostToDevice, st));
  *d = *in;
  d->stem_bytes = S.h_stem;
  d->stem_off = S.h_off + da;
  d->now = S.h_now;
  d->req_idx = S.h_req + da;
  d->unit = S.h_unit + da;
  d->flags = S.h_flags + da;
  d->limit = S.h_limit + da;
  d->hits = S.h_hits + da;
  d->rule_id = S.h_rule + da;
  return RL_OK;
}

// A compact slice: its stems and offsets straight into the staging above (at
// the same absolute offsets), the rest of its parts into h_cbuf at the host
// buffer's own offsets, then k_unpack over the slice's descriptors and
// requests writes the staging arrays. Seven copies per slice (stems, offsets,
// limit indices, request firsts, clocks, hits, the limit table) of 46 B per
// descriptor at C1, against stage_host's nine of 60 B. A malformed request
// layout fails the batch through the partition's validation word.
int stage_host_compact(CommRouter* r, Engine* e, CommSlot& S, const rl_batch* in, rl_batch* d) {
  const rl_batch_compact& cb = *S.io.cb;
  const uint32_t n = in->n, da = S.io.da, db = da + n, qa = S.io.qa, qb = in->n_requests;
  const rl_config& g = e->cfg;
  if (const int rc = ensure_stage(r, e, S)) return rc;
  if ((uint64_t)db > g.max_batch || qb > g.max_requests || qa > qb)
    return eng_fail(e, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_stem_bytes");
  if (!n) {
    *d = *in;
    return RL_OK;
  }
  if (cb.buf_bytes > S.h_cbuf_cap) {  // (the slot's previous batch is drained first)
    CHK_HIP(e, hipEventSynchronize(S.done));
    if (S.h_cbuf) CHK_HIP(e, hipFree(S.h_cbuf));
    S.h_cbuf = nullptr;
    S.h_cbuf_cap = 0;
    if (dalloc(&S.h_cbuf, cb.buf_bytes + 64) != hipSuccess)
      return breaks(r, e, RL_E_HIP, "gpu: compact slice staging allocation failed");
    S.h_cbuf_cap = cb.buf_bytes;
  }
  const uint32_t* off = reinterpret_cast<const uint32_t*>(cb.buf + cb.stem_off);
  const uint64_t a0 = off[da] & ~3u, a1 = off[db];
  if (a1 < a0 || a1 > off[cb.n])  // (offsets out of order: never read past the buffer's stems)
    return eng_fail(e, RL_E_INVALID, "gpu: compact batch stem offsets out of order");
  if (a1 > g.max_stem_bytes)
    return eng_fail(e, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_stem_bytes");
  hipStream_t st = r->scs;
  auto part = [&](uint64_t sect, uint64_t from, uint64_t bytes) {
    return bytes ? hipMemcpyAsync(S.h_cbuf + sect + from, cb.buf + sect + from, bytes, hipMemcpyHostToDevice, st)
                 : hipSuccess;
  };
  if (a1 > a0) CHK_HIP(e, hipMemcpyAsync(S.h_stem + a0, cb.buf + cb.stem_bytes + a0, a1 - a0, hipMemcpyHostToDevice, st));
  CHK_HIP(e, hipMemcpyAsync(S.h_off + da, off + da, (n + 1) * 4ull, hipMemcpyHostToDevice, st));
  CHK_HIP(e, part(cb.limit_idx, 2ull * da, 2ull * n));
  CHK_HIP(e, part(cb.req_first, 4ull * qa, 4ull * (qb - qa + 1)));
  CHK_HIP(e, part(cb.now, 4ull * qa, 4ull * (qb - qa)));
  CHK_HIP(e, part(cb.hits, 4ull * qa, 4ull * (qb - qa)));
  CHK_HIP(e, part(cb.limits, 0, 12ull * cb.n_limits));
  launch_unpack_range(cb, S.h_cbuf, da, db, qa, qb, S.h_req, S.h_unit, S.h_flags, S.h_limit, S.h_hits, S.h_rule,
                      S.h_now, e->errw + NBUF + 2, st);
  CHK_HIP(e, hipGetLastError());
  *d = *in;
  d->stem_bytes = S.h_stem;
  d->stem_off = S.h_off + da;
  d->now = S.h_now;
  d->req_idx = S.h_req + da;
  d->unit = S.h_unit + da;
  d->flags = S.h_flags + da;
  d->limit = S.h_limit + da;
  d->hits = S.h_hits + da;
  d->rule_id = S.h_rule + da;
  return RL_OK;
}

// A prefix-shared slice (request tiles [t0, t1)): its parts of the host
// buffer into h_cbuf at the buffer's own offsets (index entries t0..t1, the
// tiles' request words, clocks and hits, their descriptor words, prefix and
// suffix bytes, the limit table), then k_unpack_prefixed over those tiles
// writes the staging arrays and stems at their absolute offsets. Eight copies
// of ~31.5 B per descriptor at C1; the index entries were written by the
// batcher, so the cut reads nothing but them.
int stage_host_prefixed(CommRouter* r, Engine* e, CommSlot& S, const rl_batch* in, rl_batch* d) {
  const rl_batch_prefixed& pb = *S.io.pb;
  const uint32_t n = in->n, da = S.io.da, db = da + n, qa = S.io.qa, qb = in->n_requests;
  const rl_config& g = e->cfg;
  if (const int rc = ensure_stage(r, e, S)) return rc;
  if ((uint64_t)db > g.max_batch || qb > g.max_requests || qa > qb)
    return eng_fail(e, RL_E_CAPACITY, "gpu: batch exceeds configured max_batch/max_requests/max_stem_bytes");
  if (S.io.t1 <= S.io.t0) {
    *d = *in;
    return RL_OK;
  }
  if (pb.buf_bytes > S.h_cbuf_cap) {  // (the slot's previous batch is drained first)
    CHK_HIP(e, hipEventSynchronize(S.done));
    if (S.h_cbuf) CHK_HIP(e, hipFree(S.h_cbuf));
    S.h_cbuf = nullptr;
    S.h_cbuf_cap = 0;
    if (dalloc(&S.h_cbuf, pb.buf_bytes + 64) != hipSuccess)
      return breaks(r, e, RL_E_HIP, "gpu: prefixed slice staging allocation failed");
    S.h_cbuf_cap = pb.buf_bytes;
  }
  const uint32_t* ix = reinterpret_cast<const uint32_t*>(pb.buf + pb.index);
  const uint32_t* I0 = ix + 4ull * S.io.t0;
  const uint32_t* I1 = ix + 4ull * S.io.t1;
  const uint32_t T = (pb.n_requests + RL_PREFIXED_TILE - 1) / RL_PREFIXED_TILE;
  const uint32_t* tot = ix + 4ull * T;
  // the cut's own entries bound the copies (the device checks every tile's)
  if (I0[0] != da || I1[0] != db || I1[1] < I0[1] || I1[2] < I0[2] || I1[1] > tot[1] || I1[2] > tot[2])
    return eng_fail(e, RL_E_INVALID, "gpu: prefixed batch index out of order");
  hipStream_t st = r->scs;
  auto part = [&](uint64_t sect, uint64_t from, uint64_t bytes) {
    return bytes ? hipMemcpyAsync(S.h_cbuf + sect + from, pb.buf + sect + from, bytes, hipMemcpyHostToDevice, st)
                 : hipSuccess;
  };
  CHK_HIP(e, part(pb.index, 16ull * S.io.t0, 16ull * (S.io.t1 - S.io.t0 + 1)));
  CHK_HIP(e, part(pb.req, 4ull * qa, 4ull * (qb - qa)));
  CHK_HIP(e, part(pb.now, 4ull * qa, 4ull * (qb - qa)));
  CHK_HIP(e, part(pb.hits, 4ull * qa, 4ull * (qb - qa)));
  CHK_HIP(e, part(pb.desc, 4ull * da, 4ull * n));
  CHK_HIP(e, part(pb.prefix_bytes, I0[1], (uint64_t)I1[1] - I0[1]));
  CHK_HIP(e, part(pb.suffix_bytes, I0[2], (uint64_t)I1[2] - I0[2]));
  CHK_HIP(e, part(pb.limits, 0, 12ull * pb.n_limits));
  launch_unpack_prefixed(pb, S.h_cbuf, S.io.t0, S.io.t1, S.h_stem, S.h_off, S.h_req, S.h_unit, S.h_flags, S.h_limit,
                         S.h_hits, S.h_rule, S.h_now, e->errw + NBUF + 2, st);
  CHK_HIP(e, hipGetLastError());
  *d = *in;
  d->stem_bytes = S.h_stem;
  d->stem_off = S.h_off + da;
  d->now = S.h_now;
  d->req_idx = S.h_req + da;
  d->unit = S.h_unit + da;
  d->flags = S.h_flags + da;
  d->limit = S.h_limit + da;
  d->hits = S.h_hits + da;
  d->rule_id = S.h_rule + da;
  return RL_OK;
}

// First half of a batch (slot s): partition, counts exchange, counts to the
// host. `hostrc` != RL_OK: the slice was rejected before the partition; it
// sends zero counts. (The next call's second half waits on the host for this
// partition: from then on the inputs may be reused.)
int first_half(CommRouter* r, Engine* e, CommSlot& S, uint32_t s, const rl_batch* in, hipStream_t caller,
               int hostrc) {
  const uint32_t W = r->world, me = r->rank;
  // (one_stream: the pipeline stream this batch's owner part is predicted to
  // take: the engine buffer after the pending batches' owner parts)
  r->scs = r->one_stream ? e->pipe[(e->next + r->n_pend) % NBUF] : r->cs;
  hipStream_t cs = r->scs;
  CHK_HIP(e, hipStreamWaitEvent(cs, S.done, 0));  // the slot's previous batch is complete
  if (caller && hipStreamQuery(caller) == hipErrorNotReady) {  // the inputs' producer (still running)
    CHK_HIP(e, hipEventRecord(r->in_ready, caller));
    CHK_HIP(e, hipStreamWaitEvent(cs, r->in_ready, 0));
  }
  const uint64_t flags = S.out.status ? CNT_ISOLATE : 0;
  int rc = hostrc;
  rl_batch staged;
  if (!rc && S.io.host) {
    rc = S.io.cb   ? stage_host_compact(r, e, S, in, &staged)
         : S.io.pb ? stage_host_prefixed(r, e, S, in, &staged)
                   : stage_host(r, e, S, in, &staged);
    if (r->broken) return rc;
    in = &staged;
  }
  // world 1: no exchange, the counts go straight to the host's copy (kernel
  // stores to page-locked memory; no copy launch per batch)
  unsigned long long* hc = r->alias && r->d_hcnt ? r->d_hcnt + (size_t)s * 2 * CNT_W * W : nullptr;
  if (!rc) {
    rc = eng_route_pack(e, in, W, me, S.send_rec, S.send_stem, S.perm, (uint64_t*)S.cnt, cs, CNT_W, S.n_rules,
                        flags, r->own ? me : ROUTE_OWN_NONE, S.hash, hc, &S.pb);
    S.src = *in;  // (read by this batch's owner part, in the next call)
  }
  if (rc) {  // (a device-side malformation zeroes the counts itself and fails at rl_synchronize)
    S.err = rc;
    S.errmsg = eng_last_error(e);
    launch_cnt_fill(S.cnt, W, CNT_W, 0, flags | CNT_FAILED, cs, hc);
  }
  if (!r->alias) {
    r->ops.clear();
    for (uint32_t p = 0; p < W; p++) {
      if (p == me) continue;
      r->ops.push_back({S.cnt + (size_t)CNT_W * p, CNT_W * 8ull, p, true});
      r->ops.push_back({S.cnt + (size_t)CNT_W * (W + p), CNT_W * 8ull, p, false});
    }
    const int g = run_group(r, e, 0, cs);
    if (g) return g;
  }
  if (!hc)
    CHK_HIP(e, hipMemcpyAsync(r->h_cnt + (size_t)s * 2 * CNT_W * W, S.cnt, 2ull * CNT_W * W * 8, hipMemcpyDeviceToHost,
                              cs));
  CHK_HIP(e, hipEventRecord(S.packed, cs));
  return RL_OK;
}

// Second half (slot s): records and stems to their owners, the owner
// pipeline, results and per-source stats back, scatter.
int second_half(CommRouter* r, Engine* e, CommSlot& S, uint32_t s) {
  const uint32_t W = r->world, me = r->rank, n = S.n;
  unsigned long long* h = r->h_cnt + (size_t)s * 2 * CNT_W * W;
  unsigned long long* hr = h + (size_t)CNT_W * W;  // received
  const double t0 = now_s();
  CHK_HIP(e, hipEventSynchronize(S.packed));  // (issued one call ago)
  const double t1 = now_s();
  r->t_wait_counts += t1 - t0;
  for (uint32_t k = 0; k < CNT_W; k++) hr[CNT_W * me + k] = h[CNT_W * me + k];  // (own chunk)
  uint64_t n_send = 0, n_recv = 0, b_recv = 0, M = 0, iso = 0;
  for (uint32_t p = 0; p < W; p++) {
    n_send += h[CNT_W * p];
    r->base[p] = b_recv;
    n_recv += hr[CNT_W * p];
    b_recv += hr[CNT_W * p + 1];
    M = std::max<uint64_t>(M, hr[CNT_W * p + 2]);
    iso |= hr[CNT_W * p + 3] & CNT_ISOLATE;
  }
  if (!S.err && n_send != n && n_send != 0) {  // (0: the device rejected the slice, below)
    S.err = eng_fail(e, RL_E_INTERNAL, "gpu: routing counts do not add up");
    S.errmsg = eng_last_error(e);
  }
  // what this rank cannot run as an owner fails every record it received
  int owner_fail = RL_OK;
  if (b_recv >= (1ull << 32)) {
    owner_fail = RL_E_CAPACITY;
  } else if ((uint64_t)W * M > e->cfg.max_rules) {
    owner_fail = RL_E_CAPACITY;  // (per-source stats: an owner needs world x n_rules rule slots)
  }
  if (owner_fail && !r->sticky) {
    r->sticky = owner_fail;
    r->sticky_msg = "gpu: routed owner capacity exceeded (4 GiB of stems, or max_rules < world x n_rules)";
  }
  const uint32_t m = (uint32_t)M * RL_NUM_STATS;  // one source's stats block
  const uint32_t mb = r->part_max;
  // per-peer offsets: so_* into the send buffers, ro_* into the receive ones
  r->so_r.assign(W + 1, 0);
  r->so_b.assign(W + 1, 0);
  r->ro_r.assign(W + 1, 0);
  for (uint32_t p = 0; p < W; p++) {
    r->so_r[p + 1] = r->so_r[p] + h[CNT_W * p];
    r->so_b[p + 1] = r->so_b[p] + h[CNT_W * p + 1];
    r->ro_r[p + 1] = r->ro_r[p] + hr[CNT_W * p];
  }
  // world 1: nothing crosses the fwd stream; the owner waits on the
  // partition itself (a wait routed through fwd queued behind whatever shares
  // its hardware queue)
  hipStream_t fwd = r->one_stream ? e->pipe[e->next] : r->fwd;  // (one_stream: the owner part's stream)
  if (!r->alias) CHK_HIP(e, hipStreamWaitEvent(fwd, S.packed, 0));
  if (!r->alias) CHK_HIP(e, grow(r, S, n_recv, b_recv, 1));
  // (world 1: the partition is the received batch)
  const Wire* recv_rec = r->alias ? S.send_rec : S.recv_rec;
  const uint8_t* recv_stem = r->alias ? S.send_stem : S.recv_stem;
  if (!r->alias) {
    // records and stems to their owners; this rank's own chunk by device copy
    r->ops.clear();
    for (uint32_t p = 0; p < W; p++) {
      if (p == me) continue;
      const uint64_t sn = h[CNT_W * p], sb = h[CNT_W * p + 1], rn = hr[CNT_W * p], rb = hr[CNT_W * p + 1];
      r->ops.push_back({S.send_rec + r->so_r[p], sn * sizeof(Wire), p, true});
      r->ops.push_back({S.send_stem + r->so_b[p], sb, p, true});
      r->ops.push_back({S.recv_rec + r->ro_r[p], rn * sizeof(Wire), p, false});
      r->ops.push_back({S.recv_stem + r->base[p], rb, p, false});
    }
    const int g = run_group(r, e, 1, fwd);
    if (g) return g;
    if (h[CNT_W * me] && !r->own)
      CHK_HIP(e, hipMemcpyAsync(S.recv_rec + r->ro_r[me], S.send_rec + r->so_r[me], h[CNT_W * me] * sizeof(Wire),
                                hipMemcpyDeviceToDevice, fwd));
    if (h[CNT_W * me + 1])  // (none with the own chunk read in place)
      CHK_HIP(e, hipMemcpyAsync(S.recv_stem + r->base[me], S.send_stem + r->so_b[me], h[CNT_W * me + 1],
                                hipMemcpyDeviceToDevice, fwd));
  }
  const uint64_t own_lo = r->ro_r[me], own_hi = r->own ? r->ro_r[me + 1] : own_lo;  // (received positions)
  // an exchange answered in several owner parts (below): the records' stem
  // offsets, scanned once over all of them (one part scans its own)
  const bool scan_all = n_recv > mb && !owner_fail && n_recv > own_hi - own_lo;
  if (scan_all) {
    CHK_HIP(e, grow_woff(S, n_recv));
    if (r->alias) CHK_HIP(e, hipStreamWaitEvent(fwd, S.packed, 0));
    CHK_HIP(e, hipEventSynchronize(S.done));  // (the slot's previous batch read the staged bases)
    std::copy(r->base.begin(), r->base.end(), S.h_wbase);
    CHK_HIP(e, hipMemcpyAsync(S.wbase, S.h_wbase, (size_t)W * 8, hipMemcpyHostToDevice, fwd));
    launch_wire_offsets(recv_rec, (uint32_t)n_recv, (uint32_t)own_lo, (uint32_t)own_hi, S.wbase, W, b_recv, S.woff,
                        S.wtsum, fwd);
  }
  if (!r->alias || scan_all) CHK_HIP(e, hipEventRecord(S.sent, fwd));
  hipEvent_t const sent = r->alias && !scan_all ? S.packed : S.sent;  // (the received records are ready)
  // the owner pipeline, in parts of at most max_batch records. A part ends on
  // a request boundary (a request's descriptors check the local cache before
  // any of them sets it, fixed_cache_impl.go:50-66 then :100-109), so more
  // than max_batch received records (hash skew; rare) cost one host read of
  // the received labels.
  std::vector<uint64_t>& cut = S.cut;
  cut.assign(1, 0);
  if (n_recv > mb && !owner_fail) {
    std::vector<uint32_t> lab(n_recv);
    CHK_HIP(e, hipStreamSynchronize(fwd));
    CHK_HIP(e, hipMemcpy2D(lab.data(), 4, recv_rec, sizeof(Wire), 4, n_recv, hipMemcpyDeviceToHost));
    if (own_hi > own_lo) {  // the own chunk has no wire labels: from its slice's request indices
      std::vector<uint32_t> pi(own_hi - own_lo), rq(S.n);
      CHK_HIP(e, hipMemcpy(pi.data(), S.perm + r->so_r[me], pi.size() * 4, hipMemcpyDeviceToHost));
      CHK_HIP(e, hipMemcpy(rq.data(), S.src.req_idx, rq.size() * 4, hipMemcpyDeviceToHost));
      for (uint64_t j = own_lo; j < own_hi; j++) lab[j] = (me << ROUTE_REQ_BITS) | rq[pi[j - own_lo]];
    }
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
  const bool direct = r->alias && parts == 1 && !owner_fail;
  S.k.assign(parts, 0);
  const size_t blk = (size_t)W * m;  // one part's per-source stats
  // this rank's outputs (arrival order): the scatter writes the records that
  // come back from owners; the own chunk's owner batch answers its own in
  // place (k_finish, OwnChunk outputs), and at world 1 with one part its stats
  // land in the output directly (no per-source sum)
  const bool out_ok = !S.err && !(n && n_send != n);  // (else perm was never written: nothing is scattered)
  const rl_result& out = S.out;
  const uint32_t mine = S.n_rules * RL_NUM_STATS;  // (<= m: M is the largest n_rules sent)
  OutDev o{out.code, out.limit_remaining, out.reset_s, (unsigned long long*)out.stats, out.status};
  if (S.io.host) o = OutDev{S.h_code, S.h_rem, S.h_reset, nullptr, out.status ? S.h_status : nullptr};
  unsigned long long* stats_out = S.io.stats_host ? S.io_stats : (unsigned long long*)out.stats;
  uint32_t* src_err = out.status ? nullptr : e->errw + NBUF + 2;
  const bool own_inplace = r->own && out_ok && !owner_fail;
  const bool stats_direct = direct && out_ok && W == 1 && stats_out && mine == m && m;
  // the own chunk's records in send order (answered in place: not scattered)
  const uint32_t ol = own_inplace ? (uint32_t)r->so_r[me] : 0u, oh = own_inplace ? (uint32_t)r->so_r[me + 1] : 0u;
  // world 1, one part, everything answered in place and nothing for the host
  // to copy: the batch ends with its owner pipeline, and its completion is
  // recorded on that pipeline's stream (the return stream shares a hardware
  // queue with another pipeline stream: a marker there waits behind that
  // stream's later batches)
  const bool on_pipe = direct && !S.io.host && !S.io.stats_host &&
                       (!out_ok || ((ol == 0 && oh >= n) && (stats_direct || !mine || !stats_out)));
  const double t2 = now_s();
  // the return stream: one_stream, the last owner part's (set below), or fwd's
  // when the owner cannot run
  hipStream_t ret = r->one_stream ? fwd : r->ret;
  if (owner_fail) {
    CHK_HIP(e, hipStreamWaitEvent(ret, sent, 0));
    launch_route_fail(ret_send, (uint32_t)n_recv, (uint32_t)owner_fail, ret);
    if (blk) CHK_HIP(e, hipMemsetAsync(S.ostats, 0, blk * 8, ret));
  } else {
    for (uint32_t q = 0; q < parts; q++) {
      const uint64_t a = cut[q], b = cut[q + 1];
      // this part's share of the own chunk, read in place from the slice
      OwnChunk oc{};
      const uint64_t lo = std::max(a, own_lo), hi = std::min(b, own_hi);
      if (lo < hi) {
        const rl_batch& sb = S.src;
        oc.lo = (uint32_t)(lo - a);
        oc.n = (uint32_t)(hi - lo);
        oc.rank = me;
        oc.stem_total = e->cfg.max_stem_bytes;
        oc.src_n = sb.n;
        oc.n_rules = sb.n_rules;
        oc.idx = S.perm + r->so_r[me] + (lo - own_lo);
        oc.hash = S.hash;
        oc.stem = sb.stem_bytes;
        oc.off = sb.stem_off;
        oc.now = sb.now;
        oc.req = sb.req_idx;
        oc.unit = sb.unit;
        oc.flags = sb.flags;
        oc.limit = sb.limit;
        oc.hits = sb.hits;
        oc.rule = sb.rule_id;
        if (own_inplace) {
          oc.code = o.code;
          oc.rem = o.rem;
          oc.reset = o.reset;
          oc.status = o.status;
          oc.src_err = src_err;
        }
      }
      const int rc = eng_route_owner(e, (uint32_t)(b - a), recv_rec + a, recv_stem, b_recv, r->base.data(), W,
                                     (uint32_t)M, (uint32_t)M, stats_direct ? stats_out : S.ostats + q * blk,
                                     iso ? 1 : 0, sent, &S.k[q], &oc, scan_all ? S.woff + a : nullptr,
                                     scan_all ? S.wtsum + WIRE_SCAN_TILES(n_recv) : nullptr);
      if (rc) return breaks(r, e, rc, eng_last_error(e));  // (argument checks only: the sizes were checked above)
      // its packed results, before a later part can take the same engine buffer
      const uint32_t k = S.k[q];
      CHK_HIP(e, hipSetDevice(r->dev));
      if (on_pipe) break;
      hipStream_t rs = r->one_stream ? e->pipe[k] : r->ret;
      if (!r->one_stream) CHK_HIP(e, hipStreamWaitEvent(rs, e->b_done[k], 0));
      if (direct) break;
      launch_route_ret(e->s[k].res, (uint32_t)(b - a), e->s[k].errb, ret_send + a, rs);
      CHK_HIP(e, hipEventRecord(e->consumed[k], rs));
    }
    if (r->one_stream) {  // the return on the last part's stream, after every part's results
      ret = e->pipe[S.k[parts - 1]];
      for (uint32_t q = 0; q + 1 < parts && !direct; q++) CHK_HIP(e, hipStreamWaitEvent(ret, e->consumed[S.k[q]], 0));
    }
  }
  const double t3 = now_s();
  r->t_owner += t3 - t2;
  r->t_enq[s] = t3;
  // results and per-source stats back to their sources
  if (parts > 1 && m && !owner_fail) launch_stats_sum(S.ostats, parts, (uint32_t)blk, S.ostats, ret);
  const unsigned long long* stats_in = S.ostats;  // (world 1: this rank's block is the owner's)
  if (!r->alias) {
    r->ops.clear();
    for (uint32_t p = 0; p < W; p++) {
      if (p == me) continue;
      const uint64_t sn = h[CNT_W * p], rn = hr[CNT_W * p];
      r->ops.push_back({S.ret_send + r->ro_r[p], rn * 8, p, true});
      r->ops.push_back({S.back + r->so_r[p], sn * 8, p, false});
      r->ops.push_back({S.ostats + (size_t)p * m, (uint64_t)m * 8, p, true});
      r->ops.push_back({S.stats_stage + (size_t)p * m, (uint64_t)m * 8, p, false});
    }
    const int g = run_group(r, e, 2, ret);
    if (g) return g;
    if (h[CNT_W * me] && !own_inplace)
      CHK_HIP(e, hipMemcpyAsync(S.back + r->so_r[me], S.ret_send + r->ro_r[me], h[CNT_W * me] * 8,
                                hipMemcpyDeviceToDevice, ret));
    if (m)
      CHK_HIP(e, hipMemcpyAsync(S.stats_stage + (size_t)me * m, S.ostats + (size_t)me * m, (size_t)m * 8,
                                hipMemcpyDeviceToDevice, ret));
    stats_in = S.stats_stage;
  }
  if (direct && (!out_ok || (ol == 0 && oh >= n))) {  // (the owner's results are not read: its buffer is free)
    CHK_HIP(e, hipEventRecord(e->consumed[S.k[0]], on_pipe ? e->pipe[S.k[0]] : ret));
  }
  if (!S.err && n && n_send != n) {
    // the partition rejected the slice on the device (zero counts; its error
    // word fails the batch at rl_synchronize): perm was never written, so
    // nothing is scattered
  } else if (!S.err) {
    if (direct) {
      const uint32_t k = S.k[0];
      if (!(ol == 0 && oh >= n)) {
        launch_route_scatter(S.perm, e->s[k].res, n, o, ret, src_err, e->s[k].errb, ol, oh);
        CHK_HIP(e, hipEventRecord(e->consumed[k], ret));
      }
    } else {
      launch_route_scatter(S.perm, S.back, n, o, ret, src_err, nullptr, ol, oh);
    }
    if (mine && stats_out && !stats_direct) launch_stats_sum(stats_in, W, mine, stats_out, ret, m);
    // the answers cross back to the caller's host slice (kernel stores into
    // page-locked outputs, rl_kernels.h ToHost)
    ToHost th{};
    auto add = [&](void* dst, const void* src, uint64_t bytes) {
      th.dst[th.n] = (uint8_t*)dst;
      th.src[th.n] = (const uint8_t*)src;
      th.bytes[th.n++] = bytes;
    };
    if (S.io.stats_host && mine) add(S.io.stats_host, S.io_stats, (size_t)mine * 8);
    if (S.io.host && n) {
      add(out.code, S.h_code, n);
      add(out.limit_remaining, S.h_rem, n * 4ull);
      if (out.reset_s) add(out.reset_s, S.h_reset, n * 4ull);
      if (out.status) add(out.status, S.h_status, n);
    }
    if (th.n) CHK_HIP(e, copy_to_host(th, ret));
  } else if (!r->sticky) {
    r->sticky = S.err;
    r->sticky_msg = S.errmsg;
  }
  CHK_HIP(e, hipGetLastError());
  CHK_HIP(e, hipEventRecord(S.done, on_pipe ? e->pipe[S.k[0]] : ret));  // (outputs: read after rl_synchronize)
  r->t_second += now_s() - t1;
  r->n_steps++;
  return RL_OK;
}

}  // namespace

int comm_unique_id(uint8_t* id, std::string* err) { return rccl_unique_id(id, err); }

int comm_loopback_id(uint8_t* id, std::string* err) { return loopback_new_id(id, err); }

CommRouter* comm_create(Engine* e, uint32_t world, uint32_t rank, const uint8_t* id, std::string* err) {
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
  r->own = !getenv("RL_DEBUG_ROUTE_NOOWN");  // (A/B knob: the own chunk as wire records and copied stems)
  r->timing = getenv("RL_DEBUG_ROUTE_TIMING") != nullptr;
  if (const char* rs = getenv("RL_DEBUG_ROUTE_STREAMS")) r->one_stream = atoi(rs) != 3;
  if (const char* lg = getenv("RL_DEBUG_ROUTE_LAG"))
    r->lag = std::max<uint32_t>(1, std::min<uint32_t>(RSLOTS - 1, (uint32_t)atoi(lg)));
  if (const char* pm = getenv("RL_DEBUG_OWNER_PART"))
    r->part_max = std::max<uint32_t>(1, std::min<uint32_t>(g.max_batch, (uint32_t)atoi(pm)));
  r->tr.reset(loopback_id(id) ? loopback_join(id, world, rank, err) : rccl_join(id, world, rank, r->dev, err));
  if (!r->tr) {
    comm_destroy(r);
    return nullptr;
  }
  bool ok = hipSetDevice(r->dev) == hipSuccess &&
            rl_stream_create(&r->cs, SR_ROUTER) == hipSuccess && rl_stream_create(&r->fwd, SR_ROUTER) == hipSuccess &&
            rl_stream_create(&r->ret, SR_ROUTER) == hipSuccess &&
            hipEventCreateWithFlags(&r->in_ready, hipEventDisableTiming) == hipSuccess &&
            hipHostMalloc((void**)&r->h_cnt, (size_t)RSLOTS * 2 * CNT_W * world * 8) == hipSuccess &&
            dalloc(&r->d_floor, (size_t)world + 1) == hipSuccess;
  if (ok && world == 1 && hipHostGetDevicePointer((void**)&r->d_hcnt, r->h_cnt, 0) != hipSuccess) {
    (void)hipGetLastError();
    r->d_hcnt = nullptr;  // (then a copy per batch)
  }
  for (uint32_t s = 0; s < RSLOTS && ok; s++) {
    CommSlot& S = r->slot[s];
    ok = dalloc(&S.send_rec, g.max_batch) == hipSuccess && dalloc(&S.send_stem, (size_t)g.max_stem_bytes + 64) == hipSuccess &&
         dalloc(&S.perm, g.max_batch) == hipSuccess && dalloc(&S.hash, g.max_batch) == hipSuccess &&
         dalloc(&S.pb.dest, g.max_batch) == hipSuccess && dalloc(&S.pb.start, 2 * (size_t)world + 1) == hipSuccess &&
         dalloc(&S.pb.hist, 2ull * world * ((g.max_batch + ROUTE_TILE - 1) / ROUTE_TILE)) == hipSuccess &&
         dalloc(&S.cnt, 2 * CNT_W * (size_t)world) == hipSuccess &&
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

const char* comm_kind(const CommRouter* r) { return r && r->tr ? r->tr->kind() : ""; }

void comm_destroy(CommRouter* r) {
  if (!r) return;
  if (r->timing && r->n_steps)
    fprintf(stderr, "{\"route_host_us\": {\"call\": %.1f, \"slot_wait\": %.1f, \"first_half\": %.1f, "
                    "\"wait_counts\": %.1f, \"owner_enqueue\": %.1f, \"second_half\": %.1f, \"batches\": %llu, \"slot_busy\": %llu, \"enqueue_to_reuse\": %.1f}}\n",
            r->t_call / r->n_steps * 1e6, r->t_slot / r->n_steps * 1e6, r->t_first / r->n_steps * 1e6,
            r->t_wait_counts / r->n_steps * 1e6, r->t_owner / r->n_steps * 1e6, r->t_second / r->n_steps * 1e6,
            (unsigned long long)r->n_steps, (unsigned long long)r->n_slot_busy, r->n_lat ? r->t_lat / r->n_lat * 1e6 : 0.0);
  (void)hipSetDevice(r->dev);
  for (hipStream_t st : {r->cs, r->fwd, r->ret})
    if (st) (void)hipStreamSynchronize(st);
  (void)hipDeviceSynchronize();  // (one_stream: routed work on the engine's pipeline streams reads the slots)
  r->tr.reset();
  for (CommSlot& S : r->slot) free_slot(S);
  if (r->h_cnt) (void)hipHostFree(r->h_cnt);
  if (r->d_floor) (void)hipFree(r->d_floor);
  if (r->in_ready) (void)hipEventDestroy(r->in_ready);
  for (hipStream_t st : {r->cs, r->fwd, r->ret})
    if (st) (void)hipStreamDestroy(st);
  delete r;
}

// Completes the pending batch (collective, like every routed step), waits for
// the router's streams, then reports the first batch failure since the last
// call.
int comm_synchronize(CommRouter* r, Engine* e) {
  if (r->broken) return eng_fail(e, r->broken, r->broken_msg);
  CHK_HIP(e, hipSetDevice(r->dev));
  while (r->n_pend) {  // (oldest first: the order every rank runs its exchanges in)
    const uint32_t p = r->pend[0];
    std::copy(r->pend + 1, r->pend + r->n_pend, r->pend);
    r->n_pend--;
    const int rc = second_half(r, e, r->slot[p], p);
    if (rc) return rc;
  }
  for (hipStream_t st : {r->cs, r->fwd, r->ret}) CHK_HIP(e, hipStreamSynchronize(st));
  for (uint32_t k = 0; k < NBUF && r->one_stream; k++) CHK_HIP(e, hipStreamSynchronize(e->pipe[k]));
  if (r->sticky) {
    const int rc = eng_fail(e, r->sticky, r->sticky_msg);
    r->sticky = RL_OK;
    r->sticky_msg.clear();
    return rc;
  }
  return RL_OK;
}

// The sweep floor of the whole world: the least `now` any rank passed to its
// rl_sweep. Every rank sweeps its own shard, and an owner checks a peer's
// requests against its floor, so one floor for all ranks means a rank whose
// clock trails a peer's (or whose caller sweeps with a larger lag) never sees
// its requests refused for a time its own clock has not reached. Collective
// like the routed batches (channel 0, quiet here: comm_synchronize ran
// first). A rank whose `now` is out of range takes part with no vote (its own
// eng_sweep then refuses the time).
int comm_sweep_floor(CommRouter* r, Engine* e, int64_t now, int64_t* floor) {
  *floor = now;
  if (r->broken) return eng_fail(e, r->broken, r->broken_msg);
  if (r->world == 1) return RL_OK;
  CHK_HIP(e, hipSetDevice(r->dev));
  const bool vote = now >= 0 && now <= (int64_t)NOW_MAX;
  std::vector<long long> v(r->world + 1, INT64_MAX);
  v[0] = vote ? now : INT64_MAX;
  CHK_HIP(e, hipMemcpyAsync(r->d_floor, v.data(), 8, hipMemcpyHostToDevice, r->cs));
  r->ops.clear();
  for (uint32_t p = 0; p < r->world; p++) {
    if (p == r->rank) continue;
    r->ops.push_back({r->d_floor, 8, p, true});
    r->ops.push_back({r->d_floor + 1 + p, 8, p, false});
  }
  if (const int rc = run_group(r, e, 0, r->cs)) return rc;
  CHK_HIP(e, hipMemcpyAsync(v.data(), r->d_floor, v.size() * 8, hipMemcpyDeviceToHost, r->cs));
  CHK_HIP(e, hipStreamSynchronize(r->cs));
  if (!vote) return RL_OK;
  for (uint32_t p = 0; p < r->world; p++)
    if (p != r->rank) *floor = std::min<int64_t>(*floor, v[1 + p]);
  return RL_OK;
}

uint32_t comm_slots() { return RSLOTS; }

int comm_wait_slot(CommRouter* r, Engine* e, uint32_t s) {
  CHK_HIP(e, hipSetDevice(r->dev));
  CHK_HIP(e, hipEventSynchronize(r->slot[s % RSLOTS].done));
  return RL_OK;
}

int comm_do_limit(CommRouter* r, Engine* e, const rl_batch* in, rl_result* out, hipStream_t caller,
                  const CommIO* io, int host_rc) {
  if (r->broken) return eng_fail(e, r->broken, r->broken_msg);
  const uint32_t n = in->n, nr = in->n_rules;
  CHK_HIP(e, hipSetDevice(r->dev));
  const uint32_t s = r->next;
  r->next = (s + 1) % RSLOTS;
  CommSlot& S = r->slot[s];
  const double tc = now_s();
  // the slot's previous batch (RSLOTS calls ago) is complete: its owner part
  // read that slice's own chunk in place, so a caller may reuse a batch's
  // inputs once RSLOTS later calls have returned (long done by then: this
  // wait does not bind)
  if (r->timing && hipEventQuery(S.done) == hipErrorNotReady) r->n_slot_busy++;
  CHK_HIP(e, hipEventSynchronize(S.done));
  r->t_slot += now_s() - tc;
  if (r->t_enq[s] > 0) {
    r->t_lat += now_s() - r->t_enq[s];
    r->n_lat++;
    r->t_enq[s] = 0;
  }
  S.out = *out;
  S.n = n;
  S.n_rules = nr;
  S.err = RL_OK;
  S.errmsg.clear();
  S.io = io ? *io : CommIO{};
  if (S.io.stats_host && !S.io_stats && dalloc(&S.io_stats, r->m_max) != hipSuccess)
    return breaks(r, e, RL_E_HIP, "gpu: routing stats staging allocation failed");
  // checks the partition does not make: a failure here still takes part in
  // the exchange (zero counts) and fails this rank's batch at rl_synchronize
  int hostrc = host_rc;
  if (hostrc) {
    // (rejected by the caller: the message is the engine's last error)
  } else if (n && (!out->code || !out->limit_remaining || (!out->reset_s && !S.io.host))) {  // (host slices: reset optional)
    hostrc = eng_fail(e, RL_E_INVALID, "gpu: null result array");
  } else if ((uint64_t)r->world * nr > e->cfg.max_rules) {
    hostrc = eng_fail(e, RL_E_CAPACITY, "gpu: routed batches need max_rules >= world x n_rules (per-source stats)");
  }
  if (hostrc) S.n_rules = 0;  // (a failed slice must not widen every owner's stats stride)
  const double t0 = now_s();
  int rc = first_half(r, e, S, s, in, caller, hostrc);
  r->t_first += now_s() - t0;
  if (rc) return rc;
  r->pend[r->n_pend++] = s;
  // the batch `lag` calls back: its counts had that many calls to arrive
  if (r->n_pend > r->lag) {
    const uint32_t p = r->pend[0];
    std::copy(r->pend + 1, r->pend + r->n_pend, r->pend);
    r->n_pend--;
    rc = second_half(r, e, r->slot[p], p);
    if (rc) return rc;
  }
  r->t_call += now_s() - tc;
  return RL_OK;
}

}  // namespace rl
