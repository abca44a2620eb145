// rl_transport.hip — the RCCL and in-process loopback transports of the
// routed step (rl_transport.h).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ratelimit_hip.h"
#include "rl_transport.h"

namespace rl {

namespace {

// ---- RCCL --------------------------------------------------------------------
// Loaded with dlopen, preferring an instance already in the process (torch's,
// which shares the HIP runtime this library binds to), so the library loads
// and runs single-GPU without RCCL present.
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

// One communicator per channel, so that no exchange waits in RCCL's
// per-communicator order behind another kind of traffic.
class RcclTransport : public Transport {
 public:
  ncclComm_t comm[TRANSPORT_CHANNELS] = {};
  ~RcclTransport() override {
    for (uint32_t c = TRANSPORT_CHANNELS; c-- > 0;)
      if (comm[c]) (void)rccl().destroy(comm[c]);
  }
  const char* kind() const override { return "rccl"; }
  int group(uint32_t ch, const std::vector<Xfer>& ops, hipStream_t st, std::string* err) override {
    Rccl& R = rccl();
    ncclResult_t rc = R.gstart();
    for (const Xfer& x : ops) {
      if (rc != ncclSuccess) break;
      if (!x.bytes) continue;
      rc = x.send ? R.send(x.buf, x.bytes, ncclUint8, (int)x.peer, comm[ch], st)
                  : R.recv(x.buf, x.bytes, ncclUint8, (int)x.peer, comm[ch], st);
    }
    const ncclResult_t re = R.gend();
    if (rc == ncclSuccess) rc = re;
    if (rc != ncclSuccess) {
      *err = std::string("gpu: RCCL grouped send/recv: ") + R.estr(rc);
      return RL_E_COMM;
    }
    return RL_OK;
  }
};

// ---- loopback ----------------------------------------------------------------
// A message of one send: the receiver copies it on its own stream after the
// sender's `ready` event and answers with `done`, which the sender's stream
// then waits for (a send completes once received, as in RCCL). Every event is
// recorded before it is posted, so no stream ever waits on work submitted
// after the wait (the hardware queues are shared by every rank's streams).
struct LoopMsg {
  const void* src = nullptr;
  uint64_t bytes = 0;
  hipEvent_t ready = nullptr;
  hipEvent_t done = nullptr;
  bool done_set = false;
};

struct LoopWorld {
  uint64_t serial = 0;
  uint32_t world = 0;  // fixed by the first join
  uint32_t left = 0;
  std::vector<uint8_t> joined;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::deque<std::shared_ptr<LoopMsg>>> q;  // [ch][src][dst]
  bool aborted = false;
  std::string abort_msg;
};

constexpr char LOOP_MAGIC[8] = {'R', 'L', 'L', 'O', 'O', 'P', 'B', 'K'};

std::mutex g_reg_mu;
std::map<uint64_t, std::shared_ptr<LoopWorld>> g_reg;
uint64_t g_serial = 0;

double loop_timeout_s() {
  const char* t = getenv("RL_LOOPBACK_TIMEOUT_S");
  const double v = t ? atof(t) : 0.0;
  return v > 0 ? v : 120.0;
}

class LoopTransport : public Transport {
 public:
  std::shared_ptr<LoopWorld> w;
  uint32_t rank = 0;
  std::chrono::duration<double> timeout{120.0};

  ~LoopTransport() override {
    std::lock_guard<std::mutex> g(g_reg_mu);
    std::lock_guard<std::mutex> l(w->mu);
    if (++w->left == w->world) g_reg.erase(w->serial);
  }
  const char* kind() const override { return "loopback"; }

  size_t qi(uint32_t ch, uint32_t src, uint32_t dst) const { return ((size_t)ch * w->world + src) * w->world + dst; }

  int abort_world(std::unique_lock<std::mutex>& l, const std::string& msg, std::string* err) {
    if (!w->aborted) {
      w->aborted = true;
      w->abort_msg = msg;
    }
    w->cv.notify_all();
    *err = w->abort_msg;
    (void)l;
    return RL_E_COMM;
  }

  int group(uint32_t ch, const std::vector<Xfer>& ops, hipStream_t st, std::string* err) override {
    auto hip_fail = [&](const char* what, hipError_t e) {
      std::unique_lock<std::mutex> l(w->mu);
      return abort_world(l, std::string("gpu: loopback ") + what + ": " + hipGetErrorString(e), err);
    };
    hipError_t he;
    // 1. post every send (never blocks)
    std::vector<std::shared_ptr<LoopMsg>> mine;
    for (const Xfer& x : ops) {
      if (!x.send || !x.bytes) continue;
      auto m = std::make_shared<LoopMsg>();
      m->src = x.buf;
      m->bytes = x.bytes;
      if ((he = hipEventCreateWithFlags(&m->ready, hipEventDisableTiming)) != hipSuccess ||
          (he = hipEventRecord(m->ready, st)) != hipSuccess)
        return hip_fail("send event", he);
      std::lock_guard<std::mutex> l(w->mu);
      w->q[qi(ch, rank, x.peer)].push_back(m);
      mine.push_back(m);
    }
    w->cv.notify_all();
    const auto deadline = std::chrono::steady_clock::now() + timeout;
    // 2. receive, in order per peer: copy after the sender's ready event
    for (const Xfer& x : ops) {
      if (x.send || !x.bytes) continue;
      std::shared_ptr<LoopMsg> m;
      {
        std::unique_lock<std::mutex> l(w->mu);
        auto& dq = w->q[qi(ch, x.peer, rank)];
        if (!w->cv.wait_until(l, deadline, [&] { return w->aborted || !dq.empty(); }))
          return abort_world(l, "gpu: loopback peer " + std::to_string(x.peer) + " did not send within the timeout",
                             err);
        if (w->aborted) return abort_world(l, "", err);
        m = dq.front();
        dq.pop_front();
        if (m->bytes != x.bytes)
          return abort_world(l, "gpu: loopback message size mismatch (" + std::to_string(m->bytes) + " sent, " +
                                    std::to_string(x.bytes) + " expected)", err);
      }
      hipEvent_t d = nullptr;
      if ((he = hipStreamWaitEvent(st, m->ready, 0)) != hipSuccess ||
          (he = hipMemcpyAsync(x.buf, m->src, x.bytes, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
          (he = hipEventCreateWithFlags(&d, hipEventDisableTiming)) != hipSuccess ||
          (he = hipEventRecord(d, st)) != hipSuccess)
        return hip_fail("receive", he);
      std::lock_guard<std::mutex> l(w->mu);
      m->done = d;
      m->done_set = true;
      w->cv.notify_all();
    }
    // 3. a send completes once its receiver's copy has run
    for (auto& m : mine) {
      {
        std::unique_lock<std::mutex> l(w->mu);
        if (!w->cv.wait_until(l, deadline, [&] { return w->aborted || m->done_set; }))
          return abort_world(l, "gpu: loopback peer did not receive within the timeout", err);
        if (w->aborted) return abort_world(l, "", err);
      }
      if ((he = hipStreamWaitEvent(st, m->done, 0)) != hipSuccess) return hip_fail("send completion", he);
      // (streams already waiting on them keep the events alive)
      (void)hipEventDestroy(m->ready);
      (void)hipEventDestroy(m->done);
    }
    return RL_OK;
  }
};

}  // namespace

bool loopback_id(const uint8_t* id) { return memcmp(id, LOOP_MAGIC, sizeof(LOOP_MAGIC)) == 0; }

int loopback_new_id(uint8_t* id, std::string* err) {
  (void)err;
  auto w = std::make_shared<LoopWorld>();
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    w->serial = ++g_serial;
    g_reg[w->serial] = w;
  }
  memset(id, 0, RL_COMM_ID_BYTES);
  memcpy(id, LOOP_MAGIC, sizeof(LOOP_MAGIC));
  memcpy(id + sizeof(LOOP_MAGIC), &w->serial, sizeof(w->serial));
  return RL_OK;
}

Transport* loopback_join(const uint8_t* id, uint32_t world, uint32_t rank, std::string* err) {
  uint64_t serial = 0;
  memcpy(&serial, id + sizeof(LOOP_MAGIC), sizeof(serial));
  std::shared_ptr<LoopWorld> w;
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.find(serial);
    if (it == g_reg.end()) {
      *err = "gpu: unknown loopback id (rl_comm_loopback_id, same process)";
      return nullptr;
    }
    w = it->second;
    std::lock_guard<std::mutex> l(w->mu);
    if (!w->world) {
      w->world = world;
      w->joined.assign(world, 0);
      w->q.resize((size_t)TRANSPORT_CHANNELS * world * world);
    }
    if (w->world != world || rank >= world || w->joined[rank]) {
      *err = "gpu: loopback join: world size differs from the first rank's, or rank taken";
      return nullptr;
    }
    w->joined[rank] = 1;
  }
  auto* t = new LoopTransport();
  t->w = w;
  t->rank = rank;
  t->timeout = std::chrono::duration<double>(loop_timeout_s());
  return t;
}

int rccl_unique_id(uint8_t* id, std::string* err) {
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

Transport* rccl_join(const uint8_t* id, uint32_t world, uint32_t rank, int device, std::string* err) {
  Rccl& R = rccl();
  if (!R.ok) {
    *err = R.err;
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    *err = "gpu: hipSetDevice failed";
    return nullptr;
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  auto* t = new RcclTransport();
  // collective: every rank splits alike
  ncclResult_t nr = R.init(&t->comm[0], (int)world, u, (int)rank);
  for (uint32_t c = 1; c < TRANSPORT_CHANNELS && nr == ncclSuccess; c++)
    nr = R.split(t->comm[0], 0, (int)rank, &t->comm[c], nullptr);
  if (nr != ncclSuccess) {
    *err = std::string("gpu: RCCL communicator setup: ") + R.estr(nr);
    delete t;
    return nullptr;
  }
  return t;
}

}  // namespace rl
