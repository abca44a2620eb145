// rl_transport.h — the point-to-point exchanges of a routed step
// (rl_comm.hip), behind one interface with two implementations:
//
//   RCCL      one process per GPU, grouped ncclSend / ncclRecv over xGMI (the
//             8-GPU node; what bench.py --gpus N runs);
//   loopback  W ranks inside ONE process (one host thread and one single-shard
//             ctx each, any devices, several may share one GPU): device-to-
//             device copies through an in-process mailbox with the same
//             grouped send/recv contract. RCCL refuses two ranks on one
//             device, so this is how the multi-rank protocol runs on a
//             one-GPU machine (tests, bench.py --loopback W).
//
// Contract of group(ch, ops, stream) (both transports): every send to peer p
// matches p's receive from this rank of the same byte count, in order, on the
// same channel ch (0 = counts, 1 = records and stems, 2 = results and stats);
// channels are independent. Sends are ordered after the work already on
// `stream`; once `stream` passes the group, every receive has landed and
// every send buffer may be reused. Zero-byte operations are not posted (both
// sides skip them: the counts that size them were exchanged first).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace rl {

struct Xfer {
  void* buf;       // device memory (send: source, recv: destination)
  uint64_t bytes;
  uint32_t peer;
  bool send;
};

constexpr uint32_t TRANSPORT_CHANNELS = 3;

class Transport {
 public:
  virtual ~Transport() {}
  // RL_OK, or an rl_status with *err set (RL_E_COMM: the world is unusable)
  virtual int group(uint32_t ch, const std::vector<Xfer>& ops, hipStream_t stream, std::string* err) = 0;
  virtual const char* kind() const = 0;
};

// An id of RL_COMM_ID_BYTES for rl_comm_init: RCCL's ncclUniqueId, or a
// loopback world's (magic prefix, then the world's serial number).
bool loopback_id(const uint8_t* id);
int loopback_new_id(uint8_t* id, std::string* err);

// Joins the loopback world `id` as rank `rank` of `world` (every rank calls
// it once; the world's size is fixed by the first). Null + *err on failure.
Transport* loopback_join(const uint8_t* id, uint32_t world, uint32_t rank, std::string* err);

// RCCL (dlopen'ed): the unique id, and a transport of three communicators
// (one per channel) split from one ncclCommInitRank (collective).
int rccl_unique_id(uint8_t* id, std::string* err);
Transport* rccl_join(const uint8_t* id, uint32_t world, uint32_t rank, int device, std::string* err);

}  // namespace rl
