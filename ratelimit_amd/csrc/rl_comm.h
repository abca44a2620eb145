// rl_comm.h — multi-process routing over RCCL inside the library
// (rl_comm_* / rl_do_limit_routed_async, include/ratelimit_hip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ratelimit_hip.h"
#include "rl_engine.h"

namespace rl {

struct CommRouter;

// ncclGetUniqueId through the RCCL library loaded in the process (dlopen).
int comm_unique_id(uint8_t* id, std::string* err);
// The id of a new in-process loopback world (rl_transport.h).
int comm_loopback_id(uint8_t* id, std::string* err);
// Collective over `world` ranks: joins engine e (one GPU) to the world `id`
// (an RCCL unique id: one process per GPU; a loopback id: ranks are threads of
// this process) as `rank`. Null + *err on failure.
CommRouter* comm_create(Engine* e, uint32_t world, uint32_t rank, const uint8_t* id, std::string* err);
void comm_destroy(CommRouter* r);
const char* comm_kind(const CommRouter* r);  // "rccl" or "loopback"
// rl_sweep on a routed ctx (collective): the least `now` over the ranks
int comm_sweep_floor(CommRouter* r, Engine* e, int64_t now, int64_t* floor);
// A slice that is not plain device memory of this rank's GPU (the shards of
// one ctx, rl_api.hip). host: `in` and `out` are host memory; `in` is an
// absolute-index view of the caller's whole batch (stem_off / req_idx / unit /
// ... point at the slice's first descriptor `da`, now / stem_bytes at the
// whole batch's start, n_requests = one past the slice's last request, whose
// first is `qa`), staged into the slot's device buffers at the same absolute
// offsets, so no index is rewritten; `out` is the slice's part of the host
// results. Device (host false): `in` / `out` are device memory of any GPU with
// peer access (read and written in place). stats_host (pinned, n_rules x
// RL_NUM_STATS) receives this rank's stats deltas instead of out->stats.
struct CommIO {
  bool host = false;
  uint32_t da = 0, qa = 0;
  unsigned long long* stats_host = nullptr;
  // a compact host batch (rl_batch_compact): this slice is its descriptors
  // [da, in->n + da) and requests [qa, in->n_requests), unpacked on the device
  const rl_batch_compact* cb = nullptr;
  // a prefix-shared host batch (rl_batch_prefixed): this slice is its request
  // tiles [t0, t1) (descriptors [da, in->n + da), requests [qa, in->n_requests))
  const rl_batch_prefixed* pb = nullptr;
  uint32_t t0 = 0, t1 = 0;
};
// One routed batch: this rank's slice (device arrays, or io) -> out in arrival
// order. Enqueues the batch's first half and runs the previous batch's second
// half. host_rc != RL_OK: the caller rejected the slice (its message already
// in the engine's last error); it still takes part in the exchange, with no
// records, and fails at rl_synchronize.
int comm_do_limit(CommRouter* r, Engine* e, const rl_batch* in, rl_result* out, hipStream_t caller,
                  const CommIO* io = nullptr, int host_rc = 0);
// Batches a router keeps in flight (its slots, used round robin), and a wait
// on the host for the last batch that used slot s (its outputs and, with
// io.stats_host, its stats are then in place). Valid once the batch's second
// half ran (the next call or comm_synchronize).
uint32_t comm_slots();
int comm_wait_slot(CommRouter* r, Engine* e, uint32_t s);
// Completes the pending batch (collective) and waits for the router's streams
// (then the engine's own synchronize reports errors).
int comm_synchronize(CommRouter* r, Engine* e);

}  // namespace rl
