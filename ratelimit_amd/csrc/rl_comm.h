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
// One routed batch: this rank's slice (device arrays) -> out in arrival order.
// Enqueues the batch's first half and runs the previous batch's second half.
int comm_do_limit(CommRouter* r, Engine* e, const rl_batch* in, rl_result* out, hipStream_t caller);
// Completes the pending batch (collective) and waits for the router's streams
// (then the engine's own synchronize reports errors).
int comm_synchronize(CommRouter* r, Engine* e);

}  // namespace rl
