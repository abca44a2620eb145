package gpu

/*
#include <stdlib.h>
#include "ratelimit_hip.h"
*/
import "C"

import (
	"runtime"
	"unsafe"
)

// One service process per GPU (SURVEY §8e): every rank's ctx shares
// Config.HashSeed, rank 0 draws a communicator id and the coordinator hands
// it to every rank; the library then routes each batch to the GPU owning its
// keys over RCCL (xGMI) and back. Replaces the Redis cluster client's
// key-slot routing (src/redis/driver_impl.go:108-126).

// CommIDBytes is the size of a communicator id (an ncclUniqueId).
const CommIDBytes = int(C.RL_COMM_ID_BYTES)

// CommUniqueID draws the id on one rank. rl_last_error(NULL) is the calling
// OS thread's message, so the goroutine stays on one thread from the call to
// the read (cgo runs C on the current thread).
func CommUniqueID() ([]byte, error) {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	id := (*C.uint8_t)(C.malloc(C.size_t(CommIDBytes)))
	defer C.free(unsafe.Pointer(id))
	if rc := C.rl_comm_unique_id(id); rc != C.RL_OK {
		return nil, &Error{Status: int(rc), Msg: C.GoString(C.rl_last_error(nil))}
	}
	return C.GoBytes(unsafe.Pointer(id), C.int(CommIDBytes)), nil
}

// CommInit joins the ctx to the world as rank (collective: every rank, the same id).
func (c *Ctx) CommInit(world, rank int, id []byte) error {
	if len(id) != CommIDBytes {
		return &Error{Status: int(C.RL_E_INVALID), Msg: "gpu: communicator id of the wrong size"}
	}
	cid := (*C.uint8_t)(C.CBytes(id))
	defer C.free(unsafe.Pointer(cid))
	return c.err(C.rl_comm_init(c.c, C.uint32_t(world), C.uint32_t(rank), cid))
}

// RoutedDoLimit submits this rank's slice of the node batch (device arrays in
// *in, *out; stream a hipStream_t or nil). Collective: every rank calls it the
// same number of times; Synchronize (collective too) completes the last one.
func (c *Ctx) RoutedDoLimit(in *C.rl_batch, out *C.rl_result, stream unsafe.Pointer) error {
	return c.err(C.rl_do_limit_routed_async(c.c, in, out, stream))
}
