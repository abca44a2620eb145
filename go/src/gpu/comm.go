package gpu

/*
#include <stdlib.h>
#include "ratelimit_hip.h"
*/
import "C"

import (
	"errors"
	"io/ioutil"
	"os"
	"runtime"
	"time"
	"unsafe"
)

// One service process per GPU (SURVEY §8e): every rank's ctx shares
// Config.HashSeed, rank 0 draws a communicator id and hands it to every rank
// (CommIDFile: through a file on shared storage); the library then routes
// each batch to the GPU owning its keys over RCCL (xGMI) and back. Replaces
// the Redis cluster client's key-slot routing (src/redis/driver_impl.go:108-126).
//
// A routed ctx takes the batcher's own prefix-shared batches: Submit on it is
// rl_do_limit_prefixed_async on a ctx that joined a communicator, and each
// rank's batch is its slice of the node batch. Submit, Synchronize and Sweep
// are collective there (every rank calls them the same number of times, in
// the same order), so the batcher of a routed ctx submits one batch per tick
// of GPU_BATCH_WINDOW, empty when its process received no call, and sweeps
// on a tick count (cache_impl.go batcherRouted).

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

// CommIDFile hands the communicator id from rank 0 to the other ranks through
// path: rank 0 draws it and writes it (write then rename, so no rank reads a
// partial id); every other rank waits up to timeout for the file. A stale
// file from an earlier run must be removed before rank 0 starts.
func CommIDFile(path string, rank int, timeout time.Duration) ([]byte, error) {
	if rank == 0 {
		id, err := CommUniqueID()
		if err != nil {
			return nil, err
		}
		if err := ioutil.WriteFile(path+".tmp", id, 0600); err != nil {
			return nil, err
		}
		return id, os.Rename(path+".tmp", path)
	}
	deadline := time.Now().Add(timeout)
	for {
		id, err := ioutil.ReadFile(path)
		if err == nil && len(id) == CommIDBytes {
			return id, nil
		}
		if time.Now().After(deadline) {
			return nil, errors.New("gpu: no communicator id in " + path + " (is rank 0 up?)")
		}
		time.Sleep(50 * time.Millisecond)
	}
}

// CommInit joins the ctx to the world as rank (collective: every rank, the same id).
func (c *Ctx) CommInit(world, rank int, id []byte) error {
	if len(id) != CommIDBytes {
		return &Error{Status: int(C.RL_E_INVALID), Msg: "gpu: communicator id of the wrong size"}
	}
	cid := (*C.uint8_t)(C.CBytes(id))
	defer C.free(unsafe.Pointer(cid))
	if err := c.err(C.rl_comm_init(c.c, C.uint32_t(world), C.uint32_t(rank), cid)); err != nil {
		return err
	}
	c.routed = world > 1
	return nil
}

// Routed reports whether the ctx joined a world of two or more ranks (its
// Submit, Synchronize and Sweep are collective).
func (c *Ctx) Routed() bool { return c.routed }
