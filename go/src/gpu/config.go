package gpu

/*
#include <stdlib.h>
#include <string.h>
#include "ratelimit_hip.h"
*/
import "C"

import (
	"errors"
	"unsafe"

	"github.com/envoyproxy/ratelimit/src/config"
	"github.com/envoyproxy/ratelimit/src/stats"
)

// LoadConfig hands a loaded config to the GPU matcher (rl_config_load, the
// raw-request path rl_do_limit_requests): the trie flattened by config.Walk
// (src/config/walk.go), one rl_config_node per domain root and per
// rateLimitDescriptor (config_impl.go:45-48), parents before children, a
// node's key its domain or finalKey (config_impl.go:106-109). rule gives the
// dense stats row of a rule (the batcher's interner: the same ids DoLimit
// batches use). Call it from the goroutine that drives the ctx, on every
// reload (reloadConfig, src/service/ratelimit.go:49-90).
func (c *Ctx) LoadConfig(cfg config.RateLimitConfig, cacheKeyPrefix string,
	rule func(s stats.RateLimitStats) (uint32, bool)) error {
	type node struct {
		parent                     int
		key                        string
		rpu, rid                   uint32
		unit                       uint8
		hasLimit, unlimited, shadow bool
	}
	var nodes []node
	keyBytes := 0
	var ruleErr error
	ok := config.Walk(cfg, func(parent int, key string, l *config.RateLimit) int {
		n := node{parent: parent, key: key}
		if l != nil {
			n.hasLimit, n.unlimited, n.shadow = true, l.Unlimited, l.ShadowMode
			if l.Limit != nil {
				n.rpu, n.unit = l.Limit.RequestsPerUnit, uint8(l.Limit.Unit)
			}
			id, fits := rule(l.Stats) // keyed by l.Stats.Key (= FullKey, config_impl.go:111,139)
			if !fits {
				ruleErr = errors.New("gpu: more rules than max_rules")
			}
			n.rid = id
		}
		keyBytes += len(key)
		nodes = append(nodes, n)
		return len(nodes) - 1
	})
	if !ok {
		return errors.New("gpu: not a config loaded by src/config")
	}
	if ruleErr != nil {
		return ruleErr
	}
	// C memory for everything the library reads (a Go struct holding Go
	// pointers cannot be passed to C)
	cn := (*C.rl_config_node)(C.calloc(C.size_t(len(nodes)+1), C.size_t(unsafe.Sizeof(C.rl_config_node{}))))
	kb := (*C.uint8_t)(C.malloc(C.size_t(keyBytes + len(cacheKeyPrefix) + 1)))
	defer C.free(unsafe.Pointer(cn))
	defer C.free(unsafe.Pointer(kb))
	cns := (*[1 << 24]C.rl_config_node)(unsafe.Pointer(cn))[: len(nodes)+1 : len(nodes)+1]
	kbs := bytesAt(unsafe.Pointer(kb), keyBytes+len(cacheKeyPrefix)+1)
	off := 0
	for i, n := range nodes {
		x := &cns[i]
		x.parent = C.int32_t(n.parent)
		x.key_off = C.uint32_t(off)
		x.key_len = C.uint32_t(len(n.key))
		off += copy(kbs[off:], n.key)
		x.requests_per_unit = C.uint32_t(n.rpu)
		x.rule_id = C.uint32_t(n.rid)
		x.unit = C.uint8_t(n.unit)
		if n.hasLimit {
			x.has_limit = 1
		}
		if n.unlimited {
			x.unlimited = 1
		}
		if n.shadow {
			x.shadow_mode = 1
		}
	}
	copy(kbs[off:], cacheKeyPrefix)
	var tree C.rl_config_tree
	tree.n_nodes = C.uint32_t(len(nodes))
	tree.cache_key_prefix_len = C.uint32_t(len(cacheKeyPrefix))
	tree.nodes = cn
	tree.key_bytes = kb
	tree.key_bytes_len = C.uint64_t(keyBytes)
	tree.cache_key_prefix = (*C.uint8_t)(unsafe.Pointer(&kbs[off]))
	return c.err(C.rl_config_load(c.c, &tree))
}
