package gpu

/*
#include <string.h>
#include "ratelimit_hip.h"
*/
import "C"

import (
	"unsafe"

	pb_struct "github.com/envoyproxy/go-control-plane/envoy/extensions/common/ratelimit/v3"
	pb "github.com/envoyproxy/go-control-plane/envoy/service/ratelimit/v3"
)

// RequestBatch holds raw RateLimitRequests for rl_do_limit_requests: the
// service's GetLimit per descriptor (src/config/config_impl.go:243-298),
// DoLimit and the unlimited mapping of shouldRateLimitWorker
// (src/service/ratelimit.go:104-190), all on the GPU against the config the
// batcher loaded with LoadConfig. Host arrays in page-locked memory (cgo: C
// must not be handed Go memory that holds Go pointers, which the
// rl_request_batch struct would be), grown on demand. rl_do_limit_requests is
// synchronous: the outputs are final when DoLimitRequests returns.
type RequestBatch struct {
	In  C.rl_request_batch
	Out C.rl_request_result

	bufs []pinnedBuf

	// outputs per descriptor, in request-major order, and per-rule deltas
	Code      []uint8
	Remaining []uint32
	Reset     []uint32
	Match     []uint8
	RuleID    []uint32
	RPU       []uint32
	Unit      []uint8
	Stats     []uint64
	NDesc     int
}

// pinnedBuf is one growable page-locked array.
type pinnedBuf struct {
	p   unsafe.Pointer
	cap int
}

func (b *pinnedBuf) ensure(nbytes int) unsafe.Pointer {
	if nbytes > b.cap || b.p == nil {
		if b.p != nil {
			C.rl_free_host(b.p)
		}
		b.cap = nbytes + nbytes/4 + 64
		b.p = pinned(b.cap)
	}
	return b.p
}

const (
	rbDomain = iota
	rbDomainOff
	rbNow
	rbHits
	rbReqIdx
	rbEntryFirst
	rbDescOff
	rbDescBytes
	rbKeyLen
	rbValueLen
	rbOvFlags
	rbOvRPU
	rbOvUnit
	rbOvRule
	rbCode
	rbRem
	rbReset
	rbMatch
	rbRule
	rbRPU
	rbUnit
	rbStats
	rbCount
)

func NewRequestBatch() *RequestBatch { return &RequestBatch{bufs: make([]pinnedBuf, rbCount)} }

func u16At(p unsafe.Pointer, n int) []uint16 { return (*[1 << 30]uint16)(p)[:n:n] }
func i64At(p unsafe.Pointer, n int) []int64  { return (*[1 << 28]int64)(p)[:n:n] }

// Pack lays out the requests (arrival order) with their UnixNow(): per
// descriptor its entries' bytes Σ(key ‖ '_' ‖ value ‖ '_') (cache_key.go:65-70)
// with the key / value lengths, and its override (RateLimitDescriptor.Limit,
// config_impl.go:254-265) with the dense id overrideRule gives its stats key
// descriptorKey (config_impl.go:300-312). nRules: every rule id is below it.
func (b *RequestBatch) Pack(reqs []*pb.RateLimitRequest, nows []int64,
	overrideRule func(domain string, d *pb_struct.RateLimitDescriptor) uint32, nRules func() int) {
	nq, nd, ne, nDom, nBytes := len(reqs), 0, 0, 0, 0
	anyOverride := false
	for _, r := range reqs {
		nDom += len(r.Domain)
		nd += len(r.Descriptors)
		for _, d := range r.Descriptors {
			ne += len(d.Entries)
			for _, e := range d.Entries {
				nBytes += len(e.Key) + len(e.Value) + 2
			}
			if d.GetLimit() != nil {
				anyOverride = true
			}
		}
	}
	dom := bytesAt(b.bufs[rbDomain].ensure(nDom+1), nDom+1)
	domOff := u32At(b.bufs[rbDomainOff].ensure(4*(nq+1)), nq+1)
	now := i64At(b.bufs[rbNow].ensure(8*nq+8), nq)
	hits := u32At(b.bufs[rbHits].ensure(4*nq+4), nq)
	reqIdx := u32At(b.bufs[rbReqIdx].ensure(4*nd+4), nd)
	entryFirst := u32At(b.bufs[rbEntryFirst].ensure(4*(nd+1)), nd+1)
	descOff := u32At(b.bufs[rbDescOff].ensure(4*(nd+1)), nd+1)
	descBytes := bytesAt(b.bufs[rbDescBytes].ensure(nBytes+1), nBytes+1)
	keyLen := u16At(b.bufs[rbKeyLen].ensure(2*ne+2), ne)
	valueLen := u16At(b.bufs[rbValueLen].ensure(2*ne+2), ne)
	var ovFlags, ovUnit []uint8
	var ovRPU, ovRule []uint32
	if anyOverride {
		ovFlags = bytesAt(b.bufs[rbOvFlags].ensure(nd+1), nd)
		ovRPU = u32At(b.bufs[rbOvRPU].ensure(4*nd+4), nd)
		ovUnit = bytesAt(b.bufs[rbOvUnit].ensure(nd+1), nd)
		ovRule = u32At(b.bufs[rbOvRule].ensure(4*nd+4), nd)
	}
	pd, pb_, pe, pdesc := 0, 0, 0, 0
	domOff[0], entryFirst[0], descOff[0] = 0, 0, 0
	for q, r := range reqs {
		pd += copy(dom[pd:], r.Domain)
		domOff[q+1] = uint32(pd)
		now[q] = nows[q]
		hits[q] = r.HitsAddend // (the library applies utils.Max(1, h), fixed_cache_impl.go:41)
		for _, d := range r.Descriptors {
			reqIdx[pdesc] = uint32(q)
			for _, e := range d.Entries {
				pb_ += copy(descBytes[pb_:], e.Key)
				descBytes[pb_] = '_'
				pb_++
				pb_ += copy(descBytes[pb_:], e.Value)
				descBytes[pb_] = '_'
				pb_++
				keyLen[pe] = uint16(len(e.Key))
				valueLen[pe] = uint16(len(e.Value))
				pe++
			}
			entryFirst[pdesc+1] = uint32(pe)
			descOff[pdesc+1] = uint32(pb_)
			if anyOverride {
				ovFlags[pdesc], ovRPU[pdesc], ovUnit[pdesc], ovRule[pdesc] = 0, 0, 0, 0
				if l := d.GetLimit(); l != nil {
					ovFlags[pdesc] = 1
					ovRPU[pdesc] = l.GetRequestsPerUnit()
					ovUnit[pdesc] = uint8(l.GetUnit())
					ovRule[pdesc] = overrideRule(r.Domain, d)
				}
			}
			pdesc++
		}
	}
	b.In.n_requests = C.uint32_t(nq)
	b.In.n_descriptors = C.uint32_t(nd)
	b.In.n_entries = C.uint32_t(ne)
	b.In.n_rules = C.uint32_t(nRules())
	b.In.domain_bytes = (*C.uint8_t)(unsafe.Pointer(&dom[0]))
	b.In.domain_off = (*C.uint32_t)(unsafe.Pointer(&domOff[0]))
	b.In.now = (*C.int64_t)(b.bufs[rbNow].p)
	b.In.hits = (*C.uint32_t)(b.bufs[rbHits].p)
	b.In.req_idx = (*C.uint32_t)(b.bufs[rbReqIdx].p)
	b.In.entry_first = (*C.uint32_t)(unsafe.Pointer(&entryFirst[0]))
	b.In.desc_off = (*C.uint32_t)(unsafe.Pointer(&descOff[0]))
	b.In.desc_bytes = (*C.uint8_t)(unsafe.Pointer(&descBytes[0]))
	b.In.key_len = (*C.uint16_t)(b.bufs[rbKeyLen].p)
	b.In.value_len = (*C.uint16_t)(b.bufs[rbValueLen].p)
	b.In.override_flags, b.In.override_rpu, b.In.override_unit, b.In.override_rule = nil, nil, nil, nil
	if anyOverride {
		b.In.override_flags = (*C.uint8_t)(b.bufs[rbOvFlags].p)
		b.In.override_rpu = (*C.uint32_t)(b.bufs[rbOvRPU].p)
		b.In.override_unit = (*C.uint8_t)(b.bufs[rbOvUnit].p)
		b.In.override_rule = (*C.uint32_t)(b.bufs[rbOvRule].p)
	}
	// outputs
	m := int(b.In.n_rules) * int(C.RL_NUM_STATS)
	b.NDesc = nd
	b.Code = bytesAt(b.bufs[rbCode].ensure(nd+1), nd)
	b.Remaining = u32At(b.bufs[rbRem].ensure(4*nd+4), nd)
	b.Reset = u32At(b.bufs[rbReset].ensure(4*nd+4), nd)
	b.Match = bytesAt(b.bufs[rbMatch].ensure(nd+1), nd)
	b.RuleID = u32At(b.bufs[rbRule].ensure(4*nd+4), nd)
	b.RPU = u32At(b.bufs[rbRPU].ensure(4*nd+4), nd)
	b.Unit = bytesAt(b.bufs[rbUnit].ensure(nd+1), nd)
	b.Stats = u64At(b.bufs[rbStats].ensure(8*m+8), m)
	b.Out.code = (*C.uint8_t)(b.bufs[rbCode].p)
	b.Out.limit_remaining = (*C.uint32_t)(b.bufs[rbRem].p)
	b.Out.reset_s = (*C.uint32_t)(b.bufs[rbReset].p)
	b.Out.match = (*C.uint8_t)(b.bufs[rbMatch].p)
	b.Out.rule_id = (*C.uint32_t)(b.bufs[rbRule].p)
	b.Out.requests_per_unit = (*C.uint32_t)(b.bufs[rbRPU].p)
	b.Out.unit = (*C.uint8_t)(b.bufs[rbUnit].p)
	b.Out.stats = (*C.uint64_t)(b.bufs[rbStats].p)
}

// Match results (rl_match).
const (
	MatchNone      = uint8(C.RL_MATCH_NONE)
	MatchUnlimited = uint8(C.RL_MATCH_UNLIMITED)
	MatchLimit     = uint8(C.RL_MATCH_LIMIT)
)

// DoLimitRequests runs a packed RequestBatch (synchronous; not on a routed ctx).
func (c *Ctx) DoLimitRequests(b *RequestBatch) error {
	return c.err(C.rl_do_limit_requests(c.c, &b.In, &b.Out))
}
