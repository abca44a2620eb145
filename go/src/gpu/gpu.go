// Package gpu binds libratelimit_hip.so, the MI355X fixed-window rate-limit
// backend, to the reference service. It is added to the reference tree as
// src/gpu (Go 1.14, go.mod:3: no generics, no unsafe.Slice) next to
// src/redis and src/memcached; cache_impl.go implements
// limiter.RateLimitCache (src/limiter/cache.go:11-29) on top of it.
//
// The C side is include/ratelimit_hip.h; the library and the header are
// vendored under third_party/ratelimit_hip (INTEGRATION.md §4).
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/ratelimit_hip/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/ratelimit_hip/lib -lratelimit_hip -Wl,-rpath,${SRCDIR}/../../third_party/ratelimit_hip/lib
#include <stdlib.h>
#include <string.h>
#include "ratelimit_hip.h"
*/
import "C"

import (
	"errors"
	"unsafe"
)

// Config mirrors rl_config: the knobs NewFixedRateLimitCacheImpl receives
// (src/redis/fixed_cache_impl.go:118-125) plus the HBM sizing.
type Config struct {
	TableSlots     uint64  // 64-B slots (power of 2)
	HistoryEntries uint64  // 32-B history log entries: windows below a key's newest (0: TableSlots)
	ArenaBytes     uint64  // overflow arena for stems longer than 36 B (0: library default)
	MaxBatch       uint32  // descriptors per batch
	MaxRequests    uint32  // requests per batch (0: MaxBatch)
	MaxRules       uint32  // distinct rule ids (stats rows)
	MaxStemBytes   uint32  // unpacked stem bytes per batch (0: 128 x MaxBatch)
	NearLimitRatio float32 // NEAR_LIMIT_RATIO (settings.go:48)
	LocalCache     bool    // LOCAL_CACHE_SIZE_IN_BYTES != 0 (runner.go:95-98)
	PerSecond      bool    // REDIS_PERSECOND: SECOND keys in their own store
	JitterMax      int64   // EXPIRATION_JITTER_MAX_SECONDS (the draw is 0; older windows kept div + JitterMax s)
	Device         int     // HIP device ordinal
	HashSeed       uint64  // stem-hash key; 0: a random secret per ctx
	ShardDevices   []int   // > 1 entries: one table shard per device, routed inside the ctx
}

// The library's defaults for a zero Config field (include/ratelimit_hip.h rl_config).
const (
	DefaultMaxBatch = 1 << 20
	DefaultMaxRules = 65536
)

// Resolved returns cfg with the zero sizing fields the batcher's own buffers
// depend on replaced by the library's defaults (rl_create applies the same).
func (cfg Config) Resolved() Config {
	if cfg.MaxBatch == 0 {
		cfg.MaxBatch = DefaultMaxBatch
	}
	if cfg.MaxRules == 0 {
		cfg.MaxRules = DefaultMaxRules
	}
	return cfg
}

// Ctx owns one rl_ctx. One goroutine drives it at a time (the batcher).
type Ctx struct {
	c      *C.rl_ctx
	routed bool // joined a world of two or more ranks (comm.go)
}

func New(cfg Config) (*Ctx, error) {
	var rc C.rl_config
	rc.table_slots = C.uint64_t(cfg.TableSlots)
	rc.history_entries = C.uint64_t(cfg.HistoryEntries)
	rc.arena_bytes = C.uint64_t(cfg.ArenaBytes)
	rc.max_batch = C.uint32_t(cfg.MaxBatch)
	rc.max_requests = C.uint32_t(cfg.MaxRequests)
	rc.max_rules = C.uint32_t(cfg.MaxRules)
	rc.max_stem_bytes = C.uint32_t(cfg.MaxStemBytes)
	rc.near_limit_ratio = C.float(cfg.NearLimitRatio)
	if cfg.LocalCache {
		rc.local_cache_enabled = 1
	}
	if cfg.PerSecond {
		rc.per_second_split = 1
	}
	rc.expiration_jitter_max_seconds = C.int64_t(cfg.JitterMax)
	rc.device = C.int32_t(cfg.Device)
	rc.hash_seed = C.uint64_t(cfg.HashSeed)
	if len(cfg.ShardDevices) > 16 {
		return nil, errors.New("gpu: at most 16 shards per ctx")
	}
	if len(cfg.ShardDevices) > 1 {
		rc.n_shards = C.uint32_t(len(cfg.ShardDevices))
		for i, d := range cfg.ShardDevices {
			rc.shard_device[i] = C.int32_t(d)
		}
	}
	var msg [512]C.char
	ctx := C.rl_create(&rc, &msg[0], C.size_t(len(msg)))
	if ctx == nil {
		return nil, errors.New(C.GoString(&msg[0]))
	}
	return &Ctx{c: ctx}, nil
}

func (c *Ctx) Close() {
	if c.c != nil {
		C.rl_destroy(c.c)
		c.c = nil
	}
}

func (c *Ctx) err(rc C.int) error {
	if rc == C.RL_OK {
		return nil
	}
	return &Error{Status: int(rc), Msg: C.GoString(C.rl_last_error(c.c))}
}

// rl_status codes of a device-level failure (the GPU or its runtime, not a
// request): the batcher's health monitor fails the server's health check on them.
const (
	StatusHIP      = int(C.RL_E_HIP)
	StatusComm     = int(C.RL_E_COMM)
	StatusInternal = int(C.RL_E_INTERNAL)
)

// Error is a library failure: the adapter turns it into
// panic(redis.RedisError(...)) (src/redis/driver_impl.go:60-64).
type Error struct {
	Status int // rl_status
	Msg    string
}

func (e *Error) Error() string { return e.Msg }

// Synchronize completes every submitted batch; device-side failures of any
// of them are reported here.
func (c *Ctx) Synchronize() error { return c.err(C.rl_synchronize(c.c)) }

// Progress returns how many batches were submitted and how many of them, in
// order, have their outputs back in host memory (never waits).
func (c *Ctx) Progress() (submitted, completed uint64, err error) {
	var s, d C.uint64_t
	err = c.err(C.rl_batch_progress(c.c, &s, &d))
	return uint64(s), uint64(d), err
}

// Sweep evicts every slot whose windows and local-cache entries have expired
// at now (the EXPIRE housekeeping); now becomes the ctx's time floor.
func (c *Ctx) Sweep(now int64) (uint64, error) {
	var ev C.uint64_t
	err := c.err(C.rl_sweep(c.c, C.int64_t(now), &ev))
	return uint64(ev), err
}

// LocalCacheInfo: the localCacheStats gauges (src/limiter/local_cache_stats.go:36-43).
type LocalCacheInfo struct {
	EntryCount, LookupCount, HitCount, MissCount uint64
}

func (c *Ctx) LocalCacheInfo(now int64) (LocalCacheInfo, error) {
	var lc C.rl_local_cache_info
	if err := c.err(C.rl_local_cache_info_get(c.c, C.int64_t(now), &lc)); err != nil {
		return LocalCacheInfo{}, err
	}
	return LocalCacheInfo{EntryCount: uint64(lc.entry_count), LookupCount: uint64(lc.lookup_count),
		HitCount: uint64(lc.hit_count), MissCount: uint64(lc.miss_count)}, nil
}

// TableInfo: live slots, tombstones and arena use, summed over shards.
type TableInfo struct {
	TableSlots, LiveSlots, Tombstones, ArenaBytesUsed, ExactStems, Batches, Decisions uint64
	HistoryEntries, HistoryAppended, HistoryLost, HistorySlots, HistoryRefused      uint64
}

func (c *Ctx) TableInfo() (TableInfo, error) {
	var ti C.rl_table_info
	if err := c.err(C.rl_table_info_get(c.c, &ti)); err != nil {
		return TableInfo{}, err
	}
	return TableInfo{TableSlots: uint64(ti.table_slots), LiveSlots: uint64(ti.live_slots),
		Tombstones: uint64(ti.tombstones), ArenaBytesUsed: uint64(ti.arena_bytes_used),
		ExactStems: uint64(ti.exact_stems), Batches: uint64(ti.batches), Decisions: uint64(ti.decisions),
		HistoryEntries: uint64(ti.history_entries), HistoryAppended: uint64(ti.history_appended),
		HistoryLost: uint64(ti.history_lost), HistorySlots: uint64(ti.history_slots),
		HistoryRefused: uint64(ti.history_refused)}, nil
}

// ---- pinned host memory: Go never hands Go-heap pointers to C (cgo pointer
// rules), and the batches' PCIe copies are asynchronous from page-locked
// memory. Go 1.14 has no unsafe.Slice: slice a pointer to a large array.

func pinned(nbytes int) unsafe.Pointer {
	if nbytes == 0 {
		nbytes = 4
	}
	p := C.rl_alloc_host(C.size_t(nbytes))
	if p == nil {
		panic("gpu: rl_alloc_host failed")
	}
	C.memset(p, 0, C.size_t(nbytes))
	return p
}

func bytesAt(p unsafe.Pointer, n int) []byte        { return (*[1 << 31]byte)(p)[:n:n] }
func u32At(p unsafe.Pointer, n int) []uint32        { return (*[1 << 29]uint32)(p)[:n:n] }
func u64At(p unsafe.Pointer, n int) []uint64        { return (*[1 << 28]uint64)(p)[:n:n] }
func limitsAt(p unsafe.Pointer, n int) []C.rl_limit { return (*[1 << 24]C.rl_limit)(p)[:n:n] }

// ---- the prefix-shared batch (rl_batch_prefixed): the fed path's PCIe
// layout. Per request its shared stem prefix once, its clock and HitsAddend;
// per descriptor its suffix and an index into the batch's table of distinct
// limits; per tile of TileRequests requests the index of starting offsets.

const TileRequests = int(C.RL_PREFIXED_TILE)

// Limit is what a descriptor's config.RateLimit contributes to the batch.
type Limit struct {
	RequestsPerUnit uint32
	RuleID          uint32 // dense id of limit.Stats.Key
	Unit            uint8  // pb.RateLimitResponse_RateLimit_Unit (1..4)
	Shadow          bool   // limit.ShadowMode
}

// PrefixedBatch is one batch under construction: a pinned buffer sized for
// the batch's exact request and descriptor counts (Begin), filled request by
// request (Add), sealed (Seal), then submitted.
type PrefixedBatch struct {
	In  C.rl_batch_prefixed
	Out C.rl_result

	mem    unsafe.Pointer
	memCap int
	index  []uint32
	req    []uint32
	now    []uint32
	hits   []uint32
	desc   []uint32
	limits []C.rl_limit
	prefix []byte
	suffix []byte

	// outputs (pinned), per descriptor in packed order, and per-rule stats
	// deltas. DurationUntilReset is not copied back (rl_result.reset_s NULL, 4 B
	// per decision less over PCIe): the adapter computes it from the request's
	// clock as utils.CalculateReset does (utilities.go:32-36).
	Code      []uint8
	Remaining []uint32
	Status    []uint8
	Stats     []uint64

	n, nReq, nPrefix, nSuffix, nStem int
	limitIdx                         map[Limit]uint16
}

// NewPrefixedBatch allocates the batch's pinned outputs for at most maxDesc
// descriptors and maxRules stats rows (0: the library defaults, as rl_create
// resolves them); the input buffer grows on demand.
func NewPrefixedBatch(maxDesc, maxRules int) *PrefixedBatch {
	if maxDesc <= 0 {
		maxDesc = DefaultMaxBatch
	}
	if maxRules <= 0 {
		maxRules = DefaultMaxRules
	}
	b := &PrefixedBatch{limitIdx: make(map[Limit]uint16)}
	b.Code = bytesAt(pinned(maxDesc), maxDesc)
	b.Remaining = u32At(pinned(4*maxDesc), maxDesc)
	b.Status = bytesAt(pinned(maxDesc), maxDesc)
	b.Stats = u64At(pinned(8*maxRules*int(C.RL_NUM_STATS)), maxRules*int(C.RL_NUM_STATS))
	b.Out.code = (*C.uint8_t)(unsafe.Pointer(&b.Code[0]))
	b.Out.limit_remaining = (*C.uint32_t)(unsafe.Pointer(&b.Remaining[0]))
	b.Out.reset_s = nil
	b.Out.status = (*C.uint8_t)(unsafe.Pointer(&b.Status[0]))
	b.Out.stats = (*C.uint64_t)(unsafe.Pointer(&b.Stats[0]))
	return b
}

func align4(x int) int { return (x + 3) &^ 3 }

// Begin lays out the buffer for exactly nReq requests, nDesc descriptors and
// prefix / suffix byte totals (the batcher computes them before packing), so
// the sections abut and the batch crosses PCIe in one copy of its real size.
func (b *PrefixedBatch) Begin(nReq, nDesc, prefixBytes, suffixBytes, maxLimits int) {
	tiles := (nReq + TileRequests - 1) / TileRequests
	off := 0
	put := func(bytes int) int { o := off; off += align4(bytes); return o }
	oIndex := put(16 * (tiles + 1))
	oReq := put(4 * nReq)
	oNow := put(4 * nReq)
	oHits := put(4 * nReq)
	oDesc := put(4 * nDesc)
	oPrefix := put(prefixBytes)
	oSuffix := put(suffixBytes)
	oLimits := put(12 * maxLimits) // last: only the used entries count in buf_bytes (Seal)
	if off > b.memCap {
		if b.mem != nil {
			C.rl_free_host(b.mem)
		}
		b.memCap = off + off/4
		b.mem = pinned(b.memCap)
	}
	base := uintptr(b.mem)
	b.index = u32At(unsafe.Pointer(base+uintptr(oIndex)), 4*(tiles+1))
	b.req = u32At(unsafe.Pointer(base+uintptr(oReq)), nReq)
	b.now = u32At(unsafe.Pointer(base+uintptr(oNow)), nReq)
	b.hits = u32At(unsafe.Pointer(base+uintptr(oHits)), nReq)
	b.desc = u32At(unsafe.Pointer(base+uintptr(oDesc)), nDesc)
	b.prefix = bytesAt(unsafe.Pointer(base+uintptr(oPrefix)), prefixBytes)
	b.suffix = bytesAt(unsafe.Pointer(base+uintptr(oSuffix)), suffixBytes)
	b.limits = limitsAt(unsafe.Pointer(base+uintptr(oLimits)), maxLimits)
	b.In.buf = (*C.uint8_t)(b.mem)
	b.In.index = C.uint64_t(oIndex)
	b.In.req = C.uint64_t(oReq)
	b.In.now = C.uint64_t(oNow)
	b.In.hits = C.uint64_t(oHits)
	b.In.desc = C.uint64_t(oDesc)
	b.In.prefix_bytes = C.uint64_t(oPrefix)
	b.In.suffix_bytes = C.uint64_t(oSuffix)
	b.In.limits = C.uint64_t(oLimits)
	b.n, b.nReq, b.nPrefix, b.nSuffix, b.nStem = 0, 0, 0, 0, 0
	for k := range b.limitIdx {
		delete(b.limitIdx, k)
	}
}

// Add appends one request: its UnixNow(), HitsAddend, shared prefix and one
// suffix and limit per descriptor (stem = prefix + suffix). The prefix is at
// most 255 bytes and each suffix at most 65535.
func (b *PrefixedBatch) Add(now int64, hits uint32, prefix []byte, suffixes [][]byte, lims []Limit) error {
	if len(prefix) > 255 || len(suffixes) > 0xFFFF || len(suffixes) != len(lims) {
		return errors.New("gpu: request does not fit the prefixed layout")
	}
	if b.nReq%TileRequests == 0 {
		t := 4 * (b.nReq / TileRequests)
		b.index[t], b.index[t+1], b.index[t+2], b.index[t+3] =
			uint32(b.n), uint32(b.nPrefix), uint32(b.nSuffix), uint32(b.nStem)
	}
	q := b.nReq
	b.req[q] = uint32(len(suffixes)) | uint32(len(prefix))<<16
	b.now[q] = uint32(now)
	b.hits[q] = hits
	b.nPrefix += copy(b.prefix[b.nPrefix:], prefix)
	for i, s := range suffixes {
		if len(s) > 0xFFFF {
			return errors.New("gpu: descriptor suffix longer than 65535 bytes")
		}
		k, ok := b.limitIdx[lims[i]]
		if !ok {
			if len(b.limitIdx) == len(b.limits) {
				return errors.New("gpu: more distinct limits than the batch's table holds")
			}
			k = uint16(len(b.limitIdx))
			b.limitIdx[lims[i]] = k
			l := &b.limits[k]
			l.requests_per_unit = C.uint32_t(lims[i].RequestsPerUnit)
			l.rule_id = C.uint32_t(lims[i].RuleID)
			l.unit = C.uint8_t(lims[i].Unit)
			l.flags = 0
			if lims[i].Shadow {
				l.flags = C.uint8_t(C.RL_FLAG_SHADOW)
			}
		}
		b.desc[b.n] = uint32(k) | uint32(len(s))<<16
		b.nSuffix += copy(b.suffix[b.nSuffix:], s)
		b.nStem += len(prefix) + len(s)
		b.n++
	}
	b.nReq++
	return nil
}

// Seal writes the index totals and the batch header (nRules: rule ids < nRules).
func (b *PrefixedBatch) Seal(nRules int) {
	t := 4 * ((b.nReq + TileRequests - 1) / TileRequests)
	b.index[t], b.index[t+1], b.index[t+2], b.index[t+3] =
		uint32(b.n), uint32(b.nPrefix), uint32(b.nSuffix), uint32(b.nStem)
	b.In.n = C.uint32_t(b.n)
	b.In.n_requests = C.uint32_t(b.nReq)
	b.In.n_rules = C.uint32_t(nRules)
	b.In.n_limits = C.uint32_t(len(b.limitIdx))
	b.In.buf_bytes = C.uint64_t(uint64(b.In.limits) + uint64(12*len(b.limitIdx)))
}

// Len is the number of descriptors packed so far.
func (b *PrefixedBatch) Len() int { return b.n }

// Submit queues a sealed batch: it crosses PCIe while earlier batches
// compute; its outputs are final once Progress reports it complete, or after
// Synchronize. The batch is untouched by Go until then. On a routed ctx
// (comm.go) the batch is this rank's slice of the node batch and the call is
// collective; an empty batch (Begin(0, 0, ...)) still takes part.
func (c *Ctx) Submit(b *PrefixedBatch) error {
	return c.err(C.rl_do_limit_prefixed_async(c.c, &b.In, &b.Out))
}
