package gpu

import (
	"fmt"
	"sync/atomic"
	"time"

	"github.com/coocood/freecache"
	pb_struct "github.com/envoyproxy/go-control-plane/envoy/extensions/common/ratelimit/v3"
	pb "github.com/envoyproxy/go-control-plane/envoy/service/ratelimit/v3"
	"github.com/golang/protobuf/ptypes/duration"
	logger "github.com/sirupsen/logrus"
	"golang.org/x/net/context"

	"github.com/envoyproxy/ratelimit/src/assert"
	"github.com/envoyproxy/ratelimit/src/config"
	"github.com/envoyproxy/ratelimit/src/limiter"
	"github.com/envoyproxy/ratelimit/src/redis"
	"github.com/envoyproxy/ratelimit/src/server"
	"github.com/envoyproxy/ratelimit/src/settings"
	"github.com/envoyproxy/ratelimit/src/stats"
	"github.com/envoyproxy/ratelimit/src/utils"
)

// rateLimitCacheImpl implements limiter.RateLimitCache (src/limiter/cache.go:11-29)
// on the GPU. Many RPC goroutines call DoLimit concurrently (no lock around it
// in service.shouldRateLimitWorker, src/service/ratelimit.go:158); each
// enqueues its call. One batcher goroutine — the only one that touches the
// C library — gathers up to maxDesc descriptors or whatever arrived within
// `window`, packs them as a prefix-shared batch, submits it, and packs the
// next batch while the GPU runs this one (two batches alternate). Each call
// then gets its statuses in the reference's DescriptorStatus form.
type rateLimitCacheImpl struct {
	ctx        *Ctx
	timeSource utils.TimeSource
	prefix     string // CACHE_KEY_PREFIX (cache_key.go:62)
	queue      chan *call
	window     time.Duration
	maxDesc    int
	maxRules   int
	sweepEvery time.Duration
	sweepLag   int64
	batches    [2]*PrefixedBatch

	rules     map[string]uint32      // limit.Stats.Key -> dense rule id
	ruleStats []stats.RateLimitStats // rule id -> the counters its deltas go to

	// local-cache gauges, refreshed by the batcher (gpuLocalCacheStats reads them)
	lcEntries, lcLookups, lcHits, lcMisses uint64
}

type call struct {
	req    *pb.RateLimitRequest
	limits []*config.RateLimit
	now    int64 // timeSource.UnixNow(), read once per request (base_limiter.go:49)
	done   chan reply
}

type reply struct {
	statuses []*pb.RateLimitResponse_DescriptorStatus
	err      string // non-empty: this call failed (its batch, or one of its descriptors)
}

// flight is a submitted batch whose answers are still to be handed out.
type flight struct {
	b      *PrefixedBatch
	calls  []*call
	where  [][]int // where[ci][i] = packed index of descriptor i of call ci, -1: nil limit
	nRules int
	err    error // the submit itself failed
}

// Options are the knobs of the batcher beyond the library's Config.
type Options struct {
	Window        time.Duration // GPU_BATCH_WINDOW
	SweepInterval time.Duration // GPU_SWEEP_INTERVAL (0: never)
	SweepLag      time.Duration // GPU_SWEEP_LAG: the sweep's time floor trails the clock by this much
}

// NewRateLimitCacheImpl starts the batcher on an existing ctx.
func NewRateLimitCacheImpl(ctx *Ctx, cfg Config, opt Options, timeSource utils.TimeSource,
	cacheKeyPrefix string) *rateLimitCacheImpl {
	maxRules := int(cfg.MaxRules)
	this := &rateLimitCacheImpl{
		ctx:        ctx,
		timeSource: timeSource,
		prefix:     cacheKeyPrefix,
		queue:      make(chan *call, 4096),
		window:     opt.Window,
		maxDesc:    int(cfg.MaxBatch),
		maxRules:   maxRules,
		sweepEvery: opt.SweepInterval,
		sweepLag:   int64(opt.SweepLag / time.Second),
		rules:      map[string]uint32{},
	}
	for i := range this.batches {
		this.batches[i] = NewPrefixedBatch(this.maxDesc, maxRules)
	}
	go this.batcher()
	return this
}

// NewRateLimitCacheImplFromSettings is BACKEND_TYPE=gpu in createLimiter
// (src/service_cmd/runner/runner.go:50-74): the ctx from the settings the
// Redis backend reads (NEAR_LIMIT_RATIO, LOCAL_CACHE_SIZE_IN_BYTES != 0,
// CACHE_KEY_PREFIX, EXPIRATION_JITTER_MAX_SECONDS, REDIS_PERSECOND; settings.go:45-50,78)
// and the GPU_* knobs (settings.go, INTEGRATION.md §4). The freecache
// instance itself is not used: the local over-limit cache lives in the
// counter table, and its gauges are published under "localcache_gpu".
func NewRateLimitCacheImplFromSettings(s settings.Settings, localCache *freecache.Cache, srv server.Server,
	timeSource utils.TimeSource, statsManager stats.Manager) limiter.RateLimitCache {
	cfg := Config{
		TableSlots:     s.GpuTableSlots,
		RingLines:      s.GpuRingLines,
		ArenaBytes:     s.GpuArenaBytes,
		MaxBatch:       uint32(s.GpuBatchMaxDescriptors),
		MaxRequests:    uint32(s.GpuBatchMaxRequests),
		MaxRules:       uint32(s.GpuMaxRules),
		MaxStemBytes:   uint32(s.GpuBatchMaxStemBytes),
		NearLimitRatio: s.NearLimitRatio,
		LocalCache:     localCache != nil,
		PerSecond:      s.RedisPerSecond,
		JitterMax:      s.ExpirationJitterMaxSeconds,
		Device:         s.GpuDevice,
		HashSeed:       s.GpuHashSeed,
		ShardDevices:   s.GpuShardDevices,
	}
	ctx, err := New(cfg)
	if err != nil {
		logger.Fatalf("gpu: cannot create the GPU backend: %v", err)
	}
	impl := NewRateLimitCacheImpl(ctx, cfg, Options{Window: s.GpuBatchWindow, SweepInterval: s.GpuSweepInterval,
		SweepLag: s.GpuSweepLag}, timeSource, s.CacheKeyPrefix)
	if cfg.LocalCache && srv != nil {
		statsManager.GetStatsStore().AddStatGenerator(newLocalCacheStats(impl, srv.Scope().Scope("localcache_gpu")))
	}
	return impl
}

func (this *rateLimitCacheImpl) DoLimit(ctx context.Context, request *pb.RateLimitRequest,
	limits []*config.RateLimit) []*pb.RateLimitResponse_DescriptorStatus {
	assert.Assert(len(request.Descriptors) == len(limits)) // base_limiter.go:47
	c := &call{request, limits, this.timeSource.UnixNow(), make(chan reply, 1)}
	this.queue <- c
	r := <-c.done
	if r.err != "" {
		panic(redis.RedisError(r.err)) // driver_impl.go:60-64; recovered at ratelimit.go:252-256
	}
	return r.statuses
}

// Flush: nothing to wait for, DoLimit returns with its answers.
func (this *rateLimitCacheImpl) Flush() {}

func (this *rateLimitCacheImpl) rule(s stats.RateLimitStats) (uint32, bool) {
	id, ok := this.rules[s.Key]
	if !ok {
		if len(this.ruleStats) == this.maxRules {
			return 0, false
		}
		id = uint32(len(this.ruleStats))
		this.rules[s.Key] = id
		this.ruleStats = append(this.ruleStats, s)
	}
	return id, true
}

// batcher: the only goroutine that calls the C library.
func (this *rateLimitCacheImpl) batcher() {
	var carry *call
	var inflight *flight
	cur := 0
	lastSweep := time.Now()
	for {
		first := carry
		carry = nil
		if first == nil {
			select {
			case first = <-this.queue:
			default:
				// idle: hand out the batch in flight before waiting for more calls
				if inflight != nil {
					this.finish(inflight)
					inflight = nil
				}
				first = <-this.queue
			}
		}
		calls, total := []*call{first}, len(first.limits)
		timer := time.NewTimer(this.window)
	collect:
		for total < this.maxDesc {
			select {
			case c := <-this.queue:
				if total+len(c.limits) > this.maxDesc {
					carry = c // the next batch
					break collect
				}
				calls = append(calls, c)
				total += len(c.limits)
			case <-timer.C:
				break collect
			}
		}
		timer.Stop()
		// pack the next batch while the one in flight runs on the GPU
		f := this.pack(this.batches[cur], calls)
		if inflight != nil {
			this.finish(inflight)
		}
		if f.err == nil {
			f.err = this.ctx.Submit(f.b)
		}
		inflight = f
		cur ^= 1
		if this.sweepEvery > 0 && time.Since(lastSweep) >= this.sweepEvery {
			this.finish(inflight) // (the sweep orders after it anyway)
			inflight = nil
			this.housekeeping()
			lastSweep = time.Now()
		}
	}
}

// stem = prefix ‖ domain ‖ '_' ‖ Σ(key ‖ '_' ‖ value ‖ '_')   (cache_key.go:62-71).
// A request's shared prefix is what every one of its packed (non-nil limit)
// descriptors' stems starts with: prefix ‖ domain ‖ '_' and the leading
// entries they all carry (nested descriptors repeat their parents'), cut at
// 255 bytes. Returns the packed descriptors' count, the shared bytes and the
// packed stems' total length.
func (this *rateLimitCacheImpl) shared(c *call) (n int, shared int, total int) {
	head := len(this.prefix) + len(c.req.Domain) + 1
	var ref []*pb_struct.RateLimitDescriptor_Entry
	common := 0
	for i, d := range c.req.Descriptors {
		if c.limits[i] == nil {
			continue
		}
		total += head
		for _, e := range d.Entries {
			total += len(e.Key) + len(e.Value) + 2
		}
		if n == 0 {
			ref, common = d.Entries, len(d.Entries)
		} else {
			k := 0
			for k < common && k < len(d.Entries) && d.Entries[k].Key == ref[k].Key && d.Entries[k].Value == ref[k].Value {
				k++
			}
			common = k
		}
		n++
	}
	if n == 0 {
		return 0, 0, 0
	}
	shared = head
	for k := 0; k < common; k++ {
		shared += len(ref[k].Key) + len(ref[k].Value) + 2
	}
	if shared > 255 {
		shared = 255
	}
	return n, shared, total
}

func appendEntries(dst []byte, entries []*pb_struct.RateLimitDescriptor_Entry) []byte {
	for _, e := range entries {
		dst = append(dst, e.Key...)
		dst = append(dst, '_')
		dst = append(dst, e.Value...)
		dst = append(dst, '_')
	}
	return dst
}

// pack: every non-nil limit of the calls, in arrival order (nil limits answer
// {OK, nil, 0} without the GPU, base_limiter.go:78-81).
func (this *rateLimitCacheImpl) pack(b *PrefixedBatch, calls []*call) *flight {
	f := &flight{b: b, calls: calls, where: make([][]int, len(calls))}
	// sizes first, so the buffer's sections abut (one PCIe copy of the real size)
	nDesc, pBytes, sBytes := 0, 0, 0
	shared := make([]int, len(calls))
	for ci, c := range calls {
		n, p, total := this.shared(c)
		shared[ci] = p
		nDesc += n
		pBytes += p
		sBytes += total - n*p
	}
	b.Begin(len(calls), nDesc, pBytes, sBytes, 65536)
	var stem []byte
	suffixes := make([][]byte, 0, 8)
	lims := make([]Limit, 0, 8)
	for ci, c := range calls {
		pLen := shared[ci]
		suffixes, lims, stem = suffixes[:0], lims[:0], stem[:0]
		idx := make([]int, len(c.limits))
		for i, d := range c.req.Descriptors {
			idx[i] = -1
			l := c.limits[i]
			if l == nil {
				continue
			}
			if l.Limit.Unit == pb.RateLimitResponse_RateLimit_UNKNOWN {
				panic("should not get here") // utils.UnitToDivider (utilities.go:29)
			}
			rid, ok := this.rule(l.Stats)
			if !ok {
				f.err = fmt.Errorf("gpu: more than %d rule stats keys", this.maxRules)
				return f
			}
			s0 := len(stem)
			stem = append(stem, this.prefix...)
			stem = append(stem, c.req.Domain...)
			stem = append(stem, '_')
			stem = appendEntries(stem, d.Entries)
			idx[i] = b.Len() + len(suffixes)
			suffixes = append(suffixes, stem[s0+pLen:])
			lims = append(lims, Limit{RequestsPerUnit: l.Limit.RequestsPerUnit, RuleID: rid,
				Unit: uint8(l.Limit.Unit), Shadow: l.ShadowMode})
		}
		// (append may have moved stem: the suffixes keep the arrays they point into)
		var prefix []byte
		if len(suffixes) > 0 {
			prefix = stem[:pLen] // every packed stem of the request starts with these bytes
		}
		// HitsAddend as the request carries it: the library applies utils.Max(1, h) (fixed_cache_impl.go:41)
		if err := b.Add(c.now, c.req.HitsAddend, prefix, suffixes, lims); err != nil {
			f.err = err
			return f
		}
		f.where[ci] = idx
	}
	f.nRules = len(this.ruleStats)
	b.Seal(f.nRules)
	return f
}

// finish waits for the flight's batch and answers its calls.
func (this *rateLimitCacheImpl) finish(f *flight) {
	err := f.err
	if err == nil {
		err = this.ctx.Synchronize()
	}
	b := f.b
	for ci, c := range f.calls {
		idx := f.where[ci]
		if err != nil || idx == nil {
			msg := "gpu: batch not packed"
			if err != nil {
				msg = "gpu: " + err.Error()
			}
			c.done <- reply{err: msg}
			continue
		}
		st := make([]*pb.RateLimitResponse_DescriptorStatus, len(c.limits))
		failed := ""
		for i, j := range idx {
			if j < 0 {
				st[i] = &pb.RateLimitResponse_DescriptorStatus{Code: pb.RateLimitResponse_OK}
				continue
			}
			if b.Status[j] != 0 { // this descriptor alone could not be answered
				failed = fmt.Sprintf("gpu: descriptor failed (rl_status %d)", b.Status[j])
				continue
			}
			div := utils.UnitToDivider(c.limits[i].Limit.Unit)
			st[i] = &pb.RateLimitResponse_DescriptorStatus{ // base_limiter.go:181-197
				Code:               pb.RateLimitResponse_Code(b.Code[j]),
				CurrentLimit:       c.limits[i].Limit,
				LimitRemaining:     b.Remaining[j],
				DurationUntilReset: &duration.Duration{Seconds: div - c.now%div}, // utils.CalculateReset
			}
		}
		if failed != "" {
			c.done <- reply{err: failed}
		} else {
			c.done <- reply{statuses: st}
		}
	}
	if err != nil {
		return
	}
	// per-rule deltas in stats.RateLimitStats order (manager.go:47-55): the
	// batch's sum of what the reference Adds per descriptor
	for r := 0; r < f.nRules; r++ {
		s := this.ruleStats[r]
		d := b.Stats[6*r : 6*r+6]
		for k, ctr := range []interface{ Add(uint64) }{s.TotalHits, s.OverLimit, s.NearLimit,
			s.OverLimitWithLocalCache, s.WithinLimit, s.ShadowMode} {
			if d[k] != 0 {
				ctr.Add(d[k])
			}
		}
	}
}

// housekeeping: the EXPIRE sweep (slots whose windows all ended before now -
// lag are evicted; requests older than that floor then fail alone) and the
// local-cache gauges.
func (this *rateLimitCacheImpl) housekeeping() {
	now := this.timeSource.UnixNow()
	if _, err := this.ctx.Sweep(now - this.sweepLag); err != nil {
		logger.Errorf("gpu: sweep failed: %v", err)
	}
	if info, err := this.ctx.LocalCacheInfo(now); err == nil {
		atomic.StoreUint64(&this.lcEntries, info.EntryCount)
		atomic.StoreUint64(&this.lcLookups, info.LookupCount)
		atomic.StoreUint64(&this.lcHits, info.HitCount)
		atomic.StoreUint64(&this.lcMisses, info.MissCount)
	}
}
