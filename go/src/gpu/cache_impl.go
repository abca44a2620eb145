package gpu

import (
	"fmt"
	"math"
	"strings"
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
	routed     bool // the ctx joined a world of ranks: one collective batch per tick (batcherRouted)

	// GPU_CONFIG_MATCH (limiter.RequestRateLimitCache): the loaded config on
	// the device, raw requests matched there (rl_do_limit_requests)
	configMatch  bool
	configReady  int32 // (atomic) a config has been loaded on the device
	rb           *RequestBatch
	statsManager stats.Manager                              // override stats (config_impl.go:255-263)
	limitByKey   map[string]*pb.RateLimitResponse_RateLimit // Stats.Key -> the config rule's limit (CurrentLimit)

	rules     map[string]uint32      // limit.Stats.Key -> dense rule id
	ruleStats []stats.RateLimitStats // rule id -> the counters its deltas go to

	// local-cache gauges, refreshed by the batcher (gpuLocalCacheStats reads them)
	lcEntries, lcLookups, lcHits, lcMisses uint64

	// health (GPU_HEALTH_CHECK_DEVICE): a device-level library failure marks
	// the server's health check failed, the next success marks it OK again,
	// as the Redis pool does on its connections (src/redis/driver_impl.go:31-52)
	health healthMonitor
}

// healthMonitor flips the server's health check on device-level failures
// (rl_status RL_E_HIP, RL_E_COMM, RL_E_INTERNAL: the GPU or its runtime, not
// a request): the pod stops reporting SERVING while its device cannot answer.
// Request-level failures (RL_E_TIME, RL_E_INVALID, RL_E_CAPACITY, a full
// table) leave it as it is. Batcher goroutine only.
type healthMonitor struct {
	srv       server.Server // nil: no health check (tests, GPU_HEALTH_CHECK_DEVICE=false)
	unhealthy bool
}

func deviceFailure(err error) bool {
	e, ok := err.(*Error)
	return ok && (e.Status == StatusHIP || e.Status == StatusComm || e.Status == StatusInternal)
}

// observe: the outcome of one library call that reached the device (a batch,
// a request batch, a sweep).
func (h *healthMonitor) observe(err error) {
	if h.srv == nil {
		return
	}
	if deviceFailure(err) {
		if !h.unhealthy {
			logger.Errorf("gpu: device failure, health check failed: %v", err)
			h.srv.HealthCheckFail()
			h.unhealthy = true
		}
	} else if err == nil && h.unhealthy {
		logger.Warnf("gpu: device answering again, health check OK")
		h.srv.HealthCheckOK()
		h.unhealthy = false
	}
}

type call struct {
	req    *pb.RateLimitRequest
	limits []*config.RateLimit
	now    int64 // timeSource.UnixNow(), read once per request (base_limiter.go:49)
	done   chan reply
	raw    bool                   // DoLimitRequest: the limits are matched on the GPU
	cfg    config.RateLimitConfig // a config to load (ConfigLoaded), not a request
}

// kind of a queued call: a DoLimit call, a raw request, a config load
func (c *call) kind() int {
	if c.cfg != nil {
		return 2
	}
	if c.raw {
		return 1
	}
	return 0
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
	ConfigMatch   bool          // GPU_CONFIG_MATCH: GetLimit on the GPU (not on a routed ctx)
	StatsManager  stats.Manager // for the override stats keys the GPU match meets (ConfigMatch)
	HealthServer  server.Server // GPU_HEALTH_CHECK_DEVICE: the server whose health check device failures flip (nil: none)
}

// NewRateLimitCacheImpl starts the batcher on an existing ctx.
func NewRateLimitCacheImpl(ctx *Ctx, cfg Config, opt Options, timeSource utils.TimeSource,
	cacheKeyPrefix string) *rateLimitCacheImpl {
	cfg = cfg.Resolved() // (a zero field is the library's default: size the pinned buffers for it)
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
		routed:     ctx.Routed(),
		// (rl_do_limit_requests is not routed: a routed ctx keeps GetLimit in Go)
		configMatch:  opt.ConfigMatch && !ctx.Routed() && opt.StatsManager != nil,
		statsManager: opt.StatsManager,
		limitByKey:   map[string]*pb.RateLimitResponse_RateLimit{},
	}
	this.health.srv = opt.HealthServer
	if this.configMatch {
		this.rb = NewRequestBatch()
	}
	for i := range this.batches {
		this.batches[i] = NewPrefixedBatch(this.maxDesc, maxRules)
	}
	if this.routed {
		go this.batcherRouted()
	} else {
		go this.batcher()
	}
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
		HistoryEntries: s.GpuHistoryEntries,
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
	if s.GpuWorld > 1 {
		// one service process per GPU: this process is rank GPU_RANK of
		// GPU_WORLD, every rank with the same GPU_HASH_SEED (comm.go)
		if cfg.HashSeed == 0 {
			logger.Fatalf("gpu: GPU_WORLD > 1 needs an explicit GPU_HASH_SEED shared by every rank")
		}
		id, err := CommIDFile(s.GpuCommIDFile, s.GpuRank, s.GpuCommTimeout)
		if err == nil {
			err = ctx.CommInit(s.GpuWorld, s.GpuRank, id)
		}
		if err != nil {
			logger.Fatalf("gpu: cannot join the GPU world: %v", err)
		}
	}
	opt := Options{Window: s.GpuBatchWindow, SweepInterval: s.GpuSweepInterval, SweepLag: s.GpuSweepLag,
		ConfigMatch: s.GpuConfigMatch, StatsManager: statsManager}
	if s.GpuHealthCheckDevice && srv != nil {
		opt.HealthServer = srv
	}
	impl := NewRateLimitCacheImpl(ctx, cfg, opt, timeSource, s.CacheKeyPrefix)
	if cfg.LocalCache && srv != nil {
		statsManager.GetStatsStore().AddStatGenerator(newLocalCacheStats(impl, srv.Scope().Scope("localcache_gpu")))
	}
	return impl
}

func (this *rateLimitCacheImpl) DoLimit(ctx context.Context, request *pb.RateLimitRequest,
	limits []*config.RateLimit) []*pb.RateLimitResponse_DescriptorStatus {
	assert.Assert(len(request.Descriptors) == len(limits)) // base_limiter.go:47
	c := &call{req: request, limits: limits, now: this.timeSource.UnixNow(), done: make(chan reply, 1)}
	this.queue <- c
	r := <-c.done
	if r.err != "" {
		panic(redis.RedisError(r.err)) // driver_impl.go:60-64; recovered at ratelimit.go:252-256
	}
	return r.statuses
}

// Flush: nothing to wait for, DoLimit returns with its answers.
func (this *rateLimitCacheImpl) Flush() {}

// ConfigLoaded (limiter.RequestRateLimitCache): the batcher loads cfg on the
// device between two batches; requests queued after it are matched against it.
func (this *rateLimitCacheImpl) ConfigLoaded(cfg config.RateLimitConfig) {
	if !this.configMatch || cfg == nil {
		return
	}
	c := &call{cfg: cfg, done: make(chan reply, 1)}
	this.queue <- c
	if r := <-c.done; r.err != "" {
		// (requests keep the reference path: GetLimit in Go, then DoLimit)
		logger.Errorf("gpu: config not loaded on the device: %s", r.err)
	}
}

// DoLimitRequest (limiter.RequestRateLimitCache): GetLimit, DoLimit and the
// unlimited mapping for the whole request on the GPU. ok == false until a
// config is on the device (and always without GPU_CONFIG_MATCH).
func (this *rateLimitCacheImpl) DoLimitRequest(ctx context.Context, request *pb.RateLimitRequest) (
	[]*pb.RateLimitResponse_DescriptorStatus, bool) {
	if !this.configMatch || atomic.LoadInt32(&this.configReady) == 0 {
		return nil, false
	}
	c := &call{req: request, now: this.timeSource.UnixNow(), done: make(chan reply, 1), raw: true}
	this.queue <- c
	r := <-c.done
	if r.err != "" {
		panic(redis.RedisError(r.err)) // driver_impl.go:60-64; recovered at ratelimit.go:252-256
	}
	return r.statuses, true
}

// descriptorKey (src/config/config_impl.go:300-312): an override's stats key.
func descriptorKey(domain string, d *pb_struct.RateLimitDescriptor) string {
	parts := make([]string, 0, len(d.Entries))
	for _, e := range d.Entries {
		if e.Value != "" {
			parts = append(parts, e.Key+"_"+e.Value)
		} else {
			parts = append(parts, e.Key)
		}
	}
	return domain + "." + strings.Join(parts, ".")
}

// loadConfig (batcher goroutine): the config on the device, its rules'
// limits kept for CurrentLimit (the reference aliases limit.Limit,
// base_limiter.go:186).
func (this *rateLimitCacheImpl) loadConfig(cfg config.RateLimitConfig) error {
	limits := map[string]*pb.RateLimitResponse_RateLimit{}
	config.Walk(cfg, func(parent int, key string, l *config.RateLimit) int {
		if l != nil && l.Limit != nil {
			limits[l.Stats.Key] = l.Limit
		}
		return 0
	})
	if err := this.ctx.LoadConfig(cfg, this.prefix, this.rule); err != nil {
		return err
	}
	this.limitByKey = limits
	atomic.StoreInt32(&this.configReady, 1)
	return nil
}

// doRaw (batcher goroutine): one rl_do_limit_requests over the raw calls.
func (this *rateLimitCacheImpl) doRaw(calls []*call) {
	reqs := make([]*pb.RateLimitRequest, len(calls))
	nows := make([]int64, len(calls))
	for i, c := range calls {
		reqs[i], nows[i] = c.req, c.now
	}
	full := false
	override := func(domain string, d *pb_struct.RateLimitDescriptor) uint32 {
		key := descriptorKey(domain, d)
		id, ok := this.rules[key]
		if !ok {
			if len(this.ruleStats) == this.maxRules {
				full = true
				return 0
			}
			// GetLimit's fresh RateLimit for an override: statsManager.NewStats(key) (config_impl.go:255-263)
			id = this.ruleStatsAdd(this.statsManager.NewStats(key))
		}
		return id
	}
	b := this.rb
	b.Pack(reqs, nows, override, func() int { return len(this.ruleStats) })
	var err error
	if full {
		err = fmt.Errorf("gpu: more than %d rule stats keys", this.maxRules)
	} else {
		err = this.ctx.DoLimitRequests(b)
		this.health.observe(err)
	}
	j := 0
	for _, c := range calls {
		if err != nil {
			c.done <- reply{err: "gpu: " + err.Error()}
			continue
		}
		st := make([]*pb.RateLimitResponse_DescriptorStatus, len(c.req.Descriptors))
		for i := range st {
			switch b.Match[j] {
			case MatchLimit: // ratelimit.go:186-190: DoLimit's status
				st[i] = &pb.RateLimitResponse_DescriptorStatus{
					Code:               pb.RateLimitResponse_Code(b.Code[j]),
					CurrentLimit:       this.currentLimit(b.RuleID[j], b.RPU[j], b.Unit[j]),
					LimitRemaining:     b.Remaining[j],
					DurationUntilReset: &duration.Duration{Seconds: int64(b.Reset[j])},
				}
			case MatchUnlimited: // ratelimit.go:176-183
				st[i] = &pb.RateLimitResponse_DescriptorStatus{Code: pb.RateLimitResponse_OK,
					LimitRemaining: math.MaxUint32}
			default: // no rule: a nil limit, {OK, nil, 0} (base_limiter.go:78-81)
				st[i] = &pb.RateLimitResponse_DescriptorStatus{Code: pb.RateLimitResponse_OK}
			}
			j++
		}
		c.done <- reply{statuses: st}
	}
	if err == nil {
		this.applyStats(b.Stats, int(b.In.n_rules))
	}
}

// currentLimit: the matched config rule's limit proto (or an override's, fresh).
func (this *rateLimitCacheImpl) currentLimit(rid, rpu uint32, unit uint8) *pb.RateLimitResponse_RateLimit {
	if int(rid) < len(this.ruleStats) {
		if l := this.limitByKey[this.ruleStats[rid].Key]; l != nil && l.RequestsPerUnit == rpu && uint8(l.Unit) == unit {
			return l
		}
	}
	return &pb.RateLimitResponse_RateLimit{RequestsPerUnit: rpu, Unit: pb.RateLimitResponse_RateLimit_Unit(unit)}
}

func (this *rateLimitCacheImpl) rule(s stats.RateLimitStats) (uint32, bool) {
	id, ok := this.rules[s.Key]
	if !ok {
		if len(this.ruleStats) == this.maxRules {
			return 0, false
		}
		id = this.ruleStatsAdd(s)
	}
	return id, true
}

func (this *rateLimitCacheImpl) ruleStatsAdd(s stats.RateLimitStats) uint32 {
	id := uint32(len(this.ruleStats))
	this.rules[s.Key] = id
	this.ruleStats = append(this.ruleStats, s)
	return id
}

// applyStats adds a batch's per-rule deltas (stats.RateLimitStats order,
// manager.go:47-55) to the rules' counters: the sum of what the reference Adds
// per descriptor.
func (this *rateLimitCacheImpl) applyStats(d []uint64, nRules int) {
	for r := 0; r < nRules && r < len(this.ruleStats); r++ {
		s := this.ruleStats[r]
		for k, ctr := range []interface{ Add(uint64) }{s.TotalHits, s.OverLimit, s.NearLimit,
			s.OverLimitWithLocalCache, s.WithinLimit, s.ShadowMode} {
			if v := d[6*r+k]; v != 0 {
				ctr.Add(v)
			}
		}
	}
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
		if first.kind() == 2 { // a config load: after every batch before it
			if inflight != nil {
				this.finish(inflight)
				inflight = nil
			}
			msg := ""
			if err := this.loadConfig(first.cfg); err != nil {
				msg = err.Error()
			}
			first.done <- reply{err: msg}
			continue
		}
		size := func(c *call) int {
			if c.raw {
				return len(c.req.Descriptors)
			}
			return len(c.limits)
		}
		calls, total := []*call{first}, size(first)
		timer := time.NewTimer(this.window)
	collect:
		for total < this.maxDesc {
			select {
			case c := <-this.queue:
				// one kind per batch, in arrival order
				if c.kind() != first.kind() || total+size(c) > this.maxDesc {
					carry = c // the next batch
					break collect
				}
				calls = append(calls, c)
				total += size(c)
			case <-timer.C:
				break collect
			}
		}
		timer.Stop()
		if first.raw { // (synchronous: after the DoLimit batch in flight)
			if inflight != nil {
				this.finish(inflight)
				inflight = nil
			}
			this.doRaw(calls)
			if this.sweepEvery > 0 && time.Since(lastSweep) >= this.sweepEvery {
				this.housekeeping()
				lastSweep = time.Now()
			}
			continue
		}
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

// batcherRouted: the batcher of a routed ctx. Submit, Synchronize and Sweep
// are collective over the ranks, so every rank takes the same steps on the
// same schedule: one batch per tick of the window, holding whatever calls
// arrived (none: an empty batch, still a step of the exchange), and a sweep
// every sweepTicks ticks. A batch that cannot be packed is replaced by an
// empty one (its calls fail) so that no peer waits for this rank. The
// previous tick's calls are answered through the collective Synchronize,
// which completes every pending routed batch: one routed batch in flight per
// tick (DESIGN.md §6). Every rank sweeps on the same tick; the library applies
// the least of the ranks' floors on all of them.
func (this *rateLimitCacheImpl) batcherRouted() {
	tick := time.NewTicker(this.window)
	defer tick.Stop()
	var carry *call
	var inflight *flight
	cur := 0
	sweepTicks := uint64(0)
	if this.sweepEvery > 0 && this.window > 0 {
		sweepTicks = uint64(this.sweepEvery / this.window)
	}
	for n := uint64(1); ; n++ {
		<-tick.C
		var calls []*call
		total := 0
		if carry != nil {
			calls, total, carry = append(calls, carry), len(carry.limits), nil
		}
	drain:
		for total < this.maxDesc {
			select {
			case c := <-this.queue:
				if total+len(c.limits) > this.maxDesc {
					carry = c
					break drain
				}
				calls = append(calls, c)
				total += len(c.limits)
			default:
				break drain
			}
		}
		f := this.pack(this.batches[cur], calls)
		if inflight != nil {
			this.finish(inflight)
		}
		if f.err != nil { // take part with an empty batch; the calls fail in finish
			e := this.pack(this.batches[cur], nil)
			if err := this.ctx.Submit(e.b); err != nil {
				logger.Errorf("gpu: routed submit failed: %v", err)
			}
		} else {
			f.err = this.ctx.Submit(f.b)
		}
		inflight = f
		cur ^= 1
		if sweepTicks > 0 && n%sweepTicks == 0 {
			this.finish(inflight)
			inflight = nil
			this.housekeeping()
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
	if err == nil || this.routed { // (routed: Synchronize is collective, every rank calls it per flight)
		if serr := this.ctx.Synchronize(); err == nil {
			err = serr
		}
	}
	this.health.observe(err)
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
	this.applyStats(b.Stats, f.nRules)
}

// housekeeping: the EXPIRE sweep (slots whose windows all ended before now -
// lag are evicted; requests older than that floor then fail alone) and the
// local-cache gauges.
func (this *rateLimitCacheImpl) housekeeping() {
	now := this.timeSource.UnixNow()
	_, err := this.ctx.Sweep(now - this.sweepLag)
	if err != nil {
		logger.Errorf("gpu: sweep failed: %v", err)
	}
	this.health.observe(err)
	if info, err := this.ctx.LocalCacheInfo(now); err == nil {
		atomic.StoreUint64(&this.lcEntries, info.EntryCount)
		atomic.StoreUint64(&this.lcLookups, info.LookupCount)
		atomic.StoreUint64(&this.lcHits, info.HitCount)
		atomic.StoreUint64(&this.lcMisses, info.MissCount)
	}
}
