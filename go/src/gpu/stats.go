package gpu

import (
	"sync/atomic"

	gostats "github.com/lyft/gostats"
)

// localCacheStats publishes the GPU local over-limit cache's gauges, the
// counterpart of limiter.localCacheStats (src/limiter/local_cache_stats.go:20-43)
// for a cache that lives in the counter table: entryCount, lookupCount,
// hitCount and missCount (freecache v1.1.0's identity lookup = hit + miss).
// The batcher refreshes the values at every housekeeping pass (it alone calls
// the library); freecache's eviction, expiry, overwrite and access-time
// gauges have no counterpart.
type localCacheStats struct {
	impl        *rateLimitCacheImpl
	entryCount  gostats.Gauge
	lookupCount gostats.Gauge
	hitCount    gostats.Gauge
	missCount   gostats.Gauge
}

func newLocalCacheStats(impl *rateLimitCacheImpl, scope gostats.Scope) gostats.StatGenerator {
	return localCacheStats{
		impl:        impl,
		entryCount:  scope.NewGauge("entryCount"),
		lookupCount: scope.NewGauge("lookupCount"),
		hitCount:    scope.NewGauge("hitCount"),
		missCount:   scope.NewGauge("missCount"),
	}
}

func (s localCacheStats) GenerateStats() {
	s.entryCount.Set(atomic.LoadUint64(&s.impl.lcEntries))
	s.lookupCount.Set(atomic.LoadUint64(&s.impl.lcLookups))
	s.hitCount.Set(atomic.LoadUint64(&s.impl.lcHits))
	s.missCount.Set(atomic.LoadUint64(&s.impl.lcMisses))
}
