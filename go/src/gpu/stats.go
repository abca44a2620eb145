package gpu

import (
	"sync/atomic"

	gostats "github.com/lyft/gostats"
)

// localCacheStats publishes the GPU local over-limit cache's gauges, the
// counterpart of limiter.localCacheStats (src/limiter/local_cache_stats.go:20-43)
// for a cache that lives in the counter table: entryCount, lookupCount,
// hitCount and missCount (freecache v1.1.0's identity lookup = hit + miss),
// refreshed by the batcher at every housekeeping pass (it alone calls the
// library). The other four gauges are published under the same names, so the
// reference's dashboards and its gauge test (which checks that all eight exist,
// fixed_cache_impl_test.go:150-167) find them, and stay 0: the table never
// evicts an entry for space (evacuateCount) nor overwrites a live one
// (overwriteCount: a key is Set only while its entry is absent or expired,
// fixed_cache_impl.go:57-67, 100-106), an expired entry is not deleted by a
// Get (expiredCount: freecache counts the deletions), and no access time is
// kept (averageAccessTime).
type localCacheStats struct {
	impl              *rateLimitCacheImpl
	entryCount        gostats.Gauge
	lookupCount       gostats.Gauge
	hitCount          gostats.Gauge
	missCount         gostats.Gauge
	evacuateCount     gostats.Gauge
	expiredCount      gostats.Gauge
	averageAccessTime gostats.Gauge
	overwriteCount    gostats.Gauge
}

func newLocalCacheStats(impl *rateLimitCacheImpl, scope gostats.Scope) gostats.StatGenerator {
	return localCacheStats{
		impl:              impl,
		entryCount:        scope.NewGauge("entryCount"),
		lookupCount:       scope.NewGauge("lookupCount"),
		hitCount:          scope.NewGauge("hitCount"),
		missCount:         scope.NewGauge("missCount"),
		evacuateCount:     scope.NewGauge("evacuateCount"),
		expiredCount:      scope.NewGauge("expiredCount"),
		averageAccessTime: scope.NewGauge("averageAccessTime"),
		overwriteCount:    scope.NewGauge("overwriteCount"),
	}
}

func (s localCacheStats) GenerateStats() {
	s.entryCount.Set(atomic.LoadUint64(&s.impl.lcEntries))
	s.lookupCount.Set(atomic.LoadUint64(&s.impl.lcLookups))
	s.hitCount.Set(atomic.LoadUint64(&s.impl.lcHits))
	s.missCount.Set(atomic.LoadUint64(&s.impl.lcMisses))
	s.evacuateCount.Set(0)
	s.expiredCount.Set(0)
	s.averageAccessTime.Set(0)
	s.overwriteCount.Set(0)
}
