package limiter

import (
	pb "github.com/envoyproxy/go-control-plane/envoy/service/ratelimit/v3"
	"golang.org/x/net/context"

	"github.com/envoyproxy/ratelimit/src/config"
)

// RequestRateLimitCache is a RateLimitCache that can also resolve the limits
// itself: the GPU backend (src/gpu) walks the loaded config on the device
// (GetLimit, src/config/config_impl.go:243-298) for every descriptor of a
// batch of raw requests, instead of the service calling GetLimit per
// descriptor in Go (constructLimitsToCheck, src/service/ratelimit.go:104-146)
// before DoLimit. The service (src/service/ratelimit.go, patched) hands every
// loaded config to ConfigLoaded and asks DoLimitRequest first; ok == false
// (no config on the backend, or the backend cannot match this request) sends
// it down the reference path: GetLimit in Go, then DoLimit.
type RequestRateLimitCache interface {
	RateLimitCache

	// ConfigLoaded hands a newly loaded config to the backend (reloadConfig,
	// src/service/ratelimit.go:49-90). Requests that arrive after it are
	// matched against it.
	ConfigLoaded(cfg config.RateLimitConfig)

	// DoLimitRequest answers every descriptor of the request as
	// shouldRateLimitWorker would after GetLimit and DoLimit
	// (ratelimit.go:158-190): DoLimit's status where a limit matched
	// (CurrentLimit set), {OK, LimitRemaining: MaxUint32} for an unlimited
	// rule, {OK} where none matched. Throws RedisError like DoLimit.
	DoLimitRequest(ctx context.Context, request *pb.RateLimitRequest) (
		statuses []*pb.RateLimitResponse_DescriptorStatus, ok bool)
}
