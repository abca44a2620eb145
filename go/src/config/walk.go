package config

// Walk visits every domain root and descriptor node of a config loaded by
// this package, parents before children, for the GPU backend's matcher
// (src/gpu/config.go, rl_config_load). visit gets the parent's id (-1 for a
// domain root), the node's key — the domain name, or its finalKey: key or
// key_value (config_impl.go:106-109) — and its limit (nil without a
// rate_limit block), and returns the id its children are given. false: cfg
// was not built by NewRateLimitConfigImpl. rateLimitConfigImpl and
// rateLimitDescriptor are unexported (config_impl.go:35-48), so the walk lives
// here and hands out only exported types.
func Walk(cfg RateLimitConfig, visit func(parent int, key string, limit *RateLimit) int) bool {
	impl, ok := cfg.(*rateLimitConfigImpl)
	if !ok {
		return false
	}
	var walk func(parent int, key string, d *rateLimitDescriptor)
	walk = func(parent int, key string, d *rateLimitDescriptor) {
		self := visit(parent, key, d.limit)
		for finalKey, child := range d.descriptors {
			walk(self, finalKey, child)
		}
	}
	for domain, root := range impl.domains {
		walk(-1, domain, &root.rateLimitDescriptor)
	}
	return true
}
