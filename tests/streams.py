"""Seeded random DoLimit call streams (structured), for parity tests.

Each stream is a list of (request, limits, now) in arrival order, built from the
oracle's data model. Streams stress every row of SURVEY.md §8a: nil limits,
duplicate descriptors inside one request, hits_addend > 1, shadow rules,
per-request overrides with a different unit than the rule (so SECOND/MINUTE/
HOUR keys of one stem can share a Redis key at aligned window starts), window
rollover across second/minute/hour boundaries, and hot keys.
"""
import random
import numpy as np

from oracle import oracle as O

UNITS = [O.SECOND, O.MINUTE, O.HOUR, O.DAY]


def random_stream(seed, n_calls=300, n_stems=12, start_now=1_700_000_035, max_step=3,
                  p_override=0.1, p_nil=0.1, p_shadow=0.2, max_hits=8, max_desc=4, limit_range=(0, 40),
                  domains=("dom", "other"), zipf=False):
    rng = random.Random(seed)
    reg = {}

    def stats(key):
        if key not in reg:
            reg[key] = O.RateLimitStats(key)
        return reg[key]

    # rules: one per (domain, entries) — like a loaded config; unit fixed per rule
    rules = []
    for s in range(n_stems):
        dom = rng.choice(domains)
        depth = rng.randint(1, 4)
        entries = [("k%d" % j, "v%d_%d" % (s % 5, j)) if rng.random() < 0.8 else ("k%d" % j, "")
                   for j in range(depth)]
        unit = rng.choice(UNITS)
        shadow = rng.random() < p_shadow
        limit = rng.randint(*limit_range)
        fk = dom + "." + ".".join(k + ("_" + v if v else "") for k, v in entries)
        rules.append((dom, entries, unit, limit, shadow, fk))
    now = start_now
    calls = []
    weights = [1.0 / (i + 1) ** 1.1 for i in range(n_stems)] if zipf else None
    for _ in range(n_calls):
        now += rng.choice([0] * 6 + list(range(1, max_step + 1)))
        dom = rng.choice(domains)
        descs, limits = [], []
        for _d in range(rng.randint(1, max_desc)):
            if weights:
                r = rng.choices(rules, weights)[0]
            else:
                r = rng.choice(rules)
            rdom, entries, unit, limit, shadow, fk = r
            if rdom != dom or rng.random() < p_nil:
                descs.append(O.Descriptor(list(entries)))
                limits.append(None)
                continue
            if rng.random() < p_override:
                # config_impl.go:254-265: override -> fresh RateLimit, stats key from descriptorKey
                ou = rng.choice(UNITS)
                ol = rng.randint(*limit_range)
                key = dom + "." + ".".join(k + ("_" + v if v else "") for k, v in entries)
                descs.append(O.Descriptor(list(entries), O.Limit(ol, ou)))
                limits.append(O.RateLimit(key, stats(key), O.Limit(ol, ou), False, False))
            else:
                descs.append(O.Descriptor(list(entries)))
                limits.append(O.RateLimit(fk, stats(fk), O.Limit(limit, unit), False, shadow))
        hits = rng.choice([0, 1, 1, 1, 2, 3, rng.randint(1, max_hits)])
        calls.append((O.RateLimitRequest(dom, descs, hits), limits, now))
    return calls


def c4_stream(seed, n_calls=1500, start_now=1_700_000_037, end_now=1_700_000_043, p_override=0.01):
    """BASELINE.json configs[4]: README Example 3/4-style nested
    descriptors in domain "c4" (rules as config_impl.go:99-151 would load them):

      service=<s> -> user (any value) -> method=<m> -> path (any value): SECOND 10
                                                      -> path=/login: MINUTE 5, shadow_mode
                                                      -> path=/health: unlimited (nil at DoLimit,
                                                         ratelimit.go:140-143)
      remote_address (any value): SECOND 10;  remote_address=50.0.0.5: SECOND 0

    plus 1% per-request overrides (config_impl.go:254-265: a fresh RateLimit whose
    stats key is descriptorKey, :300-312), duplicate descriptors inside one request,
    hits_addend 1..8 and a non-decreasing clock stepping across the second and
    minute boundaries (1_700_000_040 % 60 == 0). Wildcard rules share one stats key
    for every value (config_test.go:110)."""
    rng = random.Random(seed)
    reg = {}

    def rl(key, rpu, unit, shadow=False):
        if key not in reg:
            reg[key] = O.RateLimitStats(key)
        return O.RateLimit(key, reg[key], O.Limit(rpu, unit), False, shadow)

    dom = "c4"
    services = ["svc%d" % i for i in range(3)]
    users = ["u%03d" % i for i in range(24)]
    methods = ["GET", "POST"]
    paths = ["/login", "/health", "/api/a", "/api/b", "/static"]
    ips = ["10.0.0.%d" % i for i in range(20)] + ["50.0.0.5"] * 2
    nows = sorted(rng.randint(start_now, end_now) for _ in range(n_calls))
    calls = []
    for now in nows:
        descs, limits = [], []
        for _ in range(rng.randint(1, 4)):
            if descs and rng.random() < 0.2:  # the same descriptor twice in one request
                j = rng.randrange(len(descs))
                descs.append(O.Descriptor(list(descs[j].entries), descs[j].limit))
                limits.append(limits[j])
                continue
            if rng.random() < 0.7:
                s, u, m, p = rng.choice(services), rng.choice(users), rng.choice(methods), rng.choice(paths)
                entries = [("service", s), ("user", u), ("method", m), ("path", p)]
                base = "%s.service_%s.user.method_%s" % (dom, s, m)
                if p == "/login":
                    lim = rl(base + ".path_/login", 5, O.MINUTE, True)
                elif p == "/health":
                    lim = None
                else:
                    lim = rl(base + ".path", 10, O.SECOND)
            else:
                ip = rng.choice(ips)
                entries = [("remote_address", ip)]
                lim = rl(dom + ".remote_address_50.0.0.5", 0, O.SECOND) if ip == "50.0.0.5" else \
                    rl(dom + ".remote_address", 10, O.SECOND)
            d = O.Descriptor(entries)
            if rng.random() < p_override:
                ou, ol = rng.choice([O.SECOND, O.MINUTE, O.HOUR]), rng.randint(0, 20)
                d.limit = O.Limit(ol, ou)
                key = dom + "." + ".".join(k + ("_" + v if v else "") for k, v in entries)
                lim = rl(key, ol, ou)
            descs.append(d)
            limits.append(lim)
        calls.append((O.RateLimitRequest(dom, descs, rng.randint(1, 8)), limits, now))
    return calls


def reset_stats(calls):
    seen = set()
    for _, limits, _ in calls:
        for l in limits:
            if l is not None and id(l.stats) not in seen:
                seen.add(id(l.stats))
                for f in O.STAT_FIELDS:
                    setattr(l.stats, f, 0)


def python_oracle_run(calls, ratio=0.8, local_cache=False, prefix="", per_second=False):
    """Sequential replay through the pure-Python oracle; returns (statuses per call, stats dict)."""
    reset_stats(calls)
    cache = O.OracleFixedRateLimitCache(ratio, local_cache, prefix, per_second)
    outs = [cache.do_limit(req, limits, now) for req, limits, now in calls]
    stats = {}
    for _, limits, _ in calls:
        for l in limits:
            if l is not None:
                stats[l.stats.key] = l.stats.as_tuple()
    return outs, stats


def drop_descriptors(a, n, nq, keep):
    """The packed batch without the descriptors where keep is False (the
    oracle's input when the GPU failed those alone: RL_E_TIME descriptors do
    not INCRBY)."""
    idx = np.nonzero(keep[:n])[0]
    off = a["stem_off"]
    o = np.zeros(idx.size + 1, np.uint32)
    o[1:] = np.cumsum(off[idx + 1] - off[idx])
    out = {"stem_bytes": np.concatenate([a["stem_bytes"][off[i]:off[i + 1]] for i in idx])
           if idx.size else np.zeros(0, np.uint8), "stem_off": o, "now": a["now"]}
    for k in ("req_idx", "unit", "flags", "limit", "hits", "rule_id"):
        out[k] = a[k][idx]
    return out, idx.size, nq
