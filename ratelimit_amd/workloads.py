"""Synthetic packed request streams for the BASELINE.json configs.

All generators return packed rl_batch arrays (numpy) built vectorised, so
million-descriptor batches are cheap. Simulated clocks start at
1_700_000_000 (1_700_000_000 % 60 == 20).

C0  README Example 1 (domain mongo_cps, database=users|default, 500/s) plus a
    value-less ``database`` rule (500/s, the builder's wildcard): 1 descriptor
    per request, value uniform over {users, default, db0000..db9997}.
C1  domain ``bench``: ``tenant`` (no value) -> tier=sec (second, 100) and
    tier=min (minute, 3000); 2 descriptors per request, uniform tenants.
C2  as C1 with Zipf(1.1) tenants and hits_addend uniform in 1..8.
"""
import numpy as np

NOW0 = 1_700_000_000


def _digits(vals, width):
    """ASCII zero-padded decimal digits of vals -> uint8[n, width]."""
    vals = np.asarray(vals, np.int64)
    out = np.empty((vals.size, width), np.uint8)
    v = vals.copy()
    for k in range(width - 1, -1, -1):
        out[:, k] = (v % 10) + 48
        v //= 10
    return out


def _fixed_stems(prefix: bytes, ids, width, suffix: bytes):
    """prefix ‖ zero-padded id ‖ suffix as a flat byte array + offsets."""
    n = len(ids)
    L = len(prefix) + width + len(suffix)
    rec = np.empty((n, L), np.uint8)
    rec[:, :len(prefix)] = np.frombuffer(prefix, np.uint8)
    rec[:, len(prefix):len(prefix) + width] = _digits(ids, width)
    rec[:, len(prefix) + width:] = np.frombuffer(suffix, np.uint8)
    return rec, L


class ZipfSampler:
    """Bounded Zipf(s) over ranks 0..n-1 by inverse CDF."""

    def __init__(self, n, s=1.1):
        w = 1.0 / np.arange(1, n + 1, dtype=np.float64) ** s
        self.cdf = np.cumsum(w)
        self.cdf /= self.cdf[-1]

    def sample(self, rng, size):
        return np.minimum(np.searchsorted(self.cdf, rng.random(size), side="right"), self.cdf.size - 1)


def c1_batch(tenants, now, hits=None):
    """One C1/C2 batch: request q = tenants[q]; descriptors (sec, min) per request."""
    tenants = np.asarray(tenants, np.int64)
    nq = tenants.size
    n = 2 * nq
    sec, L = _fixed_stems(b"bench_tenant_t", tenants, 10, b"_tier_sec_")
    mn, _ = _fixed_stems(b"bench_tenant_t", tenants, 10, b"_tier_min_")
    rec = np.empty((n, L), np.uint8)
    rec[0::2] = sec
    rec[1::2] = mn
    h = np.ones(nq, np.uint32) if hits is None else np.asarray(hits, np.uint32)
    return {
        "stem_bytes": rec.reshape(-1),
        "stem_off": (np.arange(n + 1, dtype=np.uint64) * L).astype(np.uint32),
        "now": np.full(nq, now, np.int64) if np.ndim(now) == 0 else np.asarray(now, np.int64),
        "req_idx": np.repeat(np.arange(nq, dtype=np.uint32), 2),
        "unit": np.tile(np.array([1, 2], np.uint8), nq),          # SECOND, MINUTE
        "flags": np.zeros(n, np.uint8),
        "limit": np.tile(np.array([100, 3000], np.uint32), nq),
        "hits": np.repeat(h, 2),
        "rule_id": np.tile(np.array([0, 1], np.uint32), nq),
    }, n, nq, 2


C1_RULES = ["bench.tenant.tier_sec", "bench.tenant.tier_min"]


def c1_batch_dev(tenants, now, hits=None, device="cuda"):
    """c1_batch built on the GPU with torch (same bytes, same arrays): used to
    fill 10^8-key tables (BASELINE C3) without host-side generation. ``tenants``
    is an int64 tensor (or array); uint32 arrays come back as int32 tensors of
    the same bits, ready for Backend.do_limit_device."""
    import torch
    t = torch.as_tensor(tenants, dtype=torch.int64, device=device)
    nq = t.numel()
    n = 2 * nq
    pre = torch.tensor(list(b"bench_tenant_t"), dtype=torch.uint8, device=device)
    sec = torch.tensor(list(b"_tier_sec_"), dtype=torch.uint8, device=device)
    mn = torch.tensor(list(b"_tier_min_"), dtype=torch.uint8, device=device)
    L = pre.numel() + 10 + sec.numel()
    dig = torch.empty((nq, 10), dtype=torch.uint8, device=device)
    v = t.clone()
    for k in range(9, -1, -1):
        dig[:, k] = (v % 10 + 48).to(torch.uint8)
        v = v // 10
    rec = torch.empty((nq, 2, L), dtype=torch.uint8, device=device)
    rec[:, :, :pre.numel()] = pre
    rec[:, :, pre.numel():pre.numel() + 10] = dig[:, None, :]
    rec[:, 0, pre.numel() + 10:] = sec
    rec[:, 1, pre.numel() + 10:] = mn
    i32 = dict(dtype=torch.int32, device=device)
    h = torch.ones(nq, **i32) if hits is None else torch.as_tensor(hits, device=device).to(torch.int32)
    return {
        "stem_bytes": rec.reshape(-1),
        "stem_off": torch.arange(n + 1, **i32) * L,
        "now": (torch.full((nq,), int(now), dtype=torch.int64, device=device) if np.ndim(now) == 0
                else torch.as_tensor(now, dtype=torch.int64, device=device)),
        "req_idx": torch.arange(nq, **i32).repeat_interleave(2),
        "unit": torch.tensor([1, 2], dtype=torch.uint8, device=device).repeat(nq),
        "flags": torch.zeros(n, dtype=torch.uint8, device=device),
        "limit": torch.tensor([100, 3000], **i32).repeat(nq),
        "hits": h.repeat_interleave(2),
        "rule_id": torch.tensor([0, 1], **i32).repeat(nq),
    }, n, nq, 2


def c1_stream(seed=0xC1, n_tenants=10_000_000, requests_per_batch=500_000, batches=4, now0=NOW0):
    rng = np.random.default_rng(seed)
    for k in range(batches):
        yield c1_batch(rng.integers(0, n_tenants, requests_per_batch), now0 + k)


def c2_stream(seed=0xC2, n_tenants=10_000_000, requests_per_batch=500_000, batches=4, now0=NOW0, s=1.1,
              sampler=None):
    rng = np.random.default_rng(seed)
    z = sampler or ZipfSampler(n_tenants, s)
    for k in range(batches):
        t = z.sample(rng, requests_per_batch)
        h = rng.integers(1, 9, requests_per_batch).astype(np.uint32)
        yield c1_batch(t, now0 + k, h)


def c2u_batch(t, now, h, rng, hot=16, p_override=0.5, override_limit=20_000):
    """A C2 batch where requests of the `hot` hottest tenants carry, with
    probability p_override, a per-request override on their ``tier=sec``
    descriptor whose unit is MINUTE (config_impl.go:254-265: a fresh RateLimit,
    its own stats key, rule id 2). The same stem is then seen under SECOND and
    MINUTE: a Redis key shared by both units whenever t % 60 == 0
    (cache_key.go:73-74), two independent keys otherwise."""
    a, n, nq, _ = c1_batch(t, now, h)
    ov = (np.asarray(t) < hot) & (rng.random(nq) < p_override)
    idx = 2 * np.nonzero(ov)[0]  # the request's sec descriptor
    a["unit"][idx] = 2
    a["limit"][idx] = override_limit
    a["rule_id"][idx] = 2
    return a, n, nq, 3


def c2u_stream(seed=0xC2, n_tenants=10_000_000, requests_per_batch=500_000, batches=4, now0=NOW0, s=1.1,
               sampler=None, hot=16, p_override=0.5, now_per_request=None):
    """C2 plus hot-tenant overrides in a second unit (c2u_batch). now_per_request:
    optional callable (batch k, nq) -> int64[nq] clock per request."""
    rng = np.random.default_rng(seed)
    z = sampler or ZipfSampler(n_tenants, s)
    for k in range(batches):
        t = z.sample(rng, requests_per_batch)
        h = rng.integers(1, 9, requests_per_batch).astype(np.uint32)
        now = now0 + k if now_per_request is None else now_per_request(k, requests_per_batch)
        yield c2u_batch(t, now, h, rng, hot, p_override)


C2U_RULES = C1_RULES + ["bench.tenant.tier_sec(override:minute)"]


def c0_batch(values, now_per_request):
    """C0: domain mongo_cps, descriptor [(database, v)], one per request."""
    values = np.asarray(values, np.int64)  # -2 users, -1 default, >=0 db%04d
    nq = values.size
    stems = []
    for v in values.tolist():
        name = "users" if v == -2 else "default" if v == -1 else "db%04d" % v
        stems.append(("mongo_cps_database_%s_" % name).encode())
    lens = np.fromiter((len(s) for s in stems), np.uint32, nq)
    off = np.zeros(nq + 1, np.uint32)
    off[1:] = np.cumsum(lens)
    rule = np.where(values == -2, 0, np.where(values == -1, 1, 2)).astype(np.uint32)
    return {"stem_bytes": np.frombuffer(b"".join(stems), np.uint8).copy(), "stem_off": off,
            "now": np.asarray(now_per_request, np.int64), "req_idx": np.arange(nq, dtype=np.uint32),
            "unit": np.ones(nq, np.uint8), "flags": np.zeros(nq, np.uint8),
            "limit": np.full(nq, 500, np.uint32), "hits": np.ones(nq, np.uint32), "rule_id": rule}, nq, nq, 3


C0_RULES = ["mongo_cps.database_users", "mongo_cps.database_default", "mongo_cps.database"]


def c0_stream(seed=0xC0, n_requests=1_000_000, per_batch=100_000, now0=NOW0):
    """1M requests over 10k keys; now advances 1 s every 100k requests."""
    rng = np.random.default_rng(seed)
    for k in range(0, n_requests, per_batch):
        m = min(per_batch, n_requests - k)
        vals = rng.integers(-2, 9998, m)
        yield c0_batch(vals, np.full(m, now0 + k // 100_000, np.int64))


def concat_batches(batches):
    """Concatenate packed batches (request indices and offsets rebased)."""
    out = {k: [] for k in ("stem_bytes", "stem_off", "now", "req_idx", "unit", "flags", "limit", "hits",
                           "rule_id")}
    n = nq = 0
    base = 0
    n_rules = 0
    for a, bn, bq, br in batches:
        out["stem_bytes"].append(a["stem_bytes"][:int(a["stem_off"][bn])])
        out["stem_off"].append(a["stem_off"][:bn].astype(np.uint64) + base)
        out["now"].append(a["now"][:bq])
        out["req_idx"].append(a["req_idx"][:bn] + nq)
        for k in ("unit", "flags", "limit", "hits", "rule_id"):
            out[k].append(a[k][:bn])
        base += int(a["stem_off"][bn])
        n += bn
        nq += bq
        n_rules = max(n_rules, br)
    res = {k: np.concatenate(v) for k, v in out.items()}
    res["stem_off"] = np.append(res["stem_off"], base).astype(np.uint32)
    res["req_idx"] = res["req_idx"].astype(np.uint32)
    return res, n, nq, n_rules


# C1 as a config file: the rules c1_batch packs by hand (rule ids 0, 1 in load order)
C1_CONFIG_YAML = """\
domain: bench
descriptors:
  - key: tenant
    descriptors:
      - key: tier
        value: sec
        rate_limit:
          unit: second
          requests_per_unit: 100
      - key: tier
        value: min
        rate_limit:
          unit: minute
          requests_per_unit: 3000
"""


def c1_requests(tenants, now, hits=None):
    """One C1/C2 batch as raw requests (rl_request_batch arrays): request q is
    domain ``bench`` with descriptors [(tenant, t), (tier, sec)] and
    [(tenant, t), (tier, min)]; matched through C1_CONFIG_YAML it is c1_batch."""
    tenants = np.asarray(tenants, np.int64)
    nq = tenants.size
    n = 2 * nq
    sec, L = _fixed_stems(b"tenant_t", tenants, 10, b"_tier_sec_")
    mn, _ = _fixed_stems(b"tenant_t", tenants, 10, b"_tier_min_")
    rec = np.empty((n, L), np.uint8)
    rec[0::2] = sec
    rec[1::2] = mn
    h = np.ones(nq, np.uint32) if hits is None else np.asarray(hits, np.uint32)
    return {
        "domain_bytes": np.tile(np.frombuffer(b"bench", np.uint8), nq),
        "domain_off": (np.arange(nq + 1, dtype=np.uint64) * 5).astype(np.uint32),
        "now": np.full(nq, now, np.int64) if np.ndim(now) == 0 else np.asarray(now, np.int64),
        "hits": h,
        "req_idx": np.repeat(np.arange(nq, dtype=np.uint32), 2),
        "entry_first": (np.arange(n + 1, dtype=np.uint64) * 2).astype(np.uint32),
        "desc_off": (np.arange(n + 1, dtype=np.uint64) * L).astype(np.uint32),
        "desc_bytes": rec.reshape(-1),
        "key_len": np.tile(np.array([6, 4], np.uint16), n),
        "value_len": np.tile(np.array([11, 3], np.uint16), n),
        "override_flags": None, "override_rpu": None, "override_unit": None, "override_rule": None,
    }
