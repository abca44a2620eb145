"""GPU parity of the request path: GetLimit on the device + DoLimit + the
service's status mapping (rl_do_limit_requests, through the C ABI) against
the oracle's config restatement and service step (oracle/config.py).

* the reference's own GetLimit cases (tests/golden/ref_config.json, from
  test/config/config_test.go) resolved on the GPU;
* random request streams over nested configs (C4 shape: 4-level nesting,
  wildcard and value rules, shadow_mode, unlimited, README Example 3's
  remote_address pair, test/config/basic_config.yaml), with unknown domains,
  unmatched and too-deep descriptors, overrides, duplicate descriptors,
  underscores inside keys/values, hits 0..8, local cache on/off, prefixes and
  the clock crossing second/minute boundaries: statuses, overall codes and
  per-rule stats bit-exact.
"""
import json
import os
import random

import numpy as np
import pytest
import yaml

from oracle import oracle as O
from oracle.config import OracleService, RateLimitConfig, StatsStore
from ratelimit_amd import abi
from ratelimit_amd.limiter import Backend, GpuRateLimitService, RedisError

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_config.json")))
SMALL = dict(table_slots=1 << 16, max_batch=1 << 14, max_rules=1 << 10)

SERVICES = ["svc0", "svc1", "svc_2"]
METHODS = ["GET", "POST"]
PATHS = ["/login", "/health", "/api/a", "/api_b", "/static"]


def c4_yaml():
    """SURVEY.md §8d C4 rules as a config file (README Example 3/4 style)."""
    method_children = [
        {"key": "path", "rate_limit": {"unit": "second", "requests_per_unit": 10}},
        {"key": "path", "value": "/login", "rate_limit": {"unit": "minute", "requests_per_unit": 5},
         "shadow_mode": True},
        {"key": "path", "value": "/health", "rate_limit": {"unlimited": True}},
    ]
    svc = [{"key": "service", "value": s, "descriptors": [
        {"key": "user", "descriptors": [{"key": "method", "value": m, "descriptors": method_children}
                                        for m in METHODS]}]} for s in SERVICES]
    doc = {"domain": "c4", "descriptors": svc + [
        {"key": "remote_address", "rate_limit": {"unit": "second", "requests_per_unit": 10}},
        {"key": "remote_address", "value": "50.0.0.5", "rate_limit": {"unit": "second", "requests_per_unit": 0}},
        {"key": "tenant", "rate_limit": {"unit": "hour", "requests_per_unit": 40},
         "descriptors": [{"key": "tier", "value": "x_y", "rate_limit": {"unit": "day", "requests_per_unit": 60}}]},
    ]}
    return yaml.safe_dump(doc)


FILES = [("c4.yaml", c4_yaml()), ("basic_config.yaml", G["files"]["basic_config.yaml"])]


def gen_requests(seed, n, start_now=1_700_000_037, end_now=1_700_000_043, p_override=0.03):
    rng = random.Random(seed)
    users = ["u%02d" % i for i in range(12)] + ["u_x"]
    ips = ["10.0.0.%d" % i for i in range(12)] + ["50.0.0.5"]
    nows = sorted(rng.randint(start_now, end_now) for _ in range(n))
    reqs = []
    for _ in range(n):
        r = rng.random()
        domain = "c4" if r < 0.75 else ("test-domain" if r < 0.95 else "nope")
        descs = []
        for _ in range(rng.randint(1, 4)):
            if descs and rng.random() < 0.15:
                j = rng.randrange(len(descs))
                descs.append(O.Descriptor(list(descs[j].entries), descs[j].limit))
                continue
            x = rng.random()
            if domain == "test-domain":
                k1 = rng.choice(["key1", "key2", "key3", "key4", "key5", "key6", "keyX"])
                v1 = rng.choice(["value1", "value2", "value3", "value5", "foo", ""])
                entries = [(k1, v1)]
                if rng.random() < 0.4:
                    entries.append((rng.choice(["subkey1", "subkey5"]), rng.choice(["subvalue1", "subvalue5", "z"])))
            elif x < 0.6:
                entries = [("service", rng.choice(SERVICES + ["svcZ"])), ("user", rng.choice(users)),
                           ("method", rng.choice(METHODS + ["PUT"])), ("path", rng.choice(PATHS))]
                cut = rng.random()
                if cut < 0.05:
                    entries = entries[:rng.randint(0, 3)]  # too shallow (no limit at that depth)
                elif cut < 0.08:
                    entries = entries + [("extra", "1")]  # deeper than the config
            elif x < 0.85:
                entries = [("remote_address", rng.choice(ips))]
            else:
                entries = [("tenant", rng.choice(["t1", "t_2", "t3"]))]
                if rng.random() < 0.5:
                    entries.append(("tier", rng.choice(["x_y", "x", "y"])))
            lim = None
            if rng.random() < p_override:
                lim = O.Limit(rng.randint(0, 12), rng.choice([O.SECOND, O.MINUTE, O.HOUR]))
            descs.append(O.Descriptor(entries, lim))
        reqs.append(O.RateLimitRequest(domain, descs, rng.choice([0, 1, 1, 2, 3, 8])))
    return reqs, nows


def st_tuple(s):
    cl = None if s.current_limit is None else (s.current_limit.requests_per_unit, s.current_limit.unit)
    return (s.code, cl, s.limit_remaining, s.duration_until_reset)


@pytest.mark.parametrize("case", G["lookups"], ids=lambda c: c["source"])
def test_gpu_get_limit_reference_cases(case):
    files = [(n, G["files"][n]) for n in case["config"]]
    svc = GpuRateLimitService(files, **SMALL)
    try:
        ov = case["override"]
        req = O.RateLimitRequest(case["domain"], [O.Descriptor([tuple(e) for e in case["entries"]],
                                                               O.Limit(*ov) if ov else None)], 1)
        from ratelimit_amd.config import pack_requests
        a = pack_requests([req], [1_700_000_000], svc.interner)
        res = svc.backend.do_limit_requests(a, max(len(svc.interner.keys), 1))
        exp = case["expect"]
        m = int(res["match"][0])
        if exp is None:
            assert m == abi.RL_MATCH_NONE
            assert (res["code"][0], res["limit_remaining"][0], res["reset_s"][0]) == (O.OK, 0, 0)
            return
        assert svc.interner.keys[res["rule_id"][0]] == exp["full_key"]
        if exp["unlimited"]:
            assert m == abi.RL_MATCH_UNLIMITED and res["limit_remaining"][0] == 0xFFFFFFFF
        else:
            assert m == abi.RL_MATCH_LIMIT
            assert (int(res["requests_per_unit"][0]), int(res["unit"][0])) == (exp["rpu"], exp["unit"])
    finally:
        svc.close()


@pytest.mark.parametrize("seed,local_cache,prefix,ratio", [
    (1, False, "", 0.8), (2, True, "", 0.8), (3, True, "prefix:", 0.9), (4, False, "p_", 0.75),
    (5, True, "", 0.8)])
def test_gpu_request_stream_matches_oracle_service(seed, local_cache, prefix, ratio):
    reqs, nows = gen_requests(seed, 1200)
    svc = GpuRateLimitService(FILES, ratio, local_cache, prefix, **SMALL)
    store = StatsStore()
    osvc = OracleService(RateLimitConfig(FILES, store), O.OracleFixedRateLimitCache(ratio, local_cache, prefix))
    rng = random.Random(seed * 7)
    try:
        i = 0
        while i < len(reqs):
            j = min(len(reqs), i + rng.choice([1, 7, 64, 300]))
            got = svc.should_rate_limit_batch(reqs[i:j], nows[i:j])
            for r, now, (gcode, gsts) in zip(reqs[i:j], nows[i:j], got):
                ocode, osts, _ = osvc.should_rate_limit(r, now)
                assert gcode == ocode
                assert [st_tuple(s) for s in gsts] == [st_tuple(s) for s in osts]
            i = j
        want = {k: list(v.as_tuple()) for k, v in store.by_key.items() if any(v.as_tuple())}
        assert svc.stats == want
    finally:
        svc.close()


@pytest.mark.parametrize("n_shards,seed,local_cache", [(2, 2, True), (3, 3, False)])
def test_gpu_request_stream_multishard_matches_oracle_service(n_shards, seed, local_cache):
    """rl_do_limit_requests on a ctx hash-sharded over 2-3 tables on cuda:0:
    the config match on shard 0, the matched descriptors routed to their
    owners; statuses, codes and per-rule stats equal the oracle service's."""
    reqs, nows = gen_requests(seed, 1200)
    svc = GpuRateLimitService(FILES, 0.8, local_cache, "", n_shards=n_shards, shard_devices=[0] * n_shards,
                              hash_seed=5, **SMALL)
    store = StatsStore()
    osvc = OracleService(RateLimitConfig(FILES, store), O.OracleFixedRateLimitCache(0.8, local_cache, ""))
    rng = random.Random(seed * 7)
    try:
        i = 0
        while i < len(reqs):
            j = min(len(reqs), i + rng.choice([1, 7, 64, 300]))
            got = svc.should_rate_limit_batch(reqs[i:j], nows[i:j])
            for r, now, (gcode, gsts) in zip(reqs[i:j], nows[i:j], got):
                ocode, osts, _ = osvc.should_rate_limit(r, now)
                assert gcode == ocode
                assert [st_tuple(s) for s in gsts] == [st_tuple(s) for s in osts]
            i = j
        want = {k: list(v.as_tuple()) for k, v in store.by_key.items() if any(v.as_tuple())}
        assert svc.stats == want
    finally:
        svc.close()


def test_gpu_request_large_batch_matches_oracle_service():
    """One 20k-request batch (~50k descriptors): compaction at scale."""
    reqs, nows = gen_requests(11, 20000, p_override=0.01)
    svc = GpuRateLimitService(FILES, 0.8, True, "", table_slots=1 << 18, max_batch=1 << 17, max_rules=1 << 12)
    store = StatsStore()
    osvc = OracleService(RateLimitConfig(FILES, store), O.OracleFixedRateLimitCache(0.8, True, ""))
    try:
        got = svc.should_rate_limit_batch(reqs, nows)
        for r, now, (gcode, gsts) in zip(reqs, nows, got):
            ocode, osts, _ = osvc.should_rate_limit(r, now)
            assert gcode == ocode
            assert [st_tuple(s) for s in gsts] == [st_tuple(s) for s in osts]
        want = {k: list(v.as_tuple()) for k, v in store.by_key.items() if any(v.as_tuple())}
        assert svc.stats == want
    finally:
        svc.close()


def test_gpu_requests_errors():
    be = Backend(**SMALL)
    try:
        from ratelimit_amd.config import ConfigTree, pack_requests
        from ratelimit_amd.packing import RuleInterner
        it = RuleInterner()
        req = O.RateLimitRequest("c4", [O.Descriptor([("remote_address", "1")])], 1)
        with pytest.raises(RedisError, match="no rate limit configuration"):
            be.do_limit_requests(pack_requests([req], [1_700_000_000], it), 1)
        tree = ConfigTree.from_yaml(FILES, "", it)
        be.load_config(tree)
        ok = be.do_limit_requests(pack_requests([req], [1_700_000_000], it), len(it.keys))
        assert ok["match"][0] == abi.RL_MATCH_LIMIT and ok["code"][0] == O.OK
        # an override with UNKNOWN unit panics in UnitToDivider in the reference
        bad = O.RateLimitRequest("c4", [O.Descriptor([("remote_address", "1")], O.Limit(5, 0))], 1)
        with pytest.raises(RedisError, match="RL_E_INVALID"):
            be.do_limit_requests(pack_requests([bad], [1_700_000_000], it), len(it.keys))
        # entry lengths that do not tile the descriptor bytes
        a = pack_requests([req], [1_700_000_000], it)
        a["key_len"] = a["key_len"] + 1
        with pytest.raises(RedisError, match="RL_E_INVALID"):
            be.do_limit_requests(a, len(it.keys))
        # the table is intact after rejected batches
        ok2 = be.do_limit_requests(pack_requests([req], [1_700_000_000], it), len(it.keys))
        assert ok2["limit_remaining"][0] == ok["limit_remaining"][0] - 1
    finally:
        be.close()


def test_gpu_request_long_entries_take_global_paths():
    """Entry bytes beyond a workgroup's LDS staging (16 KB) and stems beyond its
    assembly buffer (24 KB) take the global-memory paths of k_match /
    k_match_emit; stems > 36 B also go through the table's overflow arena."""
    rng = random.Random(99)
    reqs, nows = [], []
    vals = ["v" + "x_" * rng.randint(40, 150) + str(i) for i in range(40)]
    for i in range(1500):
        descs = [O.Descriptor([("tenant", rng.choice(vals))]),
                 O.Descriptor([("tenant", rng.choice(vals)), ("tier", "x_y")]),
                 O.Descriptor([("remote_address", rng.choice(vals))])]
        reqs.append(O.RateLimitRequest("c4", descs, rng.randint(1, 3)))
        nows.append(1_700_000_038 + i // 500)
    svc = GpuRateLimitService(FILES, 0.8, True, "prefix:", table_slots=1 << 16, max_batch=1 << 14,
                              max_rules=1 << 10, max_stem_bytes=1 << 22)
    store = StatsStore()
    osvc = OracleService(RateLimitConfig(FILES, store), O.OracleFixedRateLimitCache(0.8, True, "prefix:"))
    try:
        got = svc.should_rate_limit_batch(reqs, nows)
        for r, now, (gcode, gsts) in zip(reqs, nows, got):
            ocode, osts, _ = osvc.should_rate_limit(r, now)
            assert gcode == ocode
            assert [st_tuple(s) for s in gsts] == [st_tuple(s) for s in osts]
        want = {k: list(v.as_tuple()) for k, v in store.by_key.items() if any(v.as_tuple())}
        assert svc.stats == want
    finally:
        svc.close()


def test_gpu_serialized_requests_through_native_packer():
    """gRPC payloads (serialized RateLimitRequest) -> rl_packer -> rl_do_limit_requests:
    statuses and stats equal the oracle service's; override stats keys come back
    by name from the packer."""
    import pbwire
    from ratelimit_amd.config import ConfigTree, RequestPacker
    from ratelimit_amd.packing import RuleInterner
    reqs, nows = gen_requests(21, 1500)
    it = RuleInterner()
    tree = ConfigTree.from_yaml(FILES, "", it)
    be = Backend(0.8, True, **SMALL)
    be.load_config(tree)
    pk = RequestPacker(len(it.keys))
    store = StatsStore()
    osvc = OracleService(RateLimitConfig(FILES, store), O.OracleFixedRateLimitCache(0.8, True, ""))
    totals = {}
    try:
        for i in range(0, len(reqs), 250):
            part, pn = reqs[i:i + 250], nows[i:i + 250]
            b = pk.pack([pbwire.encode_request(r) for r in part], pn)
            res = be.do_limit_request_batch(b)
            d = 0
            for r, now in zip(part, pn):
                _, osts, _ = osvc.should_rate_limit(r, now)
                for s in osts:
                    m = int(res["match"][d])
                    cl = (int(res["requests_per_unit"][d]), int(res["unit"][d])) if m == abi.RL_MATCH_LIMIT else None
                    got = (int(res["code"][d]), cl, int(res["limit_remaining"][d]),
                           int(res["reset_s"][d]) if m == abi.RL_MATCH_LIMIT else None)
                    assert got == st_tuple(s)
                    d += 1
            st = res["stats"].reshape(-1, abi.RL_NUM_STATS)
            for rid in np.nonzero(st.any(axis=1))[0]:
                name = it.keys[rid] if rid < len(it.keys) else pk.rule_key(int(rid))
                row = totals.setdefault(name, [0] * abi.RL_NUM_STATS)
                for j in range(abi.RL_NUM_STATS):
                    row[j] += int(st[rid, j])
        want = {k: list(v.as_tuple()) for k, v in store.by_key.items() if any(v.as_tuple())}
        assert totals == want
    finally:
        pk.close()
        be.close()
