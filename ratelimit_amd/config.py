"""Host side of the device config match: the loaded rate-limit config as the
flat trie ``rl_config_load`` takes, and raw requests as an ``rl_request_batch``.

The Go adapter builds the node array by walking the
``rateLimitConfigImpl`` it already loaded (src/config/config_impl.go:200-231):
one node per domain and per ``rateLimitDescriptor``, keyed by its finalKey
(``key`` or ``key_value``, config_impl.go:106-109), with the rule's stats key
(``domain.k_v.k2``, config_impl.go:111,139) interned to a dense rule id. This
module does the same from the YAML files, with the loader's validation
(config_impl.go:96-231), so the Python mirror can load a config on its own.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

from . import abi
from .packing import RuleInterner

UNIT_VALUE = {"UNKNOWN": 0, "SECOND": 1, "MINUTE": 2, "HOUR": 3, "DAY": 4}  # rls.proto Unit_value
VALID_KEYS = {"domain", "key", "value", "descriptors", "rate_limit", "unit", "requests_per_unit", "unlimited",
              "shadow_mode"}  # config_impl.go:57-65


class RateLimitConfigError(Exception):
    """config.RateLimitConfigError: "<file>: <text>" (config_impl.go:73-76)."""


def _check_keys(name, m):
    for k, v in m.items():
        if not isinstance(k, str):
            raise RateLimitConfigError("%s: config error, key is not of type string: %s" % (name, k))
        if k not in VALID_KEYS:
            raise RateLimitConfigError("%s: config error, unknown key '%s'" % (name, k))
        if isinstance(v, list):
            for e in v:
                if not isinstance(e, dict):
                    raise RateLimitConfigError(
                        "%s: config error, yaml file contains list of type other than map: %s" % (name, e))
                _check_keys(name, e)
        elif isinstance(v, dict):
            _check_keys(name, v)


class ConfigTree:
    """Flattened config: parents before children; node i's key is ``keys[i]``."""

    def __init__(self, cache_key_prefix: str = "", interner: Optional[RuleInterner] = None):
        self.prefix = cache_key_prefix
        self.interner = interner or RuleInterner()
        self.parent: List[int] = []
        self.keys: List[bytes] = []
        self.rows: List[Tuple[int, int, int, int, int, int]] = []  # rpu, rule, unit, has_limit, unlimited, shadow
        self.full_key: List[str] = []
        self.domains: Dict[str, int] = {}

    @classmethod
    def from_yaml(cls, files: Sequence[Tuple[str, str]], cache_key_prefix: str = "",
                  interner: Optional[RuleInterner] = None) -> "ConfigTree":
        t = cls(cache_key_prefix, interner)
        for name, text in files:
            t.add_yaml(name, text)
        return t

    def _node(self, parent: int, key: str, full_key: str, rl=None, shadow=False) -> int:
        self.parent.append(parent)
        self.keys.append(key.encode())
        self.full_key.append(full_key)
        if rl is None:
            self.rows.append((0, 0, 0, 0, 0, 0))
        else:
            rpu, unit, unlimited = rl
            self.rows.append((rpu, self.interner.intern(full_key), unit, 1, int(unlimited), int(shadow)))
        return len(self.parent) - 1

    def add_yaml(self, name: str, text: str) -> None:
        """loadConfig (config_impl.go:200-231)."""
        try:
            root = yaml.safe_load(text)
        except yaml.YAMLError as e:
            raise RateLimitConfigError("%s: error loading config file: %s" % (name, e))
        root = root if isinstance(root, dict) else {}
        _check_keys(name, root)
        domain = str(root.get("domain") or "")
        if domain == "":
            raise RateLimitConfigError("%s: config file cannot have empty domain" % name)
        if domain in self.domains:
            raise RateLimitConfigError("%s: duplicate domain '%s' in config file" % (name, domain))
        idx = self._node(-1, domain, domain)
        self.domains[domain] = idx
        self._descriptors(name, idx, domain + ".", root.get("descriptors") or [])

    def _descriptors(self, name, parent: int, parent_key: str, descs) -> None:
        """loadDescriptors (config_impl.go:96-150)."""
        seen = set()
        for dc in descs:
            key = str(dc.get("key") or "")
            if key == "":
                raise RateLimitConfigError("%s: descriptor has empty key" % name)
            value = str(dc.get("value") or "")
            final = key + ("_" + value if value else "")
            full = parent_key + final
            if final in seen:
                raise RateLimitConfigError("%s: duplicate descriptor composite key '%s'" % (name, full))
            seen.add(final)
            rl = None
            y = dc.get("rate_limit")
            if y is not None:
                unlimited = bool(y.get("unlimited") or False)
                u = UNIT_VALUE.get(str(y.get("unit") or "").upper())
                valid = u is not None and u != 0
                if unlimited and valid:
                    raise RateLimitConfigError("%s: should not specify rate limit unit when unlimited" % name)
                if not unlimited and not valid:
                    raise RateLimitConfigError("%s: invalid rate limit unit '%s'" % (name, y.get("unit") or ""))
                rl = (int(y.get("requests_per_unit") or 0) & 0xFFFFFFFF, u or 0, unlimited)
            idx = self._node(parent, final, full, rl, bool(dc.get("shadow_mode") or False))
            self._descriptors(name, idx, full + ".", dc.get("descriptors") or [])

    def arrays(self):
        """-> (nodes as a structured array of rl_config_node, key bytes, prefix bytes)."""
        n = len(self.parent)
        nodes = np.zeros(n, abi.CONFIG_NODE_DTYPE)
        lens = np.array([len(k) for k in self.keys], np.uint32)
        offs = np.zeros(n, np.uint32)
        if n:
            offs[1:] = np.cumsum(lens)[:-1]
        nodes["parent"] = self.parent
        nodes["key_off"] = offs
        nodes["key_len"] = lens
        rows = np.array(self.rows, np.uint32).reshape(n, 6)
        for j, f in enumerate(("requests_per_unit", "rule_id", "unit", "has_limit", "unlimited", "shadow_mode")):
            nodes[f] = rows[:, j]
        kb = np.frombuffer(b"".join(self.keys) or b"\0", np.uint8).copy()
        pre = np.frombuffer(self.prefix.encode() or b"\0", np.uint8).copy()
        return nodes, kb, pre


def descriptor_key(domain: str, entries: Sequence[Tuple[str, str]]) -> str:
    """descriptorKey (config_impl.go:300-312): the stats key of an override."""
    parts = [k + ("_" + v if v != "" else "") for k, v in entries]
    return domain + "." + ".".join(parts)


def pack_requests(requests, nows, interner: RuleInterner) -> Dict[str, np.ndarray]:
    """RateLimitRequests (arrival order) with their ``now`` -> rl_request_batch arrays.

    ``requests`` carry ``domain``, ``descriptors`` (each with ``entries`` [(k, v)]
    and an optional ``limit`` override {requests_per_unit, unit}) and
    ``hits_addend``. Override stats keys are interned here (descriptorKey)."""
    dom = bytearray()
    dom_off = [0]
    hits, req_idx, entry_first, desc_off = [], [], [0], [0]
    desc = bytearray()
    klen, vlen = [], []
    ovf, ovr, ovu, ovrule = [], [], [], []
    for q, r in enumerate(requests):
        dom += r.domain.encode()
        dom_off.append(len(dom))
        hits.append(r.hits_addend & 0xFFFFFFFF)
        for d in r.descriptors:
            req_idx.append(q)
            for k, v in d.entries:
                kb, vb = k.encode(), v.encode()
                desc += kb + b"_" + vb + b"_"
                klen.append(len(kb))
                vlen.append(len(vb))
            entry_first.append(len(klen))
            desc_off.append(len(desc))
            lim = getattr(d, "limit", None)
            if lim is not None:
                ovf.append(1)
                ovr.append(lim.requests_per_unit)
                ovu.append(lim.unit)
                ovrule.append(interner.intern(descriptor_key(r.domain, d.entries)))
            else:
                ovf.append(0)
                ovr.append(0)
                ovu.append(0)
                ovrule.append(0)
    D = abi.REQUEST_DTYPES
    a = {"domain_bytes": np.frombuffer(bytes(dom) or b"\0", np.uint8).copy(),
         "domain_off": np.array(dom_off, D["domain_off"]), "now": np.array(nows, D["now"]),
         "hits": np.array(hits, D["hits"]), "req_idx": np.array(req_idx, D["req_idx"]),
         "entry_first": np.array(entry_first, D["entry_first"]), "desc_off": np.array(desc_off, D["desc_off"]),
         "desc_bytes": np.frombuffer(bytes(desc) or b"\0", np.uint8).copy(),
         "key_len": np.array(klen, D["key_len"]), "value_len": np.array(vlen, D["value_len"])}
    if any(ovf):
        a.update(override_flags=np.array(ovf, np.uint8), override_rpu=np.array(ovr, np.uint32),
                 override_unit=np.array(ovu, np.uint8), override_rule=np.array(ovrule, np.uint32))
    else:
        a.update(override_flags=None, override_rpu=None, override_unit=None, override_rule=None)
    return a


class RequestPacker:
    """rl_packer: serialized RateLimitRequest messages -> rl_request_batch
    (native, no per-descriptor Python objects). Override stats keys get rule
    ids from ``first_override_rule`` up (config rules take the ids below)."""

    def __init__(self, first_override_rule: int):
        import ctypes as C
        from ._lib import lib
        self._C, self._lib = C, lib()
        self.h = self._lib.rl_packer_create(first_override_rule)
        self._keep = None

    def close(self):
        if getattr(self, "h", None):
            self._lib.rl_packer_destroy(self.h)
            self.h = None

    __del__ = close

    def pack(self, messages, nows) -> "abi.RlRequestBatch":
        """-> an RlRequestBatch over packer-owned arrays (valid until the next pack)."""
        from ._lib import RedisError
        C = self._C
        buf = np.frombuffer(b"".join(messages) or b"\0", np.uint8)
        off = np.zeros(len(messages) + 1, np.uint64)
        off[1:] = np.cumsum([len(m) for m in messages])
        now = np.ascontiguousarray(nows, np.int64)
        self._keep = (buf, off, now)
        b = abi.RlRequestBatch()
        rc = self._lib.rl_packer_pack(self.h, abi.ptr(buf), abi.ptr(off), len(messages), abi.ptr(now), C.byref(b))
        if rc:
            raise RedisError(self._lib.rl_packer_last_error(self.h).decode())
        return b

    def rules(self) -> int:
        return self._lib.rl_packer_rules(self.h)

    def rule_key(self, rule_id: int):
        k = self._lib.rl_packer_rule_key(self.h, rule_id)
        return None if k is None else k.decode()


def batch_arrays(b) -> Dict[str, np.ndarray]:
    """Copy an RlRequestBatch's arrays into numpy (tests and inspection)."""
    import ctypes as C
    n, nq, ne = b.n_descriptors, b.n_requests, b.n_entries

    def arr(p, count, dt):
        if not p or count == 0:
            return np.zeros(0, dt)
        return np.ctypeslib.as_array((C.c_uint8 * (count * np.dtype(dt).itemsize)).from_address(p)).view(dt).copy()

    dom_off = arr(b.domain_off, nq + 1, np.uint32)
    desc_off = arr(b.desc_off, n + 1, np.uint32)
    return {"domain_off": dom_off, "domain_bytes": arr(b.domain_bytes, int(dom_off[-1]) if nq else 0, np.uint8),
            "now": arr(b.now, nq, np.int64), "hits": arr(b.hits, nq, np.uint32), "req_idx": arr(b.req_idx, n, np.uint32),
            "entry_first": arr(b.entry_first, n + 1, np.uint32), "desc_off": desc_off,
            "desc_bytes": arr(b.desc_bytes, int(desc_off[-1]) if n else 0, np.uint8),
            "key_len": arr(b.key_len, ne, np.uint16), "value_len": arr(b.value_len, ne, np.uint16),
            "override_flags": arr(b.override_flags, n, np.uint8), "override_rpu": arr(b.override_rpu, n, np.uint32),
            "override_unit": arr(b.override_unit, n, np.uint8), "override_rule": arr(b.override_rule, n, np.uint32)}
