"""Host packer (rl_packer, ratelimit_amd/csrc/rl_pack.cpp) on the CPU: serialized
RateLimitRequest messages -> rl_request_batch arrays, equal to the Python
packer's (ratelimit_amd.config.pack_requests) field by field; override stats
keys named as descriptorKey (config_impl.go:300-312); unknown fields skipped;
malformed messages rejected. Host code only: no GPU call."""
import random

import numpy as np
import pytest

from oracle import oracle as O
from ratelimit_amd.config import RequestPacker, batch_arrays, descriptor_key, pack_requests
from ratelimit_amd.packing import RuleInterner
from ratelimit_amd._lib import RedisError
import pbwire


def random_requests(seed, n):
    rng = random.Random(seed)
    reqs = []
    for _ in range(n):
        descs = []
        for _ in range(rng.randint(1, 4)):
            ents = [(rng.choice(["k", "key_x", "é", "remote_address", ""]), rng.choice(["", "v", "a_b", "1.2.3.4", "ü" * 3]))
                    for _ in range(rng.randint(0, 4))]
            lim = O.Limit(rng.randint(0, 50), rng.randint(0, 4)) if rng.random() < 0.2 else None
            descs.append(O.Descriptor(ents, lim))
        reqs.append(O.RateLimitRequest(rng.choice(["d", "domain_1", ""]), descs, rng.choice([0, 1, 7, 1 << 31])))
    return reqs


@pytest.mark.parametrize("seed", range(4))
def test_native_packer_equals_python_packer(seed):
    reqs = random_requests(seed, 300)
    nows = [1_700_000_000 + i // 10 for i in range(len(reqs))]
    it = RuleInterner()
    want = pack_requests(reqs, nows, it)
    pk = RequestPacker(first_override_rule=5)
    try:
        b = pk.pack([pbwire.encode_request(r, extra_unknown=(i % 3 == 0)) for i, r in enumerate(reqs)], nows)
        got = batch_arrays(b)
        for k in ("domain_off", "now", "hits", "req_idx", "entry_first", "desc_off", "key_len", "value_len"):
            assert np.array_equal(got[k], want[k]), k
        assert bytes(got["domain_bytes"]) == bytes(want["domain_bytes"][:want["domain_off"][-1]])
        assert bytes(got["desc_bytes"]) == bytes(want["desc_bytes"][:want["desc_off"][-1]])
        ovf = want["override_flags"] if want["override_flags"] is not None else np.zeros(b.n_descriptors, np.uint8)
        assert np.array_equal(got["override_flags"], ovf)
        m = ovf == 1
        if m.any():
            assert np.array_equal(got["override_rpu"][m], want["override_rpu"][m])
            assert np.array_equal(got["override_unit"][m], want["override_unit"][m])
            # same stats key names (descriptorKey), ids from 5 up
            names_got = [pk.rule_key(int(x)) for x in got["override_rule"][m]]
            names_want = [it.keys[int(x)] for x in want["override_rule"][m]]
            assert names_got == names_want
            assert min(got["override_rule"][m]) >= 5
        assert b.n_rules == 5 + len(set(names_got if m.any() else []))
        assert pk.rule_key(4) is None
    finally:
        pk.close()


def test_descriptor_key_of_packer_matches_reference_test():
    # config_test.go:211 (override FullKey = descriptorKey)
    req = O.RateLimitRequest("test-domain", [O.Descriptor([("key1", "value1"), ("subkey1", "something")],
                                                          O.Limit(10, 4))], 1)
    pk = RequestPacker(0)
    try:
        b = pk.pack([pbwire.encode_request(req)], [0])
        assert pk.rule_key(batch_arrays(b)["override_rule"][0]) == "test-domain.key1_value1.subkey1_something"
        assert descriptor_key("test-domain", [("key1", "value1"), ("subkey1", "something")]) == pk.rule_key(0)
    finally:
        pk.close()


def test_packer_rejects_malformed_messages():
    pk = RequestPacker(0)
    try:
        good = pbwire.encode_request(O.RateLimitRequest("d", [O.Descriptor([("k", "v")])], 1))
        for bad in (good[:-1], good[:5], b"\x12\xff\xff\xff\xff\x0f", b"\x0b"):
            with pytest.raises(RedisError, match="malformed"):
                pk.pack([bad], [0])
        b = pk.pack([good, b""], [0, 1])  # an empty message is an empty request
        assert b.n_requests == 2 and b.n_descriptors == 1
    finally:
        pk.close()


@pytest.mark.parametrize("where", ["request", "descriptor", "entry", "override"])
def test_packer_rejects_field_numbers_outside_protobuf_range(where):
    """field number 0 and numbers past 2^29 - 1 are invalid protobuf
    keys at every nesting level; a valid unknown field (2^29 - 1) is skipped."""
    ok_unknown = pbwire.varint((2 ** 29 - 1) << 3) + pbwire.varint(7)
    for tag, valid in ((0, False), ((2 ** 29) << 3, False), (ok_unknown, True)):
        junk = tag if isinstance(tag, bytes) else pbwire.varint(tag) + pbwire.varint(7)
        entry = pbwire.field_bytes(1, b"k") + pbwire.field_bytes(2, b"v")
        over = pbwire.field_varint(1, 5) + pbwire.field_varint(2, 1)
        if where == "entry":
            entry += junk
        if where == "override":
            over += junk
        desc = pbwire.field_bytes(1, entry) + pbwire.field_bytes(2, over)
        if where == "descriptor":
            desc += junk
        msg = pbwire.field_bytes(1, b"d") + pbwire.field_bytes(2, desc) + pbwire.field_varint(3, 1)
        if where == "request":
            msg += junk
        pk = RequestPacker(0)
        try:
            if valid:
                b = pk.pack([msg], [0])
                assert b.n_descriptors == 1
            else:
                with pytest.raises(RedisError, match="malformed"):
                    pk.pack([msg], [0])
        finally:
            pk.close()
