"""Config lookup (GetLimit) and the request-batch boundary, on the CPU:

* the oracle restatement (oracle/config.py) against the reference's own config
  tests (tests/golden/ref_config.json, transcribed from test/config/config_test.go);
* the product's flattened trie (ratelimit_amd/config.py) against the same
  files: node keys, rule ids and the loader's error messages;
* rl_config_node / rl_request_batch / rl_request_result layouts against the C
  compiler's view of include/ratelimit_hip.h.
"""
import ctypes as C
import json
import os
import subprocess

import pytest

from oracle.config import RateLimitConfig, RateLimitConfigError
from oracle.oracle import Descriptor, Limit
from ratelimit_amd import abi
from ratelimit_amd.config import ConfigTree, RateLimitConfigError as ProductConfigError, descriptor_key, \
    pack_requests
from ratelimit_amd.packing import RuleInterner
from ratelimit_amd.types import Descriptor as PDescriptor, Limit as PLimit, RateLimitRequest as PRequest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_config.json")))


def _files(names):
    return [(n, G["files"][n]) for n in names]


@pytest.mark.parametrize("case", G["lookups"], ids=lambda c: c["source"])
def test_oracle_get_limit_matches_reference_tests(case):
    cfg = RateLimitConfig(_files(case["config"]))
    ov = case["override"]
    d = Descriptor([tuple(e) for e in case["entries"]], Limit(*ov) if ov else None)
    rl = cfg.get_limit(case["domain"], d)
    exp = case["expect"]
    if exp is None:
        assert rl is None
        return
    assert rl is not None
    assert rl.full_key == exp["full_key"] and rl.stats.key == exp["full_key"]
    assert rl.unlimited == exp["unlimited"]
    if not exp["unlimited"]:
        assert (rl.limit.requests_per_unit, rl.limit.unit) == (exp["rpu"], exp["unit"])
    if exp["shadow"] is not None:
        assert rl.shadow_mode == exp["shadow"]


@pytest.mark.parametrize("case", G["load_errors"], ids=lambda c: c["source"])
def test_loader_errors_match_reference_tests(case):
    with pytest.raises(RateLimitConfigError) as e:
        RateLimitConfig(_files(case["files"]))
    assert str(e.value) == case["error"]
    with pytest.raises(ProductConfigError) as e2:
        ConfigTree.from_yaml(_files(case["files"]))
    assert str(e2.value) == case["error"]


def test_override_stats_key_is_descriptor_key():
    # config_test.go:211 / :238 / :262: FullKey of an override = descriptorKey
    assert descriptor_key("test-domain", [("key1", "value1"), ("subkey1", "something")]) == \
        "test-domain.key1_value1.subkey1_something"
    assert descriptor_key("d", [("a", ""), ("b", "c")]) == "d.a.b_c"


def test_flattened_tree_mirrors_loaded_config():
    t = ConfigTree.from_yaml(_files(["basic_config.yaml"]), "prefix:")
    nodes, kb, pre = t.arrays()
    assert bytes(pre) == b"prefix:"
    assert nodes[0]["parent"] == -1 and t.keys[0] == b"test-domain"
    keys = {t.full_key[i]: i for i in range(len(t.keys))}
    # every config rule is a node, keyed by its finalKey under its parent
    for fk, rpu, unit in (("test-domain.key1_value1.subkey1", 5, 1), ("test-domain.key2_value2", 30, 2),
                          ("test-domain.key5_value5.subkey5_subvalue5", 25, 4)):
        i = keys[fk]
        assert nodes[i]["has_limit"] == 1 and nodes[i]["requests_per_unit"] == rpu and nodes[i]["unit"] == unit
        assert t.interner.keys[nodes[i]["rule_id"]] == fk
        p = nodes[i]["parent"]
        assert t.full_key[p] + "." + t.keys[i].decode() == fk
    i = keys["test-domain.key6"]
    assert nodes[i]["unlimited"] == 1 and nodes[i]["unit"] == 0
    assert nodes[keys["test-domain.key2_value3"]]["has_limit"] == 0
    o = nodes["key_off"]
    for j in range(len(nodes)):
        assert bytes(kb[o[j]:o[j] + nodes[j]["key_len"]]) == t.keys[j]


def test_pack_requests_layout():
    it = RuleInterner()
    reqs = [PRequest("dom", [PDescriptor([("a", "1"), ("b", "")]), PDescriptor([("k", "v")], PLimit(7, 2))], 3),
            PRequest("d2", [PDescriptor([])], 0)]
    a = pack_requests(reqs, [100, 101], it)
    assert bytes(a["domain_bytes"]) == b"domd2" and list(a["domain_off"]) == [0, 3, 5]
    assert list(a["req_idx"]) == [0, 0, 1] and list(a["entry_first"]) == [0, 2, 3, 3]
    assert bytes(a["desc_bytes"][:a["desc_off"][-1]]) == b"a_1_b__k_v_"
    assert list(a["desc_off"]) == [0, 7, 11, 11]
    assert list(a["key_len"]) == [1, 1, 1] and list(a["value_len"]) == [1, 0, 1]
    assert list(a["override_flags"]) == [0, 1, 0] and a["override_rpu"][1] == 7 and a["override_unit"][1] == 2
    assert it.keys[a["override_rule"][1]] == "dom.k_v"
    assert list(a["hits"]) == [3, 0] and list(a["now"]) == [100, 101]


LAYOUT_C = r'''
#include <stddef.h>
#include <stdio.h>
#include "ratelimit_hip.h"
#define P(s, f) printf("%s.%s %zu\n", #s, #f, offsetof(s, f));
int main(void) {
  printf("rl_config_node %zu\nrl_config_tree %zu\nrl_request_batch %zu\nrl_request_result %zu\n",
         sizeof(rl_config_node), sizeof(rl_config_tree), sizeof(rl_request_batch), sizeof(rl_request_result));
  printf("rl_local_cache_info %zu\n", sizeof(rl_local_cache_info));
  P(rl_config_node, rule_id) P(rl_config_node, unit) P(rl_config_node, shadow_mode)
  P(rl_config_tree, nodes) P(rl_config_tree, key_bytes_len) P(rl_config_tree, cache_key_prefix)
  P(rl_request_batch, domain_bytes) P(rl_request_batch, override_rule)
  P(rl_request_result, match) P(rl_request_result, stats)
  return 0;
}
'''


def test_request_struct_layouts_match_c_compiler(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(l.split() for l in subprocess.check_output([str(exe)]).decode().splitlines())
    py = {"rl_config_node": C.sizeof(abi.RlConfigNode), "rl_config_tree": C.sizeof(abi.RlConfigTree),
          "rl_request_batch": C.sizeof(abi.RlRequestBatch), "rl_request_result": C.sizeof(abi.RlRequestResult),
          "rl_local_cache_info": C.sizeof(abi.RlLocalCacheInfo)}
    for k, v in py.items():
        assert int(got[k]) == v, k
    assert abi.CONFIG_NODE_DTYPE.itemsize == C.sizeof(abi.RlConfigNode)
    for s, cls in (("rl_config_node", abi.RlConfigNode), ("rl_config_tree", abi.RlConfigTree),
                   ("rl_request_batch", abi.RlRequestBatch), ("rl_request_result", abi.RlRequestResult)):
        for key, off in got.items():
            if key.startswith(s + "."):
                assert getattr(cls, key.split(".")[1]).offset == int(off), key
