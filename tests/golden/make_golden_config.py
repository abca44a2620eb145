"""Write tests/golden/ref_config.json: GetLimit known answers transcribed from
the reference's config tests (test/config/config_test.go), with the YAML data
files those tests load (test/config/*.yaml) as inputs.

Every expected value is copied by hand from the cited test line; nothing is
computed. Re-run with ``python tests/golden/make_golden_config.py``.

Schema:
  files{name: yaml text}
  lookups[]: config (file names), domain, entries [[k, v]..], override null|[rpu, unit],
             expect null | {rpu, unit, full_key, unlimited, shadow}  (shadow null = unasserted)
  load_errors[]: files, error (the panic message)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SEC, MIN, HOUR, DAY = 1, 2, 3, 4

# test/config/basic_config.yaml
BASIC = """\
domain: test-domain
descriptors:
  - key: key1
    value: value1
    descriptors:
      - key: subkey1
        rate_limit:
          unit: second
          requests_per_unit: 5
      - key: subkey1
        value: subvalue1
        rate_limit:
          unit: second
          requests_per_unit: 10
  - key: key2
    rate_limit:
      unit: minute
      requests_per_unit: 20
  - key: key2
    value: value2
    rate_limit:
      unit: minute
      requests_per_unit: 30
  - key: key2
    value: value3
  - key: key3
    rate_limit:
      unit: hour
      requests_per_unit: 1
  - key: key4
    rate_limit:
      unit: day
      requests_per_unit: 1
  - key: key5
    value: value5
    rate_limit:
      unit: day
      requests_per_unit: 15
    descriptors:
      - key: subkey5
        value: subvalue5
        rate_limit:
          unit: day
          requests_per_unit: 25
  - key: key6
    rate_limit:
      unlimited: true
"""

# test/config/shadowmode_config.yaml
SHADOW = """\
domain: test-domain
descriptors:
  - key: key1
    value: value1
    descriptors:
      - key: subkey1
        rate_limit:
          unit: second
          requests_per_unit: 5
      - key: subkey1
        value: subvalue1
        rate_limit:
          unit: second
          requests_per_unit: 10
        shadow_mode: true
  - key: key2
    rate_limit:
      unit: minute
      requests_per_unit: 20
    shadow_mode: true
  - key: key2
    value: value2
    rate_limit:
      unit: minute
      requests_per_unit: 30
"""

FILES = {
    "basic_config.yaml": BASIC,
    "shadowmode_config.yaml": SHADOW,
    # the error cases' data files (test/config/*.yaml)
    "empty_domain.yaml": "descriptors:\n",
    "duplicate_domain.yaml": "domain: test-domain\ndescriptors:\n",
    "empty_key.yaml": "domain: test-domain\ndescriptors:\n  - value: value1\n",
    "duplicate_key.yaml": ("domain: test-domain\ndescriptors:\n  - key: key1\n    value: value1\n\n"
                           "  - key: key1\n    value: value1\n"),
    "bad_limit_unit.yaml": ("domain: test-domain\ndescriptors:\n  - key: key1\n    value: value1\n"
                            "    rate_limit:\n      unit: foo\n      requests_per_unit: 5\n"),
    "misspelled_key.yaml": ("domain: test-domain\ndescriptors:\n  - key: key1\n    value: value1\n"
                            "    ratelimit:\n      unit: day\n      requests_per_unit: 5\n"),
    "misspelled_key2.yaml": ("domain: test-domain\ndescriptors:\n  - key: key1\n    value: value1\n"
                             "    rate_limit:\n      unit: day\n      requestsperunit: 5\n"),
    "non_map_list.yaml": "domain: test-domain\ndescriptors:\n  - a\n  - b\n  - c\n",
    "unlimited_with_unit.yaml": ("domain: test-domain\ndescriptors:\n  - key: foo\n    rate_limit:\n"
                                 "      unlimited: true\n      unit: day\n      requests_per_unit: 25\n"),
}


def hit(rpu, unit, key, unlimited=False, shadow=None):
    return {"rpu": rpu, "unit": unit, "full_key": key, "unlimited": unlimited, "shadow": shadow}


def look(cfg, domain, entries, expect, override=None, src=""):
    return {"config": [cfg], "domain": domain, "entries": entries, "override": override, "expect": expect,
            "source": src}


B = "basic_config.yaml"
S = "shadowmode_config.yaml"
T = "test-domain"
lookups = [
    # TestBasicConfig, config_test.go:27-180
    look(B, "foo_domain", [], None, src="config_test.go:32"),
    look(B, T, [], None, src="config_test.go:33"),
    look(B, T, [["key1", "something"]], None, src="config_test.go:35-40"),
    look(B, T, [["key1", "value1"]], None, src="config_test.go:42-47"),
    look(B, T, [["key2", "value2"], ["subkey", "subvalue"]], None, src="config_test.go:49-54"),
    look(B, T, [["key5", "value5"], ["subkey5", "subvalue"]], None, src="config_test.go:56-61"),
    look(B, T, [["key1", "value1"], ["subkey1", "something"]], hit(5, SEC, "test-domain.key1_value1.subkey1"),
         src="config_test.go:63-77"),
    look(B, T, [["key1", "value1"], ["subkey1", "subvalue1"]],
         hit(10, SEC, "test-domain.key1_value1.subkey1_subvalue1"), src="config_test.go:79-97"),
    look(B, T, [["key2", "something"]], hit(20, MIN, "test-domain.key2"), src="config_test.go:99-113"),
    look(B, T, [["key2", "value2"]], hit(30, MIN, "test-domain.key2_value2"), src="config_test.go:115-129"),
    look(B, T, [["key2", "value3"]], None, src="config_test.go:131-136"),
    look(B, T, [["key3", "foo"]], hit(1, HOUR, "test-domain.key3"), src="config_test.go:138-152"),
    look(B, T, [["key4", "foo"]], hit(1, DAY, "test-domain.key4"), src="config_test.go:154-168"),
    look(B, T, [["key6", "foo"]], hit(0, 0, "test-domain.key6", unlimited=True), src="config_test.go:170-179"),
    # TestConfigLimitOverride, config_test.go:182-271
    look(B, "foo_domain", [], None, override=[10, DAY], src="config_test.go:189-193"),
    look(B, T, [["key1", "value1"], ["subkey1", "something"]],
         hit(10, DAY, "test-domain.key1_value1.subkey1_something", shadow=False), override=[10, DAY],
         src="config_test.go:195-217"),
    look(B, T, [["key1", "value1"], ["subkey1", "something"]],
         hit(42, HOUR, "test-domain.key1_value1.subkey1_something", shadow=False), override=[42, HOUR],
         src="config_test.go:219-244"),
    look(B, T, [["key1", "value1"], ["subkey1", "something_else"]],
         hit(42, HOUR, "test-domain.key1_value1.subkey1_something_else", shadow=False), override=[42, HOUR],
         src="config_test.go:246-270"),
    # TestShadowModeConfig, config_test.go:391-466
    look(S, T, [["key1", "value1"], ["subkey1", "something"]],
         hit(5, SEC, "test-domain.key1_value1.subkey1", shadow=False), src="config_test.go:398-409"),
    look(S, T, [["key1", "value1"], ["subkey1", "subvalue1"]],
         hit(10, SEC, "test-domain.key1_value1.subkey1_subvalue1", shadow=True), src="config_test.go:415-427"),
    look(S, T, [["key2", "something"]], hit(20, MIN, "test-domain.key2", shadow=True), src="config_test.go:433-444"),
    look(S, T, [["key2", "value2"]], hit(30, MIN, "test-domain.key2_value2", shadow=False),
         src="config_test.go:450-461"),
]

load_errors = [
    {"files": ["empty_domain.yaml"], "error": "empty_domain.yaml: config file cannot have empty domain",
     "source": "config_test.go:273-281"},
    {"files": ["basic_config.yaml", "duplicate_domain.yaml"],
     "error": "duplicate_domain.yaml: duplicate domain 'test-domain' in config file", "source": "config_test.go:283-292"},
    {"files": ["empty_key.yaml"], "error": "empty_key.yaml: descriptor has empty key", "source": "config_test.go:294-303"},
    {"files": ["duplicate_key.yaml"],
     "error": "duplicate_key.yaml: duplicate descriptor composite key 'test-domain.key1_value1'",
     "source": "config_test.go:305-314"},
    {"files": ["bad_limit_unit.yaml"], "error": "bad_limit_unit.yaml: invalid rate limit unit 'foo'",
     "source": "config_test.go:316-325"},
    {"files": ["misspelled_key.yaml"], "error": "misspelled_key.yaml: config error, unknown key 'ratelimit'",
     "source": "config_test.go:338-347"},
    {"files": ["misspelled_key2.yaml"],
     "error": "misspelled_key2.yaml: config error, unknown key 'requestsperunit'", "source": "config_test.go:349-356"},
    {"files": ["non_map_list.yaml"],
     "error": "non_map_list.yaml: config error, yaml file contains list of type other than map: a",
     "source": "config_test.go:369-378"},
    {"files": ["unlimited_with_unit.yaml"],
     "error": "unlimited_with_unit.yaml: should not specify rate limit unit when unlimited",
     "source": "config_test.go:380-389"},
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "ref_config.json"), "w") as f:
        json.dump({"kind": "config", "files": FILES, "lookups": lookups, "load_errors": load_errors}, f, indent=1)
    print("wrote ref_config.json: %d lookups, %d load errors" % (len(lookups), len(load_errors)))
