/* abi_layout.c — the C ABI as a C99 compiler sees it (test program).
 *
 * Compiled with `gcc -x c -std=c99 -Wall -Wextra -pedantic` against
 * include/ratelimit_hip.h alone (no HIP, no C++): proves the header is plain
 * C, and prints one line per struct ("S name size") and per field
 * ("F struct field offset size") for tests/test_c_abi.py to compare with the
 * ctypes mirror in ratelimit_amd/abi.py, which the Python adapter (and the cgo
 * adapter in go/src/gpu) relies on. */
#include <stddef.h>
#include <stdio.h>

#include "ratelimit_hip.h"

#define S(T) printf("S %s %zu\n", #T, sizeof(T))
#define F(T, f) printf("F %s %s %zu %zu\n", #T, #f, offsetof(T, f), sizeof(((T*)0)->f))

int main(void) {
  S(rl_config);
  F(rl_config, table_slots); F(rl_config, arena_bytes); F(rl_config, max_batch); F(rl_config, max_requests);
  F(rl_config, max_rules); F(rl_config, max_stem_bytes); F(rl_config, near_limit_ratio);
  F(rl_config, local_cache_enabled); F(rl_config, per_second_split); F(rl_config, device);
  F(rl_config, expiration_jitter_max_seconds); F(rl_config, hash_seed); F(rl_config, n_shards);
  F(rl_config, debug_hash_bits); F(rl_config, shard_device); F(rl_config, history_entries);
  F(rl_config, reserved);

  S(rl_batch);
  F(rl_batch, n); F(rl_batch, n_requests); F(rl_batch, n_rules); F(rl_batch, reserved); F(rl_batch, stem_bytes);
  F(rl_batch, stem_off); F(rl_batch, now); F(rl_batch, req_idx); F(rl_batch, unit); F(rl_batch, flags);
  F(rl_batch, limit); F(rl_batch, hits); F(rl_batch, rule_id);

  S(rl_limit);
  F(rl_limit, requests_per_unit); F(rl_limit, rule_id); F(rl_limit, unit); F(rl_limit, flags); F(rl_limit, reserved);

  S(rl_batch_compact);
  F(rl_batch_compact, n); F(rl_batch_compact, n_requests); F(rl_batch_compact, n_rules);
  F(rl_batch_compact, n_limits); F(rl_batch_compact, buf); F(rl_batch_compact, buf_bytes);
  F(rl_batch_compact, stem_bytes); F(rl_batch_compact, stem_off); F(rl_batch_compact, limit_idx);
  F(rl_batch_compact, req_first); F(rl_batch_compact, now); F(rl_batch_compact, hits); F(rl_batch_compact, limits);

  S(rl_batch_prefixed);
  F(rl_batch_prefixed, n); F(rl_batch_prefixed, n_requests); F(rl_batch_prefixed, n_rules);
  F(rl_batch_prefixed, n_limits); F(rl_batch_prefixed, buf); F(rl_batch_prefixed, buf_bytes);
  F(rl_batch_prefixed, req); F(rl_batch_prefixed, now); F(rl_batch_prefixed, hits); F(rl_batch_prefixed, desc);
  F(rl_batch_prefixed, prefix_bytes); F(rl_batch_prefixed, suffix_bytes); F(rl_batch_prefixed, limits);
  F(rl_batch_prefixed, index);

  S(rl_result);
  F(rl_result, code); F(rl_result, limit_remaining); F(rl_result, reset_s); F(rl_result, stats);
  F(rl_result, status);

  S(rl_restore_batch);
  F(rl_restore_batch, n); F(rl_restore_batch, reserved); F(rl_restore_batch, stem_bytes);
  F(rl_restore_batch, stem_off); F(rl_restore_batch, unit); F(rl_restore_batch, now); F(rl_restore_batch, count);
  F(rl_restore_batch, lc);

  S(rl_table_info);
  F(rl_table_info, table_slots); F(rl_table_info, live_slots); F(rl_table_info, tombstones);
  F(rl_table_info, arena_bytes_used); F(rl_table_info, exact_stems); F(rl_table_info, batches);
  F(rl_table_info, decisions); F(rl_table_info, history_entries); F(rl_table_info, history_appended);
  F(rl_table_info, history_lost); F(rl_table_info, history_slots); F(rl_table_info, history_refused);

  S(rl_log_tear);
  F(rl_log_tear, armed); F(rl_log_tear, protocol); F(rl_log_tear, sched); F(rl_log_tear, entry);
  F(rl_log_tear, before); F(rl_log_tear, seen); F(rl_log_tear, verdict); F(rl_log_tear, reserved);

  S(rl_config_node);
  F(rl_config_node, parent); F(rl_config_node, key_off); F(rl_config_node, key_len);
  F(rl_config_node, requests_per_unit); F(rl_config_node, rule_id); F(rl_config_node, unit);
  F(rl_config_node, has_limit); F(rl_config_node, unlimited); F(rl_config_node, shadow_mode);

  S(rl_config_tree);
  F(rl_config_tree, n_nodes); F(rl_config_tree, cache_key_prefix_len); F(rl_config_tree, nodes);
  F(rl_config_tree, key_bytes); F(rl_config_tree, key_bytes_len); F(rl_config_tree, cache_key_prefix);

  S(rl_request_batch);
  F(rl_request_batch, n_requests); F(rl_request_batch, n_descriptors); F(rl_request_batch, n_entries);
  F(rl_request_batch, n_rules); F(rl_request_batch, domain_bytes); F(rl_request_batch, domain_off);
  F(rl_request_batch, now); F(rl_request_batch, hits); F(rl_request_batch, req_idx);
  F(rl_request_batch, entry_first); F(rl_request_batch, desc_off); F(rl_request_batch, desc_bytes);
  F(rl_request_batch, key_len); F(rl_request_batch, value_len); F(rl_request_batch, override_flags);
  F(rl_request_batch, override_rpu); F(rl_request_batch, override_unit); F(rl_request_batch, override_rule);

  S(rl_request_result);
  F(rl_request_result, code); F(rl_request_result, limit_remaining); F(rl_request_result, reset_s);
  F(rl_request_result, match); F(rl_request_result, rule_id); F(rl_request_result, requests_per_unit);
  F(rl_request_result, unit); F(rl_request_result, stats);

  S(rl_local_cache_info);
  F(rl_local_cache_info, entry_count); F(rl_local_cache_info, lookup_count); F(rl_local_cache_info, hit_count);
  F(rl_local_cache_info, miss_count);

  printf("C RL_ABI_VERSION %u\n", (unsigned)RL_ABI_VERSION);
  printf("C RL_NUM_STATS %u\n", (unsigned)RL_NUM_STATS);
  printf("C RL_WIRE_BYTES %u\n", (unsigned)RL_WIRE_BYTES);
  printf("C RL_COMM_ID_BYTES %u\n", (unsigned)RL_COMM_ID_BYTES);
  return 0;
}
