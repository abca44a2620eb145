/* san_run.c — the host C/C++ code under AddressSanitizer and UBSan (test
 * program; tests/test_sanitize_cpu.py builds it with -fsanitize=address,
 * undefined and -fno-sanitize-recover=all, so the first finding aborts).
 *
 * Two inputs, written by the test:
 *   packer file: groups of serialized RateLimitRequest messages, each
 *     [u32 n][u64 off[n + 1]][bytes][i64 now[n]] — valid ones, and malformed
 *     ones (every truncation, flipped bytes, bad field numbers and lengths):
 *     rl_packer_pack (ratelimit_amd/csrc/rl_pack.cpp) parses every group; the
 *     program prints the status and, on success, a digest of the batch;
 *   oracle file: packed batches [u32 n, n_requests, n_rules, mt][stem_off]
 *     [stem bytes][now][req_idx][unit][flags][limit][hits][rule_id]: run
 *     through the C restatement oracle (oracle/rl_oracle.c), sequentially and
 *     sharded over threads (mt); the program prints every answer, which the
 *     test compares with the unsanitized oracle's.
 * The reference runs its Go tests under the race detector (Makefile:66-72);
 * this is the host code's counterpart. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ratelimit_hip.h"

typedef struct rlo_ctx rlo_ctx;
typedef struct rlo_mt rlo_mt;
rlo_ctx* rlo_create(float near_limit_ratio, int local_cache, int per_second);
void rlo_destroy(rlo_ctx* c);
int rlo_do_limit(rlo_ctx* c, const rl_batch* b, rl_result* o);
rlo_mt* rlo_mt_create(float near_limit_ratio, int local_cache, int per_second, int threads);
void rlo_mt_destroy(rlo_mt* m);
int rlo_mt_do_limit(rlo_mt* m, const rl_batch* b, rl_result* o);

static uint8_t* slurp(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *len = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* p = (uint8_t*)malloc(*len ? *len : 1);
  if (fread(p, 1, *len, f) != *len) {
    fclose(f);
    free(p);
    return NULL;
  }
  fclose(f);
  return p;
}

/* a copy of len bytes at *pos in its own heap block (so ASan sees its bounds) */
static void* take(const uint8_t* buf, size_t len, size_t* pos, size_t n) {
  if (*pos + n > len) {
    fprintf(stderr, "san_run: input truncated\n");
    exit(2);
  }
  void* p = malloc(n ? n : 1);
  memcpy(p, buf + *pos, n);
  *pos += n;
  return p;
}

static uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
  return h;
}

static int run_packer(const char* path) {
  size_t len, pos = 0;
  uint8_t* buf = slurp(path, &len);
  if (!buf) return 2;
  rl_packer* k = rl_packer_create(7);
  int groups = 0;
  while (pos < len) {
    uint32_t* n = (uint32_t*)take(buf, len, &pos, 4);
    uint64_t* off = (uint64_t*)take(buf, len, &pos, 8ull * (*n + 1));
    uint8_t* msgs = (uint8_t*)take(buf, len, &pos, off[*n]);
    int64_t* now = (int64_t*)take(buf, len, &pos, 8ull * *n);
    rl_request_batch b;
    memset(&b, 0, sizeof b);
    const int rc = rl_packer_pack(k, msgs, off, *n, now, &b);
    uint64_t h = 0xcbf29ce484222325ull;
    if (rc == RL_OK) {
      h = fnv(h, b.domain_off, 4ull * (b.n_requests + 1));
      h = fnv(h, b.domain_bytes, b.domain_off[b.n_requests]);
      h = fnv(h, b.now, 8ull * b.n_requests);
      h = fnv(h, b.hits, 4ull * b.n_requests);
      h = fnv(h, b.req_idx, 4ull * b.n_descriptors);
      h = fnv(h, b.entry_first, 4ull * (b.n_descriptors + 1));
      h = fnv(h, b.desc_off, 4ull * (b.n_descriptors + 1));
      h = fnv(h, b.desc_bytes, b.desc_off[b.n_descriptors]);
      h = fnv(h, b.key_len, 2ull * b.n_entries);
      h = fnv(h, b.value_len, 2ull * b.n_entries);
      if (b.override_flags) {
        h = fnv(h, b.override_flags, b.n_descriptors);
        h = fnv(h, b.override_rpu, 4ull * b.n_descriptors);
        h = fnv(h, b.override_unit, b.n_descriptors);
        h = fnv(h, b.override_rule, 4ull * b.n_descriptors);
      }
      for (uint32_t r = 7; r < rl_packer_rules(k); r++) {
        const char* key = rl_packer_rule_key(k, r);
        h = fnv(h, key, strlen(key));
      }
    }
    printf("P %d %d %u %u %016llx\n", groups, rc, rc == RL_OK ? b.n_requests : 0u, rc == RL_OK ? b.n_descriptors : 0u,
           (unsigned long long)h);
    free(n); free(off); free(msgs); free(now);
    groups++;
  }
  rl_packer_destroy(k);
  free(buf);
  return 0;
}

static int run_oracle(const char* path) {
  size_t len, pos = 0;
  uint8_t* buf = slurp(path, &len);
  if (!buf) return 2;
  rlo_ctx* seq = rlo_create(0.8f, 1, 0);
  rlo_mt* mt = rlo_mt_create(0.8f, 1, 0, 3);
  int batches = 0;
  while (pos < len) {
    uint32_t* hd = (uint32_t*)take(buf, len, &pos, 16);
    const uint32_t n = hd[0], nq = hd[1], nr = hd[2], use_mt = hd[3];
    rl_batch b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.n_requests = nq;
    b.n_rules = nr;
    uint32_t* off = (uint32_t*)take(buf, len, &pos, 4ull * (n + 1));
    b.stem_off = off;
    b.stem_bytes = (const uint8_t*)take(buf, len, &pos, off[n]);
    b.now = (const int64_t*)take(buf, len, &pos, 8ull * nq);
    b.req_idx = (const uint32_t*)take(buf, len, &pos, 4ull * n);
    b.unit = (const uint8_t*)take(buf, len, &pos, n);
    b.flags = (const uint8_t*)take(buf, len, &pos, n);
    b.limit = (const uint32_t*)take(buf, len, &pos, 4ull * n);
    b.hits = (const uint32_t*)take(buf, len, &pos, 4ull * n);
    b.rule_id = (const uint32_t*)take(buf, len, &pos, 4ull * n);
    rl_result o;
    o.code = (uint8_t*)calloc(n ? n : 1, 1);
    o.limit_remaining = (uint32_t*)calloc(n ? n : 1, 4);
    o.reset_s = (uint32_t*)calloc(n ? n : 1, 4);
    o.stats = (uint64_t*)calloc((size_t)(nr ? nr : 1) * RL_NUM_STATS, 8);
    o.status = NULL;
    const int rc = use_mt ? rlo_mt_do_limit(mt, &b, &o) : rlo_do_limit(seq, &b, &o);
    uint64_t h = fnv(0xcbf29ce484222325ull, o.code, n);
    h = fnv(h, o.limit_remaining, 4ull * n);
    h = fnv(h, o.reset_s, 4ull * n);
    h = fnv(h, o.stats, 8ull * nr * RL_NUM_STATS);
    printf("O %d %d %016llx\n", batches, rc, (unsigned long long)h);
    free(o.code); free(o.limit_remaining); free(o.reset_s); free(o.stats);
    free((void*)b.stem_bytes); free((void*)b.now); free((void*)b.req_idx); free((void*)b.unit);
    free((void*)b.flags); free((void*)b.limit); free((void*)b.hits); free((void*)b.rule_id);
    free(off); free(hd);
    batches++;
  }
  rlo_destroy(seq);
  rlo_mt_destroy(mt);
  free(buf);
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: san_run <packer file> <oracle file>\n");
    return 2;
  }
  int rc = run_packer(argv[1]);
  if (!rc) rc = run_oracle(argv[2]);
  return rc;
}
