/* abi_run.c — DoLimit through the C ABI from a C99 program (GPU test program).
 *
 * What a cgo adapter does, minus Go: rl_create from an rl_config, one
 * rl_do_limit per packed batch (host buffers), rl_destroy. Reads the batches
 * from a fixture file written by tests/test_c_abi.py and writes every result
 * array to an output file that the test compares with the C oracle:
 *
 *   in:  "RLFX" u32 version=1, u32 n_batches, f32 near_limit_ratio, u32
 *        local_cache, u32 per_second; per batch: u32 n, n_requests, n_rules,
 *        stem bytes; stem_bytes, stem_off[n+1] u32, now[n_requests] i64,
 *        req_idx[n] u32, unit[n] u8, flags[n] u8, limit[n] u32, hits[n] u32,
 *        rule_id[n] u32
 *   out: per batch code[n] u8, limit_remaining[n] u32, reset_s[n] u32,
 *        stats[n_rules x RL_NUM_STATS] u64
 *
 * usage: abi_run <in> <out>; exit status 0 on success. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ratelimit_hip.h"

static int rd(FILE* f, void* p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

static void* grab(FILE* f, size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p || !rd(f, p, n)) {
    fprintf(stderr, "abi_run: short fixture\n");
    exit(2);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: abi_run <in> <out>\n");
    return 2;
  }
  FILE* in = fopen(argv[1], "rb");
  FILE* out = fopen(argv[2], "wb");
  if (!in || !out) {
    fprintf(stderr, "abi_run: cannot open files\n");
    return 2;
  }
  char magic[4];
  uint32_t version, n_batches, lc, ps;
  float ratio;
  if (!rd(in, magic, 4) || memcmp(magic, "RLFX", 4) || !rd(in, &version, 4) || version != 1 ||
      !rd(in, &n_batches, 4) || !rd(in, &ratio, 4) || !rd(in, &lc, 4) || !rd(in, &ps, 4)) {
    fprintf(stderr, "abi_run: bad fixture header\n");
    return 2;
  }
  if (rl_abi_version() != RL_ABI_VERSION) {
    fprintf(stderr, "abi_run: library ABI %u, header %u\n", rl_abi_version(), (unsigned)RL_ABI_VERSION);
    return 3;
  }
  rl_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.table_slots = 1u << 16;
  cfg.max_batch = 1u << 15;
  cfg.max_rules = 1024;
  cfg.near_limit_ratio = ratio;
  cfg.local_cache_enabled = (int32_t)lc;
  cfg.per_second_split = (int32_t)ps;
  char err[512];
  rl_ctx* ctx = rl_create(&cfg, err, sizeof err);
  if (!ctx) {
    fprintf(stderr, "abi_run: rl_create: %s\n", err);
    return 4;
  }
  for (uint32_t k = 0; k < n_batches; k++) {
    uint32_t hdr[4];
    if (!rd(in, hdr, sizeof hdr)) {
      fprintf(stderr, "abi_run: short fixture\n");
      return 2;
    }
    const uint32_t n = hdr[0], nq = hdr[1], nr = hdr[2], nb = hdr[3];
    rl_batch b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.n_requests = nq;
    b.n_rules = nr;
    b.stem_bytes = (const uint8_t*)grab(in, nb);
    b.stem_off = (const uint32_t*)grab(in, (n + 1) * 4ull);
    b.now = (const int64_t*)grab(in, nq * 8ull);
    b.req_idx = (const uint32_t*)grab(in, n * 4ull);
    b.unit = (const uint8_t*)grab(in, n);
    b.flags = (const uint8_t*)grab(in, n);
    b.limit = (const uint32_t*)grab(in, n * 4ull);
    b.hits = (const uint32_t*)grab(in, n * 4ull);
    b.rule_id = (const uint32_t*)grab(in, n * 4ull);
    rl_result r;
    memset(&r, 0, sizeof r);
    r.code = (uint8_t*)calloc(n ? n : 1, 1);
    r.limit_remaining = (uint32_t*)calloc(n ? n : 1, 4);
    r.reset_s = (uint32_t*)calloc(n ? n : 1, 4);
    r.stats = (uint64_t*)calloc(nr ? nr * RL_NUM_STATS : 1, 8);
    const int rc = rl_do_limit(ctx, &b, &r);
    if (rc != RL_OK) {
      fprintf(stderr, "abi_run: rl_do_limit batch %u: %d %s\n", k, rc, rl_last_error(ctx));
      return 5;
    }
    fwrite(r.code, 1, n, out);
    fwrite(r.limit_remaining, 4, n, out);
    fwrite(r.reset_s, 4, n, out);
    fwrite(r.stats, 8, (size_t)nr * RL_NUM_STATS, out);
    free((void*)b.stem_bytes); free((void*)b.stem_off); free((void*)b.now); free((void*)b.req_idx);
    free((void*)b.unit); free((void*)b.flags); free((void*)b.limit); free((void*)b.hits); free((void*)b.rule_id);
    free(r.code); free(r.limit_remaining); free(r.reset_s); free(r.stats);
  }
  rl_table_info info;
  if (rl_table_info_get(ctx, &info) != RL_OK) return 6;
  printf("{\"batches\": %u, \"live_slots\": %llu}\n", n_batches, (unsigned long long)info.live_slots);
  rl_destroy(ctx);
  fclose(in);
  fclose(out);
  return 0;
}
