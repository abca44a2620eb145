/*
 * rl_oracle.c — TEST INFRASTRUCTURE ONLY: sequential C restatement of the
 * reference's fixed-window DoLimit path, over the packed rl_batch format of
 * include/ratelimit_hip.h.  Linked/loaded only by tests/, smoke() and
 * bench.py's cpu_baseline leg; never by the product library.
 *
 * Follows, line by line (reference read as text; no Go toolchain here):
 *   fixedRateLimitCacheImpl.DoLimit       src/redis/fixed_cache_impl.go:33-113
 *   BaseRateLimiter.GenerateCacheKeys     src/limiter/base_limiter.go:45-60
 *   CacheKeyGenerator.GenerateCacheKey    src/limiter/cache_key.go:48-80
 *   IsOverLimitWithLocalCache             base_limiter.go:63-72
 *   GetResponseDescriptorStatus           base_limiter.go:76-135
 *   checkOverLimitThreshold/NearLimit     base_limiter.go:150-179
 *   UnitToDivider / CalculateReset / Max  src/utils/utilities.go:17-43
 * with redis-server INCRBY/EXPIRE (lazy expiry: live while now <= expire) and
 * freecache Get/Set (hit while now < expireAt) modelled as in oracle/oracle.py.
 * Keys are materialised as real strings: prefix‖domain‖'_'‖Σ(k‖'_'‖v‖'_') is the
 * packed stem, followed by strconv.FormatInt((now/div)*div, 10).
 * Pinned against tests/golden (see tests/test_c_oracle.py).
 */
#define _POSIX_C_SOURCE 200809L /* pthread_barrier_t under -std=c11 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ratelimit_hip.h"

/* ------------------------------------------------------------------ string map */
typedef struct {
  uint64_t h;      /* 0 = empty */
  uint64_t off;    /* key bytes in arena */
  uint32_t len;
  uint32_t count;
  int64_t expire;  /* redis: -1 = no TTL; lc: expireAt */
  int64_t slack;   /* GC_WINDOWS windows of the largest unit that wrote the key */
} ent_t;

/* Garbage collection (smap_rebuild) drops an entry only once it is dead for
 * any request up to GC_WINDOWS windows of its unit, or horizon + 2 windows,
 * behind the request that triggers the rebuild. Liveness is judged against
 * each request's own clock (lazy expiry), so with time moving backwards an
 * entry dead at one request is live again for an earlier one; the slack keeps
 * every entry a request within that lag can read (the GPU table's history
 * answers as far: HIST_W windows, or div + J seconds). GC is an
 * implementation detail of this restatement: the reference's Redis keys have
 * no window limit, so streams whose clocks lag further are outside what the
 * oracle models. */
#define GC_WINDOWS 8

typedef struct {
  ent_t* e;
  uint64_t cap, used;
  char* arena;
  uint64_t arena_used, arena_cap;
  int is_lc;  /* liveness rule differs: redis now<=expire, freecache now<expire */
  int64_t horizon;  /* extra lag kept (rlo_set_horizon): the GPU's history horizon J */
} smap_t;

static uint64_t hash_bytes(const char* p, uint32_t n) {
  uint64_t h = 1469598103934665603ull; /* FNV-1a 64 */
  for (uint32_t i = 0; i < n; i++) { h ^= (uint8_t)p[i]; h *= 1099511628211ull; }
  h ^= h >> 29; h *= 0xbf58476d1ce4e5b9ull; h ^= h >> 32;
  return h ? h : 1;
}

static int live(const smap_t* m, const ent_t* e, int64_t now) {
  if (m->is_lc) return now < e->expire;
  return e->expire < 0 || now <= e->expire;
}

static void smap_init(smap_t* m, uint64_t cap, int is_lc) {
  m->cap = cap; m->used = 0; m->is_lc = is_lc;
  m->e = (ent_t*)calloc(cap, sizeof(ent_t));
  m->arena_cap = 1 << 20; m->arena_used = 0;
  m->arena = (char*)malloc(m->arena_cap);
}

static void smap_free(smap_t* m) { free(m->e); free(m->arena); }

static ent_t* smap_find(smap_t* m, const char* k, uint32_t n, uint64_t h) {
  uint64_t mask = m->cap - 1, i = h & mask;
  for (;;) {
    ent_t* e = &m->e[i];
    if (!e->h) return e; /* empty: insertion point */
    if (e->h == h && e->len == n && memcmp(m->arena + e->off, k, n) == 0) return e;
    i = (i + 1) & mask;
  }
}

static void smap_rebuild(smap_t* m, int64_t now) {
  uint64_t live_n = 0;
  for (uint64_t i = 0; i < m->cap; i++)
    if (m->e[i].h && live(m, &m->e[i], now - m->e[i].slack)) live_n++;
  uint64_t ncap = m->cap;
  while (live_n * 4 > ncap) ncap *= 2;
  ent_t* old = m->e; uint64_t ocap = m->cap; char* oar = m->arena;
  m->e = (ent_t*)calloc(ncap, sizeof(ent_t)); m->cap = ncap; m->used = 0;
  m->arena_cap = 1 << 20; while (m->arena_cap < m->arena_used) m->arena_cap *= 2;
  m->arena = (char*)malloc(m->arena_cap); m->arena_used = 0;
  for (uint64_t i = 0; i < ocap; i++) {
    ent_t* o = &old[i];
    if (!o->h || !live(m, o, now - o->slack)) continue;
    ent_t* e = smap_find(m, oar + o->off, o->len, o->h);
    *e = *o; e->off = m->arena_used;
    memcpy(m->arena + m->arena_used, oar + o->off, o->len); m->arena_used += o->len;
    m->used++;
  }
  free(old); free(oar);
}

/* Find or create the entry for key k (a dead entry is returned as is: the
 * caller decides liveness). */
static ent_t* smap_upsert(smap_t* m, const char* k, uint32_t n, int64_t now, int64_t div, int* created) {
  uint64_t h = hash_bytes(k, n);
  ent_t* e = smap_find(m, k, n, h);
  const int64_t slack = GC_WINDOWS * div > m->horizon + 2 * div ? GC_WINDOWS * div : m->horizon + 2 * div;
  *created = 0;
  if (e->h) {
    if (e->slack < slack) e->slack = slack;
    return e;
  }
  if ((m->used + 1) * 2 > m->cap) { smap_rebuild(m, now); e = smap_find(m, k, n, h); }
  while (m->arena_used + n > m->arena_cap) { m->arena_cap *= 2; m->arena = (char*)realloc(m->arena, m->arena_cap); }
  e->h = h; e->off = m->arena_used; e->len = n; e->count = 0; e->expire = -1; e->slack = slack;
  memcpy(m->arena + m->arena_used, k, n); m->arena_used += n; m->used++;
  *created = 1;
  return e;
}

static ent_t* smap_get(smap_t* m, const char* k, uint32_t n) {
  ent_t* e = smap_find(m, k, n, hash_bytes(k, n));
  return e->h ? e : NULL;
}

/* ------------------------------------------------------------------ utils */
static int64_t unit_to_divider(uint8_t unit) { /* utilities.go:17-30 */
  switch (unit) {
    case RL_UNIT_SECOND: return 1;
    case RL_UNIT_MINUTE: return 60;
    case RL_UNIT_HOUR: return 3600;
    case RL_UNIT_DAY: return 86400;
  }
  return 0; /* reference panics("should not get here"); rejected as RL_E_INVALID */
}

static uint32_t go_f64_to_u32(double x) { /* Go uint32(float64) on amd64 */
  int64_t v;
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) v = INT64_MIN;
  else v = (int64_t)x;
  return (uint32_t)v;
}

uint32_t rlo_near_threshold(uint32_t limit, float ratio) { /* base_limiter.go:94 */
  volatile float prod = (float)limit * ratio; /* one IEEE fp32 multiply */
  return go_f64_to_u32(floor((double)prod));
}

static uint32_t fmt_i64(char* out, int64_t v) { /* strconv.FormatInt(v, 10) */
  char tmp[24]; uint32_t n = 0; uint64_t u;
  int neg = v < 0;
  u = neg ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  do { tmp[n++] = (char)('0' + u % 10); u /= 10; } while (u);
  uint32_t k = 0;
  if (neg) out[k++] = '-';
  while (n) out[k++] = tmp[--n];
  return k;
}

/* ------------------------------------------------------------------ the cache */
typedef struct rlo_ctx {
  float ratio;
  int lc_enabled, per_second;
  smap_t redis, redis_ps, lc;
  char* keybuf; uint32_t keycap;
} rlo_ctx;

rlo_ctx* rlo_create(float near_limit_ratio, int local_cache, int per_second) {
  rlo_ctx* c = (rlo_ctx*)calloc(1, sizeof(rlo_ctx));
  c->ratio = near_limit_ratio; c->lc_enabled = local_cache; c->per_second = per_second;
  smap_init(&c->redis, 1 << 16, 0);
  smap_init(&c->redis_ps, 1 << 12, 0);
  smap_init(&c->lc, 1 << 12, 1);
  c->keycap = 1 << 16; c->keybuf = (char*)malloc(c->keycap);
  return c;
}

/* Keep entries for requests lagging up to `horizon` seconds + 2 windows (the
 * GPU ctx's expiration_jitter_max_seconds). */
void rlo_set_horizon(rlo_ctx* c, int64_t horizon) {
  c->redis.horizon = c->redis_ps.horizon = c->lc.horizon = horizon;
}

void rlo_destroy(rlo_ctx* c) {
  if (!c) return;
  smap_free(&c->redis); smap_free(&c->redis_ps); smap_free(&c->lc);
  free(c->keybuf); free(c);
}

/* GenerateCacheKey for packed descriptor i, into a scratch buffer. */
static const char* build_key(rlo_ctx* c, const rl_batch* b, uint32_t i, int64_t now, uint32_t* len) {
  uint32_t s0 = b->stem_off[i], sl = b->stem_off[i + 1] - s0;
  if (sl + 24 > c->keycap) { while (sl + 24 > c->keycap) c->keycap *= 2; c->keybuf = (char*)realloc(c->keybuf, c->keycap); }
  memcpy(c->keybuf, b->stem_bytes + s0, sl);
  int64_t d = unit_to_divider(b->unit[i]);
  *len = sl + fmt_i64(c->keybuf + sl, (now / d) * d);
  return c->keybuf;
}

typedef struct { uint32_t over, near, lcs, within, shadow; uint8_t code; uint32_t rem; int set_lc; } dec_t;

/* GetResponseDescriptorStatus for a non-empty key, base_limiter.go:82-134. */
static dec_t decide(uint32_t before, uint32_t after, int lc_hit, uint32_t h, uint32_t thr,
                    float ratio, int shadow, int lc_enabled) {
  dec_t r; memset(&r, 0, sizeof r);
  int over = 0;
  if (lc_hit) {
    over = 1; r.over += h; r.lcs += h; r.code = RL_CODE_OVER_LIMIT; r.rem = 0;
  } else {
    uint32_t near = rlo_near_threshold(thr, ratio);
    if (after > thr) {
      over = 1; r.code = RL_CODE_OVER_LIMIT; r.rem = 0;
      if (before >= thr) r.over += h;
      else { r.over += after - thr; r.near += thr - (near > before ? near : before); }
      r.set_lc = lc_enabled;
    } else {
      r.code = RL_CODE_OK; r.rem = thr - after;
      if (after > near) r.near += (before >= near) ? h : after - near;
      r.within += h;
    }
  }
  if (over && shadow) { r.code = RL_CODE_OK; r.shadow += h; }
  return r;
}

/* DoLimit over the descriptors idx[0..m) of batch b (all of b when idx is
 * NULL), in that order; results at their batch positions, stats deltas added
 * into `stats` (n_rules x RL_NUM_STATS). Requests are the runs of equal req_idx. */
static int do_limit_idx(rlo_ctx* c, const rl_batch* b, const uint32_t* idx, uint32_t m, rl_result* o,
                        uint64_t* stats) {
#define AT(j) (idx ? idx[j] : (j))
  uint32_t i = 0;
  uint32_t* after = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
  uint8_t* lcf = (uint8_t*)malloc(m ? m : 1);
  while (i < m) {
    uint32_t q = b->req_idx[AT(i)], a = i, e = i;
    while (e < m && b->req_idx[AT(e)] == q) e++;
    int64_t now = b->now[q];
    /* GenerateCacheKeys: TotalHits (base_limiter.go:55-57) */
    for (uint32_t j = a; j < e; j++) {
      uint32_t k = AT(j);
      if (!unit_to_divider(b->unit[k]) || b->rule_id[k] >= b->n_rules) { free(after); free(lcf); return RL_E_INVALID; }
      uint32_t h = b->hits[k] > 1 ? b->hits[k] : 1;
      stats[(uint64_t)b->rule_id[k] * RL_NUM_STATS + RL_STAT_TOTAL_HITS] += h;
    }
    /* local cache check for every key first (fixed_cache_impl.go:51-67) */
    for (uint32_t j = a; j < e; j++) {
      uint32_t k = AT(j);
      lcf[j] = 0; after[j] = 0;
      if (!c->lc_enabled) continue;
      uint32_t kl; const char* key = build_key(c, b, k, now, &kl);
      ent_t* le = smap_get(&c->lc, key, kl);
      if (le && now < le->expire) lcf[j] = (b->flags[k] & RL_FLAG_SHADOW) ? 2 : 1; /* 2: skip, not marked */
    }
    /* PipeDo: main pipeline in order, then the per-second pipeline (:90-95) */
    for (int pass = 0; pass < 2; pass++) {
      for (uint32_t j = a; j < e; j++) {
        uint32_t k = AT(j);
        if (lcf[j]) continue;
        int ps = c->per_second && b->unit[k] == RL_UNIT_SECOND;
        if (ps != pass) continue;
        smap_t* mp = ps ? &c->redis_ps : &c->redis;
        uint32_t kl; const char* key = build_key(c, b, k, now, &kl);
        uint32_t h = b->hits[k] > 1 ? b->hits[k] : 1;
        int created; ent_t* re = smap_upsert(mp, key, kl, now, unit_to_divider(b->unit[k]), &created);
        if (!live(mp, re, now)) { re->count = 0; re->expire = -1; }
        re->count += h;                                   /* INCRBY */
        re->expire = now + unit_to_divider(b->unit[k]);   /* EXPIRE (jitter draw 0) */
        after[j] = re->count;
      }
    }
    /* statuses (fixed_cache_impl.go:100-110) */
    for (uint32_t j = a; j < e; j++) {
      uint32_t k = AT(j);
      uint32_t h = b->hits[k] > 1 ? b->hits[k] : 1;
      int64_t d = unit_to_divider(b->unit[k]);
      dec_t r = decide(after[j] - h, after[j], lcf[j] == 1, h, b->limit[k], c->ratio,
                       (b->flags[k] & RL_FLAG_SHADOW) != 0, c->lc_enabled);
      if (r.set_lc) { /* localCache.Set(key, ttl = divider) */
        uint32_t kl; const char* key = build_key(c, b, k, now, &kl);
        int created; ent_t* le = smap_upsert(&c->lc, key, kl, now, d, &created);
        le->expire = now + d;
      }
      o->code[k] = r.code; o->limit_remaining[k] = r.rem;
      o->reset_s[k] = (uint32_t)(d - now % d); /* CalculateReset */
      uint64_t* s = stats + (uint64_t)b->rule_id[k] * RL_NUM_STATS;
      s[RL_STAT_OVER_LIMIT] += r.over; s[RL_STAT_NEAR_LIMIT] += r.near;
      s[RL_STAT_OVER_LIMIT_WITH_LOCAL_CACHE] += r.lcs; s[RL_STAT_WITHIN_LIMIT] += r.within;
      s[RL_STAT_SHADOW_MODE] += r.shadow;
    }
    i = e;
  }
  free(after); free(lcf);
  return RL_OK;
#undef AT
}

int rlo_do_limit(rlo_ctx* c, const rl_batch* b, rl_result* o) {
  if (b->n_rules) memset(o->stats, 0, sizeof(uint64_t) * RL_NUM_STATS * b->n_rules);
  return do_limit_idx(c, b, NULL, b->n, o, o->stats);
}

/* ------------------------------------------------- key-sharded, multi-threaded
 * The CPU baseline of SURVEY.md §8d (i): T independent stores ("Redis" + local
 * cache), descriptors routed by a hash of their stem (so a key, and both units
 * of a stem, always land in one shard), each shard replaying its descriptors in
 * arrival order on its own thread. Keys never interact, so the results equal
 * the sequential replay's bit for bit (tests/test_c_oracle.py checks that). */
typedef struct rlo_mt rlo_mt;
typedef struct {
  rlo_mt* m;
  int t;
  uint64_t* stats;  /* this shard's per-rule deltas of the current batch */
  int rc;
} mt_worker_t;

/* A pool of T threads, created once: per batch, three phases between
 * barriers — (0) each thread hashes its slice of the descriptors to shards and
 * counts them per shard, (1) each scatters its slice into the shards' index
 * lists at offsets the main thread took from the counts (slices in order, so
 * every list is in arrival order), (2) each replays its shard's list. Every
 * phase is O(n / T) per thread: the rate scales with the cores. */
struct rlo_mt {
  int T;
  rlo_ctx** sh;
  pthread_t* th;
  mt_worker_t* w;
  pthread_barrier_t go, done;
  int phase, quit;
  const rl_batch* b;
  rl_result* o;
  uint16_t* shard;   /* [n] shard of each descriptor */
  uint32_t* cnt;     /* [T x T] cnt[t * T + s]: descriptors of slice t in shard s; then their offsets */
  uint32_t* idx;     /* [n] the shards' index lists, concatenated */
  uint32_t* base;    /* [T + 1] shard s's list starts at idx + base[s] */
  uint32_t cap;      /* n the arrays are sized for */
};

static void mt_phase(rlo_mt* m, int t) {
  const rl_batch* b = m->b;
  const int T = m->T;
  const uint32_t a = (uint32_t)((uint64_t)b->n * t / T), e = (uint32_t)((uint64_t)b->n * (t + 1) / T);
  if (m->phase == 0) {
    uint32_t* c = m->cnt + (size_t)t * T;
    memset(c, 0, sizeof(uint32_t) * T);
    for (uint32_t i = a; i < e; i++) {
      const uint32_t s0 = b->stem_off[i];
      const uint16_t s = (uint16_t)(hash_bytes((const char*)b->stem_bytes + s0, b->stem_off[i + 1] - s0) % (uint64_t)T);
      m->shard[i] = s;
      c[s]++;
    }
  } else if (m->phase == 1) {
    uint32_t* c = m->cnt + (size_t)t * T;  /* (now this slice's next position per shard) */
    for (uint32_t i = a; i < e; i++) m->idx[c[m->shard[i]]++] = i;
  } else {
    mt_worker_t* w = &m->w[t];
    memset(w->stats, 0, sizeof(uint64_t) * RL_NUM_STATS * (b->n_rules ? b->n_rules : 1));
    w->rc = do_limit_idx(m->sh[t], b, m->idx + m->base[t], m->base[t + 1] - m->base[t], m->o, w->stats);
  }
}

static void* mt_main(void* arg) {
  mt_worker_t* w = (mt_worker_t*)arg;
  rlo_mt* m = w->m;
  for (;;) {
    pthread_barrier_wait(&m->go);
    if (m->quit) return NULL;
    mt_phase(m, w->t);
    pthread_barrier_wait(&m->done);
  }
}

rlo_mt* rlo_mt_create(float near_limit_ratio, int local_cache, int per_second, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 65535) threads = 65535;
  rlo_mt* m = (rlo_mt*)calloc(1, sizeof(rlo_mt));
  m->T = threads;
  m->sh = (rlo_ctx**)calloc(threads, sizeof(rlo_ctx*));
  for (int t = 0; t < threads; t++) m->sh[t] = rlo_create(near_limit_ratio, local_cache, per_second);
  m->cnt = (uint32_t*)calloc((size_t)threads * threads, sizeof(uint32_t));
  m->base = (uint32_t*)calloc((size_t)threads + 1, sizeof(uint32_t));
  m->w = (mt_worker_t*)calloc(threads, sizeof(mt_worker_t));
  m->th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  pthread_barrier_init(&m->go, NULL, (unsigned)threads + 1);
  pthread_barrier_init(&m->done, NULL, (unsigned)threads + 1);
  for (int t = 0; t < threads; t++) {
    m->w[t].m = m;
    m->w[t].t = t;
    pthread_create(&m->th[t], NULL, mt_main, &m->w[t]);
  }
  return m;
}

void rlo_mt_destroy(rlo_mt* m) {
  if (!m) return;
  m->quit = 1;
  pthread_barrier_wait(&m->go);
  for (int t = 0; t < m->T; t++) pthread_join(m->th[t], NULL);
  pthread_barrier_destroy(&m->go);
  pthread_barrier_destroy(&m->done);
  for (int t = 0; t < m->T; t++) {
    rlo_destroy(m->sh[t]);
    free(m->w[t].stats);
  }
  free(m->sh); free(m->th); free(m->w); free(m->cnt); free(m->base);
  free(m->shard); free(m->idx);
  free(m);
}

static void mt_run(rlo_mt* m, int phase) {
  m->phase = phase;
  pthread_barrier_wait(&m->go);
  pthread_barrier_wait(&m->done);
}

int rlo_mt_do_limit(rlo_mt* m, const rl_batch* b, rl_result* o) {
  const int T = m->T;
  if (b->n > m->cap || !m->shard) {
    free(m->shard); free(m->idx);
    m->cap = b->n > m->cap ? b->n : (m->cap ? m->cap : 1);
    m->shard = (uint16_t*)malloc(sizeof(uint16_t) * m->cap);
    m->idx = (uint32_t*)malloc(sizeof(uint32_t) * m->cap);
  }
  for (int t = 0; t < T; t++) {
    free(m->w[t].stats);
    m->w[t].stats = (uint64_t*)calloc((size_t)(b->n_rules ? b->n_rules : 1) * RL_NUM_STATS, sizeof(uint64_t));
  }
  m->b = b;
  m->o = o;
  mt_run(m, 0);
  /* shard s's list: slices 0..T-1 in order */
  uint32_t pos = 0;
  for (int s = 0; s < T; s++) {
    m->base[s] = pos;
    for (int t = 0; t < T; t++) {
      const uint32_t c = m->cnt[(size_t)t * T + s];
      m->cnt[(size_t)t * T + s] = pos;
      pos += c;
    }
  }
  m->base[T] = pos;
  mt_run(m, 1);
  mt_run(m, 2);
  int rc = RL_OK;
  if (b->n_rules) memset(o->stats, 0, sizeof(uint64_t) * RL_NUM_STATS * b->n_rules);
  for (int t = 0; t < T; t++) {
    if (m->w[t].rc) rc = m->w[t].rc;
    for (uint64_t i = 0; i < (uint64_t)b->n_rules * RL_NUM_STATS; i++) o->stats[i] += m->w[t].stats[i];
  }
  return rc;
}

int rlo_restore(rlo_ctx* c, const rl_restore_batch* r) {
  for (uint32_t i = 0; i < r->n; i++) {
    int64_t d = unit_to_divider(r->unit[i]);
    if (!d) return RL_E_INVALID;
    uint32_t s0 = r->stem_off[i], sl = r->stem_off[i + 1] - s0;
    char buf[4096];
    if (sl + 24 > sizeof buf) return RL_E_INVALID;
    memcpy(buf, r->stem_bytes + s0, sl);
    uint32_t kl = sl + fmt_i64(buf + sl, (r->now[i] / d) * d);
    smap_t* m = (c->per_second && r->unit[i] == RL_UNIT_SECOND) ? &c->redis_ps : &c->redis;
    int created; ent_t* e = smap_upsert(m, buf, kl, r->now[i], d, &created);
    e->count = r->count[i]; e->expire = r->now[i] + d;
    if (r->lc && r->lc[i]) { ent_t* le = smap_upsert(&c->lc, buf, kl, r->now[i], d, &created); le->expire = r->now[i] + d; }
  }
  return RL_OK;
}

/* Materialised keys, the oracle twin of rl_debug_keys. */
int rlo_keys(rlo_ctx* c, const rl_batch* b, uint8_t* out, uint32_t* out_off, uint32_t cap) {
  uint32_t pos = 0; out_off[0] = 0;
  for (uint32_t i = 0; i < b->n; i++) {
    uint32_t kl; const char* key = build_key(c, b, i, b->now[b->req_idx[i]], &kl);
    if (pos + kl > cap) return RL_E_CAPACITY;
    memcpy(out + pos, key, kl); pos += kl; out_off[i + 1] = pos;
  }
  return RL_OK;
}

uint64_t rlo_live_keys(rlo_ctx* c) { return c->redis.used + c->redis_ps.used; }
