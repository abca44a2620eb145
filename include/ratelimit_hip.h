/*
 * ratelimit_hip.h — C ABI of libratelimit_hip.so, the MI355X fixed-window
 * rate-limit backend.
 *
 * Drop-in boundary: this library replaces the box below
 *   limiter.RateLimitCache.DoLimit           (reference src/limiter/cache.go:11-29)
 * as implemented by
 *   redis.fixedRateLimitCacheImpl.DoLimit    (src/redis/fixed_cache_impl.go:33-113)
 *   + limiter.BaseRateLimiter                (src/limiter/base_limiter.go:45-197)
 *   + limiter.CacheKeyGenerator              (src/limiter/cache_key.go:48-80)
 *   + redis-server INCRBY/EXPIRE and the freecache local over-limit cache.
 * A Go cgo adapter packs many in-flight DoLimit calls into
 * one rl_batch and calls rl_do_limit from a single batcher goroutine.
 *
 * Plain C types only: no torch, no HIP types in any signature.
 * Threading: one rl_ctx is driven by one host thread at a time.
 * Errors: every int-returning call returns RL_OK (0) or an rl_status code and
 * records a message readable with rl_last_error(); the Go adapter turns a
 * non-zero status into panic(redis.RedisError("gpu: "+msg)), exactly the
 * reference's backend-failure convention (src/redis/driver_impl.go:60-64).
 */
#ifndef RATELIMIT_HIP_H
#define RATELIMIT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RL_ABI_VERSION 6u

/* Status codes. */
enum rl_status {
  RL_OK = 0,
  RL_E_INVALID = 1,    /* malformed batch: unit out of 1..4, offsets, sizes */
  RL_E_TABLE_FULL = 2, /* open-addressing table has no free slot on the probe path */
  RL_E_ARENA_FULL = 3, /* long-stem overflow arena exhausted */
  RL_E_HIP = 4,        /* HIP runtime error */
  RL_E_CAPACITY = 5,   /* batch larger than rl_config.max_* */
  RL_E_TIME = 6,       /* now outside [0, 2^32 - 2*86400], before the last sweep, or
                          moved back more than 8 windows on one key. Note: the reference's
                          clock is int64 (utils.TimeSource); this backend's is 32-bit */
  RL_E_COMM = 7,       /* multi-GPU routing (RCCL) error */
  RL_E_INTERNAL = 8
};

/* pb.RateLimitResponse_RateLimit_Unit (go-control-plane v0.9.7 rls.proto). */
enum rl_unit { RL_UNIT_SECOND = 1, RL_UNIT_MINUTE = 2, RL_UNIT_HOUR = 3, RL_UNIT_DAY = 4 };
/* pb.RateLimitResponse_Code. */
enum rl_code { RL_CODE_OK = 1, RL_CODE_OVER_LIMIT = 2 };
/* rl_batch.flags bits. */
#define RL_FLAG_SHADOW 0x1u /* config.RateLimit.ShadowMode (src/config/config.go:24) */

/* Per-rule stats counters, in stats.RateLimitStats order (src/stats/manager.go:47-55). */
enum rl_stat {
  RL_STAT_TOTAL_HITS = 0,
  RL_STAT_OVER_LIMIT = 1,
  RL_STAT_NEAR_LIMIT = 2,
  RL_STAT_OVER_LIMIT_WITH_LOCAL_CACHE = 3,
  RL_STAT_WITHIN_LIMIT = 4,
  RL_STAT_SHADOW_MODE = 5,
  RL_NUM_STATS = 6
};

/* Backend configuration: the knobs NewFixedRateLimitCacheImpl receives
 * (src/redis/fixed_cache_impl.go:118-125, src/settings/settings.go:45-50)
 * plus capacity sizing for HBM. */
typedef struct rl_config {
  uint64_t table_slots;      /* 64-B slots in the HBM table (power of 2; 0 = default 2^24) */
  uint64_t arena_bytes;      /* overflow arena for stems longer than 36 B (0 = default 64 MiB) */
  uint32_t max_batch;        /* max descriptors per rl_do_limit call (0 = default 1<<20) */
  uint32_t max_requests;     /* max requests per call (0 = max_batch) */
  uint32_t max_rules;        /* max distinct rule ids per call (0 = default 65536) */
  uint32_t max_stem_bytes;   /* max total stem bytes per call (0 = 128 * max_batch) */
  float near_limit_ratio;    /* NEAR_LIMIT_RATIO (float32, settings.go:48) */
  int32_t local_cache_enabled;  /* LOCAL_CACHE_SIZE_IN_BYTES != 0 (runner.go:95-98) */
  int32_t per_second_split;     /* REDIS_PERSECOND: SECOND-unit keys in a separate store */
  int32_t device;               /* HIP device ordinal */
  int64_t expiration_jitter_max_seconds; /* EXPIRATION_JITTER_MAX_SECONDS (>= 0): the backend fixes
                                            the draw at 0 and keeps a key's older
                                            windows for div + this many seconds (the history horizon) */
  uint64_t hash_seed;        /* key of the stem hash (SipHash-1-3); 0 = drawn at random per ctx.
                                Descriptor values are client-controlled: keep it secret. */
  uint32_t n_shards;         /* hash shards of the table held by this ctx (0 = 1); see rl_do_limit */
  uint32_t debug_hash_bits;  /* tests only: keep the top N bits of the hash's high word (0 = all 32),
                                so that many stems share one sort key and one home region;
                                33..63: keep the top N - 32 bits and set the others (sort keys
                                at the top of the range) */
  int32_t shard_device[16];  /* HIP device of shard k < n_shards (shards may share a device);
                                unused when n_shards <= 1 (cfg.device) */
  uint64_t history_entries;  /* 32-B entries of the history log holding the windows below a key's
                                newest (0 = table_slots; rounded to 64 powers of two, at least
                                max_batch / 16 each). Append-only rings: an entry overwritten while
                                a request could still ask for its window makes that request fail
                                with RL_E_TIME (counted in rl_table_info.history_lost), never a
                                wrong count */
  int32_t reserved[6];
} rl_config;

/* One packed batch (struct of arrays). Only descriptors whose limit is
 * non-nil are packed (nil limits -> {OK, nil, 0} host-side,
 * base_limiter.go:78-81); unlimited rules are nil by then (ratelimit.go:140-143).
 * Descriptors appear in arrival order: request-major, descriptor order inside
 * the request; req_idx is non-decreasing. now[] may move backwards (the
 * reference's tests do, on different keys); per (stem, unit) the table keeps
 * the windows below the newest one written while a request could still ask
 * for them (Redis keeps a key div + jitter seconds after its last hit,
 * fixed_cache_impl.go:71-74): a request whose clock is within div +
 * expiration_jitter_max_seconds of the key's newest window, or whose window
 * is at most 8 windows back, is answered exactly; an older one whose window
 * the key may have had gets RL_E_TIME.
 * The stem is the cache key without its window suffix:
 *   prefix ‖ domain ‖ '_' ‖ Σ(key ‖ '_' ‖ value ‖ '_')   (cache_key.go:62-71)
 * The full key is stem ‖ decimal((now/div)*div) (cache_key.go:73-74). */
typedef struct rl_batch {
  uint32_t n;            /* descriptors */
  uint32_t n_requests;   /* requests (length of now[]) */
  uint32_t n_rules;      /* rule ids are < n_rules (length of stats / RL_NUM_STATS) */
  uint32_t reserved;
  const uint8_t* stem_bytes;  /* concatenated stems */
  const uint32_t* stem_off;   /* n+1 offsets into stem_bytes, stem_off[0] == 0 */
  const int64_t* now;         /* [n_requests] UnixNow() of each request (seconds). The reference's
                                 clock is int64; here it must lie in [0, 2^32 - 172800] (the table
                                 stores 32-bit times) and not before the last rl_sweep: else RL_E_TIME */
  const uint32_t* req_idx;    /* [n] request of each descriptor */
  const uint8_t* unit;        /* [n] rl_unit of the descriptor's limit */
  const uint8_t* flags;       /* [n] RL_FLAG_* */
  const uint32_t* limit;      /* [n] RequestsPerUnit */
  const uint32_t* hits;       /* [n] request.HitsAddend (max(1, h) applied by the backend) */
  const uint32_t* rule_id;    /* [n] dense id of limit.Stats.Key */
} rl_batch;

/* Results, same order as the batch. stats holds THIS call's deltas
 * (n_rules x RL_NUM_STATS, row-major, overwritten); the adapter adds them to the
 * gostats counters. CurrentLimit is re-attached host-side (= limits[i].Limit). */
typedef struct rl_result {
  uint8_t* code;              /* [n] rl_code */
  uint32_t* limit_remaining;  /* [n] LimitRemaining */
  uint32_t* reset_s;          /* [n] DurationUntilReset.Seconds (1..86400). May be NULL on the
                                 host-buffer entry points (rl_do_limit, rl_do_limit_host_async,
                                 _compact_async, _prefixed_async): not copied back, 4 B per decision less over PCIe;
                                 the caller computes it as utils.CalculateReset does
                                 (utilities.go:32-36: div - now % div, now the request's clock) */
  uint64_t* stats;            /* [n_rules * RL_NUM_STATS] */
  uint8_t* status;            /* [n] or NULL. Non-NULL: per-descriptor failure isolation. A
                                 descriptor that cannot be answered (bad unit / rule id / stem length:
                                 RL_E_INVALID; clock: RL_E_TIME; no slot: RL_E_TABLE_FULL /
                                 RL_E_ARENA_FULL) gets that rl_status here, code 0 and no stats; the
                                 rest of the batch is answered and the call returns RL_OK. The adapter
                                 fails only the RPCs holding a failed descriptor, as the reference's
                                 per-call checkError does (fixed_cache_impl.go:90-95,
                                 ratelimit.go:252-256). NULL: any such failure fails the whole call
                                 (and the batch leaves the table untouched). A malformed batch
                                 layout (offsets, request order) always fails the call. */
} rl_result;

/* Table restore / seed records: set the fixed-window counter of key
 * stem ‖ decimal(ws(now[i], unit[i])) to count[i] with EXPIRE div (as if the last
 * INCRBY happened at now[i]); lc[i] != 0 also inserts the key into the local
 * over-limit cache with TTL div. Host memory. */
typedef struct rl_restore_batch {
  uint32_t n;
  uint32_t reserved;
  const uint8_t* stem_bytes;
  const uint32_t* stem_off;   /* n+1 */
  const uint8_t* unit;        /* [n] */
  const int64_t* now;         /* [n] */
  const uint32_t* count;      /* [n] */
  const uint8_t* lc;          /* [n] */
} rl_restore_batch;

typedef struct rl_table_info {
  uint64_t table_slots;
  uint64_t live_slots;        /* occupied (non-empty, non-tombstone) slots */
  uint64_t tombstones;
  uint64_t arena_bytes_used;
  uint64_t exact_stems;       /* slots flagged multi-unit (exact slow path) */
  uint64_t batches;
  uint64_t decisions;
  uint64_t history_entries;   /* entries of the history log (rl_config.history_entries, rounded) */
  uint64_t history_appended;  /* records appended to the log since rl_create / rl_snapshot_load */
  uint64_t history_lost;      /* lookups that found an entry the log had overwritten: answered
                                 RL_E_TIME (size history_entries up) */
  uint64_t history_slots;     /* live slots with a history chain */
  uint64_t history_refused;   /* records the log refused: their partition had taken
                                 history_entries / 64 appends in one batch already (a batch's
                                 appends never wrap a partition onto its own entries); a later
                                 lookup of such a window is RL_E_TIME (size history_entries up) */
} rl_table_info;

typedef struct rl_ctx rl_ctx;

uint32_t rl_abi_version(void);

/* Create / destroy a backend on cfg->device. NULL on failure (message in err). */
rl_ctx* rl_create(const rl_config* cfg, char* err, size_t errlen);
void rl_destroy(rl_ctx* ctx);
const char* rl_last_error(const rl_ctx* ctx);

/* DoLimit for a whole batch. Host buffers (pinned via rl_alloc_host is fastest).
 * Synchronous: returns after results are in *out.
 * Multi-GPU (rl_config.n_shards > 1): the table is hash-sharded over
 * shard_device[0..n_shards) inside this one ctx (the reference's single service
 * process scaled out over a Redis cluster, src/redis/driver_impl.go:108-126).
 * Each shard has a worker thread and a router; the shards' routers form an
 * in-process world (the loopback transport: device copies, over xGMI between
 * distinct devices). A host batch is cut into one request-aligned slice per
 * shard; each shard copies its slice over its own device's link, partitions
 * it by owner, exchanges records with the other shards, runs the pipeline on
 * the keys it owns, and returns the answers to the slice's source, which
 * writes them to *out in arrival order; the stats of the slices are summed.
 * Same call, same answers. Owners keep stats per source slice, so every shard
 * is created with n_shards x max_rules rows (a batch may carry max_rules). */
int rl_do_limit(rl_ctx* ctx, const rl_batch* in, rl_result* out);

/* Same, with every pointer in *in / *out in device memory of ctx's GPU
 * (shard_device[0] when n_shards > 1), pipelined on the ctx's own streams.
 * With `stream` (a hipStream_t) the batch starts after the work already on it
 * (the inputs' producer); with NULL the inputs must be complete at the call.
 * *out is read after rl_synchronize (the caller's stream is never made to wait
 * for a batch, which would chain the next batch's inputs behind it and
 * serialise the pipeline). The inputs are read until the batch is complete
 * (rl_synchronize, or rl_batch_progress): keep them unchanged until then.
 * Returns once the work is enqueued; errors detected
 * on the GPU surface at rl_synchronize. On a multi-shard ctx shard 0 takes the
 * whole device batch as its slice (the other shards' slices are empty) and
 * routes it to the owners as above; the caller's thread waits only until every
 * shard's worker has enqueued its part, never for the GPU.
 * stem_bytes must be 4-byte aligned (any hipMalloc / torch allocation is). */
int rl_do_limit_async(rl_ctx* ctx, const rl_batch* in, rl_result* out, void* stream);

/* Host buffers in and out, like rl_do_limit, without waiting: the batch's
 * inputs cross PCIe into one of the ctx's device staging slots while earlier
 * batches compute, its outputs cross back when it is done; *out is read after
 * rl_synchronize, and the host buffers of a batch stay untouched until then.
 * Pinned buffers (rl_alloc_host) make the copies asynchronous. The fed path of
 * a batcher whose requests arrive in host memory. On a multi-shard ctx each
 * shard's worker copies its request-aligned slice over its own link and routes
 * it (rl_do_limit); out->stats is written at rl_synchronize (or once the
 * ring of batches in flight comes round to this batch again).
 * On a multi-shard ctx rl_synchronize, rl_sweep, rl_restore, the info getters
 * and the snapshot calls first complete every shard's pending batches. */
int rl_do_limit_host_async(rl_ctx* ctx, const rl_batch* in, rl_result* out);
int rl_synchronize(rl_ctx* ctx);

/* Pipelined batchers (single-shard ctx): the number of batches submitted
 * through rl_do_limit* so far and how many of them, in submission order, have
 * their outputs complete (host-fed batches: copied back). Never waits, so a
 * batcher can hand out the answers of finished batches while later ones run;
 * device-side errors are still reported by rl_synchronize. */
int rl_batch_progress(rl_ctx* ctx, uint64_t* submitted, uint64_t* completed);

/* ---- Compact host batch: the fed path's PCIe format ---------------------
 * The same batch as rl_batch, laid out for the link: ONE contiguous host
 * buffer (one copy per batch), per request its clock, HitsAddend and first
 * descriptor (the reference's per-request fields, RateLimitRequest.HitsAddend
 * and the UnixNow() of the DoLimit call, fixed_cache_impl.go:33-51), per
 * descriptor its stem and a 16-bit index into a table of the batch's distinct
 * limits (a config rule, or an interned per-request override): 46 B per
 * descriptor at BASELINE C1 (34-B stems, two descriptors per request) against
 * rl_batch's 60. Answers, errors and statuses are those of the equivalent
 * rl_batch (a limit index >= n_limits is an RL_E_INVALID descriptor). */
typedef struct rl_limit {
  uint32_t requests_per_unit;  /* RateLimit.Limit.RequestsPerUnit */
  uint32_t rule_id;            /* stats row of the limit (< n_rules) */
  uint8_t unit;                /* rl_unit */
  uint8_t flags;               /* RL_FLAG_* */
  uint16_t reserved;
} rl_limit;

/* Sections of buf, as byte offsets (each a multiple of 4, in any order). */
typedef struct rl_batch_compact {
  uint32_t n;            /* descriptors */
  uint32_t n_requests;
  uint32_t n_rules;
  uint32_t n_limits;     /* entries of the limit table (<= 65536) */
  const uint8_t* buf;    /* pinned host memory (rl_alloc_host): copied once, asynchronously */
  uint64_t buf_bytes;
  uint64_t stem_bytes;   /* concatenated stems */
  uint64_t stem_off;     /* uint32[n + 1], stem_off[0] == 0 */
  uint64_t limit_idx;    /* uint16[n] */
  uint64_t req_first;    /* uint32[n_requests + 1]: request q holds descriptors
                            [req_first[q], req_first[q+1]); req_first[0] == 0,
                            non-decreasing, req_first[n_requests] == n */
  uint64_t now;          /* uint32[n_requests] UnixNow() (< 2^32 - 172800, as rl_batch.now) */
  uint64_t hits;         /* uint32[n_requests] HitsAddend */
  uint64_t limits;       /* rl_limit[n_limits] */
} rl_batch_compact;

/* rl_do_limit_host_async on a compact batch: on a single-shard ctx buf
 * crosses PCIe in one copy into a device staging slot while earlier batches
 * compute, is unpacked on the GPU, and the batch is pipelined like any other.
 * On a multi-shard ctx it is cut into one request-aligned slice per shard;
 * each shard copies its slice's parts of buf over its own device's link,
 * unpacks them and routes them like an rl_batch host slice. *out is read
 * after rl_synchronize; buf stays untouched until then. Not on a ctx that
 * joined a communicator (rl_do_limit_routed_async takes device batches). */
int rl_do_limit_compact_async(rl_ctx* ctx, const rl_batch_compact* in, rl_result* out);

/* ---- Prefix-shared batch: the densest PCIe format ----------------------
 * Every descriptor of one RateLimitRequest starts with the same
 * prefix ‖ domain ‖ '_' and, in practice, with its request's leading entries
 * (cache_key.go:62-71; nested descriptors repeat their parents'). This layout
 * stores those shared bytes once per request and each descriptor's remaining
 * suffix: descriptor d of request q has the stem prefix[q] ‖ suffix[d]. Per
 * request: descriptor count and prefix length (one u32), UnixNow(), HitsAddend;
 * per descriptor: one u32 (limit index, suffix length). 31.5 B per decision at
 * BASELINE C1 (25-B shared prefix, two 9-B suffixes) against rl_batch_compact's
 * 46 and rl_batch's 60. Requests form tiles of RL_PREFIXED_TILE; the index
 * holds each tile's starting offsets, which the batcher has at hand while it
 * appends, so the GPU unpacks every tile independently (no scan pass) and a
 * multi-shard ctx cuts the batch at tile boundaries without reading it.
 * Answers, errors and statuses are those of the equivalent rl_batch (a limit
 * index >= n_limits, or a stem of 0 or more than 65535 bytes, is an
 * RL_E_INVALID descriptor; an index that does not match the sections fails
 * the batch with RL_E_INVALID at rl_synchronize). */
#define RL_PREFIXED_TILE 256u
typedef struct rl_batch_prefixed {
  uint32_t n;            /* descriptors */
  uint32_t n_requests;
  uint32_t n_rules;
  uint32_t n_limits;     /* entries of the limit table (<= 65536) */
  const uint8_t* buf;    /* pinned host memory (rl_alloc_host): copied once, asynchronously */
  uint64_t buf_bytes;
  /* sections of buf, as byte offsets (each a multiple of 4, in any order) */
  uint64_t req;          /* uint32[n_requests]: descriptors of the request (bits 0-15) | bytes of
                            its shared prefix (bits 16-23, at most 255) << 16; bits 24-31 zero.
                            A request's descriptors follow those of the request before it */
  uint64_t now;          /* uint32[n_requests] UnixNow() (< 2^32 - 172800, as rl_batch.now) */
  uint64_t hits;         /* uint32[n_requests] HitsAddend */
  uint64_t desc;         /* uint32[n]: limit index (bits 0-15) | suffix bytes (bits 16-31) << 16 */
  uint64_t prefix_bytes; /* the requests' shared prefixes, concatenated in request order */
  uint64_t suffix_bytes; /* the descriptors' suffixes, concatenated in descriptor order */
  uint64_t limits;       /* rl_limit[n_limits] */
  uint64_t index;        /* uint32[4 x (tiles + 1)], tiles = ceil(n_requests / RL_PREFIXED_TILE):
                            entry t = {first descriptor, first prefix byte, first suffix byte,
                            first byte of the unpacked stems} of requests [t x TILE, (t+1) x TILE);
                            entry 0 is zero, entry `tiles` the totals {n, prefix bytes, suffix
                            bytes, stem bytes (<= max_stem_bytes)} */
} rl_batch_prefixed;

/* rl_do_limit_compact_async's contract for a prefix-shared batch: buf crosses
 * PCIe in one copy (a multi-shard ctx: each shard copies the parts of its
 * tile-aligned slice over its own device's link), is unpacked on the GPU and
 * pipelined like any batch. *out is read after rl_synchronize; buf stays
 * untouched until then. Not on a ctx that joined a communicator. */
int rl_do_limit_prefixed_async(rl_ctx* ctx, const rl_batch_prefixed* in, rl_result* out);

/* Epoch sweep (replaces Redis EXPIRE): tombstones every slot whose counter
 * and local-cache entries have all expired at `now`; `now` becomes a floor
 * (later requests with an earlier time fail with RL_E_TIME). */
int rl_sweep(rl_ctx* ctx, int64_t now, uint64_t* n_evicted);

/* Seed / restore counters (host buffers). */
int rl_restore(rl_ctx* ctx, const rl_restore_batch* in);

int rl_table_info_get(rl_ctx* ctx, rl_table_info* info);  /* summed over shards */
int rl_table_info_shard(rl_ctx* ctx, uint32_t shard, rl_table_info* info);

/* Pinned host memory for the packed buffers (hipHostMalloc). */
void* rl_alloc_host(size_t bytes);
void rl_free_host(void* p);

/* Diagnostics used by the parity tests (host buffers):
 * rl_debug_keys materialises each descriptor's full Redis key
 * (stem ‖ decimal window start) on the GPU into out_bytes/out_off (n+1). */
int rl_debug_keys(rl_ctx* ctx, const rl_batch* in, uint8_t* out_bytes, uint32_t* out_off,
                  uint32_t out_cap);
/* rl_debug_decide runs the device GetResponseDescriptorStatus on explicit
 * (before, after, local-cache flag) tuples: base_limiter.go:76-135. */
int rl_debug_decide(rl_ctx* ctx, uint32_t n, const uint32_t* before, const uint32_t* after,
                    const uint8_t* lc_hit, const uint32_t* hits, const uint32_t* limit,
                    const uint8_t* unit, const uint8_t* flags, const int64_t* now,
                    uint8_t* code, uint32_t* remaining, uint32_t* reset_s,
                    uint64_t* stat_deltas /* n * RL_NUM_STATS */, uint8_t* lc_set);
/* rl_debug_log_tear (tests; libraries built with RL_LOG_TEAR, else RL_E_INVALID):
 * replays a concurrent writer of a history-log entry between a lookup's loads.
 * With arm != NULL it arms a one-shot tear: the first entry the next lookup
 * (log_find) reads is overwritten by `entry`, the writer's steps applied by the
 * reading lane itself: sched[i] of them before the reader's i-th load (header,
 * record, header re-read; non-decreasing), the rest after its verdict. With
 * out != NULL (after the batches that should have fired it) it reads the
 * outcome back and disarms. The lookup uses a record only if the writer and
 * reader protocols keep header and record of one write together; the tests
 * check that over every schedule. */
typedef struct rl_log_tear {
  uint32_t armed;      /* in: 1; out: 2 once a lookup fired it */
  uint32_t protocol;   /* 0: the library's writer (header BUSY, record, header: 3 steps);
                          1: round 5's order (header, record: 2 steps) */
  uint32_t sched[3];   /* writer steps done before the reader's header load, record load, re-read */
  uint32_t entry[8];   /* the overwriting entry: slot, tag, prev, t_app, then the record ws, count,
                          expire, lc; 0xFFFFFFFF in slot / tag / prev / t_app = the entry's own */
  uint32_t before[8];  /* out: the entry before the tear */
  uint32_t seen[12];   /* out: the reader's header, record and header re-read */
  int32_t verdict;     /* out: 1 the record was used (its window), 0 the walk moved on, -1 rejected */
  uint32_t reserved;
} rl_log_tear;
int rl_debug_log_tear(rl_ctx* ctx, const rl_log_tear* arm, rl_log_tear* out);

/* ---- Multi-GPU routing across processes (one single-shard rl_ctx per GPU) ---
 * SURVEY.md §8e. For one process per GPU (torch.distributed / RCCL), each rank
 * routes its slice of the node's requests; the collectives are the caller's
 * (ratelimit_amd/sharded.py). Every pointer is device memory of ctx's GPU, work
 * is enqueued on `stream` (a hipStream_t, NULL = ctx's stream) and never waits
 * on the host; errors surface at rl_synchronize. Every rank's ctx must share
 * rl_config.hash_seed (owner = stem hash).
 *
 * rl_route_pack (source side): stable-partitions the batch `in` by owner shard
 * and writes, in owner order, one RL_WIRE_BYTES record per descriptor (its
 * fields, its request's clock as 32 bits, and the keyed 64-bit stem hash, so
 * owners never rehash; no stem offset) to send_rec and its stem bytes to
 * send_stem (capacity: the batch's stem bytes), each owner's stems in its
 * records' order.
 * perm[j] = batch index of record j. counts[2*d], [2*d+1] (device memory) =
 * records / stem bytes for owner d (all zero when the batch is malformed). Request
 * indices must be < 2^24; the global request label is src_rank << 24 | req_idx,
 * so chunks concatenated in source-rank order are in global arrival order.
 *
 * rl_route_do_limit (owner side): DoLimit over the n records received from all
 * sources (concatenated in source-rank order) with their stems (recv_stem,
 * 4-byte aligned, recv_stem_bytes long; src_stem_base = host array of each
 * source's chunk offset in recv_stem: the chunks abut in source order, and
 * each record's stem starts where the previous record's ends), pipelined on the ctx's streams once the
 * work already on `stream` is done; then, on `stream`, ret[j] = the packed
 * result of record j (bits 0-31 remaining, 32-51 reset_s, 52-55 status, 56-61
 * code, 62 local-cache hit). stats: rule_stride == 0: n_rules x RL_NUM_STATS
 * deltas; rule_stride > 0: per source rank, n_shards blocks of rule_stride x
 * RL_NUM_STATS (the deltas of each source's own requests). isolate != 0:
 * per-descriptor statuses (rl_result.status semantics) in ret.
 *
 * rl_route_scatter (source side): results returned in record order (ret, n =
 * the batch size) -> out (device SoA, status optional) in arrival order. */
#define RL_WIRE_BYTES 32u
#define RL_MAX_SHARDS 256u
int rl_route_pack(rl_ctx* ctx, const rl_batch* in, uint32_t n_shards, uint32_t src_rank, void* send_rec,
                  uint8_t* send_stem, uint32_t* perm, uint64_t* counts, void* stream);
int rl_route_do_limit(rl_ctx* ctx, uint32_t n, const void* recv_rec, const uint8_t* recv_stem,
                      uint64_t recv_stem_bytes, const uint64_t* src_stem_base, uint32_t n_shards, uint32_t n_rules,
                      uint32_t rule_stride, uint64_t* ret, uint64_t* stats, int isolate, void* stream);
int rl_route_scatter(rl_ctx* ctx, uint32_t n, const uint32_t* perm, const uint64_t* ret, rl_result* out,
                     void* stream);

/* ---- Multi-rank routing inside the library (RCCL or in-process loopback) ---
 * SURVEY.md §8e with the exchange itself in the library (rl_comm.hip): one
 * rank per table shard, each with one single-shard ctx, every ctx created with
 * the same rl_config.hash_seed.
 *
 * rl_comm_unique_id (one rank) fills RL_COMM_ID_BYTES bytes (an ncclUniqueId)
 * that the caller hands to every rank (e.g. a torch.distributed broadcast):
 * one process per GPU, exchanges over RCCL (xGMI). RCCL is loaded then
 * (dlopen), not at library load.
 * rl_comm_loopback_id fills the id of an in-process world instead: its ranks
 * are threads of THIS process, one ctx each (any devices; several may share
 * one GPU, which RCCL refuses), exchanging by device copies with the same
 * protocol. A rank whose peers never arrive fails with RL_E_COMM after
 * RL_LOOPBACK_TIMEOUT_S seconds (default 120) instead of waiting forever.
 * rl_comm_init (collective: every rank, the same id) joins ctx to the world as
 * `rank`.
 *
 * rl_do_limit_routed_async (collective: every rank calls it the same number of
 * times in the same order; n may be 0) answers this rank's slice of the node
 * batch. Rank r's slice precedes rank r+1's in the global order (the order the
 * sequential INCRBY contract is kept in). Device arrays; the batch starts
 * after the work already on `stream` (NULL: inputs complete at the call). A
 * call enqueues its batch's partition and counts exchange and completes the
 * batch RL_ROUTED_LAG calls back, so the host never waits for work it just
 * issued and that many owner pipelines stay queued on the GPU. The
 * descriptors a rank owns of its own slice are read in place by its owner
 * batch (no copy): a batch's inputs may be reused once RL_ROUTED_INFLIGHT
 * later calls have returned, or after rl_synchronize; its outputs are read
 * after rl_synchronize (collective too on such a ctx: it completes the last
 * batch). Keep `out` valid until then. out->stats = the deltas of
 * THIS rank's requests (summed over ranks: the node's). Ranks may pass
 * different n_rules; every owner keeps stats per source with the largest
 * n_rules of the batch as stride, so it needs max_rules >= world x that. If
 * any rank passes out->status, owners answer per descriptor (isolation) for
 * the whole batch.
 * Errors never leave a peer waiting: a slice this rank rejects (sizes, null
 * outputs) takes part in the exchange with no records and fails this rank's
 * batch at rl_synchronize; an owner that cannot run what it received answers
 * every such record with its rl_status (in out->status, or failing the
 * source's batch at rl_synchronize). Only a HIP / transport runtime failure
 * leaves the ctx's router unusable (RL_E_COMM / RL_E_HIP from every later
 * call). Replaces the Redis cluster client's key-slot routing inside one
 * service process (src/redis/driver_impl.go:108-126).
 * On a routed ctx rl_synchronize, rl_sweep, rl_restore and rl_snapshot_save /
 * _load first complete the pending batches, so they are collective like the
 * batches. rl_sweep there applies one floor on every rank: the least `now`
 * the ranks passed (a rank passing an out-of-range time fails alone and does
 * not vote), so a rank's requests are never refused by an owner whose clock
 * runs ahead of its own. The read-only getters rl_table_info_get and rl_local_cache_info_get
 * are not: they see every batch but the pending ones (the last RL_ROUTED_LAG
 * submitted), and a rank may call them alone (e.g. for its gauges). */
#define RL_COMM_ID_BYTES 128u
#ifndef RL_ROUTED_INFLIGHT       /* (overridable only for A/B builds of the library) */
#define RL_ROUTED_INFLIGHT 6u  /* routed batches in flight (the input-reuse distance above) */
#endif
#ifndef RL_ROUTED_LAG
#define RL_ROUTED_LAG 3u       /* calls between a routed batch's partition and its owner pipeline */
#endif
int rl_comm_unique_id(uint8_t* id);
int rl_comm_loopback_id(uint8_t* id);
int rl_comm_init(rl_ctx* ctx, uint32_t world, uint32_t rank, const uint8_t* id);
int rl_do_limit_routed_async(rl_ctx* ctx, const rl_batch* in, rl_result* out, void* stream);

/* ---- Config match on the GPU (the caller side of DoLimit) ---
 * The service's constructLimitsToCheck (src/service/ratelimit.go:104-143) calls
 * rateLimitConfigImpl.GetLimit (src/config/config_impl.go:243-298) once per
 * descriptor, then DoLimit, then maps unlimited descriptors to
 * {OK, LimitRemaining = MaxUint32} (ratelimit.go:176-183). rl_do_limit_requests
 * does all three on the device for a batch of raw requests: the host only
 * copies domain / entry bytes; the config trie is walked per descriptor on the
 * GPU and the matched descriptors are compacted into the DoLimit pipeline.
 *
 * rl_config_load replaces the loaded config (GetCurrentConfig snapshot,
 * ratelimit.go:105) with a flattened trie: one rl_config_node per domain root
 * and per descriptor config node (rateLimitDescriptor, config_impl.go:45-48),
 * parents before children. A node's key is the domain name for a root, else
 * its finalKey: key, or key ‖ '_' ‖ value (config_impl.go:106-109). Host
 * buffers; (parent, key) pairs must be unique (RL_E_INVALID otherwise).
 * cache_key_prefix is CACHE_KEY_PREFIX (cache_key.go:62, settings.go). */
typedef struct rl_config_node {
  int32_t parent;             /* index of the parent node; -1: a domain root */
  uint32_t key_off;           /* key bytes in rl_config_tree.key_bytes */
  uint32_t key_len;
  uint32_t requests_per_unit; /* RateLimit.Limit.RequestsPerUnit */
  uint32_t rule_id;           /* dense id of the rule's Stats.Key (its full key path, config_impl.go:111,139) */
  uint8_t unit;               /* rl_unit (0 for unlimited) */
  uint8_t has_limit;          /* the node has a rate_limit block (rateLimitDescriptor.limit != nil) */
  uint8_t unlimited;          /* RateLimit.Unlimited */
  uint8_t shadow_mode;        /* RateLimit.ShadowMode */
} rl_config_node;

typedef struct rl_config_tree {
  uint32_t n_nodes;
  uint32_t cache_key_prefix_len;
  const rl_config_node* nodes;
  const uint8_t* key_bytes;
  uint64_t key_bytes_len;
  const uint8_t* cache_key_prefix;
} rl_config_tree;

int rl_config_load(rl_ctx* ctx, const rl_config_tree* tree);

/* Raw requests (RateLimitRequest, arrival order). Descriptor d belongs to
 * request req_idx[d] (non-decreasing); its entries are
 * [entry_first[d], entry_first[d+1]), and its bytes
 * desc_bytes[desc_off[d], desc_off[d+1]) (all offsets non-decreasing) are Σ(key ‖ '_' ‖ value ‖ '_') over its
 * entries (the stem tail of cache_key.go:65-70), with key_len / value_len per
 * entry. Overrides (RateLimitDescriptor.Limit, config_impl.go:255-266):
 * override_flags[d] bit 0 = present, with override_rpu / override_unit and
 * override_rule = dense id of descriptorKey(domain, descriptor) (interned
 * host-side: the one per-override string the caller builds). The three
 * override arrays may be NULL when no descriptor carries one. Host buffers. */
typedef struct rl_request_batch {
  uint32_t n_requests;
  uint32_t n_descriptors;
  uint32_t n_entries;
  uint32_t n_rules;               /* every rule id (config and override) < n_rules */
  const uint8_t* domain_bytes;    /* RateLimitRequest.Domain, concatenated */
  const uint32_t* domain_off;     /* [n_requests + 1] */
  const int64_t* now;             /* [n_requests] UnixNow() of each request */
  const uint32_t* hits;           /* [n_requests] HitsAddend */
  const uint32_t* req_idx;        /* [n_descriptors] */
  const uint32_t* entry_first;    /* [n_descriptors + 1] */
  const uint32_t* desc_off;       /* [n_descriptors + 1] */
  const uint8_t* desc_bytes;
  const uint16_t* key_len;        /* [n_entries] */
  const uint16_t* value_len;      /* [n_entries] */
  const uint8_t* override_flags;  /* [n_descriptors] or NULL */
  const uint32_t* override_rpu;   /* [n_descriptors] or NULL */
  const uint8_t* override_unit;   /* [n_descriptors] or NULL (pb_type.RateLimitUnit) */
  const uint32_t* override_rule;  /* [n_descriptors] or NULL */
} rl_request_batch;

/* Per descriptor, what the service answers (ratelimit.go:158-190). */
enum rl_match { RL_MATCH_NONE = 0, RL_MATCH_UNLIMITED = 1, RL_MATCH_LIMIT = 2 };
typedef struct rl_request_result {
  uint8_t* code;               /* [n_descriptors] rl_code */
  uint32_t* limit_remaining;   /* [n_descriptors]; MaxUint32 for unlimited */
  uint32_t* reset_s;           /* [n_descriptors]; 0 = no DurationUntilReset (nil limit) */
  uint8_t* match;              /* [n_descriptors] rl_match */
  uint32_t* rule_id;           /* [n_descriptors] matched rule (RL_MATCH_LIMIT / UNLIMITED) */
  uint32_t* requests_per_unit; /* [n_descriptors] CurrentLimit.RequestsPerUnit (RL_MATCH_LIMIT) */
  uint8_t* unit;               /* [n_descriptors] CurrentLimit.Unit (RL_MATCH_LIMIT) */
  uint64_t* stats;             /* [n_rules * RL_NUM_STATS], this call's deltas */
} rl_request_result;

/* GetLimit + DoLimit + the unlimited mapping for a batch of raw requests.
 * Synchronous. A descriptor whose override or config unit is not 1..4 fails
 * the batch with RL_E_INVALID (the reference panics in UnitToDivider). On a
 * multi-shard ctx the match runs on shard 0's GPU and the matched descriptors
 * go through the shards like a device batch (every owner answers its keys);
 * not on a ctx that joined a communicator. */
int rl_do_limit_requests(rl_ctx* ctx, const rl_request_batch* in, rl_request_result* out);

/* ---- Host packer -------------------------------------
 * Serialized envoy.service.ratelimit.v3.RateLimitRequest messages (the gRPC
 * payloads: msgs[msg_off[i], msg_off[i+1]), n + 1 offsets) with each request's
 * UnixNow() -> an rl_request_batch for rl_do_limit_requests, without building
 * per-descriptor objects. Replaces the per-descriptor Go work of
 * constructLimitsToCheck's caller side (src/service/ratelimit.go:104-143) and the
 * proto unmarshalling of the request. Override stats keys (descriptorKey,
 * src/config/config_impl.go:300-312) are interned to rule ids from
 * first_override_rule up (config rules take the ids below it);
 * rl_packer_rule_key names them. The batch's arrays are owned by the packer and
 * valid until its next rl_packer_pack. Host code; no GPU needed. */
typedef struct rl_packer rl_packer;
rl_packer* rl_packer_create(uint32_t first_override_rule);
void rl_packer_destroy(rl_packer* packer);
int rl_packer_pack(rl_packer* packer, const uint8_t* msgs, const uint64_t* msg_off, uint32_t n,
                   const int64_t* now, rl_request_batch* out);
uint32_t rl_packer_rules(const rl_packer* packer);  /* first_override_rule + interned override keys */
const char* rl_packer_rule_key(const rl_packer* packer, uint32_t rule_id);  /* NULL below first_override_rule */
const char* rl_packer_last_error(const rl_packer* packer);

/* ---- Observability and restart -----------------------
 * rl_local_cache_info_get: the local over-limit cache gauges of
 * limiter.localCacheStats (src/limiter/local_cache_stats.go:20-43):
 * lookup_count = Get calls (one per descriptor with a limit while the local cache
 * is enabled, fixed_cache_impl.go:57-67), hit_count, miss_count, and
 * entry_count = keys whose local-cache TTL has not passed at `now`. Counts are
 * cumulative since rl_create over the single-GPU batch path (rl_do_limit*,
 * rl_do_limit_requests). freecache's eviction/overwrite gauges have no
 * counterpart: entries live in the table's window records and are never evicted. */
typedef struct rl_local_cache_info {
  uint64_t entry_count;
  uint64_t lookup_count;
  uint64_t hit_count;
  uint64_t miss_count;
} rl_local_cache_info;
int rl_local_cache_info_get(rl_ctx* ctx, int64_t now, rl_local_cache_info* info);

/* Table snapshot / restore (Redis RDB-style restart): an exact image of the
 * counter table, the history log's written entries and append counters, the
 * long-stem arena, the local-cache state and the sweep time floor.
 * rl_snapshot_size gives the bytes rl_snapshot_save writes into `host`;
 * rl_snapshot_load accepts an image from a ctx with the same table_slots and
 * history_entries and an arena at least as large, whose live slots carry a
 * valid unit and long-stem arena offset (RL_E_INVALID otherwise). Both order
 * after every submitted batch. */
int rl_snapshot_size(rl_ctx* ctx, uint64_t* bytes);
int rl_snapshot_save(rl_ctx* ctx, void* host, uint64_t bytes);
int rl_snapshot_load(rl_ctx* ctx, const void* host, uint64_t bytes);

/* Per-stage device timing (HIP events on the batch stream), for benchmarks.
 * rl_profile(ctx, k) with k >= 1 starts accumulating over every k-th batch,
 * the first sampled one being the k-th submitted after the call (1 = every
 * batch; the event markers and k_table's per-workgroup clock reads cost a
 * sampled batch a few microseconds, so a sparse sample keeps the timed
 * pipeline unchanged), 0 stops;
 * rl_profile_read fills ms[0..n) with
 * the summed milliseconds of the stages {prepare, sort, segment, table, finish}
 * and *batches with the number of batches timed (it synchronises), then resets
 * the sums. "segment" runs up to the start of k_table (the table stage's
 * wait for the previous batch included), "table" brackets the single k_table
 * launch (the keys seen once and the short runs: the bulk of the table work),
 * "finish" the rest (deferrals, long runs, outputs). With n > RL_NUM_STAGES,
 * ms[RL_NUM_STAGES] is k_table's own run time per batch, AVERAGED over every
 * batch since profiling started or was last read (not only the timed
 * sample): its first workgroup's start to its last workgroup's end on the
 * device's constant clock (the kernel duration rocprofv3 reports; no event is
 * recorded for it), where "table" also holds the launch's queueing behind the
 * other streams' kernels and the event markers' own cost. */
#define RL_NUM_STAGES 5
int rl_profile(rl_ctx* ctx, int enable);
int rl_profile_read(rl_ctx* ctx, double* ms, uint32_t n, uint64_t* batches);

#ifdef __cplusplus
}
#endif
#endif /* RATELIMIT_HIP_H */
