// slotprobe.hip — the access-pattern floor of k_unique on MI355X, and slot
// layout alternatives (measurement tool; not part of the library).
//
// Every lane does what k_unique does to memory for one descriptor with no
// table logic: coalesced reads of its 32-B record and ~36-B stem (arrival
// order), one random probe of a 128-B slot in a large table, a write-back of
// the changed window record(s), and a coalesced 8-B result store. Modes:
//   0  read slot bytes 0..63; write 16 B at +12 (cur, unaligned) and 16 B at +64
//      (prev): the current layout when a window rolls
//   1  read bytes 0..63; write 16 B at +12 only (same window)
//   2  read bytes 0..127; write 32 B at +16 (cur and prev side by side, aligned)
//   3  read bytes 0..127; write 16 B at +16
//   4  read bytes 0..63 only
//   5  read bytes 0..127 only
//   6  no slot access (the streaming part alone)
// Usage: slotprobe [lanes=1048576] [table_log2=26] [reps=20]; one JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_slot(uint8_t* __restrict__ table, uint64_t mask, const uint4* __restrict__ rec,
                                              const uint8_t* __restrict__ stem, uint32_t n,
                                              unsigned long long* __restrict__ res, uint32_t salt) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4 r0 = rec[2 * (size_t)i], r1 = rec[2 * (size_t)i + 1];
  const uint4* sp = reinterpret_cast<const uint4*>(stem + (size_t)i * 36 - ((size_t)i * 36 & 15));
  const uint4 t0 = sp[0], t1 = sp[1], t2 = sp[2];
  uint32_t acc = r0.x ^ r1.y ^ t0.x ^ t1.y ^ t2.z;
  const uint64_t s = mix(((uint64_t)salt << 32) | (i ^ (acc & 1u))) & mask;
  uint4* line = reinterpret_cast<uint4*>(table + s * 128);
  if (MODE != 6) {
    uint4 a[8];
    const int nl = (MODE == 2 || MODE == 3 || MODE == 5) ? 8 : 4;
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = k < nl ? line[k] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 8; k++) acc ^= a[k].x ^ a[k].w;
    uint32_t* d = reinterpret_cast<uint32_t*>(line);
    if (MODE == 0 || MODE == 1) {  // cur at +12 (dwords 3..6)
      d[3] = acc; d[4] = a[1].x + 1; d[5] = a[1].y; d[6] = a[1].z;
      if (MODE == 0) line[4] = make_uint4(a[0].w, a[1].x, a[1].y, acc);  // prev at +64
    } else if (MODE == 2) {
      line[1] = make_uint4(acc, a[1].y + 1, a[1].z, a[1].w);
      line[2] = make_uint4(a[1].x, a[1].y, a[1].z, acc);
    } else if (MODE == 3) {
      line[1] = make_uint4(acc, a[1].y + 1, a[1].z, a[1].w);
    }
  }
  res[i] = ((unsigned long long)acc << 32) | i;
}

template <int MODE>
float run(uint8_t* table, uint64_t mask, const uint4* rec, const uint8_t* stem, uint32_t n,
          unsigned long long* res, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  k_slot<MODE><<<(n + 255) / 256, 256>>>(table, mask, rec, stem, n, res, 999);  // warm
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) k_slot<MODE><<<(n + 255) / 256, 256>>>(table, mask, rec, stem, n, res, r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const int lg = argc > 2 ? atoi(argv[2]) : 26;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const uint64_t slots = 1ull << lg;
  uint8_t *table, *stem;
  uint4* rec;
  unsigned long long* res;
  CHK(hipMalloc(&table, slots * 128));
  CHK(hipMemset(table, 0, slots * 128));
  CHK(hipMalloc(&rec, (size_t)n * 32));
  CHK(hipMemset(rec, 1, (size_t)n * 32));
  CHK(hipMalloc(&stem, (size_t)n * 36 + 64));
  CHK(hipMemset(stem, 2, (size_t)n * 36 + 64));
  CHK(hipMalloc(&res, (size_t)n * 8));
  float t[7];
  t[0] = run<0>(table, slots - 1, rec, stem, n, res, reps);
  t[1] = run<1>(table, slots - 1, rec, stem, n, res, reps);
  t[2] = run<2>(table, slots - 1, rec, stem, n, res, reps);
  t[3] = run<3>(table, slots - 1, rec, stem, n, res, reps);
  t[4] = run<4>(table, slots - 1, rec, stem, n, res, reps);
  t[5] = run<5>(table, slots - 1, rec, stem, n, res, reps);
  t[6] = run<6>(table, slots - 1, rec, stem, n, res, reps);
  printf("{\"tool\": \"slotprobe\", \"lanes\": %u, \"table_bytes\": %llu, \"us\": {\"rd64_wr_cur12_prev64\": %.1f, "
         "\"rd64_wr_cur12\": %.1f, \"rd128_wr32_at16\": %.1f, \"rd128_wr16_at16\": %.1f, \"rd64\": %.1f, "
         "\"rd128\": %.1f, \"stream_only\": %.1f}}\n",
         n, (unsigned long long)(slots * 128), t[0], t[1], t[2], t[3], t[4], t[5], t[6]);
  return 0;
}
