// randprobe.hip — the random-access floor of k_runs' memory pattern on MI355X
// (measurement tool; not part of the library).
//
// k_runs does, per run of one descriptor at C1: read the home slot's first
// 64-B sector (random in an 8.6 GB table), read the 32-B record and the ~34-B
// stem (random in the batch's arrival-order buffers), write the 16-B window
// record back into the slot and scatter an 8-B result. These kernels replay
// exactly that pattern with no table logic, over the same sizes, so the time of
// the `pattern` kernel is the floor k_runs could reach without touching fewer
// random bytes:
//   slot64   1M random 64-B sector reads (the probe alone)
//   reads    slot 64 B + record 32 B + stem 48 B random reads
//   pattern  reads + 16-B slot write + 8-B result scatter (k_runs' full pattern)
//   chain    pattern, with record and stem addresses depending on the slot data
// Usage: randprobe [lanes=1048576] [table_log2=26]; prints one JSON line.
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
__global__ __launch_bounds__(256) void k_probe(uint4* __restrict__ slots, uint64_t mask, const uint4* __restrict__ rec,
                                               const uint4* __restrict__ stem, uint32_t n, uint32_t* __restrict__ out,
                                               unsigned long long* __restrict__ res, uint32_t salt) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = mix(((uint64_t)salt << 32) | i);
  const uint64_t s = h & mask;
  uint4 a0 = slots[s * 8], a1 = slots[s * 8 + 1], a2 = slots[s * 8 + 2], a3 = slots[s * 8 + 3];
  uint32_t acc = a0.x ^ a1.y ^ a2.z ^ a3.w;
  if (MODE >= 1) {
    // record (32 B) and stem (48 B) at random positions of 1M-entry buffers
    uint32_t e = (uint32_t)(h >> 40) % n;
    if (MODE == 3) e = (e ^ (acc & 1u)) % n;  // the address depends on the slot data
    const uint4 r0 = rec[2 * (size_t)e], r1 = rec[2 * (size_t)e + 1];
    uint32_t so = (r0.x ^ (uint32_t)(h >> 20)) % n;
    if (MODE != 3) so = (uint32_t)(h >> 20) % n;
    const uint4 t0 = stem[3 * (size_t)so], t1 = stem[3 * (size_t)so + 1], t2 = stem[3 * (size_t)so + 2];
    acc ^= r0.y ^ r1.z ^ t0.x ^ t1.y ^ t2.z;
    if (MODE >= 2) {
      slots[s * 8 + 1] = make_uint4(acc, a1.y + 1, a1.z, a1.w);  // window record write-back (16 B)
      res[e] = ((unsigned long long)acc << 32) | i;             // result scatter (8 B, arrival order)
    }
  }
  out[i] = acc;
}

template <int MODE>
float run(uint4* slots, uint64_t mask, const uint4* rec, const uint4* stem, uint32_t n, uint32_t* out,
          unsigned long long* res, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const uint32_t g = (n + 255) / 256;
  k_probe<MODE><<<g, 256>>>(slots, mask, rec, stem, n, out, res, 12345u);
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) k_probe<MODE><<<g, 256>>>(slots, mask, rec, stem, n, out, res, (uint32_t)r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return ms * 1000.f / reps;  // us per launch
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const int lg = argc > 2 ? atoi(argv[2]) : 26;
  const uint64_t nslots = 1ull << lg;
  uint4 *slots, *rec, *stem;
  uint32_t* out;
  unsigned long long* res;
  CHK(hipMalloc(&slots, nslots * 128));
  CHK(hipMalloc(&rec, (size_t)n * 32));
  CHK(hipMalloc(&stem, (size_t)n * 48));
  CHK(hipMalloc(&out, (size_t)n * 4));
  CHK(hipMalloc(&res, (size_t)n * 8));
  CHK(hipMemset(slots, 1, nslots * 128));
  CHK(hipMemset(rec, 2, (size_t)n * 32));
  CHK(hipMemset(stem, 3, (size_t)n * 48));
  const int reps = 20;
  const float t0 = run<0>(slots, nslots - 1, rec, stem, n, out, res, reps);
  const float t1 = run<1>(slots, nslots - 1, rec, stem, n, out, res, reps);
  const float t2 = run<2>(slots, nslots - 1, rec, stem, n, out, res, reps);
  const float t3 = run<3>(slots, nslots - 1, rec, stem, n, out, res, reps);
  printf("{\"tool\": \"randprobe\", \"lanes\": %u, \"table_bytes\": %llu, \"us_slot64\": %.1f, \"us_reads\": %.1f, "
         "\"us_pattern\": %.1f, \"us_chain\": %.1f, \"slot64_GBps\": %.0f, \"pattern_random_bytes_per_lane\": 168}\n",
         n, (unsigned long long)(nslots * 128), t0, t1, t2, t3, n * 64.0 / (t0 * 1e3));
  CHK(hipFree(slots));
  CHK(hipFree(rec));
  CHK(hipFree(stem));
  CHK(hipFree(out));
  CHK(hipFree(res));
  return 0;
}
