// tlbprobe.hip — does the order of k_table's random slot reads matter on
// MI355X? (measurement tool; not part of the library)
//
// randprobe's size sweep (profiles/r04/randprobe_sweep.txt) shows one random
// 64-B sector read per lane running 2.3x slower from a 17 GB table than from
// a 512 MB one, with the cliff between 2 and 4 GB: address-translation reach,
// not HBM. k_table reads C1's keys seen once in arrival order, i.e. uniformly
// over the whole table at every moment. These kernels read the same number of
// random sectors from the same table in other orders:
//   uniform   lane i -> a uniform random slot (k_table today)
//   bucketed  workgroup b -> region b % R of R equal regions, random inside
//             (k_table fed bucket by bucket, one bucket per workgroup)
//   sorted    lane i -> a random slot inside the i-th of n equal strides
//             (the whole batch sorted by home slot)
//   sorted_xcd  sorted, but workgroup b takes the (b % 8) * (G/8) + b / 8-th
//             block of the sorted order (each XCD a contiguous eighth of it)
// Usage: tlbprobe [lanes=4194304] [table_log2=27] [regions=1024]; one JSON line.
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
__global__ __launch_bounds__(256) void k_probe(const uint4* __restrict__ slots, uint64_t nslots, uint32_t n,
                                               uint32_t regions, uint32_t* __restrict__ out, uint32_t salt) {
  uint32_t b = blockIdx.x;
  if (MODE == 3) {  // XCD-major: consecutive workgroups go round the 8 XCDs
    const uint32_t G = gridDim.x, per = (G + 7) / 8;
    b = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (b >= G) {
      out[blockIdx.x * 256 + threadIdx.x] = 0;
      return;
    }
  }
  const uint32_t i = b * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = mix(((uint64_t)salt << 32) | i);
  uint64_t s;
  if (MODE == 0) {
    s = h & (nslots - 1);
  } else if (MODE == 1) {
    const uint64_t rsz = nslots / regions;
    s = (uint64_t)(b % regions) * rsz + (h % rsz);
  } else {
    const uint64_t stride = nslots / n;
    s = (uint64_t)i * stride + (h % stride);
  }
  const uint4 a0 = slots[s * 4], a1 = slots[s * 4 + 1], a2 = slots[s * 4 + 2], a3 = slots[s * 4 + 3];
  out[i] = a0.x ^ a1.y ^ a2.z ^ a3.w;
}

template <int MODE>
float run(const uint4* slots, uint64_t nslots, uint32_t n, uint32_t regions, uint32_t* out, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const uint32_t g = (n + 255) / 256;
  k_probe<MODE><<<g, 256>>>(slots, nslots, n, regions, out, 777u);
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) k_probe<MODE><<<g, 256>>>(slots, nslots, n, regions, out, (uint32_t)r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 22);
  const int lg = argc > 2 ? atoi(argv[2]) : 27;
  const uint32_t regions = argc > 3 ? (uint32_t)atoi(argv[3]) : 1024;
  const uint64_t nslots = 1ull << lg;  // 64-B slots
  uint4* slots;
  uint32_t* out;
  CHK(hipMalloc(&slots, nslots * 64));
  CHK(hipMalloc(&out, (size_t)n * 4 + 4096));
  CHK(hipMemset(slots, 1, nslots * 64));
  const int reps = 20;
  const float t0 = run<0>(slots, nslots, n, regions, out, reps);
  const float t1 = run<1>(slots, nslots, n, regions, out, reps);
  const float t2 = run<2>(slots, nslots, n, regions, out, reps);
  const float t3 = run<3>(slots, nslots, n, regions, out, reps);
  printf("{\"tool\": \"tlbprobe\", \"lanes\": %u, \"table_bytes\": %llu, \"regions\": %u, \"us_uniform\": %.1f, "
         "\"us_bucketed\": %.1f, \"us_sorted\": %.1f, \"us_sorted_xcd\": %.1f, \"uniform_GBps\": %.0f, "
         "\"bucketed_GBps\": %.0f, \"sorted_GBps\": %.0f}\n",
         n, (unsigned long long)(nslots * 64), regions, t0, t1, t2, t3, n * 64.0 / (t0 * 1e3), n * 64.0 / (t1 * 1e3),
         n * 64.0 / (t2 * 1e3));
  CHK(hipFree(slots));
  CHK(hipFree(out));
  return 0;
}
