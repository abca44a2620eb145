// pmcprobe.hip — calibration of the PMC HBM byte counters for the access
// pattern of the table kernels (measurement tool; not part of the library).
//
// k_rand64: every lane reads one uniformly random, 64-B aligned 64-B sector of
// a table far larger than the caches (4 x 16-B loads) and writes 4 B, so the
// bytes moved are known exactly: 64 x lanes read, 4 x lanes written.
// k_seq: every lane reads 64 consecutive bytes of a streamed buffer (the same
// byte count, coalesced), for the streaming-side factor.
// Run under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (separate
// passes); scripts/pmc_summary.py divides the counters by these byte counts
// to get the correction factor it applies to the pipeline kernels.
//
// usage: pmcprobe [lanes=4194304] [table_log2_bytes=33] [reps=5]; one JSON line.
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

__device__ __forceinline__ unsigned long long mix(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__global__ __launch_bounds__(256) void k_rand64(const uint4* __restrict__ table, unsigned long long sectors,
                                                unsigned* __restrict__ out, unsigned n, unsigned salt) {
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned long long s = mix(((unsigned long long)salt << 32) | i) % sectors;
  const uint4* p = table + s * 4;
  const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  out[i] = a.x ^ b.y ^ c.z ^ d.w;
}

__global__ __launch_bounds__(256) void k_seq(const uint4* __restrict__ buf, unsigned* __restrict__ out, unsigned n) {
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4* p = buf + (size_t)i * 4;
  const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  out[i] = a.x ^ b.y ^ c.z ^ d.w;
}

int main(int argc, char** argv) {
  const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : (1u << 22);
  const int lg = argc > 2 ? atoi(argv[2]) : 33;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const unsigned long long bytes = 1ull << lg, sectors = bytes / 64;
  uint4 *table, *buf;
  unsigned* out;
  CHK(hipMalloc(&table, bytes));
  CHK(hipMemset(table, 1, bytes));
  CHK(hipMalloc(&buf, (size_t)n * 64));
  CHK(hipMemset(buf, 2, (size_t)n * 64));
  CHK(hipMalloc(&out, (size_t)n * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float ms_r = 0, ms_s = 0, t;
  for (int r = 0; r < reps; r++) {
    CHK(hipEventRecord(e0));
    k_rand64<<<(n + 255) / 256, 256>>>(table, sectors, out, n, (unsigned)r);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&t, e0, e1));
    ms_r += t;
    CHK(hipEventRecord(e0));
    k_seq<<<(n + 255) / 256, 256>>>(buf, out, n);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&t, e0, e1));
    ms_s += t;
  }
  printf("{\"tool\": \"pmcprobe\", \"lanes\": %u, \"table_bytes\": %llu, \"read_bytes_per_launch\": %llu, "
         "\"write_bytes_per_launch\": %llu, \"rand64_us\": %.1f, \"seq64_us\": %.1f}\n",
         n, bytes, 64ull * n, 4ull * n, ms_r * 1000.f / reps, ms_s * 1000.f / reps);
  return 0;
}
