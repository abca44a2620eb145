// dedupprobe.hip — cost of a per-batch hash set of sort keys on MI355X
// (measurement tool; not part of the library).
//
// Dedup-first stage A would insert each descriptor's 32-bit sort key into a
// set (64-bit CAS, epoch-tagged slots so the set is never cleared) and look it
// up in the next kernel to learn whether the key occurs twice or more. This
// times those two passes over a C1-shaped batch (1M keys from 10M tenants x 2
// units: ~5% of keys occur twice) next to a plain streaming read of the keys.
// Usage: dedupprobe [n=1048576] [set_log2=21] [tenants=10000000]; one JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__host__ __device__ inline uint64_t mix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

constexpr uint64_t DUPBIT = 1ull << 23;
__device__ inline bool current(uint64_t v, uint32_t ep) { return ((v >> 24) & 0xFFu) == ep; }

__global__ __launch_bounds__(256) void k_insert(const uint32_t* __restrict__ keys, uint32_t n,
                                                unsigned long long* set, uint64_t mask, uint32_t ep) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  uint64_t s = (uint64_t)(k * 0x9E3779B1u) & mask;
  const unsigned long long mine = ((unsigned long long)k << 32) | ((unsigned long long)ep << 24);
  for (uint32_t probe = 0; probe <= mask; probe++) {
    unsigned long long v = set[s];
    for (;;) {
      if (current(v, ep)) break;
      const unsigned long long o = atomicCAS(&set[s], v, mine);
      if (o == v) return;  // first of its key
      v = o;
    }
    if ((uint32_t)(v >> 32) == k) {  // seen before
      if (!(v & DUPBIT)) atomicOr(&set[s], DUPBIT);
      return;
    }
    s = (s + 1) & mask;
  }
}

__global__ __launch_bounds__(256) void k_lookup(const uint32_t* __restrict__ keys, uint32_t n,
                                                const unsigned long long* __restrict__ set, uint64_t mask,
                                                uint32_t ep, uint32_t* __restrict__ dup, uint32_t* ndup) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  bool d = false;
  if (i < n) {
    const uint32_t k = keys[i];
    uint64_t s = (uint64_t)(k * 0x9E3779B1u) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++) {
      const unsigned long long v = set[s];
      if (current(v, ep) && (uint32_t)(v >> 32) == k) {
        d = (v & DUPBIT) != 0;
        break;
      }
      s = (s + 1) & mask;
    }
    dup[i] = d;
  }
  const unsigned long long b = __ballot(d);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(ndup, (uint32_t)__popcll(b));
}

__global__ __launch_bounds__(256) void k_stream(const uint32_t* __restrict__ keys, uint32_t n,
                                                uint32_t* __restrict__ dup) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) dup[i] = keys[i] & 1u;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const uint32_t lg = argc > 2 ? (uint32_t)atoi(argv[2]) : 21u;
  const uint64_t tenants = argc > 3 ? (uint64_t)atoll(argv[3]) : 10000000ull;
  const uint64_t sz = 1ull << lg, mask = sz - 1;
  std::vector<uint32_t> h(n);
  uint64_t st = 12345;
  for (uint32_t i = 0; i < n; i += 2) {
    st = mix(st + 1);
    const uint64_t t = st % tenants;
    h[i] = (uint32_t)(mix(2 * t) >> 32);
    if (i + 1 < n) h[i + 1] = (uint32_t)(mix(2 * t + 1) >> 32);
  }
  uint32_t *keys, *dup, *ndup;
  unsigned long long* set;
  CHK(hipMalloc(&keys, n * 4ull));
  CHK(hipMalloc(&dup, n * 4ull));
  CHK(hipMalloc(&ndup, 4));
  CHK(hipMalloc(&set, sz * 8));
  CHK(hipMemcpy(keys, h.data(), n * 4ull, hipMemcpyHostToDevice));
  CHK(hipMemset(set, 0, sz * 8));
  hipEvent_t e0, e1, e2, e3;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventCreate(&e2));
  CHK(hipEventCreate(&e3));
  const uint32_t g = (n + 255) / 256;
  float ti = 0, tl = 0, ts = 0;
  uint32_t nd = 0;
  const int iters = 30;
  for (int it = 0; it < iters + 3; it++) {
    const uint32_t ep = 1 + (it % 255);
    CHK(hipMemset(ndup, 0, 4));
    CHK(hipEventRecord(e0, 0));
    k_insert<<<g, 256>>>(keys, n, set, mask, ep);
    CHK(hipEventRecord(e1, 0));
    k_lookup<<<g, 256>>>(keys, n, set, mask, ep, dup, ndup);
    CHK(hipEventRecord(e2, 0));
    k_stream<<<g, 256>>>(keys, n, dup);
    CHK(hipEventRecord(e3, 0));
    CHK(hipEventSynchronize(e3));
    float a, b, c;
    CHK(hipEventElapsedTime(&a, e0, e1));
    CHK(hipEventElapsedTime(&b, e1, e2));
    CHK(hipEventElapsedTime(&c, e2, e3));
    if (it >= 3) {
      ti += a;
      tl += b;
      ts += c;
    }
    CHK(hipMemcpy(&nd, ndup, 4, hipMemcpyDeviceToHost));
  }
  printf("{\"n\": %u, \"set_slots\": %llu, \"dup_keys\": %u, \"insert_us\": %.2f, \"lookup_us\": %.2f, "
         "\"stream_us\": %.2f}\n",
         n, (unsigned long long)sz, nd, ti / iters * 1e3, tl / iters * 1e3, ts / iters * 1e3);
  return 0;
}
