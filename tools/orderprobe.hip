// orderprobe.hip — what k_table's singleton part would cost with its lanes in
// bucket (home-region) order instead of arrival order, per data layout
// (measurement tool; not part of the library).
//
// tlbprobe.hip showed a random 64-B sector read from a multi-GB table running
// 2.2x faster when a workgroup's probes stay in 1/1024 of the table. Walking
// the keys seen once in bucket order, though, turns the batch-side accesses
// (record, stem, result) from coalesced streams into gathers unless they are
// laid out in bucket order first. One lane per descriptor, n lanes, a table of
// 2^lg 64-B slots; per lane one slot sector read, a 16-B write into it, and:
//   arrival      record 32 B + stem 34 B read coalesced, result 8 B stored
//                coalesced; the slot uniform over the table (k_table today)
//   gather       bucket order through an 8-B list: record and stem gathered
//                from arrival-order buffers, the result scattered; the slot
//                inside the lane's bucket region
//   fat          bucket order, a dense 64-B record (record + stem) read
//                coalesced, the result scattered by arrival index
//   fat_res      as fat, the result stored coalesced in bucket order
//   perm         the permutation pass fat_res would need afterwards (8-B
//                gather by position, 8-B coalesced store)
//   arrival_ovf_write / _rmw   arrival, and every other lane also writes a
//                32-B record at a random place of an overflow table (half
//                the slots' bytes) / reads it first (an open-addressing insert)
// Usage: orderprobe [lanes=1048576] [table_log2=27]; one JSON line.
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

constexpr uint32_t REGIONS = 1024;

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(uint4* __restrict__ slots, uint64_t nslots, uint4* __restrict__ ovf,
                                               uint64_t novf, const uint4* __restrict__ rec,
                                               const uint8_t* __restrict__ stem, const uint4* __restrict__ fat,
                                               const uint2* __restrict__ list, uint32_t n,
                                               unsigned long long* __restrict__ res, uint32_t salt) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = mix(((uint64_t)salt << 32) | i);
  uint64_t s;
  uint32_t acc = 0, e = i;
  if (MODE == 0 || MODE >= 4) {
    s = h & (nslots - 1);
    const uint4 r0 = rec[2 * (size_t)i], r1 = rec[2 * (size_t)i + 1];
    const uint4* sp = reinterpret_cast<const uint4*>(stem + (((size_t)i * 34) & ~(size_t)15));
    const uint4 t0 = sp[0], t1 = sp[1], t2 = sp[2];
    acc = r0.x ^ r1.y ^ t0.z ^ t1.w ^ t2.x;
  } else {
    const uint64_t rsz = nslots / REGIONS;
    s = (uint64_t)((uint64_t)i * REGIONS / n) * rsz + (h % rsz);
    if (MODE == 1) {
      const uint2 l = list[i];
      e = l.x;
      const uint4 r0 = rec[2 * (size_t)e], r1 = rec[2 * (size_t)e + 1];
      const uint4* sp = reinterpret_cast<const uint4*>(stem + (((size_t)e * 34) & ~(size_t)15));
      const uint4 t0 = sp[0], t1 = sp[1], t2 = sp[2];
      acc = l.y ^ r0.x ^ r1.y ^ t0.z ^ t1.w ^ t2.x;
    } else {
      const uint4 f0 = fat[4 * (size_t)i], f1 = fat[4 * (size_t)i + 1], f2 = fat[4 * (size_t)i + 2],
                  f3 = fat[4 * (size_t)i + 3];
      acc = f0.x ^ f1.y ^ f2.z ^ f3.w;
      e = MODE == 2 ? f0.y % n : i;  // the arrival index travels in the record
    }
  }
  const uint4 a0 = slots[s * 4], a1 = slots[s * 4 + 1], a2 = slots[s * 4 + 2], a3 = slots[s * 4 + 3];
  acc ^= a0.x ^ a1.y ^ a2.z ^ a3.w;
  slots[s * 4 + 1] = make_uint4(acc, a1.y + 1, a1.z, a1.w);  // window record write-back (16 B)
  res[e] = ((unsigned long long)acc << 32) | i;
  if (MODE >= 4 && (i & 1)) {  // the displaced window record into an overflow table (every other lane)
    const uint64_t o = mix(h) & (novf - 1);
    uint32_t t = 0;
    if (MODE == 5) t = ovf[2 * o].x;  // (probe first: an open-addressing insert)
    ovf[2 * o] = make_uint4(acc + t, i, 7u, 8u);
    ovf[2 * o + 1] = make_uint4(i, acc, 0u, 0u);
  }
}

__global__ __launch_bounds__(256) void k_perm(const unsigned long long* __restrict__ src, const uint2* __restrict__ list,
                                              uint32_t n, unsigned long long* __restrict__ dst) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  dst[i] = src[list[i].y % n];  // (y: the position of arrival index i in bucket order)
}

template <typename F>
float timed(F f, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  f(12345u);
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) f((uint32_t)r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return ms * 1000.f / reps;  // us per launch
}

__global__ void k_fill_list(uint2* list, uint4* fat, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = (uint32_t)(mix(i) % n);
  list[i] = make_uint2(e, (uint32_t)(mix(i + 7) % n));
  fat[4 * (size_t)i] = make_uint4(i, e, 5u, 6u);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const int lg = argc > 2 ? atoi(argv[2]) : 27;
  const uint64_t nslots = 1ull << lg;  // 64-B slots
  uint4 *slots, *rec, *fat;
  uint8_t* stem;
  uint2* list;
  unsigned long long *res, *res2;
  CHK(hipMalloc(&slots, nslots * 64));
  const uint64_t novf = nslots / 2;  // 32-B overflow entries: a table half the slots' bytes
  uint4* ovf;
  CHK(hipMalloc(&ovf, novf * 32));
  CHK(hipMemset(ovf, 0, novf * 32));
  CHK(hipMalloc(&rec, (size_t)n * 32));
  CHK(hipMalloc(&stem, (size_t)n * 34 + 64));
  CHK(hipMalloc(&fat, (size_t)n * 64));
  CHK(hipMalloc(&list, (size_t)n * 8));
  CHK(hipMalloc(&res, (size_t)n * 8));
  CHK(hipMalloc(&res2, (size_t)n * 8));
  CHK(hipMemset(slots, 1, nslots * 64));
  CHK(hipMemset(rec, 2, (size_t)n * 32));
  CHK(hipMemset(stem, 3, (size_t)n * 34 + 64));
  CHK(hipMemset(fat, 4, (size_t)n * 64));
  const uint32_t g = (n + 255) / 256;
  k_fill_list<<<g, 256>>>(list, fat, n);
  const int reps = 20;
  float t[7];
  t[0] = timed([&](uint32_t s) { k_probe<0><<<g, 256>>>(slots, nslots, ovf, novf, rec, stem, fat, list, n, res, s); }, reps);
  t[1] = timed([&](uint32_t s) { k_probe<1><<<g, 256>>>(slots, nslots, ovf, novf, rec, stem, fat, list, n, res, s); }, reps);
  t[2] = timed([&](uint32_t s) { k_probe<2><<<g, 256>>>(slots, nslots, ovf, novf, rec, stem, fat, list, n, res, s); }, reps);
  t[3] = timed([&](uint32_t s) { k_probe<3><<<g, 256>>>(slots, nslots, ovf, novf, rec, stem, fat, list, n, res, s); }, reps);
  t[4] = timed([&](uint32_t) { k_perm<<<g, 256>>>(res, list, n, res2); }, reps);
  t[5] = timed([&](uint32_t s) { k_probe<4><<<g, 256>>>(slots, nslots, ovf, novf, rec, stem, fat, list, n, res, s); }, reps);
  t[6] = timed([&](uint32_t s) { k_probe<5><<<g, 256>>>(slots, nslots, ovf, novf, rec, stem, fat, list, n, res, s); }, reps);
  printf("{\"tool\": \"orderprobe\", \"lanes\": %u, \"table_bytes\": %llu, \"us_arrival\": %.1f, \"us_gather\": %.1f, "
         "\"us_fat\": %.1f, \"us_fat_res\": %.1f, \"us_perm\": %.1f, \"us_arrival_ovf_write\": %.1f, \"us_arrival_ovf_rmw\": %.1f}\n",
         n, (unsigned long long)(nslots * 64), t[0], t[1], t[2], t[3], t[4], t[5], t[6]);
  return 0;
}
