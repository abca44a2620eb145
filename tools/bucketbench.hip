// bucketbench — development micro-benchmark of the stage-A grouping kernels
// (k_part + k_bucket + k_bucket_big) on 1M sort keys: kernel times,
// per-bucket phase stamps, and a check that the output is sorted, stable and
// correctly segmented.
//   bucketbench [n] [skew]   (skew e > 0: tenant = floor(u^-e), a Zipf-like mix; 10 ~ Zipf(1.1))
#define RL_BK_PROF 1
#include "rl_kernels.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace rl;

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000u;
  const double skew = argc > 2 ? atof(argv[2]) : 0.0;
  const bool zipf = skew > 0;
  const int iters = 20;
  const uint32_t ptiles = (n + PART_TILE - 1) / PART_TILE;
  std::vector<uint32_t> hk(n), hv(n), hh(n);
  std::mt19937_64 rng(11);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (uint32_t i = 0; i < n; i++) {
    uint64_t tenant = rng() % 10000000ull;
    if (zipf) tenant = std::min<uint64_t>((uint64_t)std::pow(1.0 - U(rng), -skew), 10000000ull);
    hk[i] = (uint32_t)(fmix64(tenant * 2 + (i & 1) + 1) >> 32);
    hv[i] = i;
    hh[i] = i % 7;
  }
  uint4* tl;
  uint32_t *kp[2], *vp[2], *hp[3], *info, *big_n, *work, *work_n, *cnt, *segsum, *rid, *rs, *re, *nr, *err, *ht;
  BigMeta* meta;
  for (int i = 0; i < 2; i++) {
    CK(hipMalloc(&kp[i], n * 4));
    CK(hipMalloc(&vp[i], n * 4));
  }
  for (int i = 0; i < 3; i++) CK(hipMalloc(&hp[i], n * 4));
  CK(hipMalloc(&ht, n * 4));
  CK(hipMalloc(&tl, n * 16));
  CK(hipMalloc(&info, (size_t)PART_DIGITS * ptiles * 4));
  const size_t items = n / BIG_CHUNK + 1 + PART_DIGITS;
  CK(hipMalloc(&meta, PART_DIGITS * sizeof(BigMeta)));
  CK(hipMalloc(&big_n, 4));
  CK(hipMalloc(&work, items * 4));
  CK(hipMalloc(&work_n, 4));
  CK(hipMalloc(&cnt, items * BIG_CNT * 4));
  CK(hipMalloc(&segsum, n * 4));
  CK(hipMalloc(&rid, n * 4));
  CK(hipMalloc(&rs, n * 4));
  CK(hipMalloc(&re, n * 4));
  CK(hipMalloc(&nr, 4));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  CK(hipMemcpy(hp[0], hh.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t ev[3];
  for (auto& e : ev) CK(hipEventCreate(&e));
  const size_t seg_lds = (2ull * ptiles + 1) * 4;
  double acc[2] = {0, 0};
  for (int it = 0; it < iters; it++) {
    CK(hipMemcpy(kp[0], hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(vp[0], hv.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(big_n, 0, 4));
    CK(hipMemset(work_n, 0, 4));
    CK(hipMemset(nr, 0, 4));
    CK(hipEventRecord(ev[0], 0));
    k_part<<<ptiles, 256>>>(kp[0], hp[0], tl, n, ptiles, info, err);
    CK(hipEventRecord(ev[1], 0));
    k_bucket<<<PART_DIGITS, BkSmall::THREADS, seg_lds>>>(tl, info, ptiles, kp[0], vp[0], hp[2], segsum,
                                                         rid, rs, re, nr, meta, big_n, work, work_n, err);
    k_big_count<<<BIG_ITEM_BLOCKS, BkSmall::THREADS, seg_lds>>>(tl, info, ptiles, meta, work, work_n, cnt, err);
    k_big_place<<<BIG_ITEM_BLOCKS, BkSmall::THREADS, seg_lds>>>(tl, info, ptiles, meta, work, work_n, cnt,
                                                                kp[0], vp[0], hp[2], segsum, rid, rs, re, err);
    k_bucket_big<<<BIG_BLOCKS, BkBig::THREADS, seg_lds>>>(tl, info, ptiles, kp[0], vp[0], hp[2], ht,
                                                          segsum, rid, rs, re, nr, meta, big_n, cnt, err);
    CK(hipEventRecord(ev[2], 0));
    CK(hipDeviceSynchronize());
    if (it >= 2)
      for (int j = 0; j < 2; j++) {
        float ms;
        CK(hipEventElapsedTime(&ms, ev[j], ev[j + 1]));
        acc[j] += ms;
      }
  }
  std::vector<uint32_t> ok(n), ov(n), os(n), orid(n), ors(n), ore(n);
  uint32_t onr = 0, nbig = 0;
  CK(hipMemcpy(ok.data(), kp[0], n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ov.data(), vp[0], n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(os.data(), segsum, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(orid.data(), rid, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ors.data(), rs, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ore.data(), re, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&onr, nr, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&nbig, big_n, 4, hipMemcpyDeviceToHost));
  // grouped: buckets in order, each key's elements contiguous and in arrival
  // order, every element exactly once (keys need not be sorted inside a bucket)
  bool good = true;
  uint32_t bad = 0;
  {
    std::vector<uint8_t> seen_idx(n, 0);
    std::vector<uint32_t> closed;
    for (uint32_t i = 0; i < n && good; i++) {
      bad = i;
      good = ov[i] < n && !seen_idx[ov[i]] && hk[ov[i]] == ok[i];
      if (!good) break;
      seen_idx[ov[i]] = 1;
      if (i) {
        if (ok[i] == ok[i - 1]) good = ov[i - 1] < ov[i];
        else {
          good = (ok[i - 1] >> (32 - PART_BITS)) <= (ok[i] >> (32 - PART_BITS));
          closed.push_back(ok[i - 1]);
        }
      }
    }
    if (good) {  // no key closed twice
      closed.push_back(ok[n - 1]);
      std::sort(closed.begin(), closed.end());
      good = std::adjacent_find(closed.begin(), closed.end()) == closed.end();
    }
  }
  if (!good) {  // diagnostics: the bucket holding the first bad position
    std::vector<uint32_t> cnt(PART_DIGITS, 0), keyc;
    for (uint32_t i = 0; i < n; i++) cnt[hk[i] >> (32 - PART_BITS)]++;
    const uint32_t d = ok[bad] >> (32 - PART_BITS);
    uint32_t base = 0;
    for (uint32_t e = 0; e < d; e++) base += cnt[e];
    std::vector<uint32_t> ks;
    for (uint32_t i = 0; i < n; i++)
      if ((hk[i] >> (32 - PART_BITS)) == d) ks.push_back(hk[i]);
    std::sort(ks.begin(), ks.end());
    uint32_t distinct = 0, maxrun = 0, run = 0;
    for (size_t i = 0; i < ks.size(); i++) {
      run = (i && ks[i] == ks[i - 1]) ? run + 1 : 1;
      distinct += run == 1;
      maxrun = std::max(maxrun, run);
    }
    {  // expected stable order of the bucket vs the output
      std::vector<std::pair<uint32_t, uint32_t>> ex;
      for (uint32_t i = 0; i < n; i++)
        if ((hk[i] >> (32 - PART_BITS)) == d) ex.emplace_back(hk[i], i);
      std::stable_sort(ex.begin(), ex.end(), [](auto& a, auto& b) { return a.first < b.first; });
      int shown = 0;
      uint32_t nm = 0;
      for (uint32_t q = 0; q < cnt[d]; q++) {
        if (ov[base + q] != ex[q].second) {
          nm++;
          if (shown++ < 8)
            printf("    pos %u: got val %u key %08x, expected val %u key %08x\n", q, ov[base + q], ok[base + q],
                   ex[q].second, ex[q].first);
        }
      }
      printf("    %u mismatches in the bucket\n", nm);
      std::vector<uint32_t> pl(PART_DIGITS * 16);
      if (hipMemcpyFromSymbol(pl.data(), HIP_SYMBOL(g_bk_peel), PART_DIGITS * 16 * 4) == hipSuccess) {
        const uint32_t* g = &pl[d * 16];
        printf("    peel: r %u nl %u S %u | heavy %08x %08x %08x %08x | cnt %u %u %u %u | start %u %u %u %u\n", g[0],
               g[1], g[14], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13]);
      }
    }
    printf("  first bad position %u: bucket %u (base %u, size %u, %u distinct keys, largest key %u), pos in bucket %u, "
           "key %08x prev %08x, val %u prev %u, hk[val] %08x\n", bad, d, base, cnt[d], distinct, maxrun, bad - base,
           ok[bad], bad ? ok[bad - 1] : 0u, ov[bad], bad ? ov[bad - 1] : 0u, hk[ov[bad]]);
  }
  uint32_t runs = 0, sum = 0;
  bool seg_ok = good;
  for (uint32_t i = 0; i < n && seg_ok; i++) {
    const bool head = i == 0 || ok[i - 1] != ok[i];
    const uint32_t h = hh[ov[i]] > 1 ? hh[ov[i]] : 1u;
    sum = head ? h : sum + h;
    runs += head;
    const uint32_t r = orid[i];
    seg_ok = os[i] == sum && r < onr && ors[r] <= i && i < ore[r] && (!head || ors[r] == i);
  }
  seg_ok = seg_ok && runs == onr;
  std::vector<unsigned long long> prof(PART_DIGITS * 16);
  CK(hipMemcpyFromSymbol(prof.data(), HIP_SYMBOL(g_bk_prof), PART_DIGITS * 16 * 8));
  const double us = 1.0 / 100.0;  // wall_clock64 at 100 MHz
  double ph[5] = {0, 0, 0, 0, 0}, mx = 0;
  int nb = 0;
  for (uint32_t b = 0; b < PART_DIGITS; b++) {  // fast buckets: stamps 0..5
    const unsigned long long* p = &prof[b * 16];
    if (!p[5] || p[5] < p[0] || p[1] < p[0]) continue;
    nb++;
    for (int j = 0; j < 5; j++) ph[j] += (double)(p[j + 1] - p[j]);
    mx = std::max(mx, (double)(p[5] - p[0]));
  }
  printf("n %u skew %.1f | k_part %.1f us, k_bucket + k_bucket_big %.1f us | runs %u | big buckets %u | grouped+stable %s, "
         "segments %s\n", n, skew, acc[0] * 1e3 / (iters - 2), acc[1] * 1e3 / (iters - 2), onr,
         nbig, good ? "yes" : "NO", seg_ok ? "ok" : "BAD");
  if (nb)
    printf("  %d fast buckets, per bucket: setup %.2f, load %.2f, sort %.2f, head count %.2f, segment %.2f us; "
           "max %.2f us\n", nb, ph[0] / nb * us, ph[1] / nb * us, ph[2] / nb * us, ph[3] / nb * us, ph[4] / nb * us,
           mx * us);
  for (uint32_t b = 0; b < PART_DIGITS; b++) {  // peeled large buckets: stamps 13..15, 7
    const unsigned long long* p = &prof[b * 16];
    if (!p[7] || p[7] < p[0] || !p[15] || p[15] < p[0]) continue;
    printf("  large bucket %u: setup %.2f, pass A %.2f, light sort+write %.2f, pass B %.2f, head count %.2f, "
           "segment %.2f, total %.2f us\n", b, (p[1] - p[0]) * us, (p[13] - p[1]) * us, (p[14] - p[13]) * us,
           (p[15] - p[14]) * us, (p[4] - p[15]) * us, (p[7] - p[4]) * us, (p[7] - p[0]) * us);
  }
  return good && seg_ok ? 0 : 2;
}
