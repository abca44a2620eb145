// bucketbench — development micro-benchmark of the stage-A grouping kernels
// (k_part + k_bucket) on 1M sort keys: kernel times, per-bucket phase stamps,
// and a check that the output is sorted, stable and correctly segmented.
//   bucketbench [n] [zipf]   (zipf: keys drawn from a Zipf(1.1)-like tenant mix)
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
  const bool zipf = argc > 2 && atoi(argv[2]) != 0;
  const int iters = 20;
  const uint32_t ptiles = (n + PART_TILE - 1) / PART_TILE;
  std::vector<uint32_t> hk(n), hv(n);
  std::vector<Rec> hr(n);
  std::mt19937_64 rng(11);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (uint32_t i = 0; i < n; i++) {
    uint64_t tenant = rng() % 10000000ull;
    if (zipf) tenant = std::min<uint64_t>((uint64_t)std::pow(1.0 - U(rng), -10.0), 10000000ull);
    hk[i] = (uint32_t)(fmix64(tenant * 2 + (i & 1) + 1) >> 32);
    hv[i] = i;
    hr[i] = Rec{0, 0, 0, 0, i, 0, (uint32_t)(i % 7), 100};
  }
  uint32_t *kp[2], *vp[2], *info, *tot, *segsum, *rid, *rs, *re, *nr, *err;
  Rec *rec, *rec_s;
  for (int i = 0; i < 2; i++) {
    CK(hipMalloc(&kp[i], n * 4));
    CK(hipMalloc(&vp[i], n * 4));
  }
  CK(hipMalloc(&info, 256ull * ptiles * 4));
  CK(hipMalloc(&tot, 1024));
  CK(hipMalloc(&segsum, n * 4));
  CK(hipMalloc(&rid, n * 4));
  CK(hipMalloc(&rs, n * 4));
  CK(hipMalloc(&re, n * 4));
  CK(hipMalloc(&nr, 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&rec, n * sizeof(Rec)));
  CK(hipMalloc(&rec_s, n * sizeof(Rec)));
  CK(hipMemset(err, 0, 4));
  CK(hipMemcpy(rec, hr.data(), n * sizeof(Rec), hipMemcpyHostToDevice));
  hipEvent_t ev[3];
  for (auto& e : ev) CK(hipEventCreate(&e));
  double acc[2] = {0, 0};
  for (int it = 0; it < iters; it++) {
    CK(hipMemcpy(kp[0], hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(vp[0], hv.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(tot, 0, 1024));
    CK(hipMemset(nr, 0, 4));
    CK(hipEventRecord(ev[0], 0));
    k_part<<<ptiles, 256>>>(kp[0], vp[0], kp[1], vp[1], n, ptiles, info, tot, err);
    CK(hipEventRecord(ev[1], 0));
    k_bucket<<<256, BK_THREADS>>>(kp[1], vp[1], info, tot, ptiles, rec, kp[0], vp[0], rec_s, segsum, rid, rs, re, nr,
                                  err);
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
  uint32_t onr = 0;
  CK(hipMemcpy(ok.data(), kp[0], n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ov.data(), vp[0], n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(os.data(), segsum, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(orid.data(), rid, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ors.data(), rs, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ore.data(), re, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&onr, nr, 4, hipMemcpyDeviceToHost));
  bool good = true;
  for (uint32_t i = 1; i < n && good; i++) good = ok[i - 1] < ok[i] || (ok[i - 1] == ok[i] && ov[i - 1] < ov[i]);
  for (uint32_t i = 0; i < n && good; i++) good = hk[ov[i]] == ok[i];
  uint32_t runs = 0, sum = 0;
  bool seg_ok = good;
  for (uint32_t i = 0; i < n && seg_ok; i++) {
    const bool head = i == 0 || ok[i - 1] != ok[i];
    const uint32_t h = hr[ov[i]].hits > 1 ? hr[ov[i]].hits : 1u;
    sum = head ? h : sum + h;
    runs += head;
    const uint32_t r = orid[i];
    seg_ok = os[i] == sum && r < onr && ors[r] <= i && i < ore[r] && (!head || ors[r] == i);
  }
  seg_ok = seg_ok && runs == onr;
  std::vector<unsigned long long> prof(256 * 16);
  CK(hipMemcpyFromSymbol(prof.data(), HIP_SYMBOL(g_bk_prof), 256 * 16 * 8));
  double ph[5] = {0, 0, 0, 0, 0}, fine[5] = {0, 0, 0, 0, 0}, mx = 0;
  unsigned long long t0 = ~0ull, tend = 0;
  int nb = 0;
  for (int b = 0; b < 256; b++) {
    const unsigned long long* p = &prof[b * 16];
    if (!p[5] || p[5] < p[0]) continue;  // empty / large bucket (no full stamps)
    nb++;
    for (int j = 0; j < 5; j++) ph[j] += (double)(p[j + 1] - p[j]);
    fine[0] += (double)(p[8] - p[2]);  // zero wcnt
    fine[1] += (double)(p[9] - p[8]);  // multisplit
    fine[2] += (double)(p[10] - p[9]); // digit scans
    fine[3] += (double)(p[11] - p[10]); // positions
    fine[4] += (double)(p[12] - p[11]); // LDS scatter + reload
    mx = std::max(mx, (double)(p[5] - p[0]));
    t0 = std::min(t0, p[0]);
    tend = std::max(tend, p[5]);
  }
  const double us = 1.0 / 100.0;  // wall_clock64 at 100 MHz
  printf("n %u %s | k_part %.1f us, k_bucket %.1f us | runs %u | sorted+stable %s, segments %s\n", n,
         zipf ? "zipf" : "uniform", acc[0] * 1e3 / (iters - 2), acc[1] * 1e3 / (iters - 2), onr, good ? "yes" : "NO",
         seg_ok ? "ok" : "BAD");
  if (nb)
    printf("  %d fast buckets, per bucket: setup %.2f, load %.2f, 3 passes %.2f, head count %.2f, segment %.2f us; "
           "max %.2f, span %.2f us\n",
           nb, ph[0] / nb * us, ph[1] / nb * us, ph[2] / nb * us, ph[3] / nb * us, ph[4] / nb * us, mx * us,
           (tend - t0) * us);
  if (nb)
    printf("  first pass: zero %.2f, multisplit %.2f, digit scans %.2f, positions %.2f, scatter+reload %.2f us\n",
           fine[0] / nb * us, fine[1] / nb * us, fine[2] / nb * us, fine[3] / nb * us, fine[4] / nb * us);
  return good && seg_ok ? 0 : 2;
}
