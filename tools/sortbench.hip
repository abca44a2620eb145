// sortbench — development micro-benchmark of the onesweep radix sort kernels
// (k_os_hist + 4 x k_os_pass) on 1M uniform 32-bit keys: per-kernel times,
// per-tile phase stamps of the last pass, and a sortedness/stability check.
// Built with different RL_OS_ITEMS / RL_OS_WAVES by tools/build_sortbench.sh.
#define RL_OS_PROF 1
#include "rl_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace rl;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000u;
  const int iters = 20;
  const uint32_t ntiles = (n + OS_TILE - 1) / OS_TILE;
  std::vector<uint32_t> hk(n), hv(n);
  std::mt19937 rng(7);
  for (uint32_t i = 0; i < n; i++) {
    hk[i] = rng();
    hv[i] = i;
  }
  uint32_t *k[2], *v[2], *ghist, *ctr, *err;
  unsigned long long* status;
  for (int i = 0; i < 2; i++) {
    CK(hipMalloc(&k[i], n * 4));
    CK(hipMalloc(&v[i], n * 4));
  }
  CK(hipMalloc(&ghist, 4096));
  CK(hipMalloc(&ctr, 32));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&status, 256ull * ntiles * 8));
  CK(hipMemset(status, 0, 256ull * ntiles * 8));
  CK(hipMemset(err, 0, 4));
  hipEvent_t ev[6];
  for (auto& e : ev) CK(hipEventCreate(&e));
  double acc[5] = {0, 0, 0, 0, 0};
  for (int it = 0; it < iters; it++) {
    CK(hipMemcpy(k[0], hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v[0], hv.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(ghist, 0, 4096));
    CK(hipMemset(ctr, 0, 32));
    CK(hipEventRecord(ev[0], 0));
    k_os_hist<<<ntiles < 256 ? ntiles : 256, 256>>>(k[0], n, ghist, err);
    CK(hipEventRecord(ev[1], 0));
    for (uint32_t pass = 0; pass < 4; pass++) {
      const uint32_t src = pass & 1, dst = src ^ 1;
      k_os_pass<<<ntiles, OS_THREADS>>>(k[src], v[src], k[dst], v[dst], n, pass, ghist, ctr, status,
                                        os_tag(it + 1, pass), err);
      CK(hipEventRecord(ev[2 + pass], 0));
    }
    CK(hipDeviceSynchronize());
    if (it >= 2)
      for (int j = 0; j < 5; j++) {
        float ms;
        CK(hipEventElapsedTime(&ms, ev[j], ev[j + 1 < 6 ? j + 1 : 5]));
        acc[j] += ms;
      }
  }
  std::vector<uint32_t> ok(n), ov(n);
  CK(hipMemcpy(ok.data(), k[0], n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ov.data(), v[0], n * 4, hipMemcpyDeviceToHost));
  bool good = true;
  for (uint32_t i = 1; i < n && good; i++)
    good = ok[i - 1] < ok[i] || (ok[i - 1] == ok[i] && ov[i - 1] < ov[i]);
  for (uint32_t i = 0; i < n && good; i++) good = hk[ov[i]] == ok[i];
  std::vector<unsigned long long> prof(ntiles * 8);
  CK(hipMemcpyFromSymbol(prof.data(), HIP_SYMBOL(g_os_prof), ntiles * 8 * 8));
  unsigned long long t0 = ~0ull, tend = 0;
  double rank = 0, look = 0, scat = 0;
  for (uint32_t t = 0; t < ntiles; t++) {
    const unsigned long long* p = &prof[t * 8];
    t0 = std::min(t0, p[0]);
    tend = std::max(tend, p[3]);
    rank += p[1] - p[0];
    look += p[2] - p[1];
    scat += p[3] - p[2];
  }
  unsigned long long last_start = 0;
  for (uint32_t t = 0; t < ntiles; t++) last_start = std::max(last_start, prof[t * 8] - t0);
  const double us = 1.0 / 100.0;  // wall_clock64 at 100 MHz
  printf("items %u waves %u tile %u tiles %u | hist %.1f us, passes %.1f %.1f %.1f %.1f us | sorted+stable %s\n",
         OS_ITEMS, OS_WAVES, OS_TILE, ntiles, acc[0] * 1e3 / (iters - 2), acc[1] * 1e3 / (iters - 2),
         acc[2] * 1e3 / (iters - 2), acc[3] * 1e3 / (iters - 2), acc[4] * 1e3 / (iters - 2), good ? "yes" : "NO");
  printf("  last pass per tile: load+rank %.2f us, publish+lookback %.2f us, scatter %.2f us; last tile start "
         "+%.2f us; span %.2f us\n",
         rank / ntiles * us, look / ntiles * us, scat / ntiles * us, last_start * us, (tend - t0) * us);
  return good ? 0 : 2;
}
