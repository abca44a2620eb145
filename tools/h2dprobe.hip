// h2dprobe — what a host-fed batch's input copy costs the submitting thread
// and the link. For a 29-MB page-locked
// buffer (the C1 prefix-shared batch) it times, over REPS copies:
//   host_us  the hipMemcpyAsync call itself (the submitter's time),
//   gbps     bytes / (event end - event start) on the copy stream,
// for: one copy; the same split in 2 / 4 / 8 chunks; the same from a copy
// thread (the submitter only enqueues); hipHostMalloc flags (default,
// non-coherent, write-combined, NUMA-user); and a kernel pulling the bytes
// through the mapped pointer (vector loads over PCIe).
//
//   hipcc -O3 --offload-arch=gfx950 tools/h2dprobe.hip -o build_tools/h2dprobe
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

struct Result {
  double host_us, dev_us;
};

// REPS copies of `bytes` split in `chunks`, on stream st; returns the average
// host time per batch (all chunks' calls) and device time per batch.
static Result run_copies(void* dst, const void* src, size_t bytes, int chunks, hipStream_t st, int reps) {
  std::vector<hipEvent_t> e0(reps), e1(reps);
  for (int r = 0; r < reps; r++) {
    CK(hipEventCreate(&e0[r]));
    CK(hipEventCreate(&e1[r]));
  }
  CK(hipStreamSynchronize(st));
  double host = 0;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(e0[r], st));
    const double t0 = now_us();
    const size_t c = (bytes / chunks + 4095) & ~(size_t)4095;
    for (size_t off = 0; off < bytes; off += c)
      CK(hipMemcpyAsync((char*)dst + off, (const char*)src + off, off + c > bytes ? bytes - off : c,
                        hipMemcpyHostToDevice, st));
    host += now_us() - t0;
    CK(hipEventRecord(e1[r], st));
  }
  CK(hipStreamSynchronize(st));
  double dev = 0;
  for (int r = 0; r < reps; r++) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0[r], e1[r]));
    dev += ms * 1000.0;
    CK(hipEventDestroy(e0[r]));
    CK(hipEventDestroy(e1[r]));
  }
  return {host / reps, dev / reps};
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : 29u << 20;
  const int reps = 30;
  void* d = nullptr;
  CK(hipMalloc(&d, bytes + 4096));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct Flag {
    const char* name;
    unsigned f;
  } flags[] = {{"default", hipHostMallocDefault},
               {"noncoherent", hipHostMallocNonCoherent},
               {"writecombined", hipHostMallocWriteCombined},
               {"numauser", hipHostMallocNumaUser}};
  for (const Flag& fl : flags) {
    void* h = nullptr;
    if (hipHostMalloc(&h, bytes, fl.f) != hipSuccess) {
      printf("%-14s hipHostMalloc failed\n", fl.name);
      (void)hipGetLastError();
      continue;
    }
    memset(h, 1, bytes);
    run_copies(d, h, bytes, 1, st, 3);  // warm
    for (int chunks : {1, 2, 4, 8}) {
      const Result r = run_copies(d, h, bytes, chunks, st, reps);
      printf("%-14s chunks %d  host %7.1f us  device %7.1f us  %6.1f GB/s\n", fl.name, chunks, r.host_us, r.dev_us,
             bytes / r.dev_us / 1e3);
    }
    // a copy thread: the submitter hands the batch over and returns
    {
      std::mutex mu;
      std::condition_variable cv;
      int pending = 0;
      bool stop = false;
      std::thread th([&] {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
          cv.wait(lk, [&] { return pending > 0 || stop; });
          if (!pending && stop) return;
          pending--;
          lk.unlock();
          CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
          lk.lock();
        }
      });
      CK(hipStreamSynchronize(st));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, st));
      double host = 0;
      const double t0 = now_us();
      for (int r = 0; r < reps; r++) {
        const double s0 = now_us();
        {
          std::lock_guard<std::mutex> g(mu);
          pending++;
        }
        cv.notify_one();
        host += now_us() - s0;
      }
      {
        std::lock_guard<std::mutex> g(mu);
        stop = true;
      }
      cv.notify_one();
      th.join();
      CK(hipEventRecord(b, st));
      CK(hipStreamSynchronize(st));
      const double wall = now_us() - t0;
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("%-14s thread    host %7.1f us  device %7.1f us  %6.1f GB/s (wall %.1f us per copy)\n", fl.name,
             host / reps, ms * 1000.0 / reps, bytes * (double)reps / (ms * 1e6), wall / reps);
      CK(hipEventDestroy(a));
      CK(hipEventDestroy(b));
    }
    // a kernel pulling the bytes through the mapped pointer
    {
      void* hd = nullptr;
      if (hipHostGetDevicePointer(&hd, h, 0) == hipSuccess && hd) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int grid : {256, 1024, 4096}) {
          k_pull<<<grid, 256, 0, st>>>((const uint4*)hd, (uint4*)d, bytes / 16);
          CK(hipEventRecord(a, st));
          const double t0 = now_us();
          for (int r = 0; r < reps; r++) k_pull<<<grid, 256, 0, st>>>((const uint4*)hd, (uint4*)d, bytes / 16);
          const double host = (now_us() - t0) / reps;
          CK(hipEventRecord(b, st));
          CK(hipStreamSynchronize(st));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, a, b));
          printf("%-14s pull %4d host %7.1f us  device %7.1f us  %6.1f GB/s\n", fl.name, grid, host,
                 ms * 1000.0 / reps, bytes * (double)reps / (ms * 1e6));
        }
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
      } else {
        (void)hipGetLastError();
      }
    }
    CK(hipHostFree(h));
  }
  CK(hipFree(d));
  return 0;
}
