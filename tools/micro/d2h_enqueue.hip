// Diagnostic: how long the host spends INSIDE the enqueue of a device → page-locked host copy (hipMemcpyAsync vs a copy
// kernel into the mapped buffer), for the Ceres adapter's record read-back (45 MB at the C4 sample).
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/d2h_enqueue tools/micro/d2h_enqueue.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void copyk(const uint4* s, uint4* d, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) d[i] = s[i];
}
static double now() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t bytes = 45u << 20;
  void *d = nullptr, *h1 = nullptr, *h2 = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 1, bytes));
  CK(hipHostMalloc(&h1, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&h2, bytes, hipHostMallocMapped | hipHostMallocPortable));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int rep = 0; rep < 3; ++rep) {
    for (int which = 0; which < 2; ++which) {
      void* h = which ? h2 : h1;
      void* dd = nullptr;
      const double t0 = now();
      hipError_t q = hipHostGetDevicePointer(&dd, h, 0);
      const double t1 = now();
      (void)hipGetLastError();
      // 11 chunks of the record read-back
      const size_t ch = bytes / 11 & ~(size_t)15;
      for (int c = 0; c < 11; ++c) CK(hipMemcpyAsync((char*)h + c * ch, (char*)d + c * ch, ch, hipMemcpyDeviceToHost, st));
      const double t2 = now();
      CK(hipStreamSynchronize(st));
      const double t3 = now();
      double t4 = t3, t5 = t3;
      if (q == hipSuccess && dd) {
        for (int c = 0; c < 11; ++c) {
          copyk<<<1024, 256, 0, st>>>((const uint4*)((char*)d + c * ch), (uint4*)((char*)dd + c * ch), ch / 16);
          CK(hipEventRecord(ev, st));
        }
        t4 = now();
        CK(hipStreamSynchronize(st));
        t5 = now();
      }
      printf("rep %d %s: getdeviceptr %s %.1f us | memcpyAsync x11 enqueue %.1f us, drain %.1f us | kernel x11 enqueue %.1f us, drain %.1f us\n",
             rep, which ? "mapped" : "default", q == hipSuccess ? "ok" : hipGetErrorString(q), t1 - t0, t2 - t1, t3 - t2,
             t4 - t3, t5 - t4);
    }
  }
  return 0;
}
