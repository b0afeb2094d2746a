// The chip's streaming rate for bench.py's roofline context (libstream_copy.so, loaded with ctypes): a hand-written
// 16-B copy kernel — float4 loads, non-temporal float4 stores, four independent 16-B moves per lane per iteration —
// over a buffer far larger than the 256-MB MALL, at several grid sizes; the best rate (2 × bytes per copy: read +
// write) is MI355X_MICROARCH.md's "float4 copy" figure measured on the box the bench runs on.  A measurement aid, not
// part of the engine: bench.py's `roofline.stream_copy_*` fields only.
#include <hip/hip_runtime.h>

#include <cstddef>

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

__global__ __launch_bounds__(256) void copy_nt_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                      long long n) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const f32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(src[i], dst + i);
}

__global__ __launch_bounds__(256) void fill_kernel(f32x4* __restrict__ dst, long long n) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    dst[i] = f32x4{1.0f, 2.0f, 3.0f, (float)(i & 255)};
}

}  // namespace

extern "C" {

// Best copy rate in GB/s (read + write bytes ÷ time, the best of `reps` timed launches per grid size after 3 untimed)
// over a `bytes`-byte buffer; *best_grid receives the workgroup count that achieved it.  Returns 0 on success, a HIP
// error code otherwise.  Uses the current device and the null stream.
int stream_copy_gbs(size_t bytes, int reps, double* gbs, int* best_grid) {
  const long long n = (long long)(bytes / 16);
  f32x4 *a = nullptr, *b = nullptr;
  hipError_t err = hipMalloc(&a, (size_t)n * 16);
  if (err != hipSuccess) return (int)err;
  err = hipMalloc(&b, (size_t)n * 16);
  if (err != hipSuccess) {
    (void)hipFree(a);
    return (int)err;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  fill_kernel<<<4096, 256>>>(a, n);
  double best = 0.0;
  int bg = 0;
  const int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (int g : grids) {
    for (int i = 0; i < 3; ++i) copy_nt_kernel<<<g, 256>>>(a, b, n);
    for (int r = 0; r < reps; ++r) {
      (void)hipEventRecord(e0, nullptr);
      copy_nt_kernel<<<g, 256>>>(a, b, n);
      (void)hipEventRecord(e1, nullptr);
      err = hipEventSynchronize(e1);
      if (err != hipSuccess) break;
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double r_gbs = 2.0 * (double)n * 16.0 / (ms * 1e-3) / 1e9;
      if (r_gbs > best) {
        best = r_gbs;
        bg = g;
      }
    }
    if (err != hipSuccess) break;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(a);
  (void)hipFree(b);
  if (err != hipSuccess) return (int)err;
  *gbs = best;
  if (best_grid) *best_grid = bg;
  return 0;
}

}  // extern "C"
