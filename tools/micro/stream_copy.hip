// The chip's streaming rate for bench.py's roofline context (libstream_copy.so, loaded with ctypes): hand-written 16-B
// copy kernels — float4 loads and stores, 1, 2 or 4 independent moves per lane per iteration, default or non-temporal
// policies — over a buffer far larger than the 256-MB MALL, at several grid sizes; the best rate (2 × bytes per copy: read +
// write) is MI355X_MICROARCH.md's "float4 copy" figure measured on the box the bench runs on.  A measurement aid, not
// part of the engine: bench.py's `roofline.stream_copy_*` fields only.
#include <hip/hip_runtime.h>

#include <cstddef>

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

// U independent 16-B moves per lane per iteration of a grid-stride loop; NTS / NTL: non-temporal stores / loads.
template <int U, bool NTS, bool NTL>
__global__ __launch_bounds__(256) void copy_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst, long long n) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) {
    const f32x4 v = NTL ? __builtin_nontemporal_load(src + i) : src[i];
    if (NTS) __builtin_nontemporal_store(v, dst + i);
    else dst[i] = v;
  }
}

__global__ __launch_bounds__(256) void fill_kernel(f32x4* __restrict__ dst, long long n) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    dst[i] = f32x4{1.0f, 2.0f, 3.0f, (float)(i & 255)};
}

typedef void (*copy_fn)(const f32x4*, f32x4*, long long);

}  // namespace

extern "C" {

// Best copy rate in GB/s (read + write bytes ÷ time, the best of `reps` timed launches per grid size after 3 untimed)
// over a `bytes`-byte buffer; *best_grid receives the workgroup count that achieved it.  Returns 0 on success, a HIP
// error code otherwise.  Uses the current device and the null stream.  *best_grid = workgroups × 100 + form index
// (forms: see the table below).
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
  // forms: (U, stores, loads); grids: a few waves of the chip up to one 16-B move per lane (n / 256)
  struct Form { copy_fn f; int u; };
  const Form forms[] = {{copy_kernel<1, true, false>, 1}, {copy_kernel<2, true, false>, 2}, {copy_kernel<4, true, false>, 4},
                        {copy_kernel<1, false, false>, 1}, {copy_kernel<4, false, false>, 4},
                        {copy_kernel<1, true, true>, 1}, {copy_kernel<4, true, true>, 4}};
  const long long grids[] = {2048, 8192, 32768, 0};
  for (int fi = 0; fi < (int)(sizeof(forms) / sizeof(forms[0])) && err == hipSuccess; ++fi) {
    for (long long g0 : grids) {
      const long long g = g0 ? g0 : (n + 256LL * forms[fi].u - 1) / (256LL * forms[fi].u);
      for (int i = 0; i < 2; ++i) forms[fi].f<<<(unsigned)g, 256>>>(a, b, n);
      for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(e0, nullptr);
        forms[fi].f<<<(unsigned)g, 256>>>(a, b, n);
        (void)hipEventRecord(e1, nullptr);
        err = hipEventSynchronize(e1);
        if (err != hipSuccess) break;
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double r_gbs = 2.0 * (double)n * 16.0 / (ms * 1e-3) / 1e9;
        if (r_gbs > best) {
          best = r_gbs;
          bg = (int)(g * 100 + fi);  // grid × 100 + form index
        }
      }
      if (err != hipSuccess) break;
    }
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
