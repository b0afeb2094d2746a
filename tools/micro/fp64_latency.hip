// Micro-benchmark: dependent-chain latency and independent-chain issue rate of v_fma_f64 / v_fma_f32 and
// ds_read_b64 broadcast latency for ONE wave (s_memtime cycles).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
template <class T, int CH>
__global__ void chain(T* out, T a, T b, long long* cyc, int n) {
  T v[CH];
  for (int c = 0; c < CH; ++c) v[c] = (T)threadIdx.x + c;
  long long t0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) v[c] = v[c] * a + b;
  }
  long long t1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0 && CH == 16) printf("clock64 %lld cycles in %lld wall ticks (100 MHz) -> %.2f GHz\n", t1 - t0, w1 - w0, (double)(t1 - t0) / ((w1 - w0) * 10.0));
  T s = 0;
  for (int c = 0; c < CH; ++c) s += v[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
// all-VGPR operands: v[c] -= x[c] * t0 + y[c] * t1 (the Gauss-Jordan update shape), 24 rows
__global__ void gj_shape(double* out, long long* cyc, int n) {
  double v[24], x[24], y[24];
  for (int c = 0; c < 24; ++c) { v[c] = threadIdx.x + c; x[c] = 1e-3 * c; y[c] = 2e-3 * c; }
  double t0 = 0.5 + threadIdx.x * 1e-3, t1 = 0.25;
  long long t_0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int c = 0; c < 24; ++c) v[c] = v[c] - x[c] * t0 - y[c] * t1;
    t0 = v[3] * 1e-9 + 0.5;  // step dependence like the next pivot
  }
  long long t_1 = clock64();
  double s = 0;
  for (int c = 0; c < 24; ++c) s += v[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t_1 - t_0;
}
// 24 broadcast ds_read_b128 + the 48-fma update per step (the Gauss-Jordan step without the pivot chain)
template <bool BCAST>
__global__ void lds_gj(double* out, long long* cyc, int n) {
  __shared__ double2 buf[64 * 24];
  for (int q = threadIdx.x; q < 64 * 24; q += 64) buf[q] = make_double2(1e-3 * q, 2e-3 * q);
  __syncthreads();
  double v[24];
  for (int c = 0; c < 24; ++c) v[c] = threadIdx.x + c;
  double t0 = 0.5 + threadIdx.x * 1e-3, t1 = 0.25;
  int base = 0;
  long long t_0 = clock64();
  for (int i = 0; i < n; ++i) {
    double2 cr[24];
#pragma unroll
    for (int c = 0; c < 24; ++c) cr[c] = buf[base + (BCAST ? c : c * 64 + (int)threadIdx.x) % (64 * 24)];
#pragma unroll
    for (int c = 0; c < 24; ++c) v[c] = v[c] - cr[c].x * t0 - cr[c].y * t1;
    t0 = v[3] * 1e-9 + 0.5;
    base = (base + 24) & 511;
  }
  long long t_1 = clock64();
  double s = 0;
  for (int c = 0; c < 24; ++c) s += v[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t_1 - t_0;
}
__device__ __forceinline__ double rl(double v, int l) {
  int2 p = __builtin_bit_cast(int2, v);
  p.x = __builtin_amdgcn_readlane(p.x, l);
  p.y = __builtin_amdgcn_readlane(p.y, l);
  return __builtin_bit_cast(double, p);
}
// pivot columns broadcast from lanes k, k+1 with v_readlane (SGPR operands) + the 48-fma update
__global__ void readlane_gj(double* out, long long* cyc, int n) {
  double v[24];
  for (int c = 0; c < 24; ++c) v[c] = threadIdx.x + c * 1e-3;
  double t0 = 0.5 + threadIdx.x * 1e-3, t1 = 0.25;
  long long t_0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      double c0[24], c1[24];
#pragma unroll
      for (int r = 0; r < 24; ++r) {
        c0[r] = rl(v[r], k);
        c1[r] = rl(v[r], k + 1);
      }
#pragma unroll
      for (int r = 0; r < 24; ++r) v[r] = v[r] - c0[r] * t0 - c1[r] * t1;
      t0 = v[3] * 1e-9 + 0.5;
    }
  }
  long long t_1 = clock64();
  double s = 0;
  for (int c = 0; c < 24; ++c) s += v[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t_1 - t_0;
}
__global__ void lds_lat(double* out, long long* cyc, int n) {
  __shared__ double buf[256];
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  int idx = 0;
  double acc = 0;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    const double v = buf[idx];
    acc += v;
    idx = ((int)v + 1) & 63;  // dependent address
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  double* od; float* of; long long* cyc; long long h;
  hipMalloc(&od, 256 * 8); hipMalloc(&of, 256 * 4); hipMalloc(&cyc, 8);
  const int n = 1000;
#define RUN(T, CH, O)                                                                                        \
  chain<T, CH><<<1, 64>>>(O, (T)0.999, (T)0.001, cyc, n); hipDeviceSynchronize();                             \
  chain<T, CH><<<1, 64>>>(O, (T)0.999, (T)0.001, cyc, n); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);        \
  printf("%-6s chains=%d: %.2f cycles per fma (per chain step %.2f)\n", #T, CH, (double)h / (n * 16.0 * CH), (double)h / (n * 16.0));
  RUN(double, 1, od) RUN(double, 2, od) RUN(double, 4, od) RUN(double, 8, od) RUN(double, 16, od)
  RUN(float, 1, of) RUN(float, 4, of) RUN(float, 16, of)
  gj_shape<<<1, 64>>>(od, cyc, n); hipDeviceSynchronize();
  gj_shape<<<1, 64>>>(od, cyc, n); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("GJ-shaped update (48 fma, all-VGPR operands): %.1f cycles per step\n", (double)h / n);
  lds_gj<true><<<1, 64>>>(od, cyc, n); hipDeviceSynchronize();
  lds_gj<true><<<1, 64>>>(od, cyc, n); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("24 broadcast ds_read_b128 + 48 fma: %.1f cycles per step\n", (double)h / n);
  lds_gj<false><<<1, 64>>>(od, cyc, n); hipDeviceSynchronize();
  lds_gj<false><<<1, 64>>>(od, cyc, n); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("24 per-lane ds_read_b128 + 48 fma: %.1f cycles per step\n", (double)h / n);
  readlane_gj<<<1, 64>>>(od, cyc, n); hipDeviceSynchronize();
  readlane_gj<<<1, 64>>>(od, cyc, n); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("96 v_readlane + 48 fma: %.1f cycles per step\n", (double)h / (2 * n));
  lds_lat<<<1, 64>>>(od, cyc, n); hipDeviceSynchronize();
  lds_lat<<<1, 64>>>(od, cyc, n); hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("ds_read_b64 dependent latency: %.1f cycles\n", (double)h / n);
  return 0;
}
