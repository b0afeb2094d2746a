// Micro-test: issue cost of v_mfma_f64_4x4x4_4b_f64 against v_mfma_f64_16x16x4_f64 — cycles per instruction of one wave
// with four independent accumulator chains (throughput) and with one chain (latency), by wall_clock64 (100 MHz) and
// clock64 (shader cycles) around 4096 instructions.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
template <int KIND, int CH>
__global__ void k(double* out, long long* cyc) {
  const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  double c1[CH];
  v4d c4[CH];
  for (int i = 0; i < CH; ++i) { c1[i] = 0.0; c4[i] = v4d{0, 0, 0, 0}; }
  const long long t0 = clock64();
  for (int it = 0; it < 4096 / CH; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (KIND == 0) c1[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1[i], 0, 0, 0);
      else c4[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c4[i], 0, 0, 0);
    }
  }
  double s = 0.0;
  for (int i = 0; i < CH; ++i) s += c1[i] + c4[i][0] + c4[i][3];
  const long long t1 = clock64();
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  double* d;
  long long* c;
  long long h;
  (void)hipMalloc(&d, 64 * 8);
  (void)hipMalloc(&c, 8);
#define RUN(K, CH, name)                                                              \
  k<K, CH><<<1, 64>>>(d, c);                                                          \
  k<K, CH><<<1, 64>>>(d, c);                                                          \
  (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);                                   \
  printf("%-28s chains %d: %.1f cycles per instruction\n", name, CH, (double)h / 4096.0);
  RUN(0, 1, "f64 4x4x4_4b");
  RUN(0, 4, "f64 4x4x4_4b");
  RUN(0, 8, "f64 4x4x4_4b");
  RUN(1, 1, "f64 16x16x4");
  RUN(1, 4, "f64 16x16x4");
  return 0;
}
