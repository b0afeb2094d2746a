// Micro-test: the accumulator layout of v_mfma_f64_16x16x4f64 (which (row, col) each lane's 4 values hold).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void k(double* out) {
  const int l = threadIdx.x;
  const int i = l % 16, kk = l / 16;                 // A: row i, k
  const double a = kk == 0 ? (double)(i + 1) : 0.0;  // A[i][0] = i + 1
  const double b = kk == 0 ? (double)(1000 + (l % 16)) : 0.0;  // B[0][j] = 1000 + j  (if B: k = l/16, j = l%16)
  v4d acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int v = 0; v < 4; ++v) out[l * 4 + v] = acc[v];
}
int main() {
  double* d; double h[256];
  (void)hipMalloc(&d, 256 * 8);
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, 256 * 8, hipMemcpyDeviceToHost);
  for (int l : {0, 1, 15, 16, 17, 32, 48, 63}) {
    printf("lane %2d:", l);
    for (int v = 0; v < 4; ++v) {
      const double x = h[l * 4 + v];
      // x = (row+1) * (1000 + col)
      int col = -1, row = -1;
      for (int c = 0; c < 16; ++c) { double r = x / (1000 + c); if (r == (int)r && r >= 1 && r <= 16) { col = c; row = (int)r - 1; } }
      printf("  v%d=(r%d,c%d)", v, row, col);
    }
    printf("\n");
  }
  return 0;
}
