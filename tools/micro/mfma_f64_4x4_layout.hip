// Micro-test: the operand and accumulator layouts of v_mfma_f64_4x4x4_4b_f64 (4 blocks of 4×4×4 per instruction, one
// f64 per lane for A, B and C).  Workgroup (La, Lb) puts a 1 in lane La of A and lane Lb of B only: C is non-zero in
// one lane exactly when A's (block, k) equals B's, and that lane is C's (block, i of La, j of Lb).  Prints, per A lane,
// the B lanes that pair with it and the C lane hit; then checks the layout the engine assumes.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const int l = threadIdx.x, La = blockIdx.x / 64, Lb = blockIdx.x % 64;
  const double a = l == La ? 1.0 : 0.0, b = l == Lb ? 1.0 : 0.0;
  double c = 0.0;
  c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
  const unsigned long long m = __ballot(c != 0.0);
  int hit = -1, n = 0;
  for (int q = 0; q < 64; ++q)
    if ((m >> q) & 1ull) { hit = q; ++n; }
  if (l == 0) out[blockIdx.x] = n > 1 ? -2 : hit;
}
int main() {
  int* d;
  int h[4096];
  (void)hipMalloc(&d, sizeof h);
  k<<<4096, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int La = 0; La < 64; ++La) {
    printf("A lane %2d:", La);
    for (int Lb = 0; Lb < 64; ++Lb)
      if (h[La * 64 + Lb] != -1) printf(" B%d->C%d", Lb, h[La * 64 + Lb]);
    printf("\n");
  }
  // hypothesis: block = l/16; A: i = l%4, k = (l/4)%4; B: j = l%4, k = (l/4)%4; C: i = (l/4)%4, j = l%4
  int bad = 0;
  for (int La = 0; La < 64; ++La)
    for (int Lb = 0; Lb < 64; ++Lb) {
      const bool pair = La / 16 == Lb / 16 && (La / 4) % 4 == (Lb / 4) % 4;
      const int want = pair ? (La / 16) * 16 + (La % 4) * 4 + (Lb % 4) : -1;
      bad += h[La * 64 + Lb] != want;
    }
  printf("hypothesis (block l/16; A i=l%%4 k=(l/4)%%4; B j=l%%4 k=(l/4)%%4; C i=(l/4)%%4 j=l%%4): %s (%d mismatches)\n",
         bad ? "WRONG" : "OK", bad);
  return 0;
}
