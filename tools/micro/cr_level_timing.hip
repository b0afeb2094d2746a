// Micro-benchmark: one cyclic-reduction level (the structure of cr_level_kernel, pba_gn.hip) on a synthetic SPD
// block-tridiagonal level, with wall_clock64 phase stamps (load | Gauss-Jordan | products).  Diagnostic only:
// not part of the library.  Build: hipcc -O3 --offload-arch=gfx950 -I../../photometric-bundle-adjustment_amd/csrc
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pba_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
using pba::rcp_nr;

struct CrLevel { double *D, *U, *b, *X, *x; int n; };

template <int M>
constexpr int kT = ((3 * M + 1) + 63) / 64 * 64;

template <int M, bool ST>
__device__ __forceinline__ bool gj_row(const CrLevel& L, int j, int tid, double (*colk)[2][M], double* a, long long* st) {
  constexpr int NC = 2 * M + 1, W = M + NC;
  const int c = min(tid, W - 1);
  const double* D = L.D + (long long)j * M * M;
#pragma unroll
  for (int r = 0; r < M; ++r) {
    const double* src;
    if (c < M) src = D + r * M + c;
    else if (c < 2 * M) src = L.U + (long long)(j - 1) * M * M + (c - M) * M + r;
    else if (c < 3 * M) src = (j + 1 < L.n) ? L.U + (long long)j * M * M + r * M + (c - 2 * M) : nullptr;
    else src = L.b + (long long)j * M + r;
    a[r] = src ? *src : 0.0;
  }
  if (ST) {
    double s = 0;
#pragma unroll
    for (int r = 0; r < M; ++r) s += a[r];
    if (s == 12345.678) a[0] = 0;  // force the loads to land before the stamp
    st[1] = wall_clock64();
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < M; k += 2) {
    const int buf = (k >> 1) & 1;
    if (tid == k || tid == k + 1) {
      double* dst = colk[buf][tid - k];
#pragma unroll
      for (int r = 0; r < M; ++r) dst[r] = a[r];
    }
    __syncthreads();
    const double* c0 = colk[buf][0];
    const double* c1 = colk[buf][1];
    const double p00 = c0[k], p10 = c0[k + 1], p01 = c1[k], p11 = c1[k + 1];
    const double det = p00 * p11 - p01 * p10;
    bad |= !(p00 > 0.0 && det > 0.0);
    const double rd = rcp_nr(det);
    const double ak = a[k], ak1 = a[k + 1];
    const double t0 = (p11 * ak - p01 * ak1) * rd;
    const double t1 = (p00 * ak1 - p10 * ak) * rd;
#pragma unroll
    for (int r = 0; r < M; ++r) a[r] = r == k ? t0 : (r == k + 1 ? t1 : a[r] - c0[r] * t0 - c1[r] * t1);
  }
  return !bad;
}

template <int M, bool ST>
__global__ __launch_bounds__(2 * kT<M>) void level(CrLevel L, CrLevel Ln, int* status, long long* stamps) {
  constexpr int NC = 2 * M + 1, W = M + NC, T = kT<M>;
  __shared__ __attribute__((aligned(16))) double colk[2][2][2][M];
  extern __shared__ double smem[];
  double* sUl = smem;
  double* sUi = sUl + M * M;
  double* sX[2] = {sUi + M * M, sUi + M * M + M * NC};
  long long st[5];
  st[0] = wall_clock64();
  const int i = 2 * blockIdx.x, in = blockIdx.x;
  const int half = threadIdx.x >= T ? 1 : 0, tl = threadIdx.x - half * T;
  const int j = half ? i + 1 : i - 1;
  const bool has = j >= 0 && j < L.n;
  double a[M];
  const bool ok = gj_row<M, ST>(L, has ? j : 1, tl, colk[half], a, st);
  if (!ok && has && tl == 0) atomicOr(status, 1);
  if (ST) st[2] = wall_clock64();
  if (tl >= M && tl < W) {
    double* x = sX[half] + (tl - M);
#pragma unroll
    for (int r = 0; r < M; ++r) x[r * NC] = has ? a[r] : 0.0;
    if (half && has) {
      double* X = L.X + (long long)(j / 2) * M * NC + (tl - M);
#pragma unroll
      for (int r = 0; r < M; ++r) X[r * NC] = a[r];
    }
  }
  const bool left = i - 1 >= 0, right = i + 1 < L.n;
  for (int e = threadIdx.x; e < M * M; e += 2 * T) {
    sUl[e] = left ? L.U[(long long)(i - 1) * M * M + e] : 0.0;
    sUi[e] = L.U[(long long)i * M * M + e];
  }
  __syncthreads();
  if (ST) st[3] = wall_clock64();
  const double* sXl = sX[0];
  const double* sXr = sX[1];
  for (int e = threadIdx.x; e < 2 * M * M + M; e += 2 * T) {
    if (e < M * M) {
      const int r = e / M, c = e % M;
      double v = L.D[(long long)i * M * M + e];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + M + c] + sUi[r * M + q] * sXr[q * NC + c];
      Ln.D[(long long)in * M * M + e] = v;
    } else if (e < 2 * M * M) {
      const int f = e - M * M, r = f / M, c = f % M;
      double v = 0.0;
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUi[r * M + q] * sXr[q * NC + M + c];
      Ln.U[(long long)in * M * M + f] = right ? v : 0.0;
    } else {
      const int r = e - 2 * M * M;
      double v = L.b[(long long)i * M + r];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + 2 * M] + sUi[r * M + q] * sXr[q * NC + 2 * M];
      Ln.b[(long long)in * M + r] = v;
    }
  }
  if (ST) {
    __syncthreads();
    st[4] = wall_clock64();
    if (threadIdx.x == 0)
      for (int q = 0; q < 5; ++q) stamps[blockIdx.x * 5 + q] = st[q];
  }
}

// V1: U_{i-1}, U_i, D_i, b_i for the products are loaded at kernel start (in flight with the Gauss-Jordan
// column loads) and parked in LDS; the product loop then reads only LDS.
template <int M, bool ST>
__global__ __launch_bounds__(2 * kT<M>) void level1(CrLevel L, CrLevel Ln, int* status, long long* stamps) {
  constexpr int NC = 2 * M + 1, W = M + NC, T = kT<M>, NT = 2 * T;
  constexpr int NPRE = (3 * M * M + M + NT - 1) / NT;  // per-thread share of U_{i-1}, U_i, D_i, b_i
  __shared__ __attribute__((aligned(16))) double colk[2][2][2][M];
  extern __shared__ double smem[];
  double* sUl = smem;
  double* sUi = sUl + M * M;
  double* sD = sUi + M * M;
  double* sb = sD + M * M;
  double* sX[2] = {sb + M, sb + M + M * NC};
  long long st[5];
  st[0] = wall_clock64();
  const int i = 2 * blockIdx.x, in = blockIdx.x;
  const bool left = i - 1 >= 0, right = i + 1 < L.n;
  double pre[NPRE];
#pragma unroll
  for (int u = 0; u < NPRE; ++u) {
    const int e = threadIdx.x + u * NT;
    const double* src = nullptr;
    if (e < M * M) src = left ? L.U + (long long)(i - 1) * M * M + e : nullptr;
    else if (e < 2 * M * M) src = L.U + (long long)i * M * M + (e - M * M);
    else if (e < 3 * M * M) src = L.D + (long long)i * M * M + (e - 2 * M * M);
    else if (e < 3 * M * M + M) src = L.b + (long long)i * M + (e - 3 * M * M);
    pre[u] = src ? *src : 0.0;
  }
  const int half = threadIdx.x >= T ? 1 : 0, tl = threadIdx.x - half * T;
  const int j = half ? i + 1 : i - 1;
  const bool has = j >= 0 && j < L.n;
  double a[M];
  // park the product operands (their loads were issued first; gj_row's loads follow)
#pragma unroll
  for (int u = 0; u < NPRE; ++u) {
    const int e = threadIdx.x + u * NT;
    if (e < 3 * M * M + M) smem[e] = pre[u];
  }
  const bool ok = gj_row<M, ST>(L, has ? j : 1, tl, colk[half], a, st);
  if (!ok && has && tl == 0) atomicOr(status, 1);
  if (ST) st[2] = wall_clock64();
  if (tl >= M && tl < W) {
    double* x = sX[half] + (tl - M);
#pragma unroll
    for (int r = 0; r < M; ++r) x[r * NC] = has ? a[r] : 0.0;
    if (half && has) {
      double* X = L.X + (long long)(j / 2) * M * NC + (tl - M);
#pragma unroll
      for (int r = 0; r < M; ++r) X[r * NC] = a[r];
    }
  }
  __syncthreads();
  if (ST) st[3] = wall_clock64();
  const double* sXl = sX[0];
  const double* sXr = sX[1];
  for (int e = threadIdx.x; e < 2 * M * M + M; e += NT) {
    if (e < M * M) {
      const int r = e / M, c = e % M;
      double v = sD[e];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + M + c] + sUi[r * M + q] * sXr[q * NC + c];
      Ln.D[(long long)in * M * M + e] = v;
    } else if (e < 2 * M * M) {
      const int f = e - M * M, r = f / M, c = f % M;
      double v = 0.0;
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUi[r * M + q] * sXr[q * NC + M + c];
      Ln.U[(long long)in * M * M + f] = right ? v : 0.0;
    } else {
      const int r = e - 2 * M * M;
      double v = sb[r];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + 2 * M] + sUi[r * M + q] * sXr[q * NC + 2 * M];
      Ln.b[(long long)in * M + r] = v;
    }
  }
  if (ST) {
    __syncthreads();
    st[4] = wall_clock64();
    if (threadIdx.x == 0)
      for (int q = 0; q < 5; ++q) stamps[blockIdx.x * 5 + q] = st[q];
  }
}

// V2: wave-level Gauss-Jordan.  Wave 0 eliminates row i−1 on [D | U_{i−1} | b] (49 columns), waves 1 and 2 row i+1
// on [D | U_iᵀ | b] and [D | U_{i+1}] — each wave keeps its own copy of D's columns, so the pivot columns are
// always in the same wave: published through a per-wave LDS buffer with no s_barrier (LDS ops of one wave are
// processed in order).  Wave 3 parks U_{i−1}, U_i, D_i, b_i in LDS for the products meanwhile.
__device__ long long g_step_clk[16];
template <int M, bool ST>
__device__ __forceinline__ bool gj_wave(const double* D, const double* R1, bool r1_trans, const double* R2, int ncol,
                                        int lane, double2* piv, double* a, long long* st) {
  // lane c < M: column c of D; M ≤ c < M + ncol: right-hand side column c − M (R1 columns, then R2)
  const int c = lane;
#pragma unroll
  for (int r = 0; r < M; ++r) {
    const double* src = nullptr;
    if (c < M) src = D + r * M + c;
    else if (c < 2 * M) src = R1 ? (r1_trans ? R1 + (c - M) * M + r : R1 + r * M + (c - M)) : nullptr;
    else if (c < M + ncol) src = R2 ? R2 + r : nullptr;  // b (one column)
    a[r] = src ? *src : 0.0;
  }
  if (ST) {
    double s = 0;
#pragma unroll
    for (int r = 0; r < M; ++r) s += a[r];
    if (s == 12345.678) a[0] = 0;
    st[1] = wall_clock64();
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < M; k += 2) {
    if (ST && blockIdx.x == 0 && threadIdx.x == 0) g_step_clk[k / 2] = clock64();
    if (c == k || c == k + 1) {
      double* dst = reinterpret_cast<double*>(piv) + (c - k);
#pragma unroll
      for (int r = 0; r < M; ++r) dst[2 * r] = a[r];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double2 cr[M];
#pragma unroll
    for (int r = 0; r < M; ++r) cr[r] = piv[r];  // all 24 broadcast reads in flight at once
    const double p00 = cr[k].x, p10 = cr[k + 1].x, p01 = cr[k].y, p11 = cr[k + 1].y;
    const double det = p00 * p11 - p01 * p10;
    bad |= !(p00 > 0.0 && det > 0.0);
    const double rd = rcp_nr(det);
    const double ak = a[k], ak1 = a[k + 1];
    const double t0 = (p11 * ak - p01 * ak1) * rd;
    const double t1 = (p00 * ak1 - p10 * ak) * rd;
#pragma unroll
    for (int r = 0; r < M; ++r) a[r] = r == k ? t0 : (r == k + 1 ? t1 : a[r] - cr[r].x * t0 - cr[r].y * t1);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  return !bad;
}

template <int M, bool ST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void level2(CrLevel L, CrLevel Ln, int* status, long long* stamps) {
  constexpr int NC = 2 * M + 1;
  __shared__ __attribute__((aligned(16))) double2 piv[3][M];
  extern __shared__ double smem[];
  double* sUl = smem;
  double* sUi = sUl + M * M;
  double* sD = sUi + M * M;
  double* sb = sD + M * M;
  double* sX[2] = {sb + M, sb + M + M * NC};
  long long st[5];
  st[0] = wall_clock64();
  const int i = 2 * blockIdx.x, in = blockIdx.x;
  const bool left = i - 1 >= 0, right = i + 1 < L.n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double a[M];
  if (w == 3) {  // park the product operands
    for (int e = lane; e < 3 * M * M + M; e += 64) {
      const double* src = nullptr;
      if (e < M * M) src = left ? L.U + (long long)(i - 1) * M * M + e : nullptr;
      else if (e < 2 * M * M) src = L.U + (long long)i * M * M + (e - M * M);
      else if (e < 3 * M * M) src = L.D + (long long)i * M * M + (e - 2 * M * M);
      else src = L.b + (long long)i * M + (e - 3 * M * M);
      smem[e] = src ? *src : 0.0;
    }
    if (ST) st[1] = wall_clock64();
  } else {
    const int j = w == 0 ? i - 1 : i + 1;
    const bool has = j >= 0 && j < L.n;
    const int jj = has ? j : 1;
    const double* D = L.D + (long long)jj * M * M;
    const double* bj = L.b + (long long)jj * M;
    bool ok;
    if (w == 0) ok = gj_wave<M, ST>(D, L.U + (long long)jj * M * M, false, bj, M + 1, lane, piv[0], a, st);  // [D|U_j|b]
    else if (w == 1) ok = gj_wave<M, ST>(D, L.U + (long long)(jj - 1) * M * M, true, bj, M + 1, lane, piv[1], a, st);  // [D|U_{j-1}^T|b]
    else ok = gj_wave<M, ST>(D, jj + 1 < L.n ? L.U + (long long)jj * M * M : nullptr, false, nullptr, M, lane, piv[2], a, st);
    if (!ok && has && lane == 0) atomicOr(status, 1);
    // X columns: w0 → X^U_{i−1} (cols M..2M−1) + X^b_{i−1} (2M); w1 → X^L_{i+1} (0..M−1) + X^b_{i+1}; w2 → X^U_{i+1}
    if (lane >= M && lane < 2 * M + (w == 2 ? 0 : 1)) {
      const int col = lane < 2 * M ? (w == 1 ? lane - M : lane) : 2 * M;
      double* x = sX[w == 0 ? 0 : 1] + col;
#pragma unroll
      for (int r = 0; r < M; ++r) x[r * NC] = has ? a[r] : 0.0;
      if (w != 0 && has) {
        double* X = L.X + (long long)(j / 2) * M * NC + col;
#pragma unroll
        for (int r = 0; r < M; ++r) X[r * NC] = a[r];
      }
    }
  }
  if (ST) st[2] = wall_clock64();
  __syncthreads();
  if (ST) st[3] = wall_clock64();
  const double* sXl = sX[0];
  const double* sXr = sX[1];
  for (int e = threadIdx.x; e < 2 * M * M + M; e += 256) {
    if (e < M * M) {
      const int r = e / M, c = e % M;
      double v = sD[e];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + M + c] + sUi[r * M + q] * sXr[q * NC + c];
      Ln.D[(long long)in * M * M + e] = v;
    } else if (e < 2 * M * M) {
      const int f = e - M * M, r = f / M, c = f % M;
      double v = 0.0;
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUi[r * M + q] * sXr[q * NC + M + c];
      Ln.U[(long long)in * M * M + f] = right ? v : 0.0;
    } else {
      const int r = e - 2 * M * M;
      double v = sb[r];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + 2 * M] + sUi[r * M + q] * sXr[q * NC + 2 * M];
      Ln.b[(long long)in * M + r] = v;
    }
  }
  if (ST) {
    __syncthreads();
    st[4] = wall_clock64();
    if (threadIdx.x == 0)
      for (int q = 0; q < 5; ++q) stamps[blockIdx.x * 5 + q] = st[q];
  }
}

// V3: two waves per elimination (rows 0-11 / 12-23 of every column), three eliminations per workgroup (row i−1 on
// [D|U_{i−1}|b], row i+1 on [D|U_iᵀ|b] and on [D|U_{i+1}]), 6 waves; per pivot pair one workgroup barrier with
// double-buffered pivot columns + pivot rows in LDS; products as 2×2 register tiles from LDS.
template <int M, int BASE>
__device__ __forceinline__ void gj3_step(int k, int lane, const double2* col, const double2* rowp, double* a,
                                         bool& bad) {
  constexpr int H = M / 2;
  const double2 pk = col[k], pk1 = col[k + 1];
  const double p00 = pk.x, p01 = pk.y, p10 = pk1.x, p11 = pk1.y;
  const double det = p00 * p11 - p01 * p10;
  bad |= !(p00 > 0.0 && det > 0.0);
  const double rd = rcp_nr(det);
  const double2 ar = rowp[lane];
  const double t0 = (p11 * ar.x - p01 * ar.y) * rd;
  const double t1 = (p00 * ar.y - p10 * ar.x) * rd;
  double2 cr[H];
#pragma unroll
  for (int q = 0; q < H; ++q) cr[q] = col[BASE + q];
#pragma unroll
  for (int q = 0; q < H; ++q) {
    const int r = BASE + q;
    a[q] = r == k ? t0 : (r == k + 1 ? t1 : a[q] - cr[q].x * t0 - cr[q].y * t1);
  }
}

template <int M, bool ST>
__global__ __launch_bounds__(384) void level3(CrLevel L, CrLevel Ln, int* status, long long* stamps) {
  constexpr int NC = 2 * M + 1, H = M / 2, NT = 384;
  constexpr int NPRE = (3 * M * M + M + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) double2 s_col[2][3][M];
  __shared__ __attribute__((aligned(16))) double2 s_row[2][3][64];
  extern __shared__ double smem[];
  double* sUl = smem;
  double* sUi = sUl + M * M;
  double* sD = sUi + M * M;
  double* sb = sD + M * M;
  double* sX[2] = {sb + M, sb + M + M * NC};
  long long st[5];
  st[0] = wall_clock64();
  const int i = 2 * blockIdx.x, in = blockIdx.x;
  const bool left = i - 1 >= 0, right = i + 1 < L.n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = w >> 1, hi = w & 1;  // elimination group, row half
  // product operands: loads issued first, parked in LDS after the column loads below are issued
  double pre[NPRE];
#pragma unroll
  for (int u = 0; u < NPRE; ++u) {
    const int e = threadIdx.x + u * NT;
    const double* src = nullptr;
    if (e < M * M) src = left ? L.U + (long long)(i - 1) * M * M + e : nullptr;
    else if (e < 2 * M * M) src = L.U + (long long)i * M * M + (e - M * M);
    else if (e < 3 * M * M) src = L.D + (long long)i * M * M + (e - 2 * M * M);
    else if (e < 3 * M * M + M) src = L.b + (long long)i * M + (e - 3 * M * M);
    pre[u] = src ? *src : 0.0;
  }
  const int j = g == 0 ? i - 1 : i + 1;
  const bool has = j >= 0 && j < L.n;
  const int jj = has ? j : 1;
  const double* D = L.D + (long long)jj * M * M;
  // columns: c < M: D; M ≤ c < 2M: g0 U_j, g1 U_{j−1}ᵀ, g2 U_j (if j+1 < n); c == 2M: b (g0, g1)
  const double* R1 = g == 1 ? L.U + (long long)(jj - 1) * M * M : (g == 0 || jj + 1 < L.n ? L.U + (long long)jj * M * M : nullptr);
  const bool r1t = g == 1;
  const int ncol = g == 2 ? 2 * M : 2 * M + 1;
  const int c = lane;
  double a[H];
#pragma unroll
  for (int q = 0; q < H; ++q) {
    const int r = hi * H + q;
    const double* src = nullptr;
    if (c < M) src = D + r * M + c;
    else if (c < 2 * M) src = R1 ? (r1t ? R1 + (c - M) * M + r : R1 + r * M + (c - M)) : nullptr;
    else if (c < ncol) src = L.b + (long long)jj * M + r;
    a[q] = src ? *src : 0.0;
  }
#pragma unroll
  for (int u = 0; u < NPRE; ++u) {
    const int e = threadIdx.x + u * NT;
    if (e < 3 * M * M + M) smem[e] = pre[u];
  }
  if (ST) {
    double s = 0;
#pragma unroll
    for (int q = 0; q < H; ++q) s += a[q];
    if (s == 12345.678) a[0] = 0;
    st[1] = wall_clock64();
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < M; k += 2) {
    const int buf = (k >> 1) & 1;
    double2* col = s_col[buf][g];
    double2* rowp = s_row[buf][g];
    // publish: lanes k, k+1 their column's rows; the owner half (rows k, k+1) every column's pivot-row pair
    if (c == k || c == k + 1) {
      double* dst = reinterpret_cast<double*>(col + hi * H) + (c - k);
#pragma unroll
      for (int q = 0; q < H; ++q) dst[2 * q] = a[q];
    }
    if (hi == (k >= H ? 1 : 0)) rowp[lane] = make_double2(a[k % H], a[k % H + 1]);
    __syncthreads();
    if (hi) gj3_step<M, H>(k, lane, col, rowp, a, bad);
    else gj3_step<M, 0>(k, lane, col, rowp, a, bad);
  }
  if (bad && has && lane == 0) atomicOr(status, 1);
  if (ST) st[2] = wall_clock64();
  // X columns: g0 → X^U_{i−1} (cols M..2M−1) + X^b_{i−1} (2M); g1 → X^L_{i+1} (0..M−1) + X^b_{i+1}; g2 → X^U_{i+1}
  if (c >= M && c < ncol) {
    const int colx = c < 2 * M ? (g == 1 ? c - M : c) : 2 * M;
    double* x = sX[g == 0 ? 0 : 1] + colx;
#pragma unroll
    for (int q = 0; q < H; ++q) x[(hi * H + q) * NC] = has ? a[q] : 0.0;
    if (g != 0 && has) {
      double* X = L.X + (long long)(j / 2) * M * NC + colx;
#pragma unroll
      for (int q = 0; q < H; ++q) X[(hi * H + q) * NC] = a[q];
    }
  }
  __syncthreads();
  if (ST) st[3] = wall_clock64();
  // products, 2×2 tiles: output columns 0..M−1 → D', M..2M−1 → U', 2M → b' (tile columns 2M, 2M+1: b' only)
  const double* sXl = sX[0];
  const double* sXr = sX[1];
  constexpr int TR = M / 2, TC = (2 * M + 2) / 2;
  for (int t = threadIdx.x; t < TR * TC; t += NT) {
    const int r0 = 2 * (t % TR), c0 = 2 * (t / TR);
    double v[2][2];
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int cc = c0 + x;
        v[y][x] = cc < M ? sD[(r0 + y) * M + cc] : (cc == 2 * M ? sb[r0 + y] : 0.0);
      }
    const bool dpart = c0 < M, bpart = c0 == 2 * M;
#pragma unroll 4
    for (int q = 0; q < M; ++q) {
      const double ui0 = sUi[r0 * M + q], ui1 = sUi[(r0 + 1) * M + q];
      const double xr0 = sXr[q * NC + c0], xr1 = c0 + 1 < NC ? sXr[q * NC + c0 + 1] : 0.0;
      if (dpart || bpart) {
        const double ul0 = sUl[q * M + r0], ul1 = sUl[q * M + r0 + 1];
        const double xl0 = sXl[q * NC + (bpart ? 2 * M : M + c0)], xl1 = bpart ? 0.0 : sXl[q * NC + M + c0 + 1];
        v[0][0] -= ul0 * xl0 + ui0 * xr0;
        v[0][1] -= ul0 * xl1 + ui0 * xr1;
        v[1][0] -= ul1 * xl0 + ui1 * xr0;
        v[1][1] -= ul1 * xl1 + ui1 * xr1;
      } else {
        v[0][0] -= ui0 * xr0;
        v[0][1] -= ui0 * xr1;
        v[1][0] -= ui1 * xr0;
        v[1][1] -= ui1 * xr1;
      }
    }
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int cc = c0 + x, r = r0 + y;
        if (cc < M) Ln.D[(long long)in * M * M + r * M + cc] = v[y][x];
        else if (cc < 2 * M) Ln.U[(long long)in * M * M + r * M + (cc - M)] = right ? v[y][x] : 0.0;
        else if (cc == 2 * M) Ln.b[(long long)in * M + r] = v[y][x];
      }
  }
  if (ST) {
    __syncthreads();
    st[4] = wall_clock64();
    if (threadIdx.x == 0)
      for (int q = 0; q < 5; ++q) stamps[blockIdx.x * 5 + q] = st[q];
  }
}

// V4: V2 with a rolled pivot loop (the fully unrolled one is ~40 KB of code: one wave per SIMD streams it through
// the instruction cache once); a[k], a[k+1] extracted/inserted with dynamic register indexing.
template <int M>
__device__ __forceinline__ bool gj_wave_rolled(const double* D, const double* R1, bool r1_trans, const double* R2,
                                               int ncol, int lane, double2* piv, double* a) {
  const int c = lane;
#pragma unroll
  for (int r = 0; r < M; ++r) {
    const double* src = nullptr;
    if (c < M) src = D + r * M + c;
    else if (c < 2 * M) src = R1 ? (r1_trans ? R1 + (c - M) * M + r : R1 + r * M + (c - M)) : nullptr;
    else if (c < M + ncol) src = R2 ? R2 + r : nullptr;
    a[r] = src ? *src : 0.0;
  }
  bool bad = false;
#pragma unroll 1
  for (int k = 0; k < M; k += 2) {
    if (c == k || c == k + 1) {
      double* dst = reinterpret_cast<double*>(piv) + (c - k);
#pragma unroll
      for (int r = 0; r < M; ++r) dst[2 * r] = a[r];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double2 cr[M];
#pragma unroll
    for (int r = 0; r < M; ++r) cr[r] = piv[r];
    const double2 pk = piv[k], pk1 = piv[k + 1];
    const double p00 = pk.x, p10 = pk1.x, p01 = pk.y, p11 = pk1.y;
    const double det = p00 * p11 - p01 * p10;
    bad |= !(p00 > 0.0 && det > 0.0);
    const double rd = rcp_nr(det);
    double ak = a[0], ak1 = a[1];
#pragma unroll
    for (int r = 2; r < M; r += 2) {
      ak = r == k ? a[r] : ak;
      ak1 = r == k ? a[r + 1] : ak1;
    }
    const double t0 = (p11 * ak - p01 * ak1) * rd;
    const double t1 = (p00 * ak1 - p10 * ak) * rd;
#pragma unroll
    for (int r = 0; r < M; r += 2) {
      const bool pv = r == k;
      const double u0 = a[r] - cr[r].x * t0 - cr[r].y * t1;
      const double u1 = a[r + 1] - cr[r + 1].x * t0 - cr[r + 1].y * t1;
      a[r] = pv ? t0 : u0;
      a[r + 1] = pv ? t1 : u1;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  return !bad;
}

template <int M, bool ST>
__global__ __launch_bounds__(256) void level4(CrLevel L, CrLevel Ln, int* status, long long* stamps) {
  constexpr int NC = 2 * M + 1;
  __shared__ __attribute__((aligned(16))) double2 piv[3][M];
  extern __shared__ double smem[];
  double* sUl = smem;
  double* sUi = sUl + M * M;
  double* sD = sUi + M * M;
  double* sb = sD + M * M;
  double* sX[2] = {sb + M, sb + M + M * NC};
  long long st[5];
  st[0] = wall_clock64();
  const int i = 2 * blockIdx.x, in = blockIdx.x;
  const bool left = i - 1 >= 0, right = i + 1 < L.n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double a[M];
  if (ST) st[1] = wall_clock64();
  if (w == 3) {
    for (int e = lane; e < 3 * M * M + M; e += 64) {
      const double* src = nullptr;
      if (e < M * M) src = left ? L.U + (long long)(i - 1) * M * M + e : nullptr;
      else if (e < 2 * M * M) src = L.U + (long long)i * M * M + (e - M * M);
      else if (e < 3 * M * M) src = L.D + (long long)i * M * M + (e - 2 * M * M);
      else src = L.b + (long long)i * M + (e - 3 * M * M);
      smem[e] = src ? *src : 0.0;
    }
  } else {
    const int j = w == 0 ? i - 1 : i + 1;
    const bool has = j >= 0 && j < L.n;
    const int jj = has ? j : 1;
    const double* D = L.D + (long long)jj * M * M;
    const double* bj = L.b + (long long)jj * M;
    bool ok;
    if (w == 0) ok = gj_wave_rolled<M>(D, L.U + (long long)jj * M * M, false, bj, M + 1, lane, piv[0], a);
    else if (w == 1) ok = gj_wave_rolled<M>(D, L.U + (long long)(jj - 1) * M * M, true, bj, M + 1, lane, piv[1], a);
    else ok = gj_wave_rolled<M>(D, jj + 1 < L.n ? L.U + (long long)jj * M * M : nullptr, false, nullptr, M, lane, piv[2], a);
    if (!ok && has && lane == 0) atomicOr(status, 1);
    if (lane >= M && lane < 2 * M + (w == 2 ? 0 : 1)) {
      const int col = lane < 2 * M ? (w == 1 ? lane - M : lane) : 2 * M;
      double* x = sX[w == 0 ? 0 : 1] + col;
#pragma unroll
      for (int r = 0; r < M; ++r) x[r * NC] = has ? a[r] : 0.0;
      if (w != 0 && has) {
        double* X = L.X + (long long)(j / 2) * M * NC + col;
#pragma unroll
        for (int r = 0; r < M; ++r) X[r * NC] = a[r];
      }
    }
  }
  if (ST) st[2] = wall_clock64();
  __syncthreads();
  if (ST) st[3] = wall_clock64();
  const double* sXl = sX[0];
  const double* sXr = sX[1];
  for (int e = threadIdx.x; e < 2 * M * M + M; e += 256) {
    if (e < M * M) {
      const int r = e / M, c = e % M;
      double v = sD[e];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + M + c] + sUi[r * M + q] * sXr[q * NC + c];
      Ln.D[(long long)in * M * M + e] = v;
    } else if (e < 2 * M * M) {
      const int f = e - M * M, r = f / M, c = f % M;
      double v = 0.0;
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUi[r * M + q] * sXr[q * NC + M + c];
      Ln.U[(long long)in * M * M + f] = right ? v : 0.0;
    } else {
      const int r = e - 2 * M * M;
      double v = sb[r];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + 2 * M] + sUi[r * M + q] * sXr[q * NC + 2 * M];
      Ln.b[(long long)in * M + r] = v;
    }
  }
  if (ST) {
    __syncthreads();
    st[4] = wall_clock64();
    if (threadIdx.x == 0)
      for (int q = 0; q < 5; ++q) stamps[blockIdx.x * 5 + q] = st[q];
  }
}

// V5: V2 + the row rebuild on the matrix cores: O = [D | 0 | b] − U_{i−1}ᵀ·B1 − U_i·X_{i+1} as 2 × 4 output tiles
// of v_mfma_f64_16x16x4f64 (rows padded 24 → 32, columns 49 → 64), two tiles per wave, K = 24 in 6 steps.
typedef double v4d __attribute__((ext_vector_type(4)));
template <int M, bool ST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void level5(CrLevel L, CrLevel Ln, int* status, long long* stamps) {
  constexpr int NC = 2 * M + 1;
  __shared__ __attribute__((aligned(16))) double2 piv[3][M];
  extern __shared__ double smem[];
  double* sUl = smem;
  double* sUi = sUl + M * M;
  double* sD = sUi + M * M;
  double* sb = sD + M * M;
  double* sX[2] = {sb + M, sb + M + M * NC};
  long long st[5];
  st[0] = wall_clock64();
  const int i = 2 * blockIdx.x, in = blockIdx.x;
  const bool left = i - 1 >= 0, right = i + 1 < L.n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double a[M];
  if (w == 3) {
    for (int e = lane; e < 3 * M * M + M; e += 64) {
      const double* src = nullptr;
      if (e < M * M) src = left ? L.U + (long long)(i - 1) * M * M + e : nullptr;
      else if (e < 2 * M * M) src = L.U + (long long)i * M * M + (e - M * M);
      else if (e < 3 * M * M) src = L.D + (long long)i * M * M + (e - 2 * M * M);
      else src = L.b + (long long)i * M + (e - 3 * M * M);
      smem[e] = src ? *src : 0.0;
    }
    if (ST) st[1] = wall_clock64();
  } else {
    const int j = w == 0 ? i - 1 : i + 1;
    const bool has = j >= 0 && j < L.n;
    const int jj = has ? j : 1;
    const double* D = L.D + (long long)jj * M * M;
    const double* bj = L.b + (long long)jj * M;
    bool ok;
    if (w == 0) ok = gj_wave<M, ST>(D, L.U + (long long)jj * M * M, false, bj, M + 1, lane, piv[0], a, st);
    else if (w == 1) ok = gj_wave<M, ST>(D, L.U + (long long)(jj - 1) * M * M, true, bj, M + 1, lane, piv[1], a, st);
    else ok = gj_wave<M, ST>(D, jj + 1 < L.n ? L.U + (long long)jj * M * M : nullptr, false, nullptr, M, lane, piv[2], a, st);
    if (!ok && has && lane == 0) atomicOr(status, 1);
    if (lane >= M && lane < 2 * M + (w == 2 ? 0 : 1)) {
      const int col = lane < 2 * M ? (w == 1 ? lane - M : lane) : 2 * M;
      double* x = sX[w == 0 ? 0 : 1] + col;
#pragma unroll
      for (int r = 0; r < M; ++r) x[r * NC] = has ? a[r] : 0.0;
      if (w != 0 && has) {
        double* X = L.X + (long long)(j / 2) * M * NC + col;
#pragma unroll
        for (int r = 0; r < M; ++r) X[r * NC] = a[r];
      }
    }
  }
  if (ST) st[2] = wall_clock64();
  __syncthreads();
  if (ST) st[3] = wall_clock64();
  const double* sXl = sX[0];
  const double* sXr = sX[1];
  // wave w: row tile rt = w & 1, column tiles ct = (w >> 1) * 2 + {0, 1}: the two tiles share the A operands and
  // run as two independent accumulator chains
  const int rt = w & 1;
  const int arow = 16 * rt + (lane & 15), kq = lane >> 4;  // operand A: row, k within the step
  int bcol[2];
  v4d acc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bcol[h] = 16 * ((w >> 1) * 2 + h) + (lane & 15);
#pragma unroll
    for (int v = 0; v < 4; ++v) {  // C = [D | 0 | b]; accumulator entry v of lane l: row l/16 + 4v, column l%16
      const int r = 16 * rt + (lane >> 4) + 4 * v, c = bcol[h];
      acc[h][v] = (r < M) ? (c < M ? sD[r * M + c] : (c == 2 * M ? sb[r] : 0.0)) : 0.0;
    }
  }
#pragma unroll
  for (int s4 = 0; s4 < M / 4; ++s4) {
    const int q = 4 * s4 + kq;
    const double a2 = arow < M ? -sUi[arow * M + q] : 0.0;
    const double a1 = arow < M ? -sUl[q * M + arow] : 0.0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = bcol[h];
      const double b2 = c < NC ? sXr[q * NC + c] : 0.0;
      const double b1 = c < M ? sXl[q * NC + M + c] : (c == 2 * M ? sXl[q * NC + 2 * M] : 0.0);
      acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, b2, acc[h], 0, 0, 0);
      acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[h], 0, 0, 0);
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int r = 16 * rt + (lane >> 4) + 4 * v, c = bcol[h];
      if (r < M) {
        if (c < M) Ln.D[(long long)in * M * M + r * M + c] = acc[h][v];
        else if (c < 2 * M) Ln.U[(long long)in * M * M + r * M + (c - M)] = right ? acc[h][v] : 0.0;
        else if (c == 2 * M) Ln.b[(long long)in * M + r] = acc[h][v];
      }
    }
  if (ST) {
    __syncthreads();
    st[4] = wall_clock64();
    if (threadIdx.x == 0)
      for (int q = 0; q < 5; ++q) stamps[blockIdx.x * 5 + q] = st[q];
  }
}

template <class K0, class K1>
void run(const char* name, K0 kfast, K1 kstamp, int grid, int threads, size_t lds, CrLevel L, CrLevel Ln, int* status,
         long long* stamps) {
  CK(hipFuncSetAttribute((const void*)kfast, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)kstamp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 50; ++w) kfast<<<grid, threads, lds>>>(L, Ln, status, stamps);
  CK(hipEventRecord(e0));
  const int reps = 200;
  for (int w = 0; w < reps; ++w) kfast<<<grid, threads, lds>>>(L, Ln, status, stamps);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  for (int w = 0; w < 5; ++w) kstamp<<<grid, threads, lds>>>(L, Ln, status, stamps);
  CK(hipDeviceSynchronize());
  std::vector<long long> h((size_t)grid * 5);
  CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
  double ph[4] = {0, 0, 0, 0};
  for (int g = 0; g < grid; ++g)
    for (int q = 0; q < 4; ++q) ph[q] += (h[g * 5 + q + 1] - h[g * 5 + q]) * 10.0 / 1e3;
  if (name[1] == '2') {
    long long clk[16];
    CK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_step_clk), sizeof(clk)));
    printf("V2 per-step cycles:");
    for (int q = 0; q + 1 < 12; ++q) printf(" %lld", clk[q + 1] - clk[q]);
    printf("\n");
  }
  printf("%-4s %.2f us/launch | phases us: load %.2f | GJ %.2f | X->LDS %.2f | products %.2f\n", name,
         1e3 * ms / reps, ph[0] / grid, ph[1] / grid, ph[2] / grid, ph[3] / grid);
}

int main(int argc, char** argv) {
  constexpr int M = 24, NC = 2 * M + 1;
  const int n = argc > 1 ? atoi(argv[1]) : 251;
  std::vector<double> D((size_t)n * M * M), U((size_t)n * M * M), b((size_t)n * M);
  srand(1);
  auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
  for (int I = 0; I < n; ++I) {
    for (int r = 0; r < M; ++r)
      for (int c = 0; c <= r; ++c) {
        const double v = 0.1 * rnd() + (r == c ? 10.0 : 0.0);
        D[(size_t)I * M * M + r * M + c] = D[(size_t)I * M * M + c * M + r] = v;
      }
    for (int e = 0; e < M * M; ++e) U[(size_t)I * M * M + e] = I + 1 < n ? rnd() : 0.0;
    for (int r = 0; r < M; ++r) b[(size_t)I * M + r] = rnd();
  }
  CrLevel L{}, Ln{};
  CK(hipMalloc(&L.D, D.size() * 8)); CK(hipMalloc(&L.U, U.size() * 8)); CK(hipMalloc(&L.b, b.size() * 8));
  CK(hipMalloc(&L.X, (size_t)(n / 2 + 1) * M * NC * 8));
  CK(hipMalloc(&Ln.D, D.size() * 8)); CK(hipMalloc(&Ln.U, U.size() * 8)); CK(hipMalloc(&Ln.b, b.size() * 8));
  CK(hipMemcpy(L.D, D.data(), D.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(L.U, U.data(), U.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(L.b, b.data(), b.size() * 8, hipMemcpyHostToDevice));
  L.n = n; Ln.n = (n + 1) / 2;
  int* status; CK(hipMalloc(&status, 4)); CK(hipMemset(status, 0, 4));
  long long* stamps; const int grid = (n + 1) / 2; CK(hipMalloc(&stamps, (size_t)grid * 5 * 8));
  const size_t lds0 = sizeof(double) * (2 * M * M + 2 * M * (2 * M + 1));
  const size_t lds1 = sizeof(double) * (3 * M * M + M + 2 * M * (2 * M + 1));
  printf("n=%d grid=%d\n", n, grid);
  run("V0", &level<M, false>, &level<M, true>, grid, 2 * kT<M>, lds0, L, Ln, status, stamps);
  run("V1", &level1<M, false>, &level1<M, true>, grid, 2 * kT<M>, lds1, L, Ln, status, stamps);
  run("V2", &level2<M, false>, &level2<M, true>, grid, 256, lds1, L, Ln, status, stamps);
  run("V3", &level3<M, false>, &level3<M, true>, grid, 384, lds1, L, Ln, status, stamps);
  run("V4", &level4<M, false>, &level4<M, true>, grid, 256, lds1, L, Ln, status, stamps);
  run("V5", &level5<M, false>, &level5<M, true>, grid, 256, lds1, L, Ln, status, stamps);
  {
    std::vector<double> a0((size_t)Ln.n * M * M), a2(a0.size()), u0(a0.size()), u2(a0.size());
    std::vector<double> x0((size_t)(n / 2 + 1) * M * NC), x2(x0.size());
    level<M, false><<<grid, 2 * kT<M>, lds0>>>(L, Ln, status, stamps);
    CK(hipMemcpy(a0.data(), Ln.D, a0.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(u0.data(), Ln.U, u0.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(x0.data(), L.X, (size_t)(n / 2) * M * NC * 8, hipMemcpyDeviceToHost));
    if (getenv("CMP5")) level5<M, false><<<grid, 256, lds1>>>(L, Ln, status, stamps);
    else if (getenv("CMP4")) level4<M, false><<<grid, 256, lds1>>>(L, Ln, status, stamps);
    else if (getenv("CMP3")) level3<M, false><<<grid, 384, lds1>>>(L, Ln, status, stamps);
    else level2<M, false><<<grid, 256, lds1>>>(L, Ln, status, stamps);
    CK(hipMemcpy(a2.data(), Ln.D, a2.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(u2.data(), Ln.U, u2.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(x2.data(), L.X, (size_t)(n / 2) * M * NC * 8, hipMemcpyDeviceToHost));
    double d = 0, du = 0, dx = 0;
    for (size_t q = 0; q < a0.size(); ++q) { d = std::max(d, std::abs(a0[q] - a2[q])); du = std::max(du, std::abs(u0[q] - u2[q])); }
    for (size_t q = 0; q < (size_t)(n / 2) * M * NC; ++q) dx = std::max(dx, std::abs(x0[q] - x2[q]));
    double sd = 0; for (size_t q = 0; q < a0.size(); ++q) sd = std::max(sd, std::abs(a0[q]));
    {
      std::vector<double> bb0((size_t)Ln.n * M), bb2(bb0.size());
      level<M, false><<<grid, 2 * kT<M>, lds0>>>(L, Ln, status, stamps);
      CK(hipMemcpy(bb0.data(), Ln.b, bb0.size() * 8, hipMemcpyDeviceToHost));
      if (getenv("CMP5")) level5<M, false><<<grid, 256, lds1>>>(L, Ln, status, stamps);
      CK(hipMemcpy(bb2.data(), Ln.b, bb2.size() * 8, hipMemcpyDeviceToHost));
      double db = 0; for (size_t q = 0; q < bb0.size(); ++q) db = std::max(db, std::abs(bb0[q] - bb2[q]));
      printf("  max |db'| = %g\n", db);
    }
    std::vector<double> b0((size_t)Ln.n * M), b2(b0.size());
    printf("%s vs V0 max |dD'| = %g (max |D'| %g) |dU'| = %g |dX| = %g\n", getenv("CMP5") ? "V5" : getenv("CMP4") ? "V4" : getenv("CMP3") ? "V3" : "V2", d, sd, du, dx);
  }
  {  // V1 must reproduce V0 exactly
    std::vector<double> a0((size_t)Ln.n * M * M), a1(a0.size());
    level<M, false><<<grid, 2 * kT<M>, lds0>>>(L, Ln, status, stamps);
    CK(hipMemcpy(a0.data(), Ln.D, a0.size() * 8, hipMemcpyDeviceToHost));
    level1<M, false><<<grid, 2 * kT<M>, lds1>>>(L, Ln, status, stamps);
    CK(hipMemcpy(a1.data(), Ln.D, a1.size() * 8, hipMemcpyDeviceToHost));
    double d = 0; for (size_t q = 0; q < a0.size(); ++q) d = std::max(d, std::abs(a0[q] - a1[q]));
    printf("V1 vs V0 max |dD'| = %g\n", d);
  }
  int st; CK(hipMemcpy(&st, status, 4, hipMemcpyDeviceToHost));
  printf("status %d\n", st);
  return 0;
}
