// Micro-benchmark: phase timing (s_memtime) of the Gauss-Jordan super-row elimination used by
// cr_odd_kernel (pba_gn.hip), on a synthetic SPD level.  Diagnostic tool only; not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>
#include <cmath>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int M, int VARIANT>
__global__ __launch_bounds__(256) void gj(const double* D, const double* U, const double* b, double* X, int n,
                                          long long* stamps) {
  constexpr int NC = 2 * M + 1, W = M + NC, NE = M * W, PER = (NE + 255) / 256;
  __shared__ double rowb[2][W];
  __shared__ double colb[2][M];
  const int tid = threadIdx.x;
  const int j = 2 * blockIdx.x + 1;
  long long t0 = wall_clock64();
  long long c0 = clock64();
  double a[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = min(tid + 256 * u, NE - 1), r = q / W, c = q % W;
    const double* src;
    if (c < M) src = D + (long long)j * M * M + r * M + c;
    else if (c < 2 * M) src = U + (long long)(j - 1) * M * M + (c - M) * M + r;
    else if (c < 3 * M) src = j + 1 < n ? U + (long long)j * M * M + r * M + (c - 2 * M) : nullptr;
    else src = b + (long long)j * M + r;
    a[u] = src ? *src : 0.0;
  }
  __syncthreads();
  long long c1 = clock64();
#pragma unroll 1
  for (int k = 0; k < M; ++k) {
    const int buf = k & 1;
    if (VARIANT >= 1) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int q = tid + 256 * u, r = q / W, c = q % W;
        if (q < NE) {
          if (r == k) rowb[buf][c] = a[u];
          if (c == k) colb[buf][r] = a[u];
        }
      }
    }
    __syncthreads();
    if (VARIANT >= 2) {
      const double p = rowb[buf][k];
      const double ip = VARIANT >= 3 ? 1.0 / p : p;
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int q = tid + 256 * u, r = q / W, c = q % W;
        if (q < NE && c > k) a[u] = r == k ? a[u] * ip : a[u] - colb[buf][r] * ip * rowb[buf][c];
      }
    }
  }
  __syncthreads();
  long long c2 = clock64();
  double* Xo = X + (long long)(j / 2) * M * NC;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = tid + 256 * u, r = q / W, c = q % W;
    if (q < NE && c >= M) Xo[r * NC + (c - M)] = a[u];
  }
  long long c3 = clock64();
  long long t3 = wall_clock64();
  if (tid == 0 && blockIdx.x == 0) {
    stamps[0] = c1 - c0; stamps[1] = c2 - c1; stamps[2] = c3 - c2; stamps[3] = t3 - t0;
  }
}


// Branch-free variant: every lane writes every step (to a dummy slot when it owns no pivot-row/column
// element) and updates every element with a select.
template <int M>
__global__ __launch_bounds__(256) void gj_bf(const double* D, const double* U, const double* b, double* X, int n,
                                             long long* stamps) {
  constexpr int NC = 2 * M + 1, W = M + NC, NE = M * W, PER = (NE + 255) / 256;
  __shared__ double rowb[2][W + 256];
  __shared__ double colb[2][M + 256];
  const int tid = threadIdx.x;
  const int j = 2 * blockIdx.x + 1;
  long long t0 = wall_clock64();
  long long c0 = clock64();
  double a[PER];
  int rr[PER], cc[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int q = tid + 256 * u;
    const int qq = min(q, NE - 1), r = qq / W, c = qq % W;
    rr[u] = q < NE ? r : -1;   // padding lanes own nothing
    cc[u] = c;
    const double* src;
    if (c < M) src = D + (long long)j * M * M + r * M + c;
    else if (c < 2 * M) src = U + (long long)(j - 1) * M * M + (c - M) * M + r;
    else if (c < 3 * M) src = j + 1 < n ? U + (long long)j * M * M + r * M + (c - 2 * M) : nullptr;
    else src = b + (long long)j * M + r;
    a[u] = src ? *src : 0.0;
  }
  __syncthreads();
  long long c1 = clock64();
  long long tp = 0, tb = 0, tr = 0, tu = 0;
#pragma unroll 1
  for (int k = 0; k < M; ++k) {
    const int buf = k & 1;
    const long long s0 = clock64();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      rowb[buf][rr[u] == k ? cc[u] : W + tid] = a[u];
      colb[buf][cc[u] == k && rr[u] >= 0 ? rr[u] : M + tid] = a[u];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    const long long s1 = clock64();
    __syncthreads();
    const long long s2 = clock64();
    // all LDS reads first (one wait), then mask arithmetic (no branches, no per-element waits)
    double cv[PER], rv[PER];
    const double p = rowb[buf][k];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      cv[u] = colb[buf][max(rr[u], 0)];
      rv[u] = rowb[buf][cc[u]];
    }
    const double ip = 1.0 / p;
    const long long s3 = clock64();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const bool live = cc[u] > k, pivrow = rr[u] == k;
      const double m = (live && !pivrow) ? 1.0 : 0.0;
      const double sc = (live && pivrow) ? ip : 1.0;
      a[u] = (a[u] - m * (cv[u] * ip) * rv[u]) * sc;
    }
    if (a[0] == 12345.678) a[0] += 1.0;  // keep the update ahead of the stamp
    const long long s4 = clock64();
    tp += s1 - s0; tb += s2 - s1; tr += s3 - s2; tu += s4 - s3;
  }
  __syncthreads();
  long long c2 = clock64();
  double* Xo = X + (long long)(j / 2) * M * NC;
#pragma unroll
  for (int u = 0; u < PER; ++u)
    if (rr[u] >= 0 && cc[u] >= M) Xo[rr[u] * NC + (cc[u] - M)] = a[u];
  long long c3 = clock64();
  long long t3 = wall_clock64();
  if (tid == 0 && blockIdx.x == 0) {
    stamps[0] = c1 - c0; stamps[1] = c2 - c1; stamps[2] = c3 - c2; stamps[3] = t3 - t0;
    stamps[4] = tp; stamps[5] = tb; stamps[6] = tr; stamps[7] = tu;
  }
}


// Column-owner variant: lane c holds column c of [D | RHS] in registers (steps fully unrolled, so every
// register index is static); step k: the pivot column's owner publishes its M values, one barrier, every
// lane reads them (broadcast) and updates its own column.
template <int M>
__global__ __launch_bounds__(256) void gj_col(const double* D, const double* U, const double* b, double* X, int n,
                                              long long* stamps) {
  constexpr int NC = 2 * M + 1, W = M + NC;
  __shared__ __attribute__((aligned(16))) double colk[2][M];
  const int tid = threadIdx.x;
  const int j = 2 * blockIdx.x + 1;
  long long t0 = wall_clock64();
  long long c0 = clock64();
  const int c = min(tid, W - 1);
  double a[M];
#pragma unroll
  for (int r = 0; r < M; ++r) {
    const double* src;
    if (c < M) src = D + (long long)j * M * M + r * M + c;
    else if (c < 2 * M) src = U + (long long)(j - 1) * M * M + (c - M) * M + r;
    else if (c < 3 * M) src = j + 1 < n ? U + (long long)j * M * M + r * M + (c - 2 * M) : nullptr;
    else src = b + (long long)j * M + r;
    a[r] = src ? *src : 0.0;
  }
  long long c1 = clock64();
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const int buf = k & 1;
    if (tid == k) {
#pragma unroll
      for (int r = 0; r < M; ++r) colk[buf][r] = a[r];
    }
    __syncthreads();
    double m[M];
#pragma unroll
    for (int r = 0; r < M; ++r) m[r] = colk[buf][r];
    const double ip = 1.0 / m[k];
    const double t = a[k] * ip;  // normalised pivot-row entry of this column
#pragma unroll
    for (int r = 0; r < M; ++r) a[r] = r == k ? t : a[r] - m[r] * t;
  }
  long long c2 = clock64();
  if (tid < W && tid >= M) {
    double* Xo = X + (long long)(j / 2) * M * NC;
#pragma unroll
    for (int r = 0; r < M; ++r) Xo[r * NC + (c - M)] = a[r];
  }
  long long c3 = clock64();
  long long t3 = wall_clock64();
  if (tid == 0 && blockIdx.x == 0) {
    stamps[0] = c1 - c0; stamps[1] = c2 - c1; stamps[2] = c3 - c2; stamps[3] = t3 - t0;
  }
}


// One-wave variant: lane l holds columns l and l+64 of [D | RHS]; the pivot column (lane k, compile-time k)
// is broadcast with v_readlane into SGPRs — no LDS, no barriers.
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffff), lane);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int M>
__global__ __launch_bounds__(64) void gj_wave(const double* D, const double* U, const double* b, double* X, int n,
                                              long long* stamps) {
  constexpr int NC = 2 * M + 1, W = M + NC, NS = (W + 63) / 64;
  const int tid = threadIdx.x;
  const int j = 2 * blockIdx.x + 1;
  long long t0 = wall_clock64();
  long long c0 = clock64();
  double a[NS][M];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c = min(tid + 64 * s, W - 1);
#pragma unroll
    for (int r = 0; r < M; ++r) {
      const double* src;
      if (c < M) src = D + (long long)j * M * M + r * M + c;
      else if (c < 2 * M) src = U + (long long)(j - 1) * M * M + (c - M) * M + r;
      else if (c < 3 * M) src = j + 1 < n ? U + (long long)j * M * M + r * M + (c - 2 * M) : nullptr;
      else src = b + (long long)j * M + r;
      a[s][r] = src ? *src : 0.0;
    }
  }
  long long c1 = clock64();
#pragma unroll
  for (int k = 0; k < M; ++k) {
    double m[M];
#pragma unroll
    for (int r = 0; r < M; ++r) m[r] = readlane_f64(a[0][r], k);
    double ip = __builtin_amdgcn_rcp(m[k]) ;
    ip = ip * (2.0 - m[k] * ip);
    ip = ip * (2.0 - m[k] * ip);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const double t = a[s][k] * ip;
#pragma unroll
      for (int r = 0; r < M; ++r) a[s][r] = r == k ? t : a[s][r] - m[r] * t;
    }
  }
  long long c2 = clock64();
  double* Xo = X + (long long)(j / 2) * M * NC;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c = tid + 64 * s;
    if (c >= M && c < W)
#pragma unroll
      for (int r = 0; r < M; ++r) Xo[r * NC + (c - M)] = a[s][r];
  }
  long long c3 = clock64();
  long long t3 = wall_clock64();
  if (tid == 0 && blockIdx.x == 0) {
    stamps[0] = c1 - c0; stamps[1] = c2 - c1; stamps[2] = c3 - c2; stamps[3] = t3 - t0;
  }
}

template <int M, int V>
void run(const char* name, double* D, double* U, double* b, double* X, int n, long long* st) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto launch = [&]() {
    if (V == 9) gj_bf<M><<<n / 2, 256>>>(D, U, b, X, n, st);
    else if (V == 10) gj_col<M><<<n / 2, 256>>>(D, U, b, X, n, st);
    else if (V == 11) gj_wave<M><<<n / 2, 64>>>(D, U, b, X, n, st);
    else gj<M, V><<<n / 2, 256>>>(D, U, b, X, n, st);
  };
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(e0));
  for (int w = 0; w < reps; ++w) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  long long h[8] = {0}; CK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
  int freq = 0; CK(hipDeviceGetAttribute(&freq, hipDeviceAttributeWallClockRate, 0));
  printf("%-28s n=%d: %.2f us/launch (events) | WG0 cycles: load %lld, steps %lld, store %lld | WG0 wall %.2f us\n",
         name, n, 1e3 * ms / reps, h[0], h[1], h[2], h[3] * 1e3 / (double)freq);
  if (V == 9) printf("   per-step cycles: publish %lld, barrier %lld, read+div %lld, update %lld\n", h[4] / 24, h[5] / 24, h[6] / 24, h[7] / 24);
  CK(hipMemset(st, 0, 64));
}

int main() {
  constexpr int M = 24;
  for (int n : {251, 3}) {
    std::vector<double> hD((size_t)n * M * M), hU((size_t)n * M * M), hb((size_t)n * M);
    srand(1);
    for (int I = 0; I < n; ++I)
      for (int r = 0; r < M; ++r)
        for (int c = 0; c < M; ++c) {
          hD[(size_t)I * M * M + r * M + c] = (r == c ? 10.0 : 0.0) + 0.01 * ((r * 7 + c * 7) % 5);
          hU[(size_t)I * M * M + r * M + c] = 0.001 * (rand() % 100);
        }
    for (auto& x : hb) x = 1.0;
    double *D, *U, *b, *X; long long* st;
    CK(hipMalloc(&D, hD.size() * 8)); CK(hipMalloc(&U, hU.size() * 8)); CK(hipMalloc(&b, hb.size() * 8));
    CK(hipMalloc(&X, (size_t)n * M * (2 * M + 1) * 8)); CK(hipMalloc(&st, 64));
    CK(hipMemcpy(D, hD.data(), hD.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(U, hU.data(), hU.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
    run<M, 0>("barriers only", D, U, b, X, n, st);
    run<M, 1>("+ publish", D, U, b, X, n, st);
    run<M, 2>("+ update (no div)", D, U, b, X, n, st);
    run<M, 3>("full (fp64 div)", D, U, b, X, n, st);
    std::vector<double> x3((size_t)(n / 2) * M * (2 * M + 1)), x9(x3.size());
    CK(hipMemcpy(x3.data(), X, x3.size() * 8, hipMemcpyDeviceToHost));
    run<M, 9>("branch-free", D, U, b, X, n, st);
    CK(hipMemcpy(x9.data(), X, x9.size() * 8, hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < x3.size(); ++i) md = std::max(md, std::abs(x3[i] - x9[i]));
    printf("  max |X_full - X_branchfree| = %.3e\n", md);
    run<M, 10>("column owner", D, U, b, X, n, st);
    CK(hipMemcpy(x9.data(), X, x9.size() * 8, hipMemcpyDeviceToHost));
    md = 0;
    for (size_t i = 0; i < x3.size(); ++i) md = std::max(md, std::abs(x3[i] - x9[i]) / (std::abs(x3[i]) + 1e-300));
    printf("  max rel |X_full - X_column| = %.3e\n", md);
    run<M, 11>("one wave, readlane", D, U, b, X, n, st);
    CK(hipMemcpy(x9.data(), X, x9.size() * 8, hipMemcpyDeviceToHost));
    md = 0;
    for (size_t i = 0; i < x3.size(); ++i) md = std::max(md, std::abs(x3[i] - x9[i]) / (std::abs(x3[i]) + 1e-300));
    printf("  max rel |X_full - X_wave| = %.3e\n", md);
    CK(hipFree(D)); CK(hipFree(U)); CK(hipFree(b)); CK(hipFree(X)); CK(hipFree(st));
  }
  return 0;
}
