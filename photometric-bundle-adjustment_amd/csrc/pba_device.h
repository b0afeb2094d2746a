// pba_device.h — per-lane arithmetic of the residual/Jacobian kernels (gfx950).
//
// Precision split.  The sub-pixel position u = π_t(p) decides which bilinear cell is read and the
// interpolation weights, so everything from the bearing to (u, v) runs in fp64 (unproject, warp,
// projection) — an fp32 warp puts ~3e-5 px of rounding into u at 752-px coordinates, which shows up as
// 1e-4-relative Jacobian noise through the image gradient.  The block kernel is bound by memory latency at
// full occupancy with its SIMDs ~55–60 % VALU-busy (profiles/r1_c4_v13_sq_counters.json), so the fp64 part is
// mostly hidden.  The Jacobian chain (∇I · ∂π/∂p · ∂p/∂δ) and the records are fp32.
//
// Closed-form tangent Jacobians instead of the reference's dual numbers: the
// reference differentiates BundleAdjustmentReprojectionCostFunctor (reprojection.h:83-112) with
// Jet<double,23> and maps through LocalParameterizationSE3 (residual_block.cc:136-158); here
// d r / d δ with T ⊞ δ = T·exp(δ) is written out directly:
//
//   p_t = R_th p_h + t_th ,  p_h = b / ρ                     (geometric, unscaled)
//   p̃   = R_th b + ρ t_th = ρ p_t                            (photometric, photometric_error.h:155-159)
//   ∂p̃/∂υ_h = ρ R_th   ∂p̃/∂ω_h = −R_th [b]×   ∂p̃/∂υ_t = −ρ I   ∂p̃/∂ω_t = [p̃]×   ∂p̃/∂ρ = t_th
//   ∂p/∂υ_h = R_th     ∂p/∂ω_h = −R_th [p_h]×  ∂p/∂υ_t = −I      ∂p/∂ω_t = [p]×    ∂p/∂ρ = −R_th b/ρ²
//
// For a row vector a (1×3):  a·[b]× = (a × b)ᵀ.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pba {

enum : int { CAM_PINHOLE = 0, CAM_DS = 1, CAM_EUCM = 2, CAM_KB4 = 3 };

template <class S>
struct V3 { S x, y, z; };
using Vec3 = V3<float>;
using Vec3d = V3<double>;

template <class S>
__device__ __forceinline__ V3<S> cross(const V3<S>& a, const V3<S>& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <class S>
__device__ __forceinline__ S dot(const V3<S>& a, const V3<S>& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ Vec3 to_f(const Vec3d& a) { return {(float)a.x, (float)a.y, (float)a.z}; }

// a (row) · R  (R row-major 3×3)
template <class S, class T>
__device__ __forceinline__ V3<S> row_mul(const V3<S>& a, const T* R) {
  return {a.x * (S)R[0] + a.y * (S)R[3] + a.z * (S)R[6], a.x * (S)R[1] + a.y * (S)R[4] + a.z * (S)R[7],
          a.x * (S)R[2] + a.y * (S)R[5] + a.z * (S)R[8]};
}
template <class S, class T>
__device__ __forceinline__ V3<S> mat_mul(const T* R, const V3<S>& b) {
  return {(S)R[0] * b.x + (S)R[1] * b.y + (S)R[2] * b.z, (S)R[3] * b.x + (S)R[4] * b.y + (S)R[5] * b.z,
          (S)R[6] * b.x + (S)R[7] * b.y + (S)R[8] * b.z};
}

// Reciprocal / reciprocal square root to ~1 ulp in fp64: hardware v_rcp_f64 / v_rsq_f64 seed + ONE third-order
// correction (relative seed error e ≲ 2⁻²² → e³ ≲ 2⁻⁶⁶): 1/x = y(1 + e + e²) with e = 1 − xy, 1/√x = y(1 + e/2 +
// 3e²/8) with e = 1 − xy² — 2 and 4 fp64 operations after the seed instead of the 4 and 6 of two Newton steps.  The
// IEEE division and sqrt() sequences the compiler emits otherwise (div_scale / div_fmas / div_fixup, ldexp range
// scaling) were ~15% of the block kernel's VALU instructions.  Arguments here are finite and far from the denormal
// range (focal lengths, depths inside the projection domain, |b|² ≈ 1, SPD pivots).
__device__ __forceinline__ double rcp_nr(double x) {
  const double y = __builtin_amdgcn_rcp(x);
  const double e = fma(-x, y, 1.0);
  return fma(y, fma(e, e, e), y);
}
__device__ __forceinline__ double rsqrt_nr(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double e = fma(-x * y, y, 1.0);
  return fma(y * e, fma(e, 0.375, 0.5), y);
}
__device__ __forceinline__ float rcp_s(float x) { return __builtin_amdgcn_rcpf(x); }  // 1 ulp (fp32 chain)
__device__ __forceinline__ double rcp_s(double x) { return rcp_nr(x); }

// Camera record in device memory: kCamD doubles per camera, laid out for the two uses —
//   [0..7]   projection   "tk": fx fy cx cy p1 p2 p3 p4      (camera_models.h:50; p1,p2 = ξ,α (DS) or α,β (EUCM),
//                                                         p1..p4 = k1..k4 (KB4))
//   [8..15]  unprojection "hk": cx cy 1/fx 1/fy p1 p2 p3 p4   (reciprocals precomputed on the host)
// The pair kernel copies the host camera's hk and the target camera's tk into every PairRec.
constexpr int kCamK = 8, kCamD = 2 * kCamK, kCamHk = kCamK;

__device__ __forceinline__ float atan2_s(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double atan2_s(double y, double x) { return atan2(y, x); }

// Kannala-Brandt d(θ) = θ + θ³(k1 + θ²(k2 + θ²(k3 + θ²k4))) and d'(θ) (camera_models.h:338-343, :406-420)
template <class S, class K>
__device__ __forceinline__ S kb4_d(const K* k, S th) {
  const S t2 = th * th;
  return th + t2 * th * ((S)k[0] + t2 * ((S)k[1] + t2 * ((S)k[2] + t2 * (S)k[3])));
}
template <class S, class K>
__device__ __forceinline__ S kb4_dd(const K* k, S th) {
  const S t2 = th * th;
  return S(1) + t2 * (S(3) * (S)k[0] + t2 * (S(5) * (S)k[1] + t2 * (S(7) * (S)k[2] + t2 * S(9) * (S)k[3])));
}

// Unit bearing of pixel (u, v) — camera_models.h unproject (pinhole :93-107, EUCM :162-190,
// DS :247-277) followed by normalize() (reprojection.h:104).  fp64; hk = [cx cy 1/fx 1/fy p1 p2].
template <int MODEL>
__device__ __forceinline__ Vec3d unproject(const double* hk, double u, double v) {
  const double mx = (u - hk[0]) * hk[2];
  const double my = (v - hk[1]) * hk[3];
  Vec3d b;
  if (MODEL == CAM_PINHOLE) {
    b = {mx, my, 1.0};
  } else if (MODEL == CAM_DS) {
    const double xi = hk[4], al = hk[5];
    const double r2 = mx * mx + my * my;
    const double mz = (1.0 - al * al * r2) * rcp_nr(al * sqrt(1.0 - (2.0 * al - 1.0) * r2) + 1.0 - al);
    const double fac = (mz * xi + sqrt(mz * mz + (1.0 - xi * xi) * r2)) * rcp_nr(mz * mz + r2);
    b = {fac * mx, fac * my, fac * mz - xi};
  } else if (MODEL == CAM_EUCM) {
    const double al = hk[4], be = hk[5];
    const double r2 = mx * mx + my * my;
    b = {mx, my, (1.0 - be * al * al * r2) * rcp_nr(al * sqrt(1.0 - (2.0 * al - 1.0) * be * r2) + (1.0 - al))};
  } else {  // KB4, camera_models.h:352-380: 5 Newton steps on d(θ) = r_u from θ = 0
    const double ru = sqrt(mx * mx + my * my);
    if (ru == 0.0) return {0.0, 0.0, 1.0};
    double th = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) th -= (kb4_d(hk + 4, th) - ru) / kb4_dd(hk + 4, th);
    double sn, cs;
    sincos(th, &sn, &cs);
    b = {sn * mx / ru, sn * my / ru, cs};
  }
  const double inv = rsqrt_nr(b.x * b.x + b.y * b.y + b.z * b.z);
  return {b.x * inv, b.y * inv, b.z * inv};
}

// Projection domain on the (possibly scaled) point — identical rule to oracle/oracle.cpp in_domain();
// k = tk layout [fx fy cx cy p1 p2].
template <int MODEL>
__device__ __forceinline__ bool in_domain(const double* k, const Vec3d& p) {
  if (MODEL == CAM_PINHOLE) return p.z > 1e-6;
  if (MODEL == CAM_KB4) return p.z > 0.0 || p.x * p.x + p.y * p.y > 0.0;  // all but the backward axis
  if (MODEL == CAM_EUCM) {
    const double al = k[4], be = k[5];
    const double rr = sqrt(be * (p.x * p.x + p.y * p.y) + p.z * p.z);
    const double w = al > 0.5 ? (1.0 - al) / al : al / (1.0 - al);
    return p.z > -w * rr + 1e-10;
  }
  const double xi = k[4], al = k[5];
  const double d1 = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
  const double w1 = al <= 0.5 ? al / (1.0 - al) : (1.0 - al) / al;
  const double w2 = (w1 + xi) / sqrt(2.0 * w1 * xi + xi * xi + 1.0);
  return p.z > -w2 * d1 + 1e-10;
}

// Projection (fp64) — camera_models.h project (pinhole :75-91, EUCM :140-160, DS :226-245); k = tk layout
// [fx fy cx cy p1 p2].  Returns 1/den (pinhole: 1/z), which project_jac reuses.
template <int MODEL>
__device__ __forceinline__ double project(const double* k, const Vec3d& p, double& u, double& v) {
  if (MODEL == CAM_KB4) {  // camera_models.h:316-348; returns the scale d(θ)/r (1/z at r = 0, its limit)
    const double r = sqrt(p.x * p.x + p.y * p.y);
    if (r == 0.0) {
      u = k[2];
      v = k[3];
      return rcp_nr(p.z);
    }
    const double d = kb4_d(k + 4, atan2(r, p.z));
    u = k[0] * d * p.x / r + k[2];
    v = k[1] * d * p.y / r + k[3];
    return d / r;
  }
  double den;
  if (MODEL == CAM_PINHOLE) {
    den = p.z;
  } else if (MODEL == CAM_DS) {
    const double xi = k[4], al = k[5];
    const double d1 = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    const double kk = xi * d1 + p.z;
    const double d2 = sqrt(p.x * p.x + p.y * p.y + kk * kk);
    den = al * d2 + (1.0 - al) * kk;
  } else {
    const double al = k[4], be = k[5];
    den = al * sqrt(be * (p.x * p.x + p.y * p.y) + p.z * p.z) + (1.0 - al) * p.z;
  }
  const double iden = rcp_nr(den);
  u = k[0] * (p.x * iden) + k[2];
  v = k[1] * (p.y * iden) + k[3];
  return iden;
}

__device__ __forceinline__ float sqrt_s(float x) { return sqrtf(x); }
__device__ __forceinline__ double sqrt_s(double x) { return sqrt(x); }

// 2×3 projection Jacobian (rows du/dp, dv/dp) given iden = 1/den from project(); fp32 in the Jacobian chain,
// fp64 where a product with it cancels (∂r/∂ρ).  k: the first 8 intrinsics, in S.
template <int MODEL, class S>
__device__ __forceinline__ void project_jac(const S* k, const V3<S>& p, S iden, V3<S>& du, V3<S>& dv) {
  const S fx = k[0], fy = k[1], one = S(1), zero = S(0);
  if (MODEL == CAM_KB4) {
    // u = fx·d(θ)·c + cx with (c, s) = (x, y)/r:  ∂u/∂p = fx·(d'(θ)·c·∇θ + (d/r)·(s², −cs, 0)), no cancellation
    // as r → 0 (iden = d/r from project(); at r = 0 take c = 1, s = 0, the limit)
    const S r = sqrt_s(p.x * p.x + p.y * p.y);
    const S c = r > zero ? p.x / r : one, sn = r > zero ? p.y / r : zero;
    const S ir2 = one / (r * r + p.z * p.z);
    const V3<S> gt = {p.z * c * ir2, p.z * sn * ir2, -r * ir2};
    const S dd = kb4_dd(k + 4, atan2_s(r, p.z));
    du = {fx * (dd * c * gt.x + iden * sn * sn), fx * (dd * c * gt.y - iden * c * sn), fx * dd * c * gt.z};
    dv = {fy * (dd * sn * gt.x - iden * c * sn), fy * (dd * sn * gt.y + iden * c * c), fy * dd * sn * gt.z};
    return;
  }
  if (MODEL == CAM_PINHOLE) {
    const S mx = p.x * iden, my = p.y * iden;
    du = {fx * iden, zero, -fx * mx * iden};
    dv = {zero, fy * iden, -fy * my * iden};
    return;
  }
  V3<S> dden;
  if (MODEL == CAM_DS) {
    const S xi = k[4], al = k[5];
    const S d1 = sqrt_s(p.x * p.x + p.y * p.y + p.z * p.z);
    const S kk = xi * d1 + p.z;
    const S d2 = sqrt_s(p.x * p.x + p.y * p.y + kk * kk);
    const S id1 = rcp_s(d1), id2 = rcp_s(d2);
    const V3<S> dk = {xi * p.x * id1, xi * p.y * id1, xi * p.z * id1 + one};
    const V3<S> dd2 = {(p.x + kk * dk.x) * id2, (p.y + kk * dk.y) * id2, kk * dk.z * id2};
    dden = {al * dd2.x + (one - al) * dk.x, al * dd2.y + (one - al) * dk.y, al * dd2.z + (one - al) * dk.z};
  } else {
    const S al = k[4], be = k[5];
    const S d = sqrt_s(be * (p.x * p.x + p.y * p.y) + p.z * p.z);
    const S id = rcp_s(d);
    dden = {al * be * p.x * id, al * be * p.y * id, al * p.z * id + (one - al)};
  }
  const S mx = p.x * iden, my = p.y * iden;
  du = {fx * iden * (one - mx * dden.x), -fx * iden * mx * dden.y, -fx * iden * mx * dden.z};
  dv = {-fy * iden * my * dden.x, fy * iden * (one - my * dden.y), -fy * iden * my * dden.z};
}

// ∂π/∂k (rows du, dv; 8 columns) of the projection at p with respect to the intrinsics k = [fx fy cx cy p1 p2 p3 p4]
// (tk layout), given iden from project() — the Jacobian the reference's functor takes for its sIntr_c2 parameter block
// (reprojection.h:83-86, :108; AutoDiffCostFunction<…, 8>), free when BundleAdjustmentOptions::optimize_intrinsics is set
// (map_utils.h:339-345).  fp64.  Pinhole (camera_models.h:75-91): u = fx x/z + cx.  DS (:226-245) and EUCM (:140-160):
// u = fx x/den + cx with ∂den/∂(ξ, α) = (α kk d1/d2 + (1 − α) d1, d2 − kk) resp. ∂den/∂(α, β) = (ρ − z, α (x² + y²)/2ρ).
// KB4 (:316-348): u = fx d(θ) x/r + cx with ∂d/∂k_i = θ^(2i+1).
template <int MODEL>
__device__ __forceinline__ void project_intr_jac(const double* k, const Vec3d& p, double iden, double* du, double* dv) {
#pragma unroll
  for (int j = 0; j < 8; ++j) du[j] = dv[j] = 0.0;
  du[2] = 1.0;
  dv[3] = 1.0;
  if (MODEL == CAM_KB4) {
    const double r = sqrt(p.x * p.x + p.y * p.y);
    if (r == 0.0) return;  // u = cx, v = cy
    const double c = p.x / r, s = p.y / r, th = atan2(r, p.z), t2 = th * th;
    du[0] = iden * p.x;  // d(θ)·x/r (iden = d/r from project())
    dv[1] = iden * p.y;
    double t = t2 * th;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      du[4 + i] = k[0] * c * t;
      dv[4 + i] = k[1] * s * t;
      t *= t2;
    }
    return;
  }
  const double mx = p.x * iden, my = p.y * iden;
  du[0] = mx;
  dv[1] = my;
  if (MODEL == CAM_PINHOLE) return;
  double d4, d5;  // ∂den/∂p1, ∂den/∂p2
  if (MODEL == CAM_DS) {
    const double xi = k[4], al = k[5];
    const double d1 = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    const double kk = xi * d1 + p.z;
    const double d2 = sqrt(p.x * p.x + p.y * p.y + kk * kk);
    d4 = al * kk * d1 / d2 + (1.0 - al) * d1;
    d5 = d2 - kk;
  } else {
    const double al = k[4], be = k[5];
    const double r2 = p.x * p.x + p.y * p.y;
    const double rho = sqrt(be * r2 + p.z * p.z);
    d4 = rho - p.z;
    d5 = al * r2 / (2.0 * rho);
  }
  // ∂u/∂den = −fx x/den² = −fx mx iden
  du[4] = -k[0] * mx * iden * d4;
  du[5] = -k[0] * mx * iden * d5;
  dv[4] = -k[1] * my * iden * d4;
  dv[5] = -k[1] * my * iden * d5;
}

// Keyframe images live in HBM as 16×8-texel tiles of 128 B (one L2 line): tile (x>>4, y>>3) at
// ((y>>3)·tiles_x + (x>>4))·128, texel (x&15) + 16·(y&7) inside.  A warped 8-pixel pattern plus its bilinear
// taps covers ≈6×6 texels, which touches ≈2.1 tiles against ≈6.3 lines in row-major order (DESIGN.md
// has the measured FETCH_SIZE per block before and after).  Every frame carries a kImgPad-texel apron that
// replicates its edge pixels (Grid2D's clamp, cubic_interpolation.h:403-414), so the four taps of any position
// inside the interpolation clamp [−2, W+1] are plain in-bounds reads: no per-tap clamping.
constexpr int kTileW = 16, kTileH = 8, kTileBytes = kTileW * kTileH, kImgPad = 4;
__host__ __device__ __forceinline__ int tiles_x_of(int W) { return (W + 2 * kImgPad + kTileW - 1) / kTileW; }
__host__ __device__ __forceinline__ long long tiled_frame_bytes(int W, int H) {
  return (long long)tiles_x_of(W) * ((H + 2 * kImgPad + kTileH - 1) / kTileH) * kTileBytes;
}
// byte offset of padded texel (xp, yp) = image pixel (xp − kImgPad, yp − kImgPad)
__host__ __device__ __forceinline__ unsigned texel_index(int xp, int yp, int tiles_x) {
  return (((unsigned)((yp >> 3) * tiles_x + (xp >> 4))) << 7) | ((unsigned)(yp & 7) << 4) | (unsigned)(xp & 15);
}
__host__ __device__ __forceinline__ unsigned texel_index_img(int x, int y, int tiles_x) {
  return texel_index(x + kImgPad, y + kImgPad, tiles_x);
}

// Bilinear interpolation of a tiled u8 image with Grid2D-style edge clamp (the apron); value and gradient from
// the same four taps.  u = column, v = row, positions in fp64, value weights in fp32.
// Split in two (bilinear_taps → bilinear_eval) for callers that issue several positions' taps before using any;
// bilinear() is the two back to back.
struct Taps {
  double fu, fv;       // cell fractions u − ⌊u⌋, v − ⌊v⌋ (fp64: the gradient needs them exactly)
  float I00, I10, I01, I11;
};
__device__ __forceinline__ Taps bilinear_taps(const uint8_t* __restrict__ img, double umax, double vmax, int tiles_x,
                                              double u, double v) {
  u = fmin(fmax(u, -2.0), umax);  // NaN positions clamp to −2 (maxNum): always an in-bounds read
  v = fmin(fmax(v, -2.0), vmax);
  const double xf = floor(u), yf = floor(v);
  const int xp = (int)xf + kImgPad, yp = (int)yf + kImgPad;  // ∈ [2, W+5] × [2, H+5]
  const unsigned i00 = texel_index(xp, yp, tiles_x);
  const unsigned dx = (xp & 15) == 15 ? (unsigned)(kTileBytes - 15) : 1u;                 // next column
  const unsigned dy = (yp & 7) == 7 ? (unsigned)(tiles_x * kTileBytes - 7 * kTileW) : 16u;  // next row
  Taps t;
  t.fu = u - xf;
  t.fv = v - yf;
  t.I00 = img[i00];
  t.I10 = img[i00 + dx];
  t.I01 = img[i00 + dy];
  t.I11 = img[i00 + dy + dx];
  return t;
}
__device__ __forceinline__ void bilinear_eval(const Taps& t, float& I, float& gx, float& gy) {
  const float a = (float)t.fu, b = (float)t.fv;
  const float top = t.I00 + a * (t.I10 - t.I00);
  const float bot = t.I01 + a * (t.I11 - t.I01);
  I = top + b * (bot - top);
  // ∂I/∂u, ∂I/∂v from exact integer tap differences with fp64 cell fractions: a gradient component near
  // zero is the difference of two O(255) terms, and an fp32 fraction leaves ~1.5e-5 absolute error there
  // (3e-5 relative on J_ρ at P = 1).  Dead code for residual-only callers.
  gx = (float)fma(t.fv, (double)((t.I11 - t.I01) - (t.I10 - t.I00)), (double)(t.I10 - t.I00));
  gy = (float)fma(t.fu, (double)((t.I11 - t.I10) - (t.I01 - t.I00)), (double)(t.I01 - t.I00));
}
__device__ __forceinline__ void bilinear(const uint8_t* __restrict__ img, double umax, double vmax, int tiles_x,
                                         double u, double v, float& I, float& gx, float& gy) {
  bilinear_eval(bilinear_taps(img, umax, vmax, tiles_x, u, v), I, gx, gy);
}

// Ceres' BiCubicInterpolator over Grid2D<uint8_t, 1> (cubic_interpolation.h:252-344, the interpolator of
// PhotometricError, photometric_error.h:84): four horizontal cubic Hermite (Catmull-Rom) splines through the 4×4 taps
// around (⌊v⌋, ⌊u⌋), value and ∂/∂u per row, then one vertical spline of the values (→ I, ∂I/∂v) and one of the
// row derivatives (→ ∂I/∂u).  fp64 as Ceres (CubicHermiteSpline :64-90, same operation order).  The 4-texel apron is
// Grid2D's edge clamp (:403-414) for every tap of a position inside [−2, W+1] × [−2, H+1]; beyond that all 16 taps
// of Ceres' unclamped evaluation are the same edge texel, which the clamped position reproduces (constant spline).
__device__ __forceinline__ void hermite(double p0, double p1, double p2, double p3, double x, double& f, double& df) {
  const double a = 0.5 * (-p0 + 3.0 * p1 - 3.0 * p2 + p3);
  const double b = 0.5 * (2.0 * p0 - 5.0 * p1 + 4.0 * p2 - p3);
  const double c = 0.5 * (-p0 + p2);
  const double d = p1;
  f = d + x * (c + x * (b + x * a));
  df = c + x * (2.0 * b + 3.0 * a * x);
}
__device__ __forceinline__ void bicubic(const uint8_t* __restrict__ img, double umax, double vmax, int tiles_x, double u,
                                        double v, float& I, float& gx, float& gy) {
  u = fmin(fmax(u, -2.0), umax);
  v = fmin(fmax(v, -2.0), vmax);
  const double xf = floor(u), yf = floor(v);
  const int xp = (int)xf + kImgPad, yp = (int)yf + kImgPad;  // taps xp−1 … xp+2 ∈ [1, W+7]: inside the apron
  const double x = u - xf, y = v - yf;
  double f[4], dfdc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double p[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) p[c] = (double)img[texel_index(xp - 1 + c, yp - 1 + r, tiles_x)];
    hermite(p[0], p[1], p[2], p[3], x, f[r], dfdc[r]);
  }
  double val, dfdr, dfdu, unused;
  hermite(f[0], f[1], f[2], f[3], y, val, dfdr);
  hermite(dfdc[0], dfdc[1], dfdc[2], dfdc[3], y, dfdu, unused);
  I = (float)val;
  gx = (float)dfdu;
  gy = (float)dfdr;
}

enum : int { INTERP_BILINEAR = 0, INTERP_BICUBIC = 1 };

// The kernels' photometric template parameter carries the camera model and the interpolator: PM = model + 4·interp.
__host__ __device__ constexpr int cam_of(int pm) { return pm & 3; }
__host__ __device__ constexpr int interp_of(int pm) { return pm >> 2; }

// umax, vmax = W + 1, H + 1: the interpolation clamp [−2, W+1] × [−2, H+1] (kernel arguments, not per-lane work)
template <int INTERP>
__device__ __forceinline__ void interpolate(const uint8_t* __restrict__ img, double umax, double vmax, int tiles_x,
                                            double u, double v, float& I, float& gx, float& gy) {
  if (INTERP == INTERP_BICUBIC) bicubic(img, umax, vmax, tiles_x, u, v, I, gx, gy);
  else bilinear(img, umax, vmax, tiles_x, u, v, I, gx, gy);
}

}  // namespace pba
