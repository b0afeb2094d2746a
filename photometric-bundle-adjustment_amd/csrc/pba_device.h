// pba_device.h — per-lane arithmetic of the residual/Jacobian kernels (fp32, gfx950).
//
// Closed-form tangent Jacobians instead of the reference's dual numbers:
// the reference differentiates BundleAdjustmentReprojectionCostFunctor (reprojection.h:83-112) with
// Jet<double,23> and maps through LocalParameterizationSE3 (residual_block.cc:136-158); here the
// composition d r / d δ with T ⊞ δ = T·exp(δ) is written out directly:
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

enum : int { CAM_PINHOLE = 0, CAM_DS = 1, CAM_EUCM = 2 };

struct Vec3 { float x, y, z; };

__device__ __forceinline__ Vec3 cross(const Vec3& a, const Vec3& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float dot(const Vec3& a, const Vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// a (row) · R  (R row-major 3×3)
__device__ __forceinline__ Vec3 row_mul(const Vec3& a, const float* R) {
  return {a.x * R[0] + a.y * R[3] + a.z * R[6], a.x * R[1] + a.y * R[4] + a.z * R[7],
          a.x * R[2] + a.y * R[5] + a.z * R[8]};
}
__device__ __forceinline__ Vec3 mat_mul(const float* R, const Vec3& b) {
  return {R[0] * b.x + R[1] * b.y + R[2] * b.z, R[3] * b.x + R[4] * b.y + R[5] * b.z,
          R[6] * b.x + R[7] * b.y + R[8] * b.z};
}

// Unit bearing of pixel (u, v) — camera_models.h unproject (pinhole :93-107, EUCM :162-190,
// DS :247-277) followed by normalize() (reprojection.h:104).
template <int MODEL>
__device__ __forceinline__ Vec3 unproject(const float* k, float u, float v) {
  const float mx = (u - k[2]) / k[0];
  const float my = (v - k[3]) / k[1];
  Vec3 b;
  if (MODEL == CAM_PINHOLE) {
    b = {mx, my, 1.0f};
  } else if (MODEL == CAM_DS) {
    const float xi = k[4], al = k[5];
    const float r2 = mx * mx + my * my;
    const float mz = (1.0f - al * al * r2) / (al * sqrtf(1.0f - (2.0f * al - 1.0f) * r2) + 1.0f - al);
    const float fac = (mz * xi + sqrtf(mz * mz + (1.0f - xi * xi) * r2)) / (mz * mz + r2);
    b = {fac * mx, fac * my, fac * mz - xi};
  } else {
    const float al = k[4], be = k[5];
    const float r2 = mx * mx + my * my;
    b = {mx, my, (1.0f - be * al * al * r2) / (al * sqrtf(1.0f - (2.0f * al - 1.0f) * be * r2) + (1.0f - al))};
  }
  const float inv = rsqrtf(b.x * b.x + b.y * b.y + b.z * b.z);
  return {b.x * inv, b.y * inv, b.z * inv};
}

// Projection domain on the (possibly scaled) point — identical rule to oracle/oracle.cpp in_domain().
template <int MODEL>
__device__ __forceinline__ bool in_domain(const float* k, const Vec3& p) {
  if (MODEL == CAM_PINHOLE) return p.z > 1e-6f;
  if (MODEL == CAM_EUCM) {
    const float al = k[4], be = k[5];
    const float rr = sqrtf(be * (p.x * p.x + p.y * p.y) + p.z * p.z);
    const float w = al > 0.5f ? (1.0f - al) / al : al / (1.0f - al);
    return p.z > -w * rr + 1e-10f;
  }
  const float xi = k[4], al = k[5];
  const float d1 = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
  const float w1 = al <= 0.5f ? al / (1.0f - al) : (1.0f - al) / al;
  const float w2 = (w1 + xi) / sqrtf(2.0f * w1 * xi + xi * xi + 1.0f);
  return p.z > -w2 * d1 + 1e-10f;
}

// Projection and its 2×3 Jacobian (rows du/dp, dv/dp) — camera_models.h project (pinhole :75-91,
// EUCM :140-160, DS :226-245).
template <int MODEL>
__device__ __forceinline__ void project_jac(const float* k, const Vec3& p, float& u, float& v, Vec3& du, Vec3& dv) {
  const float fx = k[0], fy = k[1], cx = k[2], cy = k[3];
  if (MODEL == CAM_PINHOLE) {
    const float iz = 1.0f / p.z;
    const float mx = p.x * iz, my = p.y * iz;
    u = fx * mx + cx;
    v = fy * my + cy;
    du = {fx * iz, 0.0f, -fx * mx * iz};
    dv = {0.0f, fy * iz, -fy * my * iz};
    return;
  }
  float den;
  Vec3 dden;
  if (MODEL == CAM_DS) {
    const float xi = k[4], al = k[5];
    const float d1 = sqrtf(p.x * p.x + p.y * p.y + p.z * p.z);
    const float kk = xi * d1 + p.z;
    const float d2 = sqrtf(p.x * p.x + p.y * p.y + kk * kk);
    den = al * d2 + (1.0f - al) * kk;
    const float id1 = 1.0f / d1, id2 = 1.0f / d2;
    const Vec3 dk = {xi * p.x * id1, xi * p.y * id1, xi * p.z * id1 + 1.0f};
    const Vec3 dd2 = {(p.x + kk * dk.x) * id2, (p.y + kk * dk.y) * id2, kk * dk.z * id2};
    dden = {al * dd2.x + (1.0f - al) * dk.x, al * dd2.y + (1.0f - al) * dk.y, al * dd2.z + (1.0f - al) * dk.z};
  } else {
    const float al = k[4], be = k[5];
    const float d = sqrtf(be * (p.x * p.x + p.y * p.y) + p.z * p.z);
    den = al * d + (1.0f - al) * p.z;
    const float id = 1.0f / d;
    dden = {al * be * p.x * id, al * be * p.y * id, al * p.z * id + (1.0f - al)};
  }
  const float iden = 1.0f / den;
  const float mx = p.x * iden, my = p.y * iden;
  u = fx * mx + cx;
  v = fy * my + cy;
  du = {fx * iden * (1.0f - mx * dden.x), -fx * iden * mx * dden.y, -fx * iden * mx * dden.z};
  dv = {-fy * iden * my * dden.x, fy * iden * (1.0f - my * dden.y), -fy * iden * my * dden.z};
}

// Bilinear interpolation of a u8 image with Grid2D-style edge clamp; value and gradient from the same
// four taps.  u = column, v = row.
__device__ __forceinline__ void bilinear(const uint8_t* __restrict__ img, int W, int H, float u, float v,
                                         float& I, float& gx, float& gy) {
  u = fminf(fmaxf(u, -2.0f), (float)W + 1.0f);
  v = fminf(fmaxf(v, -2.0f), (float)H + 1.0f);
  const float xf = floorf(u), yf = floorf(v);
  const float a = u - xf, b = v - yf;
  const int x0 = (int)xf, y0 = (int)yf;
  const int xa = min(max(x0, 0), W - 1), xb = min(max(x0 + 1, 0), W - 1);
  const int ya = min(max(y0, 0), H - 1), yb = min(max(y0 + 1, 0), H - 1);
  const float I00 = img[ya * W + xa], I10 = img[ya * W + xb];
  const float I01 = img[yb * W + xa], I11 = img[yb * W + xb];
  const float top = I00 + a * (I10 - I00);
  const float bot = I01 + a * (I11 - I01);
  I = top + b * (bot - top);
  gx = (I10 - I00) + b * ((I11 - I01) - (I10 - I00));
  gy = bot - top;
}

}  // namespace pba
