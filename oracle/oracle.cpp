// oracle/oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's hot path, used exclusively as the parity checker by
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in the product
// (photometric-bundle-adjustment_amd/) links, loads or calls this file.
//
// What it restates (all arithmetic in double, Jacobians by forward-mode dual numbers exactly as
// Ceres' AutoDiffCostFunction does, then mapped to the SE3 tangent space the way
// ResidualBlock::Evaluate does):
//
//   * Jet<N> dual numbers ............ ceres-solver/include/ceres/jet.h (value + N-vector of partials)
//   * AutoDiff seeding/extraction .... ceres-solver/include/ceres/internal/autodiff.h:309-324
//   * Sophus SO3/SE3 algebra ......... Sophus/sophus/so3.hpp:329-345 (quaternion product),
//                                      so3.hpp:362-370 (rotate point), se3.hpp:208-211 (inverse),
//                                      se3.hpp:763-784 (exp), se3.hpp:135-204 (Dx_this_mul_exp_x_at_0)
//   * J_local = J_global · P ......... ceres-solver/internal/ceres/residual_block.cc:136-158
//   * LocalParameterizationSE3 ....... include/visnav/local_parameterization_se3.hpp:43-63
//   * Huber + Corrector .............. ceres-solver/internal/ceres/loss_function.cc:48-62,
//                                      corrector.cc:42-110, residual_block.cc:161-196
//   * Camera models .................. include/visnav/camera_models.h:75-107 (pinhole),
//                                      :140-190 (EUCM), :226-277 (double sphere), :316-420 (Kannala-Brandt 4)
//   * Geometric residual ............. include/visnav/reprojection.h:83-112
//                                      r = u_obs − π_t(T_w_t⁻¹ · T_w_h · (normalize(π_h⁻¹(u_ref)) / ρ))
//   * Photometric residual ........... ceres-solver/internal/ceres/autodiff_benchmarks/photometric_error.h:139-182
//                                      (q_t_h = q_w_t* q_w_h, t_t_h = q_w_t*(t_w_h − t_w_t),
//                                       p̃_k = R_t_h b_k + ρ t_t_h, r_k = I_t(π_t(p̃_k)) − I_h,k)
//                                      with the interpolator swapped for bilinear + Grid2D edge clamp
//                                      (cubic_interpolation.h:334-344 Jet chain, :403-414 clamp), which is
//                                      the north star's interpolator.  The reference's own photometric
//                                      functor lives on an absent branch (README.md:1-2), so this part of
//                                      the spec is pinned by our own fixtures.
//
// Record layout written per residual block (R = P for photometric, 2 for geometric):
//   [ r(R) | J_host(R×6) | J_target(R×6) | J_rho(R) ]   row-major, tangent δ = [υ(3), ω(3)] (Sophus order)
// Invalid blocks (projection outside the camera's domain, or a non-finite result) get valid = 0
// and an all-zero record.

#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <map>
#include <vector>
#include <algorithm>
#include <type_traits>

namespace {

// ----------------------------------------------------------------------------------------------
// Dual numbers (restates ceres/jet.h semantics for the operations the functors use)
// ----------------------------------------------------------------------------------------------
template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0) { for (int i = 0; i < N; ++i) v[i] = 0; }
  explicit Jet(double x) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; }
  Jet(double x, int k) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; v[k] = 1; }
};
template <int N> inline Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) { Jet<N> h; h.a = f.a + g.a; for (int i = 0; i < N; ++i) h.v[i] = f.v[i] + g.v[i]; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) { Jet<N> h; h.a = f.a - g.a; for (int i = 0; i < N; ++i) h.v[i] = f.v[i] - g.v[i]; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f) { Jet<N> h; h.a = -f.a; for (int i = 0; i < N; ++i) h.v[i] = -f.v[i]; return h; }
template <int N> inline Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) { Jet<N> h; h.a = f.a * g.a; for (int i = 0; i < N; ++i) h.v[i] = f.a * g.v[i] + f.v[i] * g.a; return h; }
template <int N> inline Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
  // ceres/jet.h: (a + u)/(b + v) = a/b + (u − (a/b) v)/b
  Jet<N> h; const double ib = 1.0 / g.a; h.a = f.a * ib;
  for (int i = 0; i < N; ++i) h.v[i] = (f.v[i] - h.a * g.v[i]) * ib;
  return h;
}
template <int N> inline Jet<N> operator+(const Jet<N>& f, double s) { Jet<N> h = f; h.a += s; return h; }
template <int N> inline Jet<N> operator+(double s, const Jet<N>& f) { Jet<N> h = f; h.a += s; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f, double s) { Jet<N> h = f; h.a -= s; return h; }
template <int N> inline Jet<N> operator-(double s, const Jet<N>& f) { Jet<N> h = -f; h.a += s; return h; }
template <int N> inline Jet<N> operator*(const Jet<N>& f, double s) { Jet<N> h; h.a = f.a * s; for (int i = 0; i < N; ++i) h.v[i] = f.v[i] * s; return h; }
template <int N> inline Jet<N> operator*(double s, const Jet<N>& f) { return f * s; }
template <int N> inline Jet<N> operator/(const Jet<N>& f, double s) { return f * (1.0 / s); }
template <int N> inline Jet<N> operator/(double s, const Jet<N>& g) { Jet<N> h; const double ib = 1.0 / g.a; h.a = s * ib; const double c = -h.a * ib; for (int i = 0; i < N; ++i) h.v[i] = c * g.v[i]; return h; }
// atan2(y, x): ∂/∂y = x/(x²+y²), ∂/∂x = −y/(x²+y²) (ceres/jet.h atan2)
template <int N> inline Jet<N> atan2(const Jet<N>& y, const Jet<N>& x) {
  Jet<N> h;
  h.a = std::atan2(y.a, x.a);
  const double t = 1.0 / (x.a * x.a + y.a * y.a);
  for (int i = 0; i < N; ++i) h.v[i] = t * (x.a * y.v[i] - y.a * x.v[i]);
  return h;
}
inline double atan2(double y, double x) { return std::atan2(y, x); }
template <int N> inline Jet<N> sqrt(const Jet<N>& f) { Jet<N> h; h.a = std::sqrt(f.a); const double c = 0.5 / h.a; for (int i = 0; i < N; ++i) h.v[i] = f.v[i] * c; return h; }

inline double val(double x) { return x; }
template <int N> inline double val(const Jet<N>& x) { return x.a; }
using std::sqrt;

// ----------------------------------------------------------------------------------------------
// Sophus-style quaternion / SE3 algebra.  Storage [qx qy qz qw tx ty tz] (se3.hpp:70,976-981).
// ----------------------------------------------------------------------------------------------
template <class T> struct Quat { T x, y, z, w; };

template <class T>
inline Quat<T> qmul(const Quat<T>& a, const Quat<T>& b) {  // so3.hpp:338-345
  Quat<T> r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}
template <class T> inline Quat<T> qconj(const Quat<T>& a) { Quat<T> r{-a.x, -a.y, -a.z, a.w}; return r; }

template <class T, class P>
inline void qrot(const Quat<T>& q, const P p[3], T out[3]) {  // so3.hpp:367-370
  // uv = q.vec × p ; uv += uv ; out = p + w·uv + q.vec × uv
  T uv0 = q.y * p[2] - q.z * p[1];
  T uv1 = q.z * p[0] - q.x * p[2];
  T uv2 = q.x * p[1] - q.y * p[0];
  uv0 = uv0 + uv0; uv1 = uv1 + uv1; uv2 = uv2 + uv2;
  out[0] = p[0] + q.w * uv0 + (q.y * uv2 - q.z * uv1);
  out[1] = p[1] + q.w * uv1 + (q.z * uv0 - q.x * uv2);
  out[2] = p[2] + q.w * uv2 + (q.x * uv1 - q.y * uv0);
}

template <class T>
inline void qmatrix(const Quat<T>& q, T R[9]) {  // Eigen QuaternionBase::toRotationMatrix
  const T tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
  const T twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const T txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const T tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
  R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

// 7×6 Jacobian of the parameter vector of T·exp(δ) w.r.t. δ at δ = 0 (se3.hpp:135-204,
// local_parameterization_se3.hpp:56-63).  Rows 0-3: ∂q = ½ q ⊗ (ω,0); rows 4-6: ∂t = R(q)·υ.
inline void plus_jacobian(const double* T, double J[42]) {
  const double qx = T[0], qy = T[1], qz = T[2], qw = T[3];
  std::memset(J, 0, sizeof(double) * 42);
  // ½ q ⊗ [ω; 0] : d/dω of the quaternion part
  J[0 * 6 + 3] = 0.5 * qw;  J[0 * 6 + 4] = -0.5 * qz; J[0 * 6 + 5] = 0.5 * qy;
  J[1 * 6 + 3] = 0.5 * qz;  J[1 * 6 + 4] = 0.5 * qw;  J[1 * 6 + 5] = -0.5 * qx;
  J[2 * 6 + 3] = -0.5 * qy; J[2 * 6 + 4] = 0.5 * qx;  J[2 * 6 + 5] = 0.5 * qw;
  J[3 * 6 + 3] = -0.5 * qx; J[3 * 6 + 4] = -0.5 * qy; J[3 * 6 + 5] = -0.5 * qz;
  Quat<double> q{qx, qy, qz, qw};
  double R[9];
  qmatrix(q, R);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) J[(4 + r) * 6 + c] = R[r * 3 + c];
}

// SE3::exp (se3.hpp:763-784 with SO3::expAndTheta)
inline void se3_exp(const double d[6], double out[7]) {
  const double w0 = d[3], w1 = d[4], w2 = d[5];
  const double theta_sq = w0 * w0 + w1 * w1 + w2 * w2;
  const double theta = std::sqrt(theta_sq);
  const double half = 0.5 * theta;
  double imag, real;
  if (theta < 1e-10) {  // Sophus Constants<double>::epsilon() = 1e-10
    const double th4 = theta_sq * theta_sq;
    real = 1.0 - theta_sq / 8.0 + th4 / 384.0;
    imag = 0.5 - theta_sq / 48.0 + th4 / 3840.0;
  } else {
    real = std::cos(half);
    imag = std::sin(half) / theta;
  }
  Quat<double> q{imag * w0, imag * w1, imag * w2, real};
  double V[9];
  if (theta < 1e-10) {
    qmatrix(q, V);
  } else {
    // V = I + (1−cosθ)/θ² Ω + (θ−sinθ)/θ³ Ω²
    const double Om[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double Om2[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 3; ++k) s += Om[r * 3 + k] * Om[k * 3 + c];
        Om2[r * 3 + c] = s;
      }
    const double a = (1.0 - std::cos(theta)) / theta_sq;
    const double b = (theta - std::sin(theta)) / (theta_sq * theta);
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * Om[i] + b * Om2[i];
  }
  out[0] = q.x; out[1] = q.y; out[2] = q.z; out[3] = q.w;
  for (int r = 0; r < 3; ++r) out[4 + r] = V[r * 3 + 0] * d[0] + V[r * 3 + 1] * d[1] + V[r * 3 + 2] * d[2];
}

// SE3 product a·b (se3.hpp group multiplication: q = qa⊗qb (normalised), t = ta + qa·tb)
inline void se3_mul(const double* a, const double* b, double* out) {
  Quat<double> qa{a[0], a[1], a[2], a[3]}, qb{b[0], b[1], b[2], b[3]};
  Quat<double> q = qmul(qa, qb);
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  double tb[3] = {b[4], b[5], b[6]}, rt[3];
  qrot(qa, tb, rt);
  out[0] = q.x / n; out[1] = q.y / n; out[2] = q.z / n; out[3] = q.w / n;
  out[4] = a[4] + rt[0]; out[5] = a[5] + rt[1]; out[6] = a[6] + rt[2];
}

// ----------------------------------------------------------------------------------------------
// Camera models (include/visnav/camera_models.h).  Intrinsics vector [fx fy cx cy p1 p2 p3 p4].
// ----------------------------------------------------------------------------------------------
enum { CAM_PINHOLE = 0, CAM_DS = 1, CAM_EUCM = 2, CAM_KB4 = 3 };

template <class T, class K = double>
inline void project(int model, const K* k, const T p[3], T uv[2]) {
  const K fx = k[0], fy = k[1], cx = k[2], cy = k[3];
  if (model == CAM_PINHOLE) {  // camera_models.h:75-91
    uv[0] = fx * p[0] / p[2] + cx;
    uv[1] = fy * p[1] / p[2] + cy;
  } else if (model == CAM_DS) {  // camera_models.h:226-245
    const K xi = k[4], alpha = k[5];
    const T d1 = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    const T xi_d1_z = xi * d1 + p[2];
    const T d2 = sqrt(p[0] * p[0] + p[1] * p[1] + xi_d1_z * xi_d1_z);
    const T denom = alpha * d2 + (1.0 - alpha) * (xi * d1 + p[2]);
    uv[0] = fx * p[0] / denom + cx;
    uv[1] = fy * p[1] / denom + cy;
  } else if (model == CAM_EUCM) {  // camera_models.h:140-160
    const K alpha = k[4], beta = k[5];
    const T d = sqrt(beta * (p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]);
    uv[0] = fx * p[0] / (alpha * d + (1.0 - alpha) * p[2]) + cx;
    uv[1] = fy * p[1] / (alpha * d + (1.0 - alpha) * p[2]) + cy;
  } else {  // Kannala-Brandt 4, camera_models.h:316-348
    const K k1 = k[4], k2 = k[5], k3 = k[6], k4 = k[7];
    const T r = sqrt(p[0] * p[0] + p[1] * p[1]);
    if (val(r) == 0.0) {
      uv[0] = T(cx);
      uv[1] = T(cy);
      return;
    }
    const T theta = atan2(r, p[2]);
    const T t2 = theta * theta, t3 = t2 * theta;
    const T d = theta + t3 * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4)));
    uv[0] = fx * d * p[0] / r + cx;
    uv[1] = fy * d * p[1] / r + cy;
  }
}

// Domain of the projection, evaluated on the (scaled) point.  The reference's camera_models.h has no
// check; Ceres' PhotometricError::Project has the EUCM one (photometric_error.h:114-121).  Pinhole: z > eps.
inline bool in_domain(int model, const double* k, const double p[3]) {
  if (model == CAM_PINHOLE) return p[2] > 1e-6;
  if (model == CAM_KB4) return p[2] > 0.0 || p[0] * p[0] + p[1] * p[1] > 0.0;  // all but the backward axis
  if (model == CAM_EUCM) {
    const double alpha = k[4], beta = k[5];
    const double rho = std::sqrt(beta * (p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]);
    const double w = alpha > 0.5 ? (1.0 - alpha) / alpha : alpha / (1.0 - alpha);
    return p[2] > -w * rho + 1e-10;
  }
  // double sphere (Usenko et al. 3DV'18, eq. 43)
  const double xi = k[4], alpha = k[5];
  const double d1 = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
  const double w1 = alpha <= 0.5 ? alpha / (1.0 - alpha) : (1.0 - alpha) / alpha;
  const double w2 = (w1 + xi) / std::sqrt(2.0 * w1 * xi + xi * xi + 1.0);
  return p[2] > -w2 * d1 + 1e-10;
}

inline void unproject(int model, const double* k, const double uv[2], double b[3]) {
  const double fx = k[0], fy = k[1], cx = k[2], cy = k[3];
  const double mx = (uv[0] - cx) / fx, my = (uv[1] - cy) / fy;
  if (model == CAM_PINHOLE) {  // camera_models.h:93-107
    b[0] = mx; b[1] = my; b[2] = 1.0;
  } else if (model == CAM_DS) {  // camera_models.h:247-277
    const double xi = k[4], alpha = k[5];
    const double r2 = mx * mx + my * my;
    const double mz = (1.0 - alpha * alpha * r2) /
                      (alpha * std::sqrt(1.0 - (2.0 * alpha - 1.0) * r2) + 1.0 - alpha);
    const double factor = (mz * xi + std::sqrt(mz * mz + (1.0 - xi * xi) * r2)) / (mz * mz + r2);
    b[0] = factor * mx; b[1] = factor * my; b[2] = factor * mz - xi;
  } else if (model == CAM_EUCM) {  // camera_models.h:162-190
    const double alpha = k[4], beta = k[5];
    const double r2 = mx * mx + my * my;
    b[0] = mx; b[1] = my;
    b[2] = (1.0 - beta * alpha * alpha * r2) /
           (alpha * std::sqrt(1.0 - (2.0 * alpha - 1.0) * beta * r2) + (1.0 - alpha));
  } else {  // Kannala-Brandt 4, camera_models.h:352-380 (5 Newton steps from θ = 0)
    const double ru = std::sqrt(mx * mx + my * my);
    if (ru == 0.0) {
      b[0] = 0.0; b[1] = 0.0; b[2] = 1.0;
    } else {
      const double k1 = k[4], k2 = k[5], k3 = k[6], k4 = k[7];
      double th = 0.0;
      for (int i = 0; i < 5; ++i) {
        const double t2 = th * th;
        const double f = th + t2 * th * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4))) - ru;
        const double df = 1.0 + t2 * (3.0 * k1 + t2 * (5.0 * k2 + t2 * (7.0 * k3 + t2 * 9.0 * k4)));
        th = th - f / df;
      }
      b[0] = std::sin(th) * mx / ru; b[1] = std::sin(th) * my / ru; b[2] = std::cos(th);
    }
  }
  const double n = std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);  // res /= res.norm()
  b[0] /= n; b[1] /= n; b[2] /= n;
}

// ----------------------------------------------------------------------------------------------
// Bilinear interpolation with Grid2D-style edge clamp (value + gradient from the same 4 taps).
// u = column (left→right), v = row (top→bottom).  Jet chain as cubic_interpolation.h:334-344.
// ----------------------------------------------------------------------------------------------
inline void bilinear(const uint8_t* img, int W, int H, double u, double v, double* f, double* dfdu, double* dfdv) {
  u = std::min(std::max(u, -2.0), (double)W + 1.0);
  v = std::min(std::max(v, -2.0), (double)H + 1.0);
  const double xf = std::floor(u), yf = std::floor(v);
  const double a = u - xf, b = v - yf;
  const int x0 = (int)xf, y0 = (int)yf;
  const int xa = std::min(std::max(x0, 0), W - 1), xb = std::min(std::max(x0 + 1, 0), W - 1);
  const int ya = std::min(std::max(y0, 0), H - 1), yb = std::min(std::max(y0 + 1, 0), H - 1);
  const double I00 = img[(size_t)ya * W + xa], I10 = img[(size_t)ya * W + xb];
  const double I01 = img[(size_t)yb * W + xa], I11 = img[(size_t)yb * W + xb];
  *f = (1.0 - b) * ((1.0 - a) * I00 + a * I10) + b * ((1.0 - a) * I01 + a * I11);
  *dfdu = (1.0 - b) * (I10 - I00) + b * (I11 - I01);
  *dfdv = (1.0 - a) * (I01 - I00) + a * (I11 - I10);
}
// Ceres' BiCubicInterpolator over Grid2D<uint8_t, 1> (cubic_interpolation.h:252-344): CubicHermiteSpline (:64-90)
// along the four rows of the 4×4 neighbourhood, then along the column; Grid2D::GetValue clamps indices (:403-414).
inline void hermite(double p0, double p1, double p2, double p3, double x, double* f, double* dfdx) {
  const double a = 0.5 * (-p0 + 3.0 * p1 - 3.0 * p2 + p3);
  const double b = 0.5 * (2.0 * p0 - 5.0 * p1 + 4.0 * p2 - p3);
  const double c = 0.5 * (-p0 + p2);
  const double d = p1;
  if (f) *f = d + x * (c + x * (b + x * a));
  if (dfdx) *dfdx = c + x * (2.0 * b + 3.0 * a * x);
}
inline void bicubic(const uint8_t* img, int W, int H, double u, double v, double* f, double* dfdu, double* dfdv) {
  const double r = v, c = u;  // Evaluate(r, c): row = v, column = u (photometric_error.h:175-177)
  const int row = (int)std::floor(r), col = (int)std::floor(c);
  auto get = [&](int rr, int cc) {
    rr = std::min(std::max(rr, 0), H - 1);
    cc = std::min(std::max(cc, 0), W - 1);
    return (double)img[(size_t)rr * W + cc];
  };
  double fr[4], dfr[4];
  for (int i = 0; i < 4; ++i)
    hermite(get(row - 1 + i, col - 1), get(row - 1 + i, col), get(row - 1 + i, col + 1), get(row - 1 + i, col + 2),
            c - col, &fr[i], &dfr[i]);
  hermite(fr[0], fr[1], fr[2], fr[3], r - row, f, dfdv);
  hermite(dfr[0], dfr[1], dfr[2], dfr[3], r - row, dfdu, nullptr);
}
inline void sample(int interp_kind, const uint8_t* img, int W, int H, double u, double v, double* f, double* du,
                   double* dv) {
  if (interp_kind == 1) bicubic(img, W, H, u, v, f, du, dv);
  else bilinear(img, W, H, u, v, f, du, dv);
}
template <int N>
inline Jet<N> interp(int ik, const uint8_t* img, int W, int H, const Jet<N>& u, const Jet<N>& v) {
  double f, du, dv;
  sample(ik, img, W, H, u.a, v.a, &f, &du, &dv);
  Jet<N> r(f);
  for (int i = 0; i < N; ++i) r.v[i] = du * u.v[i] + dv * v.v[i];
  return r;
}
inline double interp(int ik, const uint8_t* img, int W, int H, double u, double v) {
  double f, du, dv;
  sample(ik, img, W, H, u, v, &f, &du, &dv);
  return f;
}

}  // namespace

// ----------------------------------------------------------------------------------------------
// Problem description shared with the Python side (ctypes Structure of the same layout).
// ----------------------------------------------------------------------------------------------
extern "C" {

typedef struct {
  int32_t kind;        // 0 photometric, 1 geometric
  int32_t model;       // 0 pinhole, 1 double sphere, 2 EUCM
  int32_t n_frames, n_points, n_blocks, n_cams;
  int32_t width, height;
  int32_t P;           // patch size (photometric)
  int32_t interp;      // 0 bilinear, 1 Ceres' bicubic (photometric)
  const double* intrinsics;     // 8 × n_cams
  const int32_t* frame_cam;     // n_frames
  const uint8_t* images;        // n_frames × height × width (photometric)
  const float* pattern;         // 2 × P  (du, dv) offsets
  const int32_t* point_host;    // n_points
  const double* u_ref;          // 2 × n_points
  const float* host_intensity;  // P × n_points (photometric)
  const int32_t* block_point;   // n_blocks
  const int32_t* block_target;  // n_blocks
  const double* u_obs;          // 2 × n_blocks (geometric)
} orc_problem;

}  // extern "C"

namespace {

constexpr int NJ = 15;  // 7 (host pose) + 7 (target pose) + 1 (ρ), as AutoDiffCostFunction<…,7,7,1>
using J15 = Jet<NJ>;

inline void seed_pose(const double* p, int off, Quat<J15>& q, J15 t[3]) {
  q.x = J15(p[0], off + 0); q.y = J15(p[1], off + 1); q.z = J15(p[2], off + 2); q.w = J15(p[3], off + 3);
  t[0] = J15(p[4], off + 4); t[1] = J15(p[5], off + 5); t[2] = J15(p[6], off + 6);
}
inline void seed_pose(const double* p, int, Quat<double>& q, double t[3]) {
  q.x = p[0]; q.y = p[1]; q.z = p[2]; q.w = p[3]; t[0] = p[4]; t[1] = p[5]; t[2] = p[6];
}
inline J15 seed_rho(double r) { return J15(r, 14); }

// Geometric functor (reprojection.h:83-112).  Returns false if a result is non-finite.  intr_state (optional): the
// target intrinsics parameter blocks sIntr_c2 (8 per camera) when they differ from the ones the host unprojection
// captured (ref_intrinsics, reprojection.h:93-98; optimize_intrinsics, map_utils.h:339-345).
template <class T>
bool geometric_block(const orc_problem& pb, const double* poses, const double* rho, int b, T res[2],
                     const double* intr_state = nullptr) {
  const int pt = pb.block_point[b], tgt = pb.block_target[b], host = pb.point_host[pt];
  const double* kh = pb.intrinsics + 8 * pb.frame_cam[host];
  const double* kt = (intr_state ? intr_state : pb.intrinsics) + 8 * pb.frame_cam[tgt];
  Quat<T> qh, qt; T th[3], tt[3];
  seed_pose(poses + 7 * host, 0, qh, th);
  seed_pose(poses + 7 * tgt, 7, qt, tt);
  T r;
  if constexpr (std::is_same<T, double>::value) r = rho[pt]; else r = seed_rho(rho[pt]);
  double bear[3];
  unproject(pb.model, kh, pb.u_ref + 2 * pt, bear);  // cam1->unproject(p_2d_ref).normalize()
  T ph[3] = {bear[0] / r, bear[1] / r, bear[2] / r};
  // T_w_t⁻¹ · T_w_h · p_h  ==  R_wt* (R_wh p_h + t_wh − t_wt)
  T pw[3];
  qrot(qh, ph, pw);
  pw[0] = pw[0] + th[0]; pw[1] = pw[1] + th[1]; pw[2] = pw[2] + th[2];
  T d[3] = {pw[0] - tt[0], pw[1] - tt[1], pw[2] - tt[2]};
  T pt3[3];
  qrot(qconj(qt), d, pt3);
  T uv[2];
  project(pb.model, kt, pt3, uv);
  res[0] = pb.u_obs[2 * b + 0] - uv[0];
  res[1] = pb.u_obs[2 * b + 1] - uv[1];
  return std::isfinite(val(res[0])) && std::isfinite(val(res[1]));
}

// ∂r/∂sIntr_c2 (2×8 row-major) of the geometric functor: the point in the target frame in double, then the projection
// with dual-number intrinsics (AutoDiffCostFunction's 4th parameter block, reprojection.h:86,108).
bool geometric_intr_jacobian(const orc_problem& pb, const double* poses, const double* rho, int b,
                             const double* intr_state, double J[16]) {
  using J8 = Jet<8>;
  const int pt = pb.block_point[b], tgt = pb.block_target[b], host = pb.point_host[pt];
  const double* kh = pb.intrinsics + 8 * pb.frame_cam[host];
  const double* kt = intr_state + 8 * pb.frame_cam[tgt];
  Quat<double> qh, qt; double th[3], tt[3];
  seed_pose(poses + 7 * host, 0, qh, th);
  seed_pose(poses + 7 * tgt, 7, qt, tt);
  double bear[3];
  unproject(pb.model, kh, pb.u_ref + 2 * pt, bear);
  const double ph[3] = {bear[0] / rho[pt], bear[1] / rho[pt], bear[2] / rho[pt]};
  double pw[3];
  qrot(qh, ph, pw);
  const double d[3] = {pw[0] + th[0] - tt[0], pw[1] + th[1] - tt[1], pw[2] + th[2] - tt[2]};
  double p3[3];
  qrot(qconj(qt), d, p3);
  J8 k[8], p[3], uv[2];
  for (int i = 0; i < 8; ++i) k[i] = J8(kt[i], i);
  for (int i = 0; i < 3; ++i) p[i] = J8(p3[i]);
  project(pb.model, k, p, uv);
  for (int r = 0; r < 2; ++r)
    for (int i = 0; i < 8; ++i) J[8 * r + i] = -uv[r].v[i];
  for (int i = 0; i < 16; ++i)
    if (!std::isfinite(J[i])) return false;
  return true;
}

// Photometric functor (photometric_error.h:139-182, bilinear or bicubic interpolator, camera per frame).
template <class T>
bool photometric_block(const orc_problem& pb, const double* poses, const double* rho, int b, T* res) {
  const int pt = pb.block_point[b], tgt = pb.block_target[b], host = pb.point_host[pt];
  const double* kh = pb.intrinsics + 8 * pb.frame_cam[host];
  const double* kt = pb.intrinsics + 8 * pb.frame_cam[tgt];
  Quat<T> qh, qt; T th[3], tt[3];
  seed_pose(poses + 7 * host, 0, qh, th);
  seed_pose(poses + 7 * tgt, 7, qt, tt);
  T idist;
  if constexpr (std::is_same<T, double>::value) idist = rho[pt]; else idist = seed_rho(rho[pt]);
  const Quat<T> qct = qconj(qt);
  const Quat<T> q_th = qmul(qct, qh);  // photometric_error.h:151
  T R[9];
  qmatrix(q_th, R);                    // :152
  T d[3] = {th[0] - tt[0], th[1] - tt[1], th[2] - tt[2]};
  T t_th[3];
  qrot(qct, d, t_th);                  // :153
  const uint8_t* img = pb.images + (size_t)tgt * pb.width * pb.height;
  for (int k = 0; k < pb.P; ++k) {
    const double uvh[2] = {pb.u_ref[2 * pt] + pb.pattern[2 * k], pb.u_ref[2 * pt + 1] + pb.pattern[2 * k + 1]};
    double bk[3];
    unproject(pb.model, kh, uvh, bk);
    T p[3];
    for (int r = 0; r < 3; ++r) p[r] = R[3 * r + 0] * bk[0] + R[3 * r + 1] * bk[1] + R[3 * r + 2] * bk[2] + idist * t_th[r];
    const double pv[3] = {val(p[0]), val(p[1]), val(p[2])};
    if (!in_domain(pb.model, kt, pv)) return false;
    T uv[2];
    project(pb.model, kt, p, uv);
    const T I = interp(pb.interp, img, pb.width, pb.height, uv[0], uv[1]);
    res[k] = I - (double)pb.host_intensity[(size_t)pb.P * pt + k];
    if (!std::isfinite(val(res[k]))) return false;
  }
  return true;
}

int record_size(const orc_problem& pb) {
  const int R = pb.kind == 0 ? pb.P : 2;
  return 14 * R;
}

void eval_range(const orc_problem& pb, const double* poses, const double* rho, int want_jac, double* out,
                uint8_t* valid, int b0, int b1, const double* intr_state = nullptr) {
  const int R = pb.kind == 0 ? pb.P : 2;
  const int rec = (intr_state ? 22 : 14) * R;
  std::vector<J15> rj(R);
  std::vector<double> rd(R);
  double Ph[42], Pt[42];
  for (int b = b0; b < b1; ++b) {
    double* o = out + (size_t)rec * b;
    std::memset(o, 0, sizeof(double) * rec);
    bool ok;
    if (!want_jac) {
      ok = pb.kind == 0 ? photometric_block<double>(pb, poses, rho, b, rd.data())
                        : geometric_block<double>(pb, poses, rho, b, rd.data(), intr_state);
      if (ok) for (int k = 0; k < R; ++k) o[k] = rd[k];
    } else {
      ok = pb.kind == 0 ? photometric_block<J15>(pb, poses, rho, b, rj.data())
                        : geometric_block<J15>(pb, poses, rho, b, rj.data(), intr_state);
      if (ok && intr_state) ok = geometric_intr_jacobian(pb, poses, rho, b, intr_state, o + 14 * R);
      if (ok) {
        const int pt = pb.block_point[b];
        const int host = pb.point_host[pt], tgt = pb.block_target[b];
        plus_jacobian(poses + 7 * host, Ph);
        plus_jacobian(poses + 7 * tgt, Pt);
        for (int k = 0; k < R; ++k) {
          o[k] = rj[k].a;
          for (int c = 0; c < 6; ++c) {  // J_local = J_global(1×7) · P(7×6)   residual_block.cc:136-158
            double sh = 0, st = 0;
            for (int g = 0; g < 7; ++g) {
              sh += rj[k].v[g] * Ph[g * 6 + c];
              st += rj[k].v[7 + g] * Pt[g * 6 + c];
            }
            o[R + 6 * k + c] = sh;
            o[7 * R + 6 * k + c] = st;
          }
          o[13 * R + k] = rj[k].v[14];
        }
        for (int i = 0; i < rec; ++i)
          if (!std::isfinite(o[i])) { ok = false; break; }
        if (!ok) std::memset(o, 0, sizeof(double) * rec);
      }
    }
    if (valid) valid[b] = ok ? 1 : 0;
  }
}

}  // namespace

extern "C" {

int orc_record_size(const orc_problem* pb) { return record_size(*pb); }

// Geometric blocks with the target intrinsics as parameters (optimize_intrinsics): records of 22·R values, the last 8·R
// being ∂r/∂sIntr_c2 (R×8) evaluated at intr_state (8·n_cams); the host unprojection uses pb->intrinsics.
int orc_evaluate_intrinsics(const orc_problem* pb, const double* poses, const double* rho, const double* intr_state,
                            int want_jac, double* out, uint8_t* valid) {
  if (!pb || !poses || !rho || !out || !intr_state || pb->kind != 1 || !pb->u_obs) return -1;
  eval_range(*pb, poses, rho, want_jac, out, valid, 0, pb->n_blocks, intr_state);
  return 0;
}

// Evaluate every residual block; `out` holds n_blocks records of record_size doubles.
int orc_evaluate(const orc_problem* pb, const double* poses, const double* rho, int want_jac, double* out,
                 uint8_t* valid, int n_threads) {
  if (!pb || !poses || !rho || !out) return -1;
  if (pb->kind == 0 && (pb->P <= 0 || !pb->images || !pb->pattern || !pb->host_intensity)) return -1;
  if (pb->kind == 1 && !pb->u_obs) return -1;
  const int nb = pb->n_blocks;
  if (n_threads <= 1 || nb < 64) {
    eval_range(*pb, poses, rho, want_jac, out, valid, 0, nb);
    return 0;
  }
  std::vector<std::thread> ts;
  const int chunk = (nb + n_threads - 1) / n_threads;
  for (int t = 0; t < n_threads; ++t) {
    const int b0 = t * chunk, b1 = std::min(nb, b0 + chunk);
    if (b0 >= b1) break;
    ts.emplace_back([=] { eval_range(*pb, poses, rho, want_jac, out, valid, b0, b1); });
  }
  for (auto& th : ts) th.join();
  return 0;
}

// Huber loss + Ceres Corrector on one block (loss_function.cc:48-62, corrector.cc:42-110,
// residual_block.cc:161-196).  Returns the block cost ½ρ(s); writes the residual/Jacobian scale.
// For Huber ρ'' ≤ 0 always, so the corrector reduces to scaling r and J by √ρ'.
double orc_huber_block(const double* r, int R, double a, double* scale) {
  double s = 0;
  for (int k = 0; k < R; ++k) s += r[k] * r[k];
  const double b = a * a;
  double rho0, rho1;
  if (a <= 0) { rho0 = s; rho1 = 1.0; }
  else if (s > b) { const double rr = std::sqrt(s); rho0 = 2.0 * a * rr - b; rho1 = std::max(2.2250738585072014e-308, a / rr); }
  else { rho0 = s; rho1 = 1.0; }
  if (scale) *scale = std::sqrt(rho1);
  return 0.5 * rho0;
}

// SE3 helpers exposed for pinning against Sophus (oracle/_ref) and for finite-difference tests.
void orc_se3_exp(const double* d6, double* out7) { se3_exp(d6, out7); }
void orc_se3_mul(const double* a7, const double* b7, double* out7) { se3_mul(a7, b7, out7); }
void orc_se3_plus(const double* T7, const double* d6, double* out7) {  // LocalParameterizationSE3::Plus
  double e[7];
  se3_exp(d6, e);
  se3_mul(T7, e, out7);
}
void orc_se3_plus_jacobian(const double* T7, double* J42) { plus_jacobian(T7, J42); }
void orc_se3_act(const double* T7, const double* p3, double* out3) {
  Quat<double> q{T7[0], T7[1], T7[2], T7[3]};
  qrot(q, p3, out3);
  out3[0] += T7[4]; out3[1] += T7[5]; out3[2] += T7[6];
}
void orc_se3_inverse(const double* T7, double* out7) {  // se3.hpp:208-211
  Quat<double> q{-T7[0], -T7[1], -T7[2], T7[3]};
  const double mt[3] = {-T7[4], -T7[5], -T7[6]};
  double t[3];
  qrot(q, mt, t);
  out7[0] = q.x; out7[1] = q.y; out7[2] = q.z; out7[3] = q.w;
  out7[4] = t[0]; out7[5] = t[1]; out7[6] = t[2];
}
void orc_project(int model, const double* k8, const double* p3, double* uv2) { project<double>(model, k8, p3, uv2); }
void orc_unproject(int model, const double* k8, const double* uv2, double* b3) { unproject(model, k8, uv2, b3); }
int orc_in_domain(int model, const double* k8, const double* p3) { return in_domain(model, k8, p3) ? 1 : 0; }
void orc_sample(int interp_kind, const uint8_t* img, int W, int H, double u, double v, double* f3) {
  sample(interp_kind, img, W, H, u, v, &f3[0], &f3[1], &f3[2]);
}
void orc_bilinear(const uint8_t* img, int W, int H, double u, double v, double* f3) {
  bilinear(img, W, H, u, v, f3, f3 + 1, f3 + 2);
}

// compute_projections + set_outlier_flags (src/sfm.cpp:1928-2008), per observation.  th = [normal px, huge px,
// camera distance m, z m].  Landmark::get_p (common_types.h:205-217) then T_w_c.inverse() * p_w with Sophus
// (se3.hpp:208-211 inverse, so3.hpp:362-370 action).
int orc_compute_projections(int model, const double* intr8, const int* frame_cam, const double* poses,
                            const int* point_host, const double* u_ref, const double* rho, int n_obs,
                            const int* obs_point, const int* obs_frame, const double* obs_uv,
                            const uint8_t* obs_outlier, const double* th, double* reproj, double* pc, double* err,
                            uint32_t* flags) {
  for (int i = 0; i < n_obs; ++i) {
    const int pt = obs_point[i], f = obs_frame[i], h = point_host[pt];
    double b[3];
    unproject(model, intr8 + 8 * frame_cam[h], u_ref + 2 * pt, b);
    const double ph[3] = {b[0] / rho[pt], b[1] / rho[pt], b[2] / rho[pt]};
    double pw[3];
    orc_se3_act(poses + 7 * h, ph, pw);
    double Ti[7], p[3];
    orc_se3_inverse(poses + 7 * f, Ti);
    orc_se3_act(Ti, pw, p);
    double uv[2];
    project<double>(model, intr8 + 8 * frame_cam[f], p, uv);
    const double e = std::sqrt((obs_uv[2 * i] - uv[0]) * (obs_uv[2 * i] - uv[0]) +
                               (obs_uv[2 * i + 1] - uv[1]) * (obs_uv[2 * i + 1] - uv[1]));
    uint32_t fl = 0;
    if (!(obs_outlier && obs_outlier[i])) {
      if (e > th[1]) fl |= 1u;                                                    // OutlierReprojectionErrorHuge
      if (e > th[0]) fl |= 2u;                                                    // OutlierReprojectionErrorNormal
      if (std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]) < th[2]) fl |= 4u;   // OutlierCameraDistance
      if (p[2] < th[3]) fl |= 8u;                                                 // OutlierZCoordinate
    }
    reproj[2 * i] = uv[0];
    reproj[2 * i + 1] = uv[1];
    for (int j = 0; j < 3; ++j) pc[3 * i + j] = p[j];
    err[i] = e;
    flags[i] = fl;
  }
  return 0;
}

// remove_outlier_landmarks (src/sfm.cpp:2028-2114): track_projections as map<track, map<frame, flags>> (the
// reference's std::map<FrameCamId, …> iteration order), then the same per-track loop.  counts = [huge,
// normal, camera distance, z, any_severe].
int orc_outlier_landmarks(int n_points, int n_obs, const int* obs_point, const int* obs_frame, const uint32_t* flags,
                          const uint8_t* obs_outlier, uint8_t* remove, int* counts) {
  std::map<int, std::map<int, uint32_t>> tracks;
  for (int i = 0; i < n_obs; ++i)
    if (!(obs_outlier && obs_outlier[i])) tracks[obs_point[i]][obs_frame[i]] = flags[i];
  bool any_severe = false;
  for (const auto& kv : tracks) {
    for (const auto& o : kv.second)
      if (o.second & ~2u) { any_severe = true; break; }
    if (any_severe) break;
  }
  int huge = 0, normal = 0, dist = 0, z = 0;
  for (int p = 0; p < n_points; ++p) remove[p] = 0;
  for (const auto& kv : tracks) {
    bool rm = false, normal_counted = false;
    for (const auto& o : kv.second) {
      if (o.second & 1u) { ++huge; rm = true; break; }
      if (o.second & 2u) {
        if (!normal_counted) { ++normal; normal_counted = true; }
        if (!any_severe) { rm = true; break; }
      }
      if (o.second & 4u) { rm = true; ++dist; break; }
      if (o.second & 8u) { rm = true; ++z; break; }
    }
    remove[kv.first] = rm;
  }
  counts[0] = huge; counts[1] = normal; counts[2] = dist; counts[3] = z; counts[4] = any_severe;
  return 0;
}

}  // extern "C"
