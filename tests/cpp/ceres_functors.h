// tests/cpp/ceres_functors.h — TEST-ONLY CPU cost functors for the real-Ceres runs of tests/cpp/ceres_lm_driver.cpp.
//
// They restate the reference's functor arithmetic for ceres::AutoDiffCostFunction (the reference's own headers
// cannot be compiled here: include/visnav/camera_models.h and reprojection.h include common_types.h, which needs
// TBB, common_types.h:43-44):
//   GeometricFunctor   = BundleAdjustmentReprojectionCostFunctor (include/visnav/reprojection.h:74-118)
//   PhotometricFunctor = ceres::PhotometricError (internal/ceres/autodiff_benchmarks/photometric_error.h:139-182)
//                        with the camera model of the problem and the bilinear interpolator of the north star
//                        (or Ceres' own BiCubicInterpolator)
//   camera models      = include/visnav/camera_models.h (pinhole :75-107, EUCM :140-190, DS :226-277, KB4 :316-380)
// The SE3 algebra is the reference's vendored Sophus, the interpolation Jet chain is Ceres' (cubic_interpolation.h
// :334-344), the local parameterisation in the CPU runs is the reference's LocalParameterizationSE3.
#pragma once

#include <ceres/ceres.h>
#include <ceres/cubic_interpolation.h>

#include <Eigen/Core>
#include <Eigen/Geometry>
#include <algorithm>
#include <cmath>
#include <sophus/se3.hpp>

namespace pba_test {

enum { CAM_PINHOLE = 0, CAM_DS = 1, CAM_EUCM = 2, CAM_KB4 = 3 };

inline double Val(double x) { return x; }
template <int N>
inline double Val(const ceres::Jet<double, N>& x) { return x.a; }

// camera_models.h project(), templated on the intrinsics' and the point's scalar types (Jets or doubles)
template <class K, class T>
Eigen::Matrix<T, 2, 1> Project(int model, const K* k, const Eigen::Matrix<T, 3, 1>& p) {
  using std::atan2;
  using std::sqrt;
  const T x = p[0], y = p[1], z = p[2];
  Eigen::Matrix<T, 2, 1> uv;
  if (model == CAM_KB4) {  // :316-348
    const T r = sqrt(x * x + y * y);
    if (Val(r) == 0.0) {
      uv << T(k[2]), T(k[3]);
      return uv;
    }
    const T th = atan2(r, z), t2 = th * th;
    const T d = th + t2 * th * (k[4] + t2 * (k[5] + t2 * (k[6] + t2 * k[7])));
    uv << k[0] * d * x / r + k[2], k[1] * d * y / r + k[3];
    return uv;
  }
  T den;
  if (model == CAM_PINHOLE) {  // :75-91
    den = z;
  } else if (model == CAM_DS) {  // :226-245
    const T d1 = sqrt(x * x + y * y + z * z);
    const T kk = k[4] * d1 + z;
    const T d2 = sqrt(x * x + y * y + kk * kk);
    den = k[5] * d2 + (1.0 - k[5]) * kk;
  } else {  // EUCM :140-160
    den = k[4] * sqrt(k[5] * (x * x + y * y) + z * z) + (1.0 - k[4]) * z;
  }
  uv << k[0] * x / den + k[2], k[1] * y / den + k[3];
  return uv;
}

// Projection domain (photometric_error.h:114-121 for EUCM; the same rule for the others as oracle/oracle.cpp)
inline bool InDomain(int model, const double* k, const Eigen::Vector3d& p) {
  if (model == CAM_PINHOLE) return p[2] > 1e-6;
  if (model == CAM_KB4) return p[2] > 0.0 || p[0] * p[0] + p[1] * p[1] > 0.0;
  if (model == CAM_EUCM) {
    const double rr = std::sqrt(k[5] * (p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]);
    const double w = k[4] > 0.5 ? (1.0 - k[4]) / k[4] : k[4] / (1.0 - k[4]);
    return p[2] > -w * rr + 1e-10;
  }
  const double d1 = p.norm();
  const double w1 = k[5] <= 0.5 ? k[5] / (1.0 - k[5]) : (1.0 - k[5]) / k[5];
  const double w2 = (w1 + k[4]) / std::sqrt(2.0 * w1 * k[4] + k[4] * k[4] + 1.0);
  return p[2] > -w2 * d1 + 1e-10;
}

// camera_models.h unproject() + normalize() (reprojection.h:104-105), double (the host intrinsics are constants)
inline Eigen::Vector3d Unproject(int model, const double* k, const Eigen::Vector2d& uv) {
  const double mx = (uv[0] - k[2]) / k[0], my = (uv[1] - k[3]) / k[1], r2 = mx * mx + my * my;
  Eigen::Vector3d b;
  if (model == CAM_PINHOLE) {  // :93-107
    b << mx, my, 1.0;
  } else if (model == CAM_DS) {  // :247-277
    const double xi = k[4], al = k[5];
    const double mz = (1.0 - al * al * r2) / (al * std::sqrt(1.0 - (2.0 * al - 1.0) * r2) + 1.0 - al);
    const double f = (mz * xi + std::sqrt(mz * mz + (1.0 - xi * xi) * r2)) / (mz * mz + r2);
    b << f * mx, f * my, f * mz - xi;
  } else if (model == CAM_EUCM) {  // :162-190
    const double al = k[4], be = k[5];
    b << mx, my, (1.0 - be * al * al * r2) / (al * std::sqrt(1.0 - (2.0 * al - 1.0) * be * r2) + (1.0 - al));
  } else {  // KB4 :352-380, 5 Newton steps from θ = 0
    const double ru = std::sqrt(r2);
    if (ru == 0.0) return Eigen::Vector3d(0, 0, 1);
    double th = 0.0;
    for (int i = 0; i < 5; ++i) {
      const double t2 = th * th;
      const double f = th + t2 * th * (k[4] + t2 * (k[5] + t2 * (k[6] + t2 * k[7]))) - ru;
      const double df = 1.0 + t2 * (3.0 * k[4] + t2 * (5.0 * k[5] + t2 * (7.0 * k[6] + t2 * 9.0 * k[7])));
      th -= f / df;
    }
    b << std::sin(th) * mx / ru, std::sin(th) * my / ru, std::cos(th);
  }
  return b.normalized();
}

// Bilinear interpolator of a u8 image with Grid2D's edge clamp (cubic_interpolation.h:403-414), same calling
// convention as Ceres' BiCubicInterpolator::Evaluate (row, column) including the Jet chain (:334-344).
class BilinearInterpolator {
 public:
  BilinearInterpolator(const uint8_t* img, int rows, int cols) : img_(img), rows_(rows), cols_(cols) {}
  void Evaluate(double r, double c, double* f, double* dfdr, double* dfdc) const {
    r = std::min(std::max(r, -2.0), rows_ + 1.0);
    c = std::min(std::max(c, -2.0), cols_ + 1.0);
    const double r0 = std::floor(r), c0 = std::floor(c), b = r - r0, a = c - c0;
    const int ra = clamp((int)r0, rows_), rb = clamp((int)r0 + 1, rows_);
    const int ca = clamp((int)c0, cols_), cb = clamp((int)c0 + 1, cols_);
    const double I00 = img_[(size_t)ra * cols_ + ca], I01 = img_[(size_t)ra * cols_ + cb];
    const double I10 = img_[(size_t)rb * cols_ + ca], I11 = img_[(size_t)rb * cols_ + cb];
    *f = (1.0 - b) * ((1.0 - a) * I00 + a * I01) + b * ((1.0 - a) * I10 + a * I11);
    if (dfdc) *dfdc = (1.0 - b) * (I01 - I00) + b * (I11 - I10);
    if (dfdr) *dfdr = (1.0 - a) * (I10 - I00) + a * (I11 - I01);
  }
  void Evaluate(double r, double c, double* f) const { Evaluate(r, c, f, nullptr, nullptr); }
  template <typename JetT>
  void Evaluate(const JetT& r, const JetT& c, JetT* f) const {
    double frc, dfdr, dfdc;
    Evaluate(r.a, c.a, &frc, &dfdr, &dfdc);
    f->a = frc;
    f->v = dfdr * r.v + dfdc * c.v;
  }

 private:
  static int clamp(int i, int n) { return std::min(std::max(i, 0), n - 1); }
  const uint8_t* img_;
  int rows_, cols_;
};

using Grid = ceres::Grid2D<uint8_t, 1>;
using BicubicInterpolator = ceres::BiCubicInterpolator<Grid>;

// BundleAdjustmentReprojectionCostFunctor (reprojection.h:74-118): r = u_obs − π_t(T_w_t⁻¹ T_w_h (b/ρ)),
// parameters (T_w_host[7], T_w_target[7], inv_depth[1], target intrinsics[8]); host intrinsics captured.
struct GeometricFunctor {
  GeometricFunctor(const Eigen::Vector2d& u_obs, const Eigen::Vector2d& u_ref, const double* host_intr, int model)
      : u_obs(u_obs), bearing(Unproject(model, host_intr, u_ref)), model(model) {}
  template <class T>
  bool operator()(const T* const sT_w_h, const T* const sT_w_t, const T* const inv_depth, const T* const intr_t,
                  T* sres) const {
    Eigen::Map<Sophus::SE3<T> const> const T_w_h(sT_w_h);
    Eigen::Map<Sophus::SE3<T> const> const T_w_t(sT_w_t);
    Eigen::Map<Eigen::Matrix<T, 2, 1>> res(sres);
    const Eigen::Matrix<T, 3, 1> p = T_w_t.inverse() * T_w_h * (bearing.cast<T>() / inv_depth[0]);
    res = u_obs.cast<T>() - Project(model, intr_t, p);
    return true;
  }
  Eigen::Vector2d u_obs;
  Eigen::Vector3d bearing;
  int model;
};

// PhotometricError<P> (photometric_error.h:139-182) for the problem's camera model and interpolator:
// p̃_k = R_th b_k + ρ t_th, r_k = I_t(π(p̃_k)) − I_h,k; false outside the projection domain.
template <int P, class Interp>
struct PhotometricFunctor {
  PhotometricFunctor(const double* I_h, const Eigen::Matrix<double, 3, P>& bearings, const Interp& image,
                     const double* intr_t, int model)
      : bearings(bearings), image(image), intr(intr_t), model(model) {
    for (int k = 0; k < P; ++k) intensities[k] = I_h[k];
  }
  template <class T>
  bool operator()(const T* const pose_h, const T* const pose_t, const T* const idist, T* res) const {
    Eigen::Map<const Eigen::Quaternion<T>> q_w_h(pose_h);
    Eigen::Map<const Eigen::Matrix<T, 3, 1>> t_w_h(pose_h + 4);
    Eigen::Map<const Eigen::Quaternion<T>> q_w_t(pose_t);
    Eigen::Map<const Eigen::Matrix<T, 3, 1>> t_w_t(pose_t + 4);
    const Eigen::Quaternion<T> q_t_h = q_w_t.conjugate() * q_w_h;
    const Eigen::Matrix<T, 3, 3> R_t_h = q_t_h.toRotationMatrix();
    const Eigen::Matrix<T, 3, 1> t_t_h = q_w_t.conjugate() * (t_w_h - t_w_t);
    for (int k = 0; k < P; ++k) {
      const Eigen::Matrix<T, 3, 1> p = R_t_h * bearings.col(k).template cast<T>() + idist[0] * t_t_h;
      if (!InDomain(model, intr, Eigen::Vector3d(Val(p[0]), Val(p[1]), Val(p[2])))) return false;
      const Eigen::Matrix<T, 2, 1> uv = Project(model, intr, p);
      T I;
      image.Evaluate(uv[1], uv[0], &I);  // (row, column), photometric_error.h:175-177
      res[k] = I - T(intensities[k]);
    }
    return true;
  }
  double intensities[P];
  Eigen::Matrix<double, 3, P> bearings;
  const Interp& image;
  const double* intr;
  int model;
};

}  // namespace pba_test
