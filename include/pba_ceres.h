// include/pba_ceres.h — Ceres plug-in adapter over the C ABI of include/pba.h (header-only, C++14).
//
// Lets the reference's Ceres problem build (map_utils.h:322-383) keep ceres::Solve unchanged while every
// residual block is evaluated by the MI355X engine in one launch per evaluation point:
//
//   * GpuEvaluator       : ceres::EvaluationCallback (evaluation_callback.h:63-76).  Registered through
//                          Problem::Options::evaluation_callback (problem.h:185).  On the solver thread,
//                          after Ceres copied the state into the user's T_w_c / inv_depth memory
//                          (program_evaluator.h:157-162), it gathers poses and inverse distances, uploads
//                          them and evaluates all blocks (pba_evaluate), then copies the records (or, for a
//                          residual-only evaluation, just the residuals) back into page-locked memory.
//   * GpuBlockCost<R,…>  : ceres::SizedCostFunction per block.  Evaluate() is a re-entrant copy out of the
//                          evaluator's record buffer (Ceres calls it from num_threads workers,
//                          program_evaluator.h:187-229); returns false for invalid blocks like a functor
//                          whose projection failed (residual_block.cc:113-131).
//   * SE3TangentParameterization : ceres::LocalParameterization with the SAME Plus as the reference's
//                          LocalParameterizationSE3 (T·exp(δ), local_parameterization_se3.hpp:43-50) and
//                          Jacobian [I₆; 0].  The engine returns tangent-space Jacobians J6; the adapter
//                          exposes the 7-wide global Jacobian [J6 | 0], so Ceres' J_global·P
//                          (residual_block.cc:136-158) reproduces J6 exactly.
//
// The loss function stays with Ceres (HuberLoss is applied after Evaluate, residual_block.cc:161-196).
// Requires <ceres/ceres.h> (Ceres ≥ 2.0, which has EvaluationCallback) and include/pba.h on the include path.
#pragma once

#include <ceres/ceres.h>

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "pba.h"

namespace pba_ceres {

inline void check(int status, const char* what) {
  if (status != PBA_OK) throw std::runtime_error(std::string(what) + ": " + pba_status_string(status) + " — " + pba_last_error());
}

// Sophus SE3 storage [qx qy qz qw tx ty tz]; exp as se3.hpp:763-784, product as se3.hpp group multiplication.
inline void se3_plus(const double* T, const double* d, double* out) {
  const double w0 = d[3], w1 = d[4], w2 = d[5];
  const double th2 = w0 * w0 + w1 * w1 + w2 * w2, th = std::sqrt(th2);
  double imag, real, A, B;
  if (th < 1e-10) {
    real = 1.0 - th2 / 8.0 + th2 * th2 / 384.0;
    imag = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0;
    A = 0.5;
    B = 1.0 / 6.0;
  } else {
    real = std::cos(0.5 * th);
    imag = std::sin(0.5 * th) / th;
    A = (1.0 - std::cos(th)) / th2;
    B = (th - std::sin(th)) / (th2 * th);
  }
  const double qx = imag * w0, qy = imag * w1, qz = imag * w2, qw = real;
  const double c0 = w1 * d[2] - w2 * d[1], c1 = w2 * d[0] - w0 * d[2], c2 = w0 * d[1] - w1 * d[0];
  const double e0 = w1 * c2 - w2 * c1, e1 = w2 * c0 - w0 * c2, e2 = w0 * c1 - w1 * c0;
  const double tx = d[0] + A * c0 + B * e0, ty = d[1] + A * c1 + B * e1, tz = d[2] + A * c2 + B * e2;
  const double ax = T[0], ay = T[1], az = T[2], aw = T[3];
  const double rw = aw * qw - ax * qx - ay * qy - az * qz, rx = aw * qx + ax * qw + ay * qz - az * qy;
  const double ry = aw * qy + ay * qw + az * qx - ax * qz, rz = aw * qz + az * qw + ax * qy - ay * qx;
  const double n = 1.0 / std::sqrt(rw * rw + rx * rx + ry * ry + rz * rz);
  double u0 = ay * tz - az * ty, u1 = az * tx - ax * tz, u2 = ax * ty - ay * tx;
  u0 += u0; u1 += u1; u2 += u2;
  out[0] = rx * n; out[1] = ry * n; out[2] = rz * n; out[3] = rw * n;
  out[4] = T[4] + tx + aw * u0 + (ay * u2 - az * u1);
  out[5] = T[5] + ty + aw * u1 + (az * u0 - ax * u2);
  out[6] = T[6] + tz + aw * u2 + (ax * u1 - ay * u0);
}

class SE3TangentParameterization : public ceres::LocalParameterization {
 public:
  bool Plus(const double* x, const double* delta, double* x_plus_delta) const override {
    se3_plus(x, delta, x_plus_delta);
    return true;
  }
  bool ComputeJacobian(const double* /*x*/, double* jacobian) const override {  // 7×6 row-major [I6; 0]
    std::memset(jacobian, 0, sizeof(double) * 42);
    for (int i = 0; i < 6; ++i) jacobian[i * 6 + i] = 1.0;
    return true;
  }
  int GlobalSize() const override { return 7; }
  int LocalSize() const override { return 6; }
};

// Page-locked host array from the engine library (pba_host_alloc): the per-evaluation read-backs are DMA copies.
template <class T>
class PinnedArray {
 public:
  PinnedArray() = default;
  PinnedArray(const PinnedArray&) = delete;
  PinnedArray& operator=(const PinnedArray&) = delete;
  ~PinnedArray() { pba_host_free(p_); }
  void resize(size_t n) {
    if (n <= n_ && p_) return;
    pba_host_free(p_);
    p_ = nullptr;
    n_ = 0;
    void* q = nullptr;
    check(pba_host_alloc(n * sizeof(T), &q), "pba_host_alloc");
    p_ = static_cast<T*>(q);
    n_ = n;
  }
  T* data() { return p_; }
  const T* data() const { return p_; }
  const T& operator[](size_t i) const { return p_[i]; }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
};

class GpuEvaluator : public ceres::EvaluationCallback {
 public:
  // poses[f] = T_w_c.data() of keyframe f (7 doubles, user memory Ceres optimises in place);
  // inv_dist[p] = &landmark.inv_depth of point p.  The engine must already hold the problem structure.
  GpuEvaluator(pba_engine* engine, std::vector<double*> poses, std::vector<double*> inv_dist)
      : engine_(engine), poses_(std::move(poses)), rho_(std::move(inv_dist)) {
    R_ = pba_residuals_per_block(engine_);
    rec_ = pba_record_floats(engine_);
  }

  // Called on the solver thread after Ceres has written the evaluation point into the user's parameter memory
  // (program_evaluator.h:157-162).  A Jacobian evaluation reads back the whole records; a residual-only one (the
  // LM candidate, trust_region_minimizer.cc:761-779) only the residuals, R of every 14R record values.  The
  // evaluation after an accepted step comes with new_evaluation_point = false (trust_region_minimizer.cc:805-822):
  // when the point was already evaluated with Jacobians nothing is recomputed.
  void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) override {
    if (!new_evaluation_point && have_point_ && (have_jac_ || !evaluate_jacobians)) return;
    state_p_.resize(7 * poses_.size());
    state_r_.resize(rho_.size());
    for (size_t f = 0; f < poses_.size(); ++f) std::memcpy(&state_p_[7 * f], poses_[f], 7 * sizeof(double));
    for (size_t p = 0; p < rho_.size(); ++p) state_r_[p] = *rho_[p];
    check(pba_set_state(engine_, state_p_.data(), state_r_.data()), "pba_set_state");
    check(pba_evaluate(engine_, evaluate_jacobians ? 1 : 0), "pba_evaluate");
    const size_t nb = (size_t)pba_num_blocks(engine_);
    valid_.resize(nb);
    if (evaluate_jacobians) {
      records_.resize(nb * rec_);
      check(pba_get_records(engine_, records_.data(), valid_.data()), "pba_get_records");
      res_ = records_.data();
      res_stride_ = rec_;
    } else {
      residuals_.resize(nb * R_);
      check(pba_get_residuals(engine_, residuals_.data(), valid_.data()), "pba_get_residuals");
      res_ = residuals_.data();
      res_stride_ = R_;
    }
    have_point_ = true;
    have_jac_ = evaluate_jacobians;
  }

  int residuals_per_block() const { return R_; }
  const float* record(int block) const { return records_.data() + (size_t)block * rec_; }  // with has_jacobians()
  const float* residuals(int block) const { return res_ + (size_t)block * res_stride_; }
  bool valid(int block) const { return valid_[block] != 0; }
  bool has_jacobians() const { return have_jac_; }

 private:
  pba_engine* engine_;
  std::vector<double*> poses_, rho_;
  std::vector<double> state_p_, state_r_;
  PinnedArray<float> records_, residuals_;
  PinnedArray<uint8_t> valid_;
  const float* res_ = nullptr;
  int res_stride_ = 0;
  int R_ = 0, rec_ = 0;
  bool have_point_ = false, have_jac_ = false;
};

// Copy one block's record into Ceres' buffers.  Parameter blocks: T_w_host[7], T_w_target[7], ρ[1], and —
// for the geometric functor's signature (reprojection.h:83-86) — the target intrinsics[8] (constant in the
// reference, map_utils.h:340-345; its Jacobian is reported as zero).
inline bool copy_block(const GpuEvaluator& ev, int block, int R, double* residuals, double** jacobians, int n_intr) {
  if (!ev.valid(block)) return false;
  const float* res = ev.residuals(block);
  for (int k = 0; k < R; ++k) residuals[k] = res[k];
  if (!jacobians) return true;
  if (!ev.has_jacobians()) return false;  // Ceres asked for J at a point evaluated residual-only
  const float* rec = ev.record(block);
  for (int k = 0; k < R; ++k) {
    if (jacobians[0]) {
      for (int c = 0; c < 6; ++c) jacobians[0][k * 7 + c] = rec[R + 6 * k + c];
      jacobians[0][k * 7 + 6] = 0.0;
    }
    if (jacobians[1]) {
      for (int c = 0; c < 6; ++c) jacobians[1][k * 7 + c] = rec[7 * R + 6 * k + c];
      jacobians[1][k * 7 + 6] = 0.0;
    }
    if (jacobians[2]) jacobians[2][k] = rec[13 * R + k];
    if (n_intr && jacobians[3])
      for (int c = 0; c < n_intr; ++c) jacobians[3][k * n_intr + c] = 0.0;
  }
  return true;
}

// Photometric block: SizedCostFunction<P, 7, 7, 1> (the PhotometricError<P> signature, photometric_error.h:79-82).
template <int P>
class GpuPhotometricCost : public ceres::SizedCostFunction<P, 7, 7, 1> {
 public:
  GpuPhotometricCost(const GpuEvaluator* ev, int block) : ev_(ev), block_(block) {}
  bool Evaluate(double const* const* /*parameters*/, double* residuals, double** jacobians) const override {
    return copy_block(*ev_, block_, P, residuals, jacobians, 0);
  }

 private:
  const GpuEvaluator* ev_;
  int block_;
};

// Geometric block: SizedCostFunction<2, 7, 7, 1, 8> — the reference's AutoDiffCostFunction signature
// (map_utils.h:365-367) so AddResidualBlock(…, T_w_host, T_w_target, &inv_depth, intrinsics) is unchanged.
class GpuReprojectionCost : public ceres::SizedCostFunction<2, 7, 7, 1, 8> {
 public:
  GpuReprojectionCost(const GpuEvaluator* ev, int block) : ev_(ev), block_(block) {}
  bool Evaluate(double const* const* /*parameters*/, double* residuals, double** jacobians) const override {
    return copy_block(*ev_, block_, 2, residuals, jacobians, 8);
  }

 private:
  const GpuEvaluator* ev_;
  int block_;
};

}  // namespace pba_ceres
