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
//   * Pose Jacobians.  The engine returns tangent-space Jacobians J6 (∂r/∂δ with T ⊞ δ = T·exp(δ)).  Ceres multiplies
//     the 7-wide global Jacobian a CostFunction returns by the LocalParameterization's 7×6 Jacobian P
//     (residual_block.cc:136-158), so the adapter writes J7 = J6·P⁺ with P⁺ = (PᵀP)⁻¹Pᵀ and P the reference's own
//     Sophus::test::LocalParameterizationSE3::ComputeJacobian = Dx_this_mul_exp_x_at_0 (local_parameterization_se3.hpp:
//     56-63, se3.hpp:135-203) at the evaluation point: J7·P = J6 for any full-rank P, so the reference's
//     bundle_adjustment() keeps its LocalParameterizationSE3 registered unchanged (map_utils.h:331-333).
//     Alternatively (PoseJacobian::kTangent) the adapter writes [J6 | 0] for SE3TangentParameterization: the SAME
//     Plus (T·exp(δ), local_parameterization_se3.hpp:43-50) with Jacobian [I₆; 0] — no per-frame P⁺ to form.
//   * Intrinsics (geometric): given the cameras' intrinsics parameter blocks, the evaluator enables the engine's target-
//     intrinsics Jacobian (pba_set_optimize_intrinsics) and uploads the blocks' current values before every
//     evaluation, so Ceres may leave them free (BundleAdjustmentOptions::optimize_intrinsics, map_utils.h:339-345).
//     Without them, a Jacobian request for an intrinsics block is refused: that Evaluate returns false and Ceres
//     stops with FAILURE instead of optimising with a zero gradient.
//
// The loss function stays with Ceres (HuberLoss is applied after Evaluate, residual_block.cc:161-196).
// Requires <ceres/ceres.h> (Ceres ≥ 2.0, which has EvaluationCallback) and include/pba.h on the include path.
#pragma once

#include <ceres/ceres.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
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

// Sophus SE3::Dx_this_mul_exp_x_at_0 (se3.hpp:135-203), 7×6 row-major: rows [q(4) | t(3)], columns [υ(3) | ω(3)];
// the quaternion rows are ½·(q ⊗ ·) on ω, the translation rows R(q) on υ.
inline void se3_plus_jacobian(const double* T, double* P) {
  const double x = T[0], y = T[1], z = T[2], w = T[3];
  for (int i = 0; i < 42; ++i) P[i] = 0.0;
  const double hx = 0.5 * x, hy = 0.5 * y, hz = 0.5 * z, hw = 0.5 * w;
  P[0 * 6 + 3] = hw;  P[0 * 6 + 4] = -hz; P[0 * 6 + 5] = hy;
  P[1 * 6 + 3] = hz;  P[1 * 6 + 4] = hw;  P[1 * 6 + 5] = -hx;
  P[2 * 6 + 3] = -hy; P[2 * 6 + 4] = hx;  P[2 * 6 + 5] = hw;
  P[3 * 6 + 3] = -hx; P[3 * 6 + 4] = -hy; P[3 * 6 + 5] = -hz;
  const double ww = w * w, xx = x * x, yy = y * y, zz = z * z;
  P[4 * 6 + 0] = ww + xx - yy - zz;     P[4 * 6 + 1] = 2 * (x * y - w * z); P[4 * 6 + 2] = 2 * (w * y + x * z);
  P[5 * 6 + 0] = 2 * (w * z + x * y);   P[5 * 6 + 1] = ww - xx + yy - zz;   P[5 * 6 + 2] = 2 * (y * z - w * x);
  P[6 * 6 + 0] = 2 * (x * z - w * y);   P[6 * 6 + 1] = 2 * (w * x + y * z); P[6 * 6 + 2] = ww - xx - yy + zz;
}

// M = (PᵀP)⁻¹Pᵀ (6×7 row-major), the left inverse of P above: MP = I₆.  PᵀP is block diagonal (the υ columns only touch
// the translation rows, the ω columns only the quaternion rows), so its inverse is two 3×3 inverses.
inline void se3_plus_jacobian_pinv(const double* T, double* M) {
  double P[42];
  se3_plus_jacobian(T, P);
  for (int i = 0; i < 42; ++i) M[i] = 0.0;
  for (int blk = 0; blk < 2; ++blk) {
    const int c0 = 3 * blk, r0 = blk == 0 ? 4 : 0, nr = blk == 0 ? 3 : 4;
    double A[9];  // PᵀP block
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double a = 0.0;
        for (int r = r0; r < r0 + nr; ++r) a += P[r * 6 + c0 + i] * P[r * 6 + c0 + j];
        A[3 * i + j] = a;
      }
    const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02, id = 1.0 / det;
    const double Ai[9] = {c00 * id, (A[2] * A[7] - A[1] * A[8]) * id, (A[1] * A[5] - A[2] * A[4]) * id,
                          c01 * id, (A[0] * A[8] - A[2] * A[6]) * id, (A[2] * A[3] - A[0] * A[5]) * id,
                          c02 * id, (A[1] * A[6] - A[0] * A[7]) * id, (A[0] * A[4] - A[1] * A[3]) * id};
    for (int i = 0; i < 3; ++i)
      for (int r = r0; r < r0 + nr; ++r) {
        double m = 0.0;
        for (int j = 0; j < 3; ++j) m += Ai[3 * i + j] * P[r * 6 + c0 + j];
        M[(c0 + i) * 7 + r] = m;
      }
  }
}

enum class PoseJacobian {
  kReferenceSE3,  // J7 = J6·P⁺ for the reference's Sophus::test::LocalParameterizationSE3 (default)
  kTangent        // [J6 | 0] for SE3TangentParameterization
};

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
  // inv_dist[p] = &landmark.inv_depth of point p; intrinsics[c] = calib_cam.intrinsics[c]->data() (8 doubles) when the
  // geometric problem's intrinsics blocks may be free (optimize_intrinsics), else empty.  The engine must already hold
  // the problem structure.
  GpuEvaluator(pba_engine* engine, std::vector<double*> poses, std::vector<double*> inv_dist,
               std::vector<double*> intrinsics = {}, PoseJacobian pose_jacobian = PoseJacobian::kReferenceSE3)
      : engine_(engine), poses_(std::move(poses)), rho_(std::move(inv_dist)), intr_(std::move(intrinsics)),
        form_(pose_jacobian) {
    if (pba_record_format(engine_) != PBA_RECORD_F32)
      throw std::runtime_error("pba_ceres: fp16 records saturate at ±65504; the adapter needs PBA_RECORD_F32");
    if (!intr_.empty()) check(pba_set_optimize_intrinsics(engine_, 1), "pba_set_optimize_intrinsics");
    R_ = pba_residuals_per_block(engine_);
    rec_ = pba_record_floats(engine_);
    // the page-locked read-back and state buffers are allocated (and mapped for the device) here, with the problem,
    // rather than inside the first evaluation Ceres times
    const size_t nb = (size_t)pba_num_blocks(engine_);
    records_.resize(nb * rec_);
    residuals_.resize(nb * R_);
    valid_.resize(nb);
    state_p_.resize(7 * poses_.size());
    state_r_.resize(rho_.size());
  }

  // Called on the solver thread after Ceres has written the evaluation point into the user's parameter memory
  // (program_evaluator.h:157-162).  A Jacobian evaluation reads back the whole records; a residual-only one (the
  // LM candidate, trust_region_minimizer.cc:761-779) only the residuals, R of every 14R record values.  The
  // evaluation after an accepted step comes with new_evaluation_point = false (trust_region_minimizer.cc:805-822):
  // when the point was already evaluated with Jacobians nothing is recomputed.
  // Where PrepareForEvaluation's time goes (seconds, summed over calls; [0] residual-only, [1] with Jacobians):
  // gather = the state into page-locked memory (+ the previous read-back's stream drain), launch = uploads + launch +
  // enqueued read-back, wait = the residual-only read-back's wait (Jacobian read-backs are waited for per chunk by
  // Evaluate on Ceres' threads: wait_s, summed over those threads).  Ceres times all of it inside "Residual only
  // evaluation" / "Jacobian & residual evaluation" (program_evaluator.h:145-162).
  struct PrepareTimes {
    double gather_s[2] = {0, 0}, launch_s[2] = {0, 0}, readback_wait_s[2] = {0, 0}, post_s[2] = {0, 0};
    double evaluate_call_s[2] = {0, 0};  // the pba_evaluate call alone (part of launch_s)
    long calls[2] = {0, 0};
  };
  const PrepareTimes& prepare_times() const { return times_; }
  double evaluate_wait_s() const { return 1e-9 * (double)wait_ns_.load(); }

  void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) override {
    if (!new_evaluation_point && have_point_ && (have_jac_ || !evaluate_jacobians)) return;
    using clk = std::chrono::steady_clock;
    const int m = evaluate_jacobians ? 1 : 0;
    const auto t0 = clk::now();
    // the state is gathered into page-locked memory, so pba_set_state's uploads are DMA copies that do not stage
    // through a driver buffer; the launch is enqueued right behind them
    const size_t nf = poses_.size(), np = rho_.size();
    if (async_) check(pba_synchronize(engine_), "pba_synchronize");  // the last upload from these buffers is done
    state_p_.resize(7 * nf);
    state_r_.resize(np);
    double* sp = state_p_.data();
    double* sr = state_r_.data();
    for (size_t f = 0; f < nf; ++f) std::memcpy(sp + 7 * f, poses_[f], 7 * sizeof(double));
    for (size_t p = 0; p < np; ++p) sr[p] = *rho_[p];
    check(pba_set_state(engine_, sp, sr), "pba_set_state");
    if (!intr_.empty()) {
      state_k_.resize(8 * intr_.size());
      for (size_t c = 0; c < intr_.size(); ++c) std::memcpy(&state_k_[8 * c], intr_[c], 8 * sizeof(double));
      check(pba_set_intrinsics_state(engine_, state_k_.data()), "pba_set_intrinsics_state");
    }
    const auto t1 = clk::now();
    check(pba_evaluate(engine_, evaluate_jacobians ? 1 : 0), "pba_evaluate");
    times_.evaluate_call_s[m] += std::chrono::duration<double>(clk::now() - t1).count();
    const size_t nb = (size_t)pba_num_blocks(engine_);
    auto t2 = clk::now(), t3 = t2;
    valid_.resize(nb);
    if (evaluate_jacobians) {
      // chunked asynchronous read-back: each block's Evaluate waits only for its chunk (wait()), so Ceres' per-block
      // work overlaps the rest of the transfer
      records_.resize(nb * rec_);
      check(pba_get_records_async(engine_, records_.data(), valid_.data(), chunk_blocks_), "pba_get_records_async");
      async_ = true;
      rec_src_ = res_ = records_.data();
      res_stride_ = rec_;
      t2 = t3 = clk::now();
      if (form_ == PoseJacobian::kReferenceSE3) {  // P⁺ of every pose at this point, while the launch and copies run
        pinv_.resize(42 * nf);
        for (size_t f = 0; f < nf; ++f) se3_plus_jacobian_pinv(sp + 7 * f, &pinv_[42 * f]);
        pinv_src_ = pinv_.data();
      }
    } else {
      t2 = clk::now();
      // residual-only: the launch also writes the residuals contiguously, so this is one plain D2H copy of 4R bytes per
      // block (not a pitched copy out of the records)
      residuals_.resize(nb * R_);
      check(pba_get_residuals(engine_, residuals_.data(), valid_.data()), "pba_get_residuals");
      async_ = false;
      rec_src_ = nullptr;
      res_ = residuals_.data();
      res_stride_ = R_;
      t3 = clk::now();
    }
    valid_src_ = valid_.data();
    const auto t4 = clk::now();
    auto sec = [](clk::duration d) { return std::chrono::duration<double>(d).count(); };
    times_.gather_s[m] += sec(t1 - t0);
    times_.launch_s[m] += sec(t2 - t1);
    times_.readback_wait_s[m] += sec(t3 - t2);
    times_.post_s[m] += sec(t4 - t3);
    times_.calls[m]++;
    have_point_ = true;
    have_jac_ = evaluate_jacobians;
  }

  // Block `block`'s record (and validity) has arrived in host memory; called by Evaluate on Ceres' worker threads.
  void wait(int block) const {
    if (!async_) return;
    const auto t0 = std::chrono::steady_clock::now();
    check(pba_wait_records(engine_, block), "pba_wait_records");
    const long long ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    if (ns > 1000) wait_ns_.fetch_add(ns, std::memory_order_relaxed);  // (an arrived chunk returns in ~100 ns)
  }
  static constexpr int kChunkBlocks = 4096;
  // blocks per read-back chunk (PBA_CERES_CHUNK_BLOCKS overrides kChunkBlocks: diagnostic)
  int chunk_blocks_ = std::getenv("PBA_CERES_CHUNK_BLOCKS") ? std::atoi(std::getenv("PBA_CERES_CHUNK_BLOCKS")) : kChunkBlocks;

  int residuals_per_block() const { return R_; }
  const float* record(int block) const { return rec_src_ + (size_t)block * rec_; }  // with has_jacobians()
  const float* residuals(int block) const { return res_ + (size_t)block * res_stride_; }
  bool valid(int block) const { return valid_src_[block] != 0; }
  bool has_jacobians() const { return have_jac_; }
  bool has_intrinsics() const { return !intr_.empty(); }
  PoseJacobian pose_jacobian() const { return form_; }
  const double* pose_pinv(int frame) const { return pinv_src_ + 42 * (size_t)frame; }  // P⁺ (6×7) at the prepared point
  // a Jacobian was requested for an intrinsics block the evaluator was not given (Evaluate returned false)
  bool refused_intrinsics() const { return refused_.load(); }
  void refuse_intrinsics() const { refused_.store(true); }

 protected:
  // What Evaluate reads (record / residuals / valid / pose_pinv): the read-back buffers below after a
  // PrepareForEvaluation; a derived evaluator may point them at host arrays of its own (tests/cpp/ceres_lm_driver.cpp's
  // replay floor: the same per-block copy with the device's work removed).
  const float* rec_src_ = nullptr;
  const uint8_t* valid_src_ = nullptr;
  const double* pinv_src_ = nullptr;
  pba_engine* engine_;
  std::vector<double*> poses_, rho_, intr_;
  PoseJacobian form_;
  bool async_ = false;
  std::vector<double> state_k_, pinv_;
  PinnedArray<double> state_p_, state_r_;
  mutable std::atomic<bool> refused_{false};
  mutable std::atomic<long long> wait_ns_{0};
  PrepareTimes times_;
  PinnedArray<float> records_, residuals_;
  PinnedArray<uint8_t> valid_;
  const float* res_ = nullptr;
  int res_stride_ = 0;
  int R_ = 0, rec_ = 0;
  bool have_point_ = false, have_jac_ = false;
};

// One pose block's global Jacobian (R×7 row-major) from the record's tangent rows J6 (stride 6).  P⁺ (6×7) has two
// non-zero blocks — the υ rows touch only the translation columns, the ω rows only the quaternion columns
// (se3_plus_jacobian_pinv) — so J7 = J6·P⁺ is a 3×4 and a 3×3 product per row: the same sums as the full 6×7 product,
// whose other terms are exact zeros, in half the multiply-adds.
template <int R>
inline void pose_jacobian_7(const GpuEvaluator& ev, int frame, const float* j6, double* out) {
  if (ev.pose_jacobian() == PoseJacobian::kTangent) {
    for (int k = 0; k < R; ++k) {
      for (int c = 0; c < 6; ++c) out[k * 7 + c] = j6[6 * k + c];
      out[k * 7 + 6] = 0.0;
    }
    return;
  }
  const double* M = ev.pose_pinv(frame);
  double mq[12], mt[9];  // ω rows × q columns, υ rows × t columns
  for (int c = 0; c < 3; ++c) {
    for (int g = 0; g < 4; ++g) mq[4 * c + g] = M[(3 + c) * 7 + g];
    for (int g = 0; g < 3; ++g) mt[3 * c + g] = M[c * 7 + 4 + g];
  }
  for (int k = 0; k < R; ++k) {
    const float* a = j6 + 6 * k;
    const double a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3], a4 = a[4], a5 = a[5];
    double* o = out + 7 * k;
    for (int g = 0; g < 4; ++g) o[g] = a3 * mq[g] + a4 * mq[4 + g] + a5 * mq[8 + g];
    for (int g = 0; g < 3; ++g) o[4 + g] = a0 * mt[g] + a1 * mt[3 + g] + a2 * mt[6 + g];
  }
}

// Copy one block's record into Ceres' buffers.  Parameter blocks: T_w_host[7], T_w_target[7], ρ[1], and — for the
// geometric functor's signature (reprojection.h:83-86) — the target intrinsics[8] (n_intr = 8).
template <int R>
inline bool copy_block(const GpuEvaluator& ev, int block, int host, int target, double* residuals, double** jacobians,
                       int n_intr) {
  ev.wait(block);
  if (!ev.valid(block)) return false;
  const float* res = ev.residuals(block);
  for (int k = 0; k < R; ++k) residuals[k] = res[k];
  if (!jacobians) return true;
  if (!ev.has_jacobians()) return false;  // Ceres asked for J at a point evaluated residual-only
  if (n_intr && jacobians[3] && !ev.has_intrinsics()) {  // a free intrinsics block the engine was not told about
    ev.refuse_intrinsics();
    return false;
  }
  const float* rec = ev.record(block);
  if (jacobians[0]) pose_jacobian_7<R>(ev, host, rec + R, jacobians[0]);
  if (jacobians[1]) pose_jacobian_7<R>(ev, target, rec + 7 * R, jacobians[1]);
  if (jacobians[2])
    for (int k = 0; k < R; ++k) jacobians[2][k] = rec[13 * R + k];
  if (n_intr && jacobians[3])  // ∂r/∂sIntr_c2, the record's tail (pba_set_optimize_intrinsics)
    for (int i = 0; i < R * n_intr; ++i) jacobians[3][i] = rec[14 * R + i];
  return true;
}

// Photometric block: SizedCostFunction<P, 7, 7, 1> (the PhotometricError<P> signature, photometric_error.h:79-82).
template <int P>
class GpuPhotometricCost : public ceres::SizedCostFunction<P, 7, 7, 1> {
 public:
  GpuPhotometricCost(const GpuEvaluator* ev, int block, int host, int target)
      : ev_(ev), block_(block), host_(host), target_(target) {}
  bool Evaluate(double const* const* /*parameters*/, double* residuals, double** jacobians) const override {
    return copy_block<P>(*ev_, block_, host_, target_, residuals, jacobians, 0);
  }

 private:
  const GpuEvaluator* ev_;
  int block_, host_, target_;
};

// Geometric block: SizedCostFunction<2, 7, 7, 1, 8> — the reference's AutoDiffCostFunction signature
// (map_utils.h:365-367) so AddResidualBlock(…, T_w_host, T_w_target, &inv_depth, intrinsics) is unchanged.
class GpuReprojectionCost : public ceres::SizedCostFunction<2, 7, 7, 1, 8> {
 public:
  GpuReprojectionCost(const GpuEvaluator* ev, int block, int host, int target)
      : ev_(ev), block_(block), host_(host), target_(target) {}
  bool Evaluate(double const* const* /*parameters*/, double* residuals, double** jacobians) const override {
    return copy_block<2>(*ev_, block_, host_, target_, residuals, jacobians, 8);
  }

 private:
  const GpuEvaluator* ev_;
  int block_, host_, target_;
};

}  // namespace pba_ceres
