// tests/cpp/ceres_lm_driver.cpp — TEST-ONLY: the reference's bundle_adjustment() solve (map_utils.h:322-383) run by
// the real Ceres Solver 2.0.0 (vendored in the reference, built by oracle/ceres.mk) in one of two modes:
//
//   cpu  the reference's CPU path: one ceres::AutoDiffCostFunction per residual block over the restated functor
//        (tests/cpp/ceres_functors.h), the reference's own LocalParameterizationSE3 (local_parameterization_se3.hpp).
//   gpu  the drop-in: the same Problem with include/pba_ceres.h — GpuEvaluator as Problem::Options::
//        evaluation_callback, GpuPhotometricCost / GpuReprojectionCost per block, and the reference's own
//        LocalParameterizationSE3 (pose_param "ref", the default: the adapter emits J7 = J6·P⁺) or the adapter's
//        SE3TangentParameterization ("tangent") — evaluated by the MI355X engine (libpba.so).  The evaluation-callback
//        protocol of
//        evaluation_callback_test.cc:79-160 is checked on every call (Prepare/Evaluate pairing, new_evaluation_point
//        semantics, Jacobians requested iff prepared with Jacobians, parameters equal to the prepared state).
//
// Both modes: HuberLoss(a) per block (map_utils.h:370-371), two constant keyframes (SetParameterBlockConstant,
// :334-336), constant intrinsics blocks for the geometric functor (:340-345), LEVENBERG_MARQUARDT + SPARSE_SCHUR
// (:378-381).  Writes a JSON summary: per-iteration cost / success / relative decrease, termination, final state,
// Ceres' evaluation timers and the protocol counters.
//
// With interp = 1 (bicubic) the GPU engine uses Ceres' BiCubicInterpolator arithmetic (pba_set_interpolator) and the
// CPU mode, for an EUCM camera, runs the vendored ceres::PhotometricError<8> itself (photometric_error.h:79-189) —
// the whole CPU side is then reference-held code.
//
// optimize_intrinsics = 1 (geometric): the intrinsics blocks are free (map_utils.h:339-345); the CPU functor keeps
// unprojecting with the captured pointer (user memory, which Ceres does not write during a solve without a callback),
// the GPU evaluator gets the blocks and enables the engine's target-intrinsics Jacobian.
//
// floor: the drop-in's floor on the drop-in's own trajectory — the gpu-mode Solve is run once while every evaluation's
//        read-back (records or residuals, validity, the poses' P⁺) is recorded, then the SAME Solve (same Problem, the
//        same GpuPhotometricCost / GpuReprojectionCost per block, the reference's LocalParameterizationSE3, Huber) is
//        run again from the same initial state with an evaluator that only points the adapter at the recorded arrays:
//        the same values give Ceres the same decisions, so both runs make the same evaluations, and "Jacobian &
//        residual evaluation" of the second run is Ceres' own work (ProgramEvaluator, the Jacobian writer, the
//        LocalParameterization products, the loss) plus the adapter's per-block copy out of its own read-back buffers
//        (staged with the recorded values between iterations, outside Ceres' timers) and its P⁺ — everything but the
//        device's part (state gather and upload, launch, read-back).  The summary is the second run's, with "replay_ok" saying whether it took
//        exactly the recorded evaluations.
// check = 0 (gpu mode): the plain adapter, without the protocol checks (the bench's C2 timing: the checks hash the whole
//        state per Prepare and count every Evaluate with an atomic shared by Ceres' threads).
//
//   usage: ceres_lm_driver <cpu|gpu|floor> <problem.bin> <out.json> [iters] [huber] [threads] [fixed,frames] [ftol]
//                          [interp] [ptol] [gtol] [optimize_intrinsics] [pose_param ref|tangent] [check 1|0]
//                          [teacher states file | -]
// teacher (cpu mode): one LM iteration from each of a list of states, each with its own initial trust-region radius —
//        the engine's iterates, so that every iteration of its solve is checked against Ceres' own step from the same
//        point (the "teacher" array of the JSON: [cost at the state, cost after the iteration, step_is_successful,
//        relative_decrease, radius after, step_norm, iterations pushed, gradient max norm at the state] per state).
//          (problem layout: tests/golden/make_golden.py write_problem)
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <immintrin.h>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "ceres_functors.h"
#include "local_parameterization_se3.hpp"  // the reference's (include/visnav/), compiled where it lies
#include "pba_ceres.h"
#include "photometric_error.h"              // ceres-solver/internal/ceres/autodiff_benchmarks/

namespace {

template <class T>
std::vector<T> rd(FILE* f, size_t n) {
  std::vector<T> v(n);
  if (n && fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "short read\n");
    exit(2);
  }
  return v;
}

uint64_t djb2(const double* p, size_t n, uint64_t h = 5381) {  // evaluation_callback_test.cc:45-56
  const unsigned char* c = reinterpret_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n * sizeof(double); ++i) h = h * 33 + c[i];
  return h;
}

struct Protocol {
  std::atomic<long> violations{0}, evaluate_calls{0};
  long prepare_calls = 0, evaluate_calls_at_prepare = 0;
  bool requested_jacobians = false, new_point = false;
  uint64_t hash = 0;
  std::vector<double> state;  // user state snapshot at the last Prepare
  std::string log;            // "J"/"r" + "n"/"s" per Prepare (jacobians?, new point?)
};

// GpuEvaluator with the checks of evaluation_callback_test.cc:79-112 (Prepare side).
class CheckedEvaluator : public pba_ceres::GpuEvaluator {
 public:
  CheckedEvaluator(pba_engine* e, std::vector<double*> poses, std::vector<double*> rho, std::vector<double*> intr,
                   pba_ceres::PoseJacobian form, int n_blocks, Protocol* pr)
      : GpuEvaluator(e, poses, rho, intr, form), poses_(poses), rho_(rho), nb_(n_blocks), pr_(pr) {}
  void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) override {
    Protocol& p = *pr_;
    std::vector<double> st;
    st.reserve(7 * poses_.size() + rho_.size());
    for (double* q : poses_) st.insert(st.end(), q, q + 7);
    for (double* r : rho_) st.push_back(*r);
    const uint64_t h = djb2(st.data(), st.size());
    // Prepare() and a full pass of Evaluate() calls alternate
    if (p.prepare_calls > 0 && p.evaluate_calls.load() - p.evaluate_calls_at_prepare != nb_) ++p.violations;
    if (p.prepare_calls > 0) {
      if (new_evaluation_point && h == p.hash) ++p.violations;   // a new point has new parameters
      if (!new_evaluation_point && h != p.hash) ++p.violations;  // the same point has the same parameters
    }
    p.prepare_calls++;
    p.evaluate_calls_at_prepare = p.evaluate_calls.load();
    p.requested_jacobians = evaluate_jacobians;
    p.new_point = new_evaluation_point;
    p.hash = h;
    p.state = std::move(st);
    p.log += evaluate_jacobians ? 'J' : 'r';
    p.log += new_evaluation_point ? 'n' : 's';
    GpuEvaluator::PrepareForEvaluation(evaluate_jacobians, new_evaluation_point);
  }

 private:
  std::vector<double*> poses_, rho_;
  long nb_;
  Protocol* pr_;
};

// The per-block side of evaluation_callback_test.cc:113-160 around the adapter's CostFunction.
class CheckedCost : public ceres::CostFunction {
 public:
  CheckedCost(ceres::CostFunction* inner, Protocol* pr, int host, int target, int point, int nf)
      : inner_(inner), pr_(pr), host_(host), target_(target), point_(point), nf_(nf) {
    set_num_residuals(inner->num_residuals());
    *mutable_parameter_block_sizes() = inner->parameter_block_sizes();
  }
  bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const override {
    Protocol& p = *pr_;
    p.evaluate_calls++;
    bool ok = p.requested_jacobians == (jacobians != nullptr);
    ok = ok && std::memcmp(parameters[0], &p.state[7 * host_], 7 * sizeof(double)) == 0;
    ok = ok && std::memcmp(parameters[1], &p.state[7 * target_], 7 * sizeof(double)) == 0;
    ok = ok && parameters[2][0] == p.state[7 * (size_t)nf_ + point_];
    if (!ok) ++p.violations;
    return inner_->Evaluate(parameters, residuals, jacobians);
  }

 private:
  std::unique_ptr<ceres::CostFunction> inner_;
  Protocol* pr_;
  int host_, target_, point_, nf_;
};

// The floor (mode floor): what one PrepareForEvaluation left for Evaluate to read — nothing when the adapter kept the
// previous point (same point, no new work).
// The arrays are page-locked host memory from the engine library, as the drop-in's own read-back buffers.
struct Snapshot {
  bool kept = false, jac = false;
  std::unique_ptr<pba_ceres::PinnedArray<float>> rec;     // records (jac) or residuals
  std::unique_ptr<pba_ceres::PinnedArray<uint8_t>> valid;
  std::vector<double> pinv;    // the poses' P⁺ (jac, reference parameterisation)
};

// Pass 1: the drop-in, recording every evaluation's read-back (waits for the whole read-back: untimed pass).
class RecordingEvaluator : public pba_ceres::GpuEvaluator {
 public:
  RecordingEvaluator(pba_engine* e, std::vector<double*> poses, std::vector<double*> rho, std::vector<double*> intr,
                     pba_ceres::PoseJacobian form, int n_blocks, int n_frames, std::vector<Snapshot>* out)
      : GpuEvaluator(e, poses, rho, intr, form), nb_(n_blocks), nf_(n_frames), out_(out) {}
  void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) override {
    const long before = prepare_times().calls[0] + prepare_times().calls[1];
    GpuEvaluator::PrepareForEvaluation(evaluate_jacobians, new_evaluation_point);
    Snapshot s;
    s.kept = prepare_times().calls[0] + prepare_times().calls[1] == before;
    if (!s.kept) {
      s.jac = has_jacobians();
      for (int b = 0; b < nb_; b += chunk_blocks_) wait(b);
      const int R = residuals_per_block(), rf = pba_record_floats(engine_);
      const size_t n = (size_t)nb_ * (s.jac ? rf : R);
      s.rec.reset(new pba_ceres::PinnedArray<float>);
      s.rec->resize(n);
      std::memcpy(s.rec->data(), s.jac ? record(0) : residuals(0), n * sizeof(float));
      s.valid.reset(new pba_ceres::PinnedArray<uint8_t>);
      s.valid->resize(nb_);
      std::memcpy(s.valid->data(), valid_src_, nb_);
      if (s.jac && pose_jacobian() == pba_ceres::PoseJacobian::kReferenceSE3) s.pinv.assign(pinv_src_, pinv_src_ + 42 * nf_);
    }
    out_->push_back(std::move(s));
  }

 private:
  int nb_, nf_;
  std::vector<Snapshot>* out_;
};

// Pass 2: the same adapter with the device's part (state gather, upload, launch, read-back) removed.  Its Evaluate reads
// the adapter's own page-locked read-back buffers, as the drop-in does, which hold the recorded values of the
// evaluation Ceres is about to make: they are staged outside Ceres' evaluation timers — before the Solve and in an
// IterationCallback after each iteration (an iteration makes at most one residual-only and one Jacobian evaluation, into
// two different buffers).  P⁺ is formed from the state in PrepareForEvaluation, as the drop-in forms it.
class ReplayEvaluator : public pba_ceres::GpuEvaluator, public ceres::IterationCallback {
 public:
  ReplayEvaluator(pba_engine* e, std::vector<double*> poses, std::vector<double*> rho, std::vector<double*> intr,
                  pba_ceres::PoseJacobian form, const std::vector<Snapshot>* snaps)
      : GpuEvaluator(e, poses, rho, intr, form), snaps_(snaps) {
    valid_r_.resize((size_t)pba_num_blocks(e));
    stage();
  }
  ceres::CallbackReturnType operator()(const ceres::IterationSummary&) override {
    stage();
    return ceres::SOLVER_CONTINUE;
  }
  void PrepareForEvaluation(bool evaluate_jacobians, bool /*new_evaluation_point*/) override {
    if (next_ >= snaps_->size()) {
      ok_ = false;
      return;
    }
    const size_t i = next_++;
    const Snapshot& s = (*snaps_)[i];
    if (s.kept) return;
    if (s.jac != evaluate_jacobians) ok_ = false;
    async_ = false;
    if (s.jac) {
      if (staged_j_ != i) ok_ = false;
      rec_src_ = res_ = records_.data();
      res_stride_ = rec_;
      valid_src_ = valid_.data();
      if (form_ == pba_ceres::PoseJacobian::kReferenceSE3) {
        pinv_.resize(42 * poses_.size());
        for (size_t f = 0; f < poses_.size(); ++f) pba_ceres::se3_plus_jacobian_pinv(poses_[f], &pinv_[42 * f]);
        pinv_src_ = pinv_.data();
      }
    } else {
      if (staged_r_ != i) ok_ = false;
      rec_src_ = nullptr;
      res_ = residuals_.data();
      res_stride_ = R_;
      valid_src_ = valid_r_.data();
    }
    have_point_ = true;
    have_jac_ = s.jac;
  }
  bool replay_ok() const { return ok_ && next_ == snaps_->size(); }

 private:
  // the next residual-only and the next Jacobian evaluation from next_ on, into the read-back buffers
  // PBA_FLOOR_COLD=1 (diagnostic): the staged arrays are flushed from the CPU caches after staging, as the drop-in's
  // read-back arrives by DMA into memory no core has cached — the floor then differs from the drop-in by the device's
  // part only, not also by where the records are read from.
  static void evict(const void* p, size_t bytes) {
    const char* c = static_cast<const char*>(p);
    for (size_t o = 0; o < bytes; o += 64) _mm_clflush(c + o);
    _mm_mfence();
  }
  void stage() {
    static const bool cold = std::getenv("PBA_FLOOR_COLD") != nullptr;
    bool r = false, j = false;
    for (size_t i = next_; i < snaps_->size() && !(r && j); ++i) {
      const Snapshot& s = (*snaps_)[i];
      if (s.kept) continue;
      const size_t nb = (size_t)pba_num_blocks(engine_);
      if (s.jac && !j) {
        if (staged_j_ != i) {
          std::memcpy(records_.data(), s.rec->data(), nb * rec_ * sizeof(float));
          std::memcpy(valid_.data(), s.valid->data(), nb);
          if (cold) {
            evict(records_.data(), nb * rec_ * sizeof(float));
            evict(valid_.data(), nb);
          }
          staged_j_ = i;
        }
        j = true;
      } else if (!s.jac && !r) {
        if (staged_r_ != i) {
          std::memcpy(residuals_.data(), s.rec->data(), nb * R_ * sizeof(float));
          std::memcpy(valid_r_.data(), s.valid->data(), nb);
          if (cold) {
            evict(residuals_.data(), nb * R_ * sizeof(float));
            evict(valid_r_.data(), nb);
          }
          staged_r_ = i;
        }
        r = true;
      }
    }
  }
  const std::vector<Snapshot>* snaps_;
  pba_ceres::PinnedArray<uint8_t> valid_r_;
  size_t next_ = 0, staged_r_ = (size_t)-1, staged_j_ = (size_t)-1;
  bool ok_ = true;
};

// ceres::PhotometricError<8> throws outside the EUCM domain (photometric_error.h:165-171); inside a solve that is an
// invalid evaluation (residual_block.cc:113-131): return false instead.
struct CeresPhotometric {
  explicit CeresPhotometric(ceres::PhotometricError<8>* f) : f_(f) {}
  template <class T>
  bool operator()(const T* const h, const T* const t, const T* const r, T* res) const {
    try {
      return (*f_)(h, t, r, res);
    } catch (const std::runtime_error&) {
      return false;
    }
  }
  std::unique_ptr<ceres::PhotometricError<8>> f_;
};

void json_array(std::ostringstream& o, const double* v, size_t n) {
  o << "[";
  char buf[40];
  for (size_t i = 0; i < n; ++i) {
    snprintf(buf, sizeof buf, "%.17g", v[i]);
    o << (i ? "," : "") << buf;
  }
  o << "]";
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <cpu|gpu> <problem.bin> <out.json> [iters] [huber] [threads] [fixed] [ftol]\n", argv[0]);
    return 1;
  }
  const bool gpu = std::string(argv[1]) == "gpu";
  const bool floor_mode = std::string(argv[1]) == "floor";
  const int iters = argc > 4 ? atoi(argv[4]) : 20;
  const double huber = argc > 5 ? atof(argv[5]) : 1.0;
  const int threads = argc > 6 ? atoi(argv[6]) : 8;
  std::vector<int> fixed;
  if (argc > 7 && argv[7][0] != '-') {
    std::stringstream ss(argv[7]);
    std::string tok;
    while (std::getline(ss, tok, ',')) fixed.push_back(atoi(tok.c_str()));
  }
  const double ftol = argc > 8 ? atof(argv[8]) : 1e-6;
  const int interp = argc > 9 ? atoi(argv[9]) : 0;
  const double ptol = argc > 10 ? atof(argv[10]) : 1e-8;
  const double gtol = argc > 11 ? atof(argv[11]) : 1e-10;
  // 0: constant intrinsics blocks; 1: free, given to the GPU evaluator; 2: free but NOT given to it (the adapter must
  // refuse the Jacobian request instead of reporting a zero gradient)
  const int intr_mode = argc > 12 ? atoi(argv[12]) : 0;
  const bool opt_intr = intr_mode != 0;
  const bool tangent = argc > 13 && std::string(argv[13]) == "tangent";
  const bool checked = !(argc > 14 && atoi(argv[14]) == 0);
  // teacher file (cpu mode): n states of [poses (7·nf) | ρ (np) | trust-region radius] doubles; one LM iteration of the
  // Solve from each (Solver::Options::initial_trust_region_radius = that radius) instead of the one solve
  const char* teacher_path = argc > 15 && std::string(argv[15]) != "-" ? argv[15] : nullptr;

  FILE* f = fopen(argv[2], "rb");
  if (!f) return 2;
  const auto hdr = rd<int32_t>(f, 9);
  const int kind = hdr[0], model = hdr[1], nf = hdr[2], np = hdr[3], nb = hdr[4], nc = hdr[5], W = hdr[6], H = hdr[7];
  const int P = hdr[8];
  auto intr = rd<double>(f, 8 * nc);
  const auto frame_cam = rd<int32_t>(f, nf);
  const auto images = rd<uint8_t>(f, kind == 0 ? (size_t)nf * W * H : 0);
  const auto pattern = rd<float>(f, kind == 0 ? 2 * P : 0);
  const auto point_host = rd<int32_t>(f, np);
  const auto u_ref = rd<double>(f, 2 * np);
  const auto host_int = rd<float>(f, kind == 0 ? (size_t)P * np : 0);
  const auto block_point = rd<int32_t>(f, nb);
  const auto block_target = rd<int32_t>(f, nb);
  const auto u_obs = rd<double>(f, kind == 1 ? 2 * nb : 0);
  const auto poses_in = rd<double>(f, 7 * nf);
  std::vector<double> rho = rd<double>(f, np);
  fclose(f);
  if (kind == 0 && P != 8) {
    fprintf(stderr, "driver is built for P = 8\n");
    return 3;
  }

  // user memory, as the reference keeps it (Camera::T_w_c, Landmark::inv_depth, calib intrinsics)
  std::vector<Sophus::SE3d> T(nf);
  for (int i = 0; i < nf; ++i) std::memcpy(T[i].data(), &poses_in[7 * i], 7 * sizeof(double));
  std::vector<double*> pose_ptr(nf), rho_ptr(np);
  for (int i = 0; i < nf; ++i) pose_ptr[i] = T[i].data();
  for (int p = 0; p < np; ++p) rho_ptr[p] = &rho[p];

  Protocol protocol;
  pba_engine* e = nullptr;
  std::unique_ptr<pba_ceres::GpuEvaluator> ev;
  const bool engine = gpu || floor_mode;
  std::vector<double*> intr_ptr;
  const auto form = tangent ? pba_ceres::PoseJacobian::kTangent : pba_ceres::PoseJacobian::kReferenceSE3;
  if (engine) {
    pba_options opt{0, kind, model, 0.0f};
    pba_ceres::check(pba_create(&opt, &e), "pba_create");
    pba_ceres::check(pba_set_cameras(e, nc, intr.data()), "cameras");
    pba_ceres::check(pba_set_frames(e, nf, frame_cam.data(), W, H, kind == 0 ? images.data() : nullptr), "frames");
    if (kind == 0) pba_ceres::check(pba_set_pattern(e, P, pattern.data()), "pattern");
    if (kind == 0) pba_ceres::check(pba_set_interpolator(e, interp), "interpolator");
    pba_ceres::check(pba_set_points(e, np, point_host.data(), u_ref.data(), kind == 0 ? host_int.data() : nullptr),
                     "points");
    pba_ceres::check(pba_set_blocks(e, nb, block_point.data(), block_target.data(), kind == 1 ? u_obs.data() : nullptr),
                     "blocks");
    if (intr_mode == 1)
      for (int c = 0; c < nc; ++c) intr_ptr.push_back(&intr[8 * c]);
  }
  // CPU photometric: one interpolator per keyframe image, host bearings per point
  using PE = ceres::PhotometricError<8>;
  const bool ceres_pe = !engine && kind == 0 && interp == 1 && model == pba_test::CAM_EUCM;
  if (!engine && kind == 0 && interp == 1 && !ceres_pe) {
    fprintf(stderr, "cpu mode: bicubic is the vendored PhotometricError<8>, EUCM cameras only\n");
    return 3;
  }
  std::vector<std::unique_ptr<pba_test::BilinearInterpolator>> bilin;
  std::vector<std::unique_ptr<pba_test::Grid>> grids;
  std::vector<std::unique_ptr<pba_test::BicubicInterpolator>> bicub;
  std::vector<Eigen::Matrix<double, 3, 8>, Eigen::aligned_allocator<Eigen::Matrix<double, 3, 8>>> bearings;
  std::vector<PE::Patch<double>, Eigen::aligned_allocator<PE::Patch<double>>> patches;
  std::vector<PE::Intrinsics, Eigen::aligned_allocator<PE::Intrinsics>> K6(nc);
  for (int c = 0; c < nc; ++c) K6[c] << intr[8 * c], intr[8 * c + 1], intr[8 * c + 2], intr[8 * c + 3], intr[8 * c + 4], intr[8 * c + 5];
  std::vector<double> host_int_d;
  if (!engine && kind == 0) {
    for (int i = 0; i < nf; ++i) {
      bilin.emplace_back(new pba_test::BilinearInterpolator(&images[(size_t)i * W * H], H, W));
      grids.emplace_back(new pba_test::Grid(&images[(size_t)i * W * H], 0, H, 0, W));
      bicub.emplace_back(new pba_test::BicubicInterpolator(*grids.back()));
    }
    bearings.resize(np);
    patches.resize(np);
    host_int_d.assign(host_int.begin(), host_int.end());
    for (int p = 0; p < np; ++p)
      for (int k = 0; k < 8; ++k) {
        bearings[p].col(k) = pba_test::Unproject(model, &intr[8 * frame_cam[point_host[p]]],
                                                 Eigen::Vector2d(u_ref[2 * p] + pattern[2 * k], u_ref[2 * p + 1] + pattern[2 * k + 1]));
        patches[p][k] = host_int[(size_t)8 * p + k];
      }
  }

  ceres::Solver::Options so;  // map_utils.h:376-381
  so.max_num_iterations = iters;
  so.linear_solver_type = ceres::SPARSE_SCHUR;
  so.num_threads = threads;
  so.function_tolerance = ftol;
  so.parameter_tolerance = ptol;
  so.gradient_tolerance = gtol;
  ceres::Solver::Summary sum;
  // bundle_adjustment()'s problem build (map_utils.h:322-375) over the evaluator ev (nullptr: AutoDiff on the CPU),
  // then ceres::Solve (:376-383)
  auto solve = [&](pba_ceres::GpuEvaluator* evaluator, bool checked_costs, ceres::IterationCallback* cb = nullptr) {
    ceres::Problem::Options popt;
    popt.evaluation_callback = evaluator;  // problem.h:185 (not owned)
    ceres::Problem problem(popt);
    for (int i = 0; i < nf; ++i) {  // map_utils.h:330-337
      ceres::LocalParameterization* lp =
          evaluator && tangent ? static_cast<ceres::LocalParameterization*>(new pba_ceres::SE3TangentParameterization)
                               : new Sophus::test::LocalParameterizationSE3;  // the reference's own, in both modes
      problem.AddParameterBlock(T[i].data(), 7, lp);
    }
    for (int i : fixed) problem.SetParameterBlockConstant(T[i].data());
    if (kind == 1 && !opt_intr)
      for (int c = 0; c < nc; ++c) {  // :340-345
        problem.AddParameterBlock(&intr[8 * c], 8);
        problem.SetParameterBlockConstant(&intr[8 * c]);
      }
    for (int b = 0; b < nb; ++b) {  // :347-375
      const int p = block_point[b], h = point_host[p], t = block_target[b];
      ceres::LossFunction* loss = huber > 0 ? new ceres::HuberLoss(huber) : nullptr;
      ceres::CostFunction* cf;
      if (evaluator) {
        ceres::CostFunction* inner = kind == 0 ? static_cast<ceres::CostFunction*>(new pba_ceres::GpuPhotometricCost<8>(evaluator, b, h, t))
                                               : new pba_ceres::GpuReprojectionCost(evaluator, b, h, t);
        cf = checked_costs ? new CheckedCost(inner, &protocol, h, t, p, nf) : inner;
      } else if (kind == 1) {
        cf = new ceres::AutoDiffCostFunction<pba_test::GeometricFunctor, 2, 7, 7, 1, 8>(new pba_test::GeometricFunctor(
            Eigen::Vector2d(u_obs[2 * b], u_obs[2 * b + 1]), Eigen::Vector2d(u_ref[2 * p], u_ref[2 * p + 1]),
            &intr[8 * frame_cam[h]], model));
      } else if (ceres_pe) {  // the vendored functor itself (it keeps references to the patch, bearings, image, K)
        cf = new ceres::AutoDiffCostFunction<CeresPhotometric, 8, 7, 7, 1>(
            new CeresPhotometric(new PE(patches[p], bearings[p], *bicub[t], K6[frame_cam[t]])));
      } else {
        using F = pba_test::PhotometricFunctor<8, pba_test::BilinearInterpolator>;
        cf = new ceres::AutoDiffCostFunction<F, 8, 7, 7, 1>(
            new F(&host_int_d[(size_t)8 * p], bearings[p], *bilin[t], &intr[8 * frame_cam[t]], model));
      }
      if (kind == 1)
        problem.AddResidualBlock(cf, loss, T[h].data(), T[t].data(), &rho[p], &intr[8 * frame_cam[t]]);
      else
        problem.AddResidualBlock(cf, loss, T[h].data(), T[t].data(), &rho[p]);
    }
    ceres::Solver::Options o = so;
    if (cb) o.callbacks.push_back(cb);
    ceres::Solve(o, &problem, &sum);
  };

  int replay_ok = -1;
  std::string teacher_json = "null";
  if (floor_mode) {
    // pass 1: the drop-in, recording its read-backs; then the same Solve from the same initial state over the recording
    std::vector<Snapshot> snaps;
    const std::vector<double> rho0 = rho, intr0 = intr;
    {
      RecordingEvaluator rec(e, pose_ptr, rho_ptr, intr_ptr, form, nb, nf, &snaps);
      solve(&rec, false);
    }
    for (int i = 0; i < nf; ++i) std::memcpy(T[i].data(), &poses_in[7 * i], 7 * sizeof(double));
    rho = rho0;
    intr = intr0;
    std::unique_ptr<ReplayEvaluator> rep(new ReplayEvaluator(e, pose_ptr, rho_ptr, intr_ptr, form, &snaps));
    solve(rep.get(), false, rep.get());
    replay_ok = rep->replay_ok() ? 1 : 0;
    ev = std::move(rep);
  } else if (gpu) {
    if (checked)
      ev.reset(new CheckedEvaluator(e, pose_ptr, rho_ptr, intr_ptr, form, nb, &protocol));
    else
      ev.reset(new pba_ceres::GpuEvaluator(e, pose_ptr, rho_ptr, intr_ptr, form));
    solve(ev.get(), checked);
  } else if (teacher_path) {
    FILE* tf = fopen(teacher_path, "rb");
    if (!tf) return 2;
    const size_t per = 7 * (size_t)nf + np + 1;
    std::vector<double> st;
    for (;;) {
      std::vector<double> v(per);
      if (fread(v.data(), sizeof(double), per, tf) != per) break;
      st.insert(st.end(), v.begin(), v.end());
    }
    fclose(tf);
    const int n_states = (int)(st.size() / per);
    const int iters_saved = so.max_num_iterations;
    so.max_num_iterations = 1;
    std::ostringstream tj;
    tj << "[";
    for (int q = 0; q < n_states; ++q) {
      const double* v = &st[(size_t)q * per];
      for (int i = 0; i < nf; ++i) std::memcpy(T[i].data(), v + 7 * i, 7 * sizeof(double));
      for (int p = 0; p < np; ++p) rho[p] = v[7 * (size_t)nf + p];
      so.initial_trust_region_radius = v[per - 1];
      solve(nullptr, false);
      char buf[400];
      const auto& it0 = sum.iterations.front();
      const auto& it1 = sum.iterations.back();
      snprintf(buf, sizeof buf, "%s[%.17g,%.17g,%d,%.17g,%.17g,%.17g,%d,%.17g]", q ? "," : "", it0.cost, it1.cost,
               it1.step_is_successful ? 1 : 0, it1.relative_decrease, it1.trust_region_radius, it1.step_norm,
               (int)sum.iterations.size(), it0.gradient_max_norm);
      tj << buf;
    }
    tj << "]";
    teacher_json = tj.str();
    so.max_num_iterations = iters_saved;
  } else {
    solve(nullptr, false);
  }

  std::ostringstream o;
  o << "{\"mode\":\"" << argv[1] << "\",\"checked\":" << (gpu && checked ? 1 : 0) << ",\"termination\":" << (int)sum.termination_type
    << ",\"message\":\"" << sum.message << "\",\"successful_steps\":" << sum.num_successful_steps
    << ",\"unsuccessful_steps\":" << sum.num_unsuccessful_steps << ",\"iterations\":[";
  for (size_t i = 0; i < sum.iterations.size(); ++i) {
    const auto& it = sum.iterations[i];
    char buf[300];
    snprintf(buf, sizeof buf, "%s[%d,%.17g,%d,%.17g,%.17g,%.17g,%.17g]", i ? "," : "", it.iteration, it.cost,
             it.step_is_successful ? 1 : 0, it.relative_decrease, it.trust_region_radius, it.step_norm,
             it.gradient_max_norm);
    o << buf;
  }
  char buf[400];
  snprintf(buf, sizeof buf, "],\"initial_cost\":%.17g,\"final_cost\":%.17g", sum.initial_cost, sum.final_cost);
  o << buf;
  snprintf(buf, sizeof buf,
           ",\"jacobian_evaluation_s\":%.6g,\"jacobian_evaluations\":%d,\"residual_evaluation_s\":%.6g,"
           "\"residual_evaluations\":%d,\"linear_solver_s\":%.6g,\"minimizer_s\":%.6g,\"total_s\":%.6g,\"threads\":%d",
           sum.jacobian_evaluation_time_in_seconds, sum.num_jacobian_evaluations, sum.residual_evaluation_time_in_seconds,
           sum.num_residual_evaluations, sum.linear_solver_time_in_seconds, sum.minimizer_time_in_seconds,
           sum.total_time_in_seconds, sum.num_threads_used);
  o << buf;
  o << ",\"protocol\":{\"prepare_calls\":" << protocol.prepare_calls << ",\"evaluate_calls\":" << protocol.evaluate_calls.load()
    << ",\"violations\":" << protocol.violations.load() << ",\"log\":\"" << protocol.log << "\"}";
  std::vector<double> pf(7 * (size_t)nf);
  for (int i = 0; i < nf; ++i) std::memcpy(&pf[7 * i], T[i].data(), 7 * sizeof(double));
  o << ",\"poses\":";
  json_array(o, pf.data(), pf.size());
  o << ",\"rho\":";
  json_array(o, rho.data(), rho.size());
  o << ",\"intrinsics\":";
  json_array(o, intr.data(), intr.size());
  o << ",\"refused_intrinsics\":" << (ev && ev->refused_intrinsics() ? 1 : 0) << ",\"replay_ok\":" << replay_ok;
  o << ",\"teacher\":" << teacher_json;
  if (ev) {  // the adapter's own breakdown of PrepareForEvaluation ([residual-only, with Jacobians], seconds)
    const auto& t = ev->prepare_times();
    snprintf(buf, sizeof buf,
             ",\"prepare\":{\"calls\":[%ld,%ld],\"gather_s\":[%.6g,%.6g],\"launch_s\":[%.6g,%.6g],"
             "\"readback_wait_s\":[%.6g,%.6g],\"post_s\":[%.6g,%.6g],\"evaluate_wait_s\":%.6g,"
             "\"evaluate_call_s\":[%.6g,%.6g]}",
             t.calls[0], t.calls[1], t.gather_s[0], t.gather_s[1], t.launch_s[0], t.launch_s[1], t.readback_wait_s[0],
             t.readback_wait_s[1], t.post_s[0], t.post_s[1], ev->evaluate_wait_s(), t.evaluate_call_s[0],
             t.evaluate_call_s[1]);
    o << buf;
  }
  o << "}\n";
  FILE* g = fopen(argv[3], "w");
  if (!g) return 4;
  fputs(o.str().c_str(), g);
  fclose(g);
  ev.reset();
  if (e) pba_destroy(e);
  return 0;
}
