// Drives include/pba_ceres.h the way Ceres' ProgramEvaluator/ResidualBlock would (program_evaluator.h:157-237,
// residual_block.cc:69-158): PrepareForEvaluation, then per block CostFunction::Evaluate with the reference's
// parameter pointers, then J_local = J_global · LocalParameterization::ComputeJacobian.  Writes the tangent
// records for comparison with the oracle (tests/test_ceres_adapter.py).
//   pose_param "ref" (default): the 7-wide Jacobians are composed with Sophus' Dx_this_mul_exp_x_at_0 at each block's
//   frames (se3_plus_jacobian, the product of the reference's LocalParameterizationSE3); "tangent": with the adapter's
//   SE3TangentParameterization.  The 7×6 P of frame 0 is written too (the test pins it against Sophus' own).
//   usage: adapter_driver <problem.bin> <out.bin> [ref|tangent]    (problem layout: tests/golden/make_golden.py)
#include <array>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "pba_ceres.h"

template <class T>
static std::vector<T> rd(FILE* f, size_t n) {
  std::vector<T> v(n);
  if (n && fread(v.data(), sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) return 1;
  const bool tangent = argc > 3 && std::string(argv[3]) == "tangent";
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  const auto hdr = rd<int32_t>(f, 9);
  const int kind = hdr[0], model = hdr[1], nf = hdr[2], np = hdr[3], nb = hdr[4], nc = hdr[5], W = hdr[6], H = hdr[7], P = hdr[8];
  const auto intr = rd<double>(f, 8 * nc);
  const auto frame_cam = rd<int32_t>(f, nf);
  const auto images = rd<uint8_t>(f, kind == 0 ? (size_t)nf * W * H : 0);
  const auto pattern = rd<float>(f, kind == 0 ? 2 * P : 0);
  const auto point_host = rd<int32_t>(f, np);
  const auto u_ref = rd<double>(f, 2 * np);
  const auto host_int = rd<float>(f, kind == 0 ? (size_t)P * np : 0);
  const auto block_point = rd<int32_t>(f, nb);
  const auto block_target = rd<int32_t>(f, nb);
  const auto u_obs = rd<double>(f, kind == 1 ? 2 * nb : 0);
  auto poses_flat = rd<double>(f, 7 * nf);
  auto rho = rd<double>(f, np);
  fclose(f);
  if (kind == 0 && P != 8) { fprintf(stderr, "driver is built for P = 8\n"); return 3; }

  pba_options opt{0, kind, model, 0.0f};
  pba_engine* e = nullptr;
  pba_ceres::check(pba_create(&opt, &e), "pba_create");
  pba_ceres::check(pba_set_cameras(e, nc, intr.data()), "cameras");
  pba_ceres::check(pba_set_frames(e, nf, frame_cam.data(), W, H, kind == 0 ? images.data() : nullptr), "frames");
  if (kind == 0) pba_ceres::check(pba_set_pattern(e, P, pattern.data()), "pattern");
  pba_ceres::check(pba_set_points(e, np, point_host.data(), u_ref.data(), kind == 0 ? host_int.data() : nullptr), "points");
  pba_ceres::check(pba_set_blocks(e, nb, block_point.data(), block_target.data(), kind == 1 ? u_obs.data() : nullptr), "blocks");

  // user memory, as the reference keeps it (Camera::T_w_c, Landmark::inv_depth)
  std::vector<std::array<double, 7>> T(nf);
  for (int i = 0; i < nf; ++i)
    for (int q = 0; q < 7; ++q) T[i][q] = poses_flat[7 * i + q];
  std::vector<double*> pose_ptr(nf), rho_ptr(np);
  for (int i = 0; i < nf; ++i) pose_ptr[i] = T[i].data();
  for (int p = 0; p < np; ++p) rho_ptr[p] = &rho[p];
  std::vector<double> intr_target(8);
  pba_ceres::GpuEvaluator ev(e, pose_ptr, rho_ptr, {},
                             tangent ? pba_ceres::PoseJacobian::kTangent : pba_ceres::PoseJacobian::kReferenceSE3);
  std::vector<std::unique_ptr<ceres::CostFunction>> cfs;
  for (int b = 0; b < nb; ++b) {
    const int h = point_host[block_point[b]], t = block_target[b];
    if (kind == 0) cfs.emplace_back(new pba_ceres::GpuPhotometricCost<8>(&ev, b, h, t));
    else cfs.emplace_back(new pba_ceres::GpuReprojectionCost(&ev, b, h, t));
  }
  pba_ceres::SE3TangentParameterization lp;
  std::vector<double> Pf(42 * (size_t)nf);  // ComputeJacobian of every frame's parameterisation
  for (int i = 0; i < nf; ++i) {
    if (tangent) lp.ComputeJacobian(T[i].data(), &Pf[42 * i]);
    else pba_ceres::se3_plus_jacobian(T[i].data(), &Pf[42 * i]);
  }

  const int R = kind == 0 ? P : 2, rec = 14 * R;
  std::vector<double> out((size_t)nb * rec, 0.0), ronly((size_t)nb * R, 0.0);
  std::vector<uint8_t> valid(nb, 0), valid_r(nb, 0);
  // residual + Jacobian evaluation (EvaluateGradientAndJacobian)
  ev.PrepareForEvaluation(true, true);
  std::vector<double> J0(R * 7), J1(R * 7), J2(R), J3(R * 8), r(R);
  for (int b = 0; b < nb; ++b) {
    const int p = block_point[b], h = point_host[p], t = block_target[b];
    const double* params[4] = {T[h].data(), T[t].data(), &rho[p], intr_target.data()};
    double* jac[4] = {J0.data(), J1.data(), J2.data(), nullptr};  // the intrinsics block is constant (map_utils.h:340-345)
    if (!cfs[b]->Evaluate(params, r.data(), jac)) continue;
    valid[b] = 1;
    double* o = &out[(size_t)b * rec];
    const double* Ph = &Pf[42 * h];
    const double* Pt = &Pf[42 * t];
    for (int k = 0; k < R; ++k) {
      o[k] = r[k];
      for (int c = 0; c < 6; ++c) {  // J_local = J_global · P   (residual_block.cc:136-158)
        double sh = 0, st = 0;
        for (int g = 0; g < 7; ++g) {
          sh += J0[k * 7 + g] * Ph[g * 6 + c];
          st += J1[k * 7 + g] * Pt[g * 6 + c];
        }
        o[R + 6 * k + c] = sh;
        o[7 * R + 6 * k + c] = st;
      }
      o[13 * R + k] = J2[k];
    }
  }
  // residual-only evaluation at a new point (candidate cost), jacobians == nullptr
  ev.PrepareForEvaluation(false, true);
  for (int b = 0; b < nb; ++b) {
    const int p = block_point[b], h = point_host[p], t = block_target[b];
    const double* params[4] = {T[h].data(), T[t].data(), &rho[p], intr_target.data()};
    if (!cfs[b]->Evaluate(params, r.data(), nullptr)) continue;
    valid_r[b] = 1;
    for (int k = 0; k < R; ++k) ronly[(size_t)b * R + k] = r[k];
  }
  // LocalParameterization::Plus on frame 0 with a fixed δ (compared with Sophus-semantics T·exp(δ))
  const double delta[6] = {0.01, -0.02, 0.03, 0.004, -0.005, 0.006};
  double plus[7];
  lp.Plus(T[0].data(), delta, plus);
  FILE* g = fopen(argv[2], "wb");
  fwrite(out.data(), sizeof(double), out.size(), g);
  fwrite(valid.data(), 1, valid.size(), g);
  fwrite(ronly.data(), sizeof(double), ronly.size(), g);
  fwrite(valid_r.data(), 1, valid_r.size(), g);
  fwrite(plus, sizeof(double), 7, g);
  fwrite(Pf.data(), sizeof(double), 42, g);  // frame 0's P
  fclose(g);
  pba_destroy(e);
  return 0;
}
