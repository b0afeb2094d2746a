// oracle/golden_ceres.cpp — TEST-ONLY golden-vector generator built on the reference's vendored Ceres Solver 2.0.0
// (oracle/ceres.mk → oracle/_ref/golden_ceres).  It runs Ceres' own code; the fixtures it writes pin the engine's
// bicubic path (tests/golden/make_ceres_golden.py):
//
//   interp <image.bin> <positions.bin> <out.bin>
//       BiCubicInterpolator<Grid2D<uint8_t, 1>>::Evaluate(r = v, c = u) (cubic_interpolation.h:264-344) at every
//       position: f, dfdr, dfdc (doubles).  image.bin = int32 H, W then H·W u8; positions = n × (u, v) doubles.
//   photometric <problem.bin> <out.bin>
//       ceres::PhotometricError<8> (internal/ceres/autodiff_benchmarks/photometric_error.h:79-189 — EUCM projection,
//       BiCubicInterpolator over the target image) through AutoDiffCostFunction<PhotometricError<8>, 8, 7, 7, 1>
//       for every block of a problem (tests/golden/make_golden.py write_problem layout, EUCM camera, P = 8).  The
//       host bearings are the normalised EUCM unprojections of u_ref + pattern offset (tests/cpp/ceres_functors.h:
//       Unproject, camera_models.h:162-190); the 8×7 pose Jacobians are mapped to the tangent space with the
//       reference's LocalParameterizationSE3::ComputeJacobian (local_parameterization_se3.hpp:56-63), as Ceres'
//       ResidualBlock::Evaluate does (residual_block.cc:136-158).  Out: per block 112 doubles
//       [r(8) | J_host(8×6) | J_target(8×6) | J_ρ(8)] and a validity byte (0 where PhotometricError throws: a
//       projection outside the EUCM domain, photometric_error.h:165-171).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ceres/ceres.h"
#include "ceres/cubic_interpolation.h"
#include "ceres_functors.h"                 // tests/cpp: Unproject (the restated camera_models.h unprojection)
#include "local_parameterization_se3.hpp"   // the reference's (include/visnav/)
#include "photometric_error.h"              // ceres-solver/internal/ceres/autodiff_benchmarks/

template <class T>
static std::vector<T> rd(FILE* f, size_t n) {
  std::vector<T> v(n);
  if (n && fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "short read\n");
    exit(2);
  }
  return v;
}

static int run_interp(const char* img_path, const char* pos_path, const char* out_path) {
  FILE* f = fopen(img_path, "rb");
  if (!f) return 2;
  const auto hw = rd<int32_t>(f, 2);
  const auto img = rd<uint8_t>(f, (size_t)hw[0] * hw[1]);
  fclose(f);
  f = fopen(pos_path, "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const size_t n = (size_t)ftell(f) / 16;
  fseek(f, 0, SEEK_SET);
  const auto uv = rd<double>(f, 2 * n);
  fclose(f);
  ceres::Grid2D<uint8_t, 1> grid(img.data(), 0, hw[0], 0, hw[1]);
  ceres::BiCubicInterpolator<ceres::Grid2D<uint8_t, 1>> interp(grid);
  std::vector<double> out(3 * n);
  for (size_t i = 0; i < n; ++i) interp.Evaluate(uv[2 * i + 1], uv[2 * i], &out[3 * i], &out[3 * i + 1], &out[3 * i + 2]);
  f = fopen(out_path, "wb");
  fwrite(out.data(), sizeof(double), out.size(), f);
  fclose(f);
  return 0;
}

static int run_photometric(const char* in_path, const char* out_path) {
  using F = ceres::PhotometricError<8>;
  FILE* f = fopen(in_path, "rb");
  if (!f) return 2;
  const auto hdr = rd<int32_t>(f, 9);
  const int kind = hdr[0], model = hdr[1], nf = hdr[2], np = hdr[3], nb = hdr[4], nc = hdr[5], W = hdr[6], H = hdr[7];
  const int P = hdr[8];
  if (kind != 0 || model != pba_test::CAM_EUCM || P != 8) {
    fprintf(stderr, "photometric mode needs an EUCM problem with P = 8\n");
    return 3;
  }
  const auto intr = rd<double>(f, 8 * nc);
  const auto frame_cam = rd<int32_t>(f, nf);
  const auto images = rd<uint8_t>(f, (size_t)nf * W * H);
  const auto pattern = rd<float>(f, 2 * P);
  const auto point_host = rd<int32_t>(f, np);
  const auto u_ref = rd<double>(f, 2 * np);
  const auto host_int = rd<float>(f, (size_t)P * np);
  const auto block_point = rd<int32_t>(f, nb);
  const auto block_target = rd<int32_t>(f, nb);
  auto poses = rd<double>(f, 7 * nf);
  auto rho = rd<double>(f, np);
  fclose(f);

  std::vector<std::unique_ptr<ceres::Grid2D<uint8_t, 1>>> grids;
  std::vector<std::unique_ptr<F::Interpolator>> interps;
  for (int i = 0; i < nf; ++i) {
    grids.emplace_back(new ceres::Grid2D<uint8_t, 1>(&images[(size_t)i * W * H], 0, H, 0, W));
    interps.emplace_back(new F::Interpolator(*grids.back()));
  }
  std::vector<F::Intrinsics, Eigen::aligned_allocator<F::Intrinsics>> K(nc);
  for (int c = 0; c < nc; ++c) K[c] << intr[8 * c], intr[8 * c + 1], intr[8 * c + 2], intr[8 * c + 3], intr[8 * c + 4],
                                       intr[8 * c + 5];
  Sophus::test::LocalParameterizationSE3 lp;
  std::vector<double> out((size_t)nb * 112, 0.0);
  std::vector<uint8_t> valid(nb, 0);
  for (int b = 0; b < nb; ++b) {
    const int p = block_point[b], h = point_host[p], t = block_target[b];
    F::Patch<double> Ih;
    F::PatchVectors<double> bear;
    for (int k = 0; k < 8; ++k) {
      Ih[k] = host_int[(size_t)8 * p + k];
      bear.col(k) = pba_test::Unproject(model, &intr[8 * frame_cam[h]],
                                        Eigen::Vector2d(u_ref[2 * p] + pattern[2 * k], u_ref[2 * p + 1] + pattern[2 * k + 1]));
    }
    ceres::AutoDiffCostFunction<F, 8, 7, 7, 1> cf(new F(Ih, bear, *interps[t], K[frame_cam[t]]));
    const double* params[3] = {&poses[7 * h], &poses[7 * t], &rho[p]};
    double r[8], J0[56], J1[56], J2[8];
    double* jac[3] = {J0, J1, J2};
    try {
      if (!cf.Evaluate(params, r, jac)) continue;
    } catch (const std::runtime_error&) {
      continue;  // "Benchmark data leads to invalid projection." (photometric_error.h:165-171)
    }
    double Ph[42], Pt[42];
    lp.ComputeJacobian(&poses[7 * h], Ph);
    lp.ComputeJacobian(&poses[7 * t], Pt);
    double* o = &out[(size_t)b * 112];
    for (int k = 0; k < 8; ++k) {
      o[k] = r[k];
      for (int c = 0; c < 6; ++c) {
        double sh = 0, st = 0;
        for (int g = 0; g < 7; ++g) {
          sh += J0[7 * k + g] * Ph[6 * g + c];
          st += J1[7 * k + g] * Pt[6 * g + c];
        }
        o[8 + 6 * k + c] = sh;
        o[56 + 6 * k + c] = st;
      }
      o[104 + k] = J2[k];
    }
    valid[b] = 1;
  }
  f = fopen(out_path, "wb");
  fwrite(out.data(), sizeof(double), out.size(), f);
  fwrite(valid.data(), 1, valid.size(), f);
  fclose(f);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 5 && std::string(argv[1]) == "interp") return run_interp(argv[2], argv[3], argv[4]);
  if (argc >= 4 && std::string(argv[1]) == "photometric") return run_photometric(argv[2], argv[3]);
  fprintf(stderr, "usage: %s interp <image.bin> <positions.bin> <out.bin> | photometric <problem.bin> <out.bin>\n", argv[0]);
  return 1;
}
