// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/, never shipped).
//
// Golden-vector generator that runs the REFERENCE'S OWN vendored SE3 library — Sophus 1.1.0 and
// Eigen 3.3.8 compiled straight from /root/reference/thirdparty (header-only, no generated code) —
// to pin oracle/oracle.cpp.  The visnav headers themselves cannot be compiled here (common_types.h:43-44
// needs TBB, which is not installed) and Ceres needs its CMake-generated config.h, so the functor
// arithmetic around Sophus is restated below; everything Lie-group related (exp, group product,
// inverse, action, Dx_this_mul_exp_x_at_0, Eigen quaternion product / toRotationMatrix) is the real
// library code.
//
// Tangent Jacobians are taken the way Ceres' LocalParameterizationSE3 defines the tangent space
// (local_parameterization_se3.hpp:43-50: T ⊞ δ = T · SE3::exp(δ)), by central differences in
// long double through Sophus itself — an estimator fully independent of the oracle's dual numbers.
// Pixels whose difference stencil crosses a bilinear cell boundary are reported (fd_ok = 0).
//
// Usage:  ref_harness se3   <in.bin> <out.bin>
//         ref_harness block <in.bin> <out.bin>      (problem layout documented in tests/golden/make_golden.py)

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <Eigen/Core>
#include <Eigen/Geometry>
#include <sophus/se3.hpp>

using LD = long double;
using SE3L = Sophus::SE3<LD>;
using V3 = Eigen::Matrix<LD, 3, 1>;
using V6 = Eigen::Matrix<LD, 6, 1>;

namespace {

struct Reader {
  FILE* f;
  template <class T> std::vector<T> vec(size_t n) {
    std::vector<T> v(n);
    if (n && fread(v.data(), sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
    return v;
  }
  int32_t i32() { return vec<int32_t>(1)[0]; }
};

SE3L pose_from(const double* p) {
  Eigen::Quaternion<LD> q((LD)p[3], (LD)p[0], (LD)p[1], (LD)p[2]);
  return SE3L(q, V3((LD)p[4], (LD)p[5], (LD)p[6]));
}

// Camera arithmetic, restated from include/visnav/camera_models.h (pinhole :75-107, EUCM :140-190,
// double sphere :226-277, Kannala-Brandt 4 :316-420) in long double.
void project(int model, const double* k, const V3& p, LD uv[2]) {
  const LD fx = k[0], fy = k[1], cx = k[2], cy = k[3];
  if (model == 0) {
    uv[0] = fx * p[0] / p[2] + cx;
    uv[1] = fy * p[1] / p[2] + cy;
  } else if (model == 1) {
    const LD xi = k[4], alpha = k[5];
    const LD d1 = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    const LD xz = xi * d1 + p[2];
    const LD d2 = std::sqrt(p[0] * p[0] + p[1] * p[1] + xz * xz);
    const LD den = alpha * d2 + (1 - alpha) * xz;
    uv[0] = fx * p[0] / den + cx;
    uv[1] = fy * p[1] / den + cy;
  } else if (model == 2) {
    const LD alpha = k[4], beta = k[5];
    const LD d = std::sqrt(beta * (p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]);
    const LD den = alpha * d + (1 - alpha) * p[2];
    uv[0] = fx * p[0] / den + cx;
    uv[1] = fy * p[1] / den + cy;
  } else {  // Kannala-Brandt 4 (camera_models.h:316-348)
    const LD r = std::sqrt(p[0] * p[0] + p[1] * p[1]);
    if (r == 0) { uv[0] = cx; uv[1] = cy; return; }
    const LD th = std::atan2(r, p[2]), t2 = th * th;
    const LD d = th + t2 * th * ((LD)k[4] + t2 * ((LD)k[5] + t2 * ((LD)k[6] + t2 * (LD)k[7])));
    uv[0] = fx * d * p[0] / r + cx;
    uv[1] = fy * d * p[1] / r + cy;
  }
}

V3 unproject(int model, const double* k, LD u, LD v) {
  const LD fx = k[0], fy = k[1], cx = k[2], cy = k[3];
  const LD mx = (u - cx) / fx, my = (v - cy) / fy;
  V3 b;
  if (model == 0) {
    b << mx, my, 1;
  } else if (model == 1) {
    const LD xi = k[4], alpha = k[5];
    const LD r2 = mx * mx + my * my;
    const LD mz = (1 - alpha * alpha * r2) / (alpha * std::sqrt(1 - (2 * alpha - 1) * r2) + 1 - alpha);
    const LD fac = (mz * xi + std::sqrt(mz * mz + (1 - xi * xi) * r2)) / (mz * mz + r2);
    b << fac * mx, fac * my, fac * mz - xi;
  } else if (model == 2) {
    const LD alpha = k[4], beta = k[5];
    const LD r2 = mx * mx + my * my;
    b << mx, my, (1 - beta * alpha * alpha * r2) / (alpha * std::sqrt(1 - (2 * alpha - 1) * beta * r2) + (1 - alpha));
  } else {  // Kannala-Brandt 4 (camera_models.h:352-380): 5 Newton steps from θ = 0
    const LD ru = std::sqrt(mx * mx + my * my);
    if (ru == 0) return V3(0, 0, 1);
    LD th = 0;
    for (int i = 0; i < 5; ++i) {
      const LD t2 = th * th;
      const LD f = th + t2 * th * ((LD)k[4] + t2 * ((LD)k[5] + t2 * ((LD)k[6] + t2 * (LD)k[7]))) - ru;
      const LD df = 1 + t2 * (3 * (LD)k[4] + t2 * (5 * (LD)k[5] + t2 * (7 * (LD)k[6] + t2 * 9 * (LD)k[7])));
      th -= f / df;
    }
    b << std::sin(th) * mx / ru, std::sin(th) * my / ru, std::cos(th);
  }
  return b.normalized();
}

// Bilinear + edge clamp; also returns the cell so a stencil that changes cell can be flagged.
LD bilinear(const uint8_t* img, int W, int H, LD u, LD v, long* cell) {
  u = std::min(std::max(u, (LD)-2), (LD)W + 1);
  v = std::min(std::max(v, (LD)-2), (LD)H + 1);
  const LD xf = std::floor(u), yf = std::floor(v);
  const LD a = u - xf, b = v - yf;
  const int x0 = (int)xf, y0 = (int)yf;
  auto cl = [](int x, int n) { return x < 0 ? 0 : (x > n - 1 ? n - 1 : x); };
  const int xa = cl(x0, W), xb = cl(x0 + 1, W), ya = cl(y0, H), yb = cl(y0 + 1, H);
  const LD I00 = img[(size_t)ya * W + xa], I10 = img[(size_t)ya * W + xb];
  const LD I01 = img[(size_t)yb * W + xa], I11 = img[(size_t)yb * W + xb];
  if (cell) *cell = (long)(x0 + 4) * 100000L + (long)(y0 + 4);
  return (1 - b) * ((1 - a) * I00 + a * I10) + b * ((1 - a) * I01 + a * I11);
}

struct Problem {
  int kind, model, nf, np, nb, nc, W, H, P;
  std::vector<double> intr, u_ref, u_obs, poses, rho;
  std::vector<int32_t> frame_cam, point_host, block_point, block_target;
  std::vector<uint8_t> images;
  std::vector<float> pattern, host_int;
};

// Residual of one block at (T_h, T_t, ρ); cells[] receives the bilinear cell of every pixel.
bool residual(const Problem& pb, int b, const SE3L& Th, const SE3L& Tt, LD rho, LD* r, long* cells) {
  const int pt = pb.block_point[b], tgt = pb.block_target[b], host = pb.point_host[pt];
  const double* kh = &pb.intr[8 * pb.frame_cam[host]];
  const double* kt = &pb.intr[8 * pb.frame_cam[tgt]];
  if (pb.kind == 1) {
    // reprojection.h:105-108  r = p_2d − π_t(T_w_t⁻¹ · T_w_h · (b / ρ))
    const V3 bear = unproject(pb.model, kh, pb.u_ref[2 * pt], pb.u_ref[2 * pt + 1]);
    const V3 p = Tt.inverse() * Th * V3(bear / rho);
    LD uv[2];
    project(pb.model, kt, p, uv);
    r[0] = (LD)pb.u_obs[2 * b] - uv[0];
    r[1] = (LD)pb.u_obs[2 * b + 1] - uv[1];
    return std::isfinite((double)r[0]) && std::isfinite((double)r[1]);
  }
  // photometric_error.h:151-179 with Eigen quaternions, bilinear interpolator
  const Eigen::Quaternion<LD> q_w_h = Th.unit_quaternion(), q_w_t = Tt.unit_quaternion();
  const Eigen::Quaternion<LD> q_t_h = q_w_t.conjugate() * q_w_h;
  const Eigen::Matrix<LD, 3, 3> R_t_h = q_t_h.toRotationMatrix();
  const V3 t_t_h = q_w_t.conjugate() * V3(Th.translation() - Tt.translation());
  const uint8_t* img = &pb.images[(size_t)tgt * pb.W * pb.H];
  for (int k = 0; k < pb.P; ++k) {
    const V3 bk = unproject(pb.model, kh, (LD)pb.u_ref[2 * pt] + pb.pattern[2 * k], (LD)pb.u_ref[2 * pt + 1] + pb.pattern[2 * k + 1]);
    const V3 p = R_t_h * bk + rho * t_t_h;
    if (pb.model == 0 && !(p[2] > 1e-6L)) return false;
    if (pb.model == 1) {  // double-sphere domain (Usenko et al. 3DV'18, eq. 43) — same rule as the oracle
      const LD xi = kt[4], al = kt[5], d1 = p.norm();
      const LD w1 = al <= 0.5L ? al / (1 - al) : (1 - al) / al;
      const LD w2 = (w1 + xi) / std::sqrt(2 * w1 * xi + xi * xi + 1);
      if (!(p[2] > -w2 * d1 + 1e-10L)) return false;
    }
    if (pb.model == 3 && !(p[2] > 0 || p[0] * p[0] + p[1] * p[1] > 0)) return false;  // KB4: all but the backward axis
    if (pb.model == 2) {  // EUCM domain, photometric_error.h:114-121
      const LD al = kt[4], be = kt[5];
      const LD rr = std::sqrt(be * (p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]);
      const LD w = al > 0.5L ? (1 - al) / al : al / (1 - al);
      if (!(p[2] > -w * rr + 1e-10L)) return false;
    }
    LD uv[2];
    project(pb.model, kt, p, uv);
    r[k] = bilinear(img, pb.W, pb.H, uv[0], uv[1], cells ? &cells[k] : nullptr) - (LD)pb.host_int[(size_t)pb.P * pt + k];
  }
  return true;
}

int run_block(const char* in, const char* out) {
  FILE* f = fopen(in, "rb");
  if (!f) return 2;
  Reader rd{f};
  Problem pb;
  pb.kind = rd.i32(); pb.model = rd.i32(); pb.nf = rd.i32(); pb.np = rd.i32(); pb.nb = rd.i32();
  pb.nc = rd.i32(); pb.W = rd.i32(); pb.H = rd.i32(); pb.P = rd.i32();
  pb.intr = rd.vec<double>(8 * pb.nc);
  pb.frame_cam = rd.vec<int32_t>(pb.nf);
  pb.images = rd.vec<uint8_t>(pb.kind == 0 ? (size_t)pb.nf * pb.W * pb.H : 0);
  pb.pattern = rd.vec<float>(pb.kind == 0 ? 2 * pb.P : 0);
  pb.point_host = rd.vec<int32_t>(pb.np);
  pb.u_ref = rd.vec<double>(2 * pb.np);
  pb.host_int = rd.vec<float>(pb.kind == 0 ? (size_t)pb.P * pb.np : 0);
  pb.block_point = rd.vec<int32_t>(pb.nb);
  pb.block_target = rd.vec<int32_t>(pb.nb);
  pb.u_obs = rd.vec<double>(pb.kind == 1 ? 2 * pb.nb : 0);
  pb.poses = rd.vec<double>(7 * pb.nf);
  pb.rho = rd.vec<double>(pb.np);
  fclose(f);

  const int R = pb.kind == 0 ? pb.P : 2;
  const int rec = 14 * R;
  std::vector<double> outv((size_t)rec * pb.nb, 0.0);
  std::vector<uint8_t> valid(pb.nb, 0), fdok(pb.nb, 1);
  const LD h = 1e-7L;
  std::vector<LD> r0(R), rp(R), rm(R);
  std::vector<long> c0(R), cp(R), cm(R);
  for (int b = 0; b < pb.nb; ++b) {
    const int pt = pb.block_point[b], tgt = pb.block_target[b], host = pb.point_host[pt];
    const SE3L Th = pose_from(&pb.poses[7 * host]), Tt = pose_from(&pb.poses[7 * tgt]);
    const LD rho = pb.rho[pt];
    if (!residual(pb, b, Th, Tt, rho, r0.data(), c0.data())) continue;
    double* o = &outv[(size_t)rec * b];
    for (int k = 0; k < R; ++k) o[k] = (double)r0[k];
    bool ok = true;
    auto fd = [&](int which, int j) {  // which: 0 host, 1 target, 2 rho
      SE3L Thp = Th, Thm = Th, Ttp = Tt, Ttm = Tt;
      LD rp_ = rho, rm_ = rho;
      if (which < 2) {
        V6 d = V6::Zero();
        d[j] = h;
        // LocalParameterizationSE3::Plus: T · exp(δ)
        if (which == 0) { Thp = Th * SE3L::exp(d); Thm = Th * SE3L::exp(-d); }
        else { Ttp = Tt * SE3L::exp(d); Ttm = Tt * SE3L::exp(-d); }
      } else {
        rp_ = rho + h * rho; rm_ = rho - h * rho;
      }
      const bool a = residual(pb, b, Thp, Ttp, rp_, rp.data(), cp.data());
      const bool c = residual(pb, b, Thm, Ttm, rm_, rm.data(), cm.data());
      if (!a || !c) { ok = false; return; }
      const LD step = which < 2 ? 2 * h : 2 * h * rho;
      for (int k = 0; k < R; ++k) {
        const LD g = (rp[k] - rm[k]) / step;
        if (pb.kind == 0 && (cp[k] != c0[k] || cm[k] != c0[k])) fdok[b] = 0;
        if (which == 0) o[R + 6 * k + j] = (double)g;
        else if (which == 1) o[7 * R + 6 * k + j] = (double)g;
        else o[13 * R + k] = (double)g;
      }
    };
    for (int j = 0; j < 6; ++j) fd(0, j);
    for (int j = 0; j < 6; ++j) fd(1, j);
    fd(2, 0);
    if (!ok) { std::memset(o, 0, sizeof(double) * rec); continue; }
    valid[b] = 1;
  }
  FILE* g = fopen(out, "wb");
  if (!g) return 3;
  fwrite(outv.data(), sizeof(double), outv.size(), g);
  fwrite(valid.data(), 1, valid.size(), g);
  fwrite(fdok.data(), 1, fdok.size(), g);
  fclose(g);
  return 0;
}

// SE3 fixtures straight from Sophus: exp, T·exp(δ), inverse, T·p, Dx_this_mul_exp_x_at_0, Ta⁻¹·Tb.
int run_se3(const char* in, const char* out) {
  FILE* f = fopen(in, "rb");
  if (!f) return 2;
  Reader rd{f};
  const int n = rd.i32();
  auto poses = rd.vec<double>(7 * n);
  auto poses2 = rd.vec<double>(7 * n);
  auto deltas = rd.vec<double>(6 * n);
  auto points = rd.vec<double>(3 * n);
  fclose(f);
  FILE* g = fopen(out, "wb");
  if (!g) return 3;
  for (int i = 0; i < n; ++i) {
    Sophus::SE3d T(Eigen::Quaterniond(poses[7 * i + 3], poses[7 * i], poses[7 * i + 1], poses[7 * i + 2]),
                   Eigen::Vector3d(poses[7 * i + 4], poses[7 * i + 5], poses[7 * i + 6]));
    Sophus::SE3d T2(Eigen::Quaterniond(poses2[7 * i + 3], poses2[7 * i], poses2[7 * i + 1], poses2[7 * i + 2]),
                    Eigen::Vector3d(poses2[7 * i + 4], poses2[7 * i + 5], poses2[7 * i + 6]));
    Eigen::Map<const Sophus::Vector6d> d(&deltas[6 * i]);
    const Sophus::SE3d E = Sophus::SE3d::exp(d);
    const Sophus::SE3d TE = T * E;
    const Sophus::SE3d Ti = T.inverse();
    const Eigen::Vector3d Tp = T * Eigen::Vector3d(points[3 * i], points[3 * i + 1], points[3 * i + 2]);
    const Eigen::Matrix<double, 7, 6, Eigen::RowMajor> J = T.Dx_this_mul_exp_x_at_0();
    const Sophus::SE3d rel = T2.inverse() * T;
    fwrite(E.data(), sizeof(double), 7, g);
    fwrite(TE.data(), sizeof(double), 7, g);
    fwrite(Ti.data(), sizeof(double), 7, g);
    fwrite(Tp.data(), sizeof(double), 3, g);
    fwrite(J.data(), sizeof(double), 42, g);
    fwrite(rel.data(), sizeof(double), 7, g);
  }
  fclose(g);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 4) { fprintf(stderr, "usage: %s se3|block in out\n", argv[0]); return 1; }
  const std::string mode = argv[1];
  if (mode == "se3") return run_se3(argv[2], argv[3]);
  if (mode == "block") return run_block(argv[2], argv[3]);
  return 1;
}
