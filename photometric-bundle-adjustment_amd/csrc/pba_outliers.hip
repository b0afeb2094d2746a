// pba_outliers.hip — reprojection of every landmark observation and the outlier flags/landmark removal that
// follow each bundle-adjustment pass in the reference:
//
//   compute_projections()      src/sfm.cpp:1956-2008  per observation (inlier and outlier obs):
//                              p_c = T_w_c⁻¹ · Landmark::get_p()   (common_types.h:205-217: the anchor's
//                              normalised bearing / inv_depth, moved to the world by T_w_host),
//                              point_reprojected = π_c(p_c), reprojection_error = ‖corner − π_c(p_c)‖
//   set_outlier_flags()        src/sfm.cpp:1928-1953  (inlier observations only)
//   remove_outlier_landmarks() src/sfm.cpp:2028-2114  (per track, in FrameCamId order, host side)
//
// One lane per observation, fp64 throughout with Sophus' operation order (T⁻¹ = (q*, −q*·t), act = q·p + t),
// so reprojections agree with the reference's double arithmetic to rounding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "pba_internal.h"

using namespace pba;
using namespace pba::detail;

namespace {

// q·p for a unit quaternion q = (x, y, z, w) (so3.hpp:362-370: p + 2w(v×p) + 2v×(v×p))
__device__ __forceinline__ Vec3d qrot(double qx, double qy, double qz, double qw, const Vec3d& p) {
  const Vec3d v = {qx, qy, qz};
  Vec3d u = cross(v, p);
  u = {u.x + u.x, u.y + u.y, u.z + u.z};
  const Vec3d vu = cross(v, u);
  return {p.x + qw * u.x + vu.x, p.y + qw * u.y + vu.y, p.z + qw * u.z + vu.z};
}

struct ProjArgs {
  const double* poses;     // 7 per frame
  const double* rho;       // per point
  const double2* u_ref;    // per point
  const int* point_host;   // per point
  const int* frame_cam;    // per frame
  const double* cams;      // kCamD per camera
  const int* obs_point;
  const int* obs_frame;
  const double2* obs_uv;
  const uint8_t* obs_outlier;  // may be null
  double2* reproj;
  double* point_c;         // 3 per observation
  double* err;
  unsigned* flags;
  double th_normal, th_huge, th_dist, th_z;
  int n_obs;
};

template <int MODEL>
__global__ void projections_kernel(const ProjArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_obs) return;
  const int pt = a.obs_point[i], f = a.obs_frame[i], h = a.point_host[pt];
  // Landmark::get_p (common_types.h:205-217): T_w_h · (normalize(unproject_h(u_ref)) / inv_depth)
  const double2 ur = a.u_ref[pt];
  const Vec3d b = unproject<MODEL>(a.cams + kCamD * a.frame_cam[h] + kCamHk, ur.x, ur.y);
  const double id = 1.0 / a.rho[pt];
  const double* H = a.poses + 7 * h;
  const Vec3d ph = qrot(H[0], H[1], H[2], H[3], Vec3d{b.x * id, b.y * id, b.z * id});
  const Vec3d pw = {ph.x + H[4], ph.y + H[5], ph.z + H[6]};
  // T_w_c.inverse() * p_w (se3.hpp:208-211: q⁻¹ = q*, t⁻¹ = −q*·t)
  const double* T = a.poses + 7 * f;
  const Vec3d ti = qrot(-T[0], -T[1], -T[2], T[3], Vec3d{-T[4], -T[5], -T[6]});
  const Vec3d pr = qrot(-T[0], -T[1], -T[2], T[3], pw);
  const Vec3d pc = {pr.x + ti.x, pr.y + ti.y, pr.z + ti.z};
  // calib_cam.intrinsics[cam_id]->project(p_c) — the plain formula, no domain check (camera_models.h)
  double u, v;
  (void)project<MODEL>(a.cams + kCamD * a.frame_cam[f], pc, u, v);
  const double2 m = a.obs_uv[i];
  const double du = m.x - u, dv = m.y - v;
  const double e = sqrt(du * du + dv * dv);
  unsigned fl = PBA_OUTLIER_NONE;
  if (!(a.obs_outlier && a.obs_outlier[i])) {  // set_outlier_flags (sfm.cpp:1928-1953)
    if (e > a.th_huge) fl |= PBA_OUTLIER_REPROJECTION_HUGE;
    if (e > a.th_normal) fl |= PBA_OUTLIER_REPROJECTION_NORMAL;
    if (sqrt(pc.x * pc.x + pc.y * pc.y + pc.z * pc.z) < a.th_dist) fl |= PBA_OUTLIER_CAMERA_DISTANCE;
    if (pc.z < a.th_z) fl |= PBA_OUTLIER_Z_COORDINATE;
  }
  a.reproj[i] = make_double2(u, v);
  a.point_c[3 * i] = pc.x;
  a.point_c[3 * i + 1] = pc.y;
  a.point_c[3 * i + 2] = pc.z;
  a.err[i] = e;
  a.flags[i] = fl;
}

}  // namespace

extern "C" {

int pba_compute_projections(pba_engine* e, int32_t n_obs, const int32_t* obs_point, const int32_t* obs_frame,
                            const double* obs_uv, const uint8_t* obs_is_outlier, const pba_outlier_thresholds* th,
                            double* reprojected, double* point_c, double* error, uint32_t* flags) {
  if (!e || n_obs < 0 || (n_obs > 0 && (!obs_point || !obs_frame || !obs_uv)))
    return fail(PBA_ERR_INVALID_ARGUMENT, "bad observation arguments");
  if (!e->state_set || e->n_points <= 0 || e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "problem/state not set");
  if (e->level != 0) return fail(PBA_ERR_NOT_READY, "projections are computed at pyramid level 0 (pba_set_level)");
  if (n_obs == 0) return PBA_OK;
  for (int i = 0; i < n_obs; ++i)
    if (obs_point[i] < 0 || obs_point[i] >= e->n_points || obs_frame[i] < 0 || obs_frame[i] >= e->n_frames)
      return fail(PBA_ERR_INVALID_ARGUMENT, "observation point/frame out of range");
  const pba_outlier_thresholds def = {3.0, 40.0, 0.1, 0.05};  // sfm.cpp:254-261
  const pba_outlier_thresholds& t = th ? *th : def;
  if (int rc = check_device(e)) return rc;
  DevBuf<int> d_pt, d_fr;
  DevBuf<double2> d_uv, d_rep;
  DevBuf<uint8_t> d_out;
  DevBuf<double> d_pc, d_err;
  DevBuf<unsigned> d_fl;
  PBA_HIP(d_pt.resize(n_obs));
  PBA_HIP(d_fr.resize(n_obs));
  PBA_HIP(d_uv.resize(n_obs));
  PBA_HIP(d_rep.resize(n_obs));
  PBA_HIP(d_pc.resize(3 * (size_t)n_obs));
  PBA_HIP(d_err.resize(n_obs));
  PBA_HIP(d_fl.resize(n_obs));
  PBA_HIP(hipMemcpyAsync(d_pt.p, obs_point, sizeof(int) * n_obs, hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(d_fr.p, obs_frame, sizeof(int) * n_obs, hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(d_uv.p, obs_uv, sizeof(double2) * n_obs, hipMemcpyHostToDevice, e->stream));
  if (obs_is_outlier) {
    PBA_HIP(d_out.resize(n_obs));
    PBA_HIP(hipMemcpyAsync(d_out.p, obs_is_outlier, n_obs, hipMemcpyHostToDevice, e->stream));
  }
  ProjArgs a{e->poses.p, e->rho.p, e->u_ref.p, e->point_host_d.p, e->frame_cam.p, e->intr_d.p, d_pt.p, d_fr.p, d_uv.p,
             obs_is_outlier ? d_out.p : nullptr, d_rep.p, d_pc.p, d_err.p, d_fl.p,
             t.reprojection_error_normal_px, t.reprojection_error_huge_px, t.camera_center_distance_m,
             t.z_coordinate_m, n_obs};
  const int grid = (n_obs + 255) / 256;
  switch (e->opt.camera_model) {
    case PBA_CAMERA_PINHOLE: projections_kernel<CAM_PINHOLE><<<grid, 256, 0, e->stream>>>(a); break;
    case PBA_CAMERA_DOUBLE_SPHERE: projections_kernel<CAM_DS><<<grid, 256, 0, e->stream>>>(a); break;
    case PBA_CAMERA_EUCM: projections_kernel<CAM_EUCM><<<grid, 256, 0, e->stream>>>(a); break;
    default: projections_kernel<CAM_KB4><<<grid, 256, 0, e->stream>>>(a); break;
  }
  PBA_HIP(hipGetLastError());
  if (reprojected) PBA_HIP(hipMemcpyAsync(reprojected, d_rep.p, sizeof(double2) * n_obs, hipMemcpyDeviceToHost, e->stream));
  if (point_c) PBA_HIP(hipMemcpyAsync(point_c, d_pc.p, sizeof(double) * 3 * n_obs, hipMemcpyDeviceToHost, e->stream));
  if (error) PBA_HIP(hipMemcpyAsync(error, d_err.p, sizeof(double) * n_obs, hipMemcpyDeviceToHost, e->stream));
  if (flags) PBA_HIP(hipMemcpyAsync(flags, d_fl.p, sizeof(unsigned) * n_obs, hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

}  // extern "C"
