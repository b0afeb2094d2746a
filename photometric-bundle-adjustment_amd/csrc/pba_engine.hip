// pba_engine.hip — HIP kernels + C ABI (include/pba.h) of the photometric BA residual/Jacobian engine.
//
// Replaces, for every residual block of a problem at once, the reference's per-block CPU evaluation:
//   ProgramEvaluator::Evaluate ParallelFor (program_evaluator.h:187-258) →
//   ResidualBlock::Evaluate (residual_block.cc:69-158) → AutoDiffCostFunction<Functor,…> →
//   BundleAdjustmentReprojectionCostFunctor (reprojection.h:83-112) / PhotometricError (photometric_error.h:139-182)
//
// Two launches per evaluation, on one stream:
//   1. pair_kernel      one lane per distinct (host, target) keyframe pair: T_th = T_w_t⁻¹ T_w_h in fp64
//                       from the fp64 state, stored as fp32 R_th|t_th (+camera ids, target frame) — 64 B/pair.
//   2. *_block_kernel   photometric: one lane per (block, pattern pixel), a wave = 64/LPB blocks;
//                       geometric:   one lane per block.
//                       SoA inputs (block_point, block_pair, u_ref, host_intensity, ρ) read coalesced,
//                       pair poses from L2, image taps gathered from the target keyframe's u8 image,
//                       Jacobian chain in registers, per-block ‖r‖² + validity by wave shuffles,
//                       records stored as one contiguous 14R-float slab per block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pba.h"
#include "pba_device.h"

using namespace pba;

namespace {

constexpr int kBlockThreads = 256;

struct KernelArgs {
  const uint8_t* images;
  int width, height;
  long long frame_stride;
  const float* intr;             // 8 floats per camera
  const int* block_point;
  const int* block_pair;
  const float4* pair_pose;       // 4 float4 per pair: R(9) t(3) host_cam target_cam target_frame pad
  const float2* u_ref;           // per point
  const float* host_int;         // P per point
  const double* rho;             // per point (state)
  const float2* u_obs;           // per block (geometric)
  float* out;                    // records
  float* cost;                   // per block
  uint8_t* valid;                // per block
  int n_blocks;
  int P;
  float huber;
  float pattern[2 * PBA_MAX_PATTERN];
};

// XCD-aware tile order: consecutive logical tiles (→ neighbouring host keyframes → shared target images)
// land on the same XCD's L2 (blocks are dealt round-robin over the 8 XCDs; speed only, never correctness).
__device__ __forceinline__ int logical_tile() {
  const int n = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3;
  const int q = n >> 3, rem = n & 7;
  return xcd * q + min(xcd, rem) + slot;
}

__device__ __forceinline__ float huber_cost(float s, float a) {
  if (a <= 0.0f || s <= a * a) return 0.5f * s;  // loss_function.cc:48-62, cost = ½ρ(s)
  return 0.5f * (2.0f * a * sqrtf(s) - a * a);
}

// ------------------------------------------------------------------------------------------------
// Pair kernel: relative poses in fp64 (avoids fp32 cancellation in t_w_h − t_w_t for long trajectories)
// ------------------------------------------------------------------------------------------------
__global__ void pair_kernel(const double* __restrict__ poses, const int* __restrict__ pair_host,
                            const int* __restrict__ pair_target, const int* __restrict__ frame_cam,
                            float4* __restrict__ pair_pose, int n_pairs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pairs) return;
  const int h = pair_host[i], t = pair_target[i];
  const double* H = poses + 7 * h;
  const double* T = poses + 7 * t;
  // q_th = q_wt* ⊗ q_wh (photometric_error.h:151, Hamilton product as so3.hpp:338-345)
  const double ax = -T[0], ay = -T[1], az = -T[2], aw = T[3];
  const double bx = H[0], by = H[1], bz = H[2], bw = H[3];
  const double qw = aw * bw - ax * bx - ay * by - az * bz;
  const double qx = aw * bx + ax * bw + ay * bz - az * by;
  const double qy = aw * by + ay * bw + az * bx - ax * bz;
  const double qz = aw * bz + az * bw + ax * by - ay * bx;
  // toRotationMatrix (photometric_error.h:152)
  const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
  const double twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                       txz - twy, tyz + twx, 1 - (txx + tyy)};
  // t_th = q_wt* · (t_wh − t_wt) (photometric_error.h:153), rotation as so3.hpp:367-370
  const double d0 = H[4] - T[4], d1 = H[5] - T[5], d2 = H[6] - T[6];
  double u0 = ay * d2 - az * d1, u1 = az * d0 - ax * d2, u2 = ax * d1 - ay * d0;
  u0 += u0; u1 += u1; u2 += u2;
  const double t0 = d0 + aw * u0 + (ay * u2 - az * u1);
  const double t1 = d1 + aw * u1 + (az * u0 - ax * u2);
  const double t2 = d2 + aw * u2 + (ax * u1 - ay * u0);
  float4* o = pair_pose + 4 * i;
  o[0] = make_float4((float)R[0], (float)R[1], (float)R[2], (float)R[3]);
  o[1] = make_float4((float)R[4], (float)R[5], (float)R[6], (float)R[7]);
  o[2] = make_float4((float)R[8], (float)t0, (float)t1, (float)t2);
  o[3] = make_float4(__int_as_float(frame_cam[h]), __int_as_float(frame_cam[t]), __int_as_float(t), 0.0f);
}

struct PairPose {
  float R[9];
  Vec3 t;
  int host_cam, target_cam, target;
};

__device__ __forceinline__ PairPose load_pair(const float4* __restrict__ pp, int pair) {
  const float4 a = pp[4 * pair + 0], b = pp[4 * pair + 1], c = pp[4 * pair + 2], d = pp[4 * pair + 3];
  PairPose r;
  r.R[0] = a.x; r.R[1] = a.y; r.R[2] = a.z; r.R[3] = a.w;
  r.R[4] = b.x; r.R[5] = b.y; r.R[6] = b.z; r.R[7] = b.w; r.R[8] = c.x;
  r.t = {c.y, c.z, c.w};
  r.host_cam = __float_as_int(d.x);
  r.target_cam = __float_as_int(d.y);
  r.target = __float_as_int(d.z);
  return r;
}

// Sum / AND over the LPB lanes of one block (LPB | 64, groups are aligned lane ranges).
template <int LPB>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = LPB / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
template <int LPB>
__device__ __forceinline__ int group_and(int v) {
#pragma unroll
  for (int m = LPB / 2; m >= 1; m >>= 1) v &= __shfl_xor(v, m, 64);
  return v;
}

// ------------------------------------------------------------------------------------------------
// Photometric block kernel: lane = (block, pixel k)
// ------------------------------------------------------------------------------------------------
template <int MODEL, int LPB, bool JAC>
__global__ __launch_bounds__(kBlockThreads) void photometric_block_kernel(const KernelArgs a) {
  const int gtid = logical_tile() * kBlockThreads + threadIdx.x;
  const int blk = gtid / LPB;
  const int k = gtid % LPB;
  if (blk >= a.n_blocks) return;  // a block's LPB lanes leave together
  const int P = a.P;
  const bool act = k < P;

  const int pt = a.block_point[blk];
  const PairPose pp = load_pair(a.pair_pose, a.block_pair[blk]);
  const float* kh = a.intr + 8 * pp.host_cam;
  const float* kt = a.intr + 8 * pp.target_cam;
  const float2 ur = a.u_ref[pt];
  const float rho = (float)a.rho[pt];
  const int kk = act ? k : 0;
  const float Ih = a.host_int[(long long)pt * P + kk];

  // warp: p̃ = R_th b_k + ρ t_th  (photometric_error.h:158-159)
  const Vec3 b = unproject<MODEL>(kh, ur.x + a.pattern[2 * kk], ur.y + a.pattern[2 * kk + 1]);
  const Vec3 Rb = mat_mul(pp.R, b);
  const Vec3 p = {Rb.x + rho * pp.t.x, Rb.y + rho * pp.t.y, Rb.z + rho * pp.t.z};
  const bool dom = in_domain<MODEL>(kt, p);
  float u, v;
  Vec3 du, dv;
  project_jac<MODEL>(kt, p, u, v, du, dv);
  float I = 0.0f, gx = 0.0f, gy = 0.0f;
  if (dom) bilinear(a.images + pp.target * a.frame_stride, a.width, a.height, u, v, I, gx, gy);
  const float r = I - Ih;  // photometric_error.h:179

  // per-block validity and ‖r‖² (wave shuffles over the block's lanes)
  const int ok = group_and<LPB>((dom && isfinite(r)) || !act);
  const float s = group_sum<LPB>(act ? r * r : 0.0f);
  float* rec = a.out + (long long)blk * 14 * P;
  if (k == 0) {
    a.valid[blk] = (uint8_t)ok;
    a.cost[blk] = ok ? huber_cost(s, a.huber) : 0.0f;
  }
  if (!act) return;
  if (!ok) {
    rec[k] = 0.0f;
    if (JAC) {
      float2* jh = reinterpret_cast<float2*>(rec + P + 6 * k);
      float2* jt = reinterpret_cast<float2*>(rec + 7 * P + 6 * k);
      jh[0] = jh[1] = jh[2] = make_float2(0.f, 0.f);
      jt[0] = jt[1] = jt[2] = make_float2(0.f, 0.f);
      rec[13 * P + k] = 0.0f;
    }
    return;
  }
  rec[k] = r;
  if (!JAC) return;
  // q = ∇I · ∂π/∂p̃  (1×3), then the chain (pba_device.h header)
  const Vec3 q = {gx * du.x + gy * dv.x, gx * du.y + gy * dv.y, gx * du.z + gy * dv.z};
  const Vec3 qR = row_mul(q, pp.R);
  const Vec3 wh = cross(b, qR);   // −(qR)×b
  const Vec3 wt = cross(q, p);    // q·[p̃]×
  const float jr = dot(q, pp.t);
  float2* jh = reinterpret_cast<float2*>(rec + P + 6 * k);
  float2* jt = reinterpret_cast<float2*>(rec + 7 * P + 6 * k);
  jh[0] = make_float2(rho * qR.x, rho * qR.y);
  jh[1] = make_float2(rho * qR.z, wh.x);
  jh[2] = make_float2(wh.y, wh.z);
  jt[0] = make_float2(-rho * q.x, -rho * q.y);
  jt[1] = make_float2(-rho * q.z, wt.x);
  jt[2] = make_float2(wt.y, wt.z);
  rec[13 * P + k] = jr;
}

// ------------------------------------------------------------------------------------------------
// Geometric block kernel (reprojection.h:105-108): lane = block, record 28 floats = 7 float4 stores
// ------------------------------------------------------------------------------------------------
template <int MODEL, bool JAC>
__global__ __launch_bounds__(kBlockThreads) void geometric_block_kernel(const KernelArgs a) {
  const int blk = logical_tile() * kBlockThreads + threadIdx.x;
  if (blk >= a.n_blocks) return;
  const int pt = a.block_point[blk];
  const PairPose pp = load_pair(a.pair_pose, a.block_pair[blk]);
  const float* kh = a.intr + 8 * pp.host_cam;
  const float* kt = a.intr + 8 * pp.target_cam;
  const float2 ur = a.u_ref[pt];
  const float2 uo = a.u_obs[blk];
  const float rho = (float)a.rho[pt];
  const float irho = 1.0f / rho;
  const Vec3 b = unproject<MODEL>(kh, ur.x, ur.y);
  const Vec3 ph = {b.x * irho, b.y * irho, b.z * irho};
  const Vec3 Rp = mat_mul(pp.R, ph);
  const Vec3 p = {Rp.x + pp.t.x, Rp.y + pp.t.y, Rp.z + pp.t.z};
  float u, v;
  Vec3 du, dv;
  project_jac<MODEL>(kt, p, u, v, du, dv);
  const float r0 = uo.x - u, r1 = uo.y - v;
  float4* rec = reinterpret_cast<float4*>(a.out + (long long)blk * 28);
  float J[28];
  J[0] = r0;
  J[1] = r1;
  bool ok = isfinite(r0) && isfinite(r1);
  if (JAC) {
    const Vec3 Rb = mat_mul(pp.R, b);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const Vec3 d = i == 0 ? du : dv;
      const Vec3 g = {-d.x, -d.y, -d.z};  // ∂r/∂p = −∂π/∂p
      const Vec3 gR = row_mul(g, pp.R);
      const Vec3 wh = cross(ph, gR);
      const Vec3 wt = cross(g, p);
      float* jh = J + 2 + 6 * i;
      float* jt = J + 14 + 6 * i;
      jh[0] = gR.x; jh[1] = gR.y; jh[2] = gR.z; jh[3] = wh.x; jh[4] = wh.y; jh[5] = wh.z;
      jt[0] = -g.x; jt[1] = -g.y; jt[2] = -g.z; jt[3] = wt.x; jt[4] = wt.y; jt[5] = wt.z;
      J[26 + i] = -dot(g, Rb) * irho * irho;
    }
#pragma unroll
    for (int i = 2; i < 28; ++i) ok = ok && isfinite(J[i]);
  }
  a.valid[blk] = (uint8_t)ok;
  a.cost[blk] = ok ? huber_cost(r0 * r0 + r1 * r1, a.huber) : 0.0f;
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 28; ++i) J[i] = 0.0f;
  }
  if (JAC) {
#pragma unroll
    for (int i = 0; i < 7; ++i) rec[i] = make_float4(J[4 * i], J[4 * i + 1], J[4 * i + 2], J[4 * i + 3]);
  } else {
    reinterpret_cast<float2*>(rec)[0] = make_float2(J[0], J[1]);
  }
}

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define PBA_HIP(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return fail(e_ == hipErrorOutOfMemory ? PBA_ERR_OUT_OF_MEMORY : PBA_ERR_DEVICE,          \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                          \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t resize(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (count == 0) return hipSuccess;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e == hipSuccess) n = count;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

}  // namespace

struct pba_engine {
  pba_options opt{};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  int n_cams = 0, n_frames = 0, n_points = 0, n_blocks = 0, n_pairs = 0;
  int width = 0, height = 0, P = 0;
  bool have_images = false;
  std::vector<int> frame_cam_h, point_host_h;
  std::vector<float> pattern_h;
  DevBuf<float> intr;
  DevBuf<int> frame_cam;
  DevBuf<uint8_t> images;
  DevBuf<float2> u_ref;
  DevBuf<float> host_int;
  DevBuf<int> block_point, block_pair;
  DevBuf<float2> u_obs;
  DevBuf<int> pair_host, pair_target;
  DevBuf<float4> pair_pose;
  DevBuf<double> poses, rho;
  DevBuf<float> out, cost;
  DevBuf<uint8_t> valid;
  bool state_set = false;
  bool evaluated = false;
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;   // start/stop pairs, reused
  size_t ev_used = 0;

  int R() const { return opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC ? P : 2; }
};

namespace {

int check_device(pba_engine* e) {
  PBA_HIP(hipSetDevice(e->opt.device));
  return PBA_OK;
}

template <int MODEL>
void launch_blocks(pba_engine* e, const KernelArgs& ka, bool jac) {
  if (e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC) {
    const int grid = (e->n_blocks + kBlockThreads - 1) / kBlockThreads;
    if (jac) geometric_block_kernel<MODEL, true><<<grid, kBlockThreads, 0, e->stream>>>(ka);
    else geometric_block_kernel<MODEL, false><<<grid, kBlockThreads, 0, e->stream>>>(ka);
    return;
  }
  const int lpb = e->P <= 8 ? 8 : (e->P <= 16 ? 16 : 32);
  const long long lanes = (long long)e->n_blocks * lpb;
  const int grid = (int)((lanes + kBlockThreads - 1) / kBlockThreads);
#define PBA_LAUNCH_PH(L)                                                                              \
  if (jac) photometric_block_kernel<MODEL, L, true><<<grid, kBlockThreads, 0, e->stream>>>(ka);      \
  else photometric_block_kernel<MODEL, L, false><<<grid, kBlockThreads, 0, e->stream>>>(ka);
  if (lpb == 8) { PBA_LAUNCH_PH(8) }
  else if (lpb == 16) { PBA_LAUNCH_PH(16) }
  else { PBA_LAUNCH_PH(32) }
#undef PBA_LAUNCH_PH
}

}  // namespace

extern "C" {

int pba_version(void) { return 100; }

const char* pba_status_string(int s) {
  switch (s) {
    case PBA_OK: return "ok";
    case PBA_ERR_INVALID_ARGUMENT: return "invalid argument";
    case PBA_ERR_DEVICE: return "device error";
    case PBA_ERR_OUT_OF_MEMORY: return "out of device memory";
    case PBA_ERR_NOT_READY: return "not ready (missing set_* call)";
    default: return "unknown status";
  }
}

const char* pba_last_error(void) { return g_last_error.c_str(); }

int pba_create(const pba_options* o, pba_engine** out) {
  if (!o || !out) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  if (o->residual_kind != PBA_RESIDUAL_PHOTOMETRIC && o->residual_kind != PBA_RESIDUAL_GEOMETRIC)
    return fail(PBA_ERR_INVALID_ARGUMENT, "unknown residual kind");
  if (o->camera_model < PBA_CAMERA_PINHOLE || o->camera_model > PBA_CAMERA_EUCM)
    return fail(PBA_ERR_INVALID_ARGUMENT, "unknown camera model");
  int n = 0;
  hipError_t err = hipGetDeviceCount(&n);
  if (err != hipSuccess || n <= 0) return fail(PBA_ERR_DEVICE, "no HIP device available");
  if (o->device < 0 || o->device >= n) return fail(PBA_ERR_INVALID_ARGUMENT, "device ordinal out of range");
  PBA_HIP(hipSetDevice(o->device));
  pba_engine* e = new pba_engine();
  e->opt = *o;
  err = hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking);
  if (err != hipSuccess) {
    delete e;
    return fail(PBA_ERR_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(err));
  }
  e->stream = e->own_stream;
  *out = e;
  return PBA_OK;
}

int pba_destroy(pba_engine* e) {
  if (!e) return PBA_OK;
  (void)hipSetDevice(e->opt.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  e->intr.release(); e->frame_cam.release(); e->images.release(); e->u_ref.release(); e->host_int.release();
  e->block_point.release(); e->block_pair.release(); e->u_obs.release(); e->pair_host.release();
  e->pair_target.release(); e->pair_pose.release(); e->poses.release(); e->rho.release(); e->out.release();
  e->cost.release(); e->valid.release();
  for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
  delete e;
  return PBA_OK;
}

int pba_set_stream(pba_engine* e, void* s) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  e->stream = s ? static_cast<hipStream_t>(s) : e->own_stream;
  return PBA_OK;
}

int pba_get_stream(pba_engine* e, void** s) {
  if (!e || !s) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  *s = e->stream;
  return PBA_OK;
}

int pba_set_cameras(pba_engine* e, int32_t n_cams, const double* intrinsics) {
  if (!e || n_cams <= 0 || !intrinsics) return fail(PBA_ERR_INVALID_ARGUMENT, "bad camera arguments");
  if (int rc = check_device(e)) return rc;
  std::vector<float> f(8 * (size_t)n_cams);
  for (size_t i = 0; i < f.size(); ++i) f[i] = (float)intrinsics[i];
  for (int c = 0; c < n_cams; ++c)
    if (!(f[8 * c] != 0.0f && f[8 * c + 1] != 0.0f)) return fail(PBA_ERR_INVALID_ARGUMENT, "zero focal length");
  PBA_HIP(e->intr.resize(f.size()));
  PBA_HIP(hipMemcpyAsync(e->intr.p, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  e->n_cams = n_cams;
  return PBA_OK;
}

static int set_frames_impl(pba_engine* e, int32_t n_frames, const int32_t* frame_cam, int32_t width,
                           int32_t height, const uint8_t* images, hipMemcpyKind kind) {
  if (!e || n_frames <= 0 || !frame_cam) return fail(PBA_ERR_INVALID_ARGUMENT, "bad frame arguments");
  if (e->n_cams <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_cameras first");
  for (int i = 0; i < n_frames; ++i)
    if (frame_cam[i] < 0 || frame_cam[i] >= e->n_cams) return fail(PBA_ERR_INVALID_ARGUMENT, "frame_cam out of range");
  const bool photometric = e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC;
  if (photometric && (!images || width <= 1 || height <= 1))
    return fail(PBA_ERR_INVALID_ARGUMENT, "photometric engines need images of at least 2x2");
  if (photometric && (long long)width * height > (1LL << 31))
    return fail(PBA_ERR_INVALID_ARGUMENT, "image too large");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(e->frame_cam.resize(n_frames));
  PBA_HIP(hipMemcpyAsync(e->frame_cam.p, frame_cam, n_frames * sizeof(int), hipMemcpyHostToDevice, e->stream));
  if (images) {
    const size_t bytes = (size_t)n_frames * width * height;
    PBA_HIP(e->images.resize(bytes));
    PBA_HIP(hipMemcpyAsync(e->images.p, images, bytes, kind, e->stream));
    e->have_images = true;
  }
  PBA_HIP(hipStreamSynchronize(e->stream));
  e->frame_cam_h.assign(frame_cam, frame_cam + n_frames);
  e->n_frames = n_frames;
  e->width = width;
  e->height = height;
  return PBA_OK;
}

int pba_set_frames(pba_engine* e, int32_t n_frames, const int32_t* frame_cam, int32_t width, int32_t height,
                   const uint8_t* images) {
  return set_frames_impl(e, n_frames, frame_cam, width, height, images, hipMemcpyHostToDevice);
}

int pba_set_frames_device(pba_engine* e, int32_t n_frames, const int32_t* frame_cam, int32_t width,
                          int32_t height, const uint8_t* d_images) {
  return set_frames_impl(e, n_frames, frame_cam, width, height, d_images, hipMemcpyDeviceToDevice);
}

int pba_set_pattern(pba_engine* e, int32_t P, const float* offsets) {
  if (!e || P <= 0 || P > PBA_MAX_PATTERN || !offsets) return fail(PBA_ERR_INVALID_ARGUMENT, "bad pattern");
  e->pattern_h.assign(offsets, offsets + 2 * P);
  e->P = P;
  return PBA_OK;
}

int pba_set_points(pba_engine* e, int32_t n_points, const int32_t* host_frame, const double* u_ref,
                   const float* host_intensity) {
  if (!e || n_points <= 0 || !host_frame || !u_ref) return fail(PBA_ERR_INVALID_ARGUMENT, "bad point arguments");
  if (e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_frames first");
  const bool photometric = e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC;
  if (photometric && (e->P <= 0 || !host_intensity))
    return fail(PBA_ERR_INVALID_ARGUMENT, "photometric points need pba_set_pattern and host intensities");
  for (int i = 0; i < n_points; ++i)
    if (host_frame[i] < 0 || host_frame[i] >= e->n_frames) return fail(PBA_ERR_INVALID_ARGUMENT, "host frame out of range");
  if (int rc = check_device(e)) return rc;
  std::vector<float2> ur(n_points);
  for (int i = 0; i < n_points; ++i) ur[i] = make_float2((float)u_ref[2 * i], (float)u_ref[2 * i + 1]);
  PBA_HIP(e->u_ref.resize(n_points));
  PBA_HIP(hipMemcpyAsync(e->u_ref.p, ur.data(), n_points * sizeof(float2), hipMemcpyHostToDevice, e->stream));
  if (photometric) {
    PBA_HIP(e->host_int.resize((size_t)n_points * e->P));
    PBA_HIP(hipMemcpyAsync(e->host_int.p, host_intensity, (size_t)n_points * e->P * sizeof(float),
                           hipMemcpyHostToDevice, e->stream));
  }
  PBA_HIP(e->rho.resize(n_points));
  PBA_HIP(hipStreamSynchronize(e->stream));
  e->point_host_h.assign(host_frame, host_frame + n_points);
  e->n_points = n_points;
  e->state_set = false;
  return PBA_OK;
}

int pba_set_blocks(pba_engine* e, int32_t n_blocks, const int32_t* block_point, const int32_t* block_target,
                   const double* u_obs) {
  if (!e || n_blocks <= 0 || !block_point || !block_target) return fail(PBA_ERR_INVALID_ARGUMENT, "bad block arguments");
  if (e->n_points <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_points first");
  const bool geometric = e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC;
  if (geometric && !u_obs) return fail(PBA_ERR_INVALID_ARGUMENT, "geometric blocks need u_obs");
  const long long rec = 14LL * e->R();
  if ((long long)n_blocks * rec >= (1LL << 40)) return fail(PBA_ERR_INVALID_ARGUMENT, "problem too large");
  // distinct (host, target) pairs, in first-seen order
  std::vector<int> pair_of(n_blocks), ph, pt;
  std::vector<long long> keys;
  {
    std::vector<std::pair<long long, int>> seen;
    seen.reserve(n_blocks);
    for (int b = 0; b < n_blocks; ++b) {
      const int p = block_point[b], t = block_target[b];
      if (p < 0 || p >= e->n_points) return fail(PBA_ERR_INVALID_ARGUMENT, "block point out of range");
      if (t < 0 || t >= e->n_frames) return fail(PBA_ERR_INVALID_ARGUMENT, "block target out of range");
      const int h = e->point_host_h[p];
      if (h == t) return fail(PBA_ERR_INVALID_ARGUMENT, "block target equals the point's host");
      seen.emplace_back((long long)h * e->n_frames + t, b);
    }
    std::sort(seen.begin(), seen.end());
    for (size_t i = 0; i < seen.size(); ++i) {
      if (i == 0 || seen[i].first != seen[i - 1].first) {
        ph.push_back((int)(seen[i].first / e->n_frames));
        pt.push_back((int)(seen[i].first % e->n_frames));
      }
      pair_of[seen[i].second] = (int)ph.size() - 1;
    }
  }
  if (int rc = check_device(e)) return rc;
  const int np = (int)ph.size();
  PBA_HIP(e->block_point.resize(n_blocks));
  PBA_HIP(e->block_pair.resize(n_blocks));
  PBA_HIP(e->pair_host.resize(np));
  PBA_HIP(e->pair_target.resize(np));
  PBA_HIP(e->pair_pose.resize(4 * (size_t)np));
  PBA_HIP(hipMemcpyAsync(e->block_point.p, block_point, n_blocks * sizeof(int), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->block_pair.p, pair_of.data(), n_blocks * sizeof(int), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->pair_host.p, ph.data(), np * sizeof(int), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->pair_target.p, pt.data(), np * sizeof(int), hipMemcpyHostToDevice, e->stream));
  if (geometric) {
    std::vector<float2> uo(n_blocks);
    for (int b = 0; b < n_blocks; ++b) uo[b] = make_float2((float)u_obs[2 * b], (float)u_obs[2 * b + 1]);
    PBA_HIP(e->u_obs.resize(n_blocks));
    PBA_HIP(hipMemcpyAsync(e->u_obs.p, uo.data(), n_blocks * sizeof(float2), hipMemcpyHostToDevice, e->stream));
    PBA_HIP(hipStreamSynchronize(e->stream));
  }
  PBA_HIP(e->out.resize((size_t)n_blocks * rec));
  PBA_HIP(e->cost.resize(n_blocks));
  PBA_HIP(e->valid.resize(n_blocks));
  PBA_HIP(hipStreamSynchronize(e->stream));
  e->n_blocks = n_blocks;
  e->n_pairs = np;
  e->evaluated = false;
  return PBA_OK;
}

int pba_set_state(pba_engine* e, const double* poses, const double* inv_dist) {
  if (!e || !poses || !inv_dist) return fail(PBA_ERR_INVALID_ARGUMENT, "null state");
  if (e->n_points <= 0 || e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "problem not set");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(e->poses.resize(7 * (size_t)e->n_frames));
  PBA_HIP(hipMemcpyAsync(e->poses.p, poses, 7 * (size_t)e->n_frames * sizeof(double), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->rho.p, inv_dist, (size_t)e->n_points * sizeof(double), hipMemcpyHostToDevice, e->stream));
  e->state_set = true;
  return PBA_OK;
}

int pba_set_state_device(pba_engine* e, const double* d_poses, const double* d_inv_dist) {
  if (!e || !d_poses || !d_inv_dist) return fail(PBA_ERR_INVALID_ARGUMENT, "null state");
  if (e->n_points <= 0 || e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "problem not set");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(e->poses.resize(7 * (size_t)e->n_frames));
  PBA_HIP(hipMemcpyAsync(e->poses.p, d_poses, 7 * (size_t)e->n_frames * sizeof(double), hipMemcpyDeviceToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->rho.p, d_inv_dist, (size_t)e->n_points * sizeof(double), hipMemcpyDeviceToDevice, e->stream));
  e->state_set = true;
  return PBA_OK;
}

int pba_evaluate(pba_engine* e, int32_t want_jacobians) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (e->n_blocks <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_blocks first");
  if (!e->state_set) return fail(PBA_ERR_NOT_READY, "pba_set_state first");
  const bool photometric = e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC;
  if (photometric && (!e->have_images || e->P <= 0)) return fail(PBA_ERR_NOT_READY, "images/pattern missing");
  if (int rc = check_device(e)) return rc;
  pair_kernel<<<(e->n_pairs + 255) / 256, 256, 0, e->stream>>>(e->poses.p, e->pair_host.p, e->pair_target.p,
                                                               e->frame_cam.p, e->pair_pose.p, e->n_pairs);
  KernelArgs ka{};
  ka.images = e->images.p;
  ka.width = e->width;
  ka.height = e->height;
  ka.frame_stride = (long long)e->width * e->height;
  ka.intr = e->intr.p;
  ka.block_point = e->block_point.p;
  ka.block_pair = e->block_pair.p;
  ka.pair_pose = e->pair_pose.p;
  ka.u_ref = e->u_ref.p;
  ka.host_int = e->host_int.p;
  ka.rho = e->rho.p;
  ka.u_obs = e->u_obs.p;
  ka.out = e->out.p;
  ka.cost = e->cost.p;
  ka.valid = e->valid.p;
  ka.n_blocks = e->n_blocks;
  ka.P = photometric ? e->P : 2;
  ka.huber = e->opt.huber_width;
  for (size_t i = 0; i < e->pattern_h.size() && i < 2 * PBA_MAX_PATTERN; ++i) ka.pattern[i] = e->pattern_h[i];
  const bool jac = want_jacobians != 0;
  hipEvent_t ev_stop = nullptr;
  if (e->timing) {
    while (e->ev_pool.size() < e->ev_used + 2) {
      hipEvent_t ev;
      PBA_HIP(hipEventCreate(&ev));
      e->ev_pool.push_back(ev);
    }
    PBA_HIP(hipEventRecord(e->ev_pool[e->ev_used], e->stream));
    ev_stop = e->ev_pool[e->ev_used + 1];
    e->ev_used += 2;
  }
  switch (e->opt.camera_model) {
    case PBA_CAMERA_PINHOLE: launch_blocks<CAM_PINHOLE>(e, ka, jac); break;
    case PBA_CAMERA_DOUBLE_SPHERE: launch_blocks<CAM_DS>(e, ka, jac); break;
    default: launch_blocks<CAM_EUCM>(e, ka, jac); break;
  }
  PBA_HIP(hipGetLastError());
  if (ev_stop) PBA_HIP(hipEventRecord(ev_stop, e->stream));
  e->evaluated = true;
  return PBA_OK;
}

int pba_enable_kernel_timing(pba_engine* e, int32_t enable) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  e->timing = enable != 0;
  return PBA_OK;
}

int pba_get_kernel_timing(pba_engine* e, double* total_ms, int32_t* launches) {
  if (!e || !total_ms) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(hipStreamSynchronize(e->stream));
  double tot = 0;
  for (size_t i = 0; i + 1 < e->ev_used; i += 2) {
    float ms = 0;
    PBA_HIP(hipEventElapsedTime(&ms, e->ev_pool[i], e->ev_pool[i + 1]));
    tot += ms;
  }
  *total_ms = tot;
  if (launches) *launches = (int32_t)(e->ev_used / 2);
  e->ev_used = 0;
  return PBA_OK;
}

int pba_synchronize(pba_engine* e) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

int pba_record_floats(const pba_engine* e) { return e ? 14 * e->R() : 0; }
int pba_residuals_per_block(const pba_engine* e) { return e ? e->R() : 0; }

int pba_get_records(pba_engine* e, float* records, uint8_t* valid) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (!e->evaluated) return fail(PBA_ERR_NOT_READY, "pba_evaluate first");
  if (int rc = check_device(e)) return rc;
  if (records)
    PBA_HIP(hipMemcpyAsync(records, e->out.p, (size_t)e->n_blocks * 14 * e->R() * sizeof(float), hipMemcpyDeviceToHost, e->stream));
  if (valid) PBA_HIP(hipMemcpyAsync(valid, e->valid.p, e->n_blocks, hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

int pba_get_block_costs(pba_engine* e, float* costs) {
  if (!e || !costs) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  if (!e->evaluated) return fail(PBA_ERR_NOT_READY, "pba_evaluate first");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(hipMemcpyAsync(costs, e->cost.p, e->n_blocks * sizeof(float), hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

int pba_get_cost(pba_engine* e, double* total, int32_t* n_valid) {
  if (!e || !total) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  std::vector<float> c(e->n_blocks);
  std::vector<uint8_t> v(e->n_blocks);
  if (int rc = pba_get_block_costs(e, c.data())) return rc;
  PBA_HIP(hipMemcpy(v.data(), e->valid.p, e->n_blocks, hipMemcpyDeviceToHost));
  double s = 0;
  int nv = 0;
  for (int i = 0; i < e->n_blocks; ++i) {
    s += c[i];
    nv += v[i];
  }
  *total = s;
  if (n_valid) *n_valid = nv;
  return PBA_OK;
}

int pba_device_records(pba_engine* e, float** d_records, uint8_t** d_valid, float** d_costs) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (d_records) *d_records = e->out.p;
  if (d_valid) *d_valid = e->valid.p;
  if (d_costs) *d_costs = e->cost.p;
  return PBA_OK;
}

}  // extern "C"
