// pba_internal.h — engine state, kernel argument blocks and the per-row residual/Jacobian arithmetic
// shared by the Ceres-mode kernels (pba_engine.hip) and the Gauss-Newton kernels (pba_gn.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <string>
#include <vector>

#include "pba.h"
#include "pba_device.h"
#include "pba_host.h"

namespace pba {
namespace detail {

// Test hooks — environment variables some GPU tests set (a forced decision mismatch, a host delay, the λ-specific
// elimination path, the 14-column A/B lineariser) — exist only in the library's test build (libpba_test.so, compiled
// with PBA_TEST_HOOKS; tests/helpers.py loads it for those tests).  The product library ignores them.
inline const char* test_hook(const char* name) {
#ifdef PBA_TEST_HOOKS
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
inline int test_hook_int(const char* name) {
  const char* v = test_hook(name);
  return v ? std::atoi(v) : 0;
}

constexpr int kBlockThreads = 256;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Relative pose of one (host, target) keyframe pair with the camera constants its residual rows need, 320 B
// (L2-resident: 4k pairs = 1.3 MB at C4).  Formed by form_pair: in the pair table (pair_kernel, state_kernel) or
// in a block kernel's LDS tile (fused state).
struct alignas(16) PairRec {
  double R[9];                 // R_th, fp64 (warp)
  double t[3];                 // t_th
  int host_cam, target_cam, target, host;
  double hk[kCamK];            // host camera, unprojection layout [cx cy 1/fx 1/fy p1 p2 p3 p4]
  double tk[kCamK];            // target camera, projection layout [fx fy cx cy p1 p2 p3 p4]
  float Rf[9], tf[3];          // fp32 R_th, t_th (Jacobian chain)
  float kf[8];                 // target camera, fp32 [fx fy 0 0 p1 p2 p3 p4] (projection Jacobian)
};
static_assert(sizeof(PairRec) == 320, "PairRec layout");
static_assert(offsetof(PairRec, hk) % 16 == 0 && offsetof(PairRec, tk) == offsetof(PairRec, hk) + 8 * kCamK,
              "camera constants: 8 contiguous 16-B parts (fused-state prologue)");

// Relative pose of pair (h, t) into r: q_th = q_wt*·q_wh, t_th = q_wt*·(t_wh − t_wt) in fp64 (photometric_error.h:
// 151-153; Hamilton product as so3.hpp:338-345, rotation as so3.hpp:367-370), with the camera constants.  The
// three parts write their fields in place, so r may live in LDS (tile prologue: one lane per part, which keeps
// the prologue's register peak below the row evaluation's) or in the pair table (pair_kernel: all three).
template <class Rec>  // PairRec or TileBlockC: fields R, Rf
__device__ __forceinline__ void pair_rotation(const double* __restrict__ H, const double* __restrict__ T, Rec& r) {
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
  double R[9];
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    r.R[j] = R[j];
    r.Rf[j] = (float)R[j];
  }
}
template <class Rec>  // PairRec or TileBlockC: fields t, tf
__device__ __forceinline__ void pair_translation(const double* __restrict__ H, const double* __restrict__ T,
                                                 Rec& r) {
  const double ax = -T[0], ay = -T[1], az = -T[2], aw = T[3];
  const double d0 = H[4] - T[4], d1 = H[5] - T[5], d2 = H[6] - T[6];
  double u0 = ay * d2 - az * d1, u1 = az * d0 - ax * d2, u2 = ax * d1 - ay * d0;
  u0 += u0; u1 += u1; u2 += u2;
  double tt[3];
  tt[0] = d0 + aw * u0 + (ay * u2 - az * u1);
  tt[1] = d1 + aw * u1 + (az * u0 - ax * u2);
  tt[2] = d2 + aw * u2 + (ax * u1 - ay * u0);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    r.t[j] = tt[j];
    r.tf[j] = (float)tt[j];
  }
}
// fp32 projection constants of the Jacobian chain from the fp64 projection layout (cx, cy unused there)
__device__ __forceinline__ void camera_kf(const double* __restrict__ tk, float* kf) {
  kf[0] = (float)tk[0];
  kf[1] = (float)tk[1];
  kf[2] = 0.0f;
  kf[3] = 0.0f;
#pragma unroll
  for (int j = 4; j < 8; ++j) kf[j] = (float)tk[j];
}
// the same from the 16-B part q ∈ [0, 4) of tk (tk[2q], tk[2q+1]) as one lane holds it in a tile prologue
__device__ __forceinline__ void camera_kf_part(const uint4& part, int q, float* kf) {
  const float2 v = q == 1 ? make_float2(0.0f, 0.0f)
                          : make_float2((float)__hiloint2double((int)part.y, (int)part.x),
                                        (float)__hiloint2double((int)part.w, (int)part.z));
  reinterpret_cast<float2*>(kf)[q] = v;
}
__device__ __forceinline__ void pair_cameras(const double* __restrict__ cams, int h, int t, int hc, int tc,
                                             PairRec& r) {
  r.host_cam = hc;
  r.target_cam = tc;
  r.target = t;
  r.host = h;
  const double* hk = cams + kCamD * hc + kCamHk;
  const double* tk = cams + kCamD * tc;
#pragma unroll
  for (int j = 0; j < kCamK; ++j) {
    r.hk[j] = hk[j];
    r.tk[j] = tk[j];
  }
  camera_kf(tk, r.kf);
}
__device__ __forceinline__ void form_pair(const double* __restrict__ poses, const int* __restrict__ frame_cam,
                                          const double* __restrict__ cams, int h, int t, PairRec& r) {
  pair_rotation(poses + 7 * h, poses + 7 * t, r);
  pair_translation(poses + 7 * h, poses + 7 * t, r);
  pair_cameras(cams, h, t, frame_cam[h], frame_cam[t], r);
}

// One block of a workgroup's tile, staged in LDS by stage_tile(): its pair record and its point.
struct alignas(16) TileBlock {
  PairRec pr;
  double2 ur;                  // u_ref (host pixel)
  double rho;                  // inverse distance (state)
  long long img;               // byte offset of the target's tiled image (target · frame_stride)
};
static_assert(sizeof(TileBlock) == 352, "TileBlock layout");
constexpr int kPairParts = sizeof(PairRec) / 16;     // 20 × 16 B
constexpr int kTileParts = sizeof(TileBlock) / 16;   // 22 × 16 B

// Compact tile block of the camera-table form (photometric_block_kernel_multi when the problem has ≤ kCamTab cameras):
// the pair's pose part and the point, 192 B instead of 352 — the two cameras' constants (160 B per block) live once
// per camera in a small LDS table (CamRec) — so the C5 kernel's 32-block tile shrinks by 5 KB and a sixth workgroup
// fits a CU.
struct alignas(16) TileBlockC {
  double R[9];
  double t[3];
  int host_cam, target_cam, target, host;
  float Rf[9], tf[3];
  double2 ur;
  double rho;
  long long img;
};
static_assert(sizeof(TileBlockC) == 192, "TileBlockC layout");
struct alignas(16) CamRec {
  double hk[kCamK];            // unprojection layout (as PairRec::hk)
  double tk[kCamK];            // projection layout (as PairRec::tk)
  float kf[8];                 // fp32 projection constants (as PairRec::kf)
};
static_assert(sizeof(CamRec) == 160, "CamRec layout");
constexpr int kCamTab = 4;     // cameras in the LDS table (mono, stereo and up to four-camera rigs)

// The pose part and the camera constants a photometric row reads, from either tile form.
struct CamView {
  const double* hk;
  const double* tk;
  const float* kf;
};
__device__ __forceinline__ const PairRec& pose_of(const TileBlock& tb) { return tb.pr; }
__device__ __forceinline__ const TileBlockC& pose_of(const TileBlockC& tb) { return tb; }
__device__ __forceinline__ CamView cams_of(const TileBlock& tb, const CamRec*) { return {tb.pr.hk, tb.pr.tk, tb.pr.kf}; }
__device__ __forceinline__ CamView cams_of(const TileBlockC& tb, const CamRec* tab) {
  return {tab[tb.host_cam].hk, tab[tb.target_cam].tk, tab[tb.target_cam].kf};
}

// Workgroups of 256 threads in one full wave of the chip (256 CUs × 8 resident workgroups at the headline kernel's 60
// VGPRs): launches up to this size store their record slabs write-through (store_slab).
constexpr int kSlabWtGrid = 2048;

struct KernelArgs {
  const uint8_t* images;
  int width, height, tiles_x;
  long long frame_stride;        // bytes per tiled frame
  double umax, vmax;             // interpolation clamp bounds W + 1, H + 1
  const float* intr;             // 8 floats per camera (Jacobian chain)
  const double* intr_d;          // kCamD doubles per camera (warp / projection; pba_device.h)
  const float* intr_t;           // the target cameras' projection constants (geometric kernels): intr, or the
  const double* intr_t_d;        // intrinsics state of pba_set_optimize_intrinsics (host unprojection stays on intr_d)
  const int* block_point;
  const int* block_pair;
  const int2* block_pp;          // per block {point, pair}
  const PairRec* pairs;          // pair table (used when poses == nullptr)
  const double* poses;           // state poses: when set, every block forms its pair record in the tile prologue
  const int4* block_rec;         // per block {point, host, target, host_cam << 16 | target_cam} (with poses)
  double* adopt_poses;           // when set, the launch also copies poses/rho (the state it evaluates at) here
  double* adopt_rho;
  int n_pose_d;                  // 7 × frames
  int n_points;
  const double2* u_ref;          // per point
  const float* host_int;         // P per point
  const double* rho;             // per point (state)
  const double2* u_obs;          // per block (geometric)
  float* out;                    // records
  float* res_out;                // residual-only launches: R contiguous fp32 residuals per block (pba_get_residuals)
  float* cost;                   // per block
  uint8_t* valid;                // per block
  int n_blocks;
  int P;
  int n_cams;                    // cameras (photometric_block_kernel_multi's camera table: ≤ kCamTab)
  float huber;
  double* wg_red;  // residual-only launches of the LM loop: per-workgroup (Σ cost, Σ valid) at slot logical_tile()
  int slab_wt;     // record slabs stored write-through (store_slab: grids of ≤ kSlabWtGrid workgroups)
  float pattern[2 * PBA_MAX_PATTERN];
};

// Camera 0's constants read through the constant address space: uniform scalar loads (photometric rows of a
// one-camera problem; the same values the tile prologues copy).
__device__ __forceinline__ CamView single_camera(const KernelArgs& a) {
  typedef const __attribute__((address_space(4))) double cdouble;
  typedef const __attribute__((address_space(4))) float cfloat;
  return {(const double*)(cdouble*)(a.intr_d + kCamHk), (const double*)(cdouble*)a.intr_d,
          (const float*)(cfloat*)a.intr};
}

// XCD-aware tile order: consecutive logical tiles (→ neighbouring host keyframes → shared target images)
// land on the same XCD's L2 (blocks are dealt round-robin over the 8 XCDs; speed only, never correctness).
__device__ __forceinline__ int logical_tile() {
  const int n = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3;
  const int q = n >> 3, rem = n & 7;
  return xcd * q + min(xcd, rem) + slot;
}

// Σ over the workgroup of two per-lane values in a fixed order (xor butterflies in each wave, then the waves in
// order): bitwise reproducible.  Every thread of the workgroup must call it; thread 0 writes out[0..1].
__device__ __forceinline__ void wg_reduce2(double a, double b, double* out) {
  __shared__ double sa[16], sb[16];
  for (int m = 32; m >= 1; m >>= 1) {
    a += __shfl_xor(a, m, 64);
    b += __shfl_xor(b, m, 64);
  }
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
  if (l == 0) { sa[w] = a; sb[w] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double x = 0, y = 0;
    for (int i = 0; i < (int)(blockDim.x / 64); ++i) { x += sa[i]; y += sb[i]; }
    out[0] = x;
    out[1] = y;
  }
}

// Huber loss (loss_function.cc:48-62): cost = ½ρ(s); Corrector weight ρ'(s) (corrector.cc:42-110 — ρ'' ≤ 0
// for Huber, so Ceres scales r and J by √ρ' and the normal equations by ρ').
__device__ __forceinline__ float huber_cost(float s, float a) {
  if (a <= 0.0f || s <= a * a) return 0.5f * s;
  return 0.5f * (2.0f * a * __builtin_amdgcn_sqrtf(s) - a * a);  // v_sqrt_f32 (1 ulp)
}
__device__ __forceinline__ float huber_weight(float s, float a) {
  if (a <= 0.0f || s <= a * a) return 1.0f;
  return fmaxf(a * rsqrtf(s), 1.17549435e-38f);
}

// All-reduce over the LPB lanes of one block (LPB | 64, groups are aligned lane ranges) with DPP lane
// moves fused into the adds: quad_perm [1,0,3,2] and [2,3,0,1] (xor 1, xor 2), row_half_mirror (pairs the two
// quads of an 8-lane group), row_mirror (the two halves of a 16-lane row), then a swizzle for 32.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int LPB>
__device__ __forceinline__ float group_sum(float v) {
  if (LPB >= 2) v += dpp<0xB1>(v);
  if (LPB >= 4) v += dpp<0x4E>(v);
  if (LPB >= 8) v += dpp<0x141>(v);
  if (LPB >= 16) v += dpp<0x140>(v);
  if (LPB >= 32) v += __shfl_xor(v, 16, 64);
  if (LPB >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
template <int LPB>
__device__ __forceinline__ int group_and(int v) {
#pragma unroll
  for (int m = LPB / 2; m >= 1; m >>= 1) v &= __shfl_xor(v, m, 64);
  return v;
}

// AND over the LPB lanes of one block from a wave ballot (the block's lanes are an aligned bit field).
// Every lane of the wave must be active.
template <int LPB>
__device__ __forceinline__ int group_all(int v) {
  const unsigned long long m = __ballot(v != 0);
  const unsigned long long grp = LPB >= 64 ? ~0ull : ((1ull << LPB) - 1ull);
  const int sh = (int)(__lane_id() & (64 - LPB));
  return ((m >> sh) & grp) == grp;
}

// One residual row with its tangent Jacobian: r, ∂r/∂[υ_h ω_h], ∂r/∂[υ_t ω_t], ∂r/∂ρ.
struct Row {
  float r = 0.0f, jr = 0.0f;
  Vec3 hv = {0, 0, 0}, hw = {0, 0, 0}, tv = {0, 0, 0}, tw = {0, 0, 0};
  int ok = 1;
};

// Cooperative tile prologue: the LPB lanes of block lb copy its pair record, u_ref and ρ into LDS as
// kTileParts 16-B parts (lane k takes parts k, k+LPB, …) — one broadcast copy per block instead of every lane
// loading the record and the point data itself — or, with a.poses set, form the pair record from the state
// (no pair-table launch before the evaluation).  Returns the block's point.  The caller barriers.
template <int LPB>
__device__ __forceinline__ int stage_tile_pp(const KernelArgs& a, TileBlock* s_tb, int lb, int k, int2 pp);
template <int LPB>
__device__ __forceinline__ int stage_tile(const KernelArgs& a, TileBlock* s_tb, int lb, int k, int blk, bool live) {
  // a dead block (past the end of the problem) stages the last block, so every lane evaluates valid data
  uint4* dst = reinterpret_cast<uint4*>(s_tb + lb);
  if (LPB >= 8 && a.poses) {  // (LPB < 8: linearize of geometric rows, always on the table path)
    // Fused state: the block's lanes issue every load first, with lane-dependent addresses and no branches (one
    // memory round trip, as on the table path), then lane 0 forms R_th, lane 1 t_th and the ids, lane k copies
    // camera part k (hk: parts 0-3, tk: 4-7), lanes 2-3 the point.  The block record carries host, target and
    // cameras, so this is as many dependent loads as the table path.
    static_assert(kCamK == 8, "fused prologue: 8 camera parts");
    const int4 br = a.block_rec[live ? blk : a.n_blocks - 1];
    const double* H = a.poses + 7 * br.y;
    const double* T = a.poses + 7 * br.z;
    double h[7], t[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      h[j] = H[j];
      t[j] = T[j];
    }
    const int hc = br.w >> 16, tc = br.w & 0xffff, kc = k & 7;
    const uint4 cam = reinterpret_cast<const uint4*>(a.intr_d + (kc < 4 ? kCamD * hc + kCamHk : kCamD * tc))[kc & 3];
    const uint4 ur = reinterpret_cast<const uint4*>(a.u_ref)[br.x];
    const double rho = a.rho[br.x];
    // every load above completes here, before the lanes diverge (otherwise the compiler sinks each load into the
    // one branch that uses it and the branches pay a memory round trip each, serially)
    asm volatile("" ::"v"(cam.x), "v"(cam.y), "v"(cam.z), "v"(cam.w), "v"(ur.x), "v"(ur.y), "v"(ur.z), "v"(ur.w),
                 "v"(rho));
#pragma unroll
    for (int j = 0; j < 7; ++j) asm volatile("" ::"v"(h[j]), "v"(t[j]));
    PairRec& pr = s_tb[lb].pr;
    if (k < 8) dst[(int)(offsetof(PairRec, hk) / 16) + k] = cam;
    if (k >= 4 && k < 8) camera_kf_part(cam, k - 4, pr.kf);
    if (k == 0) {
      pair_rotation(h, t, pr);
    } else if (k == 1) {
      pair_translation(h, t, pr);
      pr.host_cam = hc;
      pr.target_cam = tc;
      pr.target = br.z;
      pr.host = br.y;
    } else if (k == 2) {
      dst[kPairParts] = ur;
    } else if (k == 3) {
      const long long img = (long long)br.z * a.frame_stride;
      dst[kPairParts + 1] = make_uint4(__double2loint(rho), __double2hiint(rho), (unsigned)img, (unsigned)(img >> 32));
    }
    return br.x;
  }
  return stage_tile_pp<LPB>(a, s_tb, lb, k, a.block_pp[live ? blk : a.n_blocks - 1]);
}

// Table path with the block's {point, pair} already in hand (linearize_kernel reads it with its linearise record).
template <int LPB>
__device__ __forceinline__ int stage_tile_pp(const KernelArgs& a, TileBlock* s_tb, int lb, int k, int2 pp) {
  // every load first, unconditionally and at in-range addresses (a lane past the last part re-reads part 0; the point's
  // ρ and the target id are read by every lane, one request per block), then the selects: per-part branches around
  // the loads made the compiler issue and wait for them one branch at a time (three memory round trips)
  constexpr int NP = (kTileParts + LPB - 1) / LPB;
  uint4* dst = reinterpret_cast<uint4*>(s_tb + lb);
  const uint4* src = reinterpret_cast<const uint4*>(a.pairs + pp.y);
  uint4 v[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int part = k + LPB * i;
    v[i] = part == kPairParts ? reinterpret_cast<const uint4*>(a.u_ref)[pp.x] : src[part < kPairParts ? part : 0];
  }
  const double r = a.rho[pp.x];
  const int tgt = a.pairs[pp.y].target;
  asm volatile("" ::"v"(r), "v"(tgt));
#pragma unroll
  for (int i = 0; i < NP; ++i) asm volatile("" ::"v"(v[i].x), "v"(v[i].y), "v"(v[i].z), "v"(v[i].w));
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int part = k + LPB * i;
    if (part == kPairParts + 1) {
      const long long img = (long long)tgt * a.frame_stride;
      v[i] = make_uint4(__double2loint(r), __double2hiint(r), (unsigned)img, (unsigned)(img >> 32));
    }
    if (part < kTileParts) dst[part] = v[i];
  }
  return pp.x;
}

// Fused state, workgroup-cooperative form for 256-thread workgroups of 32 blocks: the four waves split the 32
// blocks' prologue by part instead of each wave staging its own 8 blocks — wave 0 forms R_th of all 32 (lane b < 32),
// wave 1 t_th and the ids, wave 2 copies the cameras' constants (lanes 0-31 the host part, 32-63 the target part
// with its fp32 copy), wave 3 the point data (lanes 0-31 u_ref, 32-63 ρ).  The fp64 relative-pose arithmetic is then
// issued once per workgroup instead of once per wave (SIMT: a wave pays for every branch any of its lanes takes, so
// the rotation and translation branches of stage_tile cost each of the four waves both).  The caller barriers.
__device__ __forceinline__ void stage_tile_wg(const KernelArgs& a, TileBlock* s_tb, int blk0) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, b = lane & 31;
  const int4 br = a.block_rec[min(blk0 + b, a.n_blocks - 1)];  // a dead block stages the last block
  PairRec& pr = s_tb[b].pr;
  uint4* dst = reinterpret_cast<uint4*>(s_tb + b);
  if (w == 0) {
    if (lane < 32) {
      const double* H = a.poses + 7 * br.y;
      const double* T = a.poses + 7 * br.z;
      double h[4], t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h[j] = H[j];
        t[j] = T[j];
      }
      pair_rotation(h, t, pr);
    }
  } else if (w == 1) {
    if (lane < 32) {
      const double* H = a.poses + 7 * br.y;
      const double* T = a.poses + 7 * br.z;
      double h[7], t[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        h[j] = H[j];
        t[j] = T[j];
      }
      pair_translation(h, t, pr);
      pr.host_cam = br.w >> 16;
      pr.target_cam = br.w & 0xffff;
      pr.target = br.z;
      pr.host = br.y;
    }
  } else if (w == 2) {
    const bool tgt = lane >= 32;
    const uint4* src = reinterpret_cast<const uint4*>(a.intr_d + (tgt ? kCamD * (br.w & 0xffff) : kCamD * (br.w >> 16) + kCamHk));
    uint4 c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = src[q];
    uint4* d = dst + (int)(offsetof(PairRec, hk) / 16) + (tgt ? 4 : 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = c[q];
    if (tgt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) camera_kf_part(c[q], q, pr.kf);
    }
  } else {
    if (lane < 32) {
      dst[kPairParts] = reinterpret_cast<const uint4*>(a.u_ref)[br.x];
    } else {
      const double rho = a.rho[br.x];
      const long long img = (long long)br.z * a.frame_stride;
      dst[kPairParts + 1] = make_uint4(__double2loint(rho), __double2hiint(rho), (unsigned)img, (unsigned)(img >> 32));
    }
  }
}

// The same for the compact tile (TileBlockC) and the LDS camera table of n_cams ≤ kCamTab cameras: waves 0, 1 and 3
// as above; wave 2 copies the camera table instead of every block's two cameras (lane = 16-B part: per camera the four
// parts of hk, the four of tk, and the fp32 kf from tk's).  The caller barriers.
__device__ __forceinline__ void stage_tile_wg_ct(const KernelArgs& a, TileBlockC* s_tb, CamRec* s_cam, int n_cams,
                                                 int blk0) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, b = lane & 31;
  const int4 br = a.block_rec[min(blk0 + b, a.n_blocks - 1)];  // a dead block stages the last block
  TileBlockC& tb = s_tb[b];
  if (w == 0) {
    if (lane < 32) {
      const double* H = a.poses + 7 * br.y;
      const double* T = a.poses + 7 * br.z;
      double h[4], t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h[j] = H[j];
        t[j] = T[j];
      }
      pair_rotation(h, t, tb);
    }
  } else if (w == 1) {
    if (lane < 32) {
      const double* H = a.poses + 7 * br.y;
      const double* T = a.poses + 7 * br.z;
      double h[7], t[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        h[j] = H[j];
        t[j] = T[j];
      }
      pair_translation(h, t, tb);
      tb.host_cam = br.w >> 16;
      tb.target_cam = br.w & 0xffff;
      tb.target = br.z;
      tb.host = br.y;
    }
  } else if (w == 2) {
    // lane = camera c (lane >> 3) × part q (lane & 7): q < 4 → hk part q, q ≥ 4 → tk part q − 4 (+ its fp32 kf)
    const int c = lane >> 3, q = lane & 7;
    if (c < n_cams) {
      const uint4 v = reinterpret_cast<const uint4*>(a.intr_d + (q < 4 ? kCamD * c + kCamHk : kCamD * c))[q & 3];
      uint4* d = reinterpret_cast<uint4*>(s_cam + c);
      d[q] = v;  // hk parts 0-3, tk parts 4-7 (CamRec: hk then tk, contiguous)
      if (q >= 4) camera_kf_part(v, q - 4, s_cam[c].kf);
    }
  } else {
    if (lane < 32) {
      tb.ur = a.u_ref[br.x];
    } else {
      tb.rho = a.rho[br.x];
      tb.img = (long long)br.z * a.frame_stride;
    }
  }
}

// Pattern offset k (k < N) read from the kernel arguments with scalar loads at constant offsets and picked per lane
// by selects.  A lane-indexed read of the argument block is a vector-memory load, and staging it through LDS made
// every workgroup wait one memory round trip before it issued any other load.
template <int N>
__device__ __forceinline__ float2 pattern_at(const KernelArgs& a, int k) {
  float2 o = make_float2(a.pattern[0], a.pattern[1]);
#pragma unroll
  for (int j = 1; j < N; ++j)
    if (k == j) o = make_float2(a.pattern[2 * j], a.pattern[2 * j + 1]);
  return o;
}

// The launch that evaluates at a caller's state also adopts it: one element per lane (grid ≥ frames·7, points).
__device__ __forceinline__ void adopt_state(const KernelArgs& a) {
  if (!a.adopt_rho) return;
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.n_points && g >= a.n_pose_d) return;
  const double r = a.rho[g < a.n_points ? g : 0], p = a.poses[g < a.n_pose_d ? g : 0];
  asm volatile("" ::"v"(r), "v"(p));  // both loads in flight together (see stage_tile)
  if (g < a.n_points) a.adopt_rho[g] = r;
  if (g < a.n_pose_d) a.adopt_poses[g] = p;
}

// Photometric row k of a staged block (photometric_error.h:139-182 with the bilinear or Ceres' bicubic interpolator; the
// Jacobian chain of pba_device.h).  Warp and projection in fp64, chain in fp32.  off = pattern offset k,
// Ih = host intensity I_h,k.
// PM = camera model + 4 · interpolator (pba_device.h cam_of / interp_of).
// TB = TileBlock (cameras in the block), or TileBlockC with the LDS camera table `tab`.
template <int PM, bool JAC, class TB = TileBlock, bool C1 = false>
__device__ __forceinline__ Row photometric_row(const KernelArgs& a, const TB& tb, float2 off, float Ih,
                                               const CamRec* tab = nullptr) {
  constexpr int MODEL = cam_of(PM);
  Row o;
  const auto& pp = pose_of(tb);
  const CamView cv = C1 ? single_camera(a) : cams_of(tb, tab);
  const double rho = tb.rho;
  // p̃ = R_th b_k + ρ t_th  (photometric_error.h:158-159)
  const Vec3d b = unproject<MODEL>(cv.hk, tb.ur.x + (double)off.x, tb.ur.y + (double)off.y);
  const Vec3d Rb = mat_mul(pp.R, b);
  const Vec3d p = {Rb.x + rho * pp.t[0], Rb.y + rho * pp.t[1], Rb.z + rho * pp.t[2]};
  // Branch-free: the projection and the taps run whatever the domain test says (the interpolator clamps any
  // position, NaN and ±inf included, to an in-bounds read), and the caller masks a block that is not ok.  A branch
  // here costs every lane the zero-initialised Row and the exec bookkeeping, and no wave ever skips it.
  const bool dom = in_domain<MODEL>(cv.tk, p);
  float I, gx, gy;
  double u, v;
  const double iden = project<MODEL>(cv.tk, p, u, v);
  interpolate<interp_of(PM)>(a.images + tb.img, a.umax, a.vmax, a.tiles_x, u, v, I, gx, gy);
  o.r = I - Ih;  // photometric_error.h:179
  o.ok = dom && isfinite(o.r);
  if (JAC) {
    // q = ∇I · ∂π/∂p̃ (1×3)
    const Vec3 pf = to_f(p), bf = to_f(b);
    Vec3 du, dv;
    project_jac<MODEL>(cv.kf, pf, (float)iden, du, dv);
    const Vec3 q = {gx * du.x + gy * dv.x, gx * du.y + gy * dv.y, gx * du.z + gy * dv.z};
    const Vec3 qR = row_mul(q, pp.Rf);
    const float rf = (float)rho;
    o.hv = {rf * qR.x, rf * qR.y, rf * qR.z};
    o.hw = cross(bf, qR);  // −(qR)×b
    o.tv = {-rf * q.x, -rf * q.y, -rf * q.z};
    o.tw = cross(q, pf);   // q·[p̃]×
    // ∂r/∂ρ = ∇I·∂π/∂p̃·t: ∂π/∂p̃·t cancels when t points along the ray (the epipolar motion is small),
    // so the cancelling part runs in fp64 (fp32 left ~3e-5 relative error on J_ρ at short baselines)
    if (MODEL == CAM_PINHOLE) {
      // ∂u/∂p̃·t = fx/z (t_x − m_x t_z), ∂v/∂p̃·t = fy/z (t_y − m_y t_z), m = p̃_xy / z (the projection's own
      // quotients): 7 fp64 operations instead of the general 2×3 Jacobian and two dot products
      const double ex = fma(-(p.x * iden), pp.t[2], pp.t[0]), ey = fma(-(p.y * iden), pp.t[2], pp.t[1]);
      o.jr = (float)(iden * fma((double)gx * cv.tk[0], ex, (double)gy * cv.tk[1] * ey));
    } else {
      Vec3d dud, dvd;
      project_jac<MODEL>(cv.tk, p, iden, dud, dvd);
      const Vec3d td = {pp.t[0], pp.t[1], pp.t[2]};
      o.jr = (float)((double)gx * dot(dud, td) + (double)gy * dot(dvd, td));
    }
  }
  return o;
}

// Geometric row k ∈ {0: u, 1: v} of block blk (reprojection.h:105-108): r = u_obs − π_t(T_th · b/ρ).
template <int MODEL, bool JAC>
__device__ __forceinline__ Row geometric_row(const KernelArgs& a, int blk, int k) {
  Row o;
  const int pt = a.block_point[blk];
  const PairRec& pp = a.pairs[a.block_pair[blk]];
  const double2 ur = a.u_ref[pt];
  const double2 uo = a.u_obs[blk];
  const double irho = rcp_nr(a.rho[pt]);
  const Vec3d b = unproject<MODEL>(a.intr_d + kCamD * pp.host_cam + kCamHk, ur.x, ur.y);
  const Vec3d ph = {b.x * irho, b.y * irho, b.z * irho};
  const Vec3d Rp = mat_mul(pp.R, ph);
  const Vec3d p = {Rp.x + pp.t[0], Rp.y + pp.t[1], Rp.z + pp.t[2]};
  double u, v;
  // the target camera projects with the intrinsics state (intr_t: the cameras, or the free intrinsics of
  // pba_set_optimize_intrinsics / a candidate's), the host unprojects with the cameras (reprojection.h:93-98)
  const double iden = project<MODEL>(a.intr_t_d + kCamD * pp.target_cam, p, u, v);
  o.r = (float)(k == 0 ? uo.x - u : uo.y - v);
  o.ok = isfinite(o.r);
  if (JAC) {
    const Vec3 pf = to_f(p), phf = to_f(ph);
    Vec3 du, dv;
    project_jac<MODEL>(a.intr_t + 8 * pp.target_cam, pf, (float)iden, du, dv);
    const Vec3 d = k == 0 ? du : dv;
    const Vec3 g = {-d.x, -d.y, -d.z};  // ∂r/∂p = −∂π/∂p
    const Vec3 gR = row_mul(g, pp.R);
    o.hv = gR;
    o.hw = cross(phf, gR);
    o.tv = d;
    o.tw = cross(g, pf);
    // ∂r/∂ρ = ∂π/∂p·R b/ρ² = −∂π/∂p·t/ρ, because ∂π/∂p·p = 0 for every central projection (π(λp) = π(p)):
    // the second form has no cancellation (the first loses ~1e-5 relative in fp32 at small baselines)
    const Vec3 tf = {(float)pp.t[0], (float)pp.t[1], (float)pp.t[2]};
    o.jr = -dot(d, tf) * (float)irho;
    o.ok = o.ok && isfinite(o.hv.x + o.hv.y + o.hv.z + o.hw.x + o.hw.y + o.hw.z) &&
           isfinite(o.tw.x + o.tw.y + o.tw.z + o.tv.x + o.tv.y + o.tv.z + o.jr);
  }
  return o;
}

// ---------------------------------------------------------------------------------------------------------
// Host-side helpers
// ---------------------------------------------------------------------------------------------------------
#define PBA_HIP(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return ::pba::detail::fail(e_ == hipErrorOutOfMemory ? PBA_ERR_OUT_OF_MEMORY : PBA_ERR_DEVICE, \
                                 std::string(#expr) + ": " + hipGetErrorString(e_));           \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
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
  hipError_t upload(const std::vector<T>& h, hipStream_t s) {
    hipError_t e = resize(h.size());
    if (e != hipSuccess || h.empty()) return e;
    return hipMemcpyAsync(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s);
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// Page-locked host buffer: the per-iteration read-backs of the LM loop are then true async DMA copies (a pageable
// destination is staged through a driver buffer, which serialised back-to-back D2H copies by ~20 µs).
template <class T>
struct PinnedBuf {
  T* p = nullptr;
  size_t n = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t resize(size_t count, unsigned flags = hipHostMallocDefault) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), (count ? count : 1) * sizeof(T), flags);
    if (e == hipSuccess) n = count;
    return e;
  }
  T* data() { return p; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
};

enum : int { SOLVER_SKYLINE = 0, SOLVER_BAND = 1, SOLVER_CR = 2 };
struct CrLevelHost {
  size_t D = 0, U = 0, b = 0, X = 0, x = 0;
  int n = 0;
};

// Gauss-Newton state: the symbolic analysis of the normal equations (built once per problem structure) and
// the device buffers of one linearisation / Schur complement / solve.  See pba_gn.hip for the layouts.
// front_solve_kernel's plan (pba_gn.hip, build_front_plan): per column k one record of kFrontHdr + 3·fm + 2·mf ints — the
// slot of k, the column's row count, the fresh-block count, then the rows' slots, indices and factor blocks, then the
// fresh blocks (source skyline block, front position) that the next column admits; the rows admitted at column 0 in init.
struct FrontPlan {
  DevBuf<int> rec;
  DevBuf<int2> init;
  DevBuf<double> lrec;  // per column: L_kk (36) | reciprocal pivots (6) | y_k (6)
  int F = 0, fm = 0, mf = 0, R = 0, n_init = 0;
  size_t lds = 0;       // 0: the profile's front does not fit (skyline_solve_kernel)
};

struct GnData {
  bool prepared = false;
  int lpb = 8, bpw = 32, ppl = 1;  // linearisation: lanes per block, blocks per chunk, rows per lane
  int n_chunks = 0, n_schur = 0, n_gn_points = 0, n_sky = 0, band = 0, band_kernel = 0, solver = 0;
  std::vector<CrLevelHost> cr_levels;  // block-cyclic-reduction level layout (offsets into cr_buf)
  int cr_pcr = -1;                     // the CR level whose rows parallel cyclic reduction solves (-1: root kernel)
  CrLevelHost pcr_bufs[2];             // PCR ping-pong buffers (D, U, b) for that level's rows
  DevBuf<double> cr_buf;
  bool force_skyline = false;
  size_t lin_slots = 0, schur_doubles = 0, schur_lds = 0;
  // linearise order (GN order regrouped by target within each host), bpw slots per chunk (a chunk's dead slots
  // repeat its first block): {block, point, pair | local target slot << 24, GN position}
  DevBuf<int4> lin_rec;
  DevBuf<int4> chunk_desc;       // linearise chunk: first linearise position, count, n_targets, partial offset
  // The normal-equation pieces are fp64: the block products of the fp32 rows are formed on the fp64 matrix cores, so
  // JᵀJ is the exact Gram matrix of the rows and stays consistent with the point elimination's W W / H (fp32 products
  // and sums gave the reduced system errors of ~1e-7 of its scale that its condition number, ~1e11 at C4, turned into
  // wrong steps once the trust region had grown: DESIGN.md §4, tests/test_gpu_configs.py).
  DevBuf<double> blk_schur;      // GN block → 8 doubles [H_ρρ g_ρ W_t(6)] (W_h follows from W_t, pair_rt: schur_chunk)
  DevBuf<double> part_lin;       // linearise chunk partials
  DevBuf<double> pair_rt, pair_rt1;  // per pair [R_th(9) t_th(3)] of the linearisation in blk_schur / blk_schur1
  DevBuf<int> schur_lvp;         // per Schur chunk (offset aux.z): the pair of each local target lv = 1 … nv − 1 …
  DevBuf<int4> schur_lvp4;       // … and its first four, read with the chunk's descriptors
  int schur_rt_off = 0;          // doubles of R, t per Schur workgroup at the start of its dynamic LDS (12 per target)
  DevBuf<double> blk_schur1, part_lin1;  // second set: the device LM loop linearises each candidate into the spare
  DevBuf<int> pt_first, pt_nblk, pt_orig;  // GN point → first GN block, block count, original point
  DevBuf<int4> pt_rec;           // GN point → {first GN block, block count, host frame, original point} (one load)
  DevBuf<int4> pt_tgt;           // GN point → the targets of its first four GN blocks (the update's x_t loads in round 2)
  DevBuf<int4> pair_rec;         // pair → {host, target, host camera, target camera}
  DevBuf<int2> pt_fb;            // Schur chunk c's point p → {first GN block, block count} at c · SCHUR_PTS + p
  DevBuf<int4> schur_desc;       // Schur chunk: first GN point, n points, n local poses, partial offset
  DevBuf<int4> schur_aux;        // Schur chunk: pair list offset, n pairs, first GN block, n blocks
  DevBuf<uchar2> schur_pairs;    // used local pose pairs (a ≤ b) of every Schur chunk
  DevBuf<int> pt_host, gn_target;  // GN point → host frame; GN block → target frame
  DevBuf<double> drho;           // last step's δρ (original point order)
  std::vector<uint8_t> fixed_eff;  // constant frames actually used (requested + unobserved)
  DevBuf<uint8_t> blk_lv;        // GN block → local pose index of its target in its Schur chunk
  DevBuf<double> part_schur;     // Schur chunk partials (fp64)
  DevBuf<double> pt_data;        // GN point → [H'll, gl, Wh(6)] of the last Schur pass (fp64); set 0 of the LM loop
  // the single-GPU LM loop's λ-free point elimination (schur_free_decide_kernel): per linearisation set the partials
  // Σ W Wᵀ/H, Σ W g/H and the point data, a flag for a point outside the LM clamp, the set the last linearisation wrote
  DevBuf<double> part_free0, part_free1, pt_data1;
  DevBuf<int> degen, lin_set;
  DevBuf<double> ts_part;  // the decision workgroups' slices of the trial sums (schur_free_decide_kernel) …
  DevBuf<int> ts_count;    // … and their arrival count
  // test build (PBA_TEST_HOOKS) only: the λ-specific point elimination on every trial (PBA_TEST_FORCE_DEGEN), the
  // 14-column linearisation (linearize_kernel) for ≤ 8-px photometric patterns instead of the adjoint form (PBA_LIN_LEGACY)
  bool force_degen = pba::detail::test_hook("PBA_TEST_FORCE_DEGEN") != nullptr;
  bool lin_legacy = pba::detail::test_hook("PBA_LIN_LEGACY") != nullptr;
  DevBuf<int> sky_first, sky_row, sky_last;  // skyline profile of the reduced camera system
  DevBuf<int> sky_cptr, g_cptr;  // contribution lists (CSR) per skyline block / per pose
  DevBuf<int2> sky_contrib, g_contrib;
  DevBuf<int> sky_blk_i, sky_blk_j;  // skyline block → (row pose, column pose)
  DevBuf<int> sky_diag, sky_off;     // the diagonal skyline blocks, the others (assemble_kernel's thread ranges)
  DevBuf<int> sky_colptr, sky_colrows;  // per column k, the rows i > k of the profile (first(i) ≤ k): skyline solve
  int n_sky_diag = 0;
  FrontPlan front;   // front_solve_kernel's plan for the local skyline profile (gn_prepare)
  // multi-GPU with free intrinsics: the summed system's profile — the exchange band K over the keyframes, the border rows
  // from frame 0 — its skyline system, factor blocks, row offsets and plan (ensure_dist_sky, for dsky_K)
  FrontPlan dfront;
  DevBuf<double> dS, dL;
  DevBuf<int> dsky_row, dsky_first, dsky_last, dsky_colptr, dsky_colrows;
  int dsky_K = -1, n_dsky = 0;
  // free intrinsics as an ARROW system (pba_gn.hip arrow_solve): the keyframe band by parallel cyclic reduction with
  // the border's columns as extra right-hand sides, then the small dense border Schur complement.  ar_n super-rows of 4
  // keyframes, ar_batches runs of kArrowNB columns side by side; buffers: level 0 (D, U and every batch's b) + two
  // ping-pong levels (per batch D, U, b of kArrowNB columns), the solutions X (6·nf rows × 16·ar_batches), the border
  // reduction's partials, the border step.
  bool arrow = false;           // the local (single-GPU) free-intrinsics system is solved as an arrow
  int ar_n = 0, ar_batches = 0;
  DevBuf<double> ar_buf, ar_X, ar_part, ar_dc;
  DevBuf<double> S, L, Sband, Lband, g, g_dir, Ddiag, Linv, x;  // skyline system, its factor, rhs, direct gradient, LM diagonal, L_kk⁻¹, step
  DevBuf<uint8_t> fixed;
  DevBuf<uint8_t> observed, fixed_req, fixed_dist;  // multi-GPU: local observation flags, requested / effective constants
  bool sband_dirty = false;                         // Sband fully written by a distributed import
  bool cr0_dirty = true;                            // CR level 0 not (re)initialised for assemble's direct writes
  bool cr0_inited = false;                          // CR level 0 has its zeros and padding (init_cr_level0)
  std::vector<uint8_t> fixed_h;
  DevBuf<double> poses_new, rho_new, red;
  DevBuf<double> red2, gmax;  // update partials: (Σ step², Σ x_new²) and max gradient component per slot (lm_decide)
  DevBuf<double> tpose;       // multi-GPU: the trial's pose-part sums (dist_sums_kernel)
  DevBuf<double> exchange;    // multi-GPU exchange buffer of pba_solve_distributed_comm
  DevBuf<int> status;
  DevBuf<PairRec> pairs_new;
  bool pairs_new_fresh = false;  // pairs_new formed by the last update_kernel (its candidate state)
  PinnedBuf<double> red_h;
  DevBuf<double> lm;         // LM decision record of the single-GPU loop (pba_gn.hip: kLm*)
  DevBuf<double> lm_init;    // the solve's initial cost and valid blocks (lm_init_kernel)
  DevBuf<double> lm_idle;    // the record host-driven steps pass to the kernels (not done, set 0, λ from the argument)
  PinnedBuf<double> lm_h;    // its host copy (+ sequence number), host-coherent, written by lm_decide_kernel
  // Intrinsics in the reduced camera system (pba_set_optimize_intrinsics, geometric engines; pba_gn.hip "intrinsics"):
  // camera c's 8 intrinsics are the system frames nf + 2c (dims 0-5) and nf + 2c + 1 (dims 6-7, four identity pads), a
  // dense border of the skyline system.  nc_sys = 0 without intrinsics; nfs = nf + 2·nc_sys system frames.
  int nc_sys = 0, nfs = 0;
  int dist_rank = -1;           // rank in a host-callback collective (pba_gn_set_rank); −1 unknown
  DevBuf<int4> ib_rec;          // GN block → {block, point, host, target}
  DevBuf<double> ib_data;       // GN block → weighted fp64 rows [J_i (2×8) | J_h (2×6) | J_t (2×6) | J_ρ (2) | r (2) | W_i (8)]
  DevBuf<double> ib_pw;         // GN point → W_c (8 per camera), W_h (6): intr_pw_kernel
  DevBuf<int> ib_bptr, ib_blist;  // border unit pair (camera c, unit u) → GN blocks of its direct terms (CSR)
  DevBuf<int> ib_pptr, ib_plist;  // … → GN points of its Schur terms (CSR); unit u < nf: frame u, else camera u − nf
  DevBuf<int4> ir_wave;           // intr_rows_kernel's point-aligned waves {first GN block, blocks, first GN point}
  int ir_waves = 0;               // their number (0: 64-block waves + intr_pw_kernel)
  DevBuf<int> ib_pblk;            // per ib_plist entry: −1 (host / camera unit), the point's block targeting frame u, −2
  DevBuf<int> ib_cam;           // GN block → its target's camera
  DevBuf<double> ib_part;       // the camera-block reductions' per-workgroup totals (intr_cam_dir / intr_cam_sch_kernel)
  DevBuf<double> intr_new_d;    // candidate intrinsics: camera records (kCamD doubles, projection part) …
  DevBuf<float> intr_new_f;     // … and their fp32 copy (8 per camera)
  double* lm_host_d = nullptr;  // lm_h's device address
  bool phase_timing = false;    // pba_set_solver_timing: stream events around the LM phases
  std::vector<pba_iteration_summary> history;  // the last LM solve's trajectory (pba_solver_iterations)
  int red_slots = 0;
};

// One pyramid level's images, cameras and points (pba_pyramid.hip); level 0 lives in the engine's own fields.
struct LevelData {
  DevBuf<uint8_t> images;
  int width = 0, height = 0;
  DevBuf<float> intr;
  DevBuf<double> intr_d;
  DevBuf<double2> u_ref;
  DevBuf<float> host_int;
};

}  // namespace detail
}  // namespace pba

#include <atomic>
#include <memory>

struct pba_engine {
  pba_options opt{};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  int n_cams = 0, n_frames = 0, n_points = 0, n_blocks = 0, n_pairs = 0;
  int width = 0, height = 0, P = 0;
  bool have_images = false;
  std::vector<int> frame_cam_h, point_host_h, block_point_h, block_target_h, pair_of_h, pair_host_h, pair_target_h;
  std::vector<float> pattern_h;
  pba::detail::DevBuf<float> intr;
  pba::detail::DevBuf<double> intr_d;
  pba::detail::DevBuf<int> frame_cam;
  pba::detail::DevBuf<uint8_t> images;
  pba::detail::DevBuf<double2> u_ref;
  pba::detail::DevBuf<int> point_host_d;   // host keyframe per point
  pba::detail::DevBuf<float> host_int;
  pba::detail::DevBuf<int> block_point, block_pair;
  pba::detail::DevBuf<int2> block_pp;
  pba::detail::DevBuf<double2> u_obs;
  pba::detail::DevBuf<int> pair_host, pair_target;
  pba::detail::DevBuf<int4> block_rec;  // {point, host, target, cams} per block (fused-state prologue)
  pba::detail::DevBuf<pba::detail::PairRec> pairs;
  pba::detail::DevBuf<double> poses, rho;
  pba::detail::DevBuf<float> out, cost;
  pba::detail::DevBuf<float> res;    // contiguous residuals of the last residual-only evaluation (R per block)
  bool res_fresh = false;            // res holds the last evaluation's residuals (it was residual-only)
  pba::detail::DevBuf<uint8_t> valid;
  int record_format = PBA_RECORD_F32;
  int interp = PBA_INTERP_BILINEAR;  // pba_set_interpolator
  bool host_int_sampled = false;     // I_h,k sampled on the device (pba_set_points without intensities)
  bool opt_intr = false;             // pba_set_optimize_intrinsics: target intrinsics state + J_intr record tail
  pba::detail::DevBuf<float> intr_state;     // its projection constants (8 floats per camera)
  pba::detail::DevBuf<double> intr_state_d;  // and fp64 camera records (kCamD per camera)
  bool state_set = false;
  bool pairs_fresh = false;          // pairs hold T_th of the current poses (pba_set_state_device forms them)
  bool evaluated = false;
  bool timing = false;
  int last_grid = 0;                 // workgroups of the last evaluation launch (launch_mode)
  std::vector<hipEvent_t> ev_pool;   // start/stop pairs, reused
  int level = 0;                     // active pyramid level (its buffers are swapped into the fields above)
  std::vector<std::unique_ptr<pba::detail::LevelData>> pyr;  // [1, n_levels); [0] unused
  size_t ev_used = 0;
  // pba_get_records_async: one event per chunk of copied records, and how many chunks are known to have arrived
  std::vector<hipEvent_t> chunk_ev;
  hipEvent_t res_ev = nullptr;       // pba_get_residuals: the copies' completion (polled, not a blocking wait)
  int chunk_blocks = 0, n_chunks_async = 0;
  std::atomic<int> chunks_arrived{0};
  pba::detail::GnData gn;

  int R() const { return opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC ? P : 2; }
  // values per record: [r | J_host | J_target | J_rho] (14R), + J_intr (8R) with pba_set_optimize_intrinsics
  int rec_floats() const { return (opt_intr ? 22 : 14) * R(); }
};

namespace pba {
namespace detail {

inline int check_device(pba_engine* e) {
  PBA_HIP(hipSetDevice(e->opt.device));
  return PBA_OK;
}

// Kernel arguments describing the engine's current problem and state.
KernelArgs make_kernel_args(pba_engine* e, const PairRec* pairs, const double* rho);

// Pair kernel launch (relative poses of every (host, target) pair from an fp64 pose array).
void launch_pairs(pba_engine* e, const double* poses, PairRec* pairs);

// Residual-only evaluation writing only per-block costs/validity (state given by pairs/rho).
// wg_red (optional): each workgroup also writes its (Σ cost, Σ valid) there; *n_slots = the launch's workgroups.
// poses (optional): evaluate at these state poses with the fused-state prologue instead of the pair table.
// intr_t / intr_t_d (optional): the target projection's intrinsics (a candidate's free intrinsics).
int launch_cost_only(pba_engine* e, const PairRec* pairs, const double* rho, double* wg_red = nullptr,
                     int* n_slots = nullptr, const double* poses = nullptr, const float* intr_t = nullptr,
                     const double* intr_t_d = nullptr);

// Collectives of the multi-GPU loop (pba_comm.hip): Σ over the ranks in place, enqueued on stream.
int comm_allreduce(pba_comm* c, double* buf, long long count, hipStream_t stream);
int comm_rank(const pba_comm* c);
int comm_size(const pba_comm* c);

// Pyramid (pba_pyramid.hip): back to level 0 and drop the levels; I_h,k sampled from the active level's host images.
void reset_pyramid(pba_engine* e);
int sample_host_intensities(pba_engine* e, const double2* u_ref, float* out);

}  // namespace detail
}  // namespace pba
