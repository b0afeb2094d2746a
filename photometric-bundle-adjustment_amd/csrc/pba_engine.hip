// pba_engine.hip — HIP kernels + C ABI (include/pba.h) of the photometric BA residual/Jacobian engine.
//
// Replaces, for every residual block of a problem at once, the reference's per-block CPU evaluation:
//   ProgramEvaluator::Evaluate ParallelFor (program_evaluator.h:187-258) →
//   ResidualBlock::Evaluate (residual_block.cc:69-158) → AutoDiffCostFunction<Functor,…> →
//   BundleAdjustmentReprojectionCostFunctor (reprojection.h:83-112) / PhotometricError (photometric_error.h:139-182)
//
// Photometric evaluation is ONE launch (photometric_block_kernel): one lane per (block, pattern pixel), a wave =
// 64/LPB blocks.  Each block's lanes form its relative pose T_th = T_w_t⁻¹ T_w_h in fp64 from the state poses in
// the tile prologue (fused state, pba_internal.h:stage_tile) — or copy it from the pair table (pair_kernel /
// state_kernel: the geometric kernels and the Gauss-Newton path) — with u_ref and ρ into LDS; image taps are
// gathered from the target keyframe's tiled u8 image, the Jacobian chain stays in registers, per-block ‖r‖² and
// validity come from wave shuffles, and the workgroup's records leave as one contiguous slab.
#include <hip/hip_runtime.h>

#include <type_traits>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pba_internal.h"

using namespace pba;
using namespace pba::detail;

namespace pba {
namespace detail {
thread_local std::string g_last_error;
}  // namespace detail
}  // namespace pba

namespace {

// ------------------------------------------------------------------------------------------------
// Pair table: relative poses in fp64 (form_pair, pba_internal.h)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void make_pair(const double* __restrict__ poses, const int* __restrict__ pair_host,
                                          const int* __restrict__ pair_target, const int* __restrict__ frame_cam,
                                          const double* __restrict__ cams, PairRec* __restrict__ pairs, int i) {
  PairRec r;
  form_pair(poses, frame_cam, cams, pair_host[i], pair_target[i], r);
  pairs[i] = r;
}

__global__ void pair_kernel(const double* __restrict__ poses, const int* __restrict__ pair_host,
                            const int* __restrict__ pair_target, const int* __restrict__ frame_cam,
                            const double* __restrict__ cams, PairRec* __restrict__ pairs, int n_pairs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_pairs) make_pair(poses, pair_host, pair_target, frame_cam, cams, pairs, i);
}

// State upload fused with the pair kernel (one launch instead of two copies + pair_kernel): workgroups
// [0, pair_wgs) form the relative poses straight from the caller's pose array, the rest copy the poses and
// inverse distances into the engine's state buffers (16 B per lane, grid-stride).
__global__ void state_kernel(const double* __restrict__ src_poses, const double* __restrict__ src_rho,
                             double* __restrict__ poses, double* __restrict__ rho, int n_pose_d, int n_points,
                             const int* __restrict__ pair_host, const int* __restrict__ pair_target,
                             const int* __restrict__ frame_cam, const double* __restrict__ cams,
                             PairRec* __restrict__ pairs, int n_pairs, int pair_wgs) {
  if ((int)blockIdx.x < pair_wgs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_pairs) make_pair(src_poses, pair_host, pair_target, frame_cam, cams, pairs, i);
    return;
  }
  const long long stride = (long long)(gridDim.x - pair_wgs) * blockDim.x;
  const long long i0 = (long long)(blockIdx.x - pair_wgs) * blockDim.x + threadIdx.x;
  for (long long i = i0; i < n_pose_d; i += stride) poses[i] = src_poses[i];
  for (long long i = i0; i < n_points; i += stride) rho[i] = src_rho[i];
}

// ------------------------------------------------------------------------------------------------
// Image relayout: row-major u8 frames → 16×8 tiles with the edge-replicating apron (pba_device.h).  One lane per
// 16-texel tile row of the padded frame; texels beyond the padded frame are zero and never read.
// ------------------------------------------------------------------------------------------------
// Device → page-locked host copy by a kernel (the host buffer is mapped into the device's address space): 16-B
// stores over the bus when both ends are 16-B aligned, bytes otherwise.  Enqueued like any launch, so the host never
// waits inside the call — hipMemcpyAsync into the same buffers returned only when the data had arrived (C4 sample:
// 2.4 ms per Jacobian read-back spent inside the enqueue, tools/probe/c2_probe.py).
__global__ void host_copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, long long bytes) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const long long n16 = bytes >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (long long i = i0; i < n16; i += stride) d4[i] = s4[i];
    for (long long i = (n16 << 4) + i0; i < bytes; i += stride) dst[i] = src[i];
  } else {
    for (long long i = i0; i < bytes; i += stride) dst[i] = src[i];
  }
}

__global__ void tile_images_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int W, int H,
                                   int tiles_x, int tiles_y, long long n_rows) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows) return;
  // i enumerates (frame, tile, row-in-tile) in destination order → 16-B coalesced stores
  const int r = (int)(i & 7);
  const long long tile = i >> 3;
  const long long tiles_per_frame = (long long)tiles_x * tiles_y;
  const long long f = tile / tiles_per_frame;
  const int t = (int)(tile - f * tiles_per_frame);
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int yp = ty * kTileH + r, xp0 = tx * kTileW;
  const int y = min(max(yp - kImgPad, 0), H - 1);
  union { uint8_t b[16]; uint4 v; } row;
  const uint8_t* s = src + f * W * (long long)H + (long long)y * W;
  const bool yin = yp < H + 2 * kImgPad;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int xp = xp0 + j;
    row.b[j] = (yin && xp < W + 2 * kImgPad) ? s[min(max(xp - kImgPad, 0), W - 1)] : (uint8_t)0;
  }
  reinterpret_cast<uint4*>(dst)[i] = row.v;
}

// A record value in the engine's format.  fp16 saturates at ±65504 (the half range) instead of rounding to ±inf: at
// full resolution a strong edge's rotation Jacobian ∇I·∂π/∂p·[b]× reaches ~1e5 intensity units per radian (measured
// up to 9.0e4 on the C5-style problem), so those entries are clamped (pba.h, PBA_RECORD_F16).
template <class T>
__device__ __forceinline__ T rec_val(float v) { return (T)v; }
template <>
__device__ __forceinline__ _Float16 rec_val<_Float16>(float v) {
  // (fmed3 would map NaN to −65504: a NaN stays NaN)
  return (_Float16)(isnan(v) ? v : __builtin_amdgcn_fmed3f(v, -65504.0f, 65504.0f));
}

// Store a workgroup's contiguous record slab (LDS → global): 16-B non-temporal stores when the slab is 16-B
// aligned, 4-B or 2-B stores otherwise (odd patterns in fp16).
// wt (wave-uniform, KernelArgs::slab_wt): non-temporal write-through stores (`nt sc1`) — for launches of at most one
// wave of workgroups (a 1/8 shard of C4: 8.29 → 8.07-8.15 µs, nothing left dirty in L2 for the kernel's end), never for
// a full C4 launch (44.9 → 46.2 µs), DESIGN.md §3.
template <class T, int NTH = kBlockThreads>
__device__ __forceinline__ void store_slab(const unsigned char* src, unsigned char* dst, int bytes, int wt = 0) {
  constexpr int kBlockThreads = NTH;  // the workgroup's threads share the slab
  if ((((uintptr_t)dst | (unsigned)bytes) & 15) == 0) {
    // non-temporal 16-B stores (write-through sc1 stores measured 49 → 71 µs for this kernel; per-lane stores
    // straight from registers, without the LDS slab, 49 → 104 µs: DESIGN.md §3)
    const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
    f32x4* d4 = reinterpret_cast<f32x4*>(dst);
    if (wt) {
      for (int i = threadIdx.x; i < (bytes >> 4); i += kBlockThreads)
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(d4 + i), "v"(s4[i]) : "memory");
    } else {
      for (int i = threadIdx.x; i < (bytes >> 4); i += kBlockThreads) __builtin_nontemporal_store(s4[i], d4 + i);
    }
  } else if (sizeof(T) == 4 || (((uintptr_t)dst | (unsigned)bytes) & 3) == 0) {
    const float* s1 = reinterpret_cast<const float*>(src);
    float* d1 = reinterpret_cast<float*>(dst);
#pragma unroll 1
    for (int i = threadIdx.x; i < (bytes >> 2); i += kBlockThreads) __builtin_nontemporal_store(s1[i], d1 + i);
  } else {
    const _Float16* s1 = reinterpret_cast<const _Float16*>(src);
    _Float16* d1 = reinterpret_cast<_Float16*>(dst);
#pragma unroll 1
    for (int i = threadIdx.x; i < (bytes >> 1); i += kBlockThreads) d1[i] = s1[i];
  }
}

template <int PM, int LPB, int MODE, class T>  // PM = camera model + 4 · interpolator
__global__ __launch_bounds__(kBlockThreads) void photometric_block_kernel(const KernelArgs a) {
  constexpr int BPW = kBlockThreads / LPB;  // blocks per workgroup
  constexpr bool JAC = MODE == 1;
  constexpr int kStageBytes = JAC ? BPW * 14 * LPB * (int)sizeof(T) : 0;
  constexpr int kTileBytes = BPW * (int)sizeof(TileBlock);
  __shared__ __attribute__((aligned(16))) unsigned char lds[kStageBytes > kTileBytes ? kStageBytes : kTileBytes];
  TileBlock* s_tb = reinterpret_cast<TileBlock*>(lds);
  const int P = a.P;
  const int rec_f = 14 * P;
  const int blk0 = logical_tile() * BPW;
  const int lb = threadIdx.x / LPB;
  const int k = threadIdx.x % LPB;
  const int blk = blk0 + lb;
  const bool live = blk < a.n_blocks;  // a block's LPB lanes agree
  const bool act = live && k < P;
  T* out = reinterpret_cast<T*>(a.out);  // records in the engine's format (fp32, or fp16 for PBA_RECORD_F16)

  const float2 off = pattern_at<LPB>(a, k);
  adopt_state(a);
  int pt;
  if (LPB == 8 && a.poses) {  // fused state: the workgroup-cooperative prologue (BPW = 32)
    static_assert(kBlockThreads == 256, "stage_tile_wg: 4 waves, 32 blocks");
    pt = a.block_rec[live ? blk : a.n_blocks - 1].x;
    stage_tile_wg(a, s_tb, blk0);
  } else {
    pt = stage_tile<LPB>(a, s_tb, lb, k, blk, live);
  }
  const float Ih = act ? a.host_int[(long long)pt * P + k] : 0.0f;
  __syncthreads();
  const Row row = photometric_row<PM, JAC>(a, s_tb[lb], off, Ih);  // dead lanes evaluate a staged block, masked by act
  // per-block validity (ballot over the wave: the block's LPB lanes are an aligned bit field) and ‖r‖²
  const int ok = group_all<LPB>(act ? row.ok : 1);
  const float s = group_sum<LPB>(act ? row.r * row.r : 0.0f);
  const float bc = ok ? huber_cost(s, a.huber) : 0.0f;
  if (live && k == 0) {
    a.valid[blk] = (uint8_t)ok;
    a.cost[blk] = bc;
  }
  if (MODE == 2) {
    if (a.wg_red) {
      const bool one = live && k == 0;
      wg_reduce2(one ? (double)bc : 0.0, one && ok ? 1.0 : 0.0, a.wg_red + 2 * logical_tile());
    }
    return;
  }
  if (!JAC) {
    if (act) {
      out[(long long)blk * rec_f + k] = rec_val<T>(ok ? row.r : 0.0f);
      if (a.res_out) a.res_out[(long long)blk * P + k] = ok ? row.r : 0.0f;  // contiguous: one D2H copy for Ceres
    }
    return;
  }
  __syncthreads();  // every lane has read its tile block: the record stage may overwrite it
  T* stage = reinterpret_cast<T*>(lds);
  // stage the record row of pixel k: r | J_host row | J_target row | J_rho  (zeros for invalid blocks)
  if (act) {
    T* s_rec = stage + lb * rec_f;
    T* h = s_rec + P + 6 * k;
    T* t = s_rec + 7 * P + 6 * k;
    if (ok) {
      s_rec[k] = rec_val<T>(row.r);
      h[0] = rec_val<T>(row.hv.x); h[1] = rec_val<T>(row.hv.y); h[2] = rec_val<T>(row.hv.z);
      h[3] = rec_val<T>(row.hw.x); h[4] = rec_val<T>(row.hw.y); h[5] = rec_val<T>(row.hw.z);
      t[0] = rec_val<T>(row.tv.x); t[1] = rec_val<T>(row.tv.y); t[2] = rec_val<T>(row.tv.z);
      t[3] = rec_val<T>(row.tw.x); t[4] = rec_val<T>(row.tw.y); t[5] = rec_val<T>(row.tw.z);
      s_rec[13 * P + k] = rec_val<T>(row.jr);
    } else {
      s_rec[k] = (T)0.0f;
      for (int j = 0; j < 6; ++j) h[j] = t[j] = (T)0.0f;
      s_rec[13 * P + k] = (T)0.0f;
    }
  }
  __syncthreads();
  const int nblk = min(BPW, a.n_blocks - blk0);
  if (nblk <= 0) return;
  store_slab<T>(lds, reinterpret_cast<unsigned char*>(out + (long long)blk0 * rec_f), nblk * rec_f * (int)sizeof(T),
                a.slab_wt);
}

// Row px of a block's staged record (r | J_host row | J_target row | J_rho; T = float or _Float16), written by the lane
// that evaluated it when act.  Every lane of the wave calls it (the fp16 form's saturation test is a ballot).
template <class T>
__device__ __forceinline__ void stage_row(T* s_rec, int P, int px, const Row& row, bool act) {
  if constexpr (std::is_same<T, _Float16>::value) {
    // fp16 records: the 14 values in 7 packed round-to-nearest conversions (v_cvt_pk_f16_f32) instead of a
    // NaN-preserving clamp + conversion each; a value beyond the half range rounds to ±inf there, which rec_val
    // saturates to ±65504 — applied afterwards, only when some lane of the wave has one (a ballot)
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const float v[14] = {row.r, row.jr, row.hv.x, row.hv.y, row.hv.z, row.hw.x, row.hw.y, row.hw.z,
                         row.tv.x, row.tv.y, row.tv.z, row.tw.x, row.tw.y, row.tw.z};
    h2 c[7];
    // a value rounds to ±inf in half precision iff |v| ≥ 65520: one max over the 14 magnitudes (v_max3 with abs
    // modifiers; a NaN drops out of the max and stays NaN) instead of a class test per converted half
    float m = 0.0f;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      c[q] = __builtin_convertvector((f2){v[2 * q], v[2 * q + 1]}, h2);
      m = fmaxf(m, fmaxf(fabsf(v[2 * q]), fabsf(v[2 * q + 1])));
    }
    const bool big = m >= 65520.0f;
    if (__ballot(act && big) != 0) {
      auto sat = [](_Float16 h) -> _Float16 {
        return __builtin_isinf(h) ? (h > (_Float16)0 ? (_Float16)65504.0f : (_Float16)-65504.0f) : h;
      };
#pragma unroll
      for (int q = 0; q < 7; ++q) c[q] = (h2){sat(c[q].x), sat(c[q].y)};
    }
    if (act) {
      // the 6-value rows as 4-byte LDS writes where they are 4-byte aligned (LDS issue is what this kernel waits on:
      // SQ_WAIT_INST_LDS ≈ 0.26 of wave time): 3 per row for even P, 1 + 2 + 1 for odd P (the inner pairs re-packed)
      T* h = s_rec + P + 6 * px;
      T* t = s_rec + 7 * P + 6 * px;
      s_rec[px] = c[0].x;
      s_rec[13 * P + px] = c[0].y;
      if ((P & 1) == 0) {
        h2* h4 = reinterpret_cast<h2*>(h);
        h2* t4 = reinterpret_cast<h2*>(t);
        h4[0] = c[1]; h4[1] = c[2]; h4[2] = c[3];
        t4[0] = c[4]; t4[1] = c[5]; t4[2] = c[6];
      } else {
        h2* h4 = reinterpret_cast<h2*>(h + 1);
        h2* t4 = reinterpret_cast<h2*>(t + 1);
        h[0] = c[1].x; h4[0] = (h2){c[1].y, c[2].x}; h4[1] = (h2){c[2].y, c[3].x}; h[5] = c[3].y;
        t[0] = c[4].x; t4[0] = (h2){c[4].y, c[5].x}; t4[1] = (h2){c[5].y, c[6].x}; t[5] = c[6].y;
      }
    }
  } else if (act) {  // record row px: r | J_host row | J_target row | J_rho
    T* h = s_rec + P + 6 * px;
    T* t = s_rec + 7 * P + 6 * px;
    s_rec[px] = rec_val<T>(row.r);
    h[0] = rec_val<T>(row.hv.x); h[1] = rec_val<T>(row.hv.y); h[2] = rec_val<T>(row.hv.z);
    h[3] = rec_val<T>(row.hw.x); h[4] = rec_val<T>(row.hw.y); h[5] = rec_val<T>(row.hw.z);
    t[0] = rec_val<T>(row.tv.x); t[1] = rec_val<T>(row.tv.y); t[2] = rec_val<T>(row.tv.z);
    t[3] = rec_val<T>(row.tw.x); t[4] = rec_val<T>(row.tw.y); t[5] = rec_val<T>(row.tw.z);
    s_rec[13 * P + px] = rec_val<T>(row.jr);
  }
}

// Patterns of 9…32 pixels (the 21-px pattern of config C5): still 8 lanes per block, each lane evaluating pixels
// k, k+8, … (PPL of them), so a wave carries 8 blocks and the per-block prologue (pair record, point) is paid once
// per 8 blocks — one lane per pixel (32 lanes per block) ran the 21-px C4 shard at 181 µs per launch with a third
// of its lanes idle and the prologue amortised over 2 blocks per wave.  Rows go to the record stage as they are
// produced (stage and tile in separate LDS regions); an invalid block's record is zeroed once its validity is known
// (the same lanes rewrite their own rows: LDS operations of one wave stay in order).  256 threads per workgroup,
// 128 when the fp32 stage of 32 blocks would not fit the 64 KiB of static LDS.
__host__ __device__ constexpr int multi_stage_bytes(int bpw, int P, int tsize) { return (bpw * 14 * P * tsize + 15) & ~15; }

template <int PPL, class T>
constexpr int kMultiThreads = 32 * 14 * 8 * PPL * (int)sizeof(T) + 32 * (int)sizeof(TileBlock) > 60 * 1024 ? 128 : 256;

// CT: the camera-table form (fused state, ≤ kCamTab cameras, 256 threads): compact 192-B tile blocks plus one LDS
// CamRec per camera instead of 352-B tile blocks carrying both cameras (the 21-px fp16 launch: 30.1 → 25.6 KB of LDS
// per workgroup, 5 → 6 workgroups per CU, which its 78 VGPRs also allow).
// C1 (with CT, one camera): the rows take the camera constants from scalar loads of the engine's camera record instead
// of the LDS table (no per-row LDS reads of them, no VGPRs).
template <int PM, int MODE, class T, int PPL, bool CT = false, bool C1 = false>
__global__ __launch_bounds__((kMultiThreads<PPL, T>)) __attribute__((amdgpu_waves_per_eu(CT ? 6 : 1, 8)))
void photometric_block_kernel_multi(const KernelArgs a) {
  constexpr int LPB = 8, NTH = kMultiThreads<PPL, T>, BPW = NTH / LPB;
  constexpr bool JAC = MODE == 1;
  static_assert(!CT || NTH == 256, "camera table: the workgroup-cooperative prologue");
  using TB = typename std::conditional<CT, TileBlockC, TileBlock>::type;
  // dynamic LDS sized for the actual P (multi_stage_bytes): the 21-px fp16 stage is 18.4 KB instead of 21 KB for
  // 24 px, which lets a fifth workgroup onto the CU (LDS is what bounds this kernel's occupancy)
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ float2 s_pat[LPB * PPL];
  __shared__ CamRec s_cam[CT ? kCamTab : 1];
  const int P = a.P;
  T* stage = reinterpret_cast<T*>(lds);
  TB* s_tb = reinterpret_cast<TB*>(lds + (JAC ? multi_stage_bytes(BPW, P, (int)sizeof(T)) : 0));
  const int rec_f = 14 * P;
  const int blk0 = logical_tile() * BPW;
  const int lb = threadIdx.x / LPB;
  const int k = threadIdx.x % LPB;
  const int blk = blk0 + lb;
  const bool live = blk < a.n_blocks;  // a block's LPB lanes agree
  T* out = reinterpret_cast<T*>(a.out);

  if ((int)threadIdx.x < LPB * PPL) s_pat[threadIdx.x] = pattern_at<LPB * PPL>(a, threadIdx.x);
  adopt_state(a);
  int pt;
  if constexpr (CT) {
    pt = a.block_rec[live ? blk : a.n_blocks - 1].x;
    stage_tile_wg_ct(a, s_tb, s_cam, a.n_cams, blk0);
  } else if (NTH == 256 && a.poses) {  // fused state: the workgroup-cooperative prologue (BPW = 32)
    pt = a.block_rec[live ? blk : a.n_blocks - 1].x;
    stage_tile_wg(a, s_tb, blk0);
  } else {
    pt = stage_tile<LPB>(a, s_tb, lb, k, blk, live);
  }
  float Ih[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int px = k + LPB * j;
    Ih[j] = live && px < P ? a.host_int[(long long)pt * P + px] : 0.0f;
  }
  __syncthreads();
  T* s_rec = stage + lb * rec_f;
  int okl = 1;
  float s = 0.0f, rr[PPL];
  auto pixel = [&](int j, float ih) {
    const int px = k + LPB * j;
    const bool act = live && px < P;
    const Row row = photometric_row<PM, JAC, TB, C1>(a, s_tb[lb], s_pat[px < P ? px : 0], ih, s_cam);  // masked by act
    okl &= act ? row.ok : 1;
    s += act ? row.r * row.r : 0.0f;
    if constexpr (JAC) stage_row<T>(s_rec, P, px, row, act);
    return row.r;
  };
  if constexpr (JAC) {
    // one pixel at a time (no unrolling: an unrolled loop interleaves the PPL rows' evaluations and needed 122 VGPRs,
    // 4 waves per SIMD); the pixel's I_h,k selected from the registers by a compare chain
#pragma unroll 1
    for (int j = 0; j < PPL; ++j) {
      float ih = Ih[0];
#pragma unroll
      for (int q = 1; q < PPL; ++q) ih = j == q ? Ih[q] : ih;
      // the tile block (pair record, cameras, point: ~70 registers) is read from LDS again by every pixel instead of
      // being hoisted out of the loop and kept live across it
      asm volatile("" ::: "memory");
      pixel(j, ih);
    }
  } else {
#pragma unroll
    for (int j = 0; j < PPL; ++j) rr[j] = pixel(j, Ih[j]);
  }
  // per-block validity (ballot over the wave: the block's LPB lanes are an aligned bit field) and ‖r‖²
  const int ok = group_all<LPB>(okl);
  s = group_sum<LPB>(s);
  const float bc = ok ? huber_cost(s, a.huber) : 0.0f;
  if (live && k == 0) {
    a.valid[blk] = (uint8_t)ok;
    a.cost[blk] = bc;
  }
  if (MODE == 2) {
    if (a.wg_red) {
      const bool one = live && k == 0;
      wg_reduce2(one ? (double)bc : 0.0, one && ok ? 1.0 : 0.0, a.wg_red + 2 * logical_tile());
    }
    return;
  }
  if (!JAC) {
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int px = k + LPB * j;
      if (live && px < P) {
        out[(long long)blk * rec_f + px] = rec_val<T>(ok ? rr[j] : 0.0f);
        if (a.res_out) a.res_out[(long long)blk * P + px] = ok ? rr[j] : 0.0f;
      }
    }
    return;
  }
  if (live && !ok) {  // an invalid block leaves a zero record (Ceres' Evaluate returning false)
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int px = k + LPB * j;
      if (px >= P) continue;
      s_rec[px] = (T)0.0f;
      s_rec[13 * P + px] = (T)0.0f;
      for (int q = 0; q < 6; ++q) s_rec[P + 6 * px + q] = s_rec[7 * P + 6 * px + q] = (T)0.0f;
    }
  }
  __syncthreads();
  const int nblk = min(BPW, a.n_blocks - blk0);
  if (nblk <= 0) return;
  store_slab<T, NTH>(lds, reinterpret_cast<unsigned char*>(out + (long long)blk0 * rec_f), nblk * rec_f * (int)sizeof(T));
}

// ------------------------------------------------------------------------------------------------
// Geometric block kernel (reprojection.h:105-108): lane = block, record 28 floats = 7 float4 stores, or with the
// target-intrinsics Jacobian (INTR, pba_set_optimize_intrinsics) 44 floats = 11 float4 stores
// ------------------------------------------------------------------------------------------------
template <int MODEL, bool JAC, bool INTR>
__global__ __launch_bounds__(kBlockThreads) void geometric_block_kernel(const KernelArgs a) {
  constexpr int NR = INTR ? 44 : 28;
  const int blk_ = logical_tile() * kBlockThreads + threadIdx.x;
  const bool live = blk_ < a.n_blocks;
  if (!live && !a.wg_red) return;  // (with wg_red every thread reaches the workgroup reduction)
  const int blk = live ? blk_ : a.n_blocks - 1;
  const int pt = a.block_point[blk];
  const PairRec& pp = a.pairs[a.block_pair[blk]];
  // the host camera unprojects with the constant intrinsics (the functor's captured ref_intrinsics, reprojection.h:
  // 93-98), the target camera projects with the intrinsics parameter block (sIntr_c2)
  const double* khd = a.intr_d + kCamD * pp.host_cam;
  const double* ktd = a.intr_t_d + kCamD * pp.target_cam;
  const double2 ur = a.u_ref[pt];
  const double2 uo = a.u_obs[blk];
  const double rho = a.rho[pt];
  const double irho = rcp_nr(rho);
  // p = T_w_t⁻¹ · T_w_h · (b / ρ) in fp64
  const Vec3d b = unproject<MODEL>(khd + kCamHk, ur.x, ur.y);
  const Vec3d ph = {b.x * irho, b.y * irho, b.z * irho};
  const Vec3d Rp = mat_mul(pp.R, ph);
  const Vec3d p = {Rp.x + pp.t[0], Rp.y + pp.t[1], Rp.z + pp.t[2]};
  double u, v;
  const double iden = project<MODEL>(ktd, p, u, v);
  const float r0 = (float)(uo.x - u), r1 = (float)(uo.y - v);
  f32x4* rec = reinterpret_cast<f32x4*>(a.out + (long long)blk * NR);
  float J[NR];
  J[0] = r0;
  J[1] = r1;
  bool ok = isfinite(r0) && isfinite(r1);
  if (JAC) {
    const Vec3 pf = to_f(p), phf = to_f(ph);
    const Vec3 tf = {(float)pp.t[0], (float)pp.t[1], (float)pp.t[2]};
    const float irf = (float)irho;
    Vec3 du, dv;
    project_jac<MODEL>(a.intr_t + 8 * pp.target_cam, pf, (float)iden, du, dv);
    if (INTR) {  // ∂r/∂k = −∂π/∂k (2×8, row-major) after J_rho
      double ku[8], kv[8];
      project_intr_jac<MODEL>(ktd, p, iden, ku, kv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        J[28 + j] = (float)-ku[j];
        J[36 + j] = (float)-kv[j];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const Vec3 d = i == 0 ? du : dv;
      const Vec3 g = {-d.x, -d.y, -d.z};  // ∂r/∂p = −∂π/∂p
      const Vec3 gR = row_mul(g, pp.R);
      const Vec3 wh = cross(phf, gR);
      const Vec3 wt = cross(g, pf);
      float* jh = J + 2 + 6 * i;
      float* jt = J + 14 + 6 * i;
      jh[0] = gR.x; jh[1] = gR.y; jh[2] = gR.z; jh[3] = wh.x; jh[4] = wh.y; jh[5] = wh.z;
      jt[0] = -g.x; jt[1] = -g.y; jt[2] = -g.z; jt[3] = wt.x; jt[4] = wt.y; jt[5] = wt.z;
      J[26 + i] = dot(g, tf) * irf;  // = ∂π/∂p·R b/ρ² without the cancellation (∂π/∂p·p = 0), pba_internal.h
    }
#pragma unroll
    for (int i = 2; i < NR; ++i) ok = ok && isfinite(J[i]);
  }
  const float bc = ok ? huber_cost(r0 * r0 + r1 * r1, a.huber) : 0.0f;
  if (a.wg_red) {
    wg_reduce2(live ? (double)bc : 0.0, live && ok ? 1.0 : 0.0, a.wg_red + 2 * logical_tile());
    if (!live) return;
  }
  a.valid[blk] = (uint8_t)ok;
  a.cost[blk] = bc;
  if (!ok) {
#pragma unroll
    for (int i = 0; i < NR; ++i) J[i] = 0.0f;
  }
  if (JAC) {
#pragma unroll
    for (int i = 0; i < NR / 4; ++i)
      __builtin_nontemporal_store(f32x4{J[4 * i], J[4 * i + 1], J[4 * i + 2], J[4 * i + 3]}, rec + i);
  } else {
    reinterpret_cast<float2*>(rec)[0] = make_float2(J[0], J[1]);
    if (a.res_out) reinterpret_cast<float2*>(a.res_out)[blk] = make_float2(J[0], J[1]);
  }
}

template <int MODEL>
void launch_geometric(pba_engine* e, const KernelArgs& ka, int mode) {
  const int grid = (e->n_blocks + kBlockThreads - 1) / kBlockThreads;
  e->last_grid = grid;
  if (mode == 1 && e->opt_intr) geometric_block_kernel<MODEL, true, true><<<grid, kBlockThreads, 0, e->stream>>>(ka);
  else if (mode == 1) geometric_block_kernel<MODEL, true, false><<<grid, kBlockThreads, 0, e->stream>>>(ka);
  else if (e->opt_intr) geometric_block_kernel<MODEL, false, true><<<grid, kBlockThreads, 0, e->stream>>>(ka);
  else geometric_block_kernel<MODEL, false, false><<<grid, kBlockThreads, 0, e->stream>>>(ka);
}

// PM = camera model + 4 · interpolator (pba_device.h)
template <int PM>
void launch_photometric(pba_engine* e, KernelArgs ka, int mode) {
  const bool h = e->record_format == PBA_RECORD_F16;
  if (e->P <= 8) {
    const int grid = (int)(((long long)e->n_blocks * 8 + kBlockThreads - 1) / kBlockThreads);
    e->last_grid = grid;
    ka.slab_wt = grid <= kSlabWtGrid;  // one wave of workgroups: write-through record stores (store_slab)
    if (mode == 1 && h) photometric_block_kernel<PM, 8, 1, _Float16><<<grid, kBlockThreads, 0, e->stream>>>(ka);
    else if (mode == 1) photometric_block_kernel<PM, 8, 1, float><<<grid, kBlockThreads, 0, e->stream>>>(ka);
    else if (mode == 0 && h) photometric_block_kernel<PM, 8, 0, _Float16><<<grid, kBlockThreads, 0, e->stream>>>(ka);
    else if (mode == 0) photometric_block_kernel<PM, 8, 0, float><<<grid, kBlockThreads, 0, e->stream>>>(ka);
    else photometric_block_kernel<PM, 8, 2, float><<<grid, kBlockThreads, 0, e->stream>>>(ka);
    return;
  }
  // 9…32 pixels: 8 lanes per block, ⌈P/8⌉ pixels per lane
  // the camera-table form for record launches at a fused state with few cameras (the C5 configuration)
  const bool ct = mode == 1 && ka.poses != nullptr && ka.n_cams <= kCamTab;
#define PBA_LAUNCH_ONE(PPL, M, TT)                                                                      \
  {                                                                                                     \
    constexpr int nth = kMultiThreads<PPL, TT>;                                                         \
    const int grid = (int)(((long long)e->n_blocks * 8 + nth - 1) / nth);                              \
    e->last_grid = grid;                                                                                \
    const size_t stage = M == 1 ? multi_stage_bytes(nth / 8, e->P, (int)sizeof(TT)) : 0;               \
    if (M == 1 && nth == 256 && ct && ka.n_cams == 1) {                                                 \
      photometric_block_kernel_multi<PM, M, TT, PPL, (M == 1 && nth == 256), (M == 1 && nth == 256)>    \
          <<<grid, nth, stage + (size_t)(nth / 8) * sizeof(TileBlockC), e->stream>>>(ka);              \
    } else if (M == 1 && nth == 256 && ct) {                                                            \
      photometric_block_kernel_multi<PM, M, TT, PPL, (M == 1 && nth == 256)>                            \
          <<<grid, nth, stage + (size_t)(nth / 8) * sizeof(TileBlockC), e->stream>>>(ka);              \
    } else {                                                                                            \
      photometric_block_kernel_multi<PM, M, TT, PPL>                                                    \
          <<<grid, nth, stage + (size_t)(nth / 8) * sizeof(TileBlock), e->stream>>>(ka);               \
    }                                                                                                   \
  }
#define PBA_LAUNCH_PPL(PPL)                                        \
  if (mode == 1 && h) PBA_LAUNCH_ONE(PPL, 1, _Float16)             \
  else if (mode == 1) PBA_LAUNCH_ONE(PPL, 1, float)                \
  else if (mode == 0 && h) PBA_LAUNCH_ONE(PPL, 0, _Float16)        \
  else if (mode == 0) PBA_LAUNCH_ONE(PPL, 0, float)                \
  else PBA_LAUNCH_ONE(PPL, 2, float)
  const int ppl = (e->P + 7) / 8;
  if (ppl == 2) { PBA_LAUNCH_PPL(2) }
  else if (ppl == 3) { PBA_LAUNCH_PPL(3) }
  else { PBA_LAUNCH_PPL(4) }
#undef PBA_LAUNCH_PPL
#undef PBA_LAUNCH_ONE
}

void launch_mode(pba_engine* e, const KernelArgs& ka, int mode) {
  if (e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC) {
    switch (e->opt.camera_model) {
      case PBA_CAMERA_PINHOLE: launch_geometric<CAM_PINHOLE>(e, ka, mode); break;
      case PBA_CAMERA_DOUBLE_SPHERE: launch_geometric<CAM_DS>(e, ka, mode); break;
      case PBA_CAMERA_EUCM: launch_geometric<CAM_EUCM>(e, ka, mode); break;
      default: launch_geometric<CAM_KB4>(e, ka, mode); break;
    }
    return;
  }
  switch (e->opt.camera_model + 4 * e->interp) {
    case 0: launch_photometric<0>(e, ka, mode); break;
    case 1: launch_photometric<1>(e, ka, mode); break;
    case 2: launch_photometric<2>(e, ka, mode); break;
    case 3: launch_photometric<3>(e, ka, mode); break;
    case 4: launch_photometric<4>(e, ka, mode); break;
    case 5: launch_photometric<5>(e, ka, mode); break;
    case 6: launch_photometric<6>(e, ka, mode); break;
    default: launch_photometric<7>(e, ka, mode); break;
  }
}

}  // namespace

namespace pba {
namespace detail {

KernelArgs make_kernel_args(pba_engine* e, const PairRec* pairs, const double* rho) {
  KernelArgs ka{};
  ka.images = e->images.p;
  ka.width = e->width;
  ka.height = e->height;
  ka.tiles_x = tiles_x_of(e->width);
  ka.frame_stride = tiled_frame_bytes(e->width, e->height);
  ka.umax = e->width + 1.0;
  ka.vmax = e->height + 1.0;
  ka.intr = e->intr.p;
  ka.intr_d = e->intr_d.p;
  ka.intr_t = e->opt_intr ? e->intr_state.p : e->intr.p;
  ka.intr_t_d = e->opt_intr ? e->intr_state_d.p : e->intr_d.p;
  ka.block_point = e->block_point.p;
  ka.block_pair = e->block_pair.p;
  ka.block_pp = e->block_pp.p;
  ka.pairs = pairs;
  ka.block_rec = e->block_rec.p;
  ka.n_pose_d = 7 * e->n_frames;
  ka.n_points = e->n_points;
  ka.u_ref = e->u_ref.p;
  ka.host_int = e->host_int.p;
  ka.rho = rho;
  ka.u_obs = e->u_obs.p;
  ka.out = e->out.p;
  ka.cost = e->cost.p;
  ka.valid = e->valid.p;
  ka.n_blocks = e->n_blocks;
  ka.n_cams = e->n_cams;
  ka.P = e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC ? e->P : 2;
  ka.huber = e->opt.huber_width;
  for (size_t i = 0; i < e->pattern_h.size() && i < 2 * PBA_MAX_PATTERN; ++i) ka.pattern[i] = e->pattern_h[i];
  return ka;
}

void launch_pairs(pba_engine* e, const double* poses, PairRec* pairs) {
  pair_kernel<<<(e->n_pairs + 255) / 256, 256, 0, e->stream>>>(poses, e->pair_host.p, e->pair_target.p,
                                                               e->frame_cam.p, e->intr_d.p, pairs, e->n_pairs);
}

int launch_cost_only(pba_engine* e, const PairRec* pairs, const double* rho, double* wg_red, int* n_slots,
                     const double* poses, const float* intr_t, const double* intr_t_d) {
  KernelArgs ka = make_kernel_args(e, pairs, rho);
  ka.poses = poses;
  if (intr_t) ka.intr_t = intr_t;
  if (intr_t_d) ka.intr_t_d = intr_t_d;
  ka.wg_red = wg_red;
  launch_mode(e, ka, 2);
  if (n_slots) *n_slots = e->last_grid;
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

}  // namespace detail
}  // namespace pba

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
  if (o->camera_model < PBA_CAMERA_PINHOLE || o->camera_model > PBA_CAMERA_KB4)
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
  e->intr.release(); e->intr_d.release(); e->frame_cam.release(); e->images.release(); e->u_ref.release(); e->host_int.release(); e->point_host_d.release();
  e->block_point.release(); e->block_pair.release(); e->block_pp.release(); e->u_obs.release(); e->pair_host.release();
  e->pair_target.release(); e->block_rec.release(); e->pairs.release(); e->poses.release(); e->rho.release(); e->out.release();
  e->cost.release(); e->valid.release();
  for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->chunk_ev) (void)hipEventDestroy(ev);
  if (e->res_ev) (void)hipEventDestroy(e->res_ev);
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

// Camera tables from 8·n intrinsics: fp32 [fx fy cx cy p1..p4] (Jacobian chain) and the fp64 records (kCamD doubles
// each, pba_device.h) [fx fy cx cy p1..p4 | cx cy 1/fx 1/fy p1..p4], uploaded to f / d on the engine stream.
static int upload_cameras(pba_engine* e, int n_cams, const double* intrinsics, DevBuf<float>& f, DevBuf<double>& d) {
  std::vector<float> hf(8 * (size_t)n_cams);
  for (size_t i = 0; i < hf.size(); ++i) hf[i] = (float)intrinsics[i];
  for (int c = 0; c < n_cams; ++c)
    if (!(hf[8 * c] != 0.0f && hf[8 * c + 1] != 0.0f)) return fail(PBA_ERR_INVALID_ARGUMENT, "zero focal length");
  std::vector<double> hd((size_t)kCamD * n_cams, 0.0);
  for (int c = 0; c < n_cams; ++c) {
    const double* k = intrinsics + 8 * c;
    double* r = hd.data() + (size_t)kCamD * c;
    for (int j = 0; j < 8; ++j) r[j] = k[j];
    r[8] = k[2]; r[9] = k[3]; r[10] = 1.0 / k[0]; r[11] = 1.0 / k[1];
    for (int j = 4; j < 8; ++j) r[8 + j] = k[j];
  }
  PBA_HIP(f.resize(hf.size()));
  PBA_HIP(d.resize(hd.size()));
  PBA_HIP(hipMemcpyAsync(f.p, hf.data(), hf.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(d.p, hd.data(), hd.size() * sizeof(double), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

int pba_set_cameras(pba_engine* e, int32_t n_cams, const double* intrinsics) {
  if (!e || n_cams <= 0 || n_cams > 32767 || !intrinsics) return fail(PBA_ERR_INVALID_ARGUMENT, "bad camera arguments");
  if (int rc = check_device(e)) return rc;
  reset_pyramid(e);
  if (int rc = upload_cameras(e, n_cams, intrinsics, e->intr, e->intr_d)) return rc;
  e->n_cams = n_cams;
  if (e->opt_intr) return upload_cameras(e, n_cams, intrinsics, e->intr_state, e->intr_state_d);
  return PBA_OK;
}

int pba_set_optimize_intrinsics(pba_engine* e, int32_t enable) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (enable && e->opt.residual_kind != PBA_RESIDUAL_GEOMETRIC)
    return fail(PBA_ERR_INVALID_ARGUMENT, "intrinsics optimisation is geometric only");
  if (enable && e->n_cams <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_cameras first");
  if (int rc = check_device(e)) return rc;
  const bool on = enable != 0;
  if (on && !e->opt_intr) {  // the state starts at the cameras' intrinsics
    std::vector<double> k((size_t)kCamD * e->n_cams), k8(8 * (size_t)e->n_cams);
    PBA_HIP(hipMemcpy(k.data(), e->intr_d.p, sizeof(double) * k.size(), hipMemcpyDeviceToHost));
    for (int c = 0; c < e->n_cams; ++c)
      for (int j = 0; j < 8; ++j) k8[8 * c + j] = k[(size_t)kCamD * c + j];
    if (int rc = upload_cameras(e, e->n_cams, k8.data(), e->intr_state, e->intr_state_d)) return rc;
  }
  e->opt_intr = on;
  e->evaluated = false;
  e->gn.prepared = false;  // the reduced camera system gains / loses its intrinsics border
  if (e->n_blocks > 0) PBA_HIP(e->out.resize((size_t)e->n_blocks * e->rec_floats()));
  return PBA_OK;
}

int pba_get_intrinsics(pba_engine* e, double* intrinsics) {
  if (!e || !intrinsics) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  if (e->n_cams <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_cameras first");
  if (int rc = check_device(e)) return rc;
  std::vector<double> k((size_t)kCamD * e->n_cams);
  PBA_HIP(hipMemcpyAsync(k.data(), e->opt_intr ? e->intr_state_d.p : e->intr_d.p, sizeof(double) * k.size(),
                         hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  for (int c = 0; c < e->n_cams; ++c)
    for (int j = 0; j < 8; ++j) intrinsics[8 * c + j] = k[(size_t)kCamD * c + j];
  return PBA_OK;
}

int pba_set_intrinsics_state(pba_engine* e, const double* intrinsics) {
  if (!e || !intrinsics) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  if (!e->opt_intr) return fail(PBA_ERR_NOT_READY, "pba_set_optimize_intrinsics first");
  if (int rc = check_device(e)) return rc;
  return upload_cameras(e, e->n_cams, intrinsics, e->intr_state, e->intr_state_d);
}

// Per-block {point, host, target, host_cam << 16 | target_cam} for the fused-state prologue (pba_internal.h
// stage_tile); rebuilt whenever blocks or frame cameras change.  Blocks that no longer fit the frames/points
// are dropped (pba_set_blocks again).
static int upload_block_records(pba_engine* e) {
  const size_t nb = e->block_point_h.size();
  if (nb == 0 || e->n_blocks <= 0) return PBA_OK;
  std::vector<int4> rec(nb);
  const int nf = (int)e->frame_cam_h.size(), np = (int)e->point_host_h.size();
  for (size_t b = 0; b < nb; ++b) {
    const int p = e->block_point_h[b], t = e->block_target_h[b];
    const int h = p < np ? e->point_host_h[p] : nf;
    if (h >= nf || t >= nf) {
      e->n_blocks = 0;
      e->block_point_h.clear();
      e->block_target_h.clear();
      return PBA_OK;
    }
    rec[b] = make_int4(p, h, t, (e->frame_cam_h[h] << 16) | e->frame_cam_h[t]);
  }
  PBA_HIP(e->block_rec.upload(rec, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
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
  reset_pyramid(e);
  PBA_HIP(e->frame_cam.resize(n_frames));
  PBA_HIP(hipMemcpyAsync(e->frame_cam.p, frame_cam, n_frames * sizeof(int), hipMemcpyHostToDevice, e->stream));
  if (images) {
    // frames arrive row-major (the reference's cv::Mat / pangolin image rows) and are re-tiled once on the
    // device; host input is staged through a transient device buffer.
    const size_t bytes = (size_t)n_frames * width * height;
    const int tx = tiles_x_of(width), ty = (height + 2 * kImgPad + kTileH - 1) / kTileH;
    PBA_HIP(e->images.resize((size_t)n_frames * tiled_frame_bytes(width, height)));
    const uint8_t* src = images;
    DevBuf<uint8_t> staging;
    if (kind == hipMemcpyHostToDevice) {
      PBA_HIP(staging.resize(bytes));
      PBA_HIP(hipMemcpyAsync(staging.p, images, bytes, kind, e->stream));
      src = staging.p;
    }
    const long long n_rows = (long long)n_frames * tx * ty * kTileH;
    tile_images_kernel<<<(unsigned)((n_rows + 255) / 256), 256, 0, e->stream>>>(src, e->images.p, width, height,
                                                                               tx, ty, n_rows);
    PBA_HIP(hipGetLastError());
    PBA_HIP(hipStreamSynchronize(e->stream));
    staging.release();
    e->have_images = true;
  }
  PBA_HIP(hipStreamSynchronize(e->stream));
  e->frame_cam_h.assign(frame_cam, frame_cam + n_frames);
  e->pairs_fresh = false;
  e->gn.prepared = false;  // the GN structure (frame count, the pairs' camera records) is re-analysed on next use
  e->n_frames = n_frames;
  e->width = width;
  e->height = height;
  return upload_block_records(e);
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
  reset_pyramid(e);
  e->pattern_h.assign(offsets, offsets + 2 * P);
  e->P = P;
  e->evaluated = false;  // the records and contiguous residuals of the last evaluation were sized for the old P
  e->res_fresh = false;
  return PBA_OK;
}

int pba_set_points(pba_engine* e, int32_t n_points, const int32_t* host_frame, const double* u_ref,
                   const float* host_intensity) {
  if (!e || n_points <= 0 || !host_frame || !u_ref) return fail(PBA_ERR_INVALID_ARGUMENT, "bad point arguments");
  if (e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_frames first");
  const bool photometric = e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC;
  if (photometric && e->P <= 0) return fail(PBA_ERR_NOT_READY, "photometric points need pba_set_pattern first");
  if (photometric && !host_intensity && !e->have_images)
    return fail(PBA_ERR_NOT_READY, "sampling host intensities needs the frames' images");
  for (int i = 0; i < n_points; ++i)
    if (host_frame[i] < 0 || host_frame[i] >= e->n_frames) return fail(PBA_ERR_INVALID_ARGUMENT, "host frame out of range");
  if (int rc = check_device(e)) return rc;
  reset_pyramid(e);
  PBA_HIP(e->u_ref.resize(n_points));
  PBA_HIP(hipMemcpyAsync(e->u_ref.p, u_ref, n_points * sizeof(double2), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(e->point_host_d.resize(n_points));
  PBA_HIP(hipMemcpyAsync(e->point_host_d.p, host_frame, n_points * sizeof(int), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(e->rho.resize(n_points));
  e->n_points = n_points;
  if (photometric) {
    PBA_HIP(e->host_int.resize((size_t)n_points * e->P));
    if (host_intensity) {
      PBA_HIP(hipMemcpyAsync(e->host_int.p, host_intensity, (size_t)n_points * e->P * sizeof(float),
                             hipMemcpyHostToDevice, e->stream));
    } else if (int rc = sample_host_intensities(e, e->u_ref.p, e->host_int.p)) {  // I_h,k from the host image
      return rc;
    }
    e->host_int_sampled = host_intensity == nullptr;
  }
  PBA_HIP(hipStreamSynchronize(e->stream));
  e->point_host_h.assign(host_frame, host_frame + n_points);
  e->state_set = false;
  return PBA_OK;
}

int pba_set_blocks(pba_engine* e, int32_t n_blocks, const int32_t* block_point, const int32_t* block_target,
                   const double* u_obs) {
  if (!e || n_blocks <= 0 || !block_point || !block_target) return fail(PBA_ERR_INVALID_ARGUMENT, "bad block arguments");
  if (e->n_points <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_points first");
  const bool geometric = e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC;
  if (geometric && !u_obs) return fail(PBA_ERR_INVALID_ARGUMENT, "geometric blocks need u_obs");
  const long long rec = e->rec_floats();
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
  PBA_HIP(e->pairs.resize((size_t)np));
  PBA_HIP(hipMemcpyAsync(e->block_point.p, block_point, n_blocks * sizeof(int), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->block_pair.p, pair_of.data(), n_blocks * sizeof(int), hipMemcpyHostToDevice, e->stream));
  std::vector<int2> pp(n_blocks);
  for (int b = 0; b < n_blocks; ++b) pp[b] = make_int2(block_point[b], pair_of[b]);
  PBA_HIP(e->block_pp.upload(pp, e->stream));
  PBA_HIP(hipMemcpyAsync(e->pair_host.p, ph.data(), np * sizeof(int), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->pair_target.p, pt.data(), np * sizeof(int), hipMemcpyHostToDevice, e->stream));
  if (geometric) {
    PBA_HIP(e->u_obs.resize(n_blocks));
    PBA_HIP(hipMemcpyAsync(e->u_obs.p, u_obs, n_blocks * sizeof(double2), hipMemcpyHostToDevice, e->stream));
  }
  PBA_HIP(e->out.resize((size_t)n_blocks * rec));
  PBA_HIP(e->cost.resize(n_blocks));
  PBA_HIP(e->valid.resize(n_blocks));
  PBA_HIP(hipStreamSynchronize(e->stream));
  e->n_blocks = n_blocks;
  e->n_pairs = np;
  e->evaluated = false;
  e->res_fresh = false;
  e->chunk_blocks = 0;
  e->n_chunks_async = 0;
  e->chunks_arrived.store(0);
  e->pairs_fresh = false;
  e->block_point_h.assign(block_point, block_point + n_blocks);
  e->block_target_h.assign(block_target, block_target + n_blocks);
  e->pair_of_h = std::move(pair_of);
  e->pair_host_h = std::move(ph);
  e->pair_target_h = std::move(pt);
  e->gn.prepared = false;
  return upload_block_records(e);
}

int pba_set_state(pba_engine* e, const double* poses, const double* inv_dist) {
  if (!e || !poses || !inv_dist) return fail(PBA_ERR_INVALID_ARGUMENT, "null state");
  if (e->n_points <= 0 || e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "problem not set");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(e->poses.resize(7 * (size_t)e->n_frames));
  PBA_HIP(hipMemcpyAsync(e->poses.p, poses, 7 * (size_t)e->n_frames * sizeof(double), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipMemcpyAsync(e->rho.p, inv_dist, (size_t)e->n_points * sizeof(double), hipMemcpyHostToDevice, e->stream));
  e->state_set = true;
  e->pairs_fresh = false;
  return PBA_OK;
}

int pba_set_state_device(pba_engine* e, const double* d_poses, const double* d_inv_dist) {
  if (!e || !d_poses || !d_inv_dist) return fail(PBA_ERR_INVALID_ARGUMENT, "null state");
  if (e->n_points <= 0 || e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "problem not set");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(e->poses.resize(7 * (size_t)e->n_frames));
  const int n_pose_d = 7 * e->n_frames;
  // the photometric evaluation forms its pairs itself (fused state); the table serves the geometric kernels
  const bool table = e->n_blocks > 0 && e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC;
  const int pair_wgs = table ? (e->n_pairs + 255) / 256 : 0;
  const int copy_wgs = std::min(1024, (std::max(n_pose_d, e->n_points) + 255) / 256);
  state_kernel<<<pair_wgs + copy_wgs, 256, 0, e->stream>>>(d_poses, d_inv_dist, e->poses.p, e->rho.p, n_pose_d,
                                                           e->n_points, e->pair_host.p, e->pair_target.p,
                                                           e->frame_cam.p, e->intr_d.p, e->pairs.p, e->n_pairs,
                                                           pair_wgs);
  PBA_HIP(hipGetLastError());
  e->state_set = true;
  e->pairs_fresh = table;
  return PBA_OK;
}

namespace {

// One evaluation launch at state (poses, rho); with `adopt`, the same launch copies that state into the engine's
// buffers (it then is the engine's state, as after pba_set_state_device).
int evaluate_at(pba_engine* e, const double* poses, const double* rho, bool adopt, bool jac) {
  const bool photometric = e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC;
  if (photometric && (!e->have_images || e->P <= 0)) return fail(PBA_ERR_NOT_READY, "images/pattern missing");
  if (int rc = check_device(e)) return rc;
  KernelArgs ka;
  if (photometric) {
    // every photometric launch runs 8 lanes per block (photometric_block_kernel / _multi, launch_blocks)
    const long long lanes = (long long)e->n_blocks * 8;
    if (adopt && lanes < std::max<long long>(7LL * e->n_frames, e->n_points)) {
      if (int rc = pba_set_state_device(e, poses, rho)) return rc;  // more state than lanes: copy first
      poses = e->poses.p;
      rho = e->rho.p;
      adopt = false;
    }
    ka = make_kernel_args(e, nullptr, rho);
    ka.poses = poses;
    if (adopt) {
      PBA_HIP(e->poses.resize(7 * (size_t)e->n_frames));
      ka.adopt_poses = e->poses.p;
      ka.adopt_rho = e->rho.p;
      e->state_set = true;
      e->pairs_fresh = false;
    }
  } else {
    if (adopt) {
      if (int rc = pba_set_state_device(e, poses, rho)) return rc;
    } else if (!e->pairs_fresh) {
      launch_pairs(e, e->poses.p, e->pairs.p);
    }
    e->pairs_fresh = true;
    ka = make_kernel_args(e, e->pairs.p, e->rho.p);
  }
  hipEvent_t ev_stop = nullptr;
  if (e->timing) {
    while (e->ev_pool.size() < e->ev_used + 2) {
      hipEvent_t ev;
      // timing-only events: no system-scope fence (no L2 writeback of the records inside the bracket)
      PBA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableSystemFence));
      e->ev_pool.push_back(ev);
    }
    PBA_HIP(hipEventRecord(e->ev_pool[e->ev_used], e->stream));
    ev_stop = e->ev_pool[e->ev_used + 1];
    e->ev_used += 2;
  }
  if (!jac) {
    PBA_HIP(e->res.resize((size_t)e->n_blocks * e->R()));
    ka.res_out = e->res.p;
  }
  launch_mode(e, ka, jac ? 1 : 0);
  PBA_HIP(hipGetLastError());
  if (ev_stop) PBA_HIP(hipEventRecord(ev_stop, e->stream));
  e->evaluated = true;
  e->res_fresh = !jac;
  // a new evaluation invalidates an earlier asynchronous read-back (pba_wait_records then fails instead of returning)
  e->chunk_blocks = 0;
  e->n_chunks_async = 0;
  e->chunks_arrived.store(0);
  return PBA_OK;
}

}  // namespace

int pba_evaluate(pba_engine* e, int32_t want_jacobians) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (e->n_blocks <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_blocks first");
  if (!e->state_set) return fail(PBA_ERR_NOT_READY, "pba_set_state first");
  return evaluate_at(e, e->poses.p, e->rho.p, false, want_jacobians != 0);
}

int pba_evaluate_state_device(pba_engine* e, const double* d_poses, const double* d_inv_dist, int32_t want_jacobians) {
  if (!e || !d_poses || !d_inv_dist) return fail(PBA_ERR_INVALID_ARGUMENT, "null state");
  if (e->n_blocks <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_blocks first");
  return evaluate_at(e, d_poses, d_inv_dist, true, want_jacobians != 0);
}

int pba_evaluate_states_device(pba_engine* e, int32_t n, const double* const* d_poses, const double* const* d_inv_dist,
                               int32_t want_jacobians) {
  if (!e || n < 0 || (n > 0 && (!d_poses || !d_inv_dist))) return fail(PBA_ERR_INVALID_ARGUMENT, "null states");
  if (e->n_blocks <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_blocks first");
  for (int i = 0; i < n; ++i) {
    if (!d_poses[i] || !d_inv_dist[i]) return fail(PBA_ERR_INVALID_ARGUMENT, "null state");
    if (int rc = evaluate_at(e, d_poses[i], d_inv_dist[i], true, want_jacobians != 0)) return rc;
  }
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

int pba_record_floats(const pba_engine* e) { return e ? e->rec_floats() : 0; }

int pba_set_record_format(pba_engine* e, int32_t format) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (format != PBA_RECORD_F32 && format != PBA_RECORD_F16) return fail(PBA_ERR_INVALID_ARGUMENT, "unknown record format");
  if (format == PBA_RECORD_F16 && e->opt.residual_kind != PBA_RESIDUAL_PHOTOMETRIC)
    return fail(PBA_ERR_INVALID_ARGUMENT, "fp16 records are photometric only");
  e->record_format = format;
  e->evaluated = false;
  e->res_fresh = false;
  return PBA_OK;
}

int pba_record_format(const pba_engine* e) { return e ? e->record_format : PBA_RECORD_F32; }
int pba_residuals_per_block(const pba_engine* e) { return e ? e->R() : 0; }
int pba_num_blocks(const pba_engine* e) { return e ? e->n_blocks : 0; }
int pba_num_points(const pba_engine* e) { return e ? e->n_points : 0; }
int pba_num_frames(const pba_engine* e) { return e ? e->n_frames : 0; }

int pba_get_records(pba_engine* e, float* records, uint8_t* valid) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (!e->evaluated) return fail(PBA_ERR_NOT_READY, "pba_evaluate first");
  if (int rc = check_device(e)) return rc;
  const size_t n = (size_t)e->n_blocks * e->rec_floats();
  std::vector<_Float16> half;
  if (records && e->record_format == PBA_RECORD_F16) {
    half.resize(n);
    PBA_HIP(hipMemcpyAsync(half.data(), e->out.p, n * sizeof(_Float16), hipMemcpyDeviceToHost, e->stream));
  } else if (records) {
    PBA_HIP(hipMemcpyAsync(records, e->out.p, n * sizeof(float), hipMemcpyDeviceToHost, e->stream));
  }
  if (valid) PBA_HIP(hipMemcpyAsync(valid, e->valid.p, e->n_blocks, hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  for (size_t i = 0; i < half.size(); ++i) records[i] = (float)half[i];
  return PBA_OK;
}

// Wait for an event by polling it (its completion signal lives in host memory) before falling back to a blocking
// wait: the read-backs of the Ceres adapter sit inside Ceres' evaluation timer, and a blocking wait's wake-up came late
// when the process's cgroup CPU quota was saturated by Ceres' own threads (C2 residual-only evaluations measured
// 0.7-1.8 ms box to box for the same work).  The poll is bounded in time (kEventSpinUs; a C2 read-back chunk arrives
// within ~0.1 ms), so a long wait — or several of Ceres' threads waiting at once — blocks instead of spinning on the
// quota Ceres' own threads need.
constexpr double kEventSpinUs = 200.0;
static hipError_t wait_event(hipEvent_t ev) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0;; ++i) {
    const hipError_t q = hipEventQuery(ev);
    if (q != hipErrorNotReady) return q;
    __builtin_ia32_pause();
    if ((i & 63u) == 63u &&
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kEventSpinUs)
      break;
  }
  return hipEventSynchronize(ev);
}

// Enqueue a device → host copy: by host_copy_kernel when the destination is page-locked memory mapped for the device
// (pba_host_alloc), else hipMemcpyAsync.
// The device address of a page-locked host buffer (the base of its allocation: an interior pointer is not found), or
// nullptr for other memory.
static void* mapped_device_ptr(void* host) {
  void* dd = nullptr;
  if (hipHostGetDevicePointer(&dd, host, 0) != hipSuccess) {
    (void)hipGetLastError();  // (not a mapped host allocation: clear the query's error)
    return nullptr;
  }
  return dd;
}

// dd: dst's device address (mapped_device_ptr of its allocation, plus the offset), or nullptr.
static int enqueue_to_host(pba_engine* e, void* dst, void* dd, const void* src, size_t bytes) {
  if (!bytes) return PBA_OK;
  if (dd) {
    const long long n16 = (long long)((bytes + 15) >> 4);
    const int grid = (int)std::min<long long>(1024, std::max<long long>(1, (n16 + 255) / 256));
    host_copy_kernel<<<grid, 256, 0, e->stream>>>(static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dd),
                                                  (long long)bytes);
    PBA_HIP(hipGetLastError());
    return PBA_OK;
  }
  PBA_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream));
  return PBA_OK;
}

// Chunked asynchronous read-back for the Ceres adapter: the copies go out on the engine stream behind the evaluation,
// an event after each chunk; a caller waiting for one block only waits for its chunk, so Ceres' per-block work
// (CostFunction::Evaluate, the Jacobian writer) overlaps the PCIe transfer of the later chunks.
int pba_get_records_async(pba_engine* e, float* records, uint8_t* valid, int32_t chunk_blocks) {
  if (!e || !records || !valid || chunk_blocks <= 0) return fail(PBA_ERR_INVALID_ARGUMENT, "bad async read-back arguments");
  if (!e->evaluated) return fail(PBA_ERR_NOT_READY, "pba_evaluate first");
  if (e->record_format != PBA_RECORD_F32) return fail(PBA_ERR_INVALID_ARGUMENT, "asynchronous read-back: fp32 records only");
  if (int rc = check_device(e)) return rc;
  const long long nb = e->n_blocks, rf = e->rec_floats();
  const int nc = (int)((nb + chunk_blocks - 1) / chunk_blocks);
  while ((int)e->chunk_ev.size() < nc) {
    hipEvent_t ev;
    PBA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    e->chunk_ev.push_back(ev);
  }
  e->chunk_blocks = chunk_blocks;
  e->n_chunks_async = nc;
  e->chunks_arrived.store(0);
  // the validity flags of every block in one copy ahead of the record chunks (a copy per chunk of chunk_blocks bytes was
  // small enough for the runtime to complete it on the host, which made every chunk's enqueue wait for the transfers
  // before it: the whole read-back then ran inside this call, 2.5 ms of the C4 sample's evaluation)
  float* rd = static_cast<float*>(mapped_device_ptr(records));
  if (int rc = enqueue_to_host(e, valid, mapped_device_ptr(valid), e->valid.p, (size_t)nb)) return rc;
  for (int c = 0; c < nc; ++c) {
    const long long b0 = (long long)c * chunk_blocks, n = std::min<long long>(chunk_blocks, nb - b0);
    if (int rc = enqueue_to_host(e, records + b0 * rf, rd ? rd + b0 * rf : nullptr, e->out.p + b0 * rf,
                                 sizeof(float) * (size_t)(n * rf)))
      return rc;
    PBA_HIP(hipEventRecord(e->chunk_ev[c], e->stream));
  }
  return PBA_OK;
}

int pba_wait_records(pba_engine* e, int32_t block) {
  if (!e || block < 0 || block >= e->n_blocks) return fail(PBA_ERR_INVALID_ARGUMENT, "bad wait arguments");
  // no read-back in flight for the current evaluation (pba_evaluate / pba_set_blocks reset it), or one that does not
  // cover this block: fail rather than report stale records as arrived
  if (e->chunk_blocks <= 0) return fail(PBA_ERR_NOT_READY, "pba_get_records_async first");
  const int c = block / e->chunk_blocks;
  if (c >= e->n_chunks_async || c >= (int)e->chunk_ev.size()) return fail(PBA_ERR_NOT_READY, "block not in the read-back");
  if (c < e->chunks_arrived.load(std::memory_order_acquire)) return PBA_OK;
  PBA_HIP(wait_event(e->chunk_ev[c]));  // chunks arrive in stream order: every chunk ≤ c is in
  int seen = e->chunks_arrived.load(std::memory_order_relaxed);
  while (seen < c + 1 && !e->chunks_arrived.compare_exchange_weak(seen, c + 1, std::memory_order_release)) {
  }
  return PBA_OK;
}

int pba_get_residuals(pba_engine* e, float* residuals, uint8_t* valid) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (!e->evaluated) return fail(PBA_ERR_NOT_READY, "pba_evaluate first");
  if (int rc = check_device(e)) return rc;
  const size_t R = (size_t)e->R(), nb = (size_t)e->n_blocks, RF = (size_t)e->rec_floats();
  std::vector<_Float16> half;
  if (residuals && nb && e->res_fresh && e->res.n >= nb * R) {
    // a residual-only evaluation also wrote its residuals contiguously: one plain device-to-host copy
    if (int rc = enqueue_to_host(e, residuals, mapped_device_ptr(residuals), e->res.p, nb * R * sizeof(float))) return rc;
  } else if (residuals && nb) {
    // the first R values of every 14R-value record: one pitched device-to-host copy
    if (e->record_format == PBA_RECORD_F16) {
      half.resize(nb * R);
      PBA_HIP(hipMemcpy2DAsync(half.data(), R * sizeof(_Float16), e->out.p, RF * sizeof(_Float16),
                               R * sizeof(_Float16), nb, hipMemcpyDeviceToHost, e->stream));
    } else {
      PBA_HIP(hipMemcpy2DAsync(residuals, R * sizeof(float), e->out.p, RF * sizeof(float), R * sizeof(float), nb,
                               hipMemcpyDeviceToHost, e->stream));
    }
  }
  if (valid)
    if (int rc = enqueue_to_host(e, valid, mapped_device_ptr(valid), e->valid.p, nb)) return rc;
  if (!e->res_ev) PBA_HIP(hipEventCreateWithFlags(&e->res_ev, hipEventDisableTiming));
  PBA_HIP(hipEventRecord(e->res_ev, e->stream));
  PBA_HIP(wait_event(e->res_ev));
  for (size_t i = 0; i < half.size(); ++i) residuals[i] = (float)half[i];
  return PBA_OK;
}

int pba_host_alloc(size_t bytes, void** ptr) {
  if (!ptr) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  *ptr = nullptr;
  // mapped into the device's address space: the read-backs into it are copy kernels (enqueue_to_host), not
  // hipMemcpyAsync, which returned only once a device-to-host copy had arrived
  PBA_HIP(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocPortable));
  // touch every page from the device now: the first device access to fresh page-locked memory maps it into the GPU's
  // page tables (tools/micro/d2h_enqueue: 18.5 ms for 45 MB, against 0.9 ms per later 45-MB read-back) — setup work that
  // otherwise lands inside the first evaluation Ceres times
  void* dd = nullptr;
  if (bytes && hipHostGetDevicePointer(&dd, *ptr, 0) == hipSuccess && dd) {
    PBA_HIP(hipMemsetAsync(dd, 0, bytes, nullptr));
    PBA_HIP(hipStreamSynchronize(nullptr));
  }
  (void)hipGetLastError();
  return PBA_OK;
}

int pba_host_free(void* ptr) {
  if (ptr) PBA_HIP(hipHostFree(ptr));
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
