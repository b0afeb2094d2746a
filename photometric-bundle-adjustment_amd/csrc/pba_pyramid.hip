// pba_pyramid.hip — image pyramid and coarse-to-fine photometric BA (BASELINE.json config C5:
// 3-level pyramid, 21-pixel pattern).  The reference's own photometric code is on the absent pba2 branch
// (README.md:1-2), so the pyramid convention is DSO's (the photometric BA this repository's north star describes):
//   level l+1 pixel (x, y) = round(mean of level-l pixels (2x..2x+1, 2y..2y+1)),   W_{l+1} = ⌊W_l / 2⌋
//   camera at level l:  fx_l = fx / 2^l,  fy_l = fy / 2^l,  c_l = (c + 0.5) / 2^l − 0.5   (pixel centres on integers;
//                       distortion parameters unchanged)
//   u_ref_l = (u_ref + 0.5) / 2^l − 0.5, the same pattern offsets (in level-l pixels) at every level,
//   I_h,k at level l = bilinear sample of the host's level-l image at u_ref_l + offset_k.
// Level 0 keeps the caller's data.  pba_set_level swaps the active level's buffers into the engine, so every
// evaluation / Gauss-Newton entry point runs unchanged on the selected level.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <vector>

#include "pba_internal.h"

using namespace pba;
using namespace pba::detail;

namespace {

// One lane per byte of the level-(l+1) tiled frames, apron included (edge replicated); pad texels zero.
__global__ void downsample_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int Ws, int Hs, int W,
                                  int H, long long frame_in, long long frame_out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long f = i / frame_out;
  const int o = (int)(i - f * frame_out);
  const int tiles_x = tiles_x_of(W), tiles_xs = tiles_x_of(Ws);
  const int tile = o >> 7, in = o & 127;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int xp = tx * kTileW + (in & 15), yp = ty * kTileH + (in >> 4);
  uint8_t v = 0;
  if (xp < W + 2 * kImgPad && yp < H + 2 * kImgPad) {
    const int x = min(max(xp - kImgPad, 0), W - 1), y = min(max(yp - kImgPad, 0), H - 1);
    const uint8_t* s = src + f * frame_in;
    const int x0 = 2 * x, y0 = 2 * y;  // 2x+1 ≤ Ws−1 and 2y+1 ≤ Hs−1 because W = ⌊Ws/2⌋, H = ⌊Hs/2⌋
    const unsigned sum = (unsigned)s[texel_index_img(x0, y0, tiles_xs)] + s[texel_index_img(x0 + 1, y0, tiles_xs)] +
                         s[texel_index_img(x0, y0 + 1, tiles_xs)] + s[texel_index_img(x0 + 1, y0 + 1, tiles_xs)];
    v = (uint8_t)((sum + 2u) >> 2);
  }
  dst[i] = v;
}

__global__ void scale_points_kernel(const double2* __restrict__ u0, double2* __restrict__ ul, double s, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ul[i] = make_double2((u0[i].x + 0.5) * s - 0.5, (u0[i].y + 0.5) * s - 0.5);
}

// I_h,k = interpolated host image at u_ref + offset_k (the engine's interpolator), one lane per (point, k)
template <int INTERP>
__global__ void host_intensity_kernel(const uint8_t* __restrict__ images, long long frame_stride, int W, int H,
                                      const double2* __restrict__ u_ref, const int* __restrict__ host,
                                      const float* __restrict__ pattern, int P, float* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int pt = (int)(i / P), k = (int)(i - (long long)pt * P);
  const double2 u = u_ref[pt];
  float I, gx, gy;
  interpolate<INTERP>(images + (long long)host[pt] * frame_stride, W + 1.0, H + 1.0, tiles_x_of(W), u.x + (double)pattern[2 * k],
                      u.y + (double)pattern[2 * k + 1], I, gx, gy);
  out[i] = I;
}

// pba_sample_image: the engine's interpolator at caller positions of one frame (value and gradient)
template <int INTERP>
__global__ void sample_image_kernel(const uint8_t* __restrict__ img, int W, int H, const double2* __restrict__ uv,
                                    float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float I, gx, gy;
  interpolate<INTERP>(img, W + 1.0, H + 1.0, tiles_x_of(W), uv[i].x, uv[i].y, I, gx, gy);
  out[3 * i] = I;
  out[3 * i + 1] = gx;
  out[3 * i + 2] = gy;
}

void swap_buf(DevBuf<uint8_t>& a, DevBuf<uint8_t>& b) { std::swap(a.p, b.p); std::swap(a.n, b.n); }
template <class T>
void swap_buf(DevBuf<T>& a, DevBuf<T>& b) { std::swap(a.p, b.p); std::swap(a.n, b.n); }

void swap_level(pba_engine* e, LevelData& L) {
  swap_buf(e->images, L.images);
  swap_buf(e->intr, L.intr);
  swap_buf(e->intr_d, L.intr_d);
  swap_buf(e->u_ref, L.u_ref);
  swap_buf(e->host_int, L.host_int);
  std::swap(e->width, L.width);
  std::swap(e->height, L.height);
}

}  // namespace

namespace pba {
namespace detail {

// Back to level 0 and drop the pyramid (any set_* call that changes images, cameras, pattern or points).
void reset_pyramid(pba_engine* e) {
  if (e->level > 0 && e->level < (int)e->pyr.size()) swap_level(e, *e->pyr[e->level]);
  e->level = 0;
  e->pyr.clear();
  e->pairs_fresh = false;
}

int sample_host_intensities(pba_engine* e, const double2* u_ref, float* out) {
  const long long n = (long long)e->n_points * e->P;
  if (n == 0) return PBA_OK;
  DevBuf<float> pat;
  PBA_HIP(pat.upload(e->pattern_h, e->stream));
  const unsigned grid = (unsigned)((n + 255) / 256);
  const long long fs = tiled_frame_bytes(e->width, e->height);
  if (e->interp == INTERP_BICUBIC)
    host_intensity_kernel<INTERP_BICUBIC><<<grid, 256, 0, e->stream>>>(e->images.p, fs, e->width, e->height, u_ref,
                                                                         e->point_host_d.p, pat.p, e->P, out, n);
  else
    host_intensity_kernel<INTERP_BILINEAR><<<grid, 256, 0, e->stream>>>(e->images.p, fs, e->width, e->height, u_ref,
                                                                          e->point_host_d.p, pat.p, e->P, out, n);
  PBA_HIP(hipGetLastError());
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

}  // namespace detail
}  // namespace pba

extern "C" {

int pba_set_interpolator(pba_engine* e, int32_t interpolator) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (interpolator != PBA_INTERP_BILINEAR && interpolator != PBA_INTERP_BICUBIC)
    return fail(PBA_ERR_INVALID_ARGUMENT, "unknown interpolator");
  const bool resample = e->host_int_sampled && interpolator != e->interp;
  e->interp = interpolator;
  e->evaluated = false;
  if (!resample) return PBA_OK;
  // I_h,k were sampled on the device with the previous interpolator: sample them again with this one, at every level
  if (int rc = check_device(e)) return rc;
  const int active = e->level;
  if (int rc = pba_set_level(e, 0)) return rc;
  if (int rc = sample_host_intensities(e, e->u_ref.p, e->host_int.p)) return rc;
  for (size_t l = 1; l < e->pyr.size(); ++l) {
    LevelData& L = *e->pyr[l];
    swap_level(e, L);
    const int rc = sample_host_intensities(e, e->u_ref.p, e->host_int.p);
    swap_level(e, L);
    if (rc) return rc;
  }
  return pba_set_level(e, active);
}

int pba_interpolator(const pba_engine* e) { return e ? e->interp : PBA_INTERP_BILINEAR; }

int pba_sample_image(pba_engine* e, int32_t frame, int32_t n, const double* uv, float* out) {
  if (!e || (n > 0 && (!uv || !out)) || n < 0) return fail(PBA_ERR_INVALID_ARGUMENT, "bad sample arguments");
  if (!e->have_images) return fail(PBA_ERR_NOT_READY, "no images");
  if (frame < 0 || frame >= e->n_frames) return fail(PBA_ERR_INVALID_ARGUMENT, "frame out of range");
  if (n == 0) return PBA_OK;
  if (int rc = check_device(e)) return rc;
  DevBuf<double2> d_uv;
  DevBuf<float> d_out;
  PBA_HIP(d_uv.resize(n));
  PBA_HIP(d_out.resize(3 * (size_t)n));
  PBA_HIP(hipMemcpyAsync(d_uv.p, uv, sizeof(double2) * n, hipMemcpyHostToDevice, e->stream));
  const uint8_t* img = e->images.p + (long long)frame * tiled_frame_bytes(e->width, e->height);
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (e->interp == INTERP_BICUBIC)
    sample_image_kernel<INTERP_BICUBIC><<<grid, 256, 0, e->stream>>>(img, e->width, e->height, d_uv.p, d_out.p, n);
  else
    sample_image_kernel<INTERP_BILINEAR><<<grid, 256, 0, e->stream>>>(img, e->width, e->height, d_uv.p, d_out.p, n);
  PBA_HIP(hipGetLastError());
  PBA_HIP(hipMemcpyAsync(out, d_out.p, sizeof(float) * 3 * n, hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

int pba_build_pyramid(pba_engine* e, int32_t n_levels) {
  if (!e || n_levels < 1 || n_levels > PBA_MAX_LEVELS) return fail(PBA_ERR_INVALID_ARGUMENT, "bad level count");
  if (e->opt.residual_kind != PBA_RESIDUAL_PHOTOMETRIC) return fail(PBA_ERR_INVALID_ARGUMENT, "pyramids are photometric only");
  if (!e->have_images || e->n_points <= 0 || e->P <= 0) return fail(PBA_ERR_NOT_READY, "frames, pattern and points first");
  if (int rc = check_device(e)) return rc;
  reset_pyramid(e);
  e->pyr.resize(n_levels);
  std::vector<double> k0(e->intr_d.n);
  PBA_HIP(hipMemcpy(k0.data(), e->intr_d.p, sizeof(double) * k0.size(), hipMemcpyDeviceToHost));
  int Ws = e->width, Hs = e->height;
  const uint8_t* prev = e->images.p;
  for (int l = 1; l < n_levels; ++l) {
    auto L = std::make_unique<LevelData>();
    L->width = Ws / 2;
    L->height = Hs / 2;
    if (L->width < 2 || L->height < 2) {
      e->pyr.clear();
      return fail(PBA_ERR_INVALID_ARGUMENT, "pyramid level smaller than 2x2");
    }
    const long long fin = tiled_frame_bytes(Ws, Hs), fout = tiled_frame_bytes(L->width, L->height);
    const long long n = fout * e->n_frames;
    PBA_HIP(L->images.resize((size_t)n));
    downsample_kernel<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(prev, L->images.p, Ws, Hs, L->width, L->height,
                                                                        fin, fout, n);
    PBA_HIP(hipGetLastError());
    // cameras at level l (kCamD records and the fp32 intrinsics, pba_device.h)
    const double s = std::ldexp(1.0, -l);
    std::vector<double> kd = k0;
    std::vector<float> kf(8 * (size_t)e->n_cams);
    for (int c = 0; c < e->n_cams; ++c) {
      double* r = kd.data() + (size_t)kCamD * c;
      r[0] *= s; r[1] *= s; r[2] = (r[2] + 0.5) * s - 0.5; r[3] = (r[3] + 0.5) * s - 0.5;
      r[kCamHk + 0] = r[2]; r[kCamHk + 1] = r[3]; r[kCamHk + 2] = 1.0 / r[0]; r[kCamHk + 3] = 1.0 / r[1];
      for (int j = 0; j < 8; ++j) kf[8 * c + j] = (float)r[j];
    }
    PBA_HIP(L->intr_d.upload(kd, e->stream));
    PBA_HIP(L->intr.upload(kf, e->stream));
    PBA_HIP(L->u_ref.resize(e->n_points));
    scale_points_kernel<<<(e->n_points + 255) / 256, 256, 0, e->stream>>>(e->u_ref.p, L->u_ref.p, s, e->n_points);
    PBA_HIP(hipGetLastError());
    PBA_HIP(L->host_int.resize((size_t)e->n_points * e->P));
    PBA_HIP(hipStreamSynchronize(e->stream));
    prev = L->images.p;
    Ws = L->width;
    Hs = L->height;
    e->pyr[l] = std::move(L);
  }
  // host intensities per level, sampled from that level's host images
  for (int l = 1; l < n_levels; ++l) {
    LevelData& L = *e->pyr[l];
    swap_level(e, L);
    const int rc = sample_host_intensities(e, e->u_ref.p, e->host_int.p);
    swap_level(e, L);
    if (rc) return rc;
  }
  return PBA_OK;
}

int pba_num_levels(const pba_engine* e) { return e ? std::max(1, (int)e->pyr.size()) : 0; }

int pba_set_level(pba_engine* e, int32_t level) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  const int n = std::max(1, (int)e->pyr.size());
  if (level < 0 || level >= n) return fail(PBA_ERR_INVALID_ARGUMENT, "level out of range (pba_build_pyramid)");
  if (level == e->level) return PBA_OK;
  if (e->level > 0) swap_level(e, *e->pyr[e->level]);
  if (level > 0) swap_level(e, *e->pyr[level]);
  e->level = level;
  e->pairs_fresh = false;
  e->evaluated = false;
  return PBA_OK;
}

int pba_get_level(const pba_engine* e, int32_t* level, int32_t* width, int32_t* height) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (level) *level = e->level;
  if (width) *width = e->width;
  if (height) *height = e->height;
  return PBA_OK;
}

int pba_get_host_intensities(pba_engine* e, float* out) {
  if (!e || !out) return fail(PBA_ERR_INVALID_ARGUMENT, "null argument");
  if (e->opt.residual_kind != PBA_RESIDUAL_PHOTOMETRIC || e->n_points <= 0) return fail(PBA_ERR_NOT_READY, "no photometric points");
  if (int rc = check_device(e)) return rc;
  PBA_HIP(hipMemcpy(out, e->host_int.p, sizeof(float) * (size_t)e->n_points * e->P, hipMemcpyDeviceToHost));
  return PBA_OK;
}

// Coarse to fine: pba_solve on levels n−1 … 0 from the current state; summary accumulates over levels
// (initial cost of the coarsest level, final cost at level 0).
int pba_solve_pyramid(pba_engine* e, const pba_solver_options* options, pba_solver_summary* summary) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  const int n = std::max(1, (int)e->pyr.size());
  pba_solver_summary acc{};
  for (int l = n - 1; l >= 0; --l) {
    if (int rc = pba_set_level(e, l)) return rc;
    pba_solver_summary s{};
    if (int rc = pba_solve(e, options, &s)) return rc;
    if (l == n - 1) acc.initial_cost = s.initial_cost;
    acc.iterations += s.iterations;
    acc.successful_steps += s.successful_steps;
    acc.unsuccessful_steps += s.unsuccessful_steps;
    acc.termination = s.termination;
    acc.stop_reason = s.stop_reason;
    acc.gradient_max_norm = s.gradient_max_norm;
    acc.final_cost = s.final_cost;
    acc.total_ms += s.total_ms;
    acc.linearize_ms += s.linearize_ms;
    acc.solve_ms += s.solve_ms;
    acc.cost_ms += s.cost_ms;
  }
  if (summary) *summary = acc;
  return PBA_OK;
}

}  // extern "C"
