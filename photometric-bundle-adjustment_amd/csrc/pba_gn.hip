// pba_gn.hip — on-device Gauss-Newton / Levenberg-Marquardt for the photometric (and geometric) BA problem.
//
// Replaces the reference's per-iteration CPU work after the cost functors: the Jacobian writer and
// gradient accumulation (program_evaluator.h:233-257), the Schur eliminator + reduced camera system
// Cholesky of SPARSE_SCHUR (schur_complement_solver.cc:138-146; Schur structure <2,1,6>), and the
// Levenberg-Marquardt trust-region loop (trust_region_minimizer.cc, levenberg_marquardt_strategy.cc).
//
// Pipeline of one single-GPU LM trial (all on the engine stream; DESIGN.md §3 has the measured times):
//   schur_gate_kernel      the previous trial's accept; only for a buffer set flagged degenerate, the λ-specific point
//                          elimination (schur_chunk) — else the λ-free partials below are used.
//   assemble_kernel        one lane (four for the long lists) per element of the reduced camera system S and of g:
//                          fixed-order fp64 sums of the partial slots, + λ·clamp(diag) (Ceres' LM diagonal), identity
//                          rows for constant frames; writes cyclic reduction's level 0 directly.
//   cr_level_wave_kernel   block (parallel) cyclic reduction, one launch per level (band ≤ 8); band_solve_kernel
//                          (band ≤ 16); front_solve_kernel (any profile: loop closures, the free-intrinsics border —
//                          the active front in LDS) or skyline_solve_kernel (global memory).
//   update_kernel          T ← T·exp(δ) (Sophus SE3::exp, fp64), δρ = −(g_ρ + Σ W_aᵀ δ_a)/H'_ρρ, the LM model
//                          decrease ½(λ δᵀDδ − gᵀδ) and the candidate pair table, in one launch.
//   linearize_adj_kernel   at the candidate (photometric, ≤ 32 px): rows of 8 lanes per block, the target's 8-column
//                          products on 4×4×4 fp64 matrix-core tiles, host blocks through the pair's adjoint, chunk
//                          partial slots (fp64) and 8 doubles of point data per block; linearize_kernel: the
//                          14-column form (geometric rows, PBA_LIN_LEGACY).
//   schur_free_decide_kernel  the λ-free point elimination of the new linearisation (P/(1 + λ) in the assembly) and,
//                          in 16 workgroups counted in by an atomic, the fixed-order trial sums and Ceres' decision.
// Free intrinsics add intr_rows_kernel and the border kernels (intr_border_*) after the elimination; several GPUs
// exchange the per-rank systems (export_band_kernel, import_kernel / import_sky_kernel, dist_* kernels).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <numeric>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "pba_internal.h"



using namespace pba;
using namespace pba::detail;

namespace {

typedef double v4f64 __attribute__((ext_vector_type(4)));

constexpr int NV = 104;          // normal-equation products per residual row
#ifndef PBA_SCHUR_PTS
#define PBA_SCHUR_PTS 128
#endif
constexpr int SCHUR_PTS = PBA_SCHUR_PTS;   // points per Schur chunk (-DPBA_SCHUR_PTS: A/B builds)
constexpr int SCHUR_W = 2048;    // points × local poses per Schur chunk (LDS budget: dynamic, 48 B each)
constexpr int kPd = 8;            // point data per GN block: [H_ρρ, g_ρ, W_t(6)] (blk_schur)
constexpr int SLOT_LIN_BASE = 42;  // H_hh(36) + g_h(6)
constexpr int SLOT_LIN_T = 78;     // H_ht(36) + H_tt(36) + g_t(6)

enum : int { C_TRANSPOSE = 1, C_SCHUR = 2 };

// x = [J_h(6) | J_t(6) | J_ρ | r]; product v = x[pa(v)] · x[pb(v)]
__host__ __device__ constexpr int upper_index(int i, int j) {  // 6×6 upper triangle, i ≤ j
  return i * 6 - i * (i - 1) / 2 + (j - i);
}
__host__ __device__ constexpr int pa(int v) {
  if (v < 21) { int i = 0; while (upper_index(i, 5) < v) ++i; return i; }
  if (v < 57) return (v - 21) / 6;
  if (v < 78) { int i = 0; while (upper_index(i, 5) < v - 57) ++i; return 6 + i; }
  if (v < 84) return v - 78;
  if (v < 90) return 6 + (v - 84);
  if (v < 92) return 12;
  if (v < 98) return v - 92;
  if (v < 104) return 6 + (v - 98);
  return 13;
}
__host__ __device__ constexpr int pb(int v) {
  if (v < 21) { const int i = pa(v); return i + (v - upper_index(i, i)); }
  if (v < 57) return 6 + (v - 21) % 6;
  if (v < 78) { const int i = pa(v) - 6; return 6 + i + (v - 57 - upper_index(i, i)); }
  if (v < 90) return 13;
  if (v == 90) return 12;
  if (v == 91) return 13;
  if (v < 104) return 12;
  return 13;
}
static_assert(pa(0) == 0 && pb(0) == 0 && pa(20) == 5 && pb(20) == 5 && pa(6) == 1 && pb(6) == 1, "table");
static_assert(pa(57) == 6 && pb(57) == 6 && pa(77) == 11 && pb(77) == 11, "table");
static_assert(pa(21) == 0 && pb(21) == 6 && pa(56) == 5 && pb(56) == 11, "table");

// LM decision record kept on the device by the single-GPU loop (lm_decide_kernel).
// The trial's outcome, then the trust-region state the next trial runs with (λ = 1/radius, read by the kernels), the
// done flag (every later kernel of the solve returns at once: 1 function tolerance, 2 consecutive invalid steps,
// 3 parameter tolerance, 4 gradient tolerance, 5 minimum trust region radius; lm_decide), the index of the
// linearisation buffer set holding the current state's normal-equation pieces (flipped on acceptance), and Ceres'
// bookkeeping: the current state's valid blocks, x_norm (−1 until the first accepted step), consecutive invalid steps,
// and the trial's step and gradient norms.
enum : int {
  kLmCost = 0, kLmCostNew = 1, kLmModel = 2, kLmRel = 3, kLmAccept = 4, kLmStatus = 5, kLmConverged = 6,
  kLmLambda = 7, kLmRadius = 8, kLmFactor = 9, kLmDone = 10, kLmSet = 11, kLmValid = 12, kLmXNorm = 13,
  kLmInvalid = 14, kLmStepNorm = 15, kLmGradNorm = 16, kLmDesync = 17, kLmFields = 18
};
// kDoneDesync (multi-GPU): the ranks' decisions of the previous trial differed (kLmDesync = 1 + the number of ranks whose
// record said done then); every rank ends the solve with an error
enum : int { kDoneFunction = 1, kDoneInvalid = 2, kDoneParameter = 3, kDoneGradient = 4, kDoneRadius = 5, kDoneDesync = 6 };

// A record's decision as a small integer, identical on ranks with identical records: accept, done != 0 and 10 bits of
// the trust-region state (λ's bits folded) — summed with its square over the ranks in the next trial's scalar all-reduce
// (N·Σw² = (Σw)² ⇔ every w equal; exact in fp64 for w < 2^12)
__device__ inline double decision_word(const double* lm) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(lm[kLmLambda]);
  unsigned h = (unsigned)(b ^ (b >> 20) ^ (b >> 40) ^ (b >> 60));
  h = (h ^ (h >> 10) ^ (h >> 20)) & 1023u;
  return (double)((h << 2) | (lm[kLmDone] != 0.0 ? 2u : 0u) | (lm[kLmAccept] != 0.0 ? 1u : 0u));
}
// The published copies of the record (host-coherent page-locked memory): a ring of kRecRing slots of kLmFields fields
// + the trial's sequence number, trial `seq` in slot seq mod kRecRing.  The host enqueues one trial ahead of the record
// it waits for, so two records can be in flight; with a single slot, a host thread descheduled for longer than a trial
// (~0.23 ms at C4) would find the next trial's record over the one it waits for and fail the solve.
#ifndef PBA_REC_RING
#define PBA_REC_RING 4
#endif
constexpr int kRecRing = PBA_REC_RING, kRecStride = kLmFields + 1;  // (-DPBA_REC_RING=1: the one-slot record, tests)
__host__ __device__ inline long long rec_slot(double seq) { return ((long long)seq % kRecRing) * kRecStride; }
// The kernels always get a record: the device loop's, or — host-driven steps — GnData::lm_idle (not done, set 0, λ NaN
// = use the kernel's λ argument).  They read it with their first loads, never behind a branch of its own (a gate
// read before anything else cost the linearisation ~8 µs of serialised scalar round trips).
struct LmView {
  double done, set, lambda, accept;
};
__device__ __forceinline__ LmView lm_view(const double* lm) {
  return LmView{lm[kLmDone], lm[kLmSet], lm[kLmLambda], lm[kLmAccept]};
}
__device__ __forceinline__ double lm_lambda(const LmView& v, double lambda) { return isnan(v.lambda) ? lambda : v.lambda; }

struct LinArgs {
  const int4* lin_rec;      // chunk slot → {block, point, pair | local target slot << 24, GN position (blk_schur index)}
  double* blk_schur1;       // the second buffer set (device LM loop: the candidate's linearisation goes to the spare)
  double* part_lin1;
  double* wg_red;           // per-chunk (Σ cost, Σ valid) slots, or nullptr
  const int4* chunk_desc;   // first linearise position, count, n_targets, partial offset (slots)
  double* blk_schur;
  double* part_lin;
  int n_chunks;
  const double* lm;         // LM record: skip when the solve is done; spare: write the set the record does not hold
  bool spare;
  int* lin_set;             // or nullptr: the set written (workgroup 0 stores it, and clears degen[set])
  int* degen;
  double* pair_rt;          // per pair [R_th(9), t_th(3)] of the linearisation (set 0 / set 1): schur_chunk forms
  double* pair_rt1;         // W_h = −W_t·Ad from them
};

// The linearisation's R_th, t_th of pair `pair` into pair_rt, by lanes k < 12 of the LPB lanes of the first block of
// each target in the wave (the same values where a pair's blocks span waves or chunks)
template <int LPB>
__device__ __forceinline__ void store_pair_rt(double* pair_rt, const double* R, const double* t, int pair, int lt, int k,
                                              bool live) {
  const int lane = threadIdx.x & 63;
  const int prev = __shfl(lt, (lane - LPB) & 63, 64);
  if (live && ((lane & ~(LPB - 1)) == 0 || prev != lt))
    for (int e = k; e < 12; e += LPB) pair_rt[(long long)pair * 12 + e] = e < 9 ? R[e] : t[e - 9];
}

// ------------------------------------------------------------------------------------------------
// linearize_kernel
// ------------------------------------------------------------------------------------------------
// Slot of the product x[r]·x[c] (r ≤ c) in the 104-product layout, or 255 when not needed (x13·x13, pad columns).
__host__ __device__ constexpr int slot_of(int r, int c) {
  for (int v = 0; v < NV; ++v)
    if (pa(v) == r && pb(v) == c) return v;
  return 255;
}
// MFMA 16×16 output held by lane l, entry m = 0..3: v_mfma_f32_16x16x4f32 C[4(l/16) + m][l%16], v_mfma_f64_16x16x4f64
// C[l/16 + 4m][l%16] (cdna_hip_programming.md: the f64 form has a layout of its own) → the four slots of lane l (upper
// triangle only, so each product is written once), packed as bytes.
__host__ __device__ constexpr unsigned slot_word(int lane, bool f64) {
  unsigned w = 0;
  for (int m = 0; m < 4; ++m) {
    const int r = f64 ? (lane >> 4) + 4 * m : 4 * (lane >> 4) + m, c = lane & 15;
    w |= (unsigned)(r <= c ? slot_of(r, c) : 255) << (8 * m);
  }
  return w;
}
template <int... L>
constexpr auto make_slot_table(bool f64, std::integer_sequence<int, L...>) {
  struct T { unsigned w[64]; };
  return T{{slot_word(L, f64)...}};
}
__constant__ const auto kSlotTable64 = make_slot_table(true, std::make_integer_sequence<int, 64>{});

// At most this many targets per linearise chunk (gn_prepare cuts chunks there): a wave's blocks then hold ≤ 4 target
// runs, so its per-run product sets (fp64) fit the LDS the fp32 ones took for 8.
constexpr int kChunkTargets = 4;


// Normal-equation products by matrix cores: weighted rows X (R × 14, padded to LPB × 16 per block; fp32) give
// XᵀX = Σ_k x_kᵀx_k as v_mfma_f64_16x16x4f64 steps (operand A = Xᵀ and B = X are the same register: lane l holds
// X[4s + l/16][l%16], converted to fp64) — the products of fp32 rows are exact in fp64, so the system is the Gram
// matrix of the rows to fp64 rounding.  A chunk's blocks are ordered by target (gn_prepare), so the blocks of one
// target are consecutive in a wave: each block's product set is added to its target run's sum, and a wave stores one
// product set per distinct target (≤ kChunkTargets) instead of one per block.
template <int KIND, int MODEL, int LPB>
constexpr int kLinWaves = KIND == PBA_RESIDUAL_PHOTOMETRIC && MODEL == CAM_PINHOLE + 4 * INTERP_BILINEAR && LPB == 8 ? 8 : 1;

template <int KIND, int MODEL, int LPB>
__global__ __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(kLinWaves<KIND, MODEL, LPB>, 8)))
void linearize_kernel(const KernelArgs a, const LinArgs g) {
  constexpr int BW = 64 / LPB;              // blocks per wave
  constexpr int NW = kBlockThreads / 64;    // waves per workgroup
  constexpr int SPB = LPB / 4;              // MFMA steps per block
  constexpr int NVP = 108;                  // 104 products, padded
  constexpr int kTileW = KIND == PBA_RESIDUAL_PHOTOMETRIC ? BW * (int)sizeof(TileBlock) : 0;
  constexpr int kRowsW = 64 * 16 * 4, kProdW = kChunkTargets * NVP * 8;
  constexpr int kArena = (kTileW > kRowsW ? (kTileW > kProdW ? kTileW : kProdW) : (kRowsW > kProdW ? kRowsW : kProdW));
  // per-wave arena, used in turn by the wave's tile blocks, its weighted rows and its per-target products
  // (each phase only touches the wave's own blocks; LDS is in order within a wave)
  __shared__ __attribute__((aligned(16))) unsigned char arena[NW][kArena];
  __shared__ int s_wlo[NW], s_wn[NW];
  __shared__ float s_bc[kBlockThreads / LPB];  // block costs (0: invalid or dead), for the chunk's cost partial
  __shared__ unsigned s_slots[NW][64];          // the product slot table (kSlotTable64), each lane's word parked in LDS
  const int chunk = logical_tile();
  const int lb = threadIdx.x / LPB;
  // one memory round: the record, the chunk descriptor, the block's linearise record and the slot table are all issued
  // before either exit (at a clamped chunk), and the exits test them together — the compiler otherwise issued the record
  // behind the chunk test, the descriptor behind the record's done test and the linearise record behind both (three
  // dependent rounds before the tile's loads)
  const int cc = min(chunk, g.n_chunks - 1);
  const int4 d = g.chunk_desc[cc];
  const int4 lr = g.lin_rec[(long long)cc * (kBlockThreads / LPB) + lb];
  const unsigned slot_w = kSlotTable64.w[threadIdx.x & 63];
  const LmView lv = lm_view(g.lm);
  asm volatile("" ::"v"(lr.x), "v"(lr.y), "v"(lr.z), "v"(lr.w), "v"(slot_w), "s"(d.x), "s"(d.y), "s"(d.z), "s"(d.w));
  s_slots[threadIdx.x >> 6][threadIdx.x & 63] = slot_w;  // (read back by the same lane: no barrier)
  if (chunk >= g.n_chunks || lv.done != 0.0) return;
  const bool s1 = (lv.set != 0.0) != g.spare;
  double* const blk_schur = s1 ? g.blk_schur1 : g.blk_schur;
  double* const part_lin = s1 ? g.part_lin1 : g.part_lin;
  if (g.lin_set && chunk == 0 && threadIdx.x == 0) {  // (the λ-free elimination after this launch reads them)
    *g.lin_set = s1 ? 1 : 0;
    g.degen[s1 ? 1 : 0] = 0;
  }
  const int count = d.y, n_t = d.z, poff = d.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int k = threadIdx.x % LPB, wb = lb % BW;
  const bool live = lb < count;
  const int R = KIND == PBA_RESIDUAL_PHOTOMETRIC ? a.P : 2;
  const bool act = live && k < R;
  // the chunk's slots are padded to the workgroup's blocks (dead slots repeat slot 0), so the record is read with the
  // chunk descriptor, not behind it, and carries the block's point and pair: the tile prologue's loads come next
  const int blk = lr.x, gpos = lr.w, lt = (int)((unsigned)lr.z >> 24);
  Row row;
  if constexpr (KIND == PBA_RESIDUAL_PHOTOMETRIC) {
    TileBlock* s_tb = reinterpret_cast<TileBlock*>(arena[wave]);
    const float2 off = pattern_at<LPB>(a, k);
    // the host intensity in the tile's memory round (its point is in the linearise record): issued behind the tile's
    // loads it cost a round of its own at the barrier
    const float Ih = act ? a.host_int[(long long)lr.y * R + k] : 0.0f;
    stage_tile_pp<LPB>(a, s_tb, wb, k, make_int2(lr.y, lr.z & 0xffffff));
    asm volatile("" ::"v"(Ih));
    __syncthreads();
#ifdef PBA_ABL_NOROW  // ablation builds (tools/build_variant.sh): timing of the parts, results are garbage
    row.r = Ih + s_tb[wb].pr.Rf[k & 7] + off.x;
    row.jr = row.hv.x = row.hv.y = row.hv.z = row.hw.x = row.hw.y = row.hw.z = row.r;
    row.tv = row.hv;
    row.tw = row.hw;
#else
    row = photometric_row<MODEL, true>(a, s_tb[wb], off, Ih);  // dead lanes evaluate a staged block, masked below
#endif
    store_pair_rt<LPB>(s1 ? g.pair_rt1 : g.pair_rt, s_tb[wb].pr.R, s_tb[wb].pr.t, lr.z & 0xffffff, lt, k, live);
  } else {
    if (act) row = geometric_row<MODEL, true>(a, blk, k);
    const PairRec& pr = a.pairs[lr.z & 0xffffff];
    store_pair_rt<LPB>(s1 ? g.pair_rt1 : g.pair_rt, pr.R, pr.t, lr.z & 0xffffff, lt, k, live);
  }
  const int ok = group_all<LPB>(act ? row.ok : 1);
  const float s = group_sum<LPB>(act && ok ? row.r * row.r : 0.0f);
  const float w = ok ? huber_weight(s, a.huber) : 0.0f;
  const float bcost = ok ? huber_cost(s, a.huber) : 0.0f;
  if (k == 0) s_bc[lb] = live && ok ? bcost : -1.0f;  // read after the barrier below
  // weighted row x̃ = √w · x  → products carry w (Ceres Corrector with ρ'' ≤ 0: J̃ = √ρ' J, r̃ = √ρ' r)
  // the product slot table, loaded in the first memory round and parked in LDS across the row (one register fewer
  // there: the row's peak pressure spilled at 8 waves/SIMD)
  const unsigned slots = s_slots[wave][lane];
  // rows outside the domain / of dead lanes are all zero (selects, not a zero weight: such a row may hold inf / NaN)
  const bool use = act && ok;
  const float sw = use ? sqrtf(w) : 0.0f;
  auto wx = [&](float v) { return use ? sw * v : 0.0f; };
  const float x[14] = {wx(row.hv.x), wx(row.hv.y), wx(row.hv.z), wx(row.hw.x), wx(row.hw.y), wx(row.hw.z),
                       wx(row.tv.x), wx(row.tv.y), wx(row.tv.z), wx(row.tw.x), wx(row.tw.y), wx(row.tw.z),
                       wx(row.jr), wx(row.r)};
  float* sX = reinterpret_cast<float*>(arena[wave]);  // the wave's 64 rows × 16 floats (overwrites its tile blocks)
  {
    float4* xr = reinterpret_cast<float4*>(sX + lane * 16);
    xr[0] = make_float4(x[0], x[1], x[2], x[3]);
    xr[1] = make_float4(x[4], x[5], x[6], x[7]);
    xr[2] = make_float4(x[8], x[9], x[10], x[11]);
    xr[3] = make_float4(x[12], x[13], 0.0f, 0.0f);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    // every operand first (the product sets below overwrite the rows), then the wave's blocks in order; each run of
    // equal local target is summed in registers and its 16×16 result scattered as the 104 products of that slot
    const int ci = lane & 15, kq = lane >> 4;
    float op[BW * SPB];
#pragma unroll
    for (int st = 0; st < BW * SPB; ++st) op[st] = sX[(4 * st + kq) * 16 + ci];
    double* sP = reinterpret_cast<double*>(arena[wave]);
    const int nbw = min(max(count - wave * BW, 0), BW);  // live blocks of this wave (wave-uniform)
    const int lo = __builtin_amdgcn_readfirstlane(lt);     // lane 0 holds the wave's first block
    auto flush = [&](const v4f64& acc, int slot) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const unsigned v = (slots >> (8 * m)) & 255u;
        if (v < (unsigned)NV) sP[slot * NVP + v] = acc[m];
      }
    };
    // per block: its own chain (SPB steps); row 12 of the result, C[12][c] in entry 3 of lanes c < 16, is the block's
    // point-elimination data x̃_ρ·x̃_c → [H_ρρ, g_ρ, W_h(6), W_t(6), 0, 0] at its GN position (schur_kernel walks
    // them point by point); the block's products are then added to its target run's sum
    // (column c of row 12: W_h for c < 6 — not stored, schur_chunk forms it from W_t — W_t for 6 ≤ c < 12, H_ρρ, g_ρ)
    const int pc = lane < 16 ? lane : -1, pq = pc >= 6 && pc < 12 ? pc - 4 : (pc == 12 ? 0 : (pc == 13 ? 1 : -1));
    v4f64 tacc = {0.0, 0.0, 0.0, 0.0};
    int cur = lo;
    // block b's chain (SPB dependent steps); a dead block's rows are zeros, so its chain is issued unconditionally
#ifndef PBA_ABL_NOMFMA
    auto chain = [&](int b) {
      v4f64 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int st = 0; st < SPB; ++st) {
        const double o = (double)op[b * SPB + st];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(o, o, acc, 0, 0, 0);
      }
      return acc;
    };
#endif
    // two blocks in flight: block b + 1's matrix-core steps are issued before block b's result is consumed (each
    // dependent fp64 step waited out its latency before the point-data store and the run sum otherwise)
#ifdef PBA_ABL_NOMFMA
    auto chain = [&](int b) {
      const double o = (double)op[b * SPB];
      return v4f64{o, o, o, o};
    };
#endif
    v4f64 nxt = chain(0);
#pragma unroll
    for (int b = 0; b < BW; ++b) {
      const v4f64 acc = nxt;
      if (b + 1 < BW) nxt = chain(b + 1);
#ifdef PBA_ABL_NOBLK
      if (b == 0) {
        tacc = acc;
        cur = lo;
      }
      if (false) {
#else
      if (b < nbw) {
#endif
        const int gpb = __builtin_amdgcn_readlane(gpos, b * LPB);
        if (pq >= 0) blk_schur[(long long)gpb * kPd + pq] = acc[3];
#ifndef PBA_ABL_NORUN
        const int ltb = __builtin_amdgcn_readlane(lt, b * LPB);
        if (ltb != cur) {
          flush(tacc, cur - lo);
          tacc = v4f64{0.0, 0.0, 0.0, 0.0};
          cur = ltb;
        }
        tacc += acc;
#endif
      }
    }
    if (nbw > 0) flush(tacc, cur - lo);
    if (lane == 0) {
      s_wlo[wave] = lo;
      s_wn[wave] = nbw > 0 ? cur - lo + 1 : 0;
    }
  }
  __syncthreads();
  // chunk partial slots, fixed summation order (wave, then slot): H_hh / g_h over every product set of the chunk,
  // H_ht / H_tt / g_t of local target j from the ≤ NW sets of j (one per wave that holds j's blocks)
  auto sset = [&](int w, int i, int v) -> double { return reinterpret_cast<const double*>(arena[w])[i * NVP + v]; };
#ifdef PBA_ABL_NOPART
  const int nout = 0;
#else
  const int nout = SLOT_LIN_BASE + SLOT_LIN_T * n_t;
#endif
  for (int o = threadIdx.x; o < nout; o += kBlockThreads) {
    int v, j = -1;
    if (o < 36) {
      const int r = o / 6, c = o % 6;
      v = upper_index(min(r, c), max(r, c));
    } else if (o < 42) {
      v = 78 + (o - 36);
    } else {
      j = (o - 42) / SLOT_LIN_T;
      const int q = (o - 42) % SLOT_LIN_T;
      if (q < 36) v = 21 + q;
      else if (q < 72) { const int r = (q - 36) / 6, c = (q - 36) % 6; v = 57 + upper_index(min(r, c), max(r, c)); }
      else v = 84 + (q - 72);
    }
    double acc = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int wl = s_wlo[w], wn = s_wn[w];
      if (j < 0) {
        for (int i = 0; i < wn; ++i) acc += sset(w, i, v);
      } else if (j >= wl && j < wl + wn) {
        acc += sset(w, j - wl, v);
      }
    }
    part_lin[(long long)poff + o] = acc;
  }
  // the block costs last: a store issued before a load makes the wait for that load wait for the store too (GFX9
  // counts loads and stores in one counter), so the stores go after every load of the kernel
  if (live && k == 0) {
    a.valid[blk] = (uint8_t)ok;
    a.cost[blk] = bcost;
  }
  if (g.wg_red && wave == 0) {  // the chunk's (Σ cost, Σ valid): lane b takes block b, xor butterflies (fixed order)
    static_assert(kBlockThreads / LPB <= 64, "one lane per block of the chunk");
    const float x = lane < count ? s_bc[lane] : -1.0f;
    double c = x >= 0.0f ? (double)x : 0.0, v = x >= 0.0f ? 1.0 : 0.0;
    for (int m = 32; m >= 1; m >>= 1) {
      c += __shfl_xor(c, m, 64);
      v += __shfl_xor(v, m, 64);
    }
    if (lane == 0) {
      g.wg_red[2 * chunk] = c;
      g.wg_red[2 * chunk + 1] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// linearize_adj_kernel: the photometric linearisation of ≤ 8-px patterns through the pair's adjoint
// ------------------------------------------------------------------------------------------------
// A photometric row's host Jacobian is its target Jacobian through the relative pose: with p̃ = R b + ρ t (R = R_th,
// t = t_th) the rows of photometric_row satisfy [hv hw] = −[tv tw]·Ad, Ad = [[R, [t]×R], [0, R]] — the SE(3) adjoint of
// T_th (exact algebra: hv = ρ qR = −tv R, hw = b × qR = −tw R − tv [t]× R).  Ceres differentiates both poses through
// the functor (photometric_error.h:146-186); the normal equations only need their products, and those follow from the
// target's: J_hᵀJ_h = Adᵀ(J_tᵀJ_t)Ad, J_hᵀJ_t = −Adᵀ(J_tᵀJ_t), J_hᵀr = −Adᵀ(J_tᵀr), J_ρᵀJ_h = −(J_ρᵀJ_t)Ad — linear in
// the per-target sums, so applied once per (chunk, target) and once per block for the point data.  The matrix cores
// then form only the 8-column products of x = √w [tv tw jr r] (36 in the upper triangle, against 104 of the 14-column
// rows): per block the three 4×4 tiles (0,0), (0,1), (1,1) of xᵀx, K = 8 rows in two steps of v_mfma_f64_4x4x4_4b_f64
// (16 cycles each, against two 64-cycle v_mfma_f64_16x16x4f64).  Same chunk partials and point data as
// linearize_kernel (the 14-column kernel, kept for the geometric rows and as PBA_LIN_LEGACY's A/B reference).
// MFMA layout (tools/micro/mfma_f64_4x4_layout.hip, measured): lane l works in 4×4 block β = (l >> 2) & 3; A holds
// A_β[l & 3][l >> 4], B holds B_β[l >> 4][l & 3], the accumulator C_β[l >> 4][l & 3].
__host__ __device__ constexpr int upper8(int r, int c) { return r * 8 - r * (r - 1) / 2 + (c - r); }  // r ≤ c < 8

// PPL > 1 (9…32 px, C5's 21): lane k evaluates pixels k, k + 8, … in PPL passes (8 lanes per block, as the evaluation's
// photometric_block_kernel_multi: a chunk stays 32 blocks, the chunk partials those of 8 px); each pass's
// unweighted rows go through the matrix cores into per-block fp64 accumulators (the chain runs on across the passes) and
// the block's Huber weight, known after its last row, scales them (x̃ᵀx̃ = w·xᵀx).  LDS per wave: the tile blocks and a
// pass's rows side by side, the run product sets over the tile once the passes are done.
#ifndef PBA_LINADJ_WAVES
#define PBA_LINADJ_WAVES 5
#endif
// NT: threads per workgroup (NT / 8 blocks per chunk).  Measured at 8 px: 512 threads (64-block chunks: the phases,
// partial slots, assembly contributions and decision slots per chunk spread over twice the blocks) 71.1 → 76.6 µs for
// the linearisation against 12.1 → 10.9 for the assembly — the 8-wave barriers cost more than the halved chunk work.
template <int MODEL, int PPL, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PPL == 1 ? 8 : PBA_LINADJ_WAVES, 8)))
void linearize_adj_kernel(const KernelArgs a, const LinArgs g) {
  constexpr int LPB = 8, BW = 64 / LPB, NW = NT / 64;
  constexpr int kRowS = 12;                  // floats per staged row (8 used): 8-lane groups of b128 stores hit 32 banks
  constexpr int NQ = 36;                     // products per run set (the 8 × 8 upper triangle)
  constexpr int kTileW = BW * (int)sizeof(TileBlock), kRowsW = 64 * kRowS * 4, kProdW = kChunkTargets * NQ * 8;
  // per wave — PPL = 1: [tile blocks, then the weighted rows over them | run product sets];
  //            PPL > 1: [tile blocks, then the run product sets over them | a pass's rows]
  constexpr int kRowsOff = PPL == 1 ? 0 : kTileW;
  constexpr int kProdOff = PPL == 1 ? (kTileW > kRowsW ? kTileW : kRowsW) : 0;
  constexpr int kArena = PPL == 1 ? kProdOff + kProdW : kTileW + kRowsW;
  static_assert(kProdW <= kTileW && kRowsW <= kTileW + 512, "regions");
  static_assert(kChunkTargets * 64 * 8 <= kRowsW, "phase data fits a rows region");
  static_assert(NT >= 64 * kChunkTargets && NT / LPB <= 64, "one thread per entry of the targets' 8 × 8 sums");
  __shared__ __attribute__((aligned(16))) unsigned char arena[NW][kArena];
  __shared__ double s_rt[kChunkTargets][12];  // R_th, t_th of each local target (the host is the chunk's)
  __shared__ double s_ad[kChunkTargets][36];  // Ad of each local target
  __shared__ int s_wlo[NW], s_wn[NW];
  __shared__ float s_bc[NT / LPB];
  __shared__ float2 s_pat[PPL == 1 ? 1 : LPB * PPL];
  const int chunk = logical_tile();
  const int lb = threadIdx.x / LPB;
  // one memory round: record, chunk descriptor and linearise record before either exit (see linearize_kernel)
  const int cc = min(chunk, g.n_chunks - 1);
  const int4 d = g.chunk_desc[cc];
  const int4 lr = g.lin_rec[(long long)cc * (NT / LPB) + lb];
  const LmView lv = lm_view(g.lm);
  asm volatile("" ::"v"(lr.x), "v"(lr.y), "v"(lr.z), "v"(lr.w), "s"(d.x), "s"(d.y), "s"(d.z), "s"(d.w));
  if (chunk >= g.n_chunks || lv.done != 0.0) return;
  const bool s1 = (lv.set != 0.0) != g.spare;
  double* const blk_schur = s1 ? g.blk_schur1 : g.blk_schur;
  double* const part_lin = s1 ? g.part_lin1 : g.part_lin;
  if (g.lin_set && chunk == 0 && threadIdx.x == 0) {  // (the λ-free elimination after this launch reads them)
    *g.lin_set = s1 ? 1 : 0;
    g.degen[s1 ? 1 : 0] = 0;
  }
  const int count = d.y, n_t = d.z, poff = d.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int k = threadIdx.x % LPB, wb = lb % BW;
  const bool live = lb < count;
  const int R = a.P;
  const int blk = lr.x, gpos = lr.w, lt = (int)((unsigned)lr.z >> 24);
  TileBlock* s_tb = reinterpret_cast<TileBlock*>(arena[wave]);
  float* sX = reinterpret_cast<float*>(arena[wave] + kRowsOff);  // the wave's 64 rows
  // lane l: 4×4 block β — tiles (0,0), (0,1), (1,1) of xᵀx, and β = 3 repeating (0,1) unused — operand columns
  // ca / cb, product (pr_, pc_)
  const int beta = (lane >> 2) & 3, i4 = lane & 3, kq = lane >> 4;
  const int I = beta == 2 ? 1 : 0, J = beta == 0 ? 0 : 1;
  const int ca = 4 * I + i4, cb = 4 * J + i4;
  auto ops = [&](int b, float* o) {  // block b's operands from the staged rows: A, B of K steps 0 and 1
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const float* xr = sX + (8 * b + 4 * st + kq) * kRowS;
      o[2 * st] = xr[ca];
      o[2 * st + 1] = xr[cb];
    }
  };
  auto save_rt = [&]() {  // R_th, t_th of the block's target from the first block of each target in the wave, for
                          // the phases below and (pair_rt) the point elimination's W_h
    const int prev = __shfl(lt, (lane - LPB) & 63, 64);
    if (live && (wb == 0 || prev != lt)) {
      const PairRec& pr = s_tb[wb].pr;
      double* prt = (s1 ? g.pair_rt1 : g.pair_rt) + (long long)(lr.z & 0xffffff) * 12;
      s_rt[lt][k] = prt[k] = pr.R[k];
      if (k < 4) s_rt[lt][8 + k] = prt[8 + k] = k == 0 ? pr.R[8] : pr.t[k - 1];
    }
  };
  int ok;
  float bcost;
  double accb[BW];  // the blocks' products (PPL > 1: unweighted over the passes, then weighted)
  if constexpr (PPL == 1) {
    const bool act = live && k < R;
    const float2 off = pattern_at<LPB>(a, k);
    const float Ih = act ? a.host_int[(long long)lr.y * R + k] : 0.0f;
    stage_tile_pp<LPB>(a, s_tb, wb, k, make_int2(lr.y, lr.z & 0xffffff));
    asm volatile("" ::"v"(Ih));
    __syncthreads();
#ifdef PBA_ABL_ROW  // ablation builds (tools/build_variant.sh): timing of the parts, results are garbage
    Row row;
    row.r = Ih + (float)s_tb[wb].pr.R[k] + off.x;
    row.jr = row.r;
    row.tv = Vec3{row.r, row.r, row.r};
    row.tw = row.tv;
#else
    const Row row = photometric_row<MODEL, true>(a, s_tb[wb], off, Ih);  // (hv, hw unused: not formed)
#endif
    save_rt();
    ok = group_all<LPB>(act ? row.ok : 1);
    const float s = group_sum<LPB>(act && ok ? row.r * row.r : 0.0f);
    const float w = ok ? huber_weight(s, a.huber) : 0.0f;
    bcost = ok ? huber_cost(s, a.huber) : 0.0f;
    const bool use = act && ok;
    const float sw = use ? sqrtf(w) : 0.0f;
    auto wx = [&](float v) { return use ? sw * v : 0.0f; };
    float4* xr = reinterpret_cast<float4*>(sX + lane * kRowS);  // (over the wave's tile blocks, read above)
    xr[0] = make_float4(wx(row.tv.x), wx(row.tv.y), wx(row.tv.z), wx(row.tw.x));
    xr[1] = make_float4(wx(row.tw.y), wx(row.tw.z), wx(row.jr), wx(row.r));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    if ((int)threadIdx.x < LPB * PPL) s_pat[threadIdx.x] = pattern_at<LPB * PPL>(a, threadIdx.x);
    float Ih[PPL];
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int px = k + LPB * j;
      Ih[j] = live && px < R ? a.host_int[(long long)lr.y * R + px] : 0.0f;
    }
    stage_tile_pp<LPB>(a, s_tb, wb, k, make_int2(lr.y, lr.z & 0xffffff));
#pragma unroll
    for (int j = 0; j < PPL; ++j) asm volatile("" ::"v"(Ih[j]));
    __syncthreads();
    save_rt();
#pragma unroll
    for (int b = 0; b < BW; ++b) accb[b] = 0.0;
    int okl = 1;
    float s = 0.0f;
#pragma unroll 1
    for (int j = 0; j < PPL; ++j) {
      const int px = k + LPB * j;
      const bool act = live && px < R;
      float ih = Ih[0];
#pragma unroll
      for (int q = 1; q < PPL; ++q) ih = j == q ? Ih[q] : ih;
      asm volatile("" ::: "memory");  // the tile is read from LDS per pass (see photometric_block_kernel_multi)
#ifdef PBA_ABL_ROW
      Row row;
      row.ok = 1;
      row.r = ih + (float)s_tb[wb].pr.R[k] + s_pat[act ? px : 0].x;
      row.jr = row.r;
      row.tv = Vec3{row.r, row.r, row.r};
      row.tw = row.tv;
#else
      const Row row = photometric_row<MODEL, true>(a, s_tb[wb], s_pat[act ? px : 0], ih);
#endif
      const bool use = act && row.ok;
      okl &= act ? row.ok : 1;
      s += use ? row.r * row.r : 0.0f;
      auto xv = [&](float v) { return use ? v : 0.0f; };  // selects: a row that is not ok may hold inf / NaN
      float4* xr = reinterpret_cast<float4*>(sX + lane * kRowS);
      xr[0] = make_float4(xv(row.tv.x), xv(row.tv.y), xv(row.tv.z), xv(row.tw.x));
      xr[1] = make_float4(xv(row.tw.y), xv(row.tw.z), xv(row.jr), xv(row.r));
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifndef PBA_ABL_MFMA
#pragma unroll
      for (int b = 0; b < BW; ++b) {
        float o[4];
        ops(b, o);
#pragma unroll
        for (int st = 0; st < 2; ++st)
          accb[b] = __builtin_amdgcn_mfma_f64_4x4x4f64((double)o[2 * st], (double)o[2 * st + 1], accb[b], 0, 0, 0);
      }
#endif
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // this pass's reads before the next pass's row stores
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    ok = group_all<LPB>(okl);
    s = group_sum<LPB>(s);
    const float w = ok ? huber_weight(s, a.huber) : 0.0f;
    bcost = ok ? huber_cost(s, a.huber) : 0.0f;
#pragma unroll
    for (int b = 0; b < BW; ++b)
      accb[b] *= (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), b * LPB));
  }
  if (k == 0) s_bc[lb] = live && ok ? bcost : -1.0f;  // read after the barrier below
  const int nbw = min(max(count - wave * BW, 0), BW);
  {
    const int pr_ = 4 * I + kq, pc_ = 4 * J + i4;
    const int pslot = beta < 3 && pr_ <= pc_ ? upper8(pr_, pc_) : -1;
    // the point data: column 6 (jr) of tiles (0,1) and (1,1) — W_t[0..3] and W_t[4..5], H_ρρ, g_ρ — at its blk_schur
    // position [H_ρρ, g_ρ, W_t(6)]
    const int ppos = i4 != 2 || beta == 0 || beta == 3 ? -1 : (beta == 1 ? 2 + kq : (kq < 2 ? 6 + kq : kq - 2));
    double* sP = reinterpret_cast<double*>(arena[wave] + kProdOff);
    const int lo = __builtin_amdgcn_readfirstlane(lt);
    if constexpr (PPL == 1) {
      // every block's products first — the two-step chains of four blocks at a time in flight together — then the
      // stores: the matrix-core latency is paid once per four blocks, and the point-data and run-set stores each run
      // under one exec mask instead of one per block
#pragma unroll
      for (int h = 0; h < BW; h += 4) {
        float o[4][4];
#pragma unroll
        for (int b = 0; b < 4; ++b) ops(h + b, o[b]);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          double acc = 0.0;
#pragma unroll
          for (int st = 0; st < 2; ++st)
            acc = __builtin_amdgcn_mfma_f64_4x4x4f64((double)o[b][2 * st], (double)o[b][2 * st + 1], acc, 0, 0, 0);
          accb[h + b] = acc;
        }
      }
    }
    int gpb[BW];  // (read in uniform control flow: a readlane of a lane the exec mask excludes reads a dead register)
#pragma unroll
    for (int b = 0; b < BW; ++b) gpb[b] = __builtin_amdgcn_readlane(gpos, b * LPB);
    if (ppos >= 0) {
#pragma unroll
      for (int b = 0; b < BW; ++b)
        if (b < nbw) blk_schur[(long long)gpb[b] * kPd + ppos] = accb[b];
    }
    double tacc = 0.0;
    int cur = lo;
#pragma unroll
    for (int b = 0; b < BW; ++b) {
      if (b < nbw) {
        const int ltb = __builtin_amdgcn_readlane(lt, b * LPB);
        if (ltb != cur) {
          if (pslot >= 0) sP[(cur - lo) * NQ + pslot] = tacc;
          tacc = 0.0;
          cur = ltb;
        }
        tacc += accb[b];
      }
    }
    if (nbw > 0 && pslot >= 0) sP[(cur - lo) * NQ + pslot] = tacc;
    if (lane == 0) {
      s_wlo[wave] = lo;
      s_wn[wave] = nbw > 0 ? cur - lo + 1 : 0;
    }
  }
#ifdef PBA_ABL_PHASE
  if (n_t > 0) return;
#endif
  __syncthreads();
  // Phase A: the chunk's product sums per local target j, as full 8 × 8 matrices (one thread per entry; the sets of j
  // over the waves in order), and Ad_j from R_th, t_th.  Over wave 0's rows.
  double* sT = reinterpret_cast<double*>(arena[0] + kRowsOff);  // [j][8][8]
  double* sN = reinterpret_cast<double*>(arena[1] + kRowsOff);  // [j][6][6]: H_tt,j·Ad_j
  {
    const int t = threadIdx.x, j = t >> 6, r = (t >> 3) & 7, c = t & 7;
    if (j < n_t && t < 64 * kChunkTargets) {
      const int u = upper8(min(r, c), max(r, c));
      double acc = 0.0;
#pragma unroll
      for (int w_ = 0; w_ < NW; ++w_) {
        const int wl = s_wlo[w_], wn = s_wn[w_];
        if (j >= wl && j < wl + wn) acc += reinterpret_cast<const double*>(arena[w_] + kProdOff)[(j - wl) * NQ + u];
      }
      sT[t] = acc;
    }
    if (t < 36 * n_t) {  // Ad = [[R, [t]×R], [0, R]]; ([t]×R)[q][c] = t[q+1] R[q+2][c] − t[q+2] R[q+1][c] (indices mod 3)
      const int jj = t / 36, e = t - 36 * jj, q = e / 6, p = e - 6 * q;
      const double* rt = s_rt[jj];
      double v = 0.0;
      if (q < 3 && p < 3) {
        v = rt[3 * q + p];
      } else if (q >= 3 && p >= 3) {
        v = rt[3 * (q - 3) + (p - 3)];
      } else if (q < 3) {
        const int c = p - 3, q1 = q == 2 ? 0 : q + 1, q2 = q == 0 ? 2 : q - 1;
        v = rt[9 + q1] * rt[3 * q2 + c] - rt[9 + q2] * rt[3 * q1 + c];
      }
      s_ad[jj][e] = v;
    }
  }
  __syncthreads();
  // Phase B: N_j = H_tt,j·Ad_j; the target outputs — H_ht = −AdᵀH_tt, H_tt, g_t — and g_h = −Σ_j Ad_jᵀ g_t,j
  const int nout = SLOT_LIN_BASE + SLOT_LIN_T * n_t;
  for (int o = threadIdx.x; o < nout; o += NT) {
    if (o < 36) {
      const int r = o / 6, c = o - 6 * (o / 6);
      for (int j = 0; j < n_t; ++j) {
        double v = 0.0;
#pragma unroll
        for (int p = 0; p < 6; ++p) v += sT[64 * j + 8 * r + p] * s_ad[j][6 * p + c];
        sN[36 * j + o] = v;
      }
      continue;
    }
    double v = 0.0;
    if (o < 42) {
      const int r = o - 36;
      for (int j = 0; j < n_t; ++j)
#pragma unroll
        for (int q = 0; q < 6; ++q) v -= s_ad[j][6 * q + r] * sT[64 * j + 8 * q + 7];
    } else {
      const int j = (o - 42) / SLOT_LIN_T, q = (o - 42) - SLOT_LIN_T * j;
      if (q < 36) {
        const int r = q / 6, c = q - 6 * (q / 6);
#pragma unroll
        for (int p = 0; p < 6; ++p) v -= s_ad[j][6 * p + r] * sT[64 * j + 8 * p + c];
      } else if (q < 72) {
        const int r = (q - 36) / 6, c = (q - 36) % 6;
        v = sT[64 * j + 8 * r + c];
      } else {
        v = sT[64 * j + 8 * (q - 72) + 7];
      }
    }
    part_lin[(long long)poff + o] = v;
  }
  __syncthreads();
  if (threadIdx.x < 36) {  // Phase C: H_hh[r][c] = Σ_j Σ_q Ad_j[q][r] N_j[q][c], (r, c) and (c, r) from one sum
    const int o = threadIdx.x, r0 = o / 6, c0 = o - 6 * (o / 6), r = min(r0, c0), c = max(r0, c0);
    double v = 0.0;
    for (int j = 0; j < n_t; ++j)
#pragma unroll
      for (int q = 0; q < 6; ++q) v += s_ad[j][6 * q + r] * sN[36 * j + 6 * q + c];
    part_lin[(long long)poff + o] = v;
  }
  if (live && k == 0) {
    a.valid[blk] = (uint8_t)ok;
    a.cost[blk] = bcost;
  }
  if (g.wg_red && wave == 0) {  // the chunk's (Σ cost, Σ valid): lane b takes block b, xor butterflies (fixed order)
    const float x = lane < count ? s_bc[lane] : -1.0f;
    double cs = x >= 0.0f ? (double)x : 0.0, vs = x >= 0.0f ? 1.0 : 0.0;
    for (int m = 32; m >= 1; m >>= 1) {
      cs += __shfl_xor(cs, m, 64);
      vs += __shfl_xor(vs, m, 64);
    }
    if (lane == 0) {
      g.wg_red[2 * chunk] = cs;
      g.wg_red[2 * chunk + 1] = vs;
    }
  }
}


struct SchurArgs {
  const int4* desc;       // first GN point, n points, n local poses, partial offset (doubles)
  const int4* aux;        // pair list offset, n pairs, first GN block, n blocks (the last two: diagnostics)
  const uchar2* pairs;    // (a, b) local pose pairs, a ≤ b
  const int2* pt_fb;       // chunk c's point p → {first GN block, block count} at c · SCHUR_PTS + p (padded table)
  const uint8_t* blk_lv;
  const double* blk_schur;
  const double* blk_schur1;  // buffer set 1 (device LM loop)
  double* part_schur;
  double* pt_data;        // per GN point [H_ρρ, g_ρ, W_h(6)] (undamped)
  int n_chunks;
  const double* lm;       // LM record (λ, set; the loop's or GnData::lm_idle)
  // device LM loop: the previous trial's accept (state ← candidate when the record says accepted), done here by the
  // workgroups before their chunks instead of by a launch of its own; poses == nullptr: nothing to apply
  double* poses;
  const double* poses_new;
  double* rho;
  const double* rho_new;
  const int* pt_orig;
  int n_pose_d, n_gn_points;
  const double* pair_rt;   // per pair [R_th, t_th] of the linearisation in blk_schur / blk_schur1 (W_h = −W_t·Ad)
  const double* pair_rt1;
  const int4* lvp4;        // per chunk: the pairs of local targets 1 … 4
  const int* lvp;          // all of them (from aux.z), for chunks of > 5 local poses
  int rt_off;              // R, t at the start of the dynamic LDS (doubles); W after it
  // free intrinsics (single-GPU LM loop): the previous trial's accept also copies the candidate intrinsics (the copies of
  // intr_accept_kernel, 8 per camera) — k_d == nullptr: not here
  const double* knew_d = nullptr;
  const float* knew_f = nullptr;
  double* k_d = nullptr;
  float* k_f = nullptr;
  int n_intr = 0;
};

// ------------------------------------------------------------------------------------------------
// schur_kernel: point elimination for damping λ
// ------------------------------------------------------------------------------------------------
// One Schur chunk c for damping λ: the points' H_ρρ, g_ρ, W sums from the block data of the linearisation set blk_schur,
// their point data into pt_out (nullptr: not stored), and the chunk's partial slots into part_out.  degen != nullptr (the
// λ-free pass of the device LM loop, λ = 0): set to 1 when a point's H_ρρ lies outside the LM diagonal's clamp [1e-6, 1e32]
// (H = 0 excepted: such a point has W = 0) — only inside it is H + λ·clamp(H) = (1 + λ)·H, the identity the λ-free pass
// relies on (schur_free_decide_kernel).
// A chunk's descriptors and point records: the first loads of its elimination (schur_head), separate so that a kernel
// can issue them in one memory round with loads of its own (schur_free_decide_kernel: the record and the set).
constexpr int kPtIter = (SCHUR_PTS + kBlockThreads / 4 - 1) / (kBlockThreads / 4);
struct SchurHead {
  int4 d, ax, lp4;
  int2 prec[kPtIter];
};
__device__ __forceinline__ SchurHead schur_head(const SchurArgs& g, int c) {
  SchurHead h;
  h.d = g.desc[c];
  h.ax = g.aux[c];
  h.lp4 = g.lvp4[c];
#pragma unroll
  for (int it = 0; it < kPtIter; ++it)
    h.prec[it] = g.pt_fb[(long long)c * SCHUR_PTS + it * (kBlockThreads / 4) + (threadIdx.x >> 2)];
  return h;
}
// The host block of W: a photometric (or geometric) row's host Jacobian is its target Jacobian through the pair's
// adjoint, J_h = −J_t·Ad with Ad = [[R, [t]×R], [0, R]] (R = R_th, t = t_th; linearize_adj_kernel), so
// W_h = J_ρᵀJ_h = −Σ_targets W_t·Ad = −Σ_lv [W_tv·R, (W_tv × t + W_tw)·R] over the point's per-target sums W[p][lv]: the
// blocks carry W_t alone (8 doubles of point data instead of 16).  Point p, all six components (one thread per point:
// per component, the reads of W and R, t were a third of the work); rt: the local targets' [R(9), t(3)] in LDS.
__device__ __forceinline__ void host_w(const double (*W)[6], const double* rt, int p, int nv, double* out) {
  double v[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int l = 1; l < nv; ++l) {
    const double2* w2 = reinterpret_cast<const double2*>(W[p * nv + l]);
    const double2* r2 = reinterpret_cast<const double2*>(rt + 12 * (l - 1));
    double w[6], R[12];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double2 x = w2[i];
      w[2 * i] = x.x;
      w[2 * i + 1] = x.y;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double2 x = r2[i];
      R[2 * i] = x.x;
      R[2 * i + 1] = x.y;
    }
    const double* t = R + 9;
    const double u0 = w[1] * t[2] - w[2] * t[1] + w[3], u1 = w[2] * t[0] - w[0] * t[2] + w[4],
                 u2 = w[0] * t[1] - w[1] * t[0] + w[5];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      v[c] += w[0] * R[c] + w[1] * R[3 + c] + w[2] * R[6 + c];
      v[3 + c] += u0 * R[c] + u1 * R[3 + c] + u2 * R[6 + c];
    }
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) out[c] = -v[c];
}
__device__ __forceinline__ void schur_chunk(const SchurArgs& g, const SchurHead& h, double lambda,
                                            const double* __restrict__ blk_schur, const double* __restrict__ pair_rt,
                                            double* __restrict__ part_out, double* __restrict__ pt_out, int* degen,
                                            double* W_dyn, double* s_inv, double* s_gl) {
  const int4 d = h.d;
  const int4 ax = h.ax;
  const int2* prec = h.prec;
  const int first = d.x, npt = d.y, nv = d.z, poff = d.w;
#ifdef PBA_FD_STAMPS
  const long long ts0 = wall_clock64();
  long long ts1 = 0, ts2 = 0, tsa = 0, tsb = 0, tsc = 0;
  auto stamp_out = [&](const char* tag) {
    const int b = blockIdx.x;
    if (threadIdx.x == 0 && (b == 17 || b == 300 || b == 600 || b == 1000))
      printf("fdphase b=%d %s zero %lld acc %lld presync %lld sync %lld wh %lld total %lld\n", b, tag, ts1 - ts0,
             tsa - ts0, tsb - ts0, tsc - ts0, ts2 - ts0, wall_clock64() - ts0);
  };
#endif
  double* const rt = W_dyn;  // the local targets' R_th, t_th (12 each)
  double (*W)[6] = reinterpret_cast<double (*)[6]>(W_dyn + g.rt_off);
  for (int i = threadIdx.x; i < npt * nv * 6; i += kBlockThreads) (&W[0][0])[i] = 0.0;
  __syncthreads();
#ifdef PBA_FD_STAMPS
  ts1 = wall_clock64();
#endif
  // the targets' R, t: loaded beside the block data (the first four pairs came with the descriptors; a chunk of more
  // local poses reads its pair list first), stored to LDS after the accumulation
  double rtv[2];
  int rti[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + u * kBlockThreads, l = i / 12;
    rti[u] = i < 12 * (nv - 1) ? i : -1;
    int pr = 0;
    if (rti[u] >= 0) pr = l < 4 ? (l == 0 ? h.lp4.x : l == 1 ? h.lp4.y : l == 2 ? h.lp4.z : h.lp4.w) : g.lvp[ax.z + l];
    rtv[u] = rti[u] >= 0 ? pair_rt[(long long)pr * 12 + (i - 12 * l)] : 0.0;
  }
  // four lanes per point, each summing one 16-B load per block of the point's blocks' 8-value records in block order:
  // q = 0: H_ρρ, g_ρ   q = 1, 2, 3: W_t[0..1], [2..3], [4..5] → W[p][lv] (staging the chunk's records in LDS
  // block-parallel instead measured slower: 23 → 35 µs at C4, its LDS halves the resident workgroups)
  bool bad = false;
  const int q = threadIdx.x & 3;
  // the first kFirst blocks of both of the lane's points in ONE memory round (a point's block loop per point cost a
  // round each), the rest of a point's blocks (more than kFirst observations) in batches after
  constexpr int kFirst = 4, kBatch = 8;
  double2 v0[kPtIter][kFirst];
  int lv0[kPtIter][kFirst];
#pragma unroll
  for (int it = 0; it < kPtIter; ++it) {
    const int fb = prec[it].x, nb = max(prec[it].y, 1);
#pragma unroll
    for (int u = 0; u < kFirst; ++u) {
      const int b = fb + min(u, nb - 1);
      v0[it][u] = reinterpret_cast<const double2*>(blk_schur + (long long)b * kPd)[q];
      lv0[it][u] = q == 0 ? 0 : g.blk_lv[b];
    }
  }
#ifdef PBA_FD_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tsa = wall_clock64();
#endif
#pragma unroll
  for (int it = 0; it < kPtIter; ++it) {
    const int p = it * (kBlockThreads / 4) + (threadIdx.x >> 2), gp = first + p;
    if (p < npt) {
      const int fb = prec[it].x, nb = prec[it].y;
      double s0 = 0.0, s1 = 0.0;
      auto add = [&](const double2& v, int lv) {
        if (q == 0) {
          s0 += v.x;
          s1 += v.y;
        } else {
          double* wt = W[p * nv + lv] + 2 * (q - 1);
          wt[0] += v.x;
          wt[1] += v.y;
        }
      };
#pragma unroll
      for (int u = 0; u < kFirst; ++u)
        if (u < nb) add(v0[it][u], lv0[it][u]);
      for (int b0 = fb + kFirst; b0 < fb + nb; b0 += kBatch) {
        double2 v[kBatch];
        int lv[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
          const int b = min(b0 + u, fb + nb - 1);
          v[u] = reinterpret_cast<const double2*>(blk_schur + (long long)b * kPd)[q];
          lv[u] = q == 0 ? 0 : g.blk_lv[b];
        }
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
          if (b0 + u < fb + nb) add(v[u], lv[u]);
      }
      if (q == 0) {
        const double D = fmin(fmax(s0, 1e-6), 1e32);
        const double Hd = s0 + lambda * D;
        s_inv[p] = Hd > 0.0 ? 1.0 / Hd : 0.0;
        s_gl[p] = s1;
        bad = s0 != 0.0 && !(s0 >= 1e-6 && s0 <= 1e32);
        if (pt_out) {
          pt_out[(long long)gp * 8] = s0;
          pt_out[(long long)gp * 8 + 1] = s1;
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (rti[u] >= 0) rt[rti[u]] = rtv[u];
  for (int i = threadIdx.x + 2 * kBlockThreads; i < 12 * (nv - 1); i += kBlockThreads)  // (> 43 local poses)
    rt[i] = pair_rt[(long long)g.lvp[ax.z + i / 12] * 12 + i % 12];
#ifdef PBA_FD_STAMPS
  tsb = wall_clock64();
#endif
  if (degen && __syncthreads_or(bad) && threadIdx.x == 0) atomicOr(degen, 1);
  __syncthreads();
#ifdef PBA_FD_STAMPS
  tsc = wall_clock64();
#endif
  for (int p = threadIdx.x; p < npt; p += kBlockThreads) {  // W_h = W[p][0] from the targets' sums
    double v[6];
    host_w(W, rt, p, nv, v);
#pragma unroll
    for (int c = 0; c < 6; ++c) W[p * nv][c] = v[c];
    if (pt_out)
#pragma unroll
      for (int c = 0; c < 6; ++c) pt_out[(long long)(first + p) * 8 + 2 + c] = v[c];
  }
  __syncthreads();
#ifdef PBA_FD_STAMPS
  ts2 = wall_clock64();
#endif
  if (nv * 6 + 1 <= 32) {
    // ≤ 5 local poses (a temporal window): the chunk's sums are one small GEMM on the matrix cores,
    // C = (W·diag(1/H'_ρρ))ᵀ [W | g_ρ] over its points (K = points, 4 per v_mfma_f64_16x16x4f64 step), 32 × 32 in
    // four 16 × 16 tiles, one per wave; C's 6 × 6 blocks (a, b) of the used pose pairs and its column nv·6 (the
    // gradient terms) are the partial slots.  Layouts as in cr_level_wave_kernel: A lane l = (row l%16, k l/16),
    // B lane l = (k l/16, column l%16), accumulator entry v of lane l = (row l/16 + 4v, column l%16).
    const int nv6 = nv * 6;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ti = wv & 1, tj = wv >> 1;
    const int ca = 16 * ti + (lane & 15), cb = 16 * tj + (lane & 15), kq = lane >> 4;
    const double* Wf = &W[0][0];
    v4f64 acc = {0.0, 0.0, 0.0, 0.0};
    // four K steps per batch: the batch's LDS reads first, at clamped indices with unconditional reads, the padding
    // zeroed by selects afterwards (conditional reads were issued and waited one step at a time)
    constexpr int KB = 4;
    const int cac = min(ca, nv6 - 1), cbc = min(cb, nv6 - 1);
    for (int p0 = 0; p0 < npt; p0 += 4 * KB) {
      double wa[KB], wb[KB], si[KB], sg[KB];
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        const int pc = min(p0 + 4 * u + kq, npt - 1);
        wa[u] = Wf[pc * nv6 + cac];
        wb[u] = Wf[pc * nv6 + cbc];
        si[u] = s_inv[pc];
        sg[u] = s_gl[pc];
      }
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        const bool pin = p0 + 4 * u + kq < npt;
        const double av = (pin && ca < nv6) ? wa[u] * si[u] : 0.0;
        const double bv = !pin ? 0.0 : (cb < nv6 ? wb[u] : (cb == nv6 ? sg[u] : 0.0));
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int r = 16 * ti + (lane >> 4) + 4 * v;
      if (r >= nv6) continue;
      if (cb < nv6) {
        // canonical pair order (gn_prepare): (0,0) (0,1) … (0,nv−1) (1,1) …; blocks of unused pairs are zero
        const int pa_ = r / 6, pb_ = cb / 6;
        const int u = pa_ * nv - pa_ * (pa_ - 1) / 2 + (pb_ - pa_);
        if (pa_ <= pb_) part_out[(long long)poff + u * 36 + (r % 6) * 6 + cb % 6] = acc[v];
      } else if (cb == nv6) {
        part_out[(long long)poff + ax.y * 36 + r] = acc[v];
      }
    }
#ifdef PBA_FD_STAMPS
    stamp_out("mfma");
#endif
    return;
  }
  const int nout = ax.y * 36 + nv * 6;
  for (int o = threadIdx.x; o < nout; o += kBlockThreads) {
    double acc = 0.0;
    if (o < ax.y * 36) {
      const uchar2 ab = g.pairs[ax.x + o / 36];
      const int r = (o % 36) / 6, cc = o % 6;
      for (int p = 0; p < npt; ++p)
        acc += W[p * nv + ab.x][r] * W[p * nv + ab.y][cc] * s_inv[p];
    } else {
      const int q = o - ax.y * 36, a = q / 6, r = q % 6;
      for (int p = 0; p < npt; ++p) acc += W[p * nv + a][r] * s_gl[p] * s_inv[p];
    }
    part_out[(long long)poff + o] = acc;
  }
}

// The accept of the device LM loop's previous trial (state ← candidate when the record says accepted; the copies of
// lm_accept_kernel): one element per thread, a grid-stride tail beyond the grid.  Loads first (with the kernel's first
// loads), stores after the kernel's own stores (loads and stores share vmcnt).
struct AcceptCopy {
  bool accepted = false;
  int ia = 0, oa = 0, ka = 0;
  double pnew = 0.0, rnew = 0.0, kdnew = 0.0;
  float kfnew = 0.0f;
  __device__ __forceinline__ void load(const SchurArgs& g, const LmView& lv) {
    accepted = g.poses && lv.accept != 0.0 && lv.done == 0.0;
    ia = blockIdx.x * blockDim.x + threadIdx.x;
    if (g.poses) {
      pnew = g.poses_new[min(ia, g.n_pose_d - 1)];
      oa = g.pt_orig[min(ia, g.n_gn_points - 1)];
      rnew = g.rho_new[oa];
    }
    if (g.k_d && ia < 8 * g.n_intr) {
      ka = kCamD * (ia >> 3) + (ia & 7);
      kdnew = g.knew_d[ka];
      kfnew = g.knew_f[ia];
    }
  }
  __device__ __forceinline__ void store(const SchurArgs& g) const {
    if (!accepted) return;
    if (ia < g.n_pose_d) g.poses[ia] = pnew;
    if (ia < g.n_gn_points) g.rho[oa] = rnew;
    if (g.k_d && ia < 8 * g.n_intr) {
      g.k_d[ka] = kdnew;
      g.k_f[ia] = kfnew;
    }
    const int n = max(g.n_pose_d, g.n_gn_points);
    for (int i = ia + gridDim.x * blockDim.x; i < n; i += gridDim.x * blockDim.x) {
      if (i < g.n_pose_d) g.poses[i] = g.poses_new[i];
      if (i < g.n_gn_points) {
        const int o = g.pt_orig[i];
        g.rho[o] = g.rho_new[o];
      }
    }
  }
};

// Point elimination for damping λ (host-driven steps, the multi-GPU loop, free intrinsics): one chunk per workgroup, the
// linearisation set of the record, plus the previous trial's accept when g.poses is set.
__global__ __launch_bounds__(kBlockThreads) void schur_kernel(const SchurArgs g, double lambda) {
  extern __shared__ __attribute__((aligned(16))) double W_dyn[];  // W [points × local poses][6] (gn_prepare: schur_lds)
  __shared__ double s_inv[SCHUR_PTS], s_gl[SCHUR_PTS];
  const int c = blockIdx.x;
  if (c >= g.n_chunks) return;  // (not gated by the record's done flag: a trial after the end only wastes time here)
  // Memory rounds (each dependent one is ~1.7 µs here): 1 — the record, the chunk descriptors, the chunk's point
  // records (padded per-chunk table) and the accept copy's sources; 2 — the points' block data (and the copied ρ);
  // the accept copy's stores come last, so no load of the chunk waits behind them (loads and stores share vmcnt).
  const LmView lv = lm_view(g.lm);
  AcceptCopy ac;
  ac.load(g, lv);
  lambda = lm_lambda(lv, lambda);
  const double* const blk_schur = lv.set != 0.0 ? g.blk_schur1 : g.blk_schur;
  schur_chunk(g, schur_head(g, c), lambda, blk_schur, lv.set != 0.0 ? g.pair_rt1 : g.pair_rt, g.part_schur, g.pt_data,
              nullptr, W_dyn, s_inv, s_gl);
  ac.store(g);
}

struct AsmArgs {
  const double* part_lin;
  const double* part_lin1;  // buffer set 1 (device LM loop)
  const double* lm;        // LM record (λ, set; the loop's or GnData::lm_idle)
  const double* part_schur;
  const int* sky_cptr;
  const int2* sky_contrib;
  const int* g_cptr;
  const int2* g_contrib;
  const int* blk_i;
  const int* blk_j;
  const uint8_t* fixed;
  double* S;
  double* g;
  double* g_dir;
  double* Ddiag;
  double* Sband;   // optional dense band copy (block c of row i = column i − B + c), B = band
  int band;
  int n_sky;
  int n_frames;
  // optional: level 0 of the block cyclic reduction written directly (super-rows of crB keyframes: D, U, b = −g; the
  // positions outside the profile and the identity padding set once by configure_solver), which replaces cr_build's
  // pass over Sband; status (the solve's failure flag) is then cleared here
  double* crD;
  double* crU;
  double* crb;
  int crB;
  int* status;
  // the single-GPU LM loop: the current set's λ-free Schur partials (scaled by 1/(1 + λ)) unless the set is flagged
  // degen (schur_free_decide_kernel); nullptr: part_schur as it is
  const double* part_free0;
  const double* part_free1;
  const int* degen;
  const int* sky_diag;  // assemble_kernel: the diagonal blocks (long contribution lists: kAsmSeg lanes per element) …
  const int* sky_off;   // … and the off-diagonal ones (one lane)
  int n_diag;
};

// Fixed-order sums over a contribution list (total, and the part that is not a Schur term — the undamped
// JᵀJ diagonal / direct gradient).  The list entries and their values are gathered 8 at a time so eight
// independent loads are in flight per lane instead of one dependent index → value chain per term.  (16 at a time with
// the next batch's entries loaded beside the current batch's values measured slower: 12.8 → 15.0 µs at C4, 128
// VGPRs and twice the clamped loads of the short off-diagonal lists.)
constexpr int GATHER = 8;
// seg / nseg: this lane's share of the list, entries beg + seg, beg + seg + nseg, … (the caller adds the nseg lanes'
// sums in a fixed order).
__device__ __forceinline__ void contrib_sums(const AsmArgs& a, const int2* __restrict__ list, int beg, int end, int e,
                                             int et, double& sum, double& dsum, double pscale = 1.0, int seg = 0,
                                             int nseg = 1) {
  sum = dsum = 0.0;
  for (int q0 = beg + seg; q0 < end; q0 += GATHER * nseg) {
    int2 c[GATHER];
    double v[GATHER];
#pragma unroll
    for (int u = 0; u < GATHER; ++u) c[u] = list[min(q0 + u * nseg, end - 1)];
#pragma unroll
    for (int u = 0; u < GATHER; ++u) {
      // both loads unconditional (the other one at a valid dummy offset): no divergent branch, no wait
      const int off = c[u].x + ((c[u].y & C_TRANSPOSE) ? et : e);
      const bool sc = (c[u].y & C_SCHUR) != 0;
      const double vs = a.part_schur[sc ? off : 0];
      const double vl = a.part_lin[sc ? 0 : off];
      v[u] = sc ? -pscale * vs : vl;
    }
#pragma unroll
    for (int u = 0; u < GATHER; ++u) {
      if (q0 + u * nseg < end) {
        sum += v[u];
        if (!(c[u].y & C_SCHUR)) dsum += v[u];
      }
    }
  }
}
// The kAsmSeg lanes of one element (aligned groups) add their list shares: lane 0 of the group gets the total, in a
// fixed order.
constexpr int kAsmSeg = 4;
__device__ __forceinline__ void seg_total(double& sum, double& dsum) {
#pragma unroll
  for (int m = 1; m < kAsmSeg; m <<= 1) {
    sum += __shfl_xor(sum, m, 64);
    dsum += __shfl_xor(dsum, m, 64);
  }
}

// ------------------------------------------------------------------------------------------------
// assemble_kernel: S (skyline, lower blocks) and g from the partial slots
// ------------------------------------------------------------------------------------------------
__global__ void assemble_kernel(AsmArgs a, double lambda) {
  const LmView lv = lm_view(a.lm);  // (no done gate: see schur_kernel)
  const int dg0 = a.degen ? a.degen[0] : 1, dg1 = a.degen ? a.degen[1] : 1;
  lambda = lm_lambda(lv, lambda);
  if (lv.set != 0.0) a.part_lin = a.part_lin1;
  double pscale = 1.0;  // the λ-free partials of the current set: P / (1 + λ)
  if (a.degen && (lv.set != 0.0 ? dg1 : dg0) == 0) {
    a.part_schur = lv.set != 0.0 ? a.part_free1 : a.part_free0;
    pscale = 1.0 / (1.0 + lambda);
  }
  // thread ranges: the diagonal blocks' elements, kAsmSeg lanes each (their lists are the long ones: every chunk hosted
  // by or targeting the keyframe, ~30 partials at C4, four dependent memory rounds on one lane), then the off-diagonal
  // blocks' elements one lane each, then the gradient rows kAsmSeg lanes each
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int nA = a.n_diag * 36 * kAsmSeg, nS = nA + (a.n_sky - a.n_diag) * 36;
  if (tid < nS) {
    const bool dg = tid < nA;
    const int w = dg ? tid / kAsmSeg : tid - nA, seg = dg ? tid % kAsmSeg : 0;
    const int s = dg ? a.sky_diag[w / 36] : a.sky_off[w / 36], e = w % 36, r = e / 6, cc = e % 6;
    const int i = a.blk_i[s], j = a.blk_j[s];
    double sum, dsum;
    contrib_sums(a, a.sky_contrib, a.sky_cptr[s], a.sky_cptr[s + 1], r * 6 + cc, cc * 6 + r, sum, dsum, pscale, seg,
                 dg ? kAsmSeg : 1);
    if (dg) {
      seg_total(sum, dsum);
      if (seg != 0) return;
    }
    const int tid_s = s * 36 + e;  // the element's position in S
    double val = sum;
    if (a.fixed[i] || a.fixed[j]) {
      val = (i == j && r == cc) ? 1.0 : 0.0;
    } else if (i == j && r == cc) {
      const double D = fmin(fmax(dsum, 1e-6), 1e32);  // levenberg_marquardt_strategy.cc min/max diagonal
      a.Ddiag[6 * i + r] = D;
      val = sum + lambda * D;
    }
    a.S[tid_s] = val;
    if (a.Sband) a.Sband[(long long)i * ((a.band + 1) * 36 + 6) + (j - i + a.band) * 36 + e] = val;
    if (a.crD) {
      const int B = a.crB, M = 6 * B, I = i / B, J = j / B;
      const int Ri = (i % B) * 6 + r, Cj = (j % B) * 6 + cc;  // row of i's entry / column of j's in their super-rows
      if (I == J) {
        // a diagonal block's (r, cc) and (cc, r) are two lanes whose sums may differ in the last bit (the Schur
        // terms' products round differently): only the lower one writes both, so D is symmetric and the solve
        // reproducible (both lanes writing both positions left whichever stored last)
        double* D = a.crD + (long long)I * M * M;
        if (i != j || r >= cc) {
          D[Ri * M + Cj] = val;
          D[Cj * M + Ri] = val;
        }
      } else {  // I == J + 1 (bandwidth ≤ B): U_J[row of j][column of i] = S[6j+cc][6i+r]
        a.crU[(long long)J * M * M + Cj * M + Ri] = val;
      }
    }
    return;
  }
  const int tg = tid - nS, t = tg / kAsmSeg, seg = tg % kAsmSeg;
  if (t >= 6 * a.n_frames) return;
  const int i = t / 6, r = t % 6;
  double sum, dsum;
  contrib_sums(a, a.g_contrib, a.g_cptr[i], a.g_cptr[i + 1], r, r, sum, dsum, pscale, seg, kAsmSeg);
  seg_total(sum, dsum);
  if (seg != 0) return;
  a.g[t] = a.fixed[i] ? 0.0 : sum;
  if (a.Sband) a.Sband[(long long)i * ((a.band + 1) * 36 + 6) + (a.band + 1) * 36 + r] = a.fixed[i] ? 0.0 : sum;
  if (a.crD) {
    a.crb[t] = a.fixed[i] ? 0.0 : -sum;  // super-row i / B, row (i % B)·6 + r: t itself (M = 6B, rows padded after N)
    if (t == 0) *a.status = 0;
  }
  a.g_dir[t] = a.fixed[i] ? 0.0 : dsum;
  if (a.fixed[i]) a.Ddiag[t] = 0.0;
}

// ------------------------------------------------------------------------------------------------
// Multi-GPU exchange (include/pba.h): this rank's partial reduced system in the banded exchange layout,
// and the finalisation of the summed system into the band solvers' input.
// ------------------------------------------------------------------------------------------------
constexpr int EX_TAIL = 24;  // g(6) | g_direct(6) | diag(A)(6) | observed | pad
__host__ __device__ constexpr long long ex_row(int K) { return (long long)(K + 1) * 36 + EX_TAIL; }

// One lane per element of the exchange buffer (the local skyline's elements by the contribution lists of
// assemble_kernel, nothing damped or fixed; the pose gradients): positions outside the local profile get their zero here, so the
// buffer needs no fill launch before it (round 3: a 5-µs hipMemsetAsync of the whole band per trial).
__global__ void export_band_kernel(AsmArgs a, const uint8_t* __restrict__ observed, const int* __restrict__ sky_first,
                                   const int* __restrict__ sky_row, double* __restrict__ X, int K) {
  if (lm_view(a.lm).set != 0.0) a.part_lin = a.part_lin1;  // (no done gate: see schur_kernel)
  // lanes [0, nf·(K+1)·36): the band elements; then 24 per frame for the tails, in waves of their own (the gradient lists
  // are long: interleaved with the band's short lists they made every wave wait for them, 12 → 21 µs at C4)
  const long long RS = ex_row(K), t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int QB = (K + 1) * 36;
  const long long nB = (long long)a.n_frames * QB;
  if (t < nB) {
    const int i = (int)(t / QB), q = (int)(t - (long long)i * QB);
    const int c = q / 36, e = q % 36, r = e / 6, cc = e % 6, j = i - K + c;
    double sum = 0.0, dsum = 0.0;
    if (j >= 0 && j >= sky_first[i]) {
      const int s = sky_row[i] + (j - sky_first[i]);
      contrib_sums(a, a.sky_contrib, a.sky_cptr[s], a.sky_cptr[s + 1], r * 6 + cc, cc * 6 + r, sum, dsum);
    }
    double* row = X + (long long)i * RS;
    row[q] = sum;
    if (i == j && r == cc) row[QB + 12 + r] = dsum;  // diag(A)
    return;
  }
  const long long u = t - nB;
  if (u >= (long long)a.n_frames * EX_TAIL) return;
  const int i = (int)(u / EX_TAIL), r = (int)(u % EX_TAIL);
  double* tail = X + (long long)i * RS + QB;
  if (r < 6) {  // g and the direct gradient from one list walk
    double sum, dsum;
    contrib_sums(a, a.g_contrib, a.g_cptr[i], a.g_cptr[i + 1], r, r, sum, dsum);
    tail[r] = sum;
    tail[6 + r] = dsum;
  } else if (r >= 18) {
    tail[r] = r == 18 && observed[i] ? 1.0 : 0.0;
  }
}

struct ImportArgs {
  const double* X;         // summed exchange buffer
  const uint8_t* fixed_req;
  double* Sband;           // band solver input, row stride (K+1)·36 + 6
  double* g;
  double* g_dir;
  double* Ddiag;
  uint8_t* fixed;          // effective constant frames: requested, or observed by no rank
  int n_frames;
  int K;
  // block cyclic reduction: level 0 written directly (super-rows of K keyframes; as assemble_kernel), else Sband
  double* crD;
  double* crU;
  double* crb;
  int* status;
};

// One lane per element of the band solver input: + λ·clamp(diag(A)) (levenberg_marquardt_strategy.cc),
// identity rows/columns for constant frames — the same arithmetic as assemble_kernel on the summed system.
__global__ void import_kernel(const ImportArgs a, double lambda, const double* __restrict__ lm) {
  lambda = lm_lambda(lm_view(lm), lambda);  // the device LM record's λ (host-driven steps: the argument)
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int K = a.K;
  const long long SR = (long long)(K + 1) * 36 + 6, RS = ex_row(K);
  if (t >= SR * a.n_frames) return;
  const int i = (int)(t / SR), q = (int)(t - (long long)i * SR);
  const double* row = a.X + (long long)i * RS;
  const double* tail = row + (K + 1) * 36;
  const bool fi = a.fixed_req[i] || tail[18] == 0.0;
  if (q < (K + 1) * 36) {
    const int c = q / 36, e = q % 36, r = e / 6, cc = e % 6, j = i - K + c;
    double val = 0.0;
    if (j >= 0) {
      const bool fj = a.fixed_req[j] || a.X[(long long)j * RS + (K + 1) * 36 + 18] == 0.0;
      val = row[q];
      if (fi || fj) {
        val = (i == j && r == cc) ? 1.0 : 0.0;
      } else if (i == j && r == cc) {
        val += lambda * fmin(fmax(tail[12 + r], 1e-6), 1e32);
      }
    }
    if (!a.crD) {
      a.Sband[t] = val;
    } else if (j >= 0) {  // the (i, j) entry into level 0 (I = i / K, J = j / K, I − J ≤ 1), as assemble_kernel
      const int M = 6 * K, I = i / K, J = j / K, Ri = (i % K) * 6 + r, Cj = (j % K) * 6 + cc;
      if (I == J) {
        if (i != j || r >= cc) {  // the lower lane writes both positions (a symmetric D, reproducible)
          double* D = a.crD + (long long)I * M * M;
          D[Ri * M + Cj] = val;
          D[Cj * M + Ri] = val;
        }
      } else {
        a.crU[(long long)J * M * M + Cj * M + Ri] = val;
      }
    }
    return;
  }
  const int r = q - (K + 1) * 36;
  if (!a.crD) a.Sband[t] = fi ? 0.0 : tail[r];
  else a.crb[6 * i + r] = fi ? 0.0 : -tail[r];
  if (a.crD && t == (K + 1) * 36) *a.status = 0;  // the solve's failure flag (cr_build_kernel clears it otherwise)
  a.g[6 * i + r] = fi ? 0.0 : tail[r];
  a.g_dir[6 * i + r] = fi ? 0.0 : tail[6 + r];
  a.Ddiag[6 * i + r] = fi ? 0.0 : fmin(fmax(tail[12 + r], 1e-6), 1e32);
  if (r == 0) a.fixed[i] = fi ? 1 : 0;
}

// Free intrinsics on several GPUs: the summed exchange — the keyframes' band rows and the 2·nc border rows (the
// border region after the band, export by intr_border_all_kernel) — into the skyline system of the summed profile
// (keyframe i: columns max(0, i − K) … i; border rows: 0 … P; row offsets `row`), with the single-GPU arithmetic of
// assemble_kernel and border_store: + λ·clamp(diag(A)), identity rows / columns for constant frames (requested, or
// observed by no rank — cameras: seen by no rank), the intrinsics pads (1 + λ on the diagonal, LM diagonal 1).  One lane
// per element, then six per frame for g, the direct gradient, the LM diagonal and the effective constant flag.
struct ImportSkyArgs {
  const double* X;          // summed exchange buffer: band rows
  const double* Xb;         // … its border region
  const uint8_t* fixed_req;
  const int* row;           // skyline row offsets of the summed profile (nfs + 1)
  double* S;
  double* g;
  double* g_dir;
  double* Ddiag;
  uint8_t* fixed;           // effective constant frames (nfs)
  int nf, nc, K;
  long long n_el;           // skyline elements (36 per block)
};
__device__ __forceinline__ bool import_fixed(const ImportSkyArgs& a, int i) {
  const int nfs = a.nf + 2 * a.nc;
  if (i < a.nf) return a.fixed_req[i] || a.X[(long long)i * ex_row(a.K) + (a.K + 1) * 36 + 18] == 0.0;
  return a.Xb[(long long)(i - a.nf) * ((long long)nfs * 36 + EX_TAIL) + (long long)nfs * 36 + 18] == 0.0;
}
__global__ void import_sky_kernel(const ImportSkyArgs a, double lambda, const double* __restrict__ lm) {
  lambda = lm_lambda(lm_view(lm), lambda);
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nfs = a.nf + 2 * a.nc, K = a.K;
  const long long RS = ex_row(K), BRS = (long long)nfs * 36 + EX_TAIL;
  auto tail_of = [&](int i) {
    return i < a.nf ? a.X + (long long)i * RS + (K + 1) * 36 : a.Xb + (long long)(i - a.nf) * BRS + (long long)nfs * 36;
  };
  if (t < a.n_el) {
    const int blk = (int)(t / 36), e = (int)(t % 36), r = e / 6, cc = e % 6;
    int lo = 0, hi = nfs;  // the row i with row[i] ≤ blk < row[i + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (a.row[mid] <= blk) lo = mid;
      else hi = mid;
    }
    const int i = lo, j = (i < a.nf ? max(0, i - K) : 0) + (blk - a.row[i]);
    double val;
    bool pad = false;
    if (i < a.nf) {
      val = a.X[(long long)i * RS + (j - i + K) * 36 + e];
    } else {
      const int p = i - a.nf, d = 6 * (p & 1) + r, d2 = j >= a.nf ? 6 * ((j - a.nf) & 1) + cc : cc;
      pad = d >= 8 || d2 >= 8;
      val = a.Xb[(long long)p * BRS + (long long)j * 36 + e];
    }
    if (import_fixed(a, i) || import_fixed(a, j)) {
      val = (i == j && r == cc) ? 1.0 : 0.0;
    } else if (pad) {
      val = (i == j && r == cc) ? 1.0 + lambda : 0.0;  // border_store: direct 1, LM diagonal 1
    } else if (i == j && r == cc) {
      val += lambda * fmin(fmax(tail_of(i)[12 + r], 1e-6), 1e32);
    }
    a.S[t] = val;
    return;
  }
  const long long u = t - a.n_el;
  if (u >= 6LL * nfs) return;
  const int i = (int)(u / 6), r = (int)(u % 6);
  const double* tail = tail_of(i);
  const bool fi = import_fixed(a, i), pad = i >= a.nf && ((i - a.nf) & 1) && r >= 2;
  a.g[u] = fi || pad ? 0.0 : tail[r];
  a.g_dir[u] = fi || pad ? 0.0 : tail[6 + r];
  a.Ddiag[u] = fi ? 0.0 : (pad ? 1.0 : fmin(fmax(tail[12 + r], 1e-6), 1e32));
  if (r == 0) a.fixed[i] = fi ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------
// skyline_solve_kernel: S δ = −g, S = LLᵀ in place (block skyline, right-looking), one workgroup
// ------------------------------------------------------------------------------------------------
// chol6 / inv_lower6: the 6×6 diagonal block's Cholesky factor and its inverse, on register arrays (fully unrolled)
__device__ __forceinline__ bool chol6_reg(const double (&A)[36], double (&L)[36]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 36; ++i) L[i] = 0.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double s = A[j * 6 + j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[j * 6 + k] * L[j * 6 + k];
    ok = ok && s > 0.0;
    const double ljj = sqrt(fmax(s, 1e-300));
    L[j * 6 + j] = ljj;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double t = A[i * 6 + j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[i * 6 + k] * L[j * 6 + k];
      L[i * 6 + j] = t / ljj;
    }
  }
  return ok;
}
__device__ __forceinline__ void inv_lower6_reg(const double (&L)[36], double (&Li)[36]) {
#pragma unroll
  for (int i = 0; i < 36; ++i) Li[i] = 0.0;
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    Li[c * 6 + c] = 1.0 / L[c * 6 + c];
#pragma unroll
    for (int r = c + 1; r < 6; ++r) {
      double s = 0.0;
#pragma unroll
      for (int k = c; k < r; ++k) s += L[r * 6 + k] * Li[k * 6 + c];
      Li[r * 6 + c] = -s / L[r * 6 + r];
    }
  }
}

struct SolveArgs {
  double* S;
  const int* first;
  const int* row;
  const int* last;
  const double* g;
  double* Linv;
  double* x;
  int* status;
  int N;
  const int* cptr;   // column k's profile rows crows[cptr[k] … cptr[k+1]) (every i > k with first(i) ≤ k, in order)
  const int* crows;
};

__device__ __forceinline__ long long sky_off(const SolveArgs& a, int i, int j) {  // block (i, j), j ≥ first(i)
  return ((long long)a.row[i] + (j - a.first[i])) * 36;
}

__global__ __launch_bounds__(256) void skyline_solve_kernel(const SolveArgs a) {
  __shared__ double sA[36], sL[36], sLi[36];
  __shared__ int s_fail;
  const int tid = threadIdx.x;
  if (tid == 0) s_fail = 0;
  for (int k = 0; k < a.N; ++k) {
    const long long okk = sky_off(a, k, k);
    if (tid < 36) sA[tid] = a.S[okk + tid];
    __syncthreads();
    if (tid == 0) {  // in registers: the LDS-pointer forms' dependent LDS round trips were most of a column's time
      double A[36], L[36], Li[36];
#pragma unroll
      for (int q = 0; q < 36; ++q) A[q] = sA[q];
      if (!chol6_reg(A, L)) {
        s_fail = k + 1;
      } else {
        inv_lower6_reg(L, Li);
#pragma unroll
        for (int q = 0; q < 36; ++q) {
          sL[q] = L[q];
          sLi[q] = Li[q];
        }
      }
    }
    __syncthreads();
    if (s_fail) {
      if (tid == 0) *a.status = s_fail;
      return;
    }
    if (tid < 36) {
      a.S[okk + tid] = sL[tid];
      a.Linv[(long long)k * 36 + tid] = sLi[tid];
    }
    // column k's profile rows: the band below the diagonal and, with free intrinsics, the dense border rows — walking
    // (k, last(k)] instead enumerated every row pair up to the border, O(N²) per column (C3 with free intrinsics: 0.7 s
    // per solve)
    const int c0 = a.cptr[k], na = a.cptr[k + 1] - c0;
    const int* rows = a.crows + c0;
    // column panel L_ik = A_ik · L_kk⁻ᵀ, 7 blocks per pass (read all, barrier, write)
    for (int i0 = 0; i0 < na; i0 += 7) {
      double val = 0.0;
      long long dst = -1;
      const int li = i0 + tid / 36;
      if (tid < 252 && li < na) {
        const int i = rows[li], e = tid % 36, r = e / 6, c = e % 6;
        const long long o = sky_off(a, i, k);
        for (int m = 0; m <= c; ++m) val += a.S[o + r * 6 + m] * sLi[c * 6 + m];
        dst = o + e;
      }
      __syncthreads();
      if (dst >= 0) a.S[dst] = val;
      __threadfence_block();
      __syncthreads();
    }
    // trailing update A_ij −= L_ik L_jkᵀ over the pairs of the column's rows (i ≥ j)
    const int npairs = na * (na + 1) / 2;
    for (int idx = tid; idx < npairs * 36; idx += 256) {
      const int pidx = idx / 36, e = idx % 36, r = e / 6, c = e % 6;
      int ii = 0;  // decode lower-triangular pair index → (ii ≥ jj)
      while ((ii + 1) * (ii + 2) / 2 <= pidx) ++ii;
      const int jj = pidx - ii * (ii + 1) / 2;
      const int i = rows[ii], j = rows[jj];
      const long long oi = sky_off(a, i, k), oj = sky_off(a, j, k);
      double s = 0.0;
      for (int m = 0; m < 6; ++m) s += a.S[oi + r * 6 + m] * a.S[oj + c * 6 + m];
      a.S[sky_off(a, i, j) + e] -= s;
    }
    __threadfence_block();
    __syncthreads();
  }
  // forward substitution L y = −g (y in x)
  for (int t = tid; t < 6 * a.N; t += 256) a.x[t] = -a.g[t];
  __threadfence_block();
  __syncthreads();
  for (int k = 0; k < a.N; ++k) {
    __shared__ double yk[6];
    if (tid < 6) {
      double s = 0.0;
      for (int m = 0; m <= tid; ++m) s += a.Linv[(long long)k * 36 + tid * 6 + m] * a.x[6 * k + m];
      yk[tid] = s;
    }
    __syncthreads();
    if (tid < 6) a.x[6 * k + tid] = yk[tid];
    const int c0 = a.cptr[k], na = a.cptr[k + 1] - c0;
    for (int idx = tid; idx < na * 6; idx += 256) {
      const int i = a.crows[c0 + idx / 6], r = idx % 6;
      const long long o = sky_off(a, i, k);
      double s = 0.0;
      for (int m = 0; m < 6; ++m) s += a.S[o + r * 6 + m] * yk[m];
      a.x[6 * i + r] -= s;
    }
    __threadfence_block();
    __syncthreads();
  }
  // back substitution Lᵀ x = y
  for (int k = a.N - 1; k >= 0; --k) {
    __shared__ double tk[6];
    if (tid < 6) {
      double s = a.x[6 * k + tid];
      for (int q = a.cptr[k]; q < a.cptr[k + 1]; ++q) {
        const int i = a.crows[q];
        const long long o = sky_off(a, i, k);
        for (int m = 0; m < 6; ++m) s -= a.S[o + m * 6 + tid] * a.x[6 * i + m];
      }
      tk[tid] = s;
    }
    __syncthreads();
    if (tid < 6) {
      double s = 0.0;
      for (int m = tid; m < 6; ++m) s += a.Linv[(long long)k * 36 + m * 6 + tid] * tk[m];
      a.x[6 * k + tid] = s;
    }
    __threadfence_block();
    __syncthreads();
  }
  if (tid == 0) *a.status = 0;
}

// rsqrt_nr (pba_device.h): hardware v_rsq_f64 seed + two Newton steps — the pivot is on the solver's
// serial critical path; this is ~3x shorter than sqrt() + division.
__device__ inline bool chol6_rcp(double* A, double* invd) {  // in place, lower; returns reciprocal pivots
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double s = A[j * 6 + j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= A[j * 6 + k] * A[j * 6 + k];
    if (!(s > 0.0)) return false;
    const double il = rsqrt_nr(s), l = s * il;
    A[j * 6 + j] = l;
    invd[j] = il;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double t = A[i * 6 + j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= A[i * 6 + k] * A[j * 6 + k];
      A[i * 6 + j] = t * il;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = i + 1; j < 6; ++j) A[i * 6 + j] = 0.0;
  return true;
}

// ------------------------------------------------------------------------------------------------
// front_solve_kernel: the same factorisation and solve with the ACTIVE FRONT in LDS (one workgroup)
// ------------------------------------------------------------------------------------------------
// Right-looking block Cholesky touches, at column k, only the blocks among {k} ∪ rows(k), rows(k) = {i > k : first(i) ≤ k}
// — the front.  It moves by one row per column: k leaves, the rows with first(i) = k + 1 enter with their blocks fresh
// from S (no earlier column touched them).  gn_prepare gives every row a static LDS slot (a row admitted for column k + 1
// never takes a slot in use at column k) and writes per column a record: the slots, row indices and factor-block
// indices of rows(k), and the fresh blocks of the next column's admissions (source skyline block → front position
// slot_hi·F + slot_lo) — build_front_plan; a multi-GPU free-intrinsics solve has a plan of its own for the summed
// profile (ensure_dist_sky).  skyline_solve_kernel walks the same factorisation through global memory, a dependent L2
// round trip per phase (≈ 9 µs per column); here the front, the forward vector and the records live in LDS and the
// next column's fresh blocks and record are loaded while this column is factored.  Free intrinsics make the profile a
// band plus 2·nc dense border rows: F = K + 1 + 2nc slots (C3/C4: 7).
// Every lane issues its share of the global loads of the record two columns ahead and of the next column's fresh
// blocks (backward: its staged factor blocks) at a column's start and stores them to LDS at its end.  (A dedicated
// loader wave measured slower: the compiler's conservative waits then stalled that wave at the barriers.)
// Forward (2 barriers per column): 6·|rows(k)| lanes form L_ik = A_ik L_kk⁻ᵀ row by row (to LDS, to L, v_i −= L_ik y_k);
// then the trailing pairs A_ij −= L_ik L_jkᵀ while one lane finishes and factors the next diagonal block (look-ahead:
// L_kk, reciprocal pivots and y_k = L_kk⁻¹ v_k were formed during column k − 1).
// Backward (2 barriers per column): 6·|rows(k)| lanes form the products L_ikᵀ x_i, six lanes add them in order and one
// solves x_k = L_kk⁻ᵀ (y_k − Σ_i L_ikᵀ x_i).
constexpr int kFrontHdr = 3;
struct FrontArgs {
  const double* S;      // the assembled skyline system
  const double* g;
  double* L;            // the factor's off-diagonal blocks (skyline layout)
  double* lrec;         // per column: L_kk | 1/pivots | y_k
  const int* rec;       // per column: kFrontHdr + 3·fm + 2·mf ints
  const int2* init;     // the rows of column 0's front: (source block, front position)
  double* x;
  int* status;
  int N, F, fm, mf, R, n_init;
};
constexpr int kFrontPf = 4;  // doubles per lane per column: fresh blocks (mf·36) / staged blocks (fm·36 + 48)
constexpr int kFrontPr = 1;  // record ints per lane (R ≤ 256)

__global__ __launch_bounds__(256) void front_solve_kernel(const FrontArgs a) {
  extern __shared__ double front_lds[];
  const int tid = threadIdx.x, N = a.N, F = a.F, fm = a.fm, mf = a.mf, R = a.R;
  const int SB = fm * 36 + 48, ld = tid;
  double* fr = front_lds;                                // F·F blocks: block (i ≥ j) at slot_i·F + slot_j
  double* ys = fr + (size_t)F * F * 36;                  // v → y → x, 6 per row
  double* stg = ys + 6 * N;                              // backward: 2 × SB
  int* recb = reinterpret_cast<int*>(stg + 2 * SB);      // 3 × R: records k, k + 1, k + 2 (backward: k, k − 1, k − 2)
  int* pairs = recb + 3 * R;                             // lower-triangle pair p → (ii << 16) | jj
  __shared__ double sL[2][36], sd[2][6], sy[2][6], sp[6 * 32];  // the diagonal factor of columns k, k + 1
  __shared__ double sDn[36];                                       // column k + 1's diagonal block (look-ahead)
  __shared__ int s_fail;
#ifdef PBA_FRONT_STAMPS  // timing variant: per-phase wall-clock sums of lanes 0, 64 and 192, written over x[0 … 29]
  unsigned long long fts[10] = {}, ft0 = 0;
#define FRONT_STAMP(i) { const unsigned long long t_ = wall_clock64(); if ((i) > 0) fts[(i) - 1] += t_ - ft0; ft0 = t_; }
#else
#define FRONT_STAMP(i)
#endif
  // the prefetch loads: unconditional (clamped addresses; the stores are guarded) — under a branch, the compiler waited
  // for every load in flight at the first use of any
  auto load_rec = [&](int k, int (&regs)[kFrontPr]) {
#pragma unroll
    for (int q = 0; q < kFrontPr; ++q)
      regs[q] = a.rec[(long long)min(max(k, 0), N - 1) * R + min(ld + 256 * q, R - 1)];
  };
  auto store_rec = [&](int k, const int (&regs)[kFrontPr]) {
#pragma unroll
    for (int q = 0; q < kFrontPr; ++q)
      if (ld + 256 * q < R) recb[(k % 3) * R + ld + 256 * q] = regs[q];
  };
  auto load_fresh = [&](const int* rk, double (&regs)[kFrontPf]) {  // the blocks column k admits for column k + 1
    const int nfr = rk[2];
    const int* fsrc = rk + kFrontHdr + 3 * fm;
#pragma unroll
    for (int q = 0; q < kFrontPf; ++q) {
      const int idx = min(ld + 256 * q, max(nfr * 36 - 1, 0));
      regs[q] = a.S[(long long)(nfr ? fsrc[idx / 36] : 0) * 36 + idx % 36];
    }
  };
  if (tid == 0) s_fail = 0;
  for (int t = tid; t < 6 * N; t += 256) ys[t] = -a.g[t];
  for (int t = tid; t < a.n_init * 36; t += 256) {
    const int2 q = a.init[t / 36];
    fr[(long long)q.y * 36 + t % 36] = a.S[(long long)q.x * 36 + t % 36];
  }
  for (int t = tid; t < 2 * R; t += 256)
    if (t / R < N) recb[t] = a.rec[t];
  for (int p = tid; p < fm * (fm + 1) / 2; p += 256) {
    int ii = 0;
    while ((ii + 1) * (ii + 2) / 2 <= p) ++ii;
    pairs[p] = (ii << 16) | (p - ii * (ii + 1) / 2);
  }
  __syncthreads();

  // the 6×6 factor of a diagonal block, y = L⁻¹ v, into buffer set q (one lane); false: not positive definite
  auto factor = [&](const double (&D)[36], int col, int q) -> bool {
    double A[36], d[6];
#pragma unroll
    for (int e = 0; e < 36; ++e) A[e] = D[e];
    if (!chol6_rcp(A, d)) return false;
    double b[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) b[r] = ys[6 * col + r];
#pragma unroll
    for (int c = 0; c < 6; ++c) {  // y_col = L⁻¹ v_col
      double t = b[c];
#pragma unroll
      for (int m = 0; m < c; ++m) t -= A[c * 6 + m] * b[m];
      b[c] = t * d[c];
    }
#pragma unroll
    for (int e = 0; e < 36; ++e) sL[q][e] = A[e];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      sd[q][r] = d[r];
      sy[q][r] = b[r];
      ys[6 * col + r] = b[r];
    }
    return true;
  };
  auto factor_lds = [&](int col, int slot, int q) {  // column col's diagonal block as it stands in the front
    double D[36];
    const double* Dk = fr + (long long)(slot * F + slot) * 36;
#pragma unroll
    for (int e = 0; e < 36; ++e) D[e] = Dk[e];
    if (!factor(D, col, q)) s_fail = col + 1;
  };
  if (N > 0 && tid == 0) factor_lds(0, recb[0], 0);
  __syncthreads();
  if (s_fail) {
    if (tid == 0) *a.status = s_fail;
    return;
  }

  // One column, LOOK-AHEAD: its diagonal block was factored during the previous column (buffer set k & 1).  Panel,
  // then — while lanes 0-191 run the trailing update — lane 192 forms column k + 1's diagonal block (its last update,
  // −L_{k+1,k} L_{k+1,k}ᵀ, when k + 1 is the column's first row) and factors it: the 6×6 factor's serial chain is off
  // the critical path.  A column k + 1 outside rows(k) (admitted fresh at k + 1) is factored after the barrier.
  // cur holds the column's admissions (loaded during the previous column), nxt receives the next column's — two
  // columns per pass with the arrays swapped (no register copies).
  auto column = [&](int k, double (&cur)[kFrontPf], double (&nxt)[kFrontPf]) -> bool {
    const int* rk = recb + (k % 3) * R;
    const int sk = rk[0], na = rk[1], nfr = rk[2], q = k & 1;
    const int* slots = rk + kFrontHdr;
    const int* rows = slots + fm;
    const int* gbl = rows + fm;
    const int* fdst = gbl + fm + mf;
    FRONT_STAMP(0);
    int pr[kFrontPr];
    load_rec(k + 2, pr);  // before the fresh loads: waiting for it must not wait for them
    if (k + 1 < N) load_fresh(recb + ((k + 1) % 3) * R, nxt);
    FRONT_STAMP(1);
    FRONT_STAMP(2);
    if (tid < na * 6) {  // panel row r of L_ik = A_ik L_kk⁻ᵀ; v_i −= L_ik y_k
      const int li = tid / 6, r = tid % 6;
      double* A = fr + (long long)(slots[li] * F + sk) * 36 + r * 6;
      double X[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        double t = A[c];
#pragma unroll
        for (int m = 0; m < c; ++m) t -= X[m] * sL[q][c * 6 + m];
        X[c] = t * sd[q][c];
      }
      double* Lg = a.L + (long long)gbl[li] * 36 + r * 6;
      double dv = 0.0;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        A[c] = X[c];
        Lg[c] = X[c];
        dv += X[c] * sy[q][c];
      }
      ys[6 * rows[li] + r] -= dv;
    } else if (tid >= 192 && tid < 240) {
      const int e = tid - 192;
      a.lrec[(long long)k * 48 + e] = e < 36 ? sL[q][e] : (e < 42 ? sd[q][e - 36] : sy[q][e - 42]);
    }
    FRONT_STAMP(3);
    __syncthreads();
    FRONT_STAMP(4);
    const bool ahead = k + 1 < N && na > 0 && rows[0] == k + 1;  // (uniform)
    const int np = na * (na + 1) / 2;  // trailing A_ij −= L_ik L_jkᵀ (i ≥ j in rows(k)); pair 0 = (k+1, k+1) if ahead
    if (tid < 192) {  // four items per lane in flight: their dependent LDS rounds (pair → slots → rows → element) overlap
      constexpr int TR = 4;
      const int i0 = ahead ? 36 : 0, ne = np * 36;
      for (int base = i0 + tid; base < ne; base += 192 * TR) {
        double acc[TR];
        int dst[TR];
#pragma unroll
        for (int u = 0; u < TR; ++u) {
          const int idx = min(base + 192 * u, ne - 1);
          const int pq = pairs[idx / 36], e = idx % 36, r = e / 6, c = e % 6;
          const int si = slots[pq >> 16], sj = slots[pq & 0xffff];
          const double* Li = fr + (si * F + sk) * 36 + r * 6;
          const double* Lj = fr + (sj * F + sk) * 36 + c * 6;
          double t = 0.0;
#pragma unroll
          for (int m = 0; m < 6; ++m) t += Li[m] * Lj[m];
          acc[u] = t;
          dst[u] = (si * F + sj) * 36 + e;
        }
#pragma unroll
        for (int u = 0; u < TR; ++u)
          if (base + 192 * u < ne) fr[dst[u]] -= acc[u];
      }
    } else if (ahead) {  // wave 3: column k + 1's diagonal block, final (lane e: entry e), then lane 192 factors it
      const int s1 = slots[0], e = tid - 192;
      if (e < 36) {
        const double* Li = fr + (long long)(s1 * F + sk) * 36 + (e / 6) * 6;
        const double* Lj = fr + (long long)(s1 * F + sk) * 36 + (e % 6) * 6;
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < 6; ++m) acc += Li[m] * Lj[m];
        sDn[e] = fr[(long long)(s1 * F + s1) * 36 + e] - acc;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (e == 0) {
        double D[36];
#pragma unroll
        for (int i = 0; i < 36; ++i) D[i] = sDn[i];
        if (!factor(D, k + 1, q ^ 1)) s_fail = k + 2;
      }
    }
#pragma unroll
    for (int qq = 0; qq < kFrontPf; ++qq) {  // column k's admissions (slots unused at column k), the record of k + 2
      const int idx = ld + 256 * qq;
      if (idx < nfr * 36) fr[(long long)fdst[idx / 36] * 36 + idx % 36] = cur[qq];
    }
    if (k + 2 < N) store_rec(k + 2, pr);
    FRONT_STAMP(5);
    __syncthreads();
    FRONT_STAMP(6);
    if (k + 1 < N && !ahead) {  // column k + 1 entered the front fresh: factor it now
      if (tid == 0) factor_lds(k + 1, recb[((k + 1) % 3) * R], q ^ 1);
      __syncthreads();
    }
    if (s_fail) {
      if (tid == 0) *a.status = s_fail;
      return false;
    }
    return true;
  };
  double pf[kFrontPf], pfn[kFrontPf];
  load_fresh(recb, pf);
  for (int k = 0; k < N; k += 2) {
    if (!column(k, pf, pfn)) return;
    if (k + 1 < N && !column(k + 1, pfn, pf)) return;
  }
  __threadfence();
  __syncthreads();

  // backward: x_k = L_kk⁻ᵀ (y_k − Σ_i L_ikᵀ x_i); column k's blocks staged during column k + 1, loaded during k + 2
  auto load_stage = [&](int k, const int* rk, double (&regs)[kFrontPf]) {
    const int na = rk[1];
    const int* gbl = rk + kFrontHdr + 2 * fm;
#pragma unroll
    for (int q = 0; q < kFrontPf; ++q) {  // unused stage entries hold any value
      const int idx = ld + 256 * q;
      const double* src = a.lrec;
      if (k >= 0 && idx < na * 36) src = a.L + (long long)gbl[idx / 36] * 36 + idx % 36;
      else if (k >= 0 && idx >= fm * 36 && idx < SB) src = a.lrec + (long long)k * 48 + idx - fm * 36;
      regs[q] = *src;
    }
  };
  auto store_stage = [&](int k, const double (&regs)[kFrontPf]) {
#pragma unroll
    for (int q = 0; q < kFrontPf; ++q)
      if (ld + 256 * q < SB) stg[(k & 1) * SB + ld + 256 * q] = regs[q];
  };
  double pb[kFrontPf], pbn[kFrontPf];  // cur / nxt of bcolumn, swapped per column as the forward pass
  for (int t = tid; t < 3 * R; t += 256) {
    const int k = N - 1 - t / R;
    if (k >= 0) recb[(k % 3) * R + t % R] = a.rec[(long long)k * R + t % R];
  }
  __syncthreads();
  {
    const int* rk = recb + ((N - 1) % 3) * R;
    for (int t = tid; t < SB; t += 256) {
      double v = 0.0;
      if (t < rk[1] * 36) v = a.L[(long long)rk[kFrontHdr + 2 * fm + t / 36] * 36 + t % 36];
      else if (t >= fm * 36) v = a.lrec[(long long)(N - 1) * 48 + t - fm * 36];
      stg[((N - 1) & 1) * SB + t] = v;
    }
  }
  load_stage(N - 2, recb + (((N - 2) % 3 + 3) % 3) * R, pb);
  __syncthreads();
  auto bcolumn = [&](int k, double (&cur)[kFrontPf], double (&nxt)[kFrontPf]) {
    const int* rk = recb + (k % 3) * R;
    const double* st = stg + (k & 1) * SB;
    const int na = rk[1];
    FRONT_STAMP(0);
    int pr[kFrontPr];
    load_rec(k - 3, pr);
    load_stage(k - 2, recb + (((k - 2) % 3 + 3) % 3) * R, nxt);
    if (tid < na * 6) {  // (L_ikᵀ x_i)_r
      const int li = tid / 6, r = tid % 6;
      const double* Lb = st + li * 36 + r;
      const double* xi = ys + 6 * rk[kFrontHdr + fm + li];
      double p = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m) p += Lb[m * 6] * xi[m];
      sp[tid] = p;
    }
    FRONT_STAMP(7);
    __syncthreads();
    FRONT_STAMP(8);
    if (tid < 64) {  // lanes 0-5 add the products of entry r in order, lane 0 solves
      double tr = 0.0;
      if (tid < 6) {
        tr = st[fm * 36 + 42 + tid];
        for (int li = 0; li < na; ++li) tr -= sp[li * 6 + tid];
      }
      double t[6];
#pragma unroll
      for (int r = 0; r < 6; ++r) t[r] = __shfl(tr, r, 64);
      if (tid == 0) {
#pragma unroll
      for (int r = 5; r >= 0; --r) {  // L_kkᵀ x = t
        double v = t[r];
#pragma unroll
        for (int m = r + 1; m < 6; ++m) v -= st[fm * 36 + m * 6 + r] * t[m];
        t[r] = v * st[fm * 36 + 36 + r];
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        ys[6 * k + r] = t[r];
        a.x[6 * k + r] = t[r];
      }
      }
    }
    if (k >= 1) store_stage(k - 1, cur);  // column k − 1's stage (not read at column k)
    if (k >= 3) store_rec(k - 3, pr);     // the record of k − 3 (over record k)
    FRONT_STAMP(9);
    __syncthreads();
    FRONT_STAMP(10);
  };
  for (int k = N - 1; k >= 0; k -= 2) {
    bcolumn(k, pb, pbn);
    if (k >= 1) bcolumn(k - 1, pbn, pb);
  }
  if (tid == 0) *a.status = 0;
#ifdef PBA_FRONT_STAMPS
  __syncthreads();
  if (tid == 0 || tid == 64 || tid == 192)
    for (int i = 0; i < 10; ++i) a.x[(tid == 0 ? 0 : (tid == 64 ? 10 : 20)) + i] = (double)fts[i];
#endif
#undef FRONT_STAMP
}

// ------------------------------------------------------------------------------------------------
// band_solve_kernel<B>: the same factorisation when every block row satisfies first(i) ≥ i − B (the
// structure of windowed/sequential BA — C3/C4 have B = 4).  The assembly also writes S in dense band
// layout (block c of row i = column i − B + c), so the next block row's address needs no indirection.
// The active window of the factor (block rows k..k+B) lives in LDS as a ring; block row k+B+2 is
// prefetched into registers two steps ahead.  Per step: one lane factors the 6×6 diagonal block
// (reciprocal pivots, no inverse), B·6 lanes solve the column panel L_ik = A_ik L_kk⁻ᵀ row by row, the
// trailing triangle is updated in parallel, and forward substitution is fused in.  Finished rows of L and
// the reciprocal pivots go to global memory for the backward pass, which prefetches one step ahead.
// ------------------------------------------------------------------------------------------------
struct BandArgs {
  const double* Sband;  // N rows × ((B+1)·36 + 6): blocks of columns i−B..i, then g_i
  double* Lcol;         // N column records × (B·36 + 48): L_(k+q),k for q = 1..B | L_kk | 1/pivots | y_k
  double* x;            // the step δ_poses
  int* status;
  int N;
};

template <int B>
__global__ __launch_bounds__(256) void band_solve_kernel(const BandArgs a) {
  constexpr int W = B + 1;
  constexpr int ROWF = W * 36;
  constexpr int ROWG = ROWF + 6;
  constexpr int COLF = B * 36 + 48;
  constexpr int CH = B <= 8 ? 16 : 4;      // rows / column records per prefetch chunk
  constexpr int STG = CH * COLF;           // ≥ CH·ROWG
  constexpr int PCH = (STG + 255) / 256;
  __shared__ double win[W * ROWG];         // ring of block rows k..k+B (slot i % W)
  __shared__ double stage[2 * STG];        // double-buffered prefetch chunks
  __shared__ double ring[W * 6];           // y (forward) / x (backward) of the last B+1 block rows
  __shared__ double sd[6], sv[6];
  __shared__ int s_fail;
  const int tid = threadIdx.x, N = a.N;

  // ---- forward: factor + fused forward substitution -------------------------------------------------
  auto load_rows = [&](int r0, double* regs) {  // rows r0 .. r0+CH−1 (zero beyond N)
#pragma unroll
    for (int q = 0; q < PCH; ++q) {
      const int idx = tid + q * 256;
      const int i = r0 + idx / ROWG;
      regs[q] = (idx < CH * ROWG && i < N) ? a.Sband[(long long)r0 * ROWG + idx] : 0.0;
    }
  };
  auto put_stage = [&](int buf, const double* regs, int n) {
#pragma unroll
    for (int q = 0; q < PCH; ++q) {
      const int idx = tid + q * 256;
      if (idx < n) stage[buf * STG + idx] = regs[q];
    }
  };
  if (tid == 0) s_fail = 0;
  for (int idx = tid; idx < W * ROWG; idx += 256)
    win[idx] = (idx / ROWG < N) ? a.Sband[idx] : 0.0;  // rows 0..B into slots 0..B
  if (tid < W * 6) ring[tid] = 0.0;
  double pf[PCH];
  load_rows(W, pf);
  put_stage(0, pf, CH * ROWG);
  __syncthreads();

  for (int k = 0; k < N; ++k) {
    const int c = k / CH, o = k % CH;
    double* rk = win + (k % W) * ROWG;
    double* Lkk = rk + B * 36;
    if (o == 0) load_rows(W + (c + 1) * CH, pf);  // next chunk, lands during the next CH steps
    if (tid == 0) {
      double A[36], d[6];
#pragma unroll
      for (int e = 0; e < 36; ++e) A[e] = Lkk[e];
      if (!chol6_rcp(A, d)) {
        s_fail = k + 1;
      } else {
#pragma unroll
        for (int e = 0; e < 36; ++e) Lkk[e] = A[e];
#pragma unroll
        for (int e = 0; e < 6; ++e) sd[e] = d[e];
      }
    } else if (tid >= 64 && tid < 70) {  // b_k = −g_k − Σ_j L_kj y_j   (L_kj final, y_j in the ring)
      const int r = tid - 64;
      double v = -rk[ROWF + r];
#pragma unroll
      for (int cc = 0; cc < B; ++cc) {
        const int j = k - B + cc;
        if (j < 0) continue;
        const double* Lb = rk + cc * 36 + r * 6;
        const double* yj = ring + (j % W) * 6;
#pragma unroll
        for (int m = 0; m < 6; ++m) v -= Lb[m] * yj[m];
      }
      sv[r] = v;
    }
    __syncthreads();
    if (s_fail) {
      if (tid == 0) *a.status = s_fail;
      return;
    }
    const int nk = min(B, N - 1 - k);
    double* rec = a.Lcol + (long long)k * COLF;
    if (tid < nk * 6) {  // panel row r of L_ik = A_ik L_kk⁻ᵀ
      const int ii = 1 + tid / 6, r = tid % 6;
      double* A = win + ((k + ii) % W) * ROWG + (B - ii) * 36 + r * 6;
      double X[6];
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) {
        double t = A[cc];
#pragma unroll
        for (int m = 0; m < cc; ++m) t -= X[m] * Lkk[cc * 6 + m];
        X[cc] = t * sd[cc];
      }
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) A[cc] = X[cc];
    } else if (tid >= 192 && tid < 228) {
      rec[B * 36 + (tid - 192)] = Lkk[tid - 192];
    } else if (tid >= 228 && tid < 234) {
      rec[B * 36 + 36 + (tid - 228)] = sd[tid - 228];
    } else if (tid == 255) {  // y_k = L_kk⁻¹ b_k
      double L[36], bb[6], d[6];
#pragma unroll
      for (int e = 0; e < 36; ++e) L[e] = Lkk[e];
#pragma unroll
      for (int r = 0; r < 6; ++r) { bb[r] = sv[r]; d[r] = sd[r]; }
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) {
        double t = bb[cc];
#pragma unroll
        for (int m = 0; m < cc; ++m) t -= L[cc * 6 + m] * bb[m];
        bb[cc] = t * d[cc];
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        ring[(k % W) * 6 + r] = bb[r];
        rec[B * 36 + 42 + r] = bb[r];
      }
    }
    __syncthreads();
    // trailing update A_ij −= L_ik L_jkᵀ (k < j ≤ i ≤ k+nk); column k of L to the record
    const int npairs = nk * (nk + 1) / 2;
    for (int idx = tid; idx < npairs * 36; idx += 256) {
      const int pidx = idx / 36, e = idx % 36, r = e / 6, cc = e % 6;
      int ii = 0;
      while ((ii + 1) * (ii + 2) / 2 <= pidx) ++ii;
      const int jj = pidx - ii * (ii + 1) / 2;
      const int i = k + 1 + ii, j = k + 1 + jj;
      const double* Li_ = win + (i % W) * ROWG + (k - i + B) * 36;
      const double* Lj_ = win + (j % W) * ROWG + (k - j + B) * 36;
      double sacc = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m) sacc += Li_[r * 6 + m] * Lj_[cc * 6 + m];
      win[(i % W) * ROWG + (j - i + B) * 36 + e] -= sacc;
    }
    for (int idx = tid; idx < B * 36; idx += 256) {
      const int q = 1 + idx / 36, e = idx % 36;
      rec[idx] = (q <= nk) ? win[((k + q) % W) * ROWG + (B - q) * 36 + e] : 0.0;
    }
    // row k+B+1 from the staged chunk into row k's slot (first read by the next step's panel)
    {
      const double* src = stage + (c & 1) * STG + o * ROWG;
      for (int idx = tid; idx < ROWG; idx += 256) rk[idx] = src[idx];
    }
    if (o == CH - 1) put_stage((c + 1) & 1, pf, CH * ROWG);
    __syncthreads();
  }
  __threadfence();
  __syncthreads();

  // ---- backward: x_k = L_kk⁻ᵀ (y_k − Σ_q L_(k+q),kᵀ x_(k+q)), column records streamed in reverse ---------
  auto load_cols = [&](int s0, double* regs) {  // records for steps s0..s0+CH−1, k = N−1−s
#pragma unroll
    for (int q = 0; q < PCH; ++q) {
      const int idx = tid + q * 256;
      const int sidx = s0 + idx / COLF;
      regs[q] = (idx < STG && sidx < N) ? a.Lcol[(long long)(N - 1 - sidx) * COLF + idx % COLF] : 0.0;
    }
  };
  if (tid < W * 6) ring[tid] = 0.0;
  load_cols(0, pf);
  put_stage(0, pf, STG);
  __syncthreads();
  for (int sstep = 0; sstep < N; ++sstep) {
    const int k = N - 1 - sstep, c = sstep / CH, o = sstep % CH;
    if (o == 0) load_cols((c + 1) * CH, pf);
    const double* rec = stage + (c & 1) * STG + o * COLF;
    if (tid < 6) {
      const int r = tid;
      double v = rec[B * 36 + 42 + r];
#pragma unroll
      for (int q = 1; q <= B; ++q) {
        if (k + q >= N) break;
        const double* Lq = rec + (q - 1) * 36;
        const double* xq = ring + ((k + q) % W) * 6;
#pragma unroll
        for (int m = 0; m < 6; ++m) v -= Lq[m * 6 + r] * xq[m];
      }
      sv[r] = v;
    }
    __syncthreads();
    if (tid == 0) {
      double L[36], t[6], id[6];
#pragma unroll
      for (int e = 0; e < 36; ++e) L[e] = rec[B * 36 + e];
#pragma unroll
      for (int r = 0; r < 6; ++r) { t[r] = sv[r]; id[r] = rec[B * 36 + 36 + r]; }
#pragma unroll
      for (int r = 5; r >= 0; --r) {  // L_kkᵀ x = t
        double v = t[r];
#pragma unroll
        for (int m = r + 1; m < 6; ++m) v -= L[m * 6 + r] * t[m];
        t[r] = v * id[r];
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        ring[(k % W) * 6 + r] = t[r];
        a.x[6 * k + r] = t[r];
      }
    }
    if (o == CH - 1) put_stage((c + 1) & 1, pf, STG);
    __syncthreads();
  }
  if (tid == 0) *a.status = 0;
}

// ------------------------------------------------------------------------------------------------
// Block cyclic reduction (bandwidth B ≤ 8 block rows).  Super-row I = block rows [I·B, (I+1)·B) turns the
// banded reduced camera system into a block-tridiagonal SPD system with m×m blocks (m = 6B): diagonal D_I,
// coupling U_I = S(I, I+1).  Each level eliminates the odd super-rows j in parallel (one workgroup each:
// dense Cholesky of D_j in LDS, X_j = D_j⁻¹ [U_{j−1}ᵀ | U_j | b_j]) and rebuilds the even ones
// (D'_i = D_i − U_{i−1}ᵀ X_{i−1}^U − U_i X_{i+1}^L, U'_i = −U_i X_{i+1}^U, b'_i likewise).  log2(N/B) levels
// replace the N-step sequential factorisation; back-substitution runs the levels in reverse
// (x_j = X_j^b − X_j^L x_{j−1} − X_j^U x_{j+1}).
// ------------------------------------------------------------------------------------------------
struct CrLevel {
  double* D;   // n × m²
  double* U;   // n × m²   (U of the last row = 0)
  double* b;   // n × m
  double* X;   // ⌊n/2⌋ × m × (2m+1)
  double* x;   // n × m
  int n;
};

template <int M>
__global__ __launch_bounds__(256) void cr_build_kernel(const double* __restrict__ Sband, CrLevel L0, int N, int B,
                                                       int* __restrict__ status) {
  // one thread per element of D_I, U_I and b_I of level 0 (rows ≥ N are identity padding); the solve's failure flag
  // is cleared here (the levels only ever set it), which saves a memset launch per solve
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid == 0) *status = 0;
  const long long nD = (long long)L0.n * M * M;
  const int ROWG = (B + 1) * 36 + 6;
  auto lower = [&](int i, int j, int r, int c) -> double {  // S[6i+r][6j+c] for i ≥ j within the band
    if (i >= N || j >= N) return (i == j && r == c) ? 1.0 : 0.0;
    if (i - j > B) return 0.0;
    return Sband[(long long)i * ROWG + (j - i + B) * 36 + r * 6 + c];
  };
  if (tid < nD) {
    const int I = (int)(tid / (M * M)), e = (int)(tid % (M * M)), R = e / M, C = e % M;
    const int i = I * B + R / 6, j = I * B + C / 6, r = R % 6, c = C % 6;
    L0.D[tid] = i >= j ? lower(i, j, r, c) : lower(j, i, c, r);
    // U_I: rows of super-row I, columns of super-row I+1 → S[6i+r][6j'+c] with j' > i
    const int jn = (I + 1) * B + C / 6;
    L0.U[tid] = (I + 1 < L0.n) ? lower(jn, i, c, r) : 0.0;
    return;
  }
  const long long t = tid - nD;
  if (t < (long long)L0.n * M) {
    const int I = (int)(t / M), R = (int)(t % M), i = I * B + R / 6;
    L0.b[t] = i < N ? -Sband[(long long)i * ROWG + (B + 1) * 36 + R % 6] : 0.0;
  }
}

// Eliminate super-row j (odd rows of the level, or the single root row when `root`): X = D⁻¹ [U_{j−1}ᵀ | U_j | b]
// by 2×2-block Gauss-Jordan on the augmented M × (3M+1) matrix [D | RHS] (no pivoting: D is SPD, so are its
// 2×2 pivot blocks).  Lane c owns column c in registers (steps fully unrolled, so every register index is
// static).  Step k: the pivot columns' owners publish their 2M values to LDS (double-buffered: one barrier per
// step), every lane reads them as broadcasts and updates its own column.  Measured on MI355X
// (tools/micro/cr_odd_timing.hip, M = 24): 12 µs per launch for 1×1 pivots against 29 µs for an element-owner
// formulation whose per-step publish/read traffic was LDS-bound.  A non-positive pivot flags the status.
template <int M>
constexpr int kCrOddThreads = ((3 * M + 1) + 63) / 64 * 64;  // one lane per column of [D | RHS], whole waves

// The elimination of one super-row by kCrOddThreads<M> lanes (tid = lane index within that group, c = its
// column); colk = the group's own publish buffers.  Every lane of the workgroup must call it (barriers).
// Returns false when a pivot block was not positive definite; a[] = column c of [D⁻¹ | D⁻¹RHS].
template <int M>
__device__ __forceinline__ bool gj_row(const CrLevel& L, int j, bool root, int tid, double (*colk)[2][M], double* a) {
  constexpr int NC = 2 * M + 1, W = M + NC;
  const int c = min(tid, W - 1);
  const double* D = L.D + (long long)j * M * M;
#pragma unroll
  for (int r = 0; r < M; ++r) {  // all of a lane's loads in flight at once
    const double* src;
    if (c < M) src = D + r * M + c;
    else if (c < 2 * M) src = root ? nullptr : L.U + (long long)(j - 1) * M * M + (c - M) * M + r;  // U_{j−1}ᵀ
    else if (c < 3 * M) src = (!root && j + 1 < L.n) ? L.U + (long long)j * M * M + r * M + (c - 2 * M) : nullptr;  // U_j
    else src = L.b + (long long)j * M + r;
    a[r] = src ? *src : 0.0;
  }
  bool bad = false;
  auto step = [&](int k) {
    const int buf = (k >> 1) & 1;
    if (tid == k || tid == k + 1) {
      double* dst = colk[buf][tid - k];
#pragma unroll
      for (int r = 0; r < M; ++r) dst[r] = a[r];
    }
    __syncthreads();
    const double* c0 = colk[buf][0];
    const double* c1 = colk[buf][1];
    const double p00 = c0[k], p10 = c0[k + 1], p01 = c1[k], p11 = c1[k + 1];
    const double det = p00 * p11 - p01 * p10;
    bad |= !(p00 > 0.0 && det > 0.0);
    const double rd = rcp_nr(det);
    double ak = a[0], ak1 = a[1];
#pragma unroll
    for (int r = 1; r < M; ++r) ak = r == k ? a[r] : ak;
#pragma unroll
    for (int r = 2; r < M; ++r) ak1 = r == k + 1 ? a[r] : ak1;
    const double t0 = (p11 * ak - p01 * ak1) * rd;
    const double t1 = (p00 * ak1 - p10 * ak) * rd;
#pragma unroll
    for (int r = 0; r < M; ++r) a[r] = r == k ? t0 : (r == k + 1 ? t1 : a[r] - c0[r] * t0 - c1[r] * t1);
  };
  if constexpr (M <= 24) {
#pragma unroll
    for (int k = 0; k < M; k += 2) step(k);
  } else {
#pragma unroll 1
    for (int k = 0; k < M; k += 2) step(k);
  }
  return !bad;
}

// One level of cyclic reduction in ONE launch: workgroup i/2 rebuilds even super-row i.  Its two halves
// eliminate the neighbouring odd rows i−1 and i+1 side by side (gj_row, redundantly with the neighbouring
// workgroups — each odd row is done twice, saving a launch and an HBM round trip of X per level), keep both X in
// LDS, store X_{i+1} for the back-substitution (every odd row is the right neighbour of exactly one even row),
// then form D'_i = D_i − U_{i−1}ᵀX^U_{i−1} − U_i X^L_{i+1}, U'_i = −U_i X^U_{i+1} and b'_i likewise.
template <int M>
constexpr size_t cr_level_lds() { return sizeof(double) * (2 * M * M + 2 * M * (2 * M + 1)); }

template <int M>
__global__ __launch_bounds__(2 * kCrOddThreads<M>) void cr_level_kernel(CrLevel L, CrLevel Ln, int* status) {
  constexpr int NC = 2 * M + 1, W = M + NC, T = kCrOddThreads<M>;
  __shared__ __attribute__((aligned(16))) double colk[2][2][2][M];
  extern __shared__ double smem[];
  double* sUl = smem;               // U_{i−1}   M×M
  double* sUi = sUl + M * M;        // U_i       M×M
  double* sX[2] = {sUi + M * M, sUi + M * M + M * NC};  // X_{i−1}, X_{i+1}   M×NC each
  const int i = 2 * blockIdx.x, in = blockIdx.x;
  const int half = threadIdx.x >= T ? 1 : 0, tl = threadIdx.x - half * T;
  const int j = half ? i + 1 : i - 1;
  const bool has = j >= 0 && j < L.n;
  double a[M];
  const bool ok = gj_row<M>(L, has ? j : 1, false, tl, colk[half], a);
  if (!ok && has && tl == 0) atomicOr(status, 1);
  if (tl >= M && tl < W) {
    double* x = sX[half] + (tl - M);
#pragma unroll
    for (int r = 0; r < M; ++r) x[r * NC] = has ? a[r] : 0.0;
    if (half && has) {
      double* X = L.X + (long long)(j / 2) * M * NC + (tl - M);
#pragma unroll
      for (int r = 0; r < M; ++r) X[r * NC] = a[r];
    }
  }
  const bool left = i - 1 >= 0, right = i + 1 < L.n;
  for (int e = threadIdx.x; e < M * M; e += 2 * T) {
    sUl[e] = left ? L.U[(long long)(i - 1) * M * M + e] : 0.0;
    sUi[e] = L.U[(long long)i * M * M + e];
  }
  __syncthreads();
  const double* sXl = sX[0];
  const double* sXr = sX[1];
  for (int e = threadIdx.x; e < 2 * M * M + M; e += 2 * T) {
    if (e < M * M) {  // D' = D − U_{i−1}ᵀ X^U_{i−1} − U_i X^L_{i+1}
      const int r = e / M, c = e % M;
      double v = L.D[(long long)i * M * M + e];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + M + c] + sUi[r * M + q] * sXr[q * NC + c];
      Ln.D[(long long)in * M * M + e] = v;
    } else if (e < 2 * M * M) {  // U' = −U_i X^U_{i+1}
      const int f = e - M * M, r = f / M, c = f % M;
      double v = 0.0;
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUi[r * M + q] * sXr[q * NC + M + c];
      Ln.U[(long long)in * M * M + f] = right ? v : 0.0;
    } else {  // b'
      const int r = e - 2 * M * M;
      double v = L.b[(long long)i * M + r];
#pragma unroll 8
      for (int q = 0; q < M; ++q) v -= sUl[q * M + r] * sXl[q * NC + 2 * M] + sUi[r * M + q] * sXr[q * NC + 2 * M];
      Ln.b[(long long)in * M + r] = v;
    }
  }
}

// Wave-level variant for super-rows of ≤ 31 unknowns (B ≤ 5 keyframes), where [D | one coupling block | b] fits one
// wave: lane c < M holds column c of D, lanes M…2M−1 the coupling block's columns, lane 2M b.  The pivot columns are
// then always in the elimination's own wave: the pivot lanes publish them to a per-wave LDS buffer and every lane
// reads them back with no s_barrier (LDS operations of one wave are processed in order).  Measured
// (tools/micro/cr_level_timing.hip, M = 24): 17.0 → 14.5 µs per level launch with 2-column pivots (13.0 with the
// rebuild on the matrix cores, below); 4-column pivot blocks (6 publish/read round trips instead of 12): C4 step
// 0.228 → 0.216 ms per LM iteration (8-column blocks: 0.216-0.220, their per-lane 8×8 solve costs what the saved
// round trips gain).
#ifndef PBA_CR_PIVOT
#define PBA_CR_PIVOT 4
#endif
constexpr int kCrPivot = PBA_CR_PIVOT;  // columns per Gauss-Jordan step of gj_wave (1, 2, 4 or 8; divides M)

// Loads of the rows a launch wrote itself (COH: the last PCR level's solve reads the rows its own workgroup has just
// stored, cr_level_wave_kernel): `sc1` (L1-bypassing) agent-scope loads; plain otherwise.
template <bool COH>
__device__ __forceinline__ double ld_row(const double* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// Pivot blocks of PB columns: lanes k … k+PB−1 publish their columns to the wave's LDS buffer (row r: PB doubles),
// every lane reads the PB×PB pivot block P and solves P t = a[k … k+PB−1] in registers (unpivoted Gauss-Jordan:
// D is SPD, so is every pivot block; all of P's pivots must be positive), then updates its other rows
// a[r] −= Σ_j piv[r][j] t_j.  The publish / read round trip is paid M/PB times instead of M/2 times; the updates are
// the same FMAs.
// b: NB right-hand-side columns, row-major (row r of column q at b[r·NB + q]); lanes 2M … M + ncol − 1 take them.
template <int M, bool COH = false, int PB = kCrPivot, int NB = 1>
__device__ __forceinline__ bool gj_wave(const double* __restrict__ D, const double* __restrict__ R1, bool r1_trans,
                                        const double* __restrict__ b, int ncol, int c, double* piv, double* a) {
  static_assert(M % PB == 0, "pivot blocks tile the system");
  // column c of [D | R1 | b] as base + r·stride: one address choice per lane, then M unconditional loads in flight
  // together (a lane without a column reads D's and keeps zeros)
  const double* base = D + min(c, M - 1);
  int stride = M;
  bool zero = c >= M + ncol;
  if (c >= M && c < 2 * M) {
    if (R1) {
      base = r1_trans ? R1 + (c - M) * M : R1 + (c - M);
      stride = r1_trans ? 1 : M;
    } else {
      zero = true;
    }
  } else if (c >= 2 * M && c < M + ncol) {
    if (b) {
      base = b + (c - 2 * M);
      stride = NB;
    } else {
      zero = true;
    }
  }
#pragma unroll
  for (int r = 0; r < M; ++r) a[r] = ld_row<COH>(base + r * stride);
#pragma unroll
  for (int r = 0; r < M; ++r) a[r] = zero ? 0.0 : a[r];
  bool bad = false;
#pragma unroll
  for (int k = 0; k < M; k += PB) {
    if (c >= k && c < k + PB) {
      double* dst = piv + (c - k);
#pragma unroll
      for (int r = 0; r < M; ++r) dst[PB * r] = a[r];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    // every pivot row of the step read at once (the pivot block's rows first): the 24·PB broadcast reads are in flight
    // during the PB×PB solve instead of one or two at a time between the update FMAs (the update was LDS-latency
    // bound: ~2200 cycles per step)
    double pr[M][PB];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int r = (i + k) % M;
#pragma unroll
      for (int j = 0; j < PB; ++j) pr[r][j] = piv[PB * r + j];
    }
    double P[PB][PB], t[PB];
#pragma unroll
    for (int i = 0; i < PB; ++i) {
#pragma unroll
      for (int j = 0; j < PB; ++j) P[i][j] = pr[k + i][j];
      t[i] = a[k + i];
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {  // t ← P⁻¹ t
      bad |= !(P[i][i] > 0.0);
      const double inv = rcp_nr(P[i][i]);
#pragma unroll
      for (int j = i + 1; j < PB; ++j) P[i][j] *= inv;
      t[i] *= inv;
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        if (q == i) continue;
        const double f = P[q][i];
#pragma unroll
        for (int j = i + 1; j < PB; ++j) P[q][j] -= f * P[i][j];
        t[q] -= f * t[i];
      }
    }
#pragma unroll
    for (int r = 0; r < M; ++r) {
      if (r >= k && r < k + PB) {
        a[r] = t[r - k];
      } else {
        double v = a[r];
#pragma unroll
        for (int j = 0; j < PB; ++j) v -= pr[r][j] * t[j];
        a[r] = v;
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  return !bad;
}


// Rebuild of super-row i (next-level index in) from the two eliminations in LDS (sXl = X_{i−1}, sXr = X_{i+1}) and
// U_{i−1}, U_i, D_i, b_i, on RB waves: 4 waves take two column tiles each, 8 waves one.  keep_u: the rebuilt row
// still has a right coupling.  Waves w ≥ RB return at once.
template <int M, int RB, int NB = 1>
__device__ __forceinline__ void cr_rebuild(int w, int lane, const double* sUl, const double* sUi, const double* sD,
                                           const double* sb, const double* sXl, const double* sXr, const CrLevel& Ln,
                                           int in, bool keep_u) {
  constexpr int NC = 2 * M + NB;  // [D | U | b] columns: b's NB columns at 2M …
  static_assert(NC <= 64, "four column tiles");
  // Rebuild of row i on the matrix cores: [D' | U' | b'] = [D | 0 | b] − U_{i−1}ᵀ·[X^U_{i−1} | 0 | X^b_{i−1}]
  // − U_i·X_{i+1}, as 2 × 4 output tiles of v_mfma_f64_16x16x4f64 (rows padded to 32, columns to 64).  Wave w takes
  // row tile w & 1 and column tiles TPW·(w >> 1) + {0 … TPW−1}: a wave's tiles share the A operands and run as
  // independent accumulator chains.  Layouts (tools/micro/mfma_f64_layout.hip): A lane l = (row l%16, k l/16),
  // B lane l = (k l/16, column l%16), accumulator entry v of lane l = (row l/16 + 4v, column l%16).
  // 3.9 → 2.7 µs per level against the scalar LDS products (tools/micro/cr_level_timing.hip, V5).
  static_assert(M % 4 == 0 && M <= 32, "K steps of 4, two row tiles");
  static_assert(RB == 4 || RB == 8, "2 × 4 tiles over the rebuild waves");
  constexpr int TPW = 8 / RB;  // column tiles per wave
  if (w >= RB) return;
  const int rt = w & 1;
  const int arow = 16 * rt + (lane & 15), kq = lane >> 4;
  // every operand of the six K steps read from LDS first, at clamped (in-range) indices and with unconditional reads,
  // then the padding zeroed by selects: conditional reads were issued and waited one at a time (~2.9 µs per level)
  constexpr int KS = M / 4;
  const bool aok = arow < M;
  const int ar = aok ? arow : 0;
  int bcol[TPW];
  double av2[KS], av1[KS], bv2[TPW][KS], bv1[TPW][KS], cv[TPW][4];
#pragma unroll
  for (int h = 0; h < TPW; ++h) {
    bcol[h] = 16 * ((w >> 1) * TPW + h) + (lane & 15);
    const int c = bcol[h];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int r = 16 * rt + (lane >> 4) + 4 * v;
      cv[h][v] = c < M ? sD[min(r, M - 1) * M + c] : sb[min(r, M - 1) * NB + min(max(c - 2 * M, 0), NB - 1)];
    }
  }
#pragma unroll
  for (int s4 = 0; s4 < KS; ++s4) {
    const int q = 4 * s4 + kq;
    av2[s4] = sUi[ar * M + q];
    av1[s4] = sUl[q * M + ar];
#pragma unroll
    for (int h = 0; h < TPW; ++h) {
      const int c = bcol[h];
      bv2[h][s4] = sXr[q * NC + min(c, NC - 1)];
      bv1[h][s4] = sXl[q * NC + (c < M ? M + c : min(max(c, 2 * M), NC - 1))];
    }
  }
  v4f64 acc[TPW];
#pragma unroll
  for (int h = 0; h < TPW; ++h) {
    const int c = bcol[h];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int r = 16 * rt + (lane >> 4) + 4 * v;
      acc[h][v] = (r < M && (c < M || (c >= 2 * M && c < NC))) ? cv[h][v] : 0.0;
    }
  }
#pragma unroll
  for (int s4 = 0; s4 < KS; ++s4) {
    const double a2 = aok ? -av2[s4] : 0.0;
    const double a1 = aok ? -av1[s4] : 0.0;
#pragma unroll
    for (int h = 0; h < TPW; ++h) {
      const int c = bcol[h];
      const double b2 = c < NC ? bv2[h][s4] : 0.0;
      const double b1 = (c < M || (c >= 2 * M && c < NC)) ? bv1[h][s4] : 0.0;
      acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, b2, acc[h], 0, 0, 0);
      acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[h], 0, 0, 0);
    }
  }
#pragma unroll
  for (int h = 0; h < TPW; ++h)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int r = 16 * rt + (lane >> 4) + 4 * v, c = bcol[h];
      if (r < M) {
        if (c < M) Ln.D[(long long)in * M * M + r * M + c] = acc[h][v];
        else if (c < 2 * M) Ln.U[(long long)in * M * M + r * M + (c - M)] = keep_u ? acc[h][v] : 0.0;
        else if (c < NC) Ln.b[((long long)in * M + r) * NB + (c - 2 * M)] = acc[h][v];
      }
    }
}

// per-wave LDS of an elimination: gj_wave's pivot columns
template <int M>
constexpr int kPivBuf = M * kCrPivot;

template <int M, int NB = 1>
constexpr size_t cr_level_wave_lds() { return sizeof(double) * (3 * M * M + M * NB + 2 * M * (2 * M + NB)); }

// One level, 4 waves per rebuilt super-row i: wave 0 eliminates its left neighbour l on [D | U_l | b] (X^U, X^b),
// waves 1 and 2 its right neighbour r on [D | U_iᵀ | b] (X^L, X^b) and [D | U_r] (X^U) — D's columns replicated per
// wave — while wave 3 parks U_l, U_i, D_i and b_i in LDS for the rebuild of row i.
//   CR  (PCR = false): i = 2·blockIdx (the even rows), l = i − 1, r = i + 1, rebuilt row i/2 of the next level; X_r
//       is stored for the back-substitution.
//   PCR (PCR = true, stride s): i = blockIdx (EVERY row), l = i − s, r = i + s, rebuilt row i of the next level
//       (couplings now at stride 2s).  Every row stays in the system, so after ⌈log2 n⌉ levels all couplings are
//       gone and x_i = D_i⁻¹ b_i (pcr_solve_kernel): no back-substitution.  A PCR level runs twice the workgroups of a
//       CR level at the same per-workgroup latency, so it is used while the rows fit one workgroup per CU.
// The D_i' are Schur complements of SPD principal submatrices ({l, i, r}), so every pivot block stays SPD.
// The level's work for row i (rebuilt as row `in` of Ln) by a 4-wave workgroup: piv = 3 × M·kCrPivot doubles, smem =
// cr_level_wave_lds<M>() bytes.
// NB > 1 (PCR only): b holds NB right-hand-side columns (row-major, b[(i·M + r)·NB + q]) — the free-intrinsics
// arrow solve's [−g | border columns] (arrow_solve).
template <int M, bool PCR, int NB = 1>
__device__ __forceinline__ void cr_wave_level(const CrLevel& L, const CrLevel& Ln, int i, int in, int s, int* status,
                                              double (*piv)[kPivBuf<M>], double* smem) {
  static_assert(2 * M + NB <= 64, "one wave per elimination");
  static_assert(PCR || NB == 1, "the back-substitution's X has one right-hand side");
  constexpr int NC = 2 * M + NB;
  double* sUl = smem;
  double* sUi = sUl + M * M;
  double* sD = sUi + M * M;
  double* sb = sD + M * M;
  double* sX[2] = {sb + M * NB, sb + M * NB + M * NC};
  const int il = i - s, ir = i + s;
  const bool left = il >= 0, right = ir < L.n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#ifdef PBA_CR_STAMPS
  long long t0 = wall_clock64(), t1 = 0, t2 = 0;
#endif
  if (w == 3) {
    // U_l, U_i, D_i, b_i → LDS: every load in flight at once (a loop of load → LDS store pays one memory round trip
    // per element, serially: measured ~10 µs of a 12.4-µs level); missing neighbours read U_i and store zeros
    constexpr int NE = 3 * M * M + M * NB, NQ = (NE + 63) / 64;
    double v[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = lane + 64 * q;
      const double* src = L.b + (long long)i * M * NB;
      if (e < M * M) src = L.U + (long long)(left ? il : i) * M * M + e;
      else if (e < 2 * M * M) src = L.U + (long long)i * M * M + (e - M * M);
      else if (e < 3 * M * M) src = L.D + (long long)i * M * M + (e - 2 * M * M);
      else if (e < NE) src = L.b + (long long)i * M * NB + (e - 3 * M * M);
      v[q] = *src;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = lane + 64 * q;
      const bool zero = (e < M * M && !left) || (e >= M * M && e < 2 * M * M && !right);
      if (e < NE) smem[e] = zero ? 0.0 : v[q];
    }
  } else {
    const int j = w == 0 ? il : ir;
    const bool has = w == 0 ? left : right;
    const int jj = has ? j : i;  // a missing neighbour eliminates a real row and contributes zeros
    const double* D = L.D + (long long)jj * M * M;
    const double* bj = L.b + (long long)jj * M * NB;
    double a[M];
    bool ok;
    if (w == 0) ok = gj_wave<M, false, kCrPivot, NB>(D, L.U + (long long)jj * M * M, false, bj, M + NB, lane, piv[0], a);
    else if (w == 1) ok = gj_wave<M, false, kCrPivot, NB>(D, L.U + (long long)i * M * M, true, bj, M + NB, lane, piv[1], a);
    else ok = gj_wave<M>(D, jj + s < L.n ? L.U + (long long)jj * M * M : nullptr, false, nullptr, M, lane, piv[2], a);
    if (!ok && has && lane == 0) atomicOr(status, 1);
    if (lane >= M && lane < 2 * M + (w == 2 ? 0 : NB)) {
      const int col = lane < 2 * M ? (w == 1 ? lane - M : lane) : lane;  // (b's columns keep their lane index)
      double* x = sX[w == 0 ? 0 : 1] + col;
#pragma unroll
      for (int r = 0; r < M; ++r) x[r * NC] = has ? a[r] : 0.0;
      if (!PCR && w != 0 && has) {  // X_{i+1} for the back-substitution
        double* X = L.X + (long long)(j / 2) * M * NC + col;
#pragma unroll
        for (int r = 0; r < M; ++r) X[r * NC] = a[r];
      }
    }
  }
#ifdef PBA_CR_STAMPS
  t1 = wall_clock64();
#endif
  __syncthreads();
#ifdef PBA_CR_STAMPS
  t2 = wall_clock64();
#endif
  cr_rebuild<M, 4, NB>(w, lane, sUl, sUi, sD, sb, sX[0], sX[1], Ln, in, PCR ? i + 2 * s < L.n : right);
#ifdef PBA_CR_STAMPS
  __syncthreads();
  const long long t3 = wall_clock64();
  if (blockIdx.x == 5 && lane == 0)
    printf("crstamp s=%d w=%d phase_end_us %.2f barrier_us %.2f rebuild_us %.2f\n", s, w, (t1 - t0) * 0.01,
           (t2 - t0) * 0.01, (t3 - t0) * 0.01);
#endif
}

// out != nullptr (the last PCR level): the workgroup then also solves its decoupled row, x_i = D'_i⁻¹ b'_i, from the
// rows it has just written (read back with L1-bypassing loads after every wave's stores completed) — pcr_solve_kernel's
// work without its launch boundary and its reload of the level (out / lim as pcr_solve_kernel).
// NB > 1: out row t = i·M + r holds the NB solution columns at out[t·ld + q].
// Several independent right-hand-side batches in one launch (the arrow solve, gridDim.y = batches): batch y reads L's
// D, U at + y·bs_du and b at + y·bs_b, writes Ln at + y·bs_n and its solution columns at out + y·NB (its own CR run
// over its own copies of the rows: the batches share only L when that is level 0).
template <int M, bool PCR, int NB = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void cr_level_wave_kernel(
    CrLevel L, CrLevel Ln, int s, int* status, double* __restrict__ out, int lim, int ld = 1, long long bs_du = 0,
    long long bs_b = 0, long long bs_n = 0) {
  __shared__ __attribute__((aligned(16))) double piv[3][kPivBuf<M>];
  extern __shared__ double smem[];
  if (blockIdx.y) {
    const long long y = blockIdx.y;
    L.D += y * bs_du;
    L.U += y * bs_du;
    L.b += y * bs_b;
    Ln.D += y * bs_n;
    Ln.U += y * bs_n;
    Ln.b += y * bs_n;
    if (out) out += y * NB;
  }
  const int i = PCR ? (int)blockIdx.x : 2 * (int)blockIdx.x;
  cr_wave_level<M, PCR, NB>(L, Ln, i, blockIdx.x, PCR ? s : 1, status, piv, smem);
  if (!PCR || !out) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's row stores have completed
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  double a[M];
  const bool ok = gj_wave<M, true, kCrPivot, NB>(Ln.D + (long long)i * M * M, nullptr, false, Ln.b + (long long)i * M * NB,
                                                 M + NB, lane, piv[0], a);
  if (!ok) {
    if (lane == 0) atomicOr(status, 1);
    return;
  }
  if (lane >= 2 * M && lane < 2 * M + NB)
#pragma unroll
    for (int r = 0; r < M; ++r)
      if (i * M + r < lim) out[((long long)i * M + r) * ld + (lane - 2 * M)] = a[r];
}

// The root super-row on one wave (lane 2M carries b; the coupling lanes are empty).
template <int M>
__global__ __launch_bounds__(64) void cr_root_wave_kernel(CrLevel L, int* status) {
  __shared__ __attribute__((aligned(16))) double piv[kPivBuf<M>];
  double a[M];
  const int lane = threadIdx.x;
  const bool ok = gj_wave<M>(L.D, nullptr, false, L.b, M + 1, lane, piv, a);
  if (!ok) {
    if (lane == 0) atomicOr(status, 1);
    return;
  }
  if (lane == 2 * M)
#pragma unroll
    for (int r = 0; r < M; ++r) L.x[r] = a[r];
}

// The last PCR level's decoupled rows: x_i = D_i⁻¹ b_i, one wave per row; x in the level-0 layout is the step itself
// (out = the step vector, lim = 6N), else the x of the CR level the PCR levels took over from.
template <int M, int NB = 1>
__global__ __launch_bounds__(64) void pcr_solve_kernel(CrLevel L, double* __restrict__ out, int lim, int* status,
                                                       int ld = 1) {
  __shared__ __attribute__((aligned(16))) double piv[kPivBuf<M>];
  const int lane = threadIdx.x, i = blockIdx.x;
  double a[M];
  const bool ok = gj_wave<M, false, kCrPivot, NB>(L.D + (long long)i * M * M, nullptr, false, L.b + (long long)i * M * NB,
                                                  M + NB, lane, piv, a);
  if (!ok) {
    if (lane == 0) atomicOr(status, 1);
    return;
  }
  if (lane >= 2 * M && lane < 2 * M + NB)
#pragma unroll
    for (int r = 0; r < M; ++r)
      if (i * M + r < lim) out[((long long)i * M + r) * ld + (lane - 2 * M)] = a[r];
}

// The root super-row (the last level): x = D⁻¹ b.
template <int M>
__global__ __launch_bounds__(kCrOddThreads<M>) void cr_root_kernel(CrLevel L, int* status) {
  constexpr int W = 3 * M + 1;
  __shared__ __attribute__((aligned(16))) double colk[2][2][M];
  double a[M];
  const bool ok = gj_row<M>(L, 0, true, threadIdx.x, colk, a);
  if (!ok) {  // uniform: every lane saw the same pivots
    if (threadIdx.x == 0) atomicOr(status, 1);
    return;
  }
  if ((int)threadIdx.x == W - 1)
#pragma unroll
    for (int r = 0; r < M; ++r) L.x[r] = a[r];
}

// Back-substitution, level L from level L+1: x_j = X_j^b − X_j^L x_{j−1} − X_j^U x_{j+1} for the odd rows, x of the
// even rows from the next level.  Level 0's x is the step δ itself (super-row I, element R ↔ block row
// I·B + R/6, component R%6), so it is written straight into the step vector.  The small levels at the bottom
// (n ≤ kCrTailRows) run in ONE workgroup with barriers between levels — one launch instead of one per level.
constexpr int kMaxCrLevels = 26;
constexpr int kCrTailRows = 32;
struct CrLevels {
  CrLevel lv[kMaxCrLevels];
  int nl;
};

template <int M>
__device__ __forceinline__ void cr_back_row(const CrLevel& L, const double* __restrict__ xn, double* out, int t) {
  constexpr int NC = 2 * M + 1;
  const int row = t / M, r = t % M;
  double v;
  if ((row & 1) == 0) {
    v = xn[(row / 2) * M + r];
  } else {
    const double* X = L.X + (long long)(row / 2) * M * NC + r * NC;
    v = X[2 * M];
    const double* xl = xn + ((row - 1) / 2) * M;
#pragma unroll 8
    for (int c = 0; c < M; ++c) v -= X[c] * xl[c];
    if (row + 1 < L.n) {
      const double* xr = xn + ((row + 1) / 2) * M;
#pragma unroll 8
      for (int c = 0; c < M; ++c) v -= X[M + c] * xr[c];
    }
  }
  out[t] = v;
}

// one (large) level, one lane per output
template <int M>
__global__ void cr_back_kernel(CrLevel L, const double* __restrict__ xn, double* __restrict__ out, int lim) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < lim) cr_back_row<M>(L, xn, out, t);
}

// levels hi … lo (all small) in one workgroup
template <int M>
__global__ __launch_bounds__(1024) void cr_back_tail_kernel(const CrLevels C, int hi, int lo, double* __restrict__ step,
                                                            int N) {
  for (int l = hi; l >= lo; --l) {
    const CrLevel& L = C.lv[l];
    double* out = l == 0 ? step : L.x;
    const int lim = l == 0 ? 6 * N : L.n * M;
    for (int t = threadIdx.x; t < lim; t += blockDim.x) cr_back_row<M>(L, C.lv[l + 1].x, out, t);
    __syncthreads();  // this level's x is read by the next (lower) level
  }
}

// ------------------------------------------------------------------------------------------------
// Free intrinsics as an arrow system (map_utils.h:339-345)
// ------------------------------------------------------------------------------------------------
// With free intrinsics the reduced camera system is S = [A B; Bᵀ C]: A the keyframes' band (bandwidth ≤ 4 keyframes), B
// the 2·nc border frames' coupling to every keyframe (dense columns), C the border's own 12nc × 12nc block.  The skyline
// factorisation (front_solve_kernel) walks the whole system column by column — one workgroup, ~3.5 µs per keyframe,
// 3.64 ms at C4.  Eliminating the keyframes first is the same factorisation order (border last), so instead:
//   X = A⁻¹ [−g_a | B]          parallel cyclic reduction over the band, the border's 12nc columns as extra right-hand
//                               sides (cr_level_wave_kernel<24, true, kArrowNB>: [D | U | b] = 24 + 24 + 16 lanes),
//                               in batches of kArrowNB columns run side by side (gridDim.y);
//   Sc = C − BᵀX_B,  rc = −g_c − BᵀX_0,  δc = Sc⁻¹ rc     (arrow_reduce_kernel: a workgroup per product;
//                               arrow_cap_kernel: one workgroup, dense Cholesky of the ≤ 48 × 48 border system);
//   δa = X_0 − X_B δc           (arrow_back_kernel).
// The skyline S stays the assembled system (pba_gn_reduced_system, the multi-GPU export read it), g its gradient.
constexpr int kArrowNB = 16;   // right-hand-side columns per cyclic-reduction run (2·24 + 16 = 64 lanes)
constexpr int kArrowMaxNc = 4; // border of ≤ 48 unknowns (arrow_cap_kernel's LDS system)

struct ArrowArgs {
  const double* S;       // skyline system (lower blocks; block (i, j) at (row[i] + j − first[i])·36, element r·6 + c)
  const int* first;
  const int* row;
  const double* g;       // gradient, 6 per system frame
  const uint8_t* fixed;  // constant keyframes (their border coupling is dropped: identity rows of S)
  CrLevel L0;            // level 0 of the band (D, U, b of kArrowNB columns)
  double* X;             // 6·nf rows × ldx: A⁻¹[−g_a | B]
  double* part;          // kArrowSeg × n_ent partial products (arrow_reduce_kernel)
  double* dc;            // the border step (12nc)
  double* x;             // the step, 6 per system frame
  int* status;
  int nf, nc, ldx, n_ent;
};

// Level 0 of the band (super-rows of 4 keyframes, identity padding past the last keyframe) and the batch's kArrowNB
// right-hand-side columns: global column 0 = −g_a, 1 + q = column q of B (border frame nf + q/6, component q % 6),
// B[6f + r][q] = S(border row, keyframe f)[q % 6][r].  Every batch's columns in one launch: batch bt's b at
// L0.b + bt·n·M·kArrowNB (the batches share level 0's D and U).
__device__ __forceinline__ void arrow_build(const ArrowArgs& a, int batches, long long tid) {
  constexpr int M = 24, B = 4, NB = kArrowNB;
  const int n = a.L0.n;
  if (tid == 0) *a.status = 0;
  auto blk = [&](int i, int j, int r, int c) -> double {  // S[6i + r][6j + c], i ≥ j, 0 outside the profile
    return j >= a.first[i] ? a.S[((long long)a.row[i] + (j - a.first[i])) * 36 + r * 6 + c] : 0.0;
  };
  const long long nDU = (long long)n * M * M;
  if (tid < 2 * nDU) {
    const bool isU = tid >= nDU;
    const long long e0 = isU ? tid - nDU : tid;
    const int I = (int)(e0 / (M * M)), e = (int)(e0 % (M * M)), R = e / M, C = e % M;
    const int i = I * B + R / 6, r = R % 6, c = C % 6;
    double v;
    if (!isU) {
      const int j = I * B + C / 6;
      if (i >= a.nf || j >= a.nf) v = (i == j && r == c) ? 1.0 : 0.0;
      else v = i >= j ? blk(i, j, r, c) : blk(j, i, c, r);
      a.L0.D[e0] = v;
    } else {
      const int j = (I + 1) * B + C / 6;
      a.L0.U[e0] = (I + 1 < n && i < a.nf && j < a.nf) ? blk(j, i, c, r) : 0.0;
    }
    return;
  }
  const long long t = tid - 2 * nDU;
  if (t >= (long long)batches * n * M * NB) return;
  const int q = (int)(t % NB), R = (int)((t / NB) % M), I = (int)((t / ((long long)NB * M)) % n);
  const int batch = (int)(t / ((long long)n * M * NB));
  const int i = I * B + R / 6, r = R % 6, gq = NB * batch + q;
  double v = 0.0;
  if (i < a.nf && !a.fixed[i]) {
    if (gq == 0) v = -a.g[6 * i + r];
    else if (gq <= 12 * a.nc) v = blk(a.nf + (gq - 1) / 6, i, (gq - 1) % 6, r);
  }
  a.L0.b[t] = v;
}
__global__ __launch_bounds__(256) void arrow_build_kernel(const ArrowArgs a, int batches) {
  arrow_build(a, batches, (long long)blockIdx.x * blockDim.x + threadIdx.x);
}

// kArrowSeg workgroups per product: entry e < nb(nb+1)/2 — (q1 ≥ q2) of BᵀX_B — then e − that: q1 of BᵀX_0 (nb = 12nc), a
// dot product over the T = 6nf keyframe rows; workgroup (e, g) takes segment g of the rows (thread k: rows k, k + 256, …
// of it; xor butterflies per wave, the four waves in order) → part[g·n_ent + e]; arrow_cap_kernel adds the kArrowSeg
// segments in order (a fixed order).
constexpr int kArrowSeg = 8;
__global__ __launch_bounds__(256) void arrow_reduce_kernel(const ArrowArgs a) {
  __shared__ double s_w[4];
  const int nb = 12 * a.nc, nsym = nb * (nb + 1) / 2, T = 6 * a.nf, e = blockIdx.x, g = blockIdx.y;
  const int t0 = (int)((long long)g * T / kArrowSeg), t1 = (int)((long long)(g + 1) * T / kArrowSeg);
  int q1, xc;
  if (e < nsym) {
    q1 = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
    while (q1 * (q1 + 1) / 2 > e) --q1;
    while ((q1 + 1) * (q1 + 2) / 2 <= e) ++q1;
    xc = 1 + (e - q1 * (q1 + 1) / 2);  // X column of q2
  } else {
    q1 = e - nsym;
    xc = 0;
  }
  const int p = a.nf + q1 / 6, c = q1 % 6;
  const double* Sp = a.S + (long long)a.row[p] * 36 + c * 6;  // border row p starts at frame 0
  double acc = 0.0;
  for (int tt = t0 + (int)threadIdx.x; tt < t1; tt += 256)
    acc += Sp[(long long)(tt / 6) * 36 + tt % 6] * a.X[(long long)tt * a.ldx + xc];
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) a.part[(long long)g * a.n_ent + e] = ((s_w[0] + s_w[1]) + s_w[2]) + s_w[3];
}

// The border system Sc = C − BᵀX_B, rc = −g_c − BᵀX_0, its elimination in LDS and δc = Sc⁻¹ rc (the border's part of
// the step); one workgroup.  (A one-wave form without workgroup barriers measured no faster: 15.4 → 17.0 µs at C4.)
__global__ __launch_bounds__(256) void arrow_cap_kernel(const ArrowArgs a) {
  constexpr int NBM = 12 * kArrowMaxNc;
  __shared__ double sc[NBM][NBM + 1];
  __shared__ double rc[NBM];
  __shared__ int bad;
  const int nb = 12 * a.nc, nsym = nb * (nb + 1) / 2, tid = threadIdx.x;
  if (tid == 0) bad = 0;
  for (int e = tid; e < a.n_ent; e += blockDim.x) {
    double acc = a.part[e];
    for (int g = 1; g < kArrowSeg; ++g) acc += a.part[(long long)g * a.n_ent + e];
    if (e < nsym) {
      int q1 = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
      while (q1 * (q1 + 1) / 2 > e) --q1;
      while ((q1 + 1) * (q1 + 2) / 2 <= e) ++q1;
      const int q2 = e - q1 * (q1 + 1) / 2;
      const int p1 = a.nf + q1 / 6, c1 = q1 % 6, p2 = a.nf + q2 / 6, c2 = q2 % 6;  // p1 ≥ p2
      const double C = a.S[((long long)a.row[p1] + (p2 - a.first[p1])) * 36 + c1 * 6 + c2];
      sc[q1][q2] = sc[q2][q1] = C - acc;
    } else {
      const int q1 = e - nsym;
      rc[q1] = -a.g[6 * (a.nf + q1 / 6) + q1 % 6] - acc;
    }
  }
  __syncthreads();
  // Gauss-Jordan on [Sc | rc] with one barrier per column (no serial triangular solves: a one-lane substitution paid an
  // LDS round trip per term, ~nb² of them — 30 µs at nb = 24): step k takes every row i ≠ k's columns j > k and rc,
  // a_ij −= a_ik·a_kj / a_kk; column k and row k are only read in step k, so the step needs no second barrier.  The
  // pivots are Gaussian elimination's (Sc is SPD: all positive), δc_i = rc_i / a_ii at the end.
  for (int k = 0; k < nb; ++k) {
    const double dkk = sc[k][k];
    if (tid == 0 && !(dkk > 0.0)) bad = 1;
    const double idk = 1.0 / fmax(dkk, 1e-300);
    const int m = nb - k;  // columns k + 1 … nb − 1, then rc
    for (int idx = tid; idx < nb * m; idx += blockDim.x) {
      const int i = idx / m, jj = idx - m * i;
      if (i == k) continue;
      const double f = sc[i][k] * idk;
      if (jj < m - 1) sc[i][k + 1 + jj] -= f * sc[k][k + 1 + jj];
      else rc[i] -= f * rc[k];
    }
    __syncthreads();
  }
  if (tid == 0 && bad) atomicOr(a.status, 2);
  __syncthreads();
  for (int q = tid; q < nb; q += blockDim.x) {
    const double v = rc[q] / fmax(sc[q][q], 1e-300);
    a.dc[q] = v;
    a.x[6 * a.nf + q] = v;
  }
}

// δa = X_0 − X_B δc, one lane per keyframe unknown.
__global__ __launch_bounds__(256) void arrow_back_kernel(const ArrowArgs a) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 6 * a.nf) return;
  const double* Xt = a.X + (long long)t * a.ldx;
  double v = Xt[0];
  for (int q = 0; q < 12 * a.nc; ++q) v -= Xt[1 + q] * a.dc[q];
  a.x[t] = v;
}

// ------------------------------------------------------------------------------------------------
// Updates: poses T·exp(δ) (se3.hpp:763-784) and back-substituted inverse distances
// ------------------------------------------------------------------------------------------------
__device__ void se3_exp_mul(const double* T, const double* d, double* out) {
  const double w0 = d[3], w1 = d[4], w2 = d[5];
  const double th2 = w0 * w0 + w1 * w1 + w2 * w2, th = sqrt(th2);
  double imag, real, A, B;
  if (th < 1e-10) {
    real = 1.0 - th2 / 8.0 + th2 * th2 / 384.0;
    imag = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0;
    A = 0.5;
    B = 1.0 / 6.0;
  } else {
    // one sincos of θ/2 (sin θ = 2 sc, 1 − cos θ = 2 s², the latter without cancellation) and one reciprocal of θ
    // instead of two sincos and three IEEE divisions: the candidate poses' fp64 chain is the update kernel's latency
    double sh, ch;
    sincos(0.5 * th, &sh, &ch);
    const double it = rcp_nr(th);
    real = ch;
    imag = sh * it;
    A = 2.0 * imag * imag;
    B = (th - 2.0 * sh * ch) * (it * it * it);
  }
  const double qx = imag * w0, qy = imag * w1, qz = imag * w2, qw = real;
  // V υ = υ + A ω×υ + B ω×(ω×υ)
  const double v0 = d[0], v1 = d[1], v2 = d[2];
  const double c0 = w1 * v2 - w2 * v1, c1 = w2 * v0 - w0 * v2, c2 = w0 * v1 - w1 * v0;
  const double cc0 = w1 * c2 - w2 * c1, cc1 = w2 * c0 - w0 * c2, cc2 = w0 * c1 - w1 * c0;
  const double tx = v0 + A * c0 + B * cc0, ty = v1 + A * c1 + B * cc1, tz = v2 + A * c2 + B * cc2;
  // T · exp(δ): q = q_T ⊗ q_δ (normalised), t = t_T + R_T t_δ
  const double ax = T[0], ay = T[1], az = T[2], aw = T[3];
  double rw = aw * qw - ax * qx - ay * qy - az * qz;
  double rx = aw * qx + ax * qw + ay * qz - az * qy;
  double ry = aw * qy + ay * qw + az * qx - ax * qz;
  double rz = aw * qz + az * qw + ax * qy - ay * qx;
  const double n = rsqrt_nr(rw * rw + rx * rx + ry * ry + rz * rz);  // (|q| ≈ 1: the seed + correction is ~1 ulp)
  double u0 = ay * tz - az * ty, u1 = az * tx - ax * tz, u2 = ax * ty - ay * tx;
  u0 += u0; u1 += u1; u2 += u2;
  out[0] = rx * n; out[1] = ry * n; out[2] = rz * n; out[3] = rw * n;
  out[4] = T[4] + tx + aw * u0 + (ay * u2 - az * u1);
  out[5] = T[5] + ty + aw * u1 + (az * u0 - ax * u2);
  out[6] = T[6] + tz + aw * u2 + (ax * u1 - ay * u0);
}


// Σ over the workgroup of N per-lane values and the max of one more, in a fixed order (xor butterflies in each wave,
// then the waves in order, as wg_reduce2): thread q < N stores sum q to *out[q], thread N the max to *out_max.  Every
// thread must call it.
template <int N>
__device__ __forceinline__ void wg_reduce_sum_max(double (&v)[N], double m, double* const (&out)[N], double* out_max) {
  __shared__ double s[N + 1][16];
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] += __shfl_xor(v[q], o, 64);
    m = fmax(m, __shfl_xor(m, o, 64));
  }
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
  if (l == 0) {
#pragma unroll
    for (int q = 0; q < N; ++q) s[q][w] = v[q];
    s[N][w] = m;
  }
  __syncthreads();
  if (threadIdx.x <= N) {  // one thread per sum, the waves in order
    const int q = threadIdx.x, nw = (int)(blockDim.x / 64);
    double x = 0.0;
    for (int i = 0; i < nw; ++i) x = q < N ? x + s[q][i] : fmax(x, s[N][i]);
    double* dst = out_max;
#pragma unroll
    for (int k = 0; k < N; ++k) dst = q == k ? out[k] : dst;
    *dst = x;
  }
}

// ib_data per GN block (free intrinsics, intr_rows_kernel): weighted fp64 rows J_i (2×8) | J_h (2×6) | J_t (2×6) | J_ρ (2) |
// r (2), and W_i = J_iᵀJ_ρ (8)
constexpr int kIbStride = 52;
constexpr int kIbJi = 0, kIbJh = 16, kIbJt = 28, kIbJr = 40, kIbR = 42, kIbWi = 44;

// The update workgroups' partials besides the model decrease (slot layout of red): Σ|x − x_new|² and Σ|x_new|² in the
// ambient parameter space (red2, two doubles per slot: Ceres' step_norm and x_norm, trust_region_minimizer.cc:706-726,
// :813-814) and max |x − (x ⊞ −g)| at the current state (gmax, one double per slot: gradient_max_norm,
// trust_region_minimizer.cc:287-299).  Constant frames and points without blocks are not parameters of the solve.
struct PoseUpdateArgs {
  const double* poses;
  const double* x;
  const double* g_dir;
  const double* Ddiag;
  const uint8_t* fixed;
  double* poses_new;
  double* red;
  double* red2;
  double* gmax;
  int n;                 // system frames: the keyframes, then two per camera with free intrinsics
  int nf;                // keyframes
  const double* kcur;    // free intrinsics: the state's camera records (projection part) …
  double* knew_d;        // … the candidate's (camera records) …
  float* knew_f;         // … and their fp32 copy (8 per camera)
};


// Frame i's update inputs, all loaded in one memory round (every dependent round trip is ~1.7 µs in these kernels):
// the pose, the step, the gradient direction, the LM diagonal and the constant flag.
struct FrameIn {
  double T[7], x[6], g[6], D[6];
  bool fixed;
};
__device__ __forceinline__ FrameIn frame_in(const PoseUpdateArgs& a, int i, bool grad) {
  FrameIn f;
  const double* P = a.poses + 7 * i;
#pragma unroll
  for (int q = 0; q < 7; ++q) f.T[q] = P[q];
  const double2* X = reinterpret_cast<const double2*>(a.x + 6 * i);
  const double2* G = reinterpret_cast<const double2*>(a.g_dir + 6 * i);
  const double2* Dd = reinterpret_cast<const double2*>(a.Ddiag + 6 * i);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double2 xv = X[q];
    f.x[2 * q] = xv.x;
    f.x[2 * q + 1] = xv.y;
    if (grad) {
      const double2 gv = G[q], dv = Dd[q];
      f.g[2 * q] = gv.x;
      f.g[2 * q + 1] = gv.y;
      f.D[2 * q] = dv.x;
      f.D[2 * q + 1] = dv.y;
    }
  }
  f.fixed = a.fixed[i] != 0;
  return f;
}
// candidate pose T·exp(δ), or T for a constant frame
__device__ __forceinline__ void candidate_pose(const FrameIn& f, double* out) {
  if (f.fixed) {
#pragma unroll
    for (int q = 0; q < 7; ++q) out[q] = f.T[q];
  } else {
    se3_exp_mul(f.T, f.x, out);
  }
}

// A free camera's intrinsics (system frames nf + 2c, nf + 2c + 1: dims 6h … 6h + 5 of the 8, the rest pads): k ← k + δ
// (a plain parameter block, no local parameterisation), with the same model-decrease, norm and gradient partials.
__device__ __forceinline__ void intr_update_frame(const PoseUpdateArgs& a, int i, double* v, double& gm) {
  const int c = (i - a.nf) >> 1, h = (i - a.nf) & 1;
  const bool fx = a.fixed[i] != 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int d = 6 * h + r;
    if (d >= 8) break;
    const double xk = a.x[6 * i + r], gk = a.g_dir[6 * i + r], Dk = a.Ddiag[6 * i + r];
    const double k = a.kcur[kCamD * c + d], kn = fx ? k : k + xk;
    a.knew_d[kCamD * c + d] = kn;
    a.knew_f[8 * c + d] = (float)kn;
    if (fx) continue;
    v[0] += xk * gk;
    v[1] += xk * xk * Dk;
    v[2] += (kn - k) * (kn - k);
    v[3] += kn * kn;
    gm = fmax(gm, fabs(gk));  // |k − (k − g)|
  }
}

__device__ __forceinline__ void pose_update_block(const PoseUpdateArgs& a, const LmView& lv, int blk) {
  const int i = blk * blockDim.x + threadIdx.x;
  double v[4] = {0.0, 0.0, 0.0, 0.0};  // x·g, x·D·x, |T − T_new|², |T_new|²
  double gm = 0.0;
  const FrameIn f = frame_in(a, min(i, a.nf - 1), true);  // in flight with the record's load; then the done test
  if (lv.done != 0.0) return;  // (uniform)
  if (i >= a.nf && i < a.n) {
    intr_update_frame(a, i, v, gm);
  } else if (i < a.n) {
    double tn[7];
    candidate_pose(f, tn);
    double* out = a.poses_new + 7 * i;
#pragma unroll
    for (int q = 0; q < 7; ++q) out[q] = tn[q];
    if (!f.fixed) {
      double ng[6], tg[7];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        v[0] += f.x[r] * f.g[r];
        v[1] += f.x[r] * f.x[r] * f.D[r];
        ng[r] = -f.g[r];
      }
      se3_exp_mul(f.T, ng, tg);  // Plus(x, −gradient)
#pragma unroll
      for (int q = 0; q < 7; ++q) {
        const double d = tn[q] - f.T[q];
        v[2] += d * d;
        v[3] += tn[q] * tn[q];
        gm = fmax(gm, fabs(f.T[q] - tg[q]));
      }
    }
  }
  double* const dst[4] = {a.red + 2 * blk, a.red + 2 * blk + 1, a.red2 + 2 * blk, a.red2 + 2 * blk + 1};
  wg_reduce_sum_max<4>(v, gm, dst, a.gmax + blk);
}

struct PointUpdateArgs {
  const double* pt_data;
  const double* pt_data1;  // the single-GPU LM loop: set 1's point data (schur_free_decide_kernel), else pt_data
  const int4* pt_rec;
  const int4* pt_tgt;
  const int* gn_target;
  const double* blk_schur;
  const double* blk_schur1;  // buffer set 1 (device LM loop)
  const double* x;
  const uint8_t* fixed;
  const double* rho;
  double* rho_new;
  double* drho;
  double* red;
  double* red2;
  double* gmax;
  int n_points;
  const double* pw;      // free intrinsics: per GN point its per-camera Σ W_i (ib_pw: intr_rows_kernel / intr_pw_kernel,
  int nc;                // 8·nc + 6 per point), the cameras and the keyframe count (the intrinsics steps start at
  int nf;                // x[6·nf], 12 per camera)
};

// blk: the point workgroup's index among the point workgroups; slot: its reduction slot
// lm: the LM record (done → return before any store; read with the point's first loads, not ahead of them)
__device__ __forceinline__ void point_update_block(const PointUpdateArgs& a, const double* lm, double lambda, int blk,
                                                   int slot) {
  const int p = blk * blockDim.x + threadIdx.x;
  double v[4] = {0.0, 0.0, 0.0, 0.0};  // δρ·g, δρ·D·δρ, δρ², ρ_new²
  double gm = 0.0;
  const LmView lv = lm_view(lm);
  const int pc = min(p, a.n_points - 1);
  const int4 pr = a.pt_rec[pc];  // first block, block count, host, original point
  const int4 pt4 = a.pt_tgt[pc];  // the targets of its first four blocks
  // both sets' point data with the record (which of them is current is the record's): no dependent round for the choice
  double pd[8], pd1[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double2 d2 = reinterpret_cast<const double2*>(a.pt_data + (long long)pc * 8)[i];
    const double2 e2 = reinterpret_cast<const double2*>(a.pt_data1 + (long long)pc * 8)[i];
    pd[2 * i] = d2.x;
    pd[2 * i + 1] = d2.y;
    pd1[2 * i] = e2.x;
    pd1[2 * i + 1] = e2.y;
  }
  if (lv.set != 0.0)
#pragma unroll
    for (int i = 0; i < 8; ++i) pd[i] = pd1[i];
  if (lv.done != 0.0) return;  // (uniform: every thread of the workgroup returns)
#ifdef PBA_UPD_STAMPS
  long long ts[4];
  ts[0] = wall_clock64();
#endif
  lambda = lm_lambda(lv, lambda);
  const double* blk_schur = lv.set != 0.0 ? a.blk_schur1 : a.blk_schur;
  if (p < a.n_points) {
    const double H = pd[0], gl = pd[1];
    const double D = fmin(fmax(H, 1e-6), 1e32);
    const double Hd = H + lambda * D;
    const int h = pr.z;
    // vector loads (16 B) and every load of a batch in flight before the first use: the target steps' loads used to sit
    // behind a data-dependent break (one memory round trip per block) and 4-B / 8-B scalar loads of scattered rows
    auto x6 = [&](int f, double* o) {
      const double2* q = reinterpret_cast<const double2*>(a.x + 6 * f);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const double2 d2 = q[i];
        o[2 * i] = d2.x;
        o[2 * i + 1] = d2.y;
      }
    };
    double xh[6];
    x6(h, xh);
    double s = gl;
    for (int i = 0; i < 6; ++i) s += pd[2 + i] * xh[i];
    const int fb = pr.x, nb = pr.y;
    constexpr int kBatch = 4;  // a batch's loads issued together, then summed in block order
    for (int b0 = fb; b0 < fb + nb; b0 += kBatch) {
      double w[kBatch][6];
      int t[kBatch];
      const bool first = b0 == fb;  // the first batch's targets came with the point record
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int b = min(b0 + u, fb + nb - 1);
        t[u] = first ? (u == 0 ? pt4.x : u == 1 ? pt4.y : u == 2 ? pt4.z : pt4.w) : a.gn_target[b];
        const double2* wt = reinterpret_cast<const double2*>(blk_schur + (long long)b * kPd + 2);  // W_t
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double2 q2 = wt[i];
          w[u][2 * i] = q2.x;
          w[u][2 * i + 1] = q2.y;
        }
      }
      double xt[kBatch][6];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) x6(t[u], xt[u]);
#pragma unroll
      for (int u = 0; u < kBatch; ++u)
        if (b0 + u < fb + nb)
#pragma unroll
          for (int i = 0; i < 6; ++i) s += w[u][i] * xt[u][i];
    }
    if (a.pw) {  // + Σ_b W_i(b)·δk(camera of b's target) = Σ_c W_c·δk_c from the point's camera sums (one load round,
                 // not a camera index then its step per block)
      const double* wc = a.pw + (long long)p * (8 * a.nc + 6);
      for (int c = 0; c < a.nc; ++c) {
        const double* xk = a.x + 6 * a.nf + 12 * c;
#pragma unroll
        for (int d = 0; d < 8; ++d) s += wc[8 * c + d] * xk[d];
      }
    }
#ifdef PBA_UPD_STAMPS
    ts[1] = wall_clock64();
#endif
    const double dr = Hd > 0.0 ? -s / Hd : 0.0;
    const int o = pr.w;
    const double rn = a.rho[o] + dr;
    a.rho_new[o] = rn;
    a.drho[o] = dr;
    v[0] = dr * gl;
    v[1] = dr * dr * D;
    v[2] = dr * dr;
    v[3] = rn * rn;
    gm = fabs(gl);  // ρ has no local parameterisation: |ρ − (ρ − g_ρ)|
  }
#ifdef PBA_UPD_STAMPS
  ts[2] = wall_clock64();
#endif
  double* const dst[4] = {a.red + 2 * slot, a.red + 2 * slot + 1, a.red2 + 2 * slot, a.red2 + 2 * slot + 1};
  wg_reduce_sum_max<4>(v, gm, dst, a.gmax + slot);
#ifdef PBA_UPD_STAMPS
  ts[3] = wall_clock64();
  if (threadIdx.x == 0 && (blk == 0 || blk == 196))
    printf("updpoint blk=%d loads %lld loop %lld stores %lld reduce %lld\n", blk, ts[0], ts[1] - ts[0], ts[2] - ts[1], ts[3] - ts[2]);
#endif
}

struct PairUpdateArgs {
  const int4* pair_rec;  // {host, target, host camera, target camera}
  const double* cams;
  PairRec* pairs_new;  // nullptr: no candidate pair table (geometric engines form theirs in the cost path too)
  int n_pairs;
};

// The step's candidate state in ONE launch: workgroups [0, gp) update the poses (T·exp(δ)) and reduce the pose part
// of the model decrease, [gp, gp + gq) back-substitute the inverse distances and reduce the point part (partial slots
// in the same fixed order as two separate launches), and the rest form the candidate pair table straight from
// T_h·exp(δ_h), T_t·exp(δ_t) — candidate_pose, the same arithmetic as the pose workgroups, so the pairs equal
// form_pair(poses_new) bit for bit — which saves the separate pair launch before the candidate cost.
__global__ __launch_bounds__(kBlockThreads) void update_kernel(const PoseUpdateArgs pa, PointUpdateArgs qa,
                                                               const PairUpdateArgs ra, int gp, int gq, double lambda,
                                                               const double* __restrict__ lm) {
  // gated: a trial after the end must not touch the last step (pba_gn_get_step).  Each part tests the record after
  // its own first loads are issued (a test ahead of them cost a memory round trip of its own)
  const int b = blockIdx.x;
#ifdef PBA_UPD_STAMPS  // timing dissection only: absolute 100-MHz stamps at the start and end of chosen workgroups
  const long long t0 = wall_clock64();
  struct Stamp {
    long long t0;
    int b;
    __device__ ~Stamp() {
      if (threadIdx.x == 0 && (b == 0 || b == 4 || b == 200 || b == 394 || b == 395 || b == 410))
        printf("updstamp b=%d start %lld end %lld\n", b, t0, wall_clock64());
    }
  } stamp{t0, b};
#endif
  if (b >= gp && b < gp + gq) {
    point_update_block(qa, lm, lambda, b - gp, b);
    return;
  }
  const LmView lv = lm_view(lm);
  if (b < gp) {
    pose_update_block(pa, lv, b);
  } else {
    // two memory rounds: the pair record, then both frames' inputs and both cameras' constants together
    const int i = (b - gp - gq) * blockDim.x + threadIdx.x;
    const int4 pr = ra.pair_rec[min(i, ra.n_pairs - 1)];
    const FrameIn fh = frame_in(pa, pr.x, false), ft = frame_in(pa, pr.y, false);
    double hk[kCamK], tk[kCamK];
#pragma unroll
    for (int j = 0; j < kCamK; ++j) {
      hk[j] = ra.cams[kCamD * pr.z + kCamHk + j];
      tk[j] = ra.cams[kCamD * pr.w + j];
    }
    if (lv.done != 0.0 || i >= ra.n_pairs) return;
    double H[7], T[7];
    candidate_pose(fh, H);
    candidate_pose(ft, T);
    PairRec r;
    pair_rotation(H, T, r);
    pair_translation(H, T, r);
    r.host_cam = pr.z;
    r.target_cam = pr.w;
    r.target = pr.y;
    r.host = pr.x;
#pragma unroll
    for (int j = 0; j < kCamK; ++j) {
      r.hk[j] = hk[j];
      r.tk[j] = tk[j];
    }
    camera_kf(tk, r.kf);
    ra.pairs_new[i] = r;
  }
}

// ------------------------------------------------------------------------------------------------
// Free intrinsics in the reduced camera system (pba_set_optimize_intrinsics; geometric engines)
// ------------------------------------------------------------------------------------------------
// bundle_adjustment() with BundleAdjustmentOptions::optimize_intrinsics leaves the cameras' 8-vector intrinsics blocks
// free (map_utils.h:339-345); the functor differentiates the TARGET camera's intrinsics (reprojection.h:83-86, :108) and
// SPARSE_SCHUR keeps those blocks among the f-blocks of the reduced camera system (schur_complement_solver.cc:138-146).
// Here camera c's intrinsics are the system frames nf + 2c (dims 0-5) and nf + 2c + 1 (dims 6-7, then four identity
// pads): a dense border of the skyline system (their profile starts at frame 0).  The keyframe part is linearised,
// eliminated and assembled as without intrinsics; the border — the blocks' direct terms J_iᵀJ_x and the points' Schur
// terms −W_i,c W_xᵀ / H'_ρρ — is formed in fp64 by the border kernels below (a wave per keyframe block, camera blocks
// split over workgroups) in a fixed order (the CSR lists of gn_prepare), from weighted fp64 rows (intr_rows_kernel) and
// schur_kernel's undamped H_ρρ; on several GPUs each rank exports its border rows undamped (import_sky_kernel sums them).
struct IntrRowsArgs {
  const int4* rec;       // GN block → {block, point, host, target}
  const double* poses;
  const double* rho;
  const double2* u_ref;
  const double2* u_obs;
  const int* frame_cam;
  const double* cams;    // host unprojection: the cameras (the functor's captured intrinsics, reprojection.h:93-98)
  const double* kt;      // target projection: the intrinsics state (camera records)
  double huber;
  double* out;           // ib_data
  int n;
  const double* lm;      // LM record: nothing to do once the solve is done
  // point-aligned waves (gn_prepare, every GN point ≤ 64 blocks): wave w takes GN blocks wave_tab[w].x … + .y − 1, whole
  // points from GN point wave_tab[w].z on, and also writes their W sums into pw (intr_pw_kernel's work); else nullptr
  const int4* wave_tab = nullptr;
  int n_waves = 0;
  double* pw = nullptr;
  int nc = 0;
};
struct PoseT {  // a relative pose for pair_rotation / pair_translation
  double R[9], t[3];
  float Rf[9], tf[3];
};

// One lane per GN block at the current state: r = u_obs − π_t(T_th b/ρ) and its Jacobians (the geometric_row chain, in
// fp64), J_i = −∂π/∂k (project_intr_jac), Ceres' Corrector weighting √ρ' (corrector.cc, ρ'' ≤ 0 for Huber), W_i = J_iᵀJ_ρ.
// The rows leave through LDS (PBA_IB_DIRECT: straight from the lanes): a lane's 416-B row stored from registers is 26
// 16-B stores 416 B apart per instruction — 64 partial lines each — so each wave stages its 64 rows in two halves of 26
// doubles and stores every half as the 13 16-B chunks of each row, consecutive lanes on consecutive chunks.
#ifndef PBA_IB_DIRECT
constexpr int kIbStage = 27;  // doubles per staged half row (26 used; odd: 2-way LDS bank conflicts at most)
#endif
template <int MODEL>
__global__ __launch_bounds__(256) void intr_rows_kernel(const IntrRowsArgs a) {
  const int lane = threadIdx.x & 63;
#ifdef PBA_IB_DIRECT
  const int gb0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (gb0 >= a.n || lm_view(a.lm).done != 0.0) return;
  const int gb = gb0;
#else
  // the wave's rows: 64 consecutive GN blocks, or (wave_tab) a point-aligned run of ≤ 64
  int row0, nrow;
  int4 wt = make_int4(0, 0, 0, 0);
  if (a.wave_tab) {
    const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= a.n_waves) return;  // (whole waves)
    wt = a.wave_tab[w];
    row0 = wt.x;
    nrow = wt.y;
  } else {
    row0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63);
    nrow = min(64, a.n - row0);
  }
  if (lm_view(a.lm).done != 0.0) return;       // (uniform)
  const int gb = row0 + max(min(lane, nrow - 1), 0);  // every lane of a wave takes part in its stores
#endif
  const int4 br = a.rec[gb];
  PoseT T;
  pair_rotation(a.poses + 7 * br.z, a.poses + 7 * br.w, T);
  pair_translation(a.poses + 7 * br.z, a.poses + 7 * br.w, T);
  const int hc = a.frame_cam[br.z], tc = a.frame_cam[br.w];
  const double* kt = a.kt + kCamD * tc;
  const double2 ur = a.u_ref[br.y], uo = a.u_obs[br.x];
  const double irho = 1.0 / a.rho[br.y];
  const Vec3d b = unproject<MODEL>(a.cams + kCamD * hc + kCamHk, ur.x, ur.y);
  const Vec3d ph = {b.x * irho, b.y * irho, b.z * irho};
  const Vec3d Rp = mat_mul(T.R, ph);
  const Vec3d p = {Rp.x + T.t[0], Rp.y + T.t[1], Rp.z + T.t[2]};
  double u, v;
  const double iden = project<MODEL>(kt, p, u, v);
  double J[kIbStride];
  J[kIbR] = uo.x - u;
  J[kIbR + 1] = uo.y - v;
  Vec3d du, dv;
  project_jac<MODEL>(kt, p, iden, du, dv);
  double ku[8], kv[8];
  project_intr_jac<MODEL>(kt, p, iden, ku, kv);
  const Vec3d td = {T.t[0], T.t[1], T.t[2]};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const Vec3d d = i == 0 ? du : dv;
    const Vec3d g = {-d.x, -d.y, -d.z};  // ∂r/∂p = −∂π/∂p
    const Vec3d gR = row_mul(g, T.R);
    const Vec3d wh = cross(ph, gR);
    const Vec3d wt = cross(g, p);
    double* jh = J + kIbJh + 6 * i;
    double* jt = J + kIbJt + 6 * i;
    jh[0] = gR.x; jh[1] = gR.y; jh[2] = gR.z; jh[3] = wh.x; jh[4] = wh.y; jh[5] = wh.z;
    jt[0] = -g.x; jt[1] = -g.y; jt[2] = -g.z; jt[3] = wt.x; jt[4] = wt.y; jt[5] = wt.z;
    J[kIbJr + i] = dot(g, td) * irho;
#pragma unroll
    for (int j = 0; j < 8; ++j) J[kIbJi + 8 * i + j] = -(i == 0 ? ku[j] : kv[j]);
  }
  bool ok = true;
#pragma unroll
  for (int q = 0; q < kIbWi; ++q) ok = ok && isfinite(J[q]);
  const double s2 = J[kIbR] * J[kIbR] + J[kIbR + 1] * J[kIbR + 1], hb = a.huber;
  const double w = (hb <= 0.0 || s2 <= hb * hb) ? 1.0 : hb / sqrt(s2);
  const double sw = ok ? sqrt(w) : 0.0;
#pragma unroll
  for (int q = 0; q < kIbWi; ++q) J[q] = ok ? sw * J[q] : 0.0;
#pragma unroll
  for (int d = 0; d < 8; ++d) J[kIbWi + d] = J[kIbJi + d] * J[kIbJr] + J[kIbJi + 8 + d] * J[kIbJr + 1];
#ifdef PBA_IB_DIRECT
  double* o = a.out + (long long)gb * kIbStride;
#pragma unroll
  for (int q = 0; q < kIbStride; q += 2) *reinterpret_cast<double2*>(o + q) = make_double2(J[q], J[q + 1]);
#else
  constexpr int HALF = kIbStride / 2, CH = HALF / 2;  // 26 doubles, 13 chunks of 16 B per half row
  __shared__ double stage[4][64 * kIbStage];
  double* st = stage[threadIdx.x >> 6];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int q = 0; q < HALF; ++q) st[lane * kIbStage + q] = J[HALF * h + q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int c0 = 0; c0 < 64 * CH; c0 += 64) {
      const int c = c0 + lane, r = c / CH, j = c - CH * r;
      if (r < nrow)
        *reinterpret_cast<double2*>(a.out + (long long)(row0 + r) * kIbStride + HALF * h + 2 * j) =
            make_double2(st[r * kIbStage + 2 * j], st[r * kIbStage + 2 * j + 1]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // this half's reads before the next half's writes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (!a.wave_tab) return;
  // the points' W sums (intr_pw_kernel's, in the same block order): each block's W_i, J_hᵀJ_ρ and camera through the
  // stage, then the first block of every point adds its point's blocks
  const int cam = a.frame_cam[br.w];
#pragma unroll
  for (int d = 0; d < 8; ++d) st[lane * kIbStage + d] = J[kIbWi + d];
#pragma unroll
  for (int k = 0; k < 6; ++k)
    st[lane * kIbStage + 8 + k] = J[kIbJh + k] * J[kIbJr] + J[kIbJh + 6 + k] * J[kIbJr + 1];
  st[lane * kIbStage + 14] = (double)cam;
  const bool live = lane < nrow;
  const int prev_pt = __shfl(br.y, (lane + 63) & 63, 64);
  const unsigned long long firsts = __ballot(live && (lane == 0 || br.y != prev_pt));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (!((firsts >> lane) & 1ull)) return;
  const unsigned long long later = lane == 63 ? 0ull : firsts >> (lane + 1);
  const int nb = later ? __builtin_ctzll(later) + 1 : nrow - lane;  // this point's blocks: lanes lane … lane + nb − 1
  const int gp = wt.z + __popcll(firsts & ((1ull << lane) - 1ull));
  double* o = a.pw + (long long)gp * (8 * a.nc + 6);
  double wh[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int c0 = 0; c0 < a.nc; c0 += 4) {  // cameras in groups of four, as intr_pw_kernel
    double wc[4][8];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int d = 0; d < 8; ++d) wc[c][d] = 0.0;
    for (int b = lane; b < lane + nb; ++b) {
      const double* sb = st + b * kIbStage;
      const int cb = (int)sb[14] - c0;
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const double w = sb[d];
#pragma unroll
        for (int c = 0; c < 4; ++c) wc[c][d] += c == cb ? w : 0.0;
      }
      if (c0 == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) wh[k] += sb[8 + k];
    }
    for (int c = 0; c < 4 && c0 + c < a.nc; ++c)
#pragma unroll
      for (int d = 0; d < 8; ++d) o[8 * (c0 + c) + d] = wc[c][d];
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) o[8 * a.nc + k] = wh[k];
#endif
}

struct IntrBorderArgs {
  const double* ib;        // ib_data
  const int4* ib_rec;      // GN block → {block, point, host, target}
  const int* ib_cam;       // GN block → its target's camera
  const int4* pt_rec;      // GN point → {first GN block, block count, host, point}
  const double* pt_data;   // GN point → [H_ρρ (undamped), g_ρ, …] (schur_kernel of this solve)
  const int* bptr;         // border unit pair (c, u) = c·(nf + nc) + u → direct-term GN blocks …
  const int* blist;        // (keyframe units: bit 31 set when the keyframe hosts the block)
  const int* pptr;         // … and Schur-term GN points
  const int* plist;
  const int* sky_first;
  const int* sky_row;
  const uint8_t* fixed;    // system frames
  const double* lm;
  double* S;
  double* g;
  double* g_dir;
  double* Ddiag;
  int nf, nc;
  double* X = nullptr;     // multi-GPU export (pba_gn_step_export): this rank's border rows, undamped, into the exchange
  long long xs = 0;        // buffer's border region (row stride nfs·36 + EX_TAIL) instead of S
  const double* pw = nullptr;  // GN point → its camera sums W_c (8 per camera) and W_h = Σ J_hᵀJ_ρ (6): intr_pw_kernel
  const int* pblk = nullptr;   // per plist entry of a keyframe unit: −1 the keyframe hosts the point, else the point's
                               // one block targeting it (−2: several — walk the point's blocks)
};

// Per GN point, over its blocks in order: W_c = Σ_{b: camera(b) = c} W_i(b) for every camera c, and W_h = Σ_b J_h(b)ᵀJ_ρ(b)
// (every block of a point has the point's host).  The border kernels' Schur terms read these 8·nc + 6 values instead of
// walking the point's blocks (4-5 × 52 doubles) once per (point, list) — at C4 that walk re-read the blocks' rows five
// times per kernel, ≈ 0.4 GB per launch.  The same sums in the same order: the border is unchanged bit for bit.
__global__ __launch_bounds__(256) void intr_pw_kernel(const IntrBorderArgs a, int n_points) {
  // 8 lanes per point: lane k sums component k of every camera's W_c and (k < 6) of W_h, over the blocks in order
  const int t = blockIdx.x * blockDim.x + threadIdx.x, gp = t >> 3, k = t & 7;
  if (gp >= n_points) return;
  const int4 pr = a.pt_rec[gp];
  const int st = 8 * a.nc + 6;
  double* o = const_cast<double*>(a.pw) + (long long)gp * st;
  double wh = 0.0;
  for (int c0 = 0; c0 < a.nc; c0 += 4) {  // cameras in groups of four (one pass over the blocks per group)
    double wc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int b = pr.x; b < pr.x + pr.y; ++b) {
      const double* B = a.ib + (long long)b * kIbStride;
      const int cb = a.ib_cam[b] - c0;
      const double w = B[kIbWi + k];
#pragma unroll
      for (int c = 0; c < 4; ++c) wc[c] += c == cb ? w : 0.0;
      if (c0 == 0 && k < 6) wh += B[kIbJh + k] * B[kIbJr] + B[kIbJh + 6 + k] * B[kIbJr + 1];
    }
    for (int c = 0; c < 4 && c0 + c < a.nc; ++c) o[8 * (c0 + c) + k] = wc[c];
  }
  if (k < 6) o[8 * a.nc + k] = wh;
}

// Element t of border row `row` (system frame P = nf + row): t < (P + 1)·36 → entry (r, cc) of block (P, y = t / 36) of
// the skyline system; t = nfs·36 … nfs·36 + 5 → g of P.  The keyframe blocks (P, x < nf) and the camera blocks (P, y ≥ nf)
// get direct − Schur terms, + λ·clamp(diag) on the diagonal (the direct part is Ceres' LM diagonal), identity pads, and
// — constant frames / unobserved cameras — identity rows and columns, as assemble_kernel.  border_store writes element t
// from its two totals (direct, Schur).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ double border_inv(const IntrBorderArgs& a, int gp, double lambda) {
  const double H = a.pt_data[(long long)gp * 8];
  const double Hd = H + lambda * fmin(fmax(H, 1e-6), 1e32);
  return Hd > 0.0 ? 1.0 / Hd : 0.0;
}
__device__ __forceinline__ void border_store(const IntrBorderArgs& a, double lambda, int row, int t, double dir,
                                             double sch) {
  const int P = a.nf + row, nfs = a.nf + 2 * a.nc, h = row & 1;
  if (a.X) {  // export: direct − Schur, the direct diagonal, g, the direct gradient, observed (import_sky_kernel damps,
              // pads and fixes the summed rows)
    double* xr = a.X + (long long)row * a.xs;
    double* tail = xr + (long long)nfs * 36;
    if (t >= nfs * 36) {
      const int r = t - nfs * 36;
      tail[r] = dir - sch;
      tail[6 + r] = dir;
      if (r == 0) tail[18] = a.fixed[P] ? 0.0 : 1.0;  // a camera this rank observes
      return;
    }
    const int y = t / 36, e = t % 36, r = e / 6, cc = e % 6, d = 6 * h + r;
    const int d2 = y >= a.nf ? 6 * ((y - a.nf) & 1) + cc : cc;
    const bool pad = d >= 8 || d2 >= 8;
    xr[(long long)y * 36 + e] = pad ? 0.0 : dir - sch;
    if (y == P && r == cc) tail[12 + r] = pad ? 0.0 : dir;
    return;
  }
  if (t >= nfs * 36) {
    const int r = t - nfs * 36;
    const bool fx = a.fixed[P] != 0;
    a.g[6 * P + r] = fx ? 0.0 : dir - sch;
    a.g_dir[6 * P + r] = fx ? 0.0 : dir;
    if (fx) a.Ddiag[6 * P + r] = 0.0;
    return;
  }
  const int y = t / 36, e = t % 36, r = e / 6, cc = e % 6, d = 6 * h + r;
  const bool cam = y >= a.nf;
  const int d2 = cam ? 6 * ((y - a.nf) & 1) + cc : cc;
  if (d >= 8 || d2 >= 8) {  // pad
    dir = (y == P && r == cc) ? 1.0 : 0.0;
    sch = 0.0;
  }
  double val = dir - sch;
  if (a.fixed[P] || a.fixed[y]) {
    val = (y == P && r == cc) ? 1.0 : 0.0;
  } else if (y == P && r == cc) {
    const double D = fmin(fmax(dir, 1e-6), 1e32);  // levenberg_marquardt_strategy.cc: the undamped JᵀJ diagonal
    a.Ddiag[6 * P + r] = D;
    val += lambda * D;
  }
  a.S[((long long)a.sky_row[P] + (y - a.sky_first[P])) * 36 + e] = val;
}

// Σ over the wave of 48 per-lane values v[0 … 47] by recursive halving (a reduce-scatter: 24 + 12 + 6 + 3 + 6 shuffles
// instead of 48 six-step butterflies): after the xor-32 / 16 / 8 / 4 steps lane l holds partial sums of the three values
// base(l) … base(l) + 2, base = 24·b5 + 12·b4 + 6·b3 + 3·b2 of l's bits, completed over its quad by xor 2 and xor 1 (a + b
// and b + a: the quad's lanes agree bit for bit).  Returns the total of value *vi = base(l) + (l & 3) for l & 3 < 3
// (*vi = −1 and 0 otherwise).  A fixed order.
__device__ __forceinline__ double wave_rs48(const double (&v)[48], int lane, int* vi) {
  double a24[24], a12[12], a6[6], a3[3];
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8, h2 = lane & 4;
#pragma unroll
  for (int i = 0; i < 24; ++i) a24[i] = (h5 ? v[24 + i] : v[i]) + __shfl_xor(h5 ? v[i] : v[24 + i], 32, 64);
#pragma unroll
  for (int i = 0; i < 12; ++i) a12[i] = (h4 ? a24[12 + i] : a24[i]) + __shfl_xor(h4 ? a24[i] : a24[12 + i], 16, 64);
#pragma unroll
  for (int i = 0; i < 6; ++i) a6[i] = (h3 ? a12[6 + i] : a12[i]) + __shfl_xor(h3 ? a12[i] : a12[6 + i], 8, 64);
#pragma unroll
  for (int i = 0; i < 3; ++i) a3[i] = (h2 ? a6[3 + i] : a6[i]) + __shfl_xor(h2 ? a6[i] : a6[3 + i], 4, 64);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    a3[i] += __shfl_xor(a3[i], 2, 64);
    a3[i] += __shfl_xor(a3[i], 1, 64);
  }
  const int j = lane & 3;
  *vi = j < 3 ? 24 * h5 + 12 * h4 + 6 * h3 + 3 * h2 + j : -1;
  return j == 0 ? a3[0] : j == 1 ? a3[1] : j == 2 ? a3[2] : 0.0;
}

// The keyframe blocks (P, y < nf) of both border rows of a camera: kpw WAVES per keyframe y (grid x: 4/kpw keyframes per
// workgroup; y: camera c) form the 8 × 6 live entries of (2c, y) and (2c + 1, y) — row 2c + 1's frame holds intrinsics 6,
// 7 and four pads — at once: a lane takes every (64·kpw)th entry of the keyframe's lists (its blocks and points seen by
// the camera), each wave adds its lanes' sums (wave_rs48) and the kpw waves' sums are added in order (a fixed order).
// kpw = 4 while the keyframe waves would not fill the SIMDs (C3, 200 keyframes), else 2 (C4: 2008 waves; 1 and 4 measured
// 80.5 and 82.4 against 76.5 µs).  Round 5 walked the lists twice (one kernel per border row: 133 + 117 µs at C4) and
// each point's blocks once per (point, list).
__device__ __forceinline__ void border_keyframes(const IntrBorderArgs& a, double lambda, int kpw, int bx, int by) {
  __shared__ double2 s_w[4][48];
  lambda = lm_lambda(lm_view(a.lm), lambda);
  const int c = by, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gw = bx * 4 + w, y0 = gw / kpw, sub = gw % kpw;
  const int y = min(y0, a.nf - 1);  // (a wave past the last keyframe walks nothing and stores nothing)
  const int L = c * (a.nf + a.nc) + y;
  const int q0 = sub * 64 + lane, dq = y0 < a.nf ? 64 * kpw : 1 << 30;
  // the 8 intrinsics rows d of camera c (border rows 2c: d = 0…5, 2c + 1: d = 6, 7) × the keyframe's 6 columns, value
  // v = 6d + cc; the direct terms first, then the Schur terms in the same registers; lane l ends with value vi (wave_rs48)
  double acc[8][6];
#pragma unroll
  for (int d = 0; d < 8; ++d)
#pragma unroll
    for (int cc = 0; cc < 6; ++cc) acc[d][cc] = 0.0;
  // the next entry's list index is loaded during this one (a list walk was two dependent memory rounds per entry: the
  // index, then the row — and the host / target test on the block record before the row's Jacobian)
  const int qb = a.bptr[L + 1];
  int q = a.bptr[L] + (y0 < a.nf ? q0 : 1 << 30);
  int bn = q < qb ? a.blist[q] : 0;
  for (; q < qb; q += dq) {
    const int bf = bn;
    if (q + dq < qb) bn = a.blist[q + dq];
    const double* B = a.ib + (long long)(bf & 0x7fffffff) * kIbStride;
    const double* Jc = B + (bf < 0 ? kIbJh : kIbJt);
    double c0[6], c1[6];
#pragma unroll
    for (int cc = 0; cc < 6; ++cc) {
      c0[cc] = Jc[cc];
      c1[cc] = Jc[6 + cc];
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const double j0 = B[kIbJi + d], j1 = B[kIbJi + 8 + d];
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) acc[d][cc] += j0 * c0[cc] + j1 * c1[cc];
    }
  }
  int vi;
  double vd = wave_rs48(reinterpret_cast<const double(&)[48]>(acc), lane, &vi);
#pragma unroll
  for (int d = 0; d < 8; ++d)
#pragma unroll
    for (int cc = 0; cc < 6; ++cc) acc[d][cc] = 0.0;
  const int qp = a.pptr[L + 1];
  q = a.pptr[L] + (y0 < a.nf ? q0 : 1 << 30);
  int gpn = q < qp ? a.plist[q] : 0, byn = q < qp ? a.pblk[q] : -1;
  for (; q < qp; q += dq) {
    const int gp = gpn, by = byn;
    if (q + dq < qp) {
      gpn = a.plist[q + dq];
      byn = a.pblk[q + dq];
    }
    double wc[8], wy[6];  // W of the point for camera c (Σ W_i over its blocks seen by c, intr_pw_kernel) and for
                          // keyframe y (Σ J_h / J_t ᵀJ_ρ over its blocks hosted / targeted by y)
    const double* pw = a.pw + (long long)gp * (8 * a.nc + 6);
#pragma unroll
    for (int d = 0; d < 8; ++d) wc[d] = pw[8 * c + d];
    if (by == -1) {  // y hosts the point: every block's J_hᵀJ_ρ (intr_pw_kernel)
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) wy[cc] = pw[8 * a.nc + cc];
    } else if (by >= 0) {  // y is a target: the point's block targeting it
      const double* B = a.ib + (long long)by * kIbStride;
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) wy[cc] = 0.0 + (B[kIbJt + cc] * B[kIbJr] + B[kIbJt + 6 + cc] * B[kIbJr + 1]);
    } else {  // several blocks of the point target y: their sum, in block order
      const int4 pr = a.pt_rec[gp];
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) wy[cc] = 0.0;
      for (int b = pr.x; b < pr.x + pr.y; ++b) {
        if (a.ib_rec[b].w != y) continue;
        const double* B = a.ib + (long long)b * kIbStride;
#pragma unroll
        for (int cc = 0; cc < 6; ++cc) wy[cc] += B[kIbJt + cc] * B[kIbJr] + B[kIbJt + 6 + cc] * B[kIbJr + 1];
      }
    }
    const double inv = border_inv(a, gp, lambda);
#pragma unroll
    for (int d = 0; d < 8; ++d)
#pragma unroll
      for (int cc = 0; cc < 6; ++cc) acc[d][cc] += inv * wc[d] * wy[cc];
  }
  double vs = wave_rs48(reinterpret_cast<const double(&)[48]>(acc), lane, &vi);
  if (kpw > 1) {  // the keyframe's kpw waves, in order
    if (vi >= 0) s_w[w][vi] = make_double2(vd, vs);
    __syncthreads();
    if (sub == 0 && vi >= 0) {
      double2 t = s_w[w][vi];
      for (int k = 1; k < kpw; ++k) {
        t.x += s_w[w + k][vi].x;
        t.y += s_w[w + k][vi].y;
      }
      vd = t.x;
      vs = t.y;
    }
    if (sub != 0) return;  // (whole waves)
  }
  // row 2c: values 0 … 35 (element v); row 2c + 1: values 36 … 47 (d = 6, 7) as its elements 0 … 11, its elements
  // 12 … 35 pads (border_store) from lanes 12 … 35
  if (y0 < a.nf) {
    if (vi >= 0) border_store(a, lambda, vi < 36 ? 2 * c : 2 * c + 1, y * 36 + (vi < 36 ? vi : vi - 36), vd, vs);
    if (lane >= 12 && lane < 36) border_store(a, lambda, 2 * c + 1, y * 36 + lane, 0.0, 0.0);
  }
}

// The camera blocks (P = nf + 2c + h, y = nf + 2c2 + h2 ≥ nf, c2 ≤ c) and the gradient rows of the border, as two
// reductions over whole lists instead of one list walk per (border row, column block) — the list of a camera holds ALL
// of its blocks (400k at C4) and points (100k), and round 5 walked it six times per trial (two row kernels × three column
// blocks, 165 µs at C4 with the finishing kernel):
//   cam_dir — per camera c, over its blocks: Σ J_iᵀJ_i (the 8 × 8 upper triangle, 36) and Σ J_iᵀr (8): the
//     direct terms (a block's intrinsics Jacobian is its target camera's, so the direct part couples a camera only with
//     itself);
//   cam_sch — per camera pair (c, c2 ≤ c), over the points seen by both: Σ_p W_c W_c2ᵀ / H'_ρρ (8 × 8) and,
//     for c2 = c, Σ_p W_c g_ρ / H'_ρρ (8): the Schur terms (W_c from intr_pw_kernel);
// each over kCamSplit workgroups (a thread takes every (256·kCamSplit)th entry; wave butterflies, then the four waves in
// order), and intr_cam_fin_kernel adds the kCamSplit totals in order per element and stores it (border_store) — a fixed
// order end to end.
constexpr int kCamSplit = 128;  // (512 measured no faster at C4, 2.7× slower for two cameras' Schur sums at C3)
constexpr int kCamDir = 44, kCamSch = 72;  // accumulators per thread

__device__ __forceinline__ int upper8i(int i, int j) { return i * 8 - i * (i - 1) / 2 + (j - i); }  // i ≤ j < 8

// Σ over the wave of N per-lane values (N a multiple of 16) into dst[0 … N) by recursive halving, as wave_rs48: after the
// xor-32 / 16 / 8 / 4 steps lane l holds partial sums of values base(l) … base(l) + N/16 − 1 (base = N/2·b5 + N/4·b4 +
// N/8·b3 + N/16·b2), completed over its quad by xor 2 and xor 1; the quad's lanes store them.  A fixed order.
template <int N>
__device__ __forceinline__ void wave_rs_lds(const double (&v)[N], int lane, double* dst) {
  static_assert(N % 16 == 0, "four halvings");
  constexpr int H1 = N / 2, H2 = N / 4, H3 = N / 8, H4 = N / 16;
  double a1[H1], a2[H2], a3[H3], a4[H4];
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8, h2 = lane & 4;
#pragma unroll
  for (int i = 0; i < H1; ++i) a1[i] = (h5 ? v[H1 + i] : v[i]) + __shfl_xor(h5 ? v[i] : v[H1 + i], 32, 64);
#pragma unroll
  for (int i = 0; i < H2; ++i) a2[i] = (h4 ? a1[H2 + i] : a1[i]) + __shfl_xor(h4 ? a1[i] : a1[H2 + i], 16, 64);
#pragma unroll
  for (int i = 0; i < H3; ++i) a3[i] = (h3 ? a2[H3 + i] : a2[i]) + __shfl_xor(h3 ? a2[i] : a2[H3 + i], 8, 64);
#pragma unroll
  for (int i = 0; i < H4; ++i) a4[i] = (h2 ? a3[H4 + i] : a3[i]) + __shfl_xor(h2 ? a3[i] : a3[H4 + i], 4, 64);
  const int base = H1 * h5 + H2 * h4 + H3 * h3 + H4 * h2;
#pragma unroll
  for (int i = 0; i < H4; ++i) {
    a4[i] += __shfl_xor(a4[i], 2, 64);
    a4[i] += __shfl_xor(a4[i], 1, 64);
    if ((i & 3) == (lane & 3)) dst[base + i] = a4[i];
  }
}
constexpr int pad16(int n) { return (n + 15) / 16 * 16; }

// Σ over the workgroup of NV per-thread accumulators in a fixed order → out[0 … NV): each wave's sums by wave_rs_lds
// into s_w (4·pad16(NV) doubles), then the four waves in order.  Every thread calls it.
template <int NV>
__device__ __forceinline__ void wg_sum_store(const double* acc, double* s_w, double* out) {
  constexpr int NP = pad16(NV);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double v[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) v[i] = i < NV ? acc[i] : 0.0;
  wave_rs_lds<NP>(v, lane, s_w + w * NP);
  __syncthreads();
  for (int i = threadIdx.x; i < NV; i += blockDim.x) out[i] = ((s_w[i] + s_w[NP + i]) + s_w[2 * NP + i]) + s_w[3 * NP + i];
}

__device__ __forceinline__ void cam_dir(const IntrBorderArgs& a, double* part, int bx, int by) {
  __shared__ double s_w[4 * pad16(kCamDir)];
  const int c = by, L = c * (a.nf + a.nc) + a.nf + c;  // (camera c, unit nf + c): every block of camera c
  double acc[kCamDir];
#pragma unroll
  for (int v = 0; v < kCamDir; ++v) acc[v] = 0.0;
  const int qe = a.bptr[L + 1];
  int q = a.bptr[L] + threadIdx.x + 256 * bx;
  int bn = q < qe ? a.blist[q] : 0;  // (the next entry's index loaded during this one)
  for (; q < qe; q += 256 * kCamSplit) {
    const double* B = a.ib + (long long)bn * kIbStride;
    if (q + 256 * kCamSplit < qe) bn = a.blist[q + 256 * kCamSplit];
    double j0[8], j1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      j0[k] = B[kIbJi + k];
      j1[k] = B[kIbJi + 8 + k];
    }
    const double r0 = B[kIbR], r1 = B[kIbR + 1];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = i; j < 8; ++j) acc[upper8i(i, j)] += j0[i] * j0[j] + j1[i] * j1[j];
      acc[36 + i] += j0[i] * r0 + j1[i] * r1;
    }
  }
  wg_sum_store<kCamDir>(acc, s_w, part + ((long long)c * kCamSplit + bx) * kCamDir);
}

__device__ __forceinline__ void cam_sch(const IntrBorderArgs& a, double lambda, double* part, int bx, int by) {
  __shared__ double s_w[4 * pad16(kCamSch)];
  lambda = lm_lambda(lm_view(a.lm), lambda);
  const int pc = by;  // camera pair (c, c2 ≤ c), pc = c(c+1)/2 + c2
  int c = 0;
  while ((c + 1) * (c + 2) / 2 <= pc) ++c;
  const int c2 = pc - c * (c + 1) / 2, L = c * (a.nf + a.nc) + a.nf + c2;  // points seen by c and c2
  const int st = 8 * a.nc + 6;
  double acc[kCamSch];
#pragma unroll
  for (int v = 0; v < kCamSch; ++v) acc[v] = 0.0;
  for (int q = a.pptr[L] + threadIdx.x + 256 * bx; q < a.pptr[L + 1]; q += 256 * kCamSplit) {
    const int gp = a.plist[q];
    const double* pw = a.pw + (long long)gp * st;
    const double inv = border_inv(a, gp, lambda), gr = a.pt_data[(long long)gp * 8 + 1];
    double wc[8], w2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      wc[k] = pw[8 * c + k];
      w2[k] = pw[8 * c2 + k];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const double iw = inv * wc[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[8 * i + j] += iw * w2[j];
      acc[64 + i] += iw * gr;
    }
  }
  wg_sum_store<kCamSch>(acc, s_w, part + ((long long)pc * kCamSplit + bx) * kCamSch);
}

__global__ __launch_bounds__(256) void intr_border_kernel(const IntrBorderArgs a, double lambda, int kpw) {
  border_keyframes(a, lambda, kpw, blockIdx.x, blockIdx.y);
}
__global__ __launch_bounds__(256) void intr_cam_dir_kernel(const IntrBorderArgs a, double* part) {
  cam_dir(a, part, blockIdx.x, blockIdx.y);
}
__global__ __launch_bounds__(256) void intr_cam_sch_kernel(const IntrBorderArgs a, double lambda, double* part) {
  cam_sch(a, lambda, part, blockIdx.x, blockIdx.y);
}
// The three border reductions are independent (they read the rows, the points' sums and the lists, and write
// different outputs): while the keyframe part is small (nf·nc < 512 keyframe blocks, the 4-waves-per-keyframe regime:
// C3), one launch runs them side by side — workgroups [0, nk) the keyframe blocks (nk_x per camera), then kCamSplit per
// camera of direct sums, then kCamSplit per camera pair of Schur sums — instead of three launches in sequence, each a
// fraction of the chip (C3: 35.3 → 24.6 µs, two cameras 41.3 → 31.1; at C4, where the keyframe part alone fills the
// chip, side by side measured 108 against 102 µs in sequence).
__global__ __launch_bounds__(256) void intr_border_all_kernel(const IntrBorderArgs a, double lambda, int kpw, int nk_x,
                                                             double* dpart, double* spart) {
  int b = blockIdx.x;
  const int nk = nk_x * a.nc, nd = kCamSplit * a.nc;
  if (b < nk) {
    border_keyframes(a, lambda, kpw, b % nk_x, b / nk_x);
    return;
  }
  b -= nk;
  if (b < nd) {
    cam_dir(a, dpart, b % kCamSplit, b / kCamSplit);
    return;
  }
  b -= nd;
  cam_sch(a, lambda, spart, b % kCamSplit, b / kCamSplit);
}

// One WAVE per (border row, camera column block yb ≤ row, entry e) and per border gradient element: lane l adds totals l,
// l + 64, … of the kCamSplit in order, the wave's lanes by xor butterflies (a fixed order); then border_store.
__device__ __forceinline__ void cam_fin(const IntrBorderArgs& a, double lambda, const double* dpart, const double* spart,
                                        int blk) {
  lambda = lm_lambda(lm_view(a.lm), lambda);
  const int nb = 2 * a.nc + 1, i = blk * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= 2 * a.nc * nb * 36) return;
  const int e = i % 36, yb = (i / 36) % nb, row = i / (36 * nb);
  const bool grad = yb == 2 * a.nc;
  if (grad ? (e % 6 != 0) : (yb > row)) return;  // (the upper camera blocks are not stored; whole waves)
  const int c = row >> 1, h = row & 1, r = e / 6, cc = e % 6, d = 6 * h + r;
  auto sum = [&](const double* p, int stride, int idx) {
    double v = 0.0;
    for (int s = lane; s < kCamSplit; s += 64) v += p[(long long)s * stride + idx];
    return wave_sum(v);
  };
  double dir = 0.0, sch = 0.0;
  if (grad) {
    if (d < 8) {
      dir = sum(dpart + (long long)c * kCamSplit * kCamDir, kCamDir, 36 + d);
      sch = sum(spart + (long long)(c * (c + 1) / 2 + c) * kCamSplit * kCamSch, kCamSch, 64 + d);
    }
    if (lane == 0) border_store(a, lambda, row, (a.nf + 2 * a.nc) * 36 + r, dir, sch);
    return;
  }
  const int c2 = yb >> 1, d2 = 6 * (yb & 1) + cc;
  if (d < 8 && d2 < 8) {  // (pads: border_store's identity rows)
    if (c2 == c) dir = sum(dpart + (long long)c * kCamSplit * kCamDir, kCamDir, upper8i(min(d, d2), max(d, d2)));
    sch = sum(spart + (long long)(c * (c + 1) / 2 + c2) * kCamSplit * kCamSch, kCamSch, 8 * d + d2);
  }
  if (lane == 0) border_store(a, lambda, row, (a.nf + yb) * 36 + e, dir, sch);
}
__global__ __launch_bounds__(256) void intr_cam_fin_kernel(const IntrBorderArgs a, double lambda, const double* dpart,
                                                          const double* spart) {
  cam_fin(a, lambda, dpart, spart, blockIdx.x);
}
// The same, with the arrow solve's level 0 (arrow_build) in workgroups fin_blocks … of the same launch: it reads the
// keyframe band and g (assemble_kernel) and the border rows' keyframe blocks (border_keyframes), nothing this launch
// writes — one launch fewer per trial.
__global__ __launch_bounds__(256) void intr_cam_fin_build_kernel(const IntrBorderArgs a, double lambda,
                                                                const double* dpart, const double* spart,
                                                                const ArrowArgs aa, int batches, int fin_blocks) {
  if ((int)blockIdx.x < fin_blocks) cam_fin(a, lambda, dpart, spart, blockIdx.x);
  else arrow_build(aa, batches, (long long)(blockIdx.x - fin_blocks) * blockDim.x + threadIdx.x);
}

// The candidate intrinsics become the state (after an accepted trial; lm == nullptr: always), fp64 records and fp32 copy.
__global__ void intr_accept_kernel(const double* __restrict__ lm, const double* __restrict__ knew_d,
                                   const float* __restrict__ knew_f, double* __restrict__ k_d, float* __restrict__ k_f,
                                   int nc) {
  if (lm && (lm[kLmAccept] == 0.0 || lm[kLmDone] != 0.0)) return;
  const int i = threadIdx.x, c = i >> 3, d = i & 7;
  if (c >= nc) return;
  k_d[kCamD * c + d] = knew_d[kCamD * c + d];
  k_f[8 * c + d] = knew_f[8 * c + d];
}

__global__ __launch_bounds__(kBlockThreads) void cost_reduce_kernel(const float* cost, const uint8_t* valid, int n,
                                                                    double* red) {
  double c = 0.0, v = 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    c += cost[i];
    v += valid[i];
  }
  wg_reduce2(c, v, red + 2 * blockIdx.x);
}

// The LM trial's decision on the device (trust_region_minimizer.cc semantics, the same sums and order as the host
// code of the distributed loop): model decrease from the update partials (slots [0, gp + gq)), candidate cost from
// the cost partials (slots [gp + gq, gp + gq + gc)), accepted when the solve succeeded, the model predicts a
// decrease and (cost − cost_new) / model > min_relative_decrease.  On acceptance the record's current cost becomes
// the candidate's.  One workgroup: strided per-thread sums, then a fixed-order tree in LDS (deterministic).
// The record is also published to page-locked, host-coherent memory (host_rec: the kLmFields values, then the trial's
// sequence number after a system-scope fence), so the host learns the decision by polling instead of through a copy
// and a stream event (each of which left the GPU idle ~6 µs).
constexpr int kDecideThreads = 1024;

// Ceres' termination options of the LM loop (solver.h:278-322; pba_solver_options)
struct DecideOpts {
  double min_rel, ftol, ptol, gtol, max_radius, min_radius;
  int max_invalid;
};

// The trial's sums: the pose part (identical on every rank of a distributed solve: same summed system, same step) and
// the point part with the candidate's cost and valid blocks (summed over the ranks).
enum : int {
  kTsPoseG = 0, kTsPoseD, kTsPoseStep2, kTsPoseXNorm2, kTsPoseGMax,
  kTsPtG, kTsPtD, kTsCost, kTsValid, kTsPtStep2, kTsPtXNorm2, kTsPtGMax, kTsCount
};

// The trial's decision (one lane): trust_region_minimizer.cc:85-133 + levenberg_marquardt_strategy.cc:146-160 over the
// summed trial quantities t[kTs*] and the record lm.  In Ceres' order:
//   gradient tolerance at the current state (FinalizeIteration… :336-355, GradientToleranceReached :668-684): checked
//     here, before the step, because this trial is the first to see the current state's gradient; the trial is void
//     (done 4, not an iteration);
//   invalid step — solver failure or no predicted decrease (:400-439) — HandleInvalidStep (:453-484): the 5th
//     consecutive one ends the solve with FAILURE (done 2, not an iteration), earlier ones shrink the radius;
//   candidate cost: infinite (DBL_MAX, :771-778) when a block valid at the current state is invalid at the candidate;
//   parameter tolerance (:706-726, step_norm ≤ ptol (x_norm + ptol) with x_norm = −1 until the first accepted step,
//     :185 / :814) → done 3;  function tolerance (:729-748) → done 1 (neither step applied);
//   IsStepSuccessful (:781-803) → accept (radius = min(max_radius, radius / max(1/3, 1 − (2ρ − 1)³)), :146-153) or
//     reject (radius /= factor, factor *= 2, :155-160);  MinTrustRegionRadiusReached (:687-703) → done 5.
__device__ void lm_decide(const double* t, int st, const DecideOpts& o, double* lm) {
  const double lambda = lm[kLmLambda];
  const double model = __dadd_rn(__dmul_rn(0.5, __dsub_rn(__dmul_rn(lambda, t[kTsPoseD]), t[kTsPoseG])),
                                 __dmul_rn(0.5, __dsub_rn(__dmul_rn(lambda, t[kTsPtD]), t[kTsPtG])));
  const double cost = lm[kLmCost];
  const double gnorm = fmax(t[kTsPoseGMax], t[kTsPtGMax]);
  double radius = lm[kLmRadius], factor = lm[kLmFactor], done = 0.0, invalid = lm[kLmInvalid];
  bool accept = false, converged = false;
  const bool valid_step = st == 0 && model > 0.0;
  const double c = t[kTsValid] < lm[kLmValid] ? DBL_MAX : t[kTsCost];
  const double step = sqrt(t[kTsPoseStep2] + t[kTsPtStep2]);
  const double rel = (cost - c) / model;
  if (gnorm <= o.gtol) {
    done = 4.0;
  } else if (!valid_step) {
    invalid += 1.0;
    if (invalid >= (double)o.max_invalid) {
      done = 2.0;
    } else {
      radius /= factor;  // StepIsInvalid = StepRejected(0)
      factor *= 2.0;
      if (radius <= o.min_radius) done = 5.0;
    }
  } else {
    invalid = 0.0;
    if (step <= o.ptol * (lm[kLmXNorm] + o.ptol)) {
      done = 3.0;
      converged = true;
    } else if (fabs(cost - c) <= o.ftol * cost) {
      done = 1.0;
      converged = true;
    } else if (rel > o.min_rel) {
      accept = true;
      const double q = 2.0 * rel - 1.0;
      radius = fmin(o.max_radius, radius / fmax(1.0 / 3.0, 1.0 - q * q * q));
      factor = 2.0;
    } else {
      radius /= factor;
      factor *= 2.0;
      if (radius <= o.min_radius) done = 5.0;
    }
  }
  lm[kLmConverged] = converged ? 1.0 : 0.0;
  lm[kLmCostNew] = c;
  lm[kLmModel] = model;
  lm[kLmRel] = rel;
  lm[kLmAccept] = accept ? 1.0 : 0.0;
  lm[kLmStatus] = (double)st;
  lm[kLmStepNorm] = step;
  lm[kLmGradNorm] = gnorm;
  if (accept) {
    lm[kLmCost] = c;
    lm[kLmValid] = t[kTsValid];
    lm[kLmXNorm] = sqrt(t[kTsPoseXNorm2] + t[kTsPtXNorm2]);
    lm[kLmSet] = 1.0 - lm[kLmSet];  // the candidate's linearisation (the spare set) is now the current one
  }
  lm[kLmInvalid] = invalid;
  lm[kLmRadius] = radius;
  lm[kLmFactor] = factor;
  lm[kLmLambda] = 1.0 / radius;
  lm[kLmDone] = done;
}

// The trial's sums from the update and cost partials (one workgroup; deterministic).  Slots: red [0, gp) poses,
// [gp, gp + gq) points (model decrease parts), [gp + gq, gp + gq + gc) the candidate's (cost, valid) — one slot per
// linearisation chunk, 12.5k at C4; red2 / gmax [0, gp + gq) (update_kernel).  The red2 / gmax slots one per
// thread, then one strided pass over red with U slots per thread in flight, then xor butterflies per wave and the
// waves in order (U loads of three arrays spilled 172 B per lane at 1024 threads: 16 µs per decision).  t: the
// totals, in LDS.
// lo, hi: only the slots [lo, hi) of both passes (a slice of the sums, schur_free_decide_kernel's decision workgroups).
template <int N>
__device__ void trial_sums(const double* __restrict__ red, const double* __restrict__ red2,
                           const double* __restrict__ gmax, int gp, int gq, int gc, double* t, int lo = 0,
                           int hi = 0x7fffffff) {
  constexpr int U = 8;
  __shared__ double part[kTsCount][N / 64];
  double v[kTsCount] = {};
  const int S0 = gp + gq, S = min(S0, hi), E = min(S0 + gc, hi);
  const double2* r1 = reinterpret_cast<const double2*>(red);
  const double2* r2 = reinterpret_cast<const double2*>(red2);
  // the update slots' norms and gradient maxima: one slot per thread, loaded before the red pass so that both are
  // in flight together (S ≤ N unless the problem has > 260k points: a tail loop then)
  const int i_s = lo + (int)threadIdx.x;
  const double2 ys = i_s < S ? r2[i_s] : make_double2(0.0, 0.0);
  const double ms = i_s < S ? gmax[i_s] : 0.0;
  for (int i0 = lo + (int)threadIdx.x; i0 < E; i0 += U * N) {
    double2 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * N;
      x[u] = i < E ? r1[i] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // selects, not a computed index (that put v in scratch memory)
      const int i = i0 + u * N;
      const bool p = i < gp, t = i >= gp && i < S0;
      v[kTsPoseG] += p ? x[u].x : 0.0;
      v[kTsPoseD] += p ? x[u].y : 0.0;
      v[kTsPtG] += t ? x[u].x : 0.0;
      v[kTsPtD] += t ? x[u].y : 0.0;
      v[kTsCost] += i >= S0 ? x[u].x : 0.0;  // (slots past E loaded as zeros)
      v[kTsValid] += i >= S0 ? x[u].y : 0.0;
    }
  }
  auto add_small = [&](int i, const double2& y, double m) {
    if (i < gp) {
      v[kTsPoseStep2] += y.x;
      v[kTsPoseXNorm2] += y.y;
      v[kTsPoseGMax] = fmax(v[kTsPoseGMax], m);
    } else if (i < S) {
      v[kTsPtStep2] += y.x;
      v[kTsPtXNorm2] += y.y;
      v[kTsPtGMax] = fmax(v[kTsPtGMax], m);
    }
  };
  add_small(i_s, ys, ms);
  for (int i = i_s + N; i < S; i += N) add_small(i, r2[i], gmax[i]);
  auto is_max = [](int q) { return q == kTsPoseGMax || q == kTsPtGMax; };
  // a wave past the update slots holds only candidate-cost sums: its other ten are zeros, not butterflied (the same
  // totals: only zeros are left out)
  const bool upd = __builtin_amdgcn_readfirstlane(lo + ((int)threadIdx.x & ~63)) < S;
#pragma unroll
  for (int q = 0; q < kTsCount; ++q) {
    if (!upd && q != kTsCost && q != kTsValid) continue;
    for (int m = 32; m >= 1; m >>= 1) {
      const double o = __shfl_xor(v[q], m, 64);
      v[q] = is_max(q) ? fmax(v[q], o) : v[q] + o;
    }
  }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < kTsCount; ++q) part[q][threadIdx.x >> 6] = v[q];
  __syncthreads();
  // the waves in order, one thread per sum (one thread summing all twelve, 192 dependent LDS reads, was ~8 µs)
  if (threadIdx.x < kTsCount) {
    const int q = threadIdx.x;
    double w16[N / 64];
#pragma unroll
    for (int w = 0; w < N / 64; ++w) w16[w] = part[q][w];
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < N / 64; ++w) s = is_max(q) ? fmax(s, w16[w]) : s + w16[w];
    t[q] = s;
  }
  __syncthreads();
}

// Publish the record to page-locked, host-coherent memory (wave 0): lane i stores field i, every store completes, then
// lane 0 stores the sequence number the host polls for with a system-scope release.
// Every store is a system-scope relaxed atomic (`sc0 sc1`: written through to memory, whatever the page's cache
// policy), and the sequence number is stored only after every field store has completed (vmcnt(0)).  A release fence
// at system scope instead (`buffer_wbl2`) wrote back every dirty line the candidate linearisation had left in L2: the
// decision launch took 14.5-16.4 µs against 8.6 µs (profiles/r3_gn_trial_trace_*).
__device__ void publish_record(const double* s_rec, double* host_rec, double seq) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int l = threadIdx.x;
  if (l < kLmFields) __hip_atomic_store(host_rec + l, s_rec[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's field store has completed
  __builtin_amdgcn_wave_barrier();
  if (l == 0) __hip_atomic_store(host_rec + kLmFields, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kDecideThreads) void lm_decide_kernel(const double* __restrict__ red,
                                                                   const double* __restrict__ red2,
                                                                   const double* __restrict__ gmax, int gp, int gq,
                                                                   int gc, const int* __restrict__ status,
                                                                   const DecideOpts o, double* __restrict__ lm,
                                                                   double* __restrict__ host_rec, double seq) {
  // a trial enqueued ahead of the one that ended the solve returns — tested after the sums, so the record's load is in
  // flight with the partials' instead of a round trip of its own before them (the partials are always readable)
  const double done = lm[kLmDone];
  __shared__ double t[kTsCount];
  trial_sums<kDecideThreads>(red, red2, gmax, gp, gq, gc, t);
  if (done != 0.0 || threadIdx.x >= 64) return;  // wave 0 publishes; lane 0 decides
  __shared__ double s_rec[kLmFields];
  if (threadIdx.x == 0) {
    lm_decide(t, *status, o, lm);
    for (int i = 0; i < kLmFields; ++i) s_rec[i] = lm[i];
  }
  if (host_rec) publish_record(s_rec, host_rec, seq);
}

// The LM record of a new solve, on the device: the initial cost and valid blocks summed from the initial linearisation's
// chunk partials (slots [0, gc) of red — the same partials, in the same order, as a trial's candidate cost), the trust
// region, nothing done, buffer set 0, x_norm −1.  The host enqueues the first trials behind it instead of reading the cost
// back first (a host round trip with the GPU idle, once per solve); init[0..1] = the initial cost and valid blocks.
__global__ __launch_bounds__(kDecideThreads) void lm_init_kernel(const double* __restrict__ red, int gc, double radius,
                                                                 double* __restrict__ lm, double* __restrict__ init) {
  __shared__ double t[kTsCount];
  trial_sums<kDecideThreads>(red, red, red, 0, 0, gc, t);
  if (threadIdx.x != 0) return;
  for (int i = 0; i < kLmFields; ++i) lm[i] = 0.0;
  lm[kLmCost] = t[kTsCost];
  lm[kLmValid] = t[kTsValid];
  lm[kLmXNorm] = -1.0;
  lm[kLmRadius] = radius;
  lm[kLmFactor] = 2.0;
  lm[kLmLambda] = 1.0 / radius;
  init[0] = t[kTsCost];
  init[1] = t[kTsValid];
}

// ---- the single-GPU LM loop's λ-free point elimination ---------------------------------------------------------------
// For a point whose H_ρρ lies inside the LM diagonal's clamp [1e-6, 1e32] (levenberg_marquardt_strategy.cc), the damped
// H' = H + λ·clamp(H) = (1 + λ)·H, so its Schur terms W Wᵀ / H' and W g / H' are (1 + λ)⁻¹ times the λ-free W Wᵀ / H and
// W g / H.  A linearisation set's λ-free partials P are therefore formed once, right after the set is linearised, and every
// trial on that set (an accepted candidate's first, or the retries after rejections) assembles A + λD − P / (1 + λ):
// no per-trial point elimination.  A set with a point outside the clamp (H ≠ 0: a point with H = 0 has W = 0) is flagged
// (degen[set]) and its trials form the λ-specific partials in schur_gate_kernel, exactly as schur_kernel does.
//
// The kernel after the candidate linearisation: workgroup 0 takes the trial's decision (lm_decide_kernel's sums and
// decision, 256 threads) — or, init, forms the record of a new solve (lm_init_kernel's) — while workgroups 1 … n_schur
// form the λ-free partials and point data of the set linearize_kernel has just written (lin_set); the two parts share no
// data, so the decision costs no launch and runs beside the elimination.  The elimination never reads the record's set
// (the decision may flip it meanwhile); only its done flag (a workgroup that sees the solve ended skips its chunk: nothing
// reads it then).
struct DecideArgs {
  const double* red;
  const double* red2;
  const double* gmax;
  int gp, gq, gc;
  const int* status;
  DecideOpts o;
  double* lm;
  double* host_rec;   // the published record slot, or nullptr
  double seq;
  int init;           // 1: a new solve's record (lm_init_kernel), 0: the trial's decision
  double radius;      // init: the initial trust-region radius
  double* init_out;   // init: [initial cost, valid blocks]
  double* ts_part;    // [kDecideWgs][kTsCount]: the decision workgroups' slices of the sums
  int* ts_count;      // their arrivals (0 between launches)
};
// Workgroups of schur_free_decide_kernel that sum the trial's partial slots, a slice each: one workgroup alone took ~20 µs
// for the 13.5k slots at C4 (seven dependent memory rounds), longer than the elimination beside it.
constexpr int kDecideWgs = 16;
struct FreeSets {
  double* part[2];    // λ-free Schur partials per linearisation set
  double* pt[2];      // point data per set ([H, g, W_h(6)] per GN point, undamped)
  int* degen;         // [2]: a point of the set outside the clamp
  const int* lin_set; // the set the last linearisation wrote
};

__global__ __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void schur_free_decide_kernel(const SchurArgs g, const DecideArgs da,
                                                                        const FreeSets fs) {
  extern __shared__ __attribute__((aligned(16))) double W_dyn[];
  __shared__ double s_inv[SCHUR_PTS], s_gl[SCHUR_PTS];
#ifdef PBA_FD_STAMPS  // timing dissection only: 100-MHz stamps at the start and end of chosen workgroups
  struct Stamp {
    long long t0 = wall_clock64();
    __device__ ~Stamp() {
      const int b = blockIdx.x;
      if (threadIdx.x == 0 && (b == 0 || b == 1 || b == 300 || b == 600 || b == (int)gridDim.x - 1))
        printf("fdstamp b=%d start %lld end %lld\n", b, t0, wall_clock64());
    }
  } stamp;
#endif
  if (blockIdx.x < kDecideWgs) {
    // a slice of the sums per workgroup → sc1 stores → (every store completed, release) → arrival count; the last
    // workgroup to arrive (acquire) adds the slices in workgroup order — the same totals whichever arrives last — and
    // decides (or, init, writes the new solve's record)
    __shared__ double t[kTsCount];
    __shared__ int s_last;
    const double done = da.init ? 0.0 : da.lm[kLmDone];  // (tested after the sums, as lm_decide_kernel)
    {
      const int E = da.init ? da.gc : da.gp + da.gq + da.gc, per = (E + kDecideWgs - 1) / kDecideWgs;
      const int lo = (int)blockIdx.x * per, hi = min(E, lo + per);
      if (da.init) trial_sums<kBlockThreads>(da.red, da.red, da.red, 0, 0, da.gc, t, lo, hi);
      else trial_sums<kBlockThreads>(da.red, da.red2, da.gmax, da.gp, da.gq, da.gc, t, lo, hi);
      if (threadIdx.x < kTsCount)
        __hip_atomic_store(da.ts_part + blockIdx.x * kTsCount + threadIdx.x, t[threadIdx.x], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = __hip_atomic_fetch_add(da.ts_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kDecideWgs - 1;
        if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (!s_last) return;
      if (threadIdx.x < kTsCount) {
        const int q = threadIdx.x;
        const bool mx = q == kTsPoseGMax || q == kTsPtGMax;
        double v = 0.0;
#pragma unroll 1
        for (int b0 = 0; b0 < kDecideWgs; b0 += 4) {  // (4 loads in flight: 16 held the elimination to 3 waves/SIMD)
          double x[4];
#pragma unroll
          for (int b = 0; b < 4; ++b)
            x[b] = __hip_atomic_load(da.ts_part + (b0 + b) * kTsCount + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int b = 0; b < 4; ++b) v = mx ? fmax(v, x[b]) : v + x[b];
        }
        t[q] = v;
      }
      if (threadIdx.x == 0) *da.ts_count = 0;  // for the next launch (ordered by the launch boundary)
      __syncthreads();
    }
    if (da.init) {
      if (threadIdx.x != 0) return;
      double* lm = da.lm;
      for (int i = 0; i < kLmFields; ++i) lm[i] = 0.0;
      lm[kLmCost] = t[kTsCost];
      lm[kLmValid] = t[kTsValid];
      lm[kLmXNorm] = -1.0;
      lm[kLmRadius] = da.radius;
      lm[kLmFactor] = 2.0;
      lm[kLmLambda] = 1.0 / da.radius;
      da.init_out[0] = t[kTsCost];
      da.init_out[1] = t[kTsValid];
      return;
    }
    if (done != 0.0 || threadIdx.x >= 64) return;
    __shared__ double s_rec[kLmFields];
    if (threadIdx.x == 0) {
      lm_decide(t, *da.status, da.o, da.lm);
      for (int i = 0; i < kLmFields; ++i) s_rec[i] = da.lm[i];
    }
    if (da.host_rec) publish_record(s_rec, da.host_rec, da.seq);
    return;
  }
  const int c = blockIdx.x - kDecideWgs;
  if (c >= g.n_chunks) return;
  // one memory round: the chunk's descriptors, the record's done flag and the set, all issued before the exit (the
  // compiler otherwise waited for the flag, then for the set, then issued the descriptors)
  const SchurHead h = schur_head(g, c);
  const double done = da.lm[kLmDone];
  const int lset = *fs.lin_set;
  asm volatile("" ::"v"(done), "v"(lset), "v"(h.d.x), "v"(h.ax.x), "v"(h.lp4.x));
#pragma unroll
  for (int it = 0; it < kPtIter; ++it) asm volatile("" ::"v"(h.prec[it].x), "v"(h.prec[it].y));
  if (!da.init && done != 0.0) return;
  const int set = lset != 0;
  schur_chunk(g, h, 0.0, set ? g.blk_schur1 : g.blk_schur, set ? g.pair_rt1 : g.pair_rt, fs.part[set], fs.pt[set],
              fs.degen + set, W_dyn, s_inv, s_gl);
}

// The single-GPU LM trial's first kernel: the previous trial's accept, and — only for a set flagged degen — the
// λ-specific point elimination of the current set into part_schur (every chunk, grid-stride), which the assembly then
// takes instead of the λ-free partials.
__global__ __launch_bounds__(kBlockThreads) void schur_gate_kernel(const SchurArgs g, const int* __restrict__ degen) {
  extern __shared__ __attribute__((aligned(16))) double W_dyn[];
  __shared__ double s_inv[SCHUR_PTS], s_gl[SCHUR_PTS];
  const LmView lv = lm_view(g.lm);
  const int dg0 = degen[0], dg1 = degen[1];
  AcceptCopy ac;
  ac.load(g, lv);
  const int set = lv.set != 0.0;
  if ((set ? dg1 : dg0) != 0 && lv.done == 0.0) {
    const double* blk_schur = set ? g.blk_schur1 : g.blk_schur;
    for (int c = blockIdx.x; c < g.n_chunks; c += gridDim.x) {
      schur_chunk(g, schur_head(g, c), lv.lambda, blk_schur, set ? g.pair_rt1 : g.pair_rt, g.part_schur, nullptr,
                  nullptr, W_dyn, s_inv, s_gl);
      __syncthreads();
    }
  }
  ac.store(g);
}

// Multi-GPU trial, before the scalar all-reduce: this rank's sums, written to the exchange buffer's kExScalars scalar
// slots Y for the Σ over ranks:
//   Y[0..7]  the point part: [δρ·g, δρ·D·δρ, candidate cost, candidate valid blocks, Σδρ², Σρ_new², points above the
//            gradient tolerance, 0] (the gradient test needs only whether some rank's point gradient exceeds the
//            tolerance: a count sums exactly);
//   Y[8..14] the pose part [g·δ, δ·D·δ, Σδ², Σx_new², max|g|] and the reduced solve's status, from rank 0 only (0 on the
//            other ranks).  Every rank computes them from the same summed system with the same kernels, so they agree
//            bit for bit anyway; summing rank 0's copy makes the decision inputs identical on every rank by construction
//            (a decision that differed between ranks would leave their collective sequences mismatched: a hang).
// rank0 = −1 (a host-callback collective, which does not know the ranks): Y[8..14] stay 0 and the decision reads the
// rank's own pose part from tpose.  tpose: [pose part (5) | this rank's point gradient max-norm | solve status].
constexpr int kExScalars = 16;
__global__ __launch_bounds__(kDecideThreads) void dist_sums_kernel(const double* __restrict__ red,
                                                                   const double* __restrict__ red2,
                                                                   const double* __restrict__ gmax, int gp, int gq, int gc,
                                                                   double gtol, const double* __restrict__ lm,
                                                                   const int* __restrict__ status, int rank0,
                                                                   double* __restrict__ tpose, double* __restrict__ Y) {
  const double done = lm[kLmDone];  // (tested after the sums, as lm_decide_kernel)
  __shared__ double t[kTsCount];
  trial_sums<kDecideThreads>(red, red2, gmax, gp, gq, gc, t);
  if (threadIdx.x != 0) return;
  // the previous decision's word, with its square, and whether it ended the solve on this rank: every rank, done or not
  const double w = decision_word(lm);
  Y[7] = done != 0.0 ? 1.0 : 0.0;
  Y[14] = w;
  Y[15] = w * w;
  if (done != 0.0) {  // (the sums are not used; zeros keep them finite)
    for (int q = 0; q < 7; ++q) Y[q] = 0.0;
    for (int q = 8; q < 14; ++q) Y[q] = 0.0;
    return;
  }
  for (int q = 0; q < 5; ++q) tpose[q] = t[kTsPoseG + q];
  tpose[5] = t[kTsPtGMax];
  tpose[6] = (double)*status;
  Y[0] = t[kTsPtG];
  Y[1] = t[kTsPtD];
  Y[2] = t[kTsCost];
  Y[3] = t[kTsValid];
  Y[4] = t[kTsPtStep2];
  Y[5] = t[kTsPtXNorm2];
  Y[6] = t[kTsPtGMax] > gtol ? 1.0 : 0.0;
  for (int q = 0; q < 5; ++q) Y[8 + q] = rank0 == 1 ? t[kTsPoseG + q] : 0.0;
  Y[13] = rank0 == 1 ? (double)*status : 0.0;
}

// Multi-GPU decision from the summed Y: the same lm_decide on every rank (identical inputs), so every rank takes the
// same decision; the reported gradient norm is this rank's view (the pose part and its own points).  First the check of
// the previous decision (decision_word over the ranks, n_ranks of them): if the ranks' records differed, every rank
// ends the solve here (done = kDoneDesync, kLmDesync = 1 + the number of ranks that had stopped) — the host loops then
// match their remaining collectives (lm_loop) and report the error instead of hanging.  The record is published even
// when the solve was already done, so a host that stopped can read this check.  perturb_seq (tests,
// PBA_TEST_PERTURB_DECISION): this rank's decision of that trial is overridden (mode 1 flips accept, 2 ends the solve).
__global__ __launch_bounds__(64) void dist_decide_kernel(const double* __restrict__ Y, const double* __restrict__ tpose,
                                                         int local, const DecideOpts o, double* __restrict__ lm,
                                                         double* __restrict__ host_rec, double seq, int n_ranks,
                                                         double perturb_seq, int perturb_mode, int verify_only) {
  __shared__ double s_rec[kLmFields];
  if (threadIdx.x == 0) {
    const bool desync = (double)n_ranks * Y[15] != Y[14] * Y[14];
    if (desync) {
      lm[kLmDone] = kDoneDesync;
      lm[kLmDesync] = Y[7] + 1.0;
      lm[kLmAccept] = 0.0;
    } else if (lm[kLmDone] == 0.0 && !verify_only) {
      const double* pose = local ? tpose : Y + 8;  // [pose part (5) | …, status at 6 resp. 5]
      double t[kTsCount];
      for (int q = 0; q < 5; ++q) t[kTsPoseG + q] = pose[q];
      t[kTsPtG] = Y[0];
      t[kTsPtD] = Y[1];
      t[kTsCost] = Y[2];
      t[kTsValid] = Y[3];
      t[kTsPtStep2] = Y[4];
      t[kTsPtXNorm2] = Y[5];
      // no rank's point gradient above the tolerance: the test then depends on the pose part alone (identical)
      t[kTsPtGMax] = Y[6] > 0.0 ? INFINITY : 0.0;
      lm_decide(t, (int)(local ? tpose[6] : Y[13]), o, lm);
      lm[kLmGradNorm] = fmax(pose[4], tpose[5]);
      if (seq == perturb_seq) {
        if (perturb_mode == 1) lm[kLmAccept] = 1.0 - lm[kLmAccept];
        else lm[kLmDone] = kDoneFunction;
      }
    }
    for (int i = 0; i < kLmFields; ++i) s_rec[i] = lm[i];
  }
  if (host_rec) publish_record(s_rec, host_rec, seq);
}

// The check of the last decision of a multi-GPU solve (no trial follows it): the decision word into Y as dist_sums_kernel
// writes it, every other slot zero.
__global__ void dist_verify_kernel(const double* __restrict__ lm, double* __restrict__ Y) {
  if (threadIdx.x != 0) return;
  const double w = decision_word(lm);
  for (int q = 0; q < kExScalars; ++q) Y[q] = 0.0;
  Y[7] = lm[kLmDone] != 0.0 ? 1.0 : 0.0;
  Y[14] = w;
  Y[15] = w * w;
}

// The accepted candidate becomes the state (device-side accept, gated by the decision record; lm == nullptr: always).
// Only the points of the Gauss-Newton problem are copied (through pt_orig): rho_new holds nothing for a point with
// no residual block, and such a point keeps its state, as a parameter Ceres never sees would.
__global__ void lm_accept_kernel(const double* __restrict__ lm, const double* __restrict__ poses_new,
                                 const double* __restrict__ rho_new, const int* __restrict__ pt_orig,
                                 double* __restrict__ poses, double* __restrict__ rho, int n_pose_d, int n_gn_points) {
  if (lm && (lm[kLmAccept] == 0.0 || lm[kLmDone] != 0.0)) return;
  const int n = max(n_pose_d, n_gn_points);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (i < n_pose_d) poses[i] = poses_new[i];
    if (i < n_gn_points) {
      const int o = pt_orig[i];
      rho[o] = rho_new[o];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
int gn_lpb(const pba_engine* e) { return e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC ? 4 : 8; }
// rows per lane of the linearisation: 1 up to 8 px (one lane per row), ⌈P/8⌉ above (linearize_adj_kernel<·, PPL>)
int gn_ppl(const pba_engine* e) { return e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC ? 1 : (e->P + 7) / 8; }

int band_kernel_for(int band) { return band <= 4 ? 4 : (band <= 8 ? 8 : (band <= 16 ? 16 : 0)); }

int configure_arrow(pba_engine* e);  // (free intrinsics' arrow solve, below)

// Reduced-system solver buffers for band K (0: skyline only): band input Sband (row stride (K+1)·36 + 6,
// zero outside the profile), band-Cholesky column records, cyclic-reduction levels.
int configure_solver(pba_engine* e, int K, int solver) {
  GnData& G = e->gn;
  const int nf = e->n_frames;
  hipStream_t st = e->stream;
  G.band_kernel = K;
  G.solver = solver;
  G.sband_dirty = false;
  if (K) {
    const size_t nb_ = (size_t)nf * ((K + 1) * 36 + 6);
    PBA_HIP(G.Lband.resize((size_t)nf * (K * 36 + 48)));  // column records
    PBA_HIP(G.Sband.resize(nb_));
    PBA_HIP(hipMemsetAsync(G.Sband.p, 0, nb_ * sizeof(double), st));  // positions outside the profile stay 0
  }
  G.cr_levels.clear();
  G.cr_pcr = -1;
  if (solver == SOLVER_CR) {
    const int M = 6 * K;
    // Parallel cyclic reduction takes over (wave kernel, M = 24) once the rows fit one workgroup per CU:
    // PBA_PCR_CAP overrides the row limit (0: cyclic reduction only) — the tests force the hybrid with small caps
    int cap = 0;
    if (M == 24) {
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->opt.device) != hipSuccess) cus = 0;
      cap = cus;
      if (const char* v = std::getenv("PBA_PCR_CAP")) cap = std::atoi(v);
    }
    std::vector<int> ns{(nf + K - 1) / K};
    while (ns.back() > (cap > 0 ? cap : 1)) ns.push_back((ns.back() + 1) / 2);
    if (cap > 0) G.cr_pcr = (int)ns.size() - 1;
    const int np = cap > 0 ? ns.back() : 0;
    size_t total = 2 * ((size_t)np * M * M * 2 + (size_t)np * M);
    for (int n : ns) total += (size_t)n * M * M * 2 + (size_t)n * M * 2 + (size_t)(n / 2) * M * (2 * M + 1);
    PBA_HIP(G.cr_buf.resize(total));
    size_t off = 0;
    for (int n : ns) {
      CrLevelHost L;
      L.n = n;
      L.D = off; off += (size_t)n * M * M;
      L.U = off; off += (size_t)n * M * M;
      L.b = off; off += (size_t)n * M;
      L.x = off; off += (size_t)n * M;
      L.X = off; off += (size_t)(n / 2) * M * (2 * M + 1);
      G.cr_levels.push_back(L);
    }
    for (CrLevelHost& P : G.pcr_bufs) {
      P.n = np;
      P.D = off; off += (size_t)np * M * M;
      P.U = off; off += (size_t)np * M * M;
      P.b = off; off += (size_t)np * M;
    }
    G.cr0_dirty = true;  // level 0 is set up for assemble_kernel's direct writes on first use
    G.cr0_inited = false;
  }
  return PBA_OK;
}

// Symbolic analysis: GN block order, chunks, slot layouts, skyline profile and contribution lists.
// The rows of each column's profile: column k → every i > k with first(i) ≤ k, in order (CSR).
void profile_columns(const std::vector<int>& first, std::vector<int>& ccptr, std::vector<int>& ccrows) {
  const int n = (int)first.size();
  std::vector<std::vector<int>> col(n);
  for (int i = 0; i < n; ++i)
    for (int k = first[i]; k < i; ++k) col[k].push_back(i);
  ccptr.assign(n + 1, 0);
  ccrows.clear();
  for (int k = 0; k < n; ++k) {
    ccptr[k + 1] = ccptr[k] + (int)col[k].size();
    ccrows.insert(ccrows.end(), col[k].begin(), col[k].end());
  }
  if (ccrows.empty()) ccrows.push_back(0);
}

// front_solve_kernel's plan for a skyline profile (first(i), row offsets rowp, column lists): static slots — a row
// admitted for column k + 1 never takes a slot in use at column k — and the per-column records (see the kernel).
// P.lds = 0 when the front does not fit (or use = false): the caller then takes skyline_solve_kernel.
int build_front_plan(const std::vector<int>& first, const std::vector<int>& rowp, const std::vector<int>& ccptr,
                     const std::vector<int>& ccrows, hipStream_t st, FrontPlan& P, bool use) {
  const int nfs = (int)first.size();
  std::vector<std::vector<int>> adm(nfs);
  for (int i = 0; i < nfs; ++i) adm[first[i]].push_back(i);
  std::vector<int> slot(nfs, -1), freel;
  int F = 0;
  auto alloc = [&]() {
    if (freel.empty()) return F++;
    auto it = std::min_element(freel.begin(), freel.end());
    const int v = *it;
    freel.erase(it);
    return v;
  };
  for (int i : adm[0]) slot[i] = alloc();
  for (int k = 0; k < nfs; ++k) {
    if (k + 1 < nfs)
      for (int i : adm[k + 1]) slot[i] = alloc();
    freel.push_back(slot[k]);
  }
  // active set after column k's admissions: (A_k \ {k}) ∪ adm(k+1), kept sorted
  std::vector<std::vector<int2>> fresh(nfs);  // per column k: the blocks of the rows admitted for k + 1
  std::vector<int2> init;
  std::vector<int> act;
  auto blk = [&](int hi, int lo) { return rowp[hi] + (lo - first[hi]); };
  auto add_rows = [&](const std::vector<int>& newr, std::vector<int>& A, std::vector<int2>& out) {
    for (int i : newr) A.push_back(i);
    std::sort(A.begin(), A.end());
    for (int i : newr)
      for (int j : A) {
        if (j > i && std::binary_search(newr.begin(), newr.end(), j)) continue;  // the pair once (from j)
        const int hi = std::max(i, j), lo = std::min(i, j);
        out.push_back(make_int2(blk(hi, lo), slot[hi] * F + slot[lo]));
      }
  };
  add_rows(adm[0], act, init);
  int fm = 1, mf = 1;
  for (int k = 0; k < nfs; ++k) {
    fm = std::max(fm, ccptr[k + 1] - ccptr[k]);
    act.erase(std::remove(act.begin(), act.end(), k), act.end());
    if (k + 1 < nfs) add_rows(adm[k + 1], act, fresh[k]);
    mf = std::max(mf, (int)fresh[k].size());
  }
  const int R = kFrontHdr + 3 * fm + 2 * mf, SB = fm * 36 + 48;
  const size_t lds = sizeof(double) * ((size_t)F * F * 36 + 6 * (size_t)nfs + 2 * SB) +
                     sizeof(int) * (3 * (size_t)R + fm * (fm + 1) / 2);
  P.lds = 0;
  if (!use || fm > 32 || mf * 36 > 256 * kFrontPf || SB > 256 * kFrontPf || R > 256 * kFrontPr || lds > 150 * 1024)
    return PBA_OK;
  std::vector<int> rec((size_t)nfs * R, 0);
  for (int k = 0; k < nfs; ++k) {
    int* r = rec.data() + (size_t)k * R;
    const int na = ccptr[k + 1] - ccptr[k];
    r[0] = slot[k];
    r[1] = na;
    r[2] = (int)fresh[k].size();
    for (int li = 0; li < na; ++li) {
      const int i = ccrows[ccptr[k] + li];
      r[kFrontHdr + li] = slot[i];
      r[kFrontHdr + fm + li] = i;
      r[kFrontHdr + 2 * fm + li] = blk(i, k);
    }
    for (int q = 0; q < (int)fresh[k].size(); ++q) {
      r[kFrontHdr + 3 * fm + q] = fresh[k][q].x;
      r[kFrontHdr + 3 * fm + mf + q] = fresh[k][q].y;
    }
  }
  PBA_HIP(P.rec.upload(rec, st));
  P.n_init = (int)init.size();
  if (init.empty()) init.push_back(make_int2(0, 0));
  PBA_HIP(P.init.upload(init, st));
  PBA_HIP(P.lrec.resize((size_t)nfs * 48));
  P.F = F;
  P.fm = fm;
  P.mf = mf;
  P.R = R;
  P.lds = lds;
  return PBA_OK;
}

// S δ = −g by front_solve_kernel with plan P (S: the profile's skyline blocks; L: room for its factor).
int launch_front(pba_engine* e, FrontPlan& P, const double* S, double* L, int N) {
  GnData& G = e->gn;
  FrontArgs fa{S, G.g.p, L, P.lrec.p, P.rec.p, P.init.p, G.x.p, G.status.p, N, P.F, P.fm, P.mf, P.R, P.n_init};
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&front_solve_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.lds);  // may exceed 64 KB
  front_solve_kernel<<<1, 256, P.lds, e->stream>>>(fa);
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

int gn_prepare(pba_engine* e) {
  GnData& G = e->gn;
  const int nb = e->n_blocks, nf = e->n_frames;
  if (nb <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_blocks first");
  G.lpb = gn_lpb(e);
  G.ppl = gn_ppl(e);
  G.bpw = kBlockThreads / G.lpb;
  const std::vector<int>& ph = e->point_host_h;
  // GN order: (host, point, target)
  std::vector<int> order(nb);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    const int pa_ = e->block_point_h[a], pb_ = e->block_point_h[b];
    if (ph[pa_] != ph[pb_]) return ph[pa_] < ph[pb_];
    if (pa_ != pb_) return pa_ < pb_;
    return e->block_target_h[a] < e->block_target_h[b];
  });
  std::vector<int> gtgt(nb);
  for (int i = 0; i < nb; ++i) gtgt[i] = e->block_target_h[order[i]];
  // linearise order: each host's GN range regrouped by target (stable), so a chunk's blocks of one target are
  // consecutive (one matrix-core chain per target run in linearize_kernel)
  std::vector<int> lpos(nb);
  std::iota(lpos.begin(), lpos.end(), 0);
  for (int i = 0; i < nb;) {
    const int h = ph[e->block_point_h[order[i]]];
    int j = i;
    while (j < nb && ph[e->block_point_h[order[j]]] == h) ++j;
    std::stable_sort(lpos.begin() + i, lpos.begin() + j, [&](int x, int y) { return gtgt[x] < gtgt[y]; });
    i = j;
  }
  // linearise chunks
  std::vector<int4> cdesc;
  std::vector<uint8_t> blt(nb);
  std::vector<std::vector<int>> chunk_targets;
  std::vector<int> chunk_host;
  size_t off = 0;
  for (int i = 0; i < nb;) {
    const int h = ph[e->block_point_h[order[lpos[i]]]];
    int j = i;
    std::vector<int> tg;
    while (j < nb && j - i < G.bpw && ph[e->block_point_h[order[lpos[j]]]] == h) {
      const int t = gtgt[lpos[j]];
      auto it = std::find(tg.begin(), tg.end(), t);
      if (it == tg.end() && (int)tg.size() == kChunkTargets) break;  // a chunk spans ≤ kChunkTargets targets
      blt[j] = (uint8_t)(it - tg.begin());
      if (it == tg.end()) tg.push_back(t);
      ++j;
    }
    cdesc.push_back(make_int4(i, j - i, (int)tg.size(), (int)off));
    off += SLOT_LIN_BASE + SLOT_LIN_T * tg.size();
    chunk_targets.push_back(tg);
    chunk_host.push_back(h);
    i = j;
  }
  G.lin_slots = off;
  G.n_chunks = (int)cdesc.size();
  // GN points
  std::vector<int> pfirst, pnblk, porig, phost;
  for (int i = 0; i < nb;) {
    const int p = e->block_point_h[order[i]];
    int j = i;
    while (j < nb && e->block_point_h[order[j]] == p) ++j;
    pfirst.push_back(i);
    pnblk.push_back(j - i);
    porig.push_back(p);
    phost.push_back(ph[p]);
    i = j;
  }
  const int ngp = (int)pfirst.size();
  G.n_gn_points = ngp;
  // Schur chunks
  G.schur_lds = 0;
  std::vector<int4> sdesc;
  std::vector<int4> saux;
  std::vector<uchar2> spairs;
  std::vector<int> lvp;
  int max_nv = 1;
  std::vector<std::vector<char>> schur_used_flag;
  std::vector<uint8_t> blv(nb, 0);
  std::vector<std::vector<int>> schur_poses;
  std::vector<std::vector<std::pair<int, int>>> schur_used;
  size_t soff = 0;
  for (int p = 0; p < ngp;) {
    const int h = phost[p];
    std::vector<int> poses{h};
    int q = p;
    while (q < ngp && q - p < SCHUR_PTS && phost[q] == h) {
      std::vector<int> add;
      for (int b = pfirst[q]; b < pfirst[q] + pnblk[q]; ++b)
        if (std::find(poses.begin(), poses.end(), gtgt[b]) == poses.end() &&
            std::find(add.begin(), add.end(), gtgt[b]) == add.end())
          add.push_back(gtgt[b]);
      const int nv = (int)(poses.size() + add.size());
      if (q > p && ((q - p + 1) * nv > SCHUR_W || nv > 255)) break;
      if (nv > 255 || nv > SCHUR_W) return fail(PBA_ERR_INVALID_ARGUMENT, "a point observes too many keyframes");
      poses.insert(poses.end(), add.begin(), add.end());
      ++q;
    }
    const int nv = (int)poses.size();
    std::vector<char> used(nv * nv, 0);
    std::vector<int> lpair(nv, 0);  // the pair (host, poses[l]) of each local target
    for (int r = p; r < q; ++r) {
      std::vector<int> lv{0};
      for (int b = pfirst[r]; b < pfirst[r] + pnblk[r]; ++b) {
        const int l = (int)(std::find(poses.begin(), poses.end(), gtgt[b]) - poses.begin());
        blv[b] = (uint8_t)l;
        lpair[l] = e->pair_of_h[order[b]];
        lv.push_back(l);
      }
      for (int x : lv)
        for (int y : lv) used[std::min(x, y) * nv + std::max(x, y)] = 1;
    }
    // pair slots: the used pairs, or every pair (a ≤ b) in canonical order when the chunk takes the matrix-core path
    // of schur_kernel (≤ 5 local poses; unused pairs are zero blocks no contribution list references)
    const bool canon = nv * 6 + 1 <= 32;
    std::vector<std::pair<int, int>> up;
    std::vector<char> upu;
    for (int x = 0; x < nv; ++x)
      for (int y = x; y < nv; ++y)
        if (canon || used[x * nv + y]) {
          up.emplace_back(x, y);
          upu.push_back(used[x * nv + y]);
        }
    const int fb0 = pfirst[p], nbc = pfirst[q - 1] + pnblk[q - 1] - fb0;
    saux.push_back(make_int4((int)spairs.size(), (int)up.size(), (int)lvp.size(), nbc));
    lvp.insert(lvp.end(), lpair.begin() + 1, lpair.end());
    max_nv = std::max(max_nv, nv);
    for (auto& pr : up) spairs.push_back(make_uchar2((unsigned char)pr.first, (unsigned char)pr.second));
    sdesc.push_back(make_int4(p, q - p, nv, (int)soff));
    G.schur_lds = std::max<size_t>(G.schur_lds, sizeof(double) * 6 * (size_t)(q - p) * nv);
    soff += 36 * up.size() + 6 * nv;
    schur_poses.push_back(poses);
    schur_used.push_back(up);
    schur_used_flag.push_back(upu);
    p = q;
  }
  G.schur_doubles = soff;
  G.schur_rt_off = 12 * (max_nv - 1);  // the chunks' target poses, then W (schur_chunk)
  G.schur_lds += sizeof(double) * G.schur_rt_off;
  G.n_schur = (int)sdesc.size();
  {  // chunk c's point p → {first GN block, block count} at c · SCHUR_PTS + p (schur_kernel reads it with its descriptor)
    std::vector<int2> fbt((size_t)G.n_schur * SCHUR_PTS, make_int2(0, 0));
    for (int c = 0; c < G.n_schur; ++c)
      for (int q = 0; q < sdesc[c].y; ++q) fbt[(size_t)c * SCHUR_PTS + q] = make_int2(pfirst[sdesc[c].x + q], pnblk[sdesc[c].x + q]);
    PBA_HIP(G.pt_fb.upload(fbt, e->stream));
  }
  // reduced camera system structure: lower blocks (i ≥ j)
  std::map<std::pair<int, int>, std::vector<int2>> contrib;
  std::vector<std::vector<int2>> gcon(nf);
  auto add = [&](int fa, int fb, int o, int flags) {  // contribution block in orientation (fa rows, fb cols)
    if (fa >= fb) contrib[{fa, fb}].push_back(make_int2(o, flags));
    else contrib[{fb, fa}].push_back(make_int2(o, flags | C_TRANSPOSE));
  };
  std::vector<char> observed(nf, 0);
  for (int c = 0; c < G.n_chunks; ++c) {
    const int h = chunk_host[c], o = cdesc[c].w;
    observed[h] = 1;
    add(h, h, o, 0);
    gcon[h].push_back(make_int2(o + 36, 0));
    for (size_t j = 0; j < chunk_targets[c].size(); ++j) {
      const int t = chunk_targets[c][j], bo = o + SLOT_LIN_BASE + SLOT_LIN_T * (int)j;
      observed[t] = 1;
      add(h, t, bo, 0);
      add(t, t, bo + 36, 0);
      gcon[t].push_back(make_int2(bo + 72, 0));
    }
  }
  for (int s = 0; s < G.n_schur; ++s) {
    const auto& poses = schur_poses[s];
    const int o = sdesc[s].w;
    for (size_t u = 0; u < schur_used[s].size(); ++u) {
      if (!schur_used_flag[s][u]) continue;
      const int fa = poses[schur_used[s][u].first], fb = poses[schur_used[s][u].second];
      add(fa, fb, o + 36 * (int)u, C_SCHUR);
    }
    for (size_t a = 0; a < poses.size(); ++a)
      gcon[poses[a]].push_back(make_int2(o + 36 * (int)schur_used[s].size() + 6 * (int)a, C_SCHUR));
  }
  // free intrinsics (geometric): two system frames per camera after the keyframes, a dense border (profile from 0)
  const int nc = (e->opt_intr && e->opt.residual_kind == PBA_RESIDUAL_GEOMETRIC) ? e->n_cams : 0;
  const int nfs = nf + 2 * nc;
  G.nc_sys = nc;
  G.nfs = nfs;
  G.dsky_K = -1;  // the multi-GPU summed profile is rebuilt for this problem (ensure_dist_sky)
  for (int i = 0; i < nfs; ++i) contrib[{i, i}];  // every diagonal block exists
  std::vector<int> first(nfs), rowp(nfs + 1), last(nfs);
  for (int i = 0; i < nfs; ++i) first[i] = i < nf ? i : 0;
  for (auto& kv : contrib) first[kv.first.first] = std::min(first[kv.first.first], kv.first.second);
  rowp[0] = 0;
  for (int i = 0; i < nfs; ++i) rowp[i + 1] = rowp[i] + (i - first[i] + 1);
  G.n_sky = rowp[nfs];
  G.band = 0;  // over the keyframes (the free-intrinsics border rows start at frame 0)
  for (int i = 0; i < nf; ++i) G.band = std::max(G.band, i - first[i]);
  for (int k = 0; k < nfs; ++k) last[k] = k;
  for (int i = 0; i < nfs; ++i)
    for (int k = first[i]; k < i; ++k) last[k] = std::max(last[k], i);
  std::vector<int> ccptr, ccrows;  // the rows of each column's profile, in order
  profile_columns(first, ccptr, ccrows);
  if (int rc = build_front_plan(first, rowp, ccptr, ccrows, e->stream, G.front, getenv("PBA_SKYLINE_GLOBAL") == nullptr))
    return rc;
  std::vector<int> cptr(G.n_sky + 1, 0), bi(G.n_sky), bj(G.n_sky);
  std::vector<std::vector<int2>> per(G.n_sky);
  for (int i = 0; i < nfs; ++i)
    for (int j = first[i]; j <= i; ++j) {
      const int s = rowp[i] + (j - first[i]);
      bi[s] = i;
      bj[s] = j;
    }
  for (auto& kv : contrib) {
    const int s = rowp[kv.first.first] + (kv.first.second - first[kv.first.first]);
    per[s] = kv.second;
  }
  std::vector<int2> flat;
  for (int s = 0; s < G.n_sky; ++s) {
    cptr[s] = (int)flat.size();
    flat.insert(flat.end(), per[s].begin(), per[s].end());
  }
  cptr[G.n_sky] = (int)flat.size();
  std::vector<int> gptr(nfs + 1);
  std::vector<int2> gflat;
  for (int i = 0; i < nfs; ++i) {
    gptr[i] = (int)gflat.size();
    if (i < nf) gflat.insert(gflat.end(), gcon[i].begin(), gcon[i].end());
  }
  gptr[nfs] = (int)gflat.size();
  // constant frames: requested + never observed; a camera whose intrinsics no block projects with is constant too
  std::vector<uint8_t> fixed(nfs, 0);
  for (int i = 0; i < nf; ++i) fixed[i] = (i < (int)G.fixed_h.size() && G.fixed_h[i]) || !observed[i];
  if (nc) {
    // the border's CSR lists: unit pair (camera c, unit u), u < nf keyframe u, u ≥ nf camera u − nf; direct terms from
    // the blocks whose target camera is c and that touch u (host or target u; u = c: every block of camera c), Schur
    // terms from the points with a block of camera c that touch u (a block of keyframe u / of camera u − nf)
    const int nu = nf + nc;
    std::vector<std::vector<int>> bl((size_t)nc * nu), pl((size_t)nc * nu), pk((size_t)nc * nu);
    const bool walk = test_hook("PBA_TEST_PBLK_WALK") != nullptr;  // (tests: every target entry walks its point's blocks)
    std::vector<int> bcam(nb);
    std::vector<int4> ibrec(nb);
    std::vector<char> cam_seen(nc, 0);
    for (int gb = 0; gb < nb; ++gb) {
      const int b = order[gb], pt = e->block_point_h[b], h = ph[pt], t = e->block_target_h[b], c = e->frame_cam_h[t];
      bcam[gb] = c;
      ibrec[gb] = make_int4(b, pt, h, t);
      cam_seen[c] = 1;
      bl[(size_t)c * nu + h].push_back((int)((unsigned)gb | 0x80000000u));  // (bit 31: the unit hosts the block)
      bl[(size_t)c * nu + t].push_back(gb);
      bl[(size_t)c * nu + nf + c].push_back(gb);
    }
    for (int q = 0; q < ngp; ++q) {
      std::vector<int> cams, units{phost[q]};
      for (int gb = pfirst[q]; gb < pfirst[q] + pnblk[q]; ++gb) {
        if (std::find(cams.begin(), cams.end(), bcam[gb]) == cams.end()) cams.push_back(bcam[gb]);
        if (std::find(units.begin(), units.end(), gtgt[gb]) == units.end()) units.push_back(gtgt[gb]);
      }
      for (int c : cams) units.push_back(nf + c);
      for (int c : cams)
        for (int u : units) {
          pl[(size_t)c * nu + u].push_back(q);
          // the border kernel's Schur term for keyframe u: −1 u hosts the point, else its one block targeting u
          int by = -1;
          if (u < nf && u != phost[q]) {
            int n_u = 0;
            for (int gb = pfirst[q]; gb < pfirst[q] + pnblk[q]; ++gb)
              if (gtgt[gb] == u) {
                by = gb;
                ++n_u;
              }
            if (n_u != 1 || walk) by = -2;
          }
          pk[(size_t)c * nu + u].push_back(by);
        }
    }
    std::vector<int> bp(1, 0), bflat, pp(1, 0), pflat, pkflat;
    for (size_t L = 0; L < bl.size(); ++L) {
      bflat.insert(bflat.end(), bl[L].begin(), bl[L].end());
      bp.push_back((int)bflat.size());
      pflat.insert(pflat.end(), pl[L].begin(), pl[L].end());
      pkflat.insert(pkflat.end(), pk[L].begin(), pk[L].end());
      pp.push_back((int)pflat.size());
    }
    if (bflat.empty()) bflat.push_back(0);
    if (pflat.empty()) pflat.push_back(0);
    if (pkflat.empty()) pkflat.push_back(-1);
    for (int c = 0; c < nc; ++c) fixed[nf + 2 * c] = fixed[nf + 2 * c + 1] = !cam_seen[c];
    hipStream_t st0 = e->stream;
    PBA_HIP(G.ib_rec.upload(ibrec, st0));
    PBA_HIP(G.ib_cam.upload(bcam, st0));
    PBA_HIP(G.ib_bptr.upload(bp, st0));
    PBA_HIP(G.ib_blist.upload(bflat, st0));
    PBA_HIP(G.ib_pptr.upload(pp, st0));
    PBA_HIP(G.ib_plist.upload(pflat, st0));
    PBA_HIP(G.ib_pblk.upload(pkflat, st0));
    // point-aligned waves for intr_rows_kernel (whole points of ≤ 64 blocks each; a longer point: consecutive waves and
    // the separate point sums of intr_pw_kernel)
    {
      std::vector<int4> wt;
      bool fits = true;
      for (int q = 0; q < ngp && fits; ++q) {
        if (pnblk[q] > 64) fits = false;
        else if (wt.empty() || wt.back().y + pnblk[q] > 64) wt.push_back(make_int4(pfirst[q], pnblk[q], q, 0));
        else wt.back().y += pnblk[q];
      }
      // (the GN points cover the GN blocks in order: pfirst[q + 1] = pfirst[q] + pnblk[q], checked here)
      for (int q = 0; q + 1 < ngp && fits; ++q) fits = pfirst[q + 1] == pfirst[q] + pnblk[q];
      fits = fits && ngp > 0 && pfirst[0] == 0 && pfirst[ngp - 1] + pnblk[ngp - 1] == nb;
      if (test_hook("PBA_TEST_ROW_WAVES64")) fits = false;  // (tests: the 64-block waves + intr_pw_kernel path)
      G.ir_waves = fits ? (int)wt.size() : 0;
      if (fits) PBA_HIP(G.ir_wave.upload(wt, st0));
    }
    PBA_HIP(G.ib_data.resize((size_t)nb * kIbStride));
    PBA_HIP(G.ib_pw.resize((size_t)std::max(ngp, 1) * (8 * nc + 6)));
    PBA_HIP(G.ib_part.resize((size_t)kCamSplit * (nc * kCamDir + nc * (nc + 1) / 2 * kCamSch)));
    PBA_HIP(G.intr_new_d.resize((size_t)kCamD * nc));
    PBA_HIP(G.intr_new_f.resize((size_t)8 * nc));
    // the candidate records start as the state's (their unprojection half is never read: hosts unproject with the cameras)
    PBA_HIP(hipMemcpyAsync(G.intr_new_d.p, e->intr_state_d.p, sizeof(double) * kCamD * nc, hipMemcpyDeviceToDevice, st0));
    PBA_HIP(hipMemcpyAsync(G.intr_new_f.p, e->intr_state.p, sizeof(float) * 8 * nc, hipMemcpyDeviceToDevice, st0));
  }
  // upload
  hipStream_t st = e->stream;
  if (e->n_pairs >= (1 << 24)) return fail(PBA_ERR_INVALID_ARGUMENT, "more than 2^24 (host, target) pairs");
  std::vector<int4> lrec((size_t)G.n_chunks * G.bpw);
  for (int c = 0; c < G.n_chunks; ++c)
    for (int s = 0; s < G.bpw; ++s) {
      const int i = cdesc[c].x + (s < cdesc[c].y ? s : 0), b = order[lpos[i]];
      lrec[(size_t)c * G.bpw + s] = make_int4(b, e->block_point_h[b], e->pair_of_h[b] | ((int)blt[i] << 24), lpos[i]);
    }
  PBA_HIP(G.lin_rec.upload(lrec, st));
  PBA_HIP(G.chunk_desc.upload(cdesc, st));
  PBA_HIP(G.blk_schur.resize((size_t)nb * kPd));
  PBA_HIP(G.part_lin.resize(std::max<size_t>(G.lin_slots, 1)));
  PBA_HIP(G.blk_schur1.resize((size_t)nb * kPd));  // the device LM loop's second linearisation set
  PBA_HIP(G.pair_rt.resize((size_t)std::max(e->n_pairs, 1) * 12));
  PBA_HIP(G.pair_rt1.resize((size_t)std::max(e->n_pairs, 1) * 12));
  PBA_HIP(G.part_lin1.resize(std::max<size_t>(G.lin_slots, 1)));
  PBA_HIP(G.pt_first.upload(pfirst, st));
  PBA_HIP(G.pt_nblk.upload(pnblk, st));
  PBA_HIP(G.pt_orig.upload(porig, st));
  PBA_HIP(G.pt_host.upload(phost, st));
  {
    std::vector<int4> prec(ngp), ptgt(ngp);
    for (int q = 0; q < ngp; ++q) {
      prec[q] = make_int4(pfirst[q], pnblk[q], phost[q], porig[q]);
      int t4[4] = {0, 0, 0, 0};
      for (int u = 0; u < 4 && u < pnblk[q]; ++u) t4[u] = gtgt[pfirst[q] + u];
      ptgt[q] = make_int4(t4[0], t4[1], t4[2], t4[3]);
    }
    PBA_HIP(G.pt_rec.upload(prec, st));
    PBA_HIP(G.pt_tgt.upload(ptgt, st));
    std::vector<int4> parec(std::max(e->n_pairs, 1), make_int4(0, 0, 0, 0));
    for (int q = 0; q < e->n_pairs; ++q) {
      const int h = e->pair_host_h[q], t = e->pair_target_h[q];
      parec[q] = make_int4(h, t, e->frame_cam_h[h], e->frame_cam_h[t]);
    }
    PBA_HIP(G.pair_rec.upload(parec, st));
  }
  PBA_HIP(G.gn_target.upload(gtgt, st));
  PBA_HIP(G.schur_desc.upload(sdesc, st));
  PBA_HIP(G.schur_aux.upload(saux, st));
  PBA_HIP(G.schur_pairs.upload(spairs, st));
  PBA_HIP(G.blk_lv.upload(blv, st));
  {
    std::vector<int4> lvp4(sdesc.size(), make_int4(0, 0, 0, 0));
    for (size_t c = 0; c < sdesc.size(); ++c) {
      int l4[4] = {0, 0, 0, 0};
      for (int l = 0; l < 4 && l < sdesc[c].z - 1; ++l) l4[l] = lvp[saux[c].z + l];
      lvp4[c] = make_int4(l4[0], l4[1], l4[2], l4[3]);
    }
    if (lvp4.empty()) lvp4.push_back(make_int4(0, 0, 0, 0));
    PBA_HIP(G.schur_lvp4.upload(lvp4, st));
  }
  if (lvp.empty()) lvp.push_back(0);
  PBA_HIP(G.schur_lvp.upload(lvp, st));
  PBA_HIP(G.part_schur.resize(std::max<size_t>(G.schur_doubles, 1)));
  PBA_HIP(G.pt_data.resize((size_t)ngp * 8));
  PBA_HIP(G.pt_data1.resize((size_t)ngp * 8));
  PBA_HIP(G.part_free0.resize(std::max<size_t>(G.schur_doubles, 1)));
  PBA_HIP(G.part_free1.resize(std::max<size_t>(G.schur_doubles, 1)));
  PBA_HIP(G.degen.resize(2));
  PBA_HIP(G.lin_set.resize(1));
  PBA_HIP(hipMemsetAsync(G.degen.p, 0, 2 * sizeof(int), st));
  PBA_HIP(G.ts_part.resize((size_t)kDecideWgs * kTsCount));
  PBA_HIP(G.ts_count.resize(1));
  PBA_HIP(hipMemsetAsync(G.ts_count.p, 0, sizeof(int), st));
  PBA_HIP(G.sky_first.upload(first, st));
  PBA_HIP(G.sky_row.upload(rowp, st));
  PBA_HIP(G.sky_last.upload(last, st));
  PBA_HIP(G.sky_colptr.upload(ccptr, st));
  PBA_HIP(G.sky_colrows.upload(ccrows, st));
  PBA_HIP(G.sky_cptr.upload(cptr, st));
  PBA_HIP(G.sky_contrib.upload(flat.empty() ? std::vector<int2>{make_int2(0, 0)} : flat, st));
  PBA_HIP(G.g_cptr.upload(gptr, st));
  PBA_HIP(G.g_contrib.upload(gflat.empty() ? std::vector<int2>{make_int2(0, 0)} : gflat, st));
  PBA_HIP(G.sky_blk_i.upload(bi, st));
  PBA_HIP(G.sky_blk_j.upload(bj, st));
  {
    std::vector<int> dg, od;
    for (int q = 0; q < (int)bi.size(); ++q) (bi[q] == bj[q] ? dg : od).push_back(q);
    G.n_sky_diag = (int)dg.size();
    if (dg.empty()) dg.push_back(0);
    if (od.empty()) od.push_back(0);
    PBA_HIP(G.sky_diag.upload(dg, st));
    PBA_HIP(G.sky_off.upload(od, st));
  }
  PBA_HIP(G.fixed.upload(fixed, st));
  PBA_HIP(G.S.resize((size_t)G.n_sky * 36));
  PBA_HIP(G.L.resize((size_t)G.n_sky * 36));
  // solver choice: block cyclic reduction (bandwidth ≤ 8), LDS-window band Cholesky (≤ 16), skyline (any).
  // PBA_SOLVER=cr|band|skyline forces one (test hook; cr/band fall back when the bandwidth does not allow).
  const int K = nc ? 0 : band_kernel_for(G.band);  // the intrinsics border: skyline
  int solver = K && K <= 8 ? SOLVER_CR : (K ? SOLVER_BAND : SOLVER_SKYLINE);
  if (const char* fs = getenv("PBA_SOLVER")) {
    const std::string f(fs);
    if (f == "skyline") solver = SOLVER_SKYLINE;
    else if (f == "band" && K) solver = SOLVER_BAND;
    else if (f == "cr" && K && K <= 8) solver = SOLVER_CR;
  }
  if (int rc = configure_solver(e, solver == SOLVER_SKYLINE ? 0 : K, solver)) return rc;
  G.ar_n = G.ar_batches = 0;  // free intrinsics: the arrow solve's buffers (arrow_for decides per solve)
  if (nc > 0 && nc <= kArrowMaxNc)
    if (int rc = configure_arrow(e)) return rc;
  PBA_HIP(G.observed.upload(std::vector<uint8_t>(observed.begin(), observed.end()), st));
  std::vector<uint8_t> req(nf, 0);
  for (int i = 0; i < nf && i < (int)G.fixed_h.size(); ++i) req[i] = G.fixed_h[i];
  PBA_HIP(G.fixed_req.upload(req, st));
  PBA_HIP(G.fixed_dist.resize(nfs));
  PBA_HIP(G.g.resize((size_t)nfs * 6));
  PBA_HIP(G.g_dir.resize((size_t)nfs * 6));
  PBA_HIP(G.Ddiag.resize((size_t)nfs * 6));
  PBA_HIP(G.Linv.resize((size_t)nfs * 36));
  PBA_HIP(G.x.resize((size_t)nfs * 6));
  PBA_HIP(G.poses_new.resize((size_t)nf * 7));
  PBA_HIP(G.rho_new.resize((size_t)e->n_points));
  PBA_HIP(G.drho.resize((size_t)e->n_points));
  PBA_HIP(G.pairs_new.resize((size_t)e->n_pairs));
  PBA_HIP(G.status.resize(1));
  const int red_pose = (nfs + kBlockThreads - 1) / kBlockThreads;
  const int red_pt = (ngp + kBlockThreads - 1) / kBlockThreads;
  // update partials, then the candidate cost's workgroup partials (≤ one per 16 blocks: launch_cost_only's grids)
  G.red_slots = red_pose + red_pt + std::max({1024, nb / 16 + 2, G.n_chunks});
  PBA_HIP(G.red.resize((size_t)2 * G.red_slots));
  PBA_HIP(G.red2.resize((size_t)2 * (red_pose + red_pt)));
  PBA_HIP(G.gmax.resize((size_t)(red_pose + red_pt)));
  PBA_HIP(G.red_h.resize(2 * G.red_slots));
  PBA_HIP(G.lm.resize(kLmFields));
  PBA_HIP(G.tpose.resize(8));  // pose part (5), point gradient max-norm, solve status
  {  // the record of host-driven steps: not done, buffer set 0, λ NaN (the kernels then use their λ argument)
    std::vector<double> idle(kLmFields, 0.0);
    idle[kLmLambda] = std::numeric_limits<double>::quiet_NaN();
    PBA_HIP(G.lm_idle.upload(idle, st));
  }
  // decision record + sequence number, written by lm_decide_kernel over the bus (fine-grained host memory)
  PBA_HIP(G.lm_h.resize(kRecRing * kRecStride, hipHostMallocCoherent | hipHostMallocMapped));
  PBA_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&G.lm_host_d), G.lm_h.p, 0));
  PBA_HIP(hipMemsetAsync(G.drho.p, 0, sizeof(double) * e->n_points, st));
  PBA_HIP(hipStreamSynchronize(st));
  G.prepared = true;
  G.pairs_new_fresh = false;
  G.fixed_eff = fixed;
  return PBA_OK;
}

template <int KIND, int MODEL>  // photometric: MODEL = camera model + 4 · interpolator
void launch_linearize(pba_engine* e, const KernelArgs& ka, const LinArgs& la) {
  const int grid = la.n_chunks;
  if constexpr (KIND == PBA_RESIDUAL_PHOTOMETRIC) {
    switch (e->gn.ppl) {  // 9…32 px: 8 lanes per block, ⌈P/8⌉ rows per lane
      case 1: break;
      case 2: linearize_adj_kernel<MODEL, 2, kBlockThreads><<<grid, kBlockThreads, 0, e->stream>>>(ka, la); return;
      case 3: linearize_adj_kernel<MODEL, 3, kBlockThreads><<<grid, kBlockThreads, 0, e->stream>>>(ka, la); return;
      default: linearize_adj_kernel<MODEL, 4, kBlockThreads><<<grid, kBlockThreads, 0, e->stream>>>(ka, la); return;
    }
    // the 14-column products of the same rows: the A/B reference of the test build (PBA_TEST_HOOKS, PBA_LIN_LEGACY)
    if (e->gn.lin_legacy) linearize_kernel<KIND, MODEL, 8><<<grid, kBlockThreads, 0, e->stream>>>(ka, la);
    else linearize_adj_kernel<MODEL, 1, kBlockThreads><<<grid, kBlockThreads, 0, e->stream>>>(ka, la);
  } else {
    linearize_kernel<KIND, MODEL, 4><<<grid, kBlockThreads, 0, e->stream>>>(ka, la);
  }
}

void launch_linearize_photometric(pba_engine* e, const KernelArgs& ka, const LinArgs& la) {
  switch (e->opt.camera_model + 4 * e->interp) {
    case 0: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 0>(e, ka, la); break;
    case 1: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 1>(e, ka, la); break;
    case 2: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 2>(e, ka, la); break;
    case 3: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 3>(e, ka, la); break;
    case 4: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 4>(e, ka, la); break;
    case 5: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 5>(e, ka, la); break;
    case 6: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 6>(e, ka, la); break;
    default: launch_linearize<PBA_RESIDUAL_PHOTOMETRIC, 7>(e, ka, la); break;
  }
}

void launch_linearize_geometric(pba_engine* e, const KernelArgs& ka, const LinArgs& la) {
  switch (e->opt.camera_model) {
    case PBA_CAMERA_PINHOLE: launch_linearize<PBA_RESIDUAL_GEOMETRIC, CAM_PINHOLE>(e, ka, la); break;
    case PBA_CAMERA_DOUBLE_SPHERE: launch_linearize<PBA_RESIDUAL_GEOMETRIC, CAM_DS>(e, ka, la); break;
    case PBA_CAMERA_EUCM: launch_linearize<PBA_RESIDUAL_GEOMETRIC, CAM_EUCM>(e, ka, la); break;
    default: launch_linearize<PBA_RESIDUAL_GEOMETRIC, CAM_KB4>(e, ka, la); break;
  }
}

int ensure_prepared(pba_engine* e) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (e->n_blocks <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_blocks first");
  if (!e->state_set) return fail(PBA_ERR_NOT_READY, "pba_set_state first");
  if (e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC && (!e->have_images || e->P <= 0))
    return fail(PBA_ERR_NOT_READY, "images/pattern missing");
  if (int rc = check_device(e)) return rc;
  if (!e->gn.prepared)
    if (int rc = gn_prepare(e)) return rc;
  return PBA_OK;
}

// Σ of 2-vectors over `slots` reduction slots, in fixed order on the host.
int read_red(pba_engine* e, int slots, double* a, double* b) {
  GnData& G = e->gn;
  PBA_HIP(hipMemcpyAsync(G.red_h.data(), G.red.p, sizeof(double) * 2 * slots, hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  double x = 0, y = 0;
  for (int i = 0; i < slots; ++i) {
    x += G.red_h[2 * i];
    y += G.red_h[2 * i + 1];
  }
  *a = x;
  if (b) *b = y;
  return PBA_OK;
}

int total_cost(pba_engine* e, double* cost, int* n_valid) {
  const int grid = std::min(1024, (e->n_blocks + kBlockThreads - 1) / kBlockThreads);
  cost_reduce_kernel<<<grid, kBlockThreads, 0, e->stream>>>(e->cost.p, e->valid.p, e->n_blocks, e->gn.red.p);
  PBA_HIP(hipGetLastError());
  double c, v;
  if (int rc = read_red(e, grid, &c, &v)) return rc;
  *cost = c;
  if (n_valid) *n_valid = (int)v;
  return PBA_OK;
}

// Linearisation at the engine's state (pairs == nullptr: formed here), or — the device LM loop — at the candidate:
// lm = the device LM record (the pieces go to the spare buffer set, nothing runs once the solve is done), pairs / rho
// the candidate's, and wg_red the slots of the per-chunk cost partials the decision sums.
// cand_intr: with free intrinsics, project with the candidate's (G.intr_new_*) instead of the state's.
// mark_set: record the set written (and clear its degen flag) for the λ-free elimination that follows.
int linearize(pba_engine* e, double* cost, const double* lm = nullptr, const PairRec* pairs = nullptr,
              const double* rho = nullptr, double* wg_red = nullptr, int* n_valid = nullptr, bool cand_intr = false,
              bool mark_set = false) {
  GnData& G = e->gn;
  if (!pairs) {
    launch_pairs(e, e->poses.p, e->pairs.p);
    pairs = e->pairs.p;
  }
  KernelArgs ka = make_kernel_args(e, pairs, rho ? rho : e->rho.p);
  if (cand_intr && G.nc_sys) {
    ka.intr_t = G.intr_new_f.p;
    ka.intr_t_d = G.intr_new_d.p;
  }
  LinArgs la{G.lin_rec.p, G.blk_schur1.p, G.part_lin1.p, wg_red, G.chunk_desc.p, G.blk_schur.p, G.part_lin.p, G.n_chunks,
             lm ? lm : G.lm_idle.p, lm != nullptr, mark_set ? G.lin_set.p : nullptr, mark_set ? G.degen.p : nullptr,
             G.pair_rt.p, G.pair_rt1.p};
  if (e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC) launch_linearize_photometric(e, ka, la);
  else launch_linearize_geometric(e, ka, la);
  PBA_HIP(hipGetLastError());
  e->evaluated = false;  // records are not written in GN mode
  if (cost) return total_cost(e, cost, n_valid);
  return PBA_OK;
}

CrLevel cr_level(GnData& G, int l) {
  const CrLevelHost& h = G.cr_levels[l];
  double* base = G.cr_buf.p;
  return CrLevel{base + h.D, base + h.U, base + h.b, base + h.X, base + h.x, h.n};
}
CrLevel pcr_level(GnData& G, int i) {  // PCR ping-pong buffer i (D, U, b of the rows of level G.cr_pcr)
  const CrLevelHost& h = G.pcr_bufs[i];
  double* base = G.cr_buf.p;
  return CrLevel{base + h.D, base + h.U, base + h.b, nullptr, nullptr, h.n};
}

// Level 0 of the cyclic reduction as assemble_kernel expects it: zeros (positions outside the reduced system's profile
// are never written), identity diagonal on the padding rows past the last keyframe.
int init_cr_level0(pba_engine* e) {
  GnData& G = e->gn;
  if (G.cr_levels.empty()) return PBA_OK;
  const int B = G.band_kernel, M = 6 * B, N = e->n_frames;
  const CrLevelHost& h = G.cr_levels[0];
  std::vector<double> z((size_t)h.n * M * M * 2 + (size_t)h.n * M, 0.0);  // D | U | b (contiguous: configure_solver)
  for (int I = 0; I < h.n; ++I)
    for (int R = 0; R < M; ++R)
      if (I * B + R / 6 >= N) z[(size_t)I * M * M + (size_t)R * M + R] = 1.0;
  PBA_HIP(hipMemcpyAsync(G.cr_buf.p + h.D, z.data(), z.size() * sizeof(double), hipMemcpyHostToDevice, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));  // z is pageable and goes out of scope
  G.cr0_dirty = false;
  G.cr0_inited = true;
  return PBA_OK;
}

// build: level 0 from Sband (cr_build_kernel); false when assemble_kernel wrote it directly
template <int M>
void cr_solve(pba_engine* e, bool build) {
  GnData& G = e->gn;
  if (cr_level_lds<M>() > 65536) {  // above the default dynamic-LDS limit (gfx950 has 160 KiB per CU)
    // the attribute is per device: set it on every solve (cheap) rather than once per process
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cr_level_kernel<M>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)cr_level_lds<M>());
  }
  const int nl = (int)G.cr_levels.size();
  CrLevel L0 = cr_level(G, 0);
  const long long nthreads = (long long)L0.n * M * M + (long long)L0.n * M;
  if (build)
    cr_build_kernel<M><<<(unsigned)((nthreads + 255) / 256), 256, 0, e->stream>>>(G.Sband.p, L0, e->n_frames,
                                                                                  G.band_kernel, G.status.p);
  // CR levels 0 … c−1 (one fused launch each: odd eliminations + even rebuild); level c is solved either by PCR
  // levels (G.cr_pcr = c) or, as the last CR level of one row, by the root kernel
  const int c = G.cr_pcr >= 0 ? G.cr_pcr : nl - 1;
  for (int l = 0; l < c; ++l) {
    CrLevel L = cr_level(G, l), Ln = cr_level(G, l + 1);
    if constexpr (2 * M + 1 <= 64) {
      cr_level_wave_kernel<M, false><<<(L.n + 1) / 2, 256, cr_level_wave_lds<M>(), e->stream>>>(L, Ln, 1, G.status.p,
                                                                                               nullptr, 0);
    } else
      cr_level_kernel<M><<<(L.n + 1) / 2, 2 * kCrOddThreads<M>, cr_level_lds<M>(), e->stream>>>(L, Ln, G.status.p);
  }
  bool solved = false;  // the step vector already written (level c = 0 solved in place)
  if constexpr (2 * M + 1 <= 64) {
    if (G.cr_pcr >= 0) {
      CrLevel src = cr_level(G, c);
      const int n = src.n;
      solved = c == 0;
      double* out = solved ? G.x.p : cr_level(G, c).x;
      const int lim = solved ? 6 * e->n_frames : n * M;
      int pi = 0;
      for (int s = 1; s < n; s *= 2, pi ^= 1) {  // the last level also solves the decoupled rows
        CrLevel dst = pcr_level(G, pi);
        const bool last = 2 * s >= n;
        cr_level_wave_kernel<M, true><<<n, 256, cr_level_wave_lds<M>(), e->stream>>>(src, dst, s, G.status.p,
                                                                                     last ? out : nullptr, lim);
        src = dst;
      }
      if (n <= 1) pcr_solve_kernel<M><<<n, 64, 0, e->stream>>>(src, out, lim, G.status.p);
    } else {
      cr_root_wave_kernel<M><<<1, 64, 0, e->stream>>>(cr_level(G, nl - 1), G.status.p);
    }
  } else {
    cr_root_kernel<M><<<1, kCrOddThreads<M>, 0, e->stream>>>(cr_level(G, nl - 1), G.status.p);
  }
  if (solved) return;
  if (c == 0) {  // a single super-row: the root's x is the step
    (void)hipMemcpyAsync(G.x.p, L0.x, sizeof(double) * 6 * e->n_frames, hipMemcpyDeviceToDevice, e->stream);
    return;
  }
  CrLevels C{};
  C.nl = nl;
  for (int l = 0; l < nl; ++l) C.lv[l] = cr_level(G, l);
  int lo = c;  // the tail: levels c−1 … lo with at most kCrTailRows super-rows, in one workgroup
  while (lo > 0 && C.lv[lo - 1].n <= kCrTailRows) --lo;
  if (lo <= c - 1) cr_back_tail_kernel<M><<<1, 1024, 0, e->stream>>>(C, c - 1, lo, G.x.p, e->n_frames);
  for (int l = lo - 1; l >= 0; --l) {
    const int lim = l == 0 ? 6 * e->n_frames : C.lv[l].n * M;
    cr_back_kernel<M><<<(lim + 255) / 256, 256, 0, e->stream>>>(C.lv[l], C.lv[l + 1].x, l == 0 ? G.x.p : C.lv[l].x, lim);
  }
}

// Free intrinsics: the arrow solve's buffers (gn_prepare; nf keyframes, nc ≤ kArrowMaxNc cameras).
int configure_arrow(pba_engine* e) {
  GnData& G = e->gn;
  constexpr int M = 24, NB = kArrowNB;
  const int nf = e->n_frames, nc = G.nc_sys, nb = 12 * nc;
  G.ar_n = (nf + 3) / 4;
  G.ar_batches = (1 + nb + NB - 1) / NB;
  // level 0: D, U (shared by the batches) and every batch's b; levels 1, 2 (ping-pong): per batch D, U, b
  const size_t lvl = (size_t)G.ar_n * M * M * 2 + (size_t)G.ar_n * M * NB;
  PBA_HIP(G.ar_buf.resize((size_t)G.ar_n * M * M * 2 + (size_t)G.ar_batches * (2 * lvl + (size_t)G.ar_n * M * NB)));
  PBA_HIP(G.ar_X.resize((size_t)6 * nf * NB * G.ar_batches));
  PBA_HIP(G.ar_part.resize((size_t)kArrowSeg * (nb * (nb + 1) / 2 + nb)));
  PBA_HIP(G.ar_dc.resize((size_t)nb));
  return PBA_OK;
}

// Whether a free-intrinsics system of keyframe bandwidth K is solved as an arrow (arrow_solve): K ≤ 4 (super-rows of 4
// keyframes, M = 24), ≤ kArrowMaxNc cameras, and PBA_SOLVER does not force the skyline solvers ("skyline" / "front":
// the A/B tests of the three solvers).
bool arrow_for(const pba_engine* e, int K) {
  const GnData& G = e->gn;
  if (!G.nc_sys || G.nc_sys > kArrowMaxNc || K > 4 || !G.ar_n) return false;
  const char* fs = getenv("PBA_SOLVER");
  return !(fs && (std::string(fs) == "skyline" || std::string(fs) == "front"));
}

// X = A⁻¹[−g_a | B] by parallel cyclic reduction (batches of kArrowNB columns), the border system, the step into G.x
// (the kernels above).  S, first, row: the skyline system and its profile; fixed: the constant frames.
// Batch 0's rows of arrow level k (configure_arrow's layout) and the arrow kernels' arguments.
CrLevel arrow_level(const GnData& G, int k) {
  constexpr int M = 24, NB = kArrowNB;
  const int n = G.ar_n, nbt = G.ar_batches;
  const size_t lvl = (size_t)n * M * M * 2 + (size_t)n * M * NB, nbq = (size_t)n * M * NB;
  double* p = G.ar_buf.p + (k == 0 ? 0 : (size_t)n * M * M * 2 + nbt * nbq + (size_t)(k - 1) * nbt * lvl);
  return CrLevel{p, p + (size_t)n * M * M, p + (size_t)2 * n * M * M, nullptr, nullptr, n};
}
ArrowArgs arrow_args(pba_engine* e, const double* S, const int* first, const int* row, const uint8_t* fixed) {
  GnData& G = e->gn;
  const int nb = 12 * G.nc_sys;
  return ArrowArgs{S, first, row, G.g.p, fixed, arrow_level(G, 0), G.ar_X.p, G.ar_part.p, G.ar_dc.p, G.x.p, G.status.p,
                   e->n_frames, G.nc_sys, kArrowNB * G.ar_batches, nb * (nb + 1) / 2 + nb};
}
// arrow_build's threads (level 0: D, U and every batch's right-hand sides)
long long arrow_build_threads(const GnData& G) {
  constexpr int M = 24;
  return 2LL * G.ar_n * M * M + (long long)G.ar_batches * G.ar_n * M * kArrowNB;
}

// built: level 0 is already in place (intr_cam_fin_build_kernel of the same trial).
int arrow_solve(pba_engine* e, const double* S, const int* first, const int* row, const uint8_t* fixed,
                bool built = false) {
  GnData& G = e->gn;
  constexpr int M = 24, NB = kArrowNB;
  const int nf = e->n_frames, n = G.ar_n;
  hipStream_t st = e->stream;
  const int nbt = G.ar_batches;
  const size_t lvl = (size_t)n * M * M * 2 + (size_t)n * M * NB, nbq = (size_t)n * M * NB;
  auto level = [&](int k) { return arrow_level(G, k); };
  const ArrowArgs aa = arrow_args(e, S, first, row, fixed);
  constexpr size_t lds = cr_level_wave_lds<M, NB>();
  static_assert(lds <= 65536, "default dynamic LDS limit");
  if (!built) arrow_build_kernel<<<(unsigned)((arrow_build_threads(G) + 255) / 256), 256, 0, st>>>(aa, nbt);
  // the batches' cyclic reductions side by side (gridDim.y): one launch per level whatever the number of cameras
  CrLevel src = level(0);
  if (n <= 1)
    for (int bt = 0; bt < nbt; ++bt) {
      CrLevel sb = src;
      sb.b += bt * nbq;
      pcr_solve_kernel<M, NB><<<n, 64, 0, st>>>(sb, G.ar_X.p + NB * bt, 6 * nf, G.status.p, aa.ldx);
    }
  int pi = 1;
  long long bs_du = 0, bs_b = (long long)nbq;  // level 0: shared D, U
  for (int s = 1; s < n; s *= 2, pi = 3 - pi) {  // the last level also solves the decoupled rows
    const CrLevel dst = level(pi);
    const bool last = 2 * s >= n;
    cr_level_wave_kernel<M, true, NB><<<dim3(n, nbt), 256, lds, st>>>(src, dst, s, G.status.p, last ? G.ar_X.p : nullptr,
                                                                      6 * nf, aa.ldx, bs_du, bs_b, (long long)lvl);
    src = dst;
    bs_du = bs_b = (long long)lvl;
  }
  arrow_reduce_kernel<<<dim3(aa.n_ent, kArrowSeg), 256, 0, st>>>(aa);
  arrow_cap_kernel<<<1, 256, 0, st>>>(aa);
  arrow_back_kernel<<<(6 * nf + 255) / 256, 256, 0, st>>>(aa);
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

// After a solve into G.x: solver status, candidate poses/points, and the two parts of the LM model decrease
// L(0) − L(δ) = −gᵀδ − ½δᵀHδ = ½(λ δᵀDδ − gᵀδ)  (since (H + λD)δ = −g): pose part and point part.
// Candidate poses/points and the model-decrease partials into reduction slots [0, gp + gq) of G.red.
// free_sets: the single-GPU LM loop's per-set point data (the record says which set is current), else G.pt_data.
void enqueue_updates(pba_engine* e, double lambda, const uint8_t* fixed, int* gp_out, int* gq_out,
                     const double* lm = nullptr, bool free_sets = false) {
  GnData& G = e->gn;
  const int nf = e->n_frames, nfs = G.nc_sys ? G.nfs : nf;
  const int gp = (nfs + kBlockThreads - 1) / kBlockThreads;
  const int gq = (G.n_gn_points + kBlockThreads - 1) / kBlockThreads;
  const int gr = (e->n_pairs + kBlockThreads - 1) / kBlockThreads;
  const bool ki = G.nc_sys > 0;
  PoseUpdateArgs pa{e->poses.p, G.x.p, G.g_dir.p, G.Ddiag.p, fixed, G.poses_new.p, G.red.p, G.red2.p, G.gmax.p, nfs, nf,
                    ki ? e->intr_state_d.p : nullptr, ki ? G.intr_new_d.p : nullptr, ki ? G.intr_new_f.p : nullptr};
  // point workgroup q writes reduction slot gp + q, as the separate launches did
  PointUpdateArgs qa{G.pt_data.p, free_sets ? G.pt_data1.p : G.pt_data.p, G.pt_rec.p, G.pt_tgt.p, G.gn_target.p,
                     G.blk_schur.p, G.blk_schur1.p, G.x.p, fixed, e->rho.p, G.rho_new.p, G.drho.p, G.red.p,
                     G.red2.p, G.gmax.p, G.n_gn_points, ki ? G.ib_pw.p : nullptr, G.nc_sys, nf};
  PairUpdateArgs ra{G.pair_rec.p, e->intr_d.p, G.pairs_new.p, e->n_pairs};
  update_kernel<<<gp + gq + gr, kBlockThreads, 0, e->stream>>>(pa, qa, ra, gp, gq, lambda, lm ? lm : G.lm_idle.p);
  G.pairs_new_fresh = true;
  *gp_out = gp;
  *gq_out = gq;
}

void model_from_slots(const GnData& G, double lambda, int gp, int gq, double* model_pose, double* model_points) {
  double dg = 0, dD = 0, qg = 0, qD = 0;
  for (int i = 0; i < gp; ++i) { dg += G.red_h[2 * i]; dD += G.red_h[2 * i + 1]; }
  for (int i = gp; i < gp + gq; ++i) { qg += G.red_h[2 * i]; qD += G.red_h[2 * i + 1]; }
  *model_pose = 0.5 * (lambda * dD - dg);
  *model_points = 0.5 * (lambda * qD - qg);
}

int finish_step(pba_engine* e, double lambda, const uint8_t* fixed, double* model_pose, double* model_points,
                int* solver_status) {
  GnData& G = e->gn;
  int status = 0;
  PBA_HIP(hipMemcpyAsync(&status, G.status.p, sizeof(int), hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  if (solver_status) *solver_status = status;
  *model_pose = *model_points = 0.0;
  if (status != 0) return PBA_OK;
  int gp = 0, gq = 0;
  enqueue_updates(e, lambda, fixed, &gp, &gq);
  PBA_HIP(hipGetLastError());
  PBA_HIP(hipMemcpyAsync(G.red_h.data(), G.red.p, sizeof(double) * 2 * (gp + gq), hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  model_from_slots(G, lambda, gp, gq, model_pose, model_points);
  return PBA_OK;
}

// Band solvers on G.Sband (block cyclic reduction for K ≤ 8, LDS-window band Cholesky for K = 16).
int band_solve(pba_engine* e, bool build = true) {
  GnData& G = e->gn;
  const int nf = e->n_frames;
  if (G.solver == SOLVER_CR) {
    if (G.band_kernel == 4) cr_solve<24>(e, build);
    else cr_solve<48>(e, build);
  } else {
    BandArgs ba{G.Sband.p, G.Lband.p, G.x.p, G.status.p, nf};
    if (G.band_kernel == 4) band_solve_kernel<4><<<1, 256, 0, e->stream>>>(ba);
    else if (G.band_kernel == 8) band_solve_kernel<8><<<1, 256, 0, e->stream>>>(ba);
    else band_solve_kernel<16><<<1, 256, 0, e->stream>>>(ba);
  }
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

// Dynamic LDS above the default 64 KiB limit (the attribute is per device: set on every launch, cheap).
void schur_lds_limit(const GnData& G) {
  if (G.schur_lds > 65536)
    for (const void* f : {reinterpret_cast<const void*>(&schur_kernel), reinterpret_cast<const void*>(&schur_gate_kernel),
                          reinterpret_cast<const void*>(&schur_free_decide_kernel)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G.schur_lds);
}

// Free intrinsics: the last trial's accept (lm: the LM record, else none; accept = false: the point elimination's
// launch has applied it), then the weighted fp64 rows at the state.
void enqueue_intr_rows(pba_engine* e, const double* lm, bool accept = true) {
  GnData& G = e->gn;
  if (lm && accept) intr_accept_kernel<<<1, 256, 0, e->stream>>>(lm, G.intr_new_d.p, G.intr_new_f.p, e->intr_state_d.p,
                                                       e->intr_state.p, G.nc_sys);
  IntrRowsArgs ra{G.ib_rec.p, e->poses.p, e->rho.p, e->u_ref.p, e->u_obs.p, e->frame_cam.p, e->intr_d.p,
                  e->intr_state_d.p, (double)e->opt.huber_width, G.ib_data.p, e->n_blocks, lm ? lm : G.lm_idle.p};
  int grid = (e->n_blocks + 255) / 256;
  if (G.ir_waves > 0) {  // point-aligned waves: the points' W sums too (no intr_pw_kernel)
    ra.wave_tab = G.ir_wave.p;
    ra.n_waves = G.ir_waves;
    ra.pw = G.ib_pw.p;
    ra.nc = G.nc_sys;
    grid = (G.ir_waves + 3) / 4;
  }
  switch (e->opt.camera_model) {
    case PBA_CAMERA_PINHOLE: intr_rows_kernel<CAM_PINHOLE><<<grid, 256, 0, e->stream>>>(ra); break;
    case PBA_CAMERA_DOUBLE_SPHERE: intr_rows_kernel<CAM_DS><<<grid, 256, 0, e->stream>>>(ra); break;
    case PBA_CAMERA_EUCM: intr_rows_kernel<CAM_EUCM><<<grid, 256, 0, e->stream>>>(ra); break;
    default: intr_rows_kernel<CAM_KB4><<<grid, 256, 0, e->stream>>>(ra); break;
  }
}

// The border rows of the reduced system (free intrinsics) into the skyline S — or, X ≠ nullptr, this rank's undamped
// border into the exchange buffer's border region (X points at it).
// arrow: the local solve is an arrow (arrow_solve follows with built = true): its level 0 is built in the same launch as
// the camera blocks.
void enqueue_border(pba_engine* e, double lambda, const double* lm, double* X, bool arrow = false) {
  GnData& G = e->gn;
  const int nf = e->n_frames, nfs = G.nfs;
  IntrBorderArgs ba{G.ib_data.p, G.ib_rec.p, G.ib_cam.p, G.pt_rec.p, G.pt_data.p, G.ib_bptr.p, G.ib_blist.p,
                    G.ib_pptr.p, G.ib_plist.p, G.sky_first.p, G.sky_row.p, G.fixed.p, lm ? lm : G.lm_idle.p, G.S.p,
                    G.g.p, G.g_dir.p, G.Ddiag.p, nf, G.nc_sys, X, (long long)nfs * 36 + EX_TAIL, G.ib_pw.p, G.ib_pblk.p};
  const int nb = 2 * G.nc_sys + 1;
  if (G.ir_waves == 0)  // (else intr_rows_kernel has formed them)
    intr_pw_kernel<<<(8 * G.n_gn_points + 255) / 256, 256, 0, e->stream>>>(ba, G.n_gn_points);
#ifndef PBA_INTR_KPW_BIG
#define PBA_INTR_KPW_BIG 2
#endif
  const int kpw = nf * G.nc_sys < 512 ? 4 : PBA_INTR_KPW_BIG;  // waves per keyframe block (border_keyframes)
  double* dpart = G.ib_part.p;
  double* spart = dpart + (size_t)G.nc_sys * kCamSplit * kCamDir;
  const int nk_x = (nf * kpw + 3) / 4, ncp = G.nc_sys * (G.nc_sys + 1) / 2;
  if (nf * G.nc_sys < 512) {
    const int n_wg = nk_x * G.nc_sys + kCamSplit * (G.nc_sys + ncp);
    intr_border_all_kernel<<<n_wg, 256, 0, e->stream>>>(ba, lambda, kpw, nk_x, dpart, spart);
  } else {
    intr_border_kernel<<<dim3(nk_x, G.nc_sys), 256, 0, e->stream>>>(ba, lambda, kpw);
    intr_cam_dir_kernel<<<dim3(kCamSplit, G.nc_sys), 256, 0, e->stream>>>(ba, dpart);
    intr_cam_sch_kernel<<<dim3(kCamSplit, ncp), 256, 0, e->stream>>>(ba, lambda, spart);
  }
  const int fin_blocks = (2 * G.nc_sys * nb * 36 + 3) / 4;
  if (arrow) {
    const ArrowArgs aa = arrow_args(e, G.S.p, G.sky_first.p, G.sky_row.p, G.fixed.p);
    const int build_blocks = (int)((arrow_build_threads(G) + 255) / 256);
    intr_cam_fin_build_kernel<<<fin_blocks + build_blocks, 256, 0, e->stream>>>(ba, lambda, dpart, spart, aa,
                                                                               G.ar_batches, fin_blocks);
  } else {
    intr_cam_fin_kernel<<<fin_blocks, 256, 0, e->stream>>>(ba, lambda, dpart, spart);
  }
}

// Schur complement for λ, assembly and reduced-system solve into G.x (enqueued only).
// lm: the device LM record (λ, buffer set, done flag read on the device; lambda unused) or nullptr.
// free_sets (the single-GPU LM loop without free intrinsics): the current set's λ-free partials, scaled in the assembly,
// and schur_gate_kernel (the accept, the λ-specific elimination only for a degen set) instead of schur_kernel.
int enqueue_solve(pba_engine* e, double lambda, const double* lm = nullptr, bool free_sets = false) {
  GnData& G = e->gn;
  const int nf = e->n_frames, nfs = G.nc_sys ? G.nfs : nf;
  SchurArgs sa{G.schur_desc.p, G.schur_aux.p, G.schur_pairs.p, G.pt_fb.p, G.blk_lv.p,
               G.blk_schur.p, G.blk_schur1.p, G.part_schur.p, G.pt_data.p, G.n_schur, lm ? lm : G.lm_idle.p,
               lm ? e->poses.p : nullptr, G.poses_new.p, e->rho.p, G.rho_new.p, G.pt_orig.p, 7 * nf, G.n_gn_points,
               G.pair_rt.p, G.pair_rt1.p, G.schur_lvp4.p, G.schur_lvp.p, G.schur_rt_off};
  // free intrinsics: the elimination's launch also applies the previous trial's intrinsics accept (no launch of its own)
  const bool kacc = G.nc_sys && lm && !free_sets && G.n_schur > 0;
  if (kacc) {
    sa.knew_d = G.intr_new_d.p;
    sa.knew_f = G.intr_new_f.p;
    sa.k_d = e->intr_state_d.p;
    sa.k_f = e->intr_state.p;
    sa.n_intr = G.nc_sys;
  }
  schur_lds_limit(G);
  if (free_sets)
    schur_gate_kernel<<<std::max(1, std::min(G.n_schur, 512)), kBlockThreads, G.schur_lds, e->stream>>>(sa, G.degen.p);
  else
    schur_kernel<<<G.n_schur, kBlockThreads, G.schur_lds, e->stream>>>(sa, lambda);
  if (G.nc_sys) enqueue_intr_rows(e, lm, !kacc);
  // block cyclic reduction: assemble writes its level 0 directly (no Sband, no cr_build pass)
  const bool direct = G.band_kernel && G.solver == SOLVER_CR;
  if (direct && G.cr0_dirty)  // a distributed solve rebuilt level 0 over the whole band: back to zeros + padding
    if (int rc = init_cr_level0(e)) return rc;
  CrLevel L0 = direct ? cr_level(G, 0) : CrLevel{};
  AsmArgs aa{G.part_lin.p, G.part_lin1.p, lm ? lm : G.lm_idle.p, G.part_schur.p, G.sky_cptr.p, G.sky_contrib.p, G.g_cptr.p,
             G.g_contrib.p, G.sky_blk_i.p, G.sky_blk_j.p, G.fixed.p, G.S.p, G.g.p, G.g_dir.p, G.Ddiag.p,
             G.band_kernel && !direct ? G.Sband.p : nullptr, G.band_kernel, G.n_sky, nfs,
             direct ? L0.D : nullptr, L0.U, L0.b, G.band_kernel, G.status.p, free_sets ? G.part_free0.p : nullptr,
             free_sets ? G.part_free1.p : nullptr, free_sets ? G.degen.p : nullptr, G.sky_diag.p, G.sky_off.p,
             G.n_sky_diag};
  if (G.sband_dirty && G.band_kernel && !direct) {  // a distributed import filled the whole band: clear the off-profile part
    PBA_HIP(hipMemsetAsync(G.Sband.p, 0, sizeof(double) * (size_t)nf * ((G.band_kernel + 1) * 36 + 6), e->stream));
    G.sband_dirty = false;
  }
  const int nthreads = (G.n_sky + (kAsmSeg - 1) * G.n_sky_diag) * 36 + 6 * nfs * kAsmSeg;
  assemble_kernel<<<(nthreads + 255) / 256, 256, 0, e->stream>>>(aa, lambda);
  // the intrinsics rows of the skyline system (over assemble's zeros); an arrow solve's level 0 in the same launch
  const bool arrow = G.nc_sys && !G.band_kernel && arrow_for(e, G.band);
  if (G.nc_sys) enqueue_border(e, lambda, lm, nullptr, arrow);
  if (G.band_kernel) {
    if (int rc = band_solve(e, !direct)) return rc;
  } else {
    if (arrow) return arrow_solve(e, G.S.p, G.sky_first.p, G.sky_row.p, G.fixed.p, true);
    if (G.front.lds) return launch_front(e, G.front, G.S.p, G.L.p, nfs);
    PBA_HIP(hipMemcpyAsync(G.L.p, G.S.p, sizeof(double) * 36 * (size_t)G.n_sky, hipMemcpyDeviceToDevice, e->stream));
    SolveArgs so{G.L.p, G.sky_first.p, G.sky_row.p, G.sky_last.p, G.g.p, G.Linv.p, G.x.p, G.status.p, nfs,
                 G.sky_colptr.p, G.sky_colrows.p};
    skyline_solve_kernel<<<1, 256, 0, e->stream>>>(so);
  }
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

// Schur complement for λ, assembly, solve and candidate state; returns the LM model decrease.
int gn_step(pba_engine* e, double lambda, double* model_decrease, int* solver_status) {
  if (int rc = enqueue_solve(e, lambda)) return rc;
  double mp = 0.0, mq = 0.0;
  if (int rc = finish_step(e, lambda, e->gn.fixed.p, &mp, &mq, solver_status)) return rc;
  if (model_decrease) *model_decrease = mp + mq;
  return PBA_OK;
}

// state ← candidate (poses, and the inverse distances of the Gauss-Newton points), gated by lm when given
void launch_accept(pba_engine* e, const double* lm) {
  GnData& G = e->gn;
  const int npd = 7 * e->n_frames;
  const int na = std::max(npd, G.n_gn_points);
  lm_accept_kernel<<<std::min(1024, (na + 255) / 256), 256, 0, e->stream>>>(lm, G.poses_new.p, G.rho_new.p, G.pt_orig.p,
                                                                             e->poses.p, e->rho.p, npd, G.n_gn_points);
  if (G.nc_sys)
    intr_accept_kernel<<<1, 256, 0, e->stream>>>(lm, G.intr_new_d.p, G.intr_new_f.p, e->intr_state_d.p, e->intr_state.p,
                                                 G.nc_sys);
  e->pairs_fresh = false;
}

// Wait for trial `seq`'s decision record, published by lm_decide_kernel into host-coherent memory: a poll, not a
// stream event (an event left the GPU idle ~6 µs each) — while the host polls, the GPU runs on into the gated accept
// and linearisation.  The stream is queried now and then so a device error or a record that never comes ends the wait.
double now_ms();
constexpr double kDecisionTimeoutMs = 60000.0;  // one trial takes ~0.25 ms at C4

int wait_decision(pba_engine* e, double seq, double* d) {
  volatile double* r = e->gn.lm_h.p + rec_slot(seq);
  // the stream is queried only after 2 ms without the record (a trial takes ~0.23 ms at C4), then every 2 ms: a
  // hipStreamQuery every few hundred spins idled the GPU 5.7 µs before every trial's first kernel
  // (profiles/r2_gn_trial_trace_v7.txt → v9)
  // A device that stops making progress ends the wait after kDecisionTimeoutMs with PBA_ERR_DEVICE.
  const double t0 = now_ms();
  double next_query = t0 + 2.0;
  for (unsigned spins = 1;; ++spins) {
    if (r[kLmFields] == seq) break;
    if ((spins & 255u) == 0u && now_ms() >= next_query) {
      next_query = now_ms() + 2.0;
      const hipError_t q = hipStreamQuery(e->stream);
      if (q == hipSuccess && r[kLmFields] != seq) return fail(PBA_ERR_DEVICE, "LM decision record was not published");
      if (q != hipSuccess && q != hipErrorNotReady) return fail(PBA_ERR_DEVICE, std::string("HIP: ") + hipGetErrorString(q));
      if (next_query - t0 > kDecisionTimeoutMs)
        return fail(PBA_ERR_DEVICE, "LM decision record not published within " + std::to_string(kDecisionTimeoutMs / 1000) + " s");
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  for (int i = 0; i < kLmFields; ++i) d[i] = r[i];
  return PBA_OK;
}

// One LM trial on a single GPU, enqueued whole and steered by the device LM record G.lm (λ, buffer set, done):
// Schur complement + reduced solve → candidate state (poses, ρ, pair table) and model-decrease partials →
// linearisation AT the candidate into the spare buffer set, whose per-chunk cost partials are the candidate cost →
// the decision on the device (accept, the next trust radius, done; published to the host); the accept itself is applied
// by the next trial's first kernel.  An accepted
// step's linearisation is then already done (a rejected one cost a linearisation instead of a residual-only pass), and
// since every kernel returns at once when the solve is done, the host enqueues the next trial before it has seen this
// one's decision: no host round trip between trials.  The candidate is evaluated even when the solve failed (its
// numbers are then discarded): a garbage state is memory-safe in every evaluation kernel.  ev (phase timing only,
// else nullptr): begin | candidate state | candidate linearisation | decision.
// The λ-free point elimination's launch after a linearisation (schur_free_decide_kernel): workgroup 0 the decision of
// trial seq (init: the record of a new solve), the others the set's partials.
void launch_free_decide(pba_engine* e, const DecideOpts& dopt, double seq, int gp, int gq, bool init, double radius) {
  GnData& G = e->gn;
  const int nf = e->n_frames;
  SchurArgs sa{G.schur_desc.p, G.schur_aux.p, G.schur_pairs.p, G.pt_fb.p, G.blk_lv.p,
               G.blk_schur.p, G.blk_schur1.p, G.part_schur.p, G.pt_data.p, G.n_schur, G.lm.p,
               nullptr, nullptr, nullptr, nullptr, nullptr, 7 * nf, G.n_gn_points,
               G.pair_rt.p, G.pair_rt1.p, G.schur_lvp4.p, G.schur_lvp.p, G.schur_rt_off};
  DecideArgs da{G.red.p, G.red2.p, G.gmax.p, gp, gq, G.n_chunks, G.status.p, dopt, G.lm.p,
                init ? nullptr : G.lm_host_d + rec_slot(seq), seq, init ? 1 : 0, radius, G.lm_init.p,
                G.ts_part.p, G.ts_count.p};
  FreeSets fs{{G.part_free0.p, G.part_free1.p}, {G.pt_data.p, G.pt_data1.p}, G.degen.p, G.lin_set.p};
  schur_lds_limit(G);
  schur_free_decide_kernel<<<kDecideWgs + G.n_schur, kBlockThreads, G.schur_lds, e->stream>>>(sa, da, fs);
  // tests: every set flagged, so every trial takes the λ-specific elimination (the degenerate-point path)
  if (G.force_degen) (void)hipMemsetAsync(G.degen.p, 0x01, 2 * sizeof(int), e->stream);
}

// free intrinsics keep the per-trial elimination (their border kernels read its point data at the trial's λ)
bool lm_free_sets(const pba_engine* e) { return e->gn.nc_sys == 0 && e->gn.n_schur > 0; }

int lm_trial(pba_engine* e, const DecideOpts& dopt, double seq, const hipEvent_t* ev) {
  GnData& G = e->gn;
  const bool fs = lm_free_sets(e);
  if (ev) PBA_HIP(hipEventRecord(ev[0], e->stream));
  if (int rc = enqueue_solve(e, 0.0, G.lm.p, fs)) return rc;
  int gp = 0, gq = 0;
  enqueue_updates(e, 0.0, G.fixed.p, &gp, &gq, G.lm.p, fs);
  if (ev) PBA_HIP(hipEventRecord(ev[1], e->stream));
  if (int rc = linearize(e, nullptr, G.lm.p, G.pairs_new.p, G.rho_new.p, G.red.p + 2 * (gp + gq), nullptr, true, fs))
    return rc;
  if (ev) PBA_HIP(hipEventRecord(ev[2], e->stream));
  if (fs)
    launch_free_decide(e, dopt, seq, gp, gq, false, 0.0);
  else
    lm_decide_kernel<<<1, kDecideThreads, 0, e->stream>>>(G.red.p, G.red2.p, G.gmax.p, gp, gq, G.n_chunks, G.status.p,
                                                          dopt, G.lm.p, G.lm_host_d + rec_slot(seq), seq);
  PBA_HIP(hipGetLastError());
  if (ev) PBA_HIP(hipEventRecord(ev[3], e->stream));
  return PBA_OK;  // an accepted candidate becomes the state in the next trial's first kernel (or after the loop)
}

int candidate_cost(pba_engine* e, double* cost) {
  GnData& G = e->gn;
  if (e->opt.residual_kind == PBA_RESIDUAL_PHOTOMETRIC) {
    // the candidate poses straight into the fused-state prologue: no pair-table launch (C4: 32.4 → 29.8 µs for the
    // cost launch, and the 7.6-µs pair launch gone)
    if (int rc = launch_cost_only(e, G.pairs_new.p, G.rho_new.p, nullptr, nullptr, G.poses_new.p)) return rc;
    return total_cost(e, cost, nullptr);
  }
  if (!G.pairs_new_fresh) launch_pairs(e, G.poses_new.p, G.pairs_new.p);
  if (int rc = launch_cost_only(e, G.pairs_new.p, G.rho_new.p, nullptr, nullptr, nullptr,
                                G.nc_sys ? G.intr_new_f.p : nullptr, G.nc_sys ? G.intr_new_d.p : nullptr))
    return rc;
  return total_cost(e, cost, nullptr);
}

int accept(pba_engine* e) {
  launch_accept(e, nullptr);
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

// ---- multi-GPU step (include/pba.h) ------------------------------------------------------------
int exchange_K(pba_engine* e, int band, int* K) {
  *K = band_kernel_for(std::max(band, e->gn.band));
  if (band < e->gn.band) return fail(PBA_ERR_INVALID_ARGUMENT, "band below this rank's reduced-system bandwidth");
  if (*K == 0) return fail(PBA_ERR_INVALID_ARGUMENT, "distributed solve needs a reduced-system bandwidth <= 16");
  return PBA_OK;
}

// The exchange buffer: the keyframes' band rows (nf × ex_row(K)), with free intrinsics the 2·nc border rows
// (nfs·36 + EX_TAIL each), then the kExScalars scalar slots of the device-steered loop.
long long ex_border(const pba_engine* e) {
  const GnData& G = e->gn;
  return G.nc_sys ? 2LL * G.nc_sys * ((long long)G.nfs * 36 + EX_TAIL) : 0;
}
long long ex_scalar_off(const pba_engine* e, int K) { return (long long)e->n_frames * ex_row(K) + ex_border(e); }
long long exchange_count(pba_engine* e, int K) { return ex_scalar_off(e, K) + kExScalars; }

// The summed profile of a multi-GPU free-intrinsics solve (band K over the keyframes, border rows from frame 0): its
// skyline layout and front_solve_kernel plan, built once per K.
int ensure_dist_sky(pba_engine* e, int K) {
  GnData& G = e->gn;
  if (G.dsky_K == K) return PBA_OK;
  const int nf = e->n_frames, nfs = G.nfs;
  std::vector<int> first(nfs), rowp(nfs + 1, 0), ccptr, ccrows;
  for (int i = 0; i < nfs; ++i) first[i] = i < nf ? std::max(0, i - K) : 0;
  for (int i = 0; i < nfs; ++i) rowp[i + 1] = rowp[i] + (i - first[i] + 1);
  profile_columns(first, ccptr, ccrows);
  if (int rc = build_front_plan(first, rowp, ccptr, ccrows, e->stream, G.dfront, true)) return rc;
  // (a front beyond LDS — many cameras or a wide band — is solved through global memory, skyline_solve_kernel)
  std::vector<int> last(nfs);
  for (int k = 0; k < nfs; ++k) last[k] = k;
  for (int i = 0; i < nfs; ++i)
    for (int k = first[i]; k < i; ++k) last[k] = std::max(last[k], i);
  G.n_dsky = rowp[nfs];
  PBA_HIP(G.dS.resize((size_t)G.n_dsky * 36));
  PBA_HIP(G.dL.resize((size_t)G.n_dsky * 36));
  PBA_HIP(G.dsky_row.upload(rowp, e->stream));
  PBA_HIP(G.dsky_first.upload(first, e->stream));
  PBA_HIP(G.dsky_last.upload(last, e->stream));
  PBA_HIP(G.dsky_colptr.upload(ccptr, e->stream));
  PBA_HIP(G.dsky_colrows.upload(ccrows.empty() ? std::vector<int>{0} : ccrows, e->stream));
  G.dsky_K = K;
  return PBA_OK;
}

// This rank's partial system into the exchange buffer X (every element written: no fill launch); with free
// intrinsics also the border rows (after this trial's accept and point elimination: the rows at the state, the Schur
// terms at λ — the LM record's, or `lambda` for a host-driven step).
int enqueue_export(pba_engine* e, double lambda, const double* lm, double* X, int K) {
  GnData& G = e->gn;
  const int nf = e->n_frames;
  AsmArgs aa{G.part_lin.p, G.part_lin1.p, lm, G.part_schur.p, G.sky_cptr.p, G.sky_contrib.p, G.g_cptr.p,
             G.g_contrib.p, G.sky_blk_i.p, G.sky_blk_j.p, G.fixed.p, G.S.p, G.g.p, G.g_dir.p, G.Ddiag.p, nullptr, K,
             G.n_sky, nf, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr};
  const long long n = (long long)nf * ex_row(K);  // (K+1)·36 band + EX_TAIL tail lanes per frame
  export_band_kernel<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(aa, G.observed.p, G.sky_first.p, G.sky_row.p,
                                                                        X, K);
  if (G.nc_sys) {
    enqueue_intr_rows(e, lm == G.lm_idle.p ? nullptr : lm);
    enqueue_border(e, lambda, lm, X + n);
  }
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

// The summed exchange → damping, constant frames and the band solver's input — for block cyclic reduction its level 0
// directly (no Sband, no cr_build pass), as assemble_kernel does on one GPU — then the reduced solve into G.x.
int enqueue_import(pba_engine* e, double lambda, const double* lm, const double* X, int K) {
  GnData& G = e->gn;
  const int nf = e->n_frames;
  if (G.nc_sys) {  // free intrinsics: the summed skyline system (band + border) — an arrow, or the skyline solvers
    if (int rc = ensure_dist_sky(e, K)) return rc;
    const int nfs = G.nfs;
    ImportSkyArgs ia{X, X + (long long)nf * ex_row(K), G.fixed_req.p, G.dsky_row.p, G.dS.p, G.g.p, G.g_dir.p,
                     G.Ddiag.p, G.fixed_dist.p, nf, G.nc_sys, K, (long long)G.n_dsky * 36};
    const long long n = ia.n_el + 6LL * nfs;
    import_sky_kernel<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(ia, lambda, lm);
    PBA_HIP(hipGetLastError());
    if (arrow_for(e, K)) return arrow_solve(e, G.dS.p, G.dsky_first.p, G.dsky_row.p, G.fixed_dist.p);
    if (G.dfront.lds) return launch_front(e, G.dfront, G.dS.p, G.dL.p, nfs);
    PBA_HIP(hipMemcpyAsync(G.dL.p, G.dS.p, sizeof(double) * 36 * (size_t)G.n_dsky, hipMemcpyDeviceToDevice, e->stream));
    SolveArgs so{G.dL.p, G.dsky_first.p, G.dsky_row.p, G.dsky_last.p, G.g.p, G.Linv.p, G.x.p, G.status.p, nfs,
                 G.dsky_colptr.p, G.dsky_colrows.p};
    skyline_solve_kernel<<<1, 256, 0, e->stream>>>(so);
    PBA_HIP(hipGetLastError());
    return PBA_OK;
  }
  const bool direct = G.solver == SOLVER_CR;
  if (direct && !G.cr0_inited)  // zeros outside the band, identity padding rows
    if (int rc = init_cr_level0(e)) return rc;
  CrLevel L0 = direct ? cr_level(G, 0) : CrLevel{};
  ImportArgs ia{X, G.fixed_req.p, G.Sband.p, G.g.p, G.g_dir.p, G.Ddiag.p, G.fixed_dist.p, nf, K,
                direct ? L0.D : nullptr, L0.U, L0.b, G.status.p};
  const long long n = (long long)nf * ((K + 1) * 36 + 6);
  import_kernel<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(ia, lambda, lm);
  PBA_HIP(hipGetLastError());
  G.sband_dirty = !direct;
  G.cr0_dirty = true;  // level 0 holds the whole band now: a single-GPU assembly re-initialises it first
  return band_solve(e, !direct);
}

int step_export(pba_engine* e, double lambda, int band, double* X) {
  GnData& G = e->gn;
  int K;
  if (int rc = exchange_K(e, band, &K)) return rc;
  const int nf = e->n_frames;
  SchurArgs sa{G.schur_desc.p, G.schur_aux.p, G.schur_pairs.p, G.pt_fb.p, G.blk_lv.p,
               G.blk_schur.p, G.blk_schur1.p, G.part_schur.p, G.pt_data.p, G.n_schur, G.lm_idle.p,
               nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0,
               G.pair_rt.p, G.pair_rt1.p, G.schur_lvp4.p, G.schur_lvp.p, G.schur_rt_off};
  schur_lds_limit(G);
  if (G.n_schur > 0) schur_kernel<<<G.n_schur, kBlockThreads, G.schur_lds, e->stream>>>(sa, lambda);
  (void)nf;
  return enqueue_export(e, lambda, G.lm_idle.p, X, K);
}

int step_import(pba_engine* e, double lambda, int band, const double* X, double* model_pose, double* model_points,
                int* solver_status) {
  GnData& G = e->gn;
  int K;
  if (int rc = exchange_K(e, band, &K)) return rc;
  if (!G.nc_sys && (G.band_kernel != K || G.solver == SOLVER_SKYLINE)) {
    const char* fs = getenv("PBA_SOLVER");
    const int solver = (K <= 8 && !(fs && std::string(fs) == "band")) ? SOLVER_CR : SOLVER_BAND;
    if (int rc = configure_solver(e, K, solver)) return rc;
  }
  if (int rc = enqueue_import(e, lambda, G.lm_idle.p, X, K)) return rc;
  return finish_step(e, lambda, G.fixed_dist.p, model_pose, model_points, solver_status);
}


double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" {

int pba_set_fixed_frames(pba_engine* e, int32_t n, const int32_t* frames) {
  if (!e || n < 0 || (n > 0 && !frames)) return fail(PBA_ERR_INVALID_ARGUMENT, "bad fixed-frame arguments");
  if (e->n_frames <= 0) return fail(PBA_ERR_NOT_READY, "pba_set_frames first");
  std::vector<uint8_t> f(e->n_frames, 0);
  for (int i = 0; i < n; ++i) {
    if (frames[i] < 0 || frames[i] >= e->n_frames) return fail(PBA_ERR_INVALID_ARGUMENT, "fixed frame out of range");
    f[frames[i]] = 1;
  }
  e->gn.fixed_h = f;
  e->gn.prepared = false;
  return PBA_OK;
}

int pba_gn_linearize(pba_engine* e, double* cost) {
  if (int rc = ensure_prepared(e)) return rc;
  return linearize(e, cost);
}

int pba_gn_step(pba_engine* e, double lambda, double* model_decrease, int32_t* solver_status) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!(lambda >= 0.0)) return fail(PBA_ERR_INVALID_ARGUMENT, "lambda must be >= 0");
  int st = 0;
  const int rc = gn_step(e, lambda, model_decrease, &st);
  if (solver_status) *solver_status = st;
  return rc;
}

int pba_gn_candidate_cost(pba_engine* e, double* cost) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!cost) return fail(PBA_ERR_INVALID_ARGUMENT, "null cost");
  return candidate_cost(e, cost);
}

int pba_gn_accept(pba_engine* e) {
  if (int rc = ensure_prepared(e)) return rc;
  return accept(e);
}

int pba_get_state(pba_engine* e, double* poses, double* inv_dist) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  if (!e->state_set) return fail(PBA_ERR_NOT_READY, "pba_set_state first");
  if (int rc = check_device(e)) return rc;
  if (poses) PBA_HIP(hipMemcpyAsync(poses, e->poses.p, sizeof(double) * 7 * e->n_frames, hipMemcpyDeviceToHost, e->stream));
  if (inv_dist) PBA_HIP(hipMemcpyAsync(inv_dist, e->rho.p, sizeof(double) * e->n_points, hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

int pba_gn_get_reduced_system(pba_engine* e, double* S_dense, double* g) {
  if (int rc = ensure_prepared(e)) return rc;
  GnData& G = e->gn;
  const int nf = G.nc_sys ? G.nfs : e->n_frames;  // system frames (pba_gn_system_size)
  std::vector<int> first(nf), row(nf + 1);
  PBA_HIP(hipMemcpy(first.data(), G.sky_first.p, sizeof(int) * nf, hipMemcpyDeviceToHost));
  PBA_HIP(hipMemcpy(row.data(), G.sky_row.p, sizeof(int) * (nf + 1), hipMemcpyDeviceToHost));
  if (S_dense) {
    std::vector<double> sky((size_t)G.n_sky * 36);
    PBA_HIP(hipMemcpy(sky.data(), G.S.p, sizeof(double) * sky.size(), hipMemcpyDeviceToHost));
    const size_t n = 6 * (size_t)nf;
    std::fill(S_dense, S_dense + n * n, 0.0);
    for (int i = 0; i < nf; ++i)
      for (int j = first[i]; j <= i; ++j) {
        const double* B = &sky[((size_t)row[i] + (j - first[i])) * 36];
        for (int r = 0; r < 6; ++r)
          for (int c = 0; c < 6; ++c) {
            S_dense[(6 * i + r) * n + 6 * j + c] = B[r * 6 + c];
            S_dense[(6 * j + c) * n + 6 * i + r] = B[r * 6 + c];
          }
      }
  }
  if (g) PBA_HIP(hipMemcpy(g, G.g.p, sizeof(double) * 6 * nf, hipMemcpyDeviceToHost));
  return PBA_OK;
}

int pba_gn_get_step(pba_engine* e, double* dposes, double* drho) {
  if (int rc = ensure_prepared(e)) return rc;
  GnData& G = e->gn;
  if (dposes) PBA_HIP(hipMemcpy(dposes, G.x.p, sizeof(double) * 6 * e->n_frames, hipMemcpyDeviceToHost));
  if (drho) PBA_HIP(hipMemcpy(drho, G.drho.p, sizeof(double) * e->n_points, hipMemcpyDeviceToHost));
  return PBA_OK;
}

int pba_gn_set_rank(pba_engine* e, int32_t rank) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  e->gn.dist_rank = rank < 0 ? -1 : rank;
  return PBA_OK;
}

int pba_gn_system_size(pba_engine* e, int32_t* n) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!n) return fail(PBA_ERR_INVALID_ARGUMENT, "null size");
  *n = 6 * (e->gn.nc_sys ? e->gn.nfs : e->n_frames);
  return PBA_OK;
}

int pba_gn_band(pba_engine* e, int32_t* band) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!band) return fail(PBA_ERR_INVALID_ARGUMENT, "null band");
  *band = e->gn.band;
  return PBA_OK;
}

int pba_gn_exchange_size(pba_engine* e, int32_t band, int64_t* count) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!count) return fail(PBA_ERR_INVALID_ARGUMENT, "null count");
  int K;
  if (int rc = exchange_K(e, band, &K)) return rc;
  *count = exchange_count(e, K);
  return PBA_OK;
}

int pba_gn_step_export(pba_engine* e, double lambda, int32_t band, double* d_exchange) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!d_exchange) return fail(PBA_ERR_INVALID_ARGUMENT, "null exchange buffer");
  if (!(lambda >= 0.0)) return fail(PBA_ERR_INVALID_ARGUMENT, "lambda must be >= 0");
  if (int rc = step_export(e, lambda, band, d_exchange)) return rc;
  PBA_HIP(hipStreamSynchronize(e->stream));
  return PBA_OK;
}

int pba_gn_step_import(pba_engine* e, double lambda, int32_t band, const double* d_exchange, double* model_pose,
                       double* model_points, int32_t* solver_status) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!d_exchange) return fail(PBA_ERR_INVALID_ARGUMENT, "null exchange buffer");
  if (!(lambda >= 0.0)) return fail(PBA_ERR_INVALID_ARGUMENT, "lambda must be >= 0");
  double mp = 0.0, mq = 0.0;
  int st = 0;
  if (int rc = step_import(e, lambda, band, d_exchange, &mp, &mq, &st)) return rc;
  if (model_pose) *model_pose = mp;
  if (model_points) *model_points = mq;
  if (solver_status) *solver_status = st;
  return PBA_OK;
}

}  // extern "C"

namespace {

// The collective of the multi-GPU loop: stream-ordered (a pba_comm: RCCL or an in-process group) or a host callback
// that is called once the engine's stream has drained and is complete when it returns.
struct Collective {
  pba_allreduce_fn fn = nullptr;
  void* user = nullptr;
  pba_comm* comm = nullptr;
  int allreduce(pba_engine* e, double* buf, long long n) const {
    if (comm) return comm_allreduce(comm, buf, n, e->stream);
    PBA_HIP(hipStreamSynchronize(e->stream));
    if (int rc = fn(user, buf, n)) return fail(PBA_ERR_DEVICE, "allreduce callback failed (" + std::to_string(rc) + ")");
    return PBA_OK;
  }
  // dist_sums_kernel's rank flag: 1 rank 0, 0 another rank, −1 unknown (a host callback without pba_gn_set_rank)
  int rank0(const pba_engine* e) const {
    const int r = comm ? comm_rank(comm) : e->gn.dist_rank;
    return r < 0 ? -1 : (r == 0 ? 1 : 0);
  }
};

// Levenberg-Marquardt (trust_region_minimizer.cc + levenberg_marquardt_strategy.cc semantics):
// μ = 1/radius, step accepted when (cost − cost_new)/model_decrease > min_relative_decrease (1e-3);
// success: radius /= max(1/3, 1 − (2ρ − 1)³), decrease factor 2; failure: radius /= factor, factor *= 2.
// With a Reducer every cost, model decrease and the reduced system are sums over ranks, so all ranks take
// the same decisions and the same pose steps.
pba_solver_options lm_options(const pba_solver_options* o) {
  pba_solver_options opt{};  // Ceres' defaults (solver.h:278-322), max_num_iterations as map_utils.h:318
  opt.max_iterations = 20;
  opt.max_num_consecutive_invalid_steps = 5;
  opt.initial_trust_region_radius = 1e4;
  opt.function_tolerance = 1e-6;
  opt.parameter_tolerance = 1e-8;
  opt.min_relative_decrease = 1e-3;
  opt.gradient_tolerance = 1e-10;
  opt.max_trust_region_radius = 1e16;
  opt.min_trust_region_radius = 1e-32;
  if (o) opt = *o;
  if (opt.max_num_consecutive_invalid_steps <= 0) opt.max_num_consecutive_invalid_steps = 5;
  return opt;
}

DecideOpts decide_opts(const pba_solver_options& o) {
  return DecideOpts{o.min_relative_decrease, o.function_tolerance, o.parameter_tolerance, o.gradient_tolerance,
                    o.max_trust_region_radius, o.min_trust_region_radius, o.max_num_consecutive_invalid_steps};
}

// The summary's outcome from a published decision record (done != 0).  Returns whether the trial counts as an
// iteration (Ceres pushes no IterationSummary for a gradient-tolerance stop, which happens before the step, nor for the
// consecutive-invalid-steps failure).
bool finish_summary(double done, pba_solver_summary& s) {
  switch ((int)done) {
    case kDoneFunction: s.termination = PBA_TERMINATION_CONVERGENCE; s.stop_reason = PBA_STOP_FUNCTION_TOLERANCE; return true;
    case kDoneParameter: s.termination = PBA_TERMINATION_CONVERGENCE; s.stop_reason = PBA_STOP_PARAMETER_TOLERANCE; return true;
    case kDoneGradient: s.termination = PBA_TERMINATION_CONVERGENCE; s.stop_reason = PBA_STOP_GRADIENT_TOLERANCE; return false;
    case kDoneRadius: s.termination = PBA_TERMINATION_CONVERGENCE; s.stop_reason = PBA_STOP_MIN_TRUST_REGION_RADIUS; return true;
    default: s.termination = PBA_TERMINATION_FAILURE; s.stop_reason = PBA_STOP_INVALID_STEPS; return false;
  }
}

// The trajectory of a solve, as Ceres' Solver::Summary::iterations (pba.h, pba_iteration_summary): entry 0 the initial
// state, then one entry per trial Ceres pushes.  Filled from the published decision records as the host reads them; the
// costs and cost changes are completed by finish() once the initial cost is known (pba_solve reads it after the loop).
struct Trajectory {
  std::vector<pba_iteration_summary>& it;
  explicit Trajectory(std::vector<pba_iteration_summary>& v, double radius) : it(v) {
    it.clear();
    pba_iteration_summary z{};
    z.step_is_successful = z.step_is_valid = 1;
    z.trust_region_radius = radius;
    z.gradient_max_norm = NAN;
    it.push_back(z);
  }
  // trial record d (kLm* fields): its gradient is the one at the state the trial started from, i.e. the state the last
  // entry ended in, if that entry has none yet (the initial state, an accepted step)
  void trial(const double* d) {
    if (std::isnan(it.back().gradient_max_norm)) it.back().gradient_max_norm = d[kLmGradNorm];
    const double done = d[kLmDone];
    if (done != 0.0 && done != kDoneRadius) return;  // a tolerance or the invalid-step limit: Minimize returns first
    pba_iteration_summary x{};
    x.iteration = (int)it.size();
    x.step_is_valid = d[kLmStatus] == 0.0 && d[kLmModel] > 0.0;
    x.step_is_successful = d[kLmAccept] != 0.0;
    x.cost = d[kLmCostNew];  // (the candidate's; finish() puts the current cost on invalid steps)
    x.relative_decrease = x.step_is_valid ? d[kLmRel] : 0.0;
    x.trust_region_radius = d[kLmRadius];
    x.step_norm = x.step_is_valid ? d[kLmStepNorm] : 0.0;
    x.gradient_max_norm = x.step_is_successful ? NAN : it.back().gradient_max_norm;
    it.push_back(x);
  }
  void finish(double initial_cost) {
    double cur = initial_cost;
    it[0].cost = initial_cost;
    for (size_t k = 1; k < it.size(); ++k) {
      pba_iteration_summary& x = it[k];
      if (!x.step_is_valid) {
        x.cost = cur;
        x.cost_change = 0.0;
        continue;
      }
      x.cost_change = cur - x.cost;
      if (x.step_is_successful) cur = x.cost;
    }
  }
};

// Single GPU: every trial is enqueued whole (lm_trial) and the accept/reject decision is taken on the device, so
// the host only reads the decision record back; the breakdown is device time between stream events.
int lm_loop_single(pba_engine* e, const pba_solver_options* o, pba_solver_summary* sum) {
  GnData& G = e->gn;
  const pba_solver_options opt = lm_options(o);
  pba_solver_summary s{};
  struct Events {  // phase timing (pba_set_solver_timing): two sets of 4 (a trial is enqueued ahead)
    hipEvent_t ev[8] = {};
    ~Events() {
      for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    }
  } events;
  const bool timed = G.phase_timing;
  if (timed)
    for (int i = 0; i < 8; ++i) PBA_HIP(hipEventCreate(&events.ev[i]));
  const double t0 = now_ms();
  double cost = 0.0;
  // the initial linearisation (set 0) with its chunk cost partials in red, and the device record formed from them
  // (lm_init_kernel): no host round trip before the first trial
  const bool fs = lm_free_sets(e);
  if (int rc = linearize(e, nullptr, nullptr, nullptr, nullptr, G.red.p, nullptr, false, fs)) return rc;
  if (G.lm_init.n < 2) PBA_HIP(G.lm_init.resize(2));
  if (fs)  // the record and set 0's λ-free partials in one launch
    launch_free_decide(e, decide_opts(opt), 0.0, 0, 0, true, opt.initial_trust_region_radius);
  else
    lm_init_kernel<<<1, kDecideThreads, 0, e->stream>>>(G.red.p, G.n_chunks, opt.initial_trust_region_radius, G.lm.p,
                                                         G.lm_init.p);
  PBA_HIP(hipGetLastError());
  for (int r = 0; r < kRecRing; ++r) G.lm_h[r * kRecStride + kLmFields] = 0.0;  // no trial published yet
  // PBA_LM_HOST_DELAY_US (test build only, PBA_TEST_HOOKS): the host thread sleeps this long before each wait, as a
  // descheduled thread would
  const int delay_us = test_hook_int("PBA_LM_HOST_DELAY_US");
  const int n = std::max(0, opt.max_iterations);
  const DecideOpts dopt = decide_opts(opt);
  auto enqueue = [&](int i) { return lm_trial(e, dopt, (double)(i + 1), timed ? events.ev + 4 * (i & 1) : nullptr); };
  Trajectory traj(G.history, opt.initial_trust_region_radius);
  if (n > 0)
    if (int rc = enqueue(0)) return rc;
  int iter = 0, set = 0;
  s.termination = PBA_TERMINATION_MAX_ITERATIONS;
  s.stop_reason = PBA_STOP_MAX_ITERATIONS;
  for (; iter < n; ++iter) {
    if (iter + 1 < n)
      if (int rc = enqueue(iter + 1)) return rc;  // ahead of this trial's decision
    if (delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
    double d[kLmFields];
    if (int rc = wait_decision(e, (double)(iter + 1), d)) return rc;
    set = (int)d[kLmSet];
    traj.trial(d);
    if (timed) {
      const hipEvent_t* ev = events.ev + 4 * (iter & 1);
      float ms = 0.0f;
      PBA_HIP(hipEventSynchronize(ev[3]));
      PBA_HIP(hipEventElapsedTime(&ms, ev[0], ev[1]));
      s.solve_ms += ms;
      PBA_HIP(hipEventElapsedTime(&ms, ev[1], ev[2]));
      s.linearize_ms += ms;
      PBA_HIP(hipEventElapsedTime(&ms, ev[2], ev[3]));
      s.cost_ms += ms;
    }
    s.gradient_max_norm = d[kLmGradNorm];
    const double done = d[kLmDone];
    if (done != 0.0 && done != kDoneRadius) {  // a tolerance (the step is not applied) or the invalid-step limit
      if (finish_summary(done, s)) ++iter;
      break;
    }
    if (d[kLmAccept] == 0.0) {  // invalid step (failed solve, no predicted decrease) or too little actual decrease
      ++s.unsuccessful_steps;
      if (done != 0.0) {  // the trust region collapsed
        finish_summary(done, s);
        ++iter;
        break;
      }
      continue;
    }
    ++s.successful_steps;
    cost = d[kLmCostNew];
  }
  launch_accept(e, G.lm.p);  // the last trial's accept (no trial after it to apply it)
  double init[2] = {0.0, 0.0};
  PBA_HIP(hipMemcpyAsync(init, G.lm_init.p, sizeof init, hipMemcpyDeviceToHost, e->stream));
  PBA_HIP(hipStreamSynchronize(e->stream));
  s.initial_cost = init[0];
  traj.finish(init[0]);
  if (s.successful_steps == 0) cost = init[0];
  if (set == 1) {  // the current state's pieces are in set 1: make it set 0 for the host-driven entry points
    std::swap(G.blk_schur.p, G.blk_schur1.p);
    std::swap(G.blk_schur.n, G.blk_schur1.n);
    std::swap(G.pair_rt.p, G.pair_rt1.p);
    std::swap(G.pair_rt.n, G.pair_rt1.n);
    std::swap(G.part_lin.p, G.part_lin1.p);
    std::swap(G.part_lin.n, G.part_lin1.n);
  }
  s.iterations = iter;
  s.final_cost = cost;
  s.total_ms = now_ms() - t0;
  if (sum) *sum = s;
  return PBA_OK;
}

// One multi-GPU LM trial, enqueued whole on the engine stream and steered by the device LM record like lm_trial:
// point elimination for the record's λ (the previous trial's accept applied first) → this rank's banded partial system
// into X → Σ over ranks → damping, constant frames (requested, or observed by no rank), solve → candidate state and the
// update partials → candidate linearisation into the spare buffer set (its chunk partials are this rank's candidate
// cost) → this rank's trial sums, the point part Σ over ranks (kExScalars doubles) → the decision, the same on every
// rank, published to the host.  Two collectives per trial: λ of trial i + 1 depends on the decision of trial i, and the
// point elimination (hence this rank's system) on λ.  With a stream-ordered collective the host enqueues the next trial
// before this one's decision is known, as on one GPU; every rank enqueues the same trials (the decisions agree), so the
// collectives match.
// PBA_TEST_PERTURB_DECISION = "rank:trial:mode" (tests): that rank's decision of that trial is overridden (mode 1: the
// accept flag flipped, 2: the solve ended) — the ranks' records then differ, which the next trial's check must catch.
struct DistCheck {
  int n_ranks = 1;
  double perturb_seq = -1.0;
  int perturb_mode = 0;
};

int dist_trial(pba_engine* e, const Collective& coll, const DecideOpts& dopt, double* X, int K, double seq,
               const DistCheck& chk) {
  GnData& G = e->gn;
  const int nf = e->n_frames;
  SchurArgs sa{G.schur_desc.p, G.schur_aux.p, G.schur_pairs.p, G.pt_fb.p, G.blk_lv.p,
               G.blk_schur.p, G.blk_schur1.p, G.part_schur.p, G.pt_data.p, G.n_schur, G.lm.p,
               e->poses.p, G.poses_new.p, e->rho.p, G.rho_new.p, G.pt_orig.p, 7 * nf, G.n_gn_points,
               G.pair_rt.p, G.pair_rt1.p, G.schur_lvp4.p, G.schur_lvp.p, G.schur_rt_off};
  schur_lds_limit(G);
  if (G.n_schur > 0) schur_kernel<<<G.n_schur, kBlockThreads, G.schur_lds, e->stream>>>(sa, 0.0);
  else launch_accept(e, G.lm.p);  // no points on this rank: the accept alone
  const long long nx = ex_scalar_off(e, K);  // the band rows and, with free intrinsics, the border rows
  if (int rc = enqueue_export(e, 0.0, G.lm.p, X, K)) return rc;
  if (int rc = coll.allreduce(e, X, nx)) return rc;
  if (int rc = enqueue_import(e, 0.0, G.lm.p, X, K)) return rc;
  int gp = 0, gq = 0;
  enqueue_updates(e, 0.0, G.fixed_dist.p, &gp, &gq, G.lm.p);
  if (G.n_chunks > 0)
    if (int rc = linearize(e, nullptr, G.lm.p, G.pairs_new.p, G.rho_new.p, G.red.p + 2 * (gp + gq), nullptr, true))
      return rc;  // (at the candidate intrinsics too)
  double* Y = X + nx;
  dist_sums_kernel<<<1, kDecideThreads, 0, e->stream>>>(G.red.p, G.red2.p, G.gmax.p, gp, gq, G.n_chunks, dopt.gtol,
                                                         G.lm.p, G.status.p, coll.rank0(e), G.tpose.p, Y);
  PBA_HIP(hipGetLastError());
  if (int rc = coll.allreduce(e, Y, kExScalars)) return rc;
  dist_decide_kernel<<<1, 64, 0, e->stream>>>(Y, G.tpose.p, coll.rank0(e) < 0 ? 1 : 0, dopt, G.lm.p,
                                              G.lm_host_d + rec_slot(seq), seq, chk.n_ranks, chk.perturb_seq,
                                              chk.perturb_mode, 0);
  PBA_HIP(hipGetLastError());
  return PBA_OK;
}

// The LM loop over one GPU (coll == nullptr) or all ranks: the host enqueues trial i + 1, then waits for the published
// decision of trial i and builds Ceres' summary from it; after the loop the last accepted candidate becomes the state and
// the current linearisation is moved to buffer set 0 for the host-driven entry points.
int lm_loop(pba_engine* e, const pba_solver_options* o, const Collective* coll, double* X, int K, pba_solver_summary* sum) {
  if (!coll) return lm_loop_single(e, o, sum);
  GnData& G = e->gn;
  const pba_solver_options opt = lm_options(o);
  pba_solver_summary s{};
  const double t0 = now_ms();
  if (!G.nc_sys && (G.band_kernel != K || G.solver == SOLVER_SKYLINE)) {
    const char* fs = getenv("PBA_SOLVER");
    const int solver = (K <= 8 && !(fs && std::string(fs) == "band")) ? SOLVER_CR : SOLVER_BAND;
    if (int rc = configure_solver(e, K, solver)) return rc;
  }
  double cost = 0.0;
  int n_valid = 0;
  if (int rc = linearize(e, &cost, nullptr, nullptr, nullptr, nullptr, &n_valid)) return rc;
  DistCheck chk;
  {  // Σ over ranks of the initial cost and valid blocks — and of 1: the number of ranks — through the scalar slots
    double v[3] = {cost, (double)n_valid, 1.0};
    double* Y = X + ex_scalar_off(e, K);
    PBA_HIP(hipMemcpyAsync(Y, v, sizeof v, hipMemcpyHostToDevice, e->stream));
    if (int rc = coll->allreduce(e, Y, 3)) return rc;
    PBA_HIP(hipMemcpyAsync(v, Y, sizeof v, hipMemcpyDeviceToHost, e->stream));
    PBA_HIP(hipStreamSynchronize(e->stream));
    cost = v[0];
    n_valid = (int)v[1];
    chk.n_ranks = (int)v[2];
  }
  if (const char* pv = test_hook("PBA_TEST_PERTURB_DECISION")) {  // test build: "rank:trial:mode"
    int pr = -1, pt = -1, pm = 1;
    if (std::sscanf(pv, "%d:%d:%d", &pr, &pt, &pm) >= 2 && pr == (coll->comm ? comm_rank(coll->comm) : G.dist_rank)) {
      chk.perturb_seq = pt;
      chk.perturb_mode = pm;
    }
  }
  s.linearize_ms = now_ms() - t0;
  s.initial_cost = cost;
  for (int i = 0; i < kRecRing * kRecStride; ++i) G.lm_h[i] = 0.0;  // (slot 0 stages the initial record below)
  G.lm_h[kLmCost] = cost;
  G.lm_h[kLmValid] = n_valid;
  G.lm_h[kLmXNorm] = -1.0;
  G.lm_h[kLmRadius] = opt.initial_trust_region_radius;
  G.lm_h[kLmFactor] = 2.0;
  G.lm_h[kLmLambda] = 1.0 / opt.initial_trust_region_radius;
  PBA_HIP(hipMemcpyAsync(G.lm.p, G.lm_h.data(), sizeof(double) * kLmFields, hipMemcpyHostToDevice, e->stream));
  const int n = std::max(0, opt.max_iterations);
  const DecideOpts dopt = decide_opts(opt);
  Trajectory traj(G.history, opt.initial_trust_region_radius);
  int last_enq = 0;  // the last trial enqueued (collectives included)
  if (n > 0) {
    if (int rc = dist_trial(e, *coll, dopt, X, K, 1.0, chk)) return rc;
    last_enq = 1;
  }
  int iter = 0, set = 0, stop_seq = 0;  // stop_seq: the trial whose record ended the loop
  double stop_done = 0.0;
  s.termination = PBA_TERMINATION_MAX_ITERATIONS;
  s.stop_reason = PBA_STOP_MAX_ITERATIONS;
  for (; iter < n; ++iter) {
    if (iter + 1 < n) {
      if (int rc = dist_trial(e, *coll, dopt, X, K, (double)(iter + 2), chk)) return rc;  // ahead of this decision
      last_enq = iter + 2;
    }
    double d[kLmFields];
    if (int rc = wait_decision(e, (double)(iter + 1), d)) return rc;
    set = (int)d[kLmSet];
    s.gradient_max_norm = d[kLmGradNorm];
    const double done = d[kLmDone];
    if (done == kDoneDesync) {
      stop_seq = iter + 1;
      stop_done = done;
      break;
    }
    traj.trial(d);
    if (done != 0.0 && done != kDoneRadius) {
      stop_seq = iter + 1;
      stop_done = done;
      if (finish_summary(done, s)) ++iter;
      break;
    }
    if (d[kLmAccept] == 0.0) {
      ++s.unsuccessful_steps;
      if (done != 0.0) {
        stop_seq = iter + 1;
        stop_done = done;
        finish_summary(done, s);
        ++iter;
        break;
      }
      continue;
    }
    ++s.successful_steps;
    cost = d[kLmCostNew];
  }
  // Every rank must leave with the same collectives issued.  Ranks whose records agree stop on the same trial; if they
  // differed at trial k, the next trial's check ends the solve everywhere (kDoneDesync), but a rank whose record k said
  // done has enqueued one trial fewer than a rank that went on (which enqueued k + 2 ahead): it reads record k + 1 (always
  // published) and, when ranks went on, issues trial k + 2 too.  Then the last decision is checked by one more scalar
  // all-reduce on every rank.
  bool desync = stop_done == kDoneDesync;
  int desync_at = desync ? stop_seq - 1 : 0;
  if (!desync && stop_seq > 0 && last_enq > stop_seq) {
    double d2[kLmFields];
    if (int rc = wait_decision(e, (double)(stop_seq + 1), d2)) return rc;
    if (d2[kLmDone] == kDoneDesync) {
      desync = true;
      desync_at = stop_seq;
      const int stopped = (int)d2[kLmDesync] - 1;  // ranks whose record stop_seq ended the solve
      if (stopped < chk.n_ranks && stop_seq + 2 <= n) {
        if (int rc = dist_trial(e, *coll, dopt, X, K, (double)(stop_seq + 2), chk)) return rc;
        last_enq = stop_seq + 2;
      }
    }
  }
  {
    double* Y = X + ex_scalar_off(e, K);
    dist_verify_kernel<<<1, 64, 0, e->stream>>>(G.lm.p, Y);
    PBA_HIP(hipGetLastError());
    if (int rc = coll->allreduce(e, Y, kExScalars)) return rc;
    const double vseq = (double)(last_enq + 1);
    dist_decide_kernel<<<1, 64, 0, e->stream>>>(Y, G.tpose.p, 1, dopt, G.lm.p, G.lm_host_d + rec_slot(vseq), vseq,
                                                chk.n_ranks, -1.0, 0, 1);
    PBA_HIP(hipGetLastError());
    double d3[kLmFields];
    if (int rc = wait_decision(e, vseq, d3)) return rc;
    if (!desync && d3[kLmDone] == kDoneDesync) {
      desync = true;
      desync_at = last_enq;
    }
  }
  launch_accept(e, G.lm.p);
  PBA_HIP(hipStreamSynchronize(e->stream));
  if (desync)
    return fail(PBA_ERR_DEVICE, "multi-GPU solve: the ranks' LM decisions differed at trial " + std::to_string(desync_at) +
                                    " (decision-word check); every rank ended the solve");
  traj.finish(s.initial_cost);
  if (set == 1) {
    std::swap(G.blk_schur.p, G.blk_schur1.p);
    std::swap(G.blk_schur.n, G.blk_schur1.n);
    std::swap(G.pair_rt.p, G.pair_rt1.p);
    std::swap(G.pair_rt.n, G.pair_rt1.n);
    std::swap(G.part_lin.p, G.part_lin1.p);
    std::swap(G.part_lin.n, G.part_lin1.n);
  }
  s.iterations = iter;
  s.final_cost = cost;
  s.total_ms = now_ms() - t0;
  if (sum) *sum = s;
  return PBA_OK;
}

}  // namespace

extern "C" {

int pba_solve(pba_engine* e, const pba_solver_options* o, pba_solver_summary* sum) {
  if (int rc = ensure_prepared(e)) return rc;
  return lm_loop(e, o, nullptr, nullptr, 0, sum);
}

int pba_solver_iterations(const pba_engine* e, int32_t capacity, pba_iteration_summary* out, int32_t* count) {
  if (!e || !count || capacity < 0 || (capacity > 0 && !out)) return fail(PBA_ERR_INVALID_ARGUMENT, "bad arguments");
  const std::vector<pba_iteration_summary>& h = e->gn.history;
  const int n = std::min<int>(capacity, (int)h.size());
  for (int i = 0; i < n; ++i) out[i] = h[i];
  *count = (int)h.size();
  return PBA_OK;
}

int pba_set_solver_timing(pba_engine* e, int32_t enable) {
  if (!e) return fail(PBA_ERR_INVALID_ARGUMENT, "null engine");
  e->gn.phase_timing = enable != 0;
  return PBA_OK;
}

int pba_solve_distributed(pba_engine* e, const pba_solver_options* o, int32_t band, double* d_exchange,
                          pba_allreduce_fn allreduce, void* user, pba_solver_summary* sum) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!d_exchange || !allreduce) return fail(PBA_ERR_INVALID_ARGUMENT, "null exchange buffer or allreduce");
  int K;
  if (int rc = exchange_K(e, band, &K)) return rc;
  Collective c;
  c.fn = allreduce;
  c.user = user;
  return lm_loop(e, o, &c, d_exchange, K, sum);
}

int pba_solve_distributed_comm(pba_engine* e, const pba_solver_options* o, int32_t band, pba_comm* comm,
                               pba_solver_summary* sum) {
  if (int rc = ensure_prepared(e)) return rc;
  if (!comm) return fail(PBA_ERR_INVALID_ARGUMENT, "null communicator");
  int K;
  if (int rc = exchange_K(e, band, &K)) return rc;
  GnData& G = e->gn;
  PBA_HIP(G.exchange.resize((size_t)exchange_count(e, K)));
  Collective c;
  c.comm = comm;
  return lm_loop(e, o, &c, G.exchange.p, K, sum);
}

}  // extern "C"
