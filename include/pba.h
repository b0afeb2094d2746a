/* include/pba.h — C ABI of the MI355X photometric bundle-adjustment residual/Jacobian engine.
 *
 * This is the drop-in boundary for the reference's hot path.  In the reference every residual block is
 * a separate Ceres AutoDiffCostFunction evaluated on CPU threads:
 *
 *   map_utils.h:347-375      problem build: one AutoDiffCostFunction<Functor,2,7,7,1,8> + HuberLoss per
 *                            (landmark, non-anchor observation); parameters (T_w_host, T_w_target, ρ, intr)
 *   reprojection.h:83-112    BundleAdjustmentReprojectionCostFunctor::operator()  (geometric residual)
 *   photometric_error.h:139-182  PhotometricError<8>::operator()                 (photometric residual)
 *   program_evaluator.h:139-258  ProgramEvaluator::Evaluate — the per-block ParallelFor this replaces
 *   residual_block.cc:69-198     ResidualBlock::Evaluate   — J_local = J_global · P(7×6)
 *   evaluation_callback.h:63-76  EvaluationCallback::PrepareForEvaluation — where pba_evaluate is called
 *
 * One engine evaluates ALL blocks of a problem in one launch on one GPU.  Conventions:
 *   pose        Sophus SE3d storage [qx qy qz qw tx ty tz], camera-to-world T_w_c (common_types.h:174-179)
 *   tangent     δ = [υ(3), ω(3)], right update T·exp(δ)  (local_parameterization_se3.hpp:43-50)
 *   point       anchored at its host keyframe; inverse DISTANCE ρ along the unit bearing of u_ref
 *               (common_types.h:205-217; reprojection.h:105-108)
 *   intrinsics  8-vector [fx fy cx cy p1 p2 p3 p4] (camera_models.h:50); model shared by all cameras,
 *               host camera model used for the target too (reprojection.h:99-100)
 *   block       (point, target keyframe); host = the point's host keyframe
 *   residuals   geometric: r = u_obs − π_t(T_w_t⁻¹ T_w_h b/ρ)                    (R = 2)
 *               photometric: r_k = I_t(π_t(R_th b_k + ρ t_th)) − I_h,k, k < P      (R = P)
 *               bilinear (default) or Ceres' bicubic interpolation of the u8 target image (pba_set_interpolator),
 *               Grid2D edge clamp
 *   record      per block, R×14 floats: [ r(R) | J_host(R×6) | J_target(R×6) | J_rho(R) ], row-major,
 *               tangent-space (= Ceres' J_global·P of residual_block.cc:136-158), NOT robustified
 *               (the loss stays with the caller, residual_block.cc:161-196).
 *   valid       per block 1/0; 0 when a projection leaves the camera's domain or a value is non-finite;
 *               the record is then all zeros (a Ceres adapter returns false for such a block,
 *               matching residual_block.cc:113-131).
 *
 * Memory: every pointer argument is a HOST pointer unless the function name ends in _device.  The engine
 * owns its device buffers; the caller owns its host buffers.  One engine per GPU; calls on one engine
 * must be serialised by the caller (thread-compatible, not thread-safe).  All functions return PBA_OK
 * (0) or a negative status; pba_last_error() describes the most recent failure of the calling thread.
 */
#ifndef PBA_H_
#define PBA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBA_OK 0
#define PBA_ERR_INVALID_ARGUMENT (-1)
#define PBA_ERR_DEVICE (-2)          /* HIP runtime error (no device, launch failure, …) */
#define PBA_ERR_OUT_OF_MEMORY (-3)
#define PBA_ERR_NOT_READY (-4)       /* a set_* call required by this call has not been made */

#define PBA_RESIDUAL_PHOTOMETRIC 0
#define PBA_RESIDUAL_GEOMETRIC 1

#define PBA_CAMERA_PINHOLE 0        /* camera_models.h:48-114  */
#define PBA_CAMERA_DOUBLE_SPHERE 1  /* camera_models.h:198-284 */
#define PBA_CAMERA_EUCM 2           /* camera_models.h:116-196 */
#define PBA_CAMERA_KB4 3            /* camera_models.h:286-421 (Kannala-Brandt, 4 distortion terms) */

#define PBA_MAX_PATTERN 32

typedef struct pba_engine pba_engine;

typedef struct pba_options {
  int32_t device;         /* HIP device ordinal */
  int32_t residual_kind;  /* PBA_RESIDUAL_* */
  int32_t camera_model;   /* PBA_CAMERA_* */
  float huber_width;      /* a of HuberLoss(a) for the per-block cost (loss_function.cc:48-62); <= 0: squared */
} pba_options;

/* Lifecycle ------------------------------------------------------------------------------------- */
int pba_create(const pba_options* options, pba_engine** out_engine);
int pba_destroy(pba_engine* engine);
const char* pba_status_string(int status);
const char* pba_last_error(void);
int pba_version(void);  /* 100·major + minor */

/* Problem description (BundleAdjustment problem build, map_utils.h:322-375) ---------------------- */
/* intrinsics: 8·n_cams doubles */
int pba_set_cameras(pba_engine* engine, int32_t n_cams, const double* intrinsics);
/* frame_cam[n_frames]: camera index of every keyframe; images: n_frames·height·width u8, row-major,
 * required for photometric engines (may be NULL for geometric ones). */
int pba_set_frames(pba_engine* engine, int32_t n_frames, const int32_t* frame_cam, int32_t width,
                   int32_t height, const uint8_t* images);
/* same, with the images already in device memory (copied device-to-device on the engine stream) */
int pba_set_frames_device(pba_engine* engine, int32_t n_frames, const int32_t* frame_cam, int32_t width,
                          int32_t height, const uint8_t* d_images);
/* residual pattern: P (du, dv) pairs, P <= PBA_MAX_PATTERN (photometric only) */
int pba_set_pattern(pba_engine* engine, int32_t P, const float* offsets);
/* points: host keyframe, u_ref (2 doubles, pixel in the host image), host_intensity (P floats,
 * photometric only — the I_h,k of photometric_error.h:179; NULL: sampled on the device from the host keyframe's
 * image at u_ref + pattern offset, with the engine's interpolator; a later pba_set_interpolator samples them again). */
int pba_set_points(pba_engine* engine, int32_t n_points, const int32_t* host_frame, const double* u_ref,
                   const float* host_intensity);
/* blocks: point index and target keyframe per block; u_obs (2 doubles per block) for geometric engines.
 * target != host(point) is required. */
int pba_set_blocks(pba_engine* engine, int32_t n_blocks, const int32_t* block_point,
                   const int32_t* block_target, const double* u_obs);

/* Evaluation (EvaluationCallback::PrepareForEvaluation → one launch) ----------------------------- */
/* poses: 7·n_frames doubles; inv_dist: n_points doubles (host memory; copied to the device) */
int pba_set_state(pba_engine* engine, const double* poses, const double* inv_dist);
int pba_set_state_device(pba_engine* engine, const double* d_poses, const double* d_inv_dist);
/* Enqueue the evaluation of every block on the engine's stream.  want_jacobians = 0 writes only the
 * residual part of each record (Ceres' residual-only evaluation, trust_region_minimizer.cc:761-779). */
int pba_evaluate(pba_engine* engine, int32_t want_jacobians);
/* Evaluate at a device-resident state and adopt it (afterwards it is the engine's state, as after
 * pba_set_state_device): Ceres' Evaluator::Evaluate(state, …) (program_evaluator.h:139-258), which reads the
 * parameter state straight from the caller's array.  Photometric engines do it in ONE launch — each block forms
 * its relative pose from the poses in its prologue and the launch copies the state — so no pair-table or copy
 * launch precedes the evaluation.  d_poses / d_inv_dist must stay valid until the launch has run. */
int pba_evaluate_state_device(pba_engine* engine, const double* d_poses, const double* d_inv_dist,
                              int32_t want_jacobians);
/* n evaluations back to back — state i = (d_poses[i], d_inv_dist[i]), each as pba_evaluate_state_device (one launch
 * that adopts it), enqueued by one call: a caller stepping through candidate states (a line search, a benchmark's
 * steps) pays the host-side launch cost in C instead of per foreign-function call.  Replaces n calls of
 * Evaluator::Evaluate (program_evaluator.h:139-258); the records hold the last state's evaluation. */
int pba_evaluate_states_device(pba_engine* engine, int32_t n, const double* const* d_poses,
                               const double* const* d_inv_dist, int32_t want_jacobians);
int pba_synchronize(pba_engine* engine);

/* Results ---------------------------------------------------------------------------------------- */
int pba_record_floats(const pba_engine* engine);   /* 14·R (22·R with pba_set_optimize_intrinsics) values per record */
/* Record storage format (photometric engines): PBA_RECORD_F32 (default) or PBA_RECORD_F16 — IEEE half records,
 * half the HBM write traffic (config C5's "fp16 residuals"; evaluation stays fp64 warp + fp32 chain, rounding
 * only at the store: ≤ 2⁻¹¹ relative per value; values beyond the half range saturate at ±65504 — at full
 * resolution a strong edge's rotation Jacobian can exceed it; the on-device GN path never reads records, it
 * accumulates JᵀJ from fp32 rows).  pba_get_records returns floats either way;
 * pba_device_records' pointer then addresses 14·R halves per block. */
#define PBA_RECORD_F32 0
#define PBA_RECORD_F16 1
int pba_set_record_format(pba_engine* engine, int32_t format);
int pba_record_format(const pba_engine* engine);
/* Target-intrinsics Jacobian (geometric engines; BundleAdjustmentOptions::optimize_intrinsics, map_utils.h:339-345):
 * the reference functor takes the TARGET camera's intrinsics as its 4th parameter block (sIntr_c2, reprojection.h:83-86,
 * :108) and unprojects the host pixel with the intrinsics captured at problem build (ref_intrinsics, :93-98; Ceres never
 * writes user memory during a solve without an evaluation callback, so those stay at their initial values).  Enabled,
 * every projection uses the intrinsics state (pba_set_intrinsics_state, 8·n_cams doubles; initially the cameras'),
 * host unprojection keeps the pba_set_cameras values, and each record grows by J_intr (R×8, row-major) after J_rho:
 * 22·R values.  The on-device Gauss-Newton (pba_gn_*, pba_solve) then optimises the intrinsics too: each camera's 8
 * intrinsics are 12 unknowns of the reduced camera system after the keyframes' (two 6-dim blocks, the last four pads
 * with identity rows), a dense border of the skyline system (SPARSE_SCHUR keeps the intrinsics blocks among the f-blocks,
 * schur_complement_solver.cc:138-146); k ← k + δk, Ceres' LM diagonal over them too.  The multi-GPU entry points
 * exchange the border rows too (pba_gn_exchange_size). */
int pba_set_optimize_intrinsics(pba_engine* engine, int32_t enable);
int pba_set_intrinsics_state(pba_engine* engine, const double* intrinsics);
/* the intrinsics state (8·n_cams doubles: the free intrinsics with pba_set_optimize_intrinsics, else the cameras') */
int pba_get_intrinsics(pba_engine* engine, double* intrinsics);
/* Image interpolator of the photometric residual (and of the device-sampled I_h,k): PBA_INTERP_BILINEAR (default,
 * the north star's) or PBA_INTERP_BICUBIC — Ceres' BiCubicInterpolator over Grid2D<uint8_t, 1>
 * (cubic_interpolation.h:252-344, edge clamp :403-414), the interpolator of PhotometricError<8>
 * (photometric_error.h:84): with PBA_CAMERA_EUCM the engine then evaluates that functor's residual exactly.
 * Applies to every evaluation and Gauss-Newton entry point. */
#define PBA_INTERP_BILINEAR 0
#define PBA_INTERP_BICUBIC 1
int pba_set_interpolator(pba_engine* engine, int32_t interpolator);
int pba_interpolator(const pba_engine* engine);
/* The interpolator at n positions uv (2 doubles each, (column, row) pixels, any value: outside the image the edge is
 * clamped as Grid2D does) of one frame of the active level: out = 3 floats per position [I, ∂I/∂u, ∂I/∂v]
 * (BiCubicInterpolator::Evaluate(r = v, c = u) returns f, dfdr = ∂I/∂v, dfdc = ∂I/∂u).  Synchronises. */
int pba_sample_image(pba_engine* engine, int32_t frame, int32_t n, const double* uv, float* out);
int pba_num_blocks(const pba_engine* engine);
int pba_num_points(const pba_engine* engine);
int pba_num_frames(const pba_engine* engine);
int pba_residuals_per_block(const pba_engine* engine);
/* records: n_blocks·record_floats floats; valid: n_blocks bytes (either may be NULL).  Synchronises. */
int pba_get_records(pba_engine* engine, float* records, uint8_t* valid);
/* residuals only: n_blocks·R floats (the first R values of every record, one strided DMA copy instead of the
 * whole record — what a residual-only evaluation needs, trust_region_minimizer.cc:761-779); valid may be NULL.
 * Synchronises. */
int pba_get_residuals(pba_engine* engine, float* residuals, uint8_t* valid);
/* Asynchronous read-back in chunks (fp32 records): enqueues the copies of records and validity into caller-owned
 * page-locked memory behind the evaluation, chunk_blocks blocks per copy, and returns at once; pba_wait_records returns
 * once the chunk holding `block` has arrived.  Thread-safe for concurrent waiters (Ceres' evaluator threads), so the
 * per-block CostFunction::Evaluate work overlaps the transfer of later chunks (program_evaluator.h:187-258). */
int pba_get_records_async(pba_engine* engine, float* records, uint8_t* valid, int32_t chunk_blocks);
int pba_wait_records(pba_engine* engine, int32_t block);
/* page-locked host memory for the read-back buffers of an adapter (records / residuals then arrive by DMA at
 * full PCIe rate instead of being staged through a driver buffer) */
int pba_host_alloc(size_t bytes, void** ptr);
int pba_host_free(void* ptr);
/* per-block cost ½ρ(‖r‖²) with the engine's Huber width (0 for invalid blocks) */
int pba_get_block_costs(pba_engine* engine, float* costs);
/* Σ block costs, summed in double on the host; n_valid may be NULL */
int pba_get_cost(pba_engine* engine, double* total_cost, int32_t* n_valid);

/* Device-side access for in-process consumers (zero copy) ----------------------------------------- */
/* hipStream_t the engine enqueues on (may be replaced with pba_set_stream; NULL = engine's own) */
int pba_set_stream(pba_engine* engine, void* hip_stream);
int pba_get_stream(pba_engine* engine, void** hip_stream);
int pba_device_records(pba_engine* engine, float** d_records, uint8_t** d_valid, float** d_costs);

/* Kernel timing: when enabled, every pba_evaluate brackets its residual/Jacobian block kernel with
 * hipEvents on the engine stream; pba_get_kernel_timing synchronises, returns the summed device time of
 * the block kernel (ms) and the launch count since the last call, and resets. */
int pba_enable_kernel_timing(pba_engine* engine, int32_t enable);
int pba_get_kernel_timing(pba_engine* engine, double* total_ms, int32_t* launches);

/* On-device Gauss-Newton / Levenberg-Marquardt --------------------------------
 * Replaces the solver side of ceres::Solve for this problem (map_utils.h:378-383: LM, SPARSE_SCHUR): the
 * normal equations JᵀJ / Jᵀr are accumulated on the device with the Huber corrector of
 * residual_block.cc:161-196, the inverse distances are eliminated (Schur complement; the <2,1,6>
 * structure of schur_complement_solver.cc:138-146), and the reduced camera system is factorised on the
 * device (block-skyline Cholesky, fp64).  Damping follows levenberg_marquardt_strategy.cc: (H + λ·D)δ = −g
 * with D = diag(JᵀJ) clamped to [1e-6, 1e32], λ = 1/trust-region radius. */
/* Termination as Ceres' TerminationType (types.h): CONVERGENCE on a tolerance or the minimum trust region radius,
 * NO_CONVERGENCE (here MAX_ITERATIONS) after max_iterations, FAILURE after max_num_consecutive_invalid_steps invalid
 * steps; stop_reason says which test ended the solve (trust_region_minimizer.cc, in its order of evaluation):
 *   gradient tolerance   max |x − (x ⊞ −∇)| ≤ gradient_tolerance at an accepted state (or the initial one), :668-684
 *   parameter tolerance  |x − x_candidate| ≤ parameter_tolerance (|x| + parameter_tolerance) for a valid step, with
 *                        |x| = −1 until the first accepted step (x_norm_, :185 / :814), :706-726
 *   function tolerance   |cost − candidate cost| ≤ function_tolerance · cost for a valid step, :729-748
 *   (neither candidate is applied) — norms in the ambient parameter space of the non-constant parameter blocks
 *   (poses as Sophus [q | t], inverse distances).  A candidate that leaves a block invalid which is valid at the current
 *   state has infinite cost (Ceres' failed Evaluate, :771-778). */
#define PBA_TERMINATION_CONVERGENCE 0
#define PBA_TERMINATION_MAX_ITERATIONS 1
#define PBA_TERMINATION_FAILURE 2

#define PBA_STOP_MAX_ITERATIONS 0
#define PBA_STOP_FUNCTION_TOLERANCE 1
#define PBA_STOP_PARAMETER_TOLERANCE 2
#define PBA_STOP_GRADIENT_TOLERANCE 3
#define PBA_STOP_MIN_TRUST_REGION_RADIUS 4
#define PBA_STOP_INVALID_STEPS 5

typedef struct pba_solver_options {
  int32_t max_iterations;                     /* BundleAdjustmentOptions::max_num_iterations (20, map_utils.h:318) */
  int32_t max_num_consecutive_invalid_steps;  /* Ceres default 5 (<= 0: 5) */
  double initial_trust_region_radius;         /* Ceres default 1e4 */
  double function_tolerance;                  /* Ceres default 1e-6 */
  double parameter_tolerance;                 /* Ceres default 1e-8 */
  double min_relative_decrease;               /* Ceres default 1e-3 */
  double gradient_tolerance;                  /* Ceres default 1e-10 */
  double max_trust_region_radius;             /* Ceres default 1e16 */
  double min_trust_region_radius;             /* Ceres default 1e-32 */
} pba_solver_options;

typedef struct pba_solver_summary {
  int32_t iterations;                   /* trials, the one that met a function / parameter tolerance included */
  int32_t successful_steps, unsuccessful_steps, termination;
  double initial_cost, final_cost;      /* Σ ½ρ(‖r‖²) */
  /* total_ms: host wall clock of the whole solve.  The parts: pba_solve — device time between stream events, only
   * with pba_set_solver_timing(engine, 1) (the events cost the GPU a few µs of idle time each, so they are off by
   * default and the parts are then 0): solve_ms = Schur complement + reduced solve + candidate state, linearize_ms =
   * the linearisation at each candidate (which is also its cost; plus the initial one), cost_ms = the decision; pba_solve_distributed — host wall clock of each phase, collectives included. */
  double total_ms, linearize_ms, solve_ms, cost_ms;
  double gradient_max_norm;             /* at the last state whose gradient was evaluated; pba_solve_distributed(_comm):
                                         * rank-local — max(the global pose part, this rank's points) */
  int32_t stop_reason, pad_;            /* PBA_STOP_* */
} pba_solver_summary;
/* per-phase device timing of pba_solve (linearize_ms / solve_ms / cost_ms of the summary); default off */
int pba_set_solver_timing(pba_engine* engine, int32_t enable);

/* One entry of the last solve's trajectory — Ceres' Solver::Summary::iterations (IterationSummary, iteration_callback.h;
 * filled as trust_region_minimizer.cc does): entry 0 is the initial state (successful, cost = the initial cost, radius =
 * the initial radius); then one entry per trial Ceres would push — accepted, rejected, invalid (:476-483) or ending on the
 * minimum trust-region radius — but not the trial that met the parameter / function tolerance or the invalid-step limit
 * (Minimize returns before FinalizeIteration, :110-115, :453-466).  cost: accepted — the new state's; rejected — the
 * candidate's (:124); invalid — the current state's.  trust_region_radius: after this iteration's update (:327).
 * gradient_max_norm: at the state the iteration ended in (a rejected step keeps the previous one, :130); after a
 * distributed solve it is rank-local (the global pose part, this rank's points), where Ceres reports the global value. */
typedef struct pba_iteration_summary {
  int32_t iteration, step_is_successful, step_is_valid, pad_;
  double cost, cost_change, relative_decrease, trust_region_radius, step_norm, gradient_max_norm;
} pba_iteration_summary;
/* copies min(capacity, entries) entries of the last pba_solve / pba_solve_distributed(_comm) into out (may be NULL with
 * capacity 0) and the number of entries into count; replaces reading Solver::Summary::iterations (map_utils.h:384-392) */
int pba_solver_iterations(const pba_engine* engine, int32_t capacity, pba_iteration_summary* out, int32_t* count);

/* constant parameter blocks (Problem::SetParameterBlockConstant, map_utils.h:334-336) */
int pba_set_fixed_frames(pba_engine* engine, int32_t n, const int32_t* frames);
/* Jacobian evaluation at the current state + normal-equation pieces; cost may be NULL */
int pba_gn_linearize(pba_engine* engine, double* cost);
/* Schur complement for damping lambda, reduced-system solve, candidate state; solver_status ≠ 0 when the
 * reduced system was not positive definite (the candidate is then not formed) */
int pba_gn_step(pba_engine* engine, double lambda, double* model_decrease, int32_t* solver_status);
int pba_gn_candidate_cost(pba_engine* engine, double* cost);
int pba_gn_accept(pba_engine* engine);   /* state ← candidate */
/* full LM loop (trust_region_minimizer.cc semantics); options may be NULL (Ceres defaults, 20 iterations).
 * A candidate counts as a failed evaluation (cost DBL_MAX, trust_region_minimizer.cc:771-778) when it has fewer valid
 * blocks than the current state — exactly Ceres' rule when every block is valid at the current state (the normal case:
 * an invalid block has no residual for Ceres either); from a state that already has invalid blocks, a block turning
 * valid can mask another turning invalid. */
int pba_solve(pba_engine* engine, const pba_solver_options* options, pba_solver_summary* summary);
/* read back the state (7·n_frames poses, n_points inverse distances) */
int pba_get_state(pba_engine* engine, double* poses, double* inv_dist);
/* testing/inspection: reduced camera system as a dense n² matrix, n = pba_gn_system_size (6·n_frames, + 12 per camera
 * with free intrinsics), and its right-hand side g (the solve is S δ = −g), and the last step (δ poses 6·n_frames, δρ
 * n_points) */
int pba_gn_system_size(pba_engine* engine, int32_t* n);
int pba_gn_get_reduced_system(pba_engine* engine, double* S_dense, double* g);
int pba_gn_get_step(pba_engine* engine, double* d_poses, double* d_inv_dist);

/* Multi-GPU Gauss-Newton ------------------------------------------------------------
 * One engine per GPU.  Every engine holds ALL keyframes (global frame indices, identical poses) and the
 * points hosted by its shard of keyframes with all their blocks, so the inverse distances are eliminated
 * locally (a point's blocks never leave its host's rank).  The only exchange is the sum of the per-rank
 * reduced camera systems: rank r contributes S_r = A_r − B_r (C_r + λD_C)⁻¹ B_rᵀ, its gradients and the
 * undamped pose diagonal; after the all-reduce every rank adds λ·clamp(diag), applies the constant frames
 * and solves the same system (block cyclic reduction / band Cholesky), then back-substitutes its own points.
 *
 * The exchange buffer is a DEVICE array of pba_gn_exchange_size doubles, banded with K ∈ {4, 8, 16} block
 * rows, K ≥ max over ranks of pba_gn_band: per frame i, (K+1) 6×6 blocks (block c = column i−K+c, row
 * major) followed by 24 doubles [g(6) | g_direct(6) | diag(A)(6) | observed | 0…]; with free intrinsics
 * (pba_set_optimize_intrinsics) then the 2·n_cams border rows of nfs = n_frames + 2·n_cams frames: per row, nfs 6×6
 * blocks (block y = column y; those right of the diagonal unused) and the same 24-double tail (observed = a camera this
 * rank observes) — the summed system is then solved as a skyline with its active front in LDS; then 16 scalar
 * slots. */
int pba_gn_band(pba_engine* engine, int32_t* band);   /* local reduced-system bandwidth (block rows) */
int pba_gn_exchange_size(pba_engine* engine, int32_t band, int64_t* count);
/* after pba_gn_linearize: point elimination for lambda + this rank's partial system into d_exchange */
int pba_gn_step_export(pba_engine* engine, double lambda, int32_t band, double* d_exchange);
/* d_exchange holds the sum over ranks: damping, constant frames, solve, candidate state.  model_pose is the
 * pose part of the LM model decrease (identical on every rank), model_points this rank's point part. */
int pba_gn_step_import(pba_engine* engine, double lambda, int32_t band, const double* d_exchange,
                       double* model_pose, double* model_points, int32_t* solver_status);
/* pba_solve over all ranks, steered by the device LM record as on one GPU: per trial, the banded partial systems
 * (and border rows; count = pba_gn_exchange_size − 16 doubles) and then 16 scalars are summed over the ranks: the point part (model
 * decrease, candidate cost and valid blocks, step and state norms, points above the gradient tolerance) from every
 * rank, and — with a pba_comm — the pose part and the reduced solve's status from rank 0 alone, so every rank takes the
 * same decision on the device from bit-identical inputs.  Two collectives per trial (trial i + 1's damping, hence its point elimination, depends
 * on trial i's decision).
 *
 * The collective is either a host callback — the in-place sum over all ranks of count doubles at d_buf (device memory
 * of this engine's GPU), called after the engine's stream has drained and complete when it returns — or a pba_comm,
 * whose sums are enqueued on the engine's stream (the host then enqueues trial i + 1 before trial i's decision is
 * known, as pba_solve does). */
typedef int (*pba_allreduce_fn)(void* user, double* d_buf, int64_t count);
/* This engine's rank in the host-callback collective of pba_solve_distributed (a pba_comm knows its own): rank 0 then
 * contributes the pose part and the solve status to the scalar sum as with a pba_comm; −1 (the default) leaves every
 * rank deciding from its own, bit-identical, copy. */
int pba_gn_set_rank(pba_engine* engine, int32_t rank);
int pba_solve_distributed(pba_engine* engine, const pba_solver_options* options, int32_t band, double* d_exchange,
                          pba_allreduce_fn allreduce, void* user, pba_solver_summary* summary);
/* Communicators.  RCCL (one process per GPU, over xGMI): rank 0 gets a 128-byte id from pba_comm_unique_id and shares
 * it (e.g. with torch.distributed.broadcast); every rank calls pba_comm_init (collective).  librccl.so.1 is opened at
 * run time.  In-process group (tests / one-GPU rehearsal): pba_comm_init_local(n, device, comms) fills comms[0..n) for n
 * engines on one device driven by n host threads; sums in rank order through events.  pba_comm_allreduce enqueues the
 * in-place sum of count doubles at d_buf on hip_stream (every rank, same order). */
typedef struct pba_comm pba_comm;
int pba_comm_unique_id(void* id128);
int pba_comm_init(const void* id128, int32_t n_ranks, int32_t rank, int32_t device, pba_comm** out_comm);
int pba_comm_init_local(int32_t n_ranks, int32_t device, pba_comm** out_comms);
int pba_comm_destroy(pba_comm* comm);
int pba_comm_rank(const pba_comm* comm);
int pba_comm_size(const pba_comm* comm);
int pba_comm_allreduce(pba_comm* comm, double* d_buf, int64_t count, void* hip_stream);
/* pba_solve_distributed over a communicator, with an exchange buffer owned by the engine */
int pba_solve_distributed_comm(pba_engine* engine, const pba_solver_options* options, int32_t band, pba_comm* comm,
                               pba_solver_summary* summary);

/* Image pyramid / coarse-to-fine ------------------------------------------
 * pba_build_pyramid builds levels 1 … n−1 on the device from the current frames, cameras and points (DSO
 * convention): level l+1 pixel = round(mean of a 2×2 level-l block), W_{l+1} = ⌊W_l/2⌋; camera fx_l = fx/2^l,
 * c_l = (c + 0.5)/2^l − 0.5 (distortion unchanged); u_ref_l likewise; the same pattern offsets; I_h,k re-sampled
 * from the host's level-l image.  pba_set_level selects the level every evaluation / Gauss-Newton entry point
 * runs on (state and problem structure are shared by all levels).  Any pba_set_cameras/frames/pattern/points
 * call returns to level 0 and drops the pyramid.  Photometric engines only. */
#define PBA_MAX_LEVELS 8
int pba_build_pyramid(pba_engine* engine, int32_t n_levels);
int pba_num_levels(const pba_engine* engine);
int pba_set_level(pba_engine* engine, int32_t level);
int pba_get_level(const pba_engine* engine, int32_t* level, int32_t* width, int32_t* height);
/* the active level's I_h,k (n_points·P floats) */
int pba_get_host_intensities(pba_engine* engine, float* host_intensity);
/* pba_solve on levels n−1 … 0 (coarse to fine); the summary sums iterations/timings, initial cost of the
 * coarsest level, final cost at level 0 */
int pba_solve_pyramid(pba_engine* engine, const pba_solver_options* options, pba_solver_summary* summary);

/* Reprojections and outlier flags after a bundle-adjustment pass -------------------
 * pba_compute_projections replaces compute_projections() + set_outlier_flags() of src/sfm.cpp:1928-2008 for
 * any list of observations (inlier and outlier obs; the anchor's own observation included, as the reference
 * does): with the engine's current state, per observation i of point p in frame f
 *   p_c = T_w_f⁻¹ · T_w_host(p) · (normalize(π_host⁻¹(u_ref(p))) / ρ_p)   (Landmark::get_p, common_types.h:205-217)
 *   reprojected = π_f(p_c), error = ‖obs_uv − reprojected‖, and for inlier observations the flags below
 *   (thresholds: sfm.cpp:254-261 defaults 3 px, 40 px, 0.1 m, 0.05 m when th == NULL).
 * fp64 throughout, at pyramid level 0.  All pointers are host pointers; obs_is_outlier, reprojected, point_c,
 * error, flags may be NULL. */
#define PBA_OUTLIER_NONE 0u
#define PBA_OUTLIER_REPROJECTION_HUGE 1u     /* error > huge threshold       (common_types.h:279) */
#define PBA_OUTLIER_REPROJECTION_NORMAL 2u   /* error > normal threshold     (common_types.h:281) */
#define PBA_OUTLIER_CAMERA_DISTANCE 4u       /* ‖p_c‖ < distance threshold    (common_types.h:283) */
#define PBA_OUTLIER_Z_COORDINATE 8u          /* p_c.z < z threshold           (common_types.h:285) */

typedef struct pba_outlier_thresholds {
  double reprojection_error_normal_px;  /* reprojection_error_outlier_threshold_normal_pixel (3.0)  */
  double reprojection_error_huge_px;    /* reprojection_error_outlier_threshold_huge_pixel (40.0)   */
  double camera_center_distance_m;      /* camera_center_distance_outlier_threshold_meter (0.1)     */
  double z_coordinate_m;                /* z_coordinate_outlier_threshold_meter (0.05)              */
} pba_outlier_thresholds;

int pba_compute_projections(pba_engine* engine, int32_t n_obs, const int32_t* obs_point, const int32_t* obs_frame,
                            const double* obs_uv, const uint8_t* obs_is_outlier, const pba_outlier_thresholds* th,
                            double* reprojected, double* point_c, double* error, uint32_t* flags);
/* remove_outlier_landmarks (sfm.cpp:2028-2114): remove[p] = 1 for points to drop.  Each point's inlier
 * observations are visited in frame-index order (= FrameCamId order when frames are indexed that way, as
 * pba_map_load does) and the first decisive flag wins; the normal-error flag removes a point only when no
 * observation anywhere carries another flag.  counts (may be NULL): [huge, normal, camera distance, z,
 * any_severe].  Host-only (no device needed). */
int pba_outlier_landmarks(int32_t n_points, int32_t n_obs, const int32_t* obs_point, const int32_t* obs_frame,
                          const uint32_t* flags, const uint8_t* obs_is_outlier, uint8_t* remove, int32_t* counts);

/* Problem loader from the reference's files ----------------------------------------
 * map.cereal (save_map_file, map_utils.h:58-86: cereal binary archive of corners, matches, tracks, outlier
 * tracks, cameras, landmarks; serializers serialization.h:155-205) + opt_calib.json (cereal JSON of the
 * Calibration, serialization.h:115-143; the DoubleSphere LoadCalibration form is accepted too), turned into
 * the arrays of pba_set_cameras/frames/points/blocks exactly as bundle_adjustment builds its problem
 * (map_utils.h:322-375): frames = map cameras in FrameCamId order (frame_cam = cam_id), points = landmarks in
 * TrackId order anchored at their smallest observing FrameCamId (u_ref = that corner, ρ = inv_depth),
 * blocks = the other observations (u_obs = their corners).  Host-only; the getters copy into caller arrays
 * sized from pba_map_info (any pointer may be NULL). */
typedef struct pba_map pba_map;
typedef struct pba_map_info {
  int32_t n_frames, n_points, n_blocks, n_cams;
  int32_t camera_model;      /* PBA_CAMERA_* shared by all cameras */
  int32_t n_outlier_obs;     /* Landmark::outlier_obs entries */
  int32_t width, height;     /* from the calibration (0 when absent) */
} pba_map_info;
int pba_map_load(const char* map_path, const char* calib_path, pba_map** out_map);
int pba_map_destroy(pba_map* map);
int pba_map_get_info(const pba_map* map, pba_map_info* info);
/* intrinsics 8·n_cams [fx fy cx cy p1 p2 p3 p4]; T_i_c 7·n_cams (Sophus storage) */
int pba_map_get_cameras(const pba_map* map, double* intrinsics, double* T_i_c);
/* FrameCamId.frame_id, cam_id (= camera index) and T_w_c per frame */
int pba_map_get_frames(const pba_map* map, int64_t* frame_id, int32_t* frame_cam, double* poses);
int pba_map_get_points(const pba_map* map, int64_t* track_id, int32_t* host_frame, double* u_ref, double* inv_dist);
int pba_map_get_blocks(const pba_map* map, int32_t* block_point, int32_t* block_target, double* u_obs);
int pba_map_get_outlier_obs(const pba_map* map, int32_t* point, int32_t* frame, double* uv);

#ifdef __cplusplus
}
#endif

#endif /* PBA_H_ */
