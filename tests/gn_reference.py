"""Dense double-precision Gauss-Newton / LM reference built on the oracle's residuals and Jacobians.

Test infrastructure: restates what Ceres does around the cost functors for this problem so the engine's
on-device normal equations, Schur complement, step and LM loop can be checked element by element.
  * robust weighting: HuberLoss + Corrector (loss_function.cc:48-62, corrector.cc:42-110): w = ρ'(‖r‖²),
    JᵀWJ / JᵀWr (ρ'' ≤ 0 → first-order form), cost ½ρ(s)
  * LM damping (levenberg_marquardt_strategy.cc): D = clamp(diag(JᵀJ), 1e-6, 1e32), (H + λD)δ = −g
  * Schur elimination of the inverse distances (schur_complement_solver.cc), dense solve here
  * trust region (trust_region_minimizer.cc): ρ = Δcost / model decrease > 1e-3 accepts;
    radius /= max(1/3, 1 − (2ρ−1)³) on success, radius /= factor, factor *= 2 on failure
Small problems only (dense matrices).
"""
from __future__ import annotations

import numpy as np

import oracle as O
from helpers import synth


def huber(s, a):
    if a <= 0:
        return 0.5 * s, np.ones_like(s)
    out = s > a * a
    rs = np.sqrt(np.where(out, s, 1.0))
    cost = np.where(out, 0.5 * (2 * a * rs - a * a), 0.5 * s)
    w = np.where(out, a / rs, 1.0)
    return cost, w


def linearize(pb, poses, rho, a, fixed=(), n_valid=None):
    """H (N×N), g (N), cost, with N = 6·n_frames + n_points; fixed frames' columns zeroed.  n_valid (a list): the
    number of valid blocks is appended."""
    rec, valid = O.evaluate(pb, poses=poses, rho=rho, want_jac=True)
    if n_valid is not None:
        n_valid.append(int(valid.sum()))
    R = pb.R
    r, Jh, Jt, Jr = O.split_record(rec, R)
    s = (r ** 2).sum(1)
    cost_b, w = huber(s, a)
    w = np.where(valid == 1, w, 0.0)
    cost = float(np.where(valid == 1, cost_b, 0.0).sum())
    nf, npt = pb.n_frames, pb.n_points
    N = 6 * nf + npt
    fixed = set(int(f) for f in fixed)
    H = np.zeros((N, N))
    g = np.zeros(N)
    for b in range(pb.n_blocks):
        if w[b] == 0:
            continue
        p = pb.block_point[b]
        h, t = pb.point_host[p], pb.block_target[b]
        J = np.zeros((R, N))
        if h not in fixed:
            J[:, 6 * h:6 * h + 6] = Jh[b]
        if t not in fixed:
            J[:, 6 * t:6 * t + 6] = Jt[b]
        J[:, 6 * nf + p] = Jr[b]
        H += w[b] * J.T @ J
        g += w[b] * J.T @ r[b]
    return H, g, cost


def schur_step(H, g, nf, lam, fixed=()):
    """(S, gS, δ_poses, δ_points, model_decrease) of (H + λD)δ = −g with the points eliminated."""
    P = 6 * nf
    D = np.clip(np.diag(H), 1e-6, 1e32)
    fx = np.zeros(P, bool)
    for f in fixed:
        fx[6 * f:6 * f + 6] = True
    # frames never observed are constant too (engine: unobserved frames are fixed)
    for i in range(nf):
        if not np.any(H[6 * i:6 * i + 6, :]):
            fx[6 * i:6 * i + 6] = True
    Ha = H + lam * np.diag(D)
    A = Ha[:P, :P].copy()
    B = Ha[:P, P:].copy()
    C = np.diag(Ha[P:, P:]).copy()
    gp, gl = g[:P].copy(), g[P:].copy()
    A[fx, :] = 0
    A[:, fx] = 0
    A[fx, fx] = 1.0
    B[fx, :] = 0
    gp[fx] = 0
    Ci = np.where(C > 0, 1.0 / np.where(C > 0, C, 1.0), 0.0)
    S = A - (B * Ci) @ B.T
    gS = gp - B @ (Ci * gl)
    S[fx, :] = 0
    S[:, fx] = 0
    S[fx, fx] = 1.0
    gS[fx] = 0
    dp = np.linalg.solve(S, -gS)
    dl = -(gl + B.T @ dp) * Ci
    delta = np.concatenate([dp, dl])
    Dm = D.copy()
    Dm[:P][fx] = 0
    gfull = np.concatenate([gp, gl])
    model = 0.5 * (lam * float(delta @ (Dm * delta)) - float(gfull @ delta))
    return S, gS, dp.reshape(nf, 6), dl, model


def apply_step(poses, rho, dp, dl):
    return synth.se3_plus(poses, dp), rho + dl


def lm(pb, a, fixed=(), max_iterations=20, radius=1e4, function_tolerance=1e-6, min_relative_decrease=1e-3,
       parameter_tolerance=1e-8, gradient_tolerance=1e-10, max_trust_region_radius=1e16, min_trust_region_radius=1e-32,
       max_num_consecutive_invalid_steps=5, summary=False):
    """Ceres' trust-region loop with the LM strategy (trust_region_minimizer.cc:67-136, levenberg_marquardt_strategy.cc),
    in its order of tests:
      * FinalizeIteration (:312-355) after iteration 0 and every successful step: gradient tolerance
        max|x − (x ⊞ −g)| ≤ gradient_tolerance → CONVERGENCE (no further iteration);
      * invalid step (no predicted decrease, :434): the max_num_consecutive_invalid_steps-th in a row ends the solve
        with FAILURE (HandleInvalidStep :453-467, not counted as an iteration), the others act as a rejection;
      * candidate: infinite cost when a block valid at x is invalid there (Evaluate failing, :771-778);
      * parameter tolerance |x − x_new| ≤ ptol (x_norm + ptol), x_norm = −1 until the first successful step
        (:185, :706-726, :814); function tolerance |Δcost| ≤ ftol · cost (:729-748) — neither step applied;
      * IsStepSuccessful: relative decrease > min_relative_decrease (:781-803); StepAccepted radius update clamped at
        max_trust_region_radius (:146-153), StepRejected (:155-160); MinTrustRegionRadius (:687-703) → CONVERGENCE.
    Norms in the ambient space of the non-constant parameter blocks (free observed poses as [q | t], inverse distances
    of points with blocks)."""
    poses, rho = pb.poses.copy(), pb.rho.copy()
    nf = pb.n_frames
    nv = []
    H, g, cost = linearize(pb, poses, rho, a, fixed, nv)
    valid_cur = nv[-1]
    cost0 = cost
    free = np.array([f not in set(int(x) for x in fixed) and np.any(H[6 * f:6 * f + 6, :]) for f in range(nf)])
    has_blocks = np.zeros(pb.n_points, bool)
    has_blocks[pb.block_point] = True

    def gnorm(poses, g):
        tg = synth.se3_plus(poses, -g[:6 * nf].reshape(nf, 6))
        gp = np.abs(poses - tg)[free].max() if free.any() else 0.0
        gl = np.abs(g[6 * nf:])[has_blocks].max() if has_blocks.any() else 0.0
        return max(gp, gl)

    def xvec(poses, rho):
        return np.concatenate([poses[free].ravel(), rho[has_blocks]])

    factor = 2.0
    ok = bad = 0
    it = 0
    x_norm = -1.0
    invalid = 0
    invalid_candidates = 0
    history = []  # per valid step: (iteration, accepted, step norm, x_norm before it, gradient max norm after it)
    reason = "max_iterations"
    if gnorm(poses, g) <= gradient_tolerance:
        reason = "gradient_tolerance"
    else:
        for it in range(1, max_iterations + 1):
            lam = 1.0 / radius
            _, _, dp, dl, model = schur_step(H, g, nf, lam, fixed)
            if not model > 0:
                invalid += 1
                if invalid >= max_num_consecutive_invalid_steps:
                    reason = "invalid_steps"
                    it -= 1
                    break
                radius /= factor
                factor *= 2
                bad += 1
                if radius <= min_trust_region_radius:
                    reason = "min_trust_region_radius"
                    break
                continue
            invalid = 0
            np_, nr = apply_step(poses, rho, dp, dl)
            nv = []
            H1, g1, cost_new = linearize(pb, np_, nr, a, fixed, nv)
            if nv[-1] < valid_cur:
                cost_new = np.finfo(np.float64).max
                invalid_candidates += 1
            step = np.linalg.norm(xvec(np_, nr) - xvec(poses, rho))
            history.append([it, False, step, x_norm, None])
            if step <= parameter_tolerance * (x_norm + parameter_tolerance):
                reason = "parameter_tolerance"
                break
            if abs(cost - cost_new) <= function_tolerance * cost:
                reason = "function_tolerance"
                break
            rel = (cost - cost_new) / model
            if rel > min_relative_decrease:
                poses, rho, cost, valid_cur = np_, nr, cost_new, nv[-1]
                x_norm = float(np.linalg.norm(xvec(poses, rho)))
                radius = min(max_trust_region_radius, radius / max(1.0 / 3.0, 1.0 - (2.0 * rel - 1.0) ** 3))
                factor = 2.0
                ok += 1
                H, g = H1, g1
                history[-1][1] = True
                history[-1][4] = gnorm(poses, g)
                if it < max_iterations and history[-1][4] <= gradient_tolerance:
                    reason = "gradient_tolerance"
                    break
            else:
                radius /= factor
                factor *= 2
                bad += 1
                if radius <= min_trust_region_radius:
                    reason = "min_trust_region_radius"
                    break
    converged = reason not in ("max_iterations", "invalid_steps")
    if summary:
        return poses, rho, cost0, cost, it, {"successful_steps": ok, "unsuccessful_steps": bad, "converged": converged,
                                             "stop_reason": reason, "invalid_candidates": invalid_candidates,
                                             "history": history, "gnorm0": gnorm(pb.poses, linearize(pb, pb.poses, pb.rho, a, fixed)[1])}
    return poses, rho, cost0, cost, it


def partial_system(pb, poses, rho, a, lam):
    """One rank's contribution to the multi-GPU exchange (include/pba.h): nothing damped or fixed on the
    pose side, the rank's own points eliminated with their damping.  Returns (S_r, g_r, g_direct_r,
    diag(A_r), observed_r) with S_r = A_r − B_r (C_r + λ·clamp(C_r))⁻¹ B_rᵀ, g_r = g_p − B_r (C_r + λD_C)⁻¹ g_l."""
    H, g, _ = linearize(pb, poses, rho, a, ())
    P = 6 * pb.n_frames
    A, B = H[:P, :P], H[:P, P:]
    C = np.diag(H[P:, P:])
    Cd = C + lam * np.clip(C, 1e-6, 1e32)
    Ci = np.where(Cd > 0, 1.0 / np.where(Cd > 0, Cd, 1.0), 0.0)
    S = A - (B * Ci) @ B.T
    gS = g[:P] - B @ (Ci * g[P:])
    obs = np.array([np.any(H[6 * i:6 * i + 6, :]) for i in range(pb.n_frames)], np.float64)
    return S, gS, g[:P].copy(), np.diag(A).copy(), obs


def finalize_system(S, gS, dA, obs, lam, fixed=()):
    """The import side: + λ·clamp(diag(A)) and constant frames (requested or observed by no rank)."""
    n = len(obs)
    fx = np.zeros(6 * n, bool)
    for i in range(n):
        if i in set(int(f) for f in fixed) or obs[i] == 0:
            fx[6 * i:6 * i + 6] = True
    S = S + lam * np.diag(np.clip(dA, 1e-6, 1e32))
    gS = gS.copy()
    S[fx, :] = 0
    S[:, fx] = 0
    S[fx, fx] = 1.0
    gS[fx] = 0
    return S, gS


def reduced_system_sparse(pb, poses, rho, a, lam, fixed=(), n_threads=16):
    """The damped reduced camera system S (6·n_frames square, dense) and its right-hand side g_S of (H + λD)δ = −g with
    the inverse distances eliminated — the same quantities as schur_step, built block-sparsely in fp64 from the oracle's
    Jacobians so that C3-sized problems (200 keyframes × 20k points) fit: A and the point terms are scattered with
    bincount, the per-point Schur terms −W_p W_pᵀ / C'_p over the ≤ K + 1 frames each point touches.  Constant frames
    (requested, or observed by no block) get identity rows/columns and zero gradient, as in schur_step."""
    rec, valid = O.evaluate(pb, poses=poses, rho=rho, want_jac=True, n_threads=n_threads)
    return reduced_system_from_records(pb, rec, valid, a, lam, fixed)


def reduced_system_from_records(pb, rec, valid, a, lam, fixed=()):
    """reduced_system_sparse's system from given records ([r | J_h | J_t | J_ρ] per block, tangent space), every
    product and sum in fp64 — from the oracle's fp64 records, or from the engine's fp32 ones (what fp64 normal-equation
    products over the engine's fp32 rows would give: tools/probe/c4_lm_divergence.py)."""
    rec = np.asarray(rec, np.float64)
    R = pb.R
    r, Jh, Jt, Jr = O.split_record(rec, R)
    s = (r ** 2).sum(1)
    cost_b, w = huber(s, a)
    w = np.where(valid == 1, w, 0.0)
    nf, npt = pb.n_frames, pb.n_points
    N = 6 * nf
    h = pb.point_host[pb.block_point].astype(np.int64)
    t = pb.block_target.astype(np.int64)
    p = pb.block_point.astype(np.int64)
    fx = np.zeros(nf, bool)
    fx[list(int(f) for f in fixed)] = True
    obs = np.zeros(nf, bool)
    obs[h[w > 0]] = True
    obs[t[w > 0]] = True
    fx |= ~obs
    Jh = np.where(fx[h][:, None, None], 0.0, Jh) * np.sqrt(w)[:, None, None]
    Jt = np.where(fx[t][:, None, None], 0.0, Jt) * np.sqrt(w)[:, None, None]
    Jr = Jr * np.sqrt(w)[:, None]
    rw = r * np.sqrt(w)[:, None]
    six = np.arange(6)

    def scatter(fi, fj, blocks):  # Σ of 6×6 blocks into S[6fi:6fi+6, 6fj:6fj+6]
        idx = ((fi[:, None, None] * 6 + six[None, :, None]) * N + fj[:, None, None] * 6 + six[None, None, :]).ravel()
        return np.bincount(idx, weights=blocks.ravel(), minlength=N * N)

    S = scatter(h, h, np.einsum("bki,bkj->bij", Jh, Jh)) + scatter(t, t, np.einsum("bki,bkj->bij", Jt, Jt))
    Ht = np.einsum("bki,bkj->bij", Jh, Jt)
    S += scatter(h, t, Ht) + scatter(t, h, np.swapaxes(Ht, 1, 2))
    S = S.reshape(N, N)
    gp = np.bincount((h[:, None] * 6 + six).ravel(), weights=np.einsum("bki,bk->bi", Jh, rw).ravel(), minlength=N)
    gp += np.bincount((t[:, None] * 6 + six).ravel(), weights=np.einsum("bki,bk->bi", Jt, rw).ravel(), minlength=N)
    # points: C_p, g_p and W_p over the host (one entry per point) and each block's target
    C = np.bincount(p, weights=(Jr * Jr).sum(1), minlength=npt)
    gl = np.bincount(p, weights=(Jr * rw).sum(1), minlength=npt)
    Wh = np.stack([np.bincount(p, weights=(Jh[:, :, i] * Jr).sum(1), minlength=npt) for i in range(6)], 1)
    Wt = np.einsum("bki,bk->bi", Jt, Jr)  # per block (its target)
    Cd = C + lam * np.clip(C, 1e-6, 1e32)
    Ci = np.where(Cd > 0, 1.0 / np.where(Cd > 0, Cd, 1.0), 0.0)
    # entries per point: host first, then its blocks in order
    order = np.argsort(p, kind="stable")
    counts = np.bincount(p, minlength=npt)
    M = int(counts.max()) + 1
    F = np.full((npt, M), -1, np.int64)
    V = np.zeros((npt, M, 6))
    F[:, 0] = pb.point_host
    V[:, 0] = Wh
    start = np.concatenate([[0], np.cumsum(counts)[:-1]])
    slot = np.empty(len(p), np.int64)
    slot[order] = np.arange(len(p)) - np.repeat(start, counts)
    F[p, 1 + slot] = t
    V[p, 1 + slot] = Wt
    mask = F >= 0
    Fz = np.where(mask, F, 0)
    outer = np.einsum("pmi,pnj->pmnij", V, V) * Ci[:, None, None, None, None]
    fi = np.broadcast_to(Fz[:, :, None], (npt, M, M))
    fj = np.broadcast_to(Fz[:, None, :], (npt, M, M))
    mm = mask[:, :, None] & mask[:, None, :]
    S -= scatter(fi[mm], fj[mm], outer[mm]).reshape(N, N)
    gp -= np.bincount((Fz[mask][:, None] * 6 + six).ravel(),
                      weights=(V[mask] * (Ci * gl)[np.nonzero(mask)[0]][:, None]).ravel(), minlength=N)
    diagA = np.clip(scatter(h, h, np.einsum("bki,bkj->bij", Jh, Jh)).reshape(N, N).diagonal()
                    + scatter(t, t, np.einsum("bki,bkj->bij", Jt, Jt)).reshape(N, N).diagonal(), 1e-6, 1e32)
    S[np.arange(N), np.arange(N)] += lam * diagA
    fxe = np.repeat(fx, 6)
    S[fxe, :] = 0.0
    S[:, fxe] = 0.0
    S[fxe, fxe] = 1.0
    gp[fxe] = 0.0
    cost = float(np.where(valid == 1, cost_b, 0.0).sum())
    return S, gp, cost


def linearize_intrinsics(pb, poses, rho, intr, a, fixed=()):
    """Geometric blocks with the TARGET camera's intrinsics free (optimize_intrinsics, map_utils.h:339-345; the functor's
    sIntr_c2 block, reprojection.h:83-86): H (N×N), g, cost with N = 6·n_frames + 8·n_cams + n_points (unknowns in that
    order), from the oracle's 44-value records (orc_evaluate_intrinsics: projection with `intr`, host unprojection with
    pb.intrinsics); fixed frames' columns zeroed."""
    rec, valid = O.evaluate_intrinsics(pb, intr, poses=poses, rho=rho)
    r, Jh, Jt, Jr = O.split_record(rec[:, :28], 2)
    Ji = rec[:, 28:44].reshape(-1, 2, 8)
    s = (r ** 2).sum(1)
    cost_b, w = huber(s, a)
    w = np.where(valid == 1, w, 0.0)
    cost = float(np.where(valid == 1, cost_b, 0.0).sum())
    nf, nc, npt = pb.n_frames, pb.intrinsics.shape[0], pb.n_points
    K0 = 6 * nf
    N = K0 + 8 * nc + npt
    fixed = set(int(f) for f in fixed)
    H = np.zeros((N, N))
    g = np.zeros(N)
    for b in range(pb.n_blocks):
        if w[b] == 0:
            continue
        p = pb.block_point[b]
        h, t = pb.point_host[p], pb.block_target[b]
        c = pb.frame_cam[t]
        J = np.zeros((2, N))
        if h not in fixed:
            J[:, 6 * h:6 * h + 6] = Jh[b]
        if t not in fixed:
            J[:, 6 * t:6 * t + 6] = Jt[b]
        J[:, K0 + 8 * c:K0 + 8 * c + 8] = Ji[b]
        J[:, K0 + 8 * nc + p] = Jr[b]
        H += w[b] * J.T @ J
        g += w[b] * J.T @ r[b]
    return H, g, cost


def schur_step_intrinsics(H, g, nf, nc, lam, fixed=()):
    """schur_step over the f-blocks (poses, then the cameras' intrinsics): (S, gS, δ_f, δ_points, model_decrease) of
    (H + λD)δ = −g with the points eliminated; constant frames and never-observed frames / cameras get identity rows."""
    P = 6 * nf + 8 * nc
    D = np.clip(np.diag(H), 1e-6, 1e32)
    fx = np.zeros(P, bool)
    for f in fixed:
        fx[6 * f:6 * f + 6] = True
    for i in range(nf):
        if not np.any(H[6 * i:6 * i + 6, :]):
            fx[6 * i:6 * i + 6] = True
    for c in range(nc):
        sl = slice(6 * nf + 8 * c, 6 * nf + 8 * c + 8)
        if not np.any(H[sl, :]):
            fx[sl] = True
    Ha = H + lam * np.diag(D)
    A, B, C = Ha[:P, :P].copy(), Ha[:P, P:].copy(), np.diag(Ha[P:, P:]).copy()
    gp, gl = g[:P].copy(), g[P:].copy()
    A[fx, :] = 0
    A[:, fx] = 0
    A[fx, fx] = 1.0
    B[fx, :] = 0
    gp[fx] = 0
    Ci = np.where(C > 0, 1.0 / np.where(C > 0, C, 1.0), 0.0)
    S = A - (B * Ci) @ B.T
    gS = gp - B @ (Ci * gl)
    S[fx, :] = 0
    S[:, fx] = 0
    S[fx, fx] = 1.0
    gS[fx] = 0
    df = np.linalg.solve(S, -gS)
    dl = -(gl + B.T @ df) * Ci
    delta = np.concatenate([df, dl])
    Dm = D.copy()
    Dm[:P][fx] = 0
    model = 0.5 * (lam * float(delta @ (Dm * delta)) - float(np.concatenate([gp, gl]) @ delta))
    return S, gS, df, dl, model


def intrinsics_system_index(nf, nc):
    """Indices of the 6·nf + 8·nc f-block unknowns in the engine's reduced camera system (pba_gn_system_size: 6 per
    keyframe, then 12 per camera of which the first 8 are its intrinsics)."""
    return np.concatenate([np.arange(6 * nf)] + [6 * nf + 12 * c + np.arange(8) for c in range(nc)])
