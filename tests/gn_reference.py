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


def linearize(pb, poses, rho, a, fixed=()):
    """H (N×N), g (N), cost, with N = 6·n_frames + n_points; fixed frames' columns zeroed."""
    rec, valid = O.evaluate(pb, poses=poses, rho=rho, want_jac=True)
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
       summary=False):
    """Ceres' trust-region loop (trust_region_minimizer.cc:67-136): an invalid step (no predicted decrease) and a
    rejected one shrink the radius; a valid step whose |cost change| ≤ function_tolerance · cost ends the solve
    WITHOUT being applied (FunctionToleranceReached, :115-117, checked before IsStepSuccessful)."""
    poses, rho = pb.poses.copy(), pb.rho.copy()
    H, g, cost = linearize(pb, poses, rho, a, fixed)
    cost0 = cost
    factor = 2.0
    it = 0
    ok = bad = 0
    converged = False
    for it in range(1, max_iterations + 1):
        lam = 1.0 / radius
        _, _, dp, dl, model = schur_step(H, g, pb.n_frames, lam, fixed)
        if not model > 0:
            radius /= factor
            factor *= 2
            bad += 1
            continue
        np_, nr = apply_step(poses, rho, dp, dl)
        _, _, cost_new = linearize(pb, np_, nr, a, fixed)
        if abs(cost - cost_new) <= function_tolerance * cost:
            converged = True
            break
        rel = (cost - cost_new) / model
        if rel > min_relative_decrease:
            poses, rho, cost = np_, nr, cost_new
            radius = radius / max(1.0 / 3.0, 1.0 - (2.0 * rel - 1.0) ** 3)
            factor = 2.0
            ok += 1
            H, g, cost = linearize(pb, poses, rho, a, fixed)
        else:
            radius /= factor
            factor *= 2
            bad += 1
    if summary:
        return poses, rho, cost0, cost, it, {"successful_steps": ok, "unsuccessful_steps": bad, "converged": converged}
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
