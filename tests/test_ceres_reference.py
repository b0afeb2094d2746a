"""CPU tests against the REAL Ceres Solver 2.0.0 vendored in the reference (built by oracle/ceres.mk, no CMake):

* include/pba_ceres.h and tests/cpp/adapter_driver.cpp compile against the real ceres/ceres.h (not only against the
  test double tests/cpp/mock_ceres);
* the reference's CPU path — ceres::Solve (LM, SPARSE_SCHUR) over AutoDiff of the restated functors with the
  reference's own LocalParameterizationSE3 (tests/cpp/ceres_lm_driver.cpp, cpu mode) — takes exactly the trajectory
  of tests/gn_reference.lm, which the GPU LM tests compare against.  This pins the Python LM reference (trust-region
  radius updates, function-tolerance stop, Huber corrector, Schur step) to Ceres itself.
Skipped where /root/reference (compile test) or the built driver is absent.
"""
import os
import subprocess

import numpy as np
import pytest

import ceres_runner as CR
import gn_reference as GR
from helpers import ROOT, synth

REF = "/root/reference"
needs_driver = pytest.mark.skipif(not CR.available(), reason="oracle/_ref/ceres_lm_driver not built")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "thirdparty", "ceres-solver")), reason="reference absent")
def test_adapter_compiles_against_real_ceres():
    flags = subprocess.run(["make", "-s", "-f", "ceres.mk", "print-flags"], cwd=os.path.join(ROOT, "oracle"),
                           check=True, capture_output=True, text=True).stdout.split()
    for src in ("adapter_driver.cpp", "ceres_lm_driver.cpp"):
        cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Wno-deprecated",
               "-Wno-deprecated-declarations", "-Wno-sign-compare", "-Wno-ignored-qualifiers", "-Wno-misleading-indentation",
               *[f for f in flags if f.startswith(("-D", "-I"))],
               "-I", os.path.join(REF, "thirdparty", "Sophus"), "-I", os.path.join(REF, "include", "visnav"),
               "-I", os.path.join(REF, "thirdparty", "ceres-solver", "internal", "ceres", "autodiff_benchmarks"),
               "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "tests", "cpp"),
               os.path.join(ROOT, "tests", "cpp", src)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-4000:]


@needs_driver
@pytest.mark.parametrize("kind,model,huber", [(1, 0, 1.0), (1, 1, 1.0), (0, 0, 9.0), (0, 1, 9.0)])
def test_real_ceres_lm_equals_python_reference(kind, model, huber):
    pb = synth.make_problem(kind=kind, model=model, n_frames=8, n_points=120, width=376, height=240, seed=31,
                            border=12, obs_sigma=0.3)
    pb.poses[:2] = pb.poses_gt[:2]
    got = CR.run("cpu", pb, iters=15, huber=huber, threads=4)
    p_ref, r_ref, c0, c1, it, info = GR.lm(pb, huber, (0, 1), max_iterations=15, summary=True)
    assert abs(got["costs"][0] - c0) <= 1e-12 * c0
    assert abs(got["final_cost"] - c1) <= 1e-9 * c1
    # Ceres counts iteration 0 as a successful step (trust_region_minimizer.cc:313-320)
    assert got["successful_steps"] == info["successful_steps"] + 1
    assert got["unsuccessful_steps"] == info["unsuccessful_steps"]
    assert (got["termination"] == 0) == info["converged"]  # ceres::CONVERGENCE == 0
    np.testing.assert_allclose(got["poses"], p_ref, atol=1e-12)
    np.testing.assert_allclose(got["rho"], r_ref, rtol=1e-10)


@needs_driver
def test_real_photometric_error_lm_equals_python_reference():
    """EUCM + bicubic: real Ceres LM over the vendored ceres::PhotometricError<8> (reference-held functor) takes the
    trajectory of tests/gn_reference.lm over the oracle — pins the oracle's bicubic functor inside a whole solve."""
    from test_ceres_golden import load_ceres_photometric
    pb, _, _ = load_ceres_photometric()
    pb.poses[:2] = synth.se3_plus(pb.poses[:2], np.zeros((2, 6)))
    got = CR.run("cpu", pb, iters=10, huber=9.0, threads=4)
    p_ref, r_ref, c0, c1, it, info = GR.lm(pb, 9.0, (0, 1), max_iterations=10, summary=True)
    assert abs(got["costs"][0] - c0) <= 1e-10 * c0
    assert abs(got["final_cost"] - c1) <= 1e-8 * c1, (got["final_cost"], c1)
    assert got["successful_steps"] == info["successful_steps"] + 1
    assert got["unsuccessful_steps"] == info["unsuccessful_steps"]
    np.testing.assert_allclose(got["poses"], p_ref, atol=1e-10)
    np.testing.assert_allclose(got["rho"], r_ref, rtol=1e-8)


@needs_driver
def test_real_ceres_c1_sized_solve_converges():
    """configs[0] (C1) on the reference's CPU path: 40 stereo frames, 2k landmarks, 8k blocks, EuRoC DS calibration."""
    pb = synth.c1_problem()
    pb.poses[:2] = pb.poses_gt[:2]
    got = CR.run("cpu", pb, iters=20, huber=1.0, threads=os.cpu_count() or 8)
    assert got["termination"] == 0, got["message"]
    assert got["final_cost"] < 0.2 * got["costs"][0]
    # the least-squares optimum lies at or below the cost of the true state (the observations carry 0.5 px noise)
    import oracle as O
    out, valid = O.evaluate(pb, poses=pb.poses_gt, rho=pb.rho_gt, want_jac=False)
    c_true = sum(O.huber_block(out[b, :2], 1.0)[0] for b in range(pb.n_blocks) if valid[b])
    assert got["final_cost"] <= c_true, (got["final_cost"], c_true)


@needs_driver
def test_teacher_mode_reproduces_the_free_solve():
    """ceres_lm_driver's teacher mode (one LM iteration from each given state and trust-region radius — how the GPU
    tests check every iteration of the engine's solve against Ceres' own step from the same point): from the initial
    state with the default radius it takes the free solve's first iteration (cost before and after, accept, radius after)."""
    pb = synth.make_problem(n_frames=8, n_points=120, width=376, height=240, seed=21, border=14)
    free = CR.run("cpu", pb, iters=3, huber=9.0, threads=2)
    tr = CR.run("cpu", pb, iters=3, huber=9.0, threads=2, teacher=[(pb.poses, pb.rho, 1e4), (pb.poses, pb.rho, 1e4)])
    t = tr["teacher"]
    assert t.shape == (2, 8)
    for row in t:
        assert row[0] == pytest.approx(free["costs"][0], rel=1e-12)
        assert row[1] == pytest.approx(free["costs"][1], rel=1e-12)
        assert bool(row[2]) == bool(free["step_ok"][1])
        assert row[4] == pytest.approx(free["radius"][1], rel=1e-12)
