"""CPU tests: the oracle (test infrastructure) against the reference-compiled golden vectors.

Golden vectors come from oracle/ref_harness.cpp compiled against the reference's own vendored Sophus 1.1.0 /
Eigen 3.3.8 (tests/golden/make_golden.py); this pins the oracle before any GPU result is compared with it.
"""
import numpy as np
import pytest

import oracle as O
from helpers import BLOCK_FIXTURES, load_golden, synth

SE3 = np.load(__import__("os").path.join(__import__("helpers").GOLDEN, "sophus_se3.npz"))


@pytest.mark.parametrize("i", range(0, 256, 5))
def test_se3_ops_match_sophus(i):
    T, T2, d, p = SE3["poses"][i], SE3["poses2"][i], SE3["deltas"][i], SE3["points"][i]
    np.testing.assert_allclose(O.se3_exp(d), SE3["exp"][i], atol=1e-13)
    np.testing.assert_allclose(O.se3_plus(T, d), SE3["plus"][i], atol=1e-12)
    np.testing.assert_allclose(O.se3_inverse(T), SE3["inverse"][i], atol=1e-12)
    np.testing.assert_allclose(O.se3_act(T, p), SE3["act"][i], atol=1e-12)
    np.testing.assert_allclose(O.se3_plus_jacobian(T), SE3["plus_jacobian"][i], atol=1e-14)
    np.testing.assert_allclose(O.se3_mul(O.se3_inverse(T2), T), SE3["rel"][i], atol=1e-12)


def test_numpy_se3_helpers_match_sophus():
    np.testing.assert_allclose(synth.se3_exp(SE3["deltas"]), SE3["exp"], atol=1e-12)
    np.testing.assert_allclose(synth.se3_plus(SE3["poses"], SE3["deltas"]), SE3["plus"], atol=1e-11)


@pytest.mark.parametrize("name", BLOCK_FIXTURES)
def test_oracle_matches_reference_harness(name):
    pb, z = load_golden(name)
    out, valid = O.evaluate(pb)
    exp, ev, fdok = z["expect_record"], z["expect_valid"], z["expect_fd_ok"].astype(bool)
    assert np.array_equal(valid, ev)
    R = pb.R
    m = (ev == 1) & fdok
    np.testing.assert_allclose(out[m, :R], exp[m, :R], atol=1e-9)
    for lo, hi in ((R, 7 * R), (7 * R, 13 * R), (13 * R, 14 * R)):
        scale = np.maximum(np.abs(exp[m, lo:hi]).max(1, keepdims=True), 1e-12)
        assert (np.abs(out[m, lo:hi] - exp[m, lo:hi]) / scale).max() < 1e-6
    assert np.all(out[ev == 0] == 0)


@pytest.mark.parametrize("kind,model", [(0, 0), (0, 1), (0, 2), (0, 3), (1, 0), (1, 1), (1, 2), (1, 3)])
def test_oracle_jacobians_vs_finite_differences(kind, model):
    pb = synth.make_problem(n_frames=6, n_points=12, width=320, height=200, kind=kind, model=model, seed=3 + model,
                            border=12)
    out, valid = O.evaluate(pb)
    R = pb.R
    r0, Jh, Jt, Jr = O.split_record(out, R)
    h = 1e-6
    for b in range(0, pb.n_blocks, 5):
        if not valid[b]:
            continue
        host, tgt, pt = pb.point_host[pb.block_point[b]], pb.block_target[b], pb.block_point[b]
        for which, J in ((host, Jh), (tgt, Jt)):
            for j in range(6):
                d = np.zeros(6)
                d[j] = h
                pp, pm = pb.poses.copy(), pb.poses.copy()
                pp[which] = synth.se3_plus(pb.poses[which], d)
                pm[which] = synth.se3_plus(pb.poses[which], -d)
                op, _ = O.evaluate(pb, poses=pp, want_jac=False, block_slice=slice(b, b + 1))
                om, _ = O.evaluate(pb, poses=pm, want_jac=False, block_slice=slice(b, b + 1))
                fd = (op[0, :R] - om[0, :R]) / (2 * h)
                scale = max(np.abs(J[b]).max(), 1e-9)
                # skip pixels whose stencil crosses a bilinear cell edge (gradient discontinuity)
                ok = np.abs(fd - J[b, :, j]) / scale < 1e-4
                assert ok.mean() >= 0.75, (b, which, j, fd, J[b, :, j])


def test_residual_only_matches_full():
    pb = synth.make_problem(n_frames=6, n_points=40, width=320, height=200, seed=5, border=12)
    full, v1 = O.evaluate(pb, want_jac=True)
    ronly, v2 = O.evaluate(pb, want_jac=False)
    assert np.array_equal(v1, v2)
    np.testing.assert_allclose(full[:, :pb.R], ronly[:, :pb.R], atol=1e-9)  # Jet value path rounds differently


def test_threaded_oracle_is_deterministic():
    pb = synth.make_problem(n_frames=8, n_points=200, width=320, height=200, seed=9, border=12)
    a, va = O.evaluate(pb, n_threads=1)
    b, vb = O.evaluate(pb, n_threads=4)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(va, vb)


def test_huber_corrector_semantics():
    # loss_function.cc:48-62 + corrector.cc: inlier → unit scale, cost ½s; outlier → √(a/‖r‖), cost ½(2a‖r‖ − a²)
    c, s = O.huber_block(np.array([0.3, 0.4]), 1.0)
    assert s == 1.0 and abs(c - 0.125) < 1e-15
    c, s = O.huber_block(np.array([3.0, 4.0]), 1.0)
    assert abs(s - np.sqrt(1.0 / 5.0)) < 1e-15 and abs(c - 0.5 * (2 * 5.0 - 1.0)) < 1e-12


def test_rendered_problem_is_photoconsistent_at_ground_truth():
    pb = synth.make_problem(n_frames=7, n_points=200, width=376, height=240, seed=21, border=12)
    out, valid = O.evaluate(pb, poses=pb.poses_gt, rho=pb.rho_gt, want_jac=False)
    r = out[valid == 1, :pb.R]
    assert valid.mean() > 0.95
    assert np.median(np.abs(r)) < 2.0  # quantisation + interpolation only
    out_p, _ = O.evaluate(pb, want_jac=False)
    assert np.median(np.abs(out_p[valid == 1, :pb.R])) > np.median(np.abs(r))
