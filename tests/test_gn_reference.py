"""CPU tests of the dense GN/LM reference (tests/gn_reference.py) used to check the on-device solver."""
import numpy as np

import gn_reference as GR
from helpers import synth


def test_reference_lm_recovers_geometric_problem():
    pb = synth.make_problem(kind="geometric", n_frames=7, n_points=80, seed=3, obs_sigma=0.0, pose_sigma=0.002,
                            rho_sigma=0.02)
    pb.poses[:2] = pb.poses_gt[:2]  # gauge: two constant frames, as map_utils.h:334-336 / sfm.cpp:1903
    poses, rho, c0, c1, it = GR.lm(pb, a=1.0, fixed=(0, 1))
    assert c1 < 1e-8 * max(c0, 1.0) + 1e-12
    np.testing.assert_allclose(poses[:, 4:], pb.poses_gt[:, 4:], atol=1e-6)
    np.testing.assert_allclose(rho, pb.rho_gt, rtol=1e-6)


def test_schur_step_equals_full_solve():
    pb = synth.make_problem(n_frames=6, n_points=40, width=320, height=200, seed=4, border=12)
    H, g, _ = GR.linearize(pb, pb.poses, pb.rho, 9.0, fixed=(0,))
    lam = 1e-3
    S, gS, dp, dl, model = GR.schur_step(H, g, pb.n_frames, lam, fixed=(0,))
    # full damped system with frame 0 removed
    D = np.clip(np.diag(H), 1e-6, 1e32)
    keep = np.ones(H.shape[0], bool)
    keep[:6] = False
    Ha = (H + lam * np.diag(D))[np.ix_(keep, keep)]
    full = np.linalg.solve(Ha, -g[keep])
    np.testing.assert_allclose(np.concatenate([dp.ravel()[6:], dl]), full, rtol=1e-6, atol=1e-9)
    assert model > 0
