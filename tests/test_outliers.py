"""Reprojections, outlier flags and landmark removal after a BA pass (src/sfm.cpp:1928-2114).

CPU tests: the product's host-side removal logic (pba_outlier_landmarks in libpba.so, no device call) against
the oracle's restatement of remove_outlier_landmarks over map<track, map<FrameCamId, flags>>.
GPU tests: pba_compute_projections against the oracle's double restatement of compute_projections +
set_outlier_flags — reprojections within 1e-8 px, camera-frame points within 1e-12 relative, flags identical
away from the thresholds (|error − threshold| > 1e-7 px, |‖p_c‖ − d| and |z − z_th| > 1e-9 m), and the
resulting removal decisions identical.
"""
import numpy as np
import pytest

import oracle as O
from helpers import engine_module, synth

E = engine_module()
TH = (3.0, 40.0, 0.1, 0.05)  # src/sfm.cpp:254-261


def random_flags(rng, n_points, n_obs, p_flag):
    obs_point = rng.integers(0, n_points, n_obs).astype(np.int32)
    obs_frame = rng.integers(0, 40, n_obs).astype(np.int32)
    # one observation per (point, frame), as in a FeatureTrack map
    key = obs_point.astype(np.int64) * 1000 + obs_frame
    _, first = np.unique(key, return_index=True)
    obs_point, obs_frame = obs_point[first], obs_frame[first]
    n = len(obs_point)
    flags = np.zeros(n, np.uint32)
    for bit, p in zip((1, 2, 4, 8), p_flag):
        flags |= np.where(rng.random(n) < p, bit, 0).astype(np.uint32)
    flags |= np.where(flags & 1, 2, 0).astype(np.uint32)  # huge ⊂ normal, as set_outlier_flags produces
    outlier = (rng.random(n) < 0.05).astype(np.uint8)
    flags[outlier.astype(bool)] = 0
    return obs_point, obs_frame, flags, outlier


@pytest.mark.parametrize("p_flag", [(0.0, 0.05, 0.0, 0.0), (0.01, 0.05, 0.01, 0.01), (0.0, 0.0, 0.0, 0.0),
                                    (0.2, 0.3, 0.2, 0.2)])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_outlier_landmarks_host_logic_matches_reference(p_flag, seed):
    rng = np.random.default_rng(seed)
    n_points = 500
    op, of, fl, oo = random_flags(rng, n_points, 4000, p_flag)
    perm = rng.permutation(len(op))  # input order must not matter (tracks are visited in frame order)
    rm, counts = E.outlier_landmarks(n_points, op[perm], of[perm], fl[perm], oo[perm])
    rm_ref, counts_ref = O.outlier_landmarks(n_points, op, of, fl, oo)
    assert np.array_equal(rm, rm_ref)
    assert counts == counts_ref


def test_outlier_landmarks_normal_only_when_no_severe():
    # point 0: normal only; point 1: z flag → severe present → the normal-only point stays
    op = np.array([0, 0, 1, 1], np.int32)
    of = np.array([0, 1, 0, 1], np.int32)
    fl = np.array([0, 2, 0, 8], np.uint32)
    rm, c = E.outlier_landmarks(2, op, of, fl)
    assert rm.tolist() == [False, True] and c["normal"] == 1 and c["z"] == 1 and c["any_severe"] == 1
    rm, c = E.outlier_landmarks(2, op, of, np.array([0, 2, 0, 0], np.uint32))
    assert rm.tolist() == [True, False] and c["any_severe"] == 0


def observations(pb, rng):
    """Every observation of every point: its anchor (u_ref in the host) and its blocks' u_obs, some of them
    corrupted to trigger each flag, a few marked as outlier_obs."""
    n = pb.n_points
    op = np.concatenate([np.arange(n, dtype=np.int32), pb.block_point]).astype(np.int32)
    of = np.concatenate([pb.point_host, pb.block_target]).astype(np.int32)
    uv = np.concatenate([pb.u_ref, pb.u_obs]).astype(np.float64)
    m = len(op)
    sel = rng.random(m) < 0.03
    uv[sel] += rng.normal(0, 60.0, (sel.sum(), 2))            # huge
    sel = rng.random(m) < 0.05
    uv[sel] += rng.normal(0, 4.0, (sel.sum(), 2))             # normal
    outlier = (rng.random(m) < 0.03).astype(np.uint8)
    return op, of, uv, outlier


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["pinhole", "ds", "eucm", "kb4"])
def test_compute_projections_match_reference(model):
    rng = np.random.default_rng(11)
    pb = synth.make_problem(kind="geometric", model=model, n_frames=20, n_points=800, seed=21, obs_sigma=0.3)
    rho = pb.rho.copy()
    rho[:15] = 1.0 / rng.uniform(0.01, 0.09, 15)   # closer than the 0.1 m camera-distance threshold
    op, of, uv, oo = observations(pb, rng)
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, rho)
        got = eng.compute_projections(op, of, uv, oo, TH)
    ref = O.compute_projections(pb, pb.poses, rho, op, of, uv, oo, TH)
    assert np.abs(got["reprojected"] - ref["reprojected"]).max() <= 1e-8
    assert np.abs(got["point_c"] - ref["point_c"]).max() <= 1e-12 * max(1.0, np.abs(ref["point_c"]).max())
    assert np.abs(got["error"] - ref["error"]).max() <= 1e-8
    e, d, z = ref["error"], np.linalg.norm(ref["point_c"], axis=1), ref["point_c"][:, 2]
    clear = ((np.abs(e - TH[0]) > 1e-7) & (np.abs(e - TH[1]) > 1e-7) & (np.abs(d - TH[2]) > 1e-9) &
             (np.abs(z - TH[3]) > 1e-9))
    assert np.array_equal(got["flags"][clear], ref["flags"][clear])
    for bit in (1, 2, 4):
        assert (ref["flags"] & bit).any(), f"fixture should exercise flag {bit}"
    rm, c = E.outlier_landmarks(pb.n_points, op, of, got["flags"], oo)
    rm_ref, c_ref = O.outlier_landmarks(pb.n_points, op, of, ref["flags"], oo)
    assert np.array_equal(rm, rm_ref) and c == c_ref


@pytest.mark.gpu
def test_compute_projections_default_thresholds_and_anchor():
    """The anchor's own observation reprojects onto u_ref (the reference projects it too, sfm.cpp:1968)."""
    pb = synth.make_problem(kind="geometric", n_frames=8, n_points=64, seed=3)
    op = np.arange(pb.n_points, dtype=np.int32)
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        got = eng.compute_projections(op, pb.point_host, pb.u_ref)
    assert np.abs(got["reprojected"] - pb.u_ref).max() < 1e-9
    assert (got["flags"] == 0).all()
