"""Image pyramid, coarse-to-fine solve and fp16 records (BASELINE.json config C5).

Pyramid parity: at every level the engine's records equal the oracle's on the level problem restated in numpy
(synth.level_problem: images downsampled by round(mean 2×2), c_l = (c + 0.5)/2^l − 0.5, fx_l = fx/2^l) with the
engine's own level-l host intensities, which in turn match double-precision bilinear sampling of the host's
level-l image (≤ 1e-3 intensity units: fp32 interpolation weights).  Record tolerances as tests/helpers.py.
fp16 records: every value within 2⁻¹¹ relative of the fp32 record (IEEE half rounding of the same evaluation;
absolute floor 2⁻¹⁴ for values near zero; Jacobian entries formed by cancellation may differ by 1e-6 of the block's
Jacobian scale between the two instantiations — helpers.fp16_violations) and identical validity.
"""
import numpy as np
import pytest

import oracle as O
from helpers import compare_records, engine_module, fp16_violations, projected_uv, synth

pytestmark = pytest.mark.gpu
E = engine_module()


@pytest.mark.parametrize("model", ["pinhole", "ds", "kb4"])
def test_pyramid_levels_match_oracle(model):
    pb = synth.make_problem(n_frames=7, n_points=200, width=320, height=200, model=model, seed=61, border=16)
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        eng.build_pyramid(3)
        for level in (2, 1, 0):
            eng.set_level(level)
            assert eng.level() == (level, 320 >> level, 200 >> level)
            eng.evaluate(True)
            rec, valid = eng.records()
            hi = eng.host_intensities()
            lp = synth.level_problem(pb, level)
            assert np.abs(hi - lp.host_intensity).max() <= 1e-3
            lp.host_intensity = hi
            ref, vref = O.evaluate(lp)
            assert valid.sum() > 0.8 * pb.n_blocks
            compare_records(0, pb.P, rec, ref, valid, vref, projected_uv(lp))


def test_host_intensities_sampled_on_device():
    """pba_set_points with host_intensity = NULL samples I_h,k from the host keyframe (bilinear)."""
    pb = synth.make_problem(n_frames=6, n_points=150, width=320, height=200, seed=62, border=12)
    pb.u_ref = pb.u_ref + np.random.default_rng(1).uniform(-0.5, 0.5, pb.u_ref.shape)  # sub-pixel anchors
    expect = synth.level_problem(pb, 0).host_intensity
    pb.host_intensity = None
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        got = eng.host_intensities()
    assert np.abs(got - expect).max() <= 1e-3


def test_pyramid_rejects_bad_use():
    pb = synth.make_problem(n_frames=6, n_points=40, width=64, height=32, seed=63, border=8)
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        with pytest.raises(E.PbaError):
            eng.build_pyramid(6)  # 64×32 → 2×1 at level 5
        eng.build_pyramid(2)
        with pytest.raises(E.PbaError):
            eng.set_level(2)
        eng.set_level(1)
        eng.set_problem(pb)  # new problem → back to level 0, pyramid dropped
        assert eng.level()[0] == 0
        with pytest.raises(E.PbaError):
            eng.set_level(1)
    g = synth.make_problem(kind="geometric", n_frames=6, n_points=20, seed=64)
    with E.Engine(g.kind, g.model) as eng:
        eng.set_problem(g)
        with pytest.raises(E.PbaError):
            eng.build_pyramid(2)


def test_coarse_to_fine_widens_the_basin():
    """Rendered plane scene at 4× the single-level LM test's pose error: LM on level 0 alone stalls far from the
    ground-truth cost, the 3-level coarse-to-fine solve reaches it (measured on MI355X: 135.5k vs 21.1k against a
    ground-truth cost of 20.4k; pose error 0.035 vs 0.0042 from 0.0128)."""
    pb = synth.make_problem(n_frames=10, n_points=1000, width=376, height=240, seed=41, border=16,
                            pose_sigma=0.008, rho_sigma=0.02)
    pb.poses[:2] = pb.poses_gt[:2]
    out, valid = O.evaluate(pb, poses=pb.poses_gt, rho=pb.rho_gt, want_jac=False)
    cost_gt = sum(O.huber_block(out[b, :pb.R], 9.0)[0] for b in range(pb.n_blocks) if valid[b])
    res = {}
    for mode in ("single", "pyramid"):
        with E.Engine(pb.kind, pb.model, huber_width=9.0) as eng:
            eng.set_problem(pb)
            eng.set_fixed_frames(np.array([0, 1], np.int32))
            eng.set_state(pb.poses, pb.rho)
            if mode == "pyramid":
                eng.build_pyramid(3)
                s = eng.solve_pyramid(max_iterations=15)
                assert eng.level()[0] == 0
                eng.evaluate(False)
                assert abs(s["final_cost"] - eng.cost()[0]) <= 1e-3 * s["final_cost"]
            else:
                s = eng.solve(max_iterations=45)
            poses, _ = eng.get_state()
        res[mode] = (s["final_cost"], np.abs(poses[2:, 4:] - pb.poses_gt[2:, 4:]).max(1).mean())
    err0 = np.abs(pb.poses[2:, 4:] - pb.poses_gt[2:, 4:]).max(1).mean()
    assert res["pyramid"][0] <= 1.1 * cost_gt, (res, cost_gt)
    assert res["pyramid"][1] < 0.5 * err0, (res, err0)
    assert res["single"][0] > 2.0 * res["pyramid"][0], res


@pytest.mark.parametrize("P", [8, 21, 5, 30])
def test_fp16_records(P):
    rng = np.random.default_rng(P)
    pat = synth.PATTERN8 if P == 8 else rng.integers(-3, 4, (P, 2)).astype(np.float32)
    pb = synth.make_problem(n_frames=7, n_points=300, width=320, height=200, pattern=pat, seed=70 + P, border=16)
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        eng.evaluate(True)
        r32, v32 = eng.records()
        eng.set_record_format(E.RECORD_F16)
        eng.evaluate(True)
        r16, v16 = eng.records()
        eng.evaluate(False)  # residual-only path in fp16 too
        ro, _ = eng.records()
    assert np.array_equal(v32, v16)
    bad = fp16_violations(r16, r32, projected_uv(pb), P)
    assert not bad.any(), (bad.sum(), np.unique(np.nonzero(bad)[1]))
    tol = 2.0 ** -11 * np.abs(r32[:, :P]) + 2.0 ** -14  # residuals: no cancellation, plain half rounding
    assert (np.abs(ro[:, :P] - r32[:, :P]) <= tol).all()


@pytest.mark.parametrize("n_cams", [1, 2])
@pytest.mark.parametrize("P", [21, 30])
def test_multi_pixel_kernel_forms_agree_bitwise(P, n_cams):
    """The 9-32 px kernel at a device state takes its camera constants three ways: once per lane from the camera
    record (one-camera problems), from the LDS camera table (≤ 4 cameras), or from each block's tile (more cameras).
    The per-block form is reached by the same problem registered with 6 cameras, the extra ones copies that no frame
    uses: the same values in the same arithmetic, so fp32 and fp16 records must be bit-identical."""
    import torch
    rng = np.random.default_rng(P + n_cams)
    pat = rng.integers(-3, 4, (P, 2)).astype(np.float32)
    intr = np.array([synth.DEFAULT_INTRINSICS[synth.PINHOLE]] * n_cams, np.float64)
    intr[:, :4] *= 320 / 752.0  # (explicit intrinsics are quoted for the image size)
    if n_cams == 2:
        intr[1, :4] *= [1.01, 0.99, 1.0, 1.0]
    pb = synth.make_problem(n_frames=9, n_points=400, width=320, height=200, pattern=pat, seed=80 + P, border=16,
                            intrinsics=intr, frame_cam=None if n_cams == 1 else np.arange(9) % 2)
    pb6 = synth.Problem(**{**pb.__dict__, "intrinsics": np.concatenate([intr, np.repeat(intr[:1], 6 - n_cams, 0)])})
    poses = torch.from_numpy(np.ascontiguousarray(pb.poses)).cuda()
    rho = torch.from_numpy(np.ascontiguousarray(pb.rho)).cuda()
    out = {}
    for form, prob in (("default", pb), ("per-block", pb6)):
        with E.Engine(pb.kind, pb.model) as eng:
            eng.set_problem(prob)
            eng.evaluate_state_device(poses.data_ptr(), rho.data_ptr(), True)
            r32, v32 = eng.records()
            c32 = eng.block_costs().copy()
            eng.set_record_format(E.RECORD_F16)
            eng.evaluate_state_device(poses.data_ptr(), rho.data_ptr(), True)
            r16, v16 = eng.records()
        out[form] = (r32.copy(), v32.copy(), r16.copy(), v16.copy(), c32)
    a, b = out["default"], out["per-block"]
    assert np.array_equal(a[4].view(np.uint32), b[4].view(np.uint32))  # block costs
    assert a[1].sum() > 0.8 * pb.n_blocks
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[3], b[3])
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    assert np.array_equal(a[2].view(np.uint16), b[2].view(np.uint16))
