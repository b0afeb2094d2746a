"""GPU parity of the bicubic interpolator (pba_set_interpolator(PBA_INTERP_BICUBIC)) against the reference-held
arithmetic of the vendored Ceres 2.0.0 (tests/golden/make_ceres_golden.py):

* pba_sample_image (the tiled, apron-padded u8 frames and the device interpolator) against Ceres'
  BiCubicInterpolator<Grid2D<uint8_t,1>> at 3000 positions in and around an EuRoC crop, at the out-of-bounds
  integer positions of cubic_interpolation_test.cc:114-149 (Grid2D edge clamp: exact grid values), and on the integer
  quadratic that the spline reproduces exactly (cubic_interpolation_test.cc:331-367);
* the whole residual/Jacobian evaluation with EUCM + bicubic against ceres::PhotometricError<8> through
  AutoDiffCostFunction (photometric_error.h:79-189) with LocalParameterizationSE3 tangent Jacobians: the photometric
  residual pinned by reference-held code, not only by the build's own restatement.
Tolerances: sampled values |Δ| ≤ 1e-4 (fp32 output of fp64 arithmetic on a 0-255 scale), gradients |Δ| ≤ 1e-4;
records as tests/helpers.compare_records (1e-4 intensity, 1e-5 relative Jacobians); validity identical.
"""
import os

import numpy as np
import pytest

from helpers import GOLDEN, compare_records, engine_module, projected_uv, synth
from test_ceres_golden import load_ceres_photometric

pytestmark = pytest.mark.gpu
E = engine_module()


def sampler(img, interp):
    pb = synth.Problem(kind=0, model=0, width=img.shape[1], height=img.shape[0],
                       intrinsics=np.array([[100.0, 100.0, img.shape[1] / 2, img.shape[0] / 2, 0, 0, 0, 0]]),
                       frame_cam=np.zeros(2, np.int32), images=np.stack([img, img]), pattern=synth.PATTERN8,
                       point_host=np.zeros(1, np.int32), u_ref=np.array([[1.0, 1.0]]),
                       host_intensity=np.zeros((1, 8), np.float32), block_point=np.zeros(1, np.int32),
                       block_target=np.ones(1, np.int32), u_obs=None, poses=np.tile([0, 0, 0, 1.0, 0, 0, 0], (2, 1)),
                       rho=np.ones(1), interp=interp)
    eng = E.Engine(0, 0)
    eng.set_problem(pb)
    return eng


@pytest.mark.parametrize("case", ["rand", "grid", "quad"])
def test_sample_image_matches_ceres_bicubic(case):
    z = np.load(os.path.join(GOLDEN, "ceres_bicubic.npz"))
    img = {"rand": z["crop"], "grid": z["grid"], "quad": z["quad"]}[case]
    uv, ref = z["uv_" + case], z["out_" + case]  # ref: [f, dfdr, dfdc]
    with sampler(img, 1) as eng:
        got = eng.sample_image(0, uv).astype(np.float64)  # [I, ∂I/∂u, ∂I/∂v]
    np.testing.assert_allclose(got[:, 0], ref[:, 0], atol=1e-4)
    np.testing.assert_allclose(got[:, 1], ref[:, 2], atol=1e-4)
    np.testing.assert_allclose(got[:, 2], ref[:, 1], atol=1e-4)
    if case == "grid":  # Grid2D out-of-bounds expectations, exactly
        np.testing.assert_array_equal(got[:, 0], z["expect_grid"])


def test_sample_image_bilinear_matches_oracle():
    import oracle as O
    z = np.load(os.path.join(GOLDEN, "ceres_bicubic.npz"))
    img, uv = z["crop"], z["uv_rand"]
    with sampler(img, 0) as eng:
        got = eng.sample_image(1, uv).astype(np.float64)
    ref = O.sample(img, uv, interp=0)
    np.testing.assert_allclose(got, ref, atol=1e-4)


def test_eucm_bicubic_records_match_ceres_photometric_error():
    pb, ref, vref = load_ceres_photometric()
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        eng.evaluate(True)
        rec, valid = eng.records()
        eng.evaluate(False)
        res, valid_r = eng.residuals()
    # bicubic has a continuous gradient: no cell-edge masking needed
    st = compare_records(0, 8, rec, ref, valid, vref)
    assert np.array_equal(valid_r, vref)
    np.testing.assert_allclose(res[vref == 1], ref[vref == 1, :8], atol=1e-4)
    print("\nEUCM+bicubic vs Ceres PhotometricError<8>:", st)


def test_ceres_dropin_matches_vendored_photometric_error_solve():
    """Real Ceres LM with the GPU EvaluationCallback (EUCM + bicubic on the engine) against real Ceres LM over the
    vendored ceres::PhotometricError<8> — a reference-held CPU path end to end: same accept/reject sequence, costs to
    1e-5 relative per iteration, protocol of evaluation_callback_test.cc:79-160 on every call."""
    import ceres_runner as CR
    if not CR.available():
        pytest.skip("oracle/_ref/ceres_lm_driver not built")
    pb, _, _ = load_ceres_photometric()
    threads = int(os.environ.get("OMP_NUM_THREADS", "8"))
    ref = CR.run("cpu", pb, iters=10, huber=9.0, threads=threads)
    got = CR.run("gpu", pb, iters=10, huber=9.0, threads=threads)
    assert got["protocol"]["violations"] == 0, got["protocol"]
    assert len(got["costs"]) == len(ref["costs"]) and np.array_equal(got["step_ok"], ref["step_ok"])
    np.testing.assert_allclose(got["costs"], ref["costs"], rtol=1e-5)
    np.testing.assert_allclose(got["poses"][:, 4:], ref["poses"][:, 4:], atol=1e-5)
    np.testing.assert_allclose(got["rho"], ref["rho"], rtol=1e-4, atol=1e-4 * np.abs(ref["rho"]).max())
