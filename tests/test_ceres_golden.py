"""CPU: the oracle's bicubic interpolator and photometric functor against golden vectors written by the reference's
vendored Ceres 2.0.0 itself (tests/golden/make_ceres_golden.py → oracle/_ref/golden_ceres):
BiCubicInterpolator<Grid2D<uint8_t,1>> (cubic_interpolation.h:252-344, edge clamp :403-414) and PhotometricError<8>
(photometric_error.h:79-189) through AutoDiffCostFunction with LocalParameterizationSE3 tangent Jacobians.  Both sides
are fp64: agreement to 1e-10 relative (Ceres' Jet arithmetic vs the oracle's dual numbers differ only in rounding)."""
import os

import numpy as np

import oracle as O
from helpers import GOLDEN, synth


def test_oracle_bicubic_matches_ceres_interpolator():
    z = np.load(os.path.join(GOLDEN, "ceres_bicubic.npz"))
    for img, uv, ref in ((z["crop"], z["uv_rand"], z["out_rand"]), (z["grid"], z["uv_grid"], z["out_grid"]),
                         (z["quad"], z["uv_quad"], z["out_quad"])):
        got = O.sample(img, uv, interp=1)  # [f, ∂/∂u, ∂/∂v]
        np.testing.assert_allclose(got[:, 0], ref[:, 0], atol=1e-10)
        np.testing.assert_allclose(got[:, 1], ref[:, 2], atol=1e-10)  # dfdc
        np.testing.assert_allclose(got[:, 2], ref[:, 1], atol=1e-10)  # dfdr
    # cubic_interpolation_test.cc:114-149 (Grid2D out of bounds) and :331-367 (quadratics reproduced exactly)
    np.testing.assert_array_equal(z["out_grid"][:, 0], z["expect_grid"])
    uv = z["uv_quad"]
    r, c = uv[:, 1], uv[:, 0]
    np.testing.assert_allclose(z["out_quad"][:, 0], r * r + r * c + c + 3, atol=1e-9)
    np.testing.assert_allclose(z["out_quad"][:, 1], 2 * r + c, atol=1e-9)
    np.testing.assert_allclose(z["out_quad"][:, 2], r + 1, atol=1e-9)


def load_ceres_photometric():
    z = np.load(os.path.join(GOLDEN, "ceres_photometric_eucm.npz"))
    pb = synth.Problem(kind=int(z["kind"]), model=int(z["model"]), width=int(z["width"]), height=int(z["height"]),
                       intrinsics=z["intrinsics"], frame_cam=z["frame_cam"], images=z["images"], pattern=z["pattern"],
                       point_host=z["point_host"], u_ref=z["u_ref"], host_intensity=z["host_intensity"],
                       block_point=z["block_point"], block_target=z["block_target"], u_obs=None, poses=z["poses"],
                       rho=z["rho"], interp=int(z["interp"]))
    return pb, z["records"], z["valid"]


def test_oracle_matches_ceres_photometric_error():
    pb, ref, vref = load_ceres_photometric()
    assert pb.model == synth.EUCM and pb.interp == 1 and vref.all()
    out, valid = O.evaluate(pb)
    assert np.array_equal(valid, vref)
    # per block, relative to the block's largest record value
    scale = np.maximum(np.abs(ref).max(1, keepdims=True), 1.0)
    rel = (np.abs(out - ref) / scale).max()
    assert rel <= 1e-10, rel
