"""The Ceres adapter (include/pba_ceres.h) driven like Ceres' evaluator (tests/cpp/adapter_driver.cpp).

CPU: the adapter compiles against the Ceres 2.0 interface (test double tests/cpp/mock_ceres; against the real
vendored Ceres in tests/test_ceres_reference.py).
GPU: per-block Evaluate through the adapter reproduces the oracle's tangent records after Ceres'
J_global·P step; residual-only evaluations and LocalParameterization::Plus agree too.  The driver is the one linked
against real Ceres 2.0.0 (oracle/_ref/adapter_driver, oracle/ceres.mk) when it was built, else the test-double build.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

import oracle as O
from helpers import R_ATOL_GEOMETRIC, R_ATOL_PHOTOMETRIC, ROOT, compare_records, engine_module, projected_uv, synth

E = engine_module()
DRIVER_SRC = os.path.join(ROOT, "tests", "cpp", "adapter_driver.cpp")
REAL_CERES_DRIVER = os.path.join(ROOT, "oracle", "_ref", "adapter_driver")


def build_driver(out_dir):
    exe = os.path.join(out_dir, "adapter_driver")
    libdir = os.path.dirname(E.LIB_PATH)
    cmd = ["g++", "-std=c++14", "-O2", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "tests", "cpp", "mock_ceres"), DRIVER_SRC, "-o", exe,
           "-L", libdir, "-lpba", f"-Wl,-rpath,{libdir}", "-Wl,--allow-shlib-undefined"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_adapter_compiles_against_ceres_interface():
    E.build()
    with tempfile.TemporaryDirectory() as td:
        assert os.path.exists(build_driver(td))


@pytest.mark.gpu
@pytest.mark.parametrize("pose_param", ["ref", "tangent"])
@pytest.mark.parametrize("kind,model", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_adapter_records_match_oracle(kind, model, pose_param):
    """pose_param "ref": the adapter's 7-wide Jacobians J6·P⁺ composed with the reference LocalParameterizationSE3's
    Jacobian (Sophus Dx_this_mul_exp_x_at_0) give back the oracle's tangent records; "tangent": [J6 | 0] with
    SE3TangentParameterization's [I₆; 0]."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import write_problem
    pb = synth.make_problem(kind=kind, model=model, n_frames=8, n_points=100, width=376, height=240, seed=61,
                            border=10)
    with tempfile.TemporaryDirectory() as td:
        exe = REAL_CERES_DRIVER if os.access(REAL_CERES_DRIVER, os.X_OK) else build_driver(td)
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as f:
            write_problem(f, pb)
        subprocess.run([exe, fin, fout, pose_param], check=True)
        raw = np.fromfile(fout, np.uint8)
    R, nb = pb.R, pb.n_blocks
    o = 0
    rec = raw[o:o + 8 * nb * 14 * R].view(np.float64).reshape(nb, 14 * R); o += 8 * nb * 14 * R
    valid = raw[o:o + nb]; o += nb
    ronly = raw[o:o + 8 * nb * R].view(np.float64).reshape(nb, R); o += 8 * nb * R
    valid_r = raw[o:o + nb]; o += nb
    plus = raw[o:o + 56].view(np.float64); o += 56
    P0 = raw[o:o + 8 * 42].view(np.float64).reshape(7, 6)
    if pose_param == "ref":  # the adapter's restated Sophus plus-Jacobian against the oracle's (pinned by Sophus)
        np.testing.assert_allclose(P0, O.se3_plus_jacobian(pb.poses[0]).reshape(7, 6), atol=1e-15)
    ref, vref = O.evaluate(pb)
    compare_records(kind, R, rec.astype(np.float32), ref, valid, vref, projected_uv(pb) if kind == 0 else None)
    assert np.array_equal(valid_r, vref)
    np.testing.assert_allclose(ronly[vref == 1], ref[vref == 1, :R], atol=R_ATOL_PHOTOMETRIC if kind == 0 else R_ATOL_GEOMETRIC)
    delta = np.array([0.01, -0.02, 0.03, 0.004, -0.005, 0.006])
    np.testing.assert_allclose(plus, O.se3_plus(pb.poses[0], delta), atol=1e-14)
