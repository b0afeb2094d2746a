"""Problem loader from the reference's files: map.cereal + opt_calib.json → SoA problem.

Fixture: tests/golden/map_small/ written by oracle/map_writer.cpp with the reference's vendored cereal library
(tests/golden/make_map_fixture.sh), together with expect.bin — the problem bundle_adjustment() would build
(map_utils.h:322-375) in the loader's order.  The EuRoC double-sphere calibration file is the reference's own
data/euroc_calib/calibration-double-sphere.json (LoadCalibration form).

CPU: the loader (host-only C++ in libpba.so) reproduces expect.bin bit for bit, rejects truncated/corrupt input.
GPU: the loaded stereo map runs through the geometric engine — Ceres-mode records against the oracle, an LM
solve that lowers the cost, and the outlier pass (pba_compute_projections + pba_outlier_landmarks).
"""
import os

import numpy as np
import pytest

import oracle as O
from helpers import GOLDEN, compare_records, engine_module

E = engine_module()
MAP_DIR = os.path.join(GOLDEN, "map_small")
MAP, CALIB = os.path.join(MAP_DIR, "map.cereal"), os.path.join(MAP_DIR, "opt_calib.json")


def read_expect():
    raw = open(os.path.join(MAP_DIR, "expect.bin"), "rb").read()
    off, out = 0, []
    for dt in (np.float64, np.int32, np.float64, np.int64, np.int32, np.float64, np.float64, np.int32, np.int32,
               np.float64, np.int32, np.int32, np.float64):
        n = int(np.frombuffer(raw, np.uint64, 1, off)[0])
        off += 8
        a = np.frombuffer(raw, dt, n, off)
        off += n * np.dtype(dt).itemsize
        out.append(a)
    keys = ("intr", "frame_cam", "poses", "track_id", "host", "u_ref", "rho", "bp", "bt", "u_obs", "op", "of", "ouv")
    return dict(zip(keys, out))


def test_map_loader_matches_bundle_adjustment_build():
    pb, ex = E.load_map(MAP, CALIB)
    x = read_expect()
    assert pb.model == 1 and pb.width == 752 and pb.height == 480  # "ds"
    assert np.array_equal(pb.intrinsics.ravel(), x["intr"])
    assert np.array_equal(pb.frame_cam, x["frame_cam"])
    assert np.array_equal(pb.poses.ravel(), x["poses"])
    assert np.array_equal(ex["track_id"], x["track_id"])
    assert np.array_equal(pb.point_host, x["host"])
    assert np.array_equal(pb.u_ref.ravel(), x["u_ref"])
    assert np.array_equal(pb.rho, x["rho"])
    assert np.array_equal(pb.block_point, x["bp"]) and np.array_equal(pb.block_target, x["bt"])
    assert np.array_equal(pb.u_obs.ravel(), x["u_obs"])
    assert np.array_equal(ex["outlier_point"], x["op"]) and np.array_equal(ex["outlier_frame"], x["of"])
    assert np.array_equal(ex["outlier_uv"].ravel(), x["ouv"])
    # anchor = smallest observing FrameCamId: every block targets a later frame index than its host
    assert (pb.block_target > pb.point_host[pb.block_point]).all()
    assert np.allclose(ex["T_i_c"][1, 4:], [0.11, 0.0, 0.0])
    assert sorted(set(ex["frame_id"].tolist())) == list(range(10))


def test_euroc_double_sphere_calibration_form():
    """The reference's own EuRoC calibration (LoadCalibration<DoubleSphereCamera>: fx fy cx cy xi alpha)."""
    pb, _ = E.load_map(MAP, os.path.join(MAP_DIR, "euroc_calibration-double-sphere.json"))
    assert pb.model == 1
    assert np.allclose(pb.intrinsics[0, :6], [370.3418125824944, 370.3418125824944, 375.5, 239.5, 0.0, 0.5])
    assert np.allclose(pb.intrinsics[1, :4], [361.91730176280108, 361.91730176280108, 375.5, 239.5])


def test_map_loader_rejects_bad_input(tmp_path):
    raw = open(MAP, "rb").read()
    bad = tmp_path / "trunc.cereal"
    bad.write_bytes(raw[: len(raw) // 2])
    with pytest.raises(E.PbaError):
        E.load_map(str(bad), CALIB)
    with pytest.raises(E.PbaError):
        E.load_map(str(tmp_path / "missing.cereal"), CALIB)
    js = tmp_path / "calib.json"
    js.write_text(open(CALIB).read().replace('"ds"', '"fov"'))
    with pytest.raises(E.PbaError):
        E.load_map(MAP, str(js))
    js.write_text("{ not json")
    with pytest.raises(E.PbaError):
        E.load_map(MAP, str(js))


@pytest.mark.gpu
def test_loaded_map_evaluates_and_solves():
    pb, ex = E.load_map(MAP, CALIB)
    with E.Engine(pb.kind, pb.model, huber_width=1.0) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        eng.evaluate(True)
        rec, valid = eng.records()
        ref, vref = O.evaluate(pb)
        compare_records(pb.kind, 2, rec, ref, valid, vref)
        # bundle_adjustment: first camera pair fixed (map_utils.h:334-336 — fixed_cameras {0,0}, {0,1})
        eng.set_fixed_frames(np.array([0, 1], np.int32))
        s = eng.solve(max_iterations=20)
        assert s["final_cost"] < s["initial_cost"]
        poses, rho = eng.get_state()
        n = pb.n_points
        op = np.concatenate([np.arange(n, dtype=np.int32), pb.block_point, ex["outlier_point"]])
        of = np.concatenate([pb.point_host, pb.block_target, ex["outlier_frame"]])
        uv = np.concatenate([pb.u_ref, pb.u_obs, ex["outlier_uv"]])
        oo = np.concatenate([np.zeros(n + pb.n_blocks, np.uint8), np.ones(len(ex["outlier_point"]), np.uint8)])
        got = eng.compute_projections(op, of, uv, oo)
    refp = O.compute_projections(pb, poses, rho, op, of, uv, oo)
    assert np.abs(got["reprojected"] - refp["reprojected"]).max() <= 1e-8
    rm, c = E.outlier_landmarks(n, op, of, got["flags"], oo)
    rm_ref, c_ref = O.outlier_landmarks(n, op, of, refp["flags"], oo)
    assert np.array_equal(rm, rm_ref) and c == c_ref
    assert c["huge"] + c["normal"] > 0  # the fixture corrupts ~3% of the corners by ~25 px
