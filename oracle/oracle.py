"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker
(never as the thing measured or shipped).  See oracle.cpp for what it restates (file:line).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OrcProblem(C.Structure):
    _fields_ = [("kind", C.c_int32), ("model", C.c_int32), ("n_frames", C.c_int32), ("n_points", C.c_int32),
                ("n_blocks", C.c_int32), ("n_cams", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
                ("P", C.c_int32), ("interp", C.c_int32),
                ("intrinsics", C.c_void_p), ("frame_cam", C.c_void_p), ("images", C.c_void_p),
                ("pattern", C.c_void_p), ("point_host", C.c_void_p), ("u_ref", C.c_void_p),
                ("host_intensity", C.c_void_p), ("block_point", C.c_void_p), ("block_target", C.c_void_p),
                ("u_obs", C.c_void_p)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        src = os.path.join(_HERE, "oracle.cpp")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            build()
        L = C.CDLL(path)
        L.orc_evaluate.argtypes = [C.POINTER(OrcProblem), C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_evaluate.restype = C.c_int
        L.orc_evaluate_intrinsics.argtypes = [C.POINTER(OrcProblem), C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                              C.c_void_p, C.c_void_p]
        L.orc_evaluate_intrinsics.restype = C.c_int
        L.orc_huber_block.argtypes = [C.c_void_p, C.c_int, C.c_double, C.POINTER(C.c_double)]
        L.orc_huber_block.restype = C.c_double
        for name, n in [("orc_se3_exp", 2), ("orc_se3_mul", 3), ("orc_se3_plus", 3), ("orc_se3_plus_jacobian", 2),
                        ("orc_se3_act", 3), ("orc_se3_inverse", 2)]:
            getattr(L, name).argtypes = [C.c_void_p] * n
            getattr(L, name).restype = None
        L.orc_project.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_unproject.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_in_domain.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
        L.orc_in_domain.restype = C.c_int
        L.orc_bilinear.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_void_p]
        L.orc_sample.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_void_p]
        L.orc_compute_projections.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_int] + [C.c_void_p] * 9
        L.orc_compute_projections.restype = C.c_int
        L.orc_outlier_landmarks.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 6
        L.orc_outlier_landmarks.restype = C.c_int
        _LIB = L
    return _LIB


def _ptr(a):
    return None if a is None else a.ctypes.data


class _Keep:
    """Holds contiguous copies alive for the duration of a call."""

    def __init__(self):
        self.refs = []

    def __call__(self, a, dtype):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=dtype)
        self.refs.append(a)
        return a


def make_problem_struct(pb, keep: _Keep) -> OrcProblem:
    s = OrcProblem()
    s.kind, s.model = pb.kind, pb.model
    s.n_frames, s.n_points, s.n_blocks = pb.n_frames, pb.n_points, pb.n_blocks
    s.n_cams = pb.intrinsics.shape[0]
    s.width, s.height = pb.width, pb.height
    s.P = pb.pattern.shape[0] if pb.kind == 0 else 2
    s.interp = int(getattr(pb, "interp", 0))
    s.intrinsics = _ptr(keep(pb.intrinsics, np.float64))
    s.frame_cam = _ptr(keep(pb.frame_cam, np.int32))
    s.images = _ptr(keep(pb.images, np.uint8))
    s.pattern = _ptr(keep(pb.pattern, np.float32))
    s.point_host = _ptr(keep(pb.point_host, np.int32))
    s.u_ref = _ptr(keep(pb.u_ref, np.float64))
    s.host_intensity = _ptr(keep(pb.host_intensity, np.float32))
    s.block_point = _ptr(keep(pb.block_point, np.int32))
    s.block_target = _ptr(keep(pb.block_target, np.int32))
    s.u_obs = _ptr(keep(pb.u_obs, np.float64))
    return s


def evaluate(pb, poses=None, rho=None, want_jac: bool = True, n_threads: int = 1, block_slice=None):
    """Returns (records (n_blocks, 14R) float64, valid (n_blocks,) uint8)."""
    L = lib()
    keep = _Keep()
    if block_slice is not None:
        import copy
        pb = copy.copy(pb)
        pb.block_point = pb.block_point[block_slice]
        pb.block_target = pb.block_target[block_slice]
        if pb.u_obs is not None:
            pb.u_obs = pb.u_obs[block_slice]
    s = make_problem_struct(pb, keep)
    poses = keep(pb.poses if poses is None else poses, np.float64)
    rho = keep(pb.rho if rho is None else rho, np.float64)
    R = s.P if pb.kind == 0 else 2
    out = np.zeros((pb.n_blocks, 14 * R), np.float64)
    valid = np.zeros(pb.n_blocks, np.uint8)
    rc = L.orc_evaluate(C.byref(s), _ptr(poses), _ptr(rho), int(bool(want_jac)), _ptr(out), _ptr(valid), int(n_threads))
    if rc != 0:
        raise RuntimeError(f"orc_evaluate failed ({rc})")
    return out, valid


def evaluate_intrinsics(pb, intr_state, poses=None, rho=None, want_jac: bool = True):
    """Geometric blocks with the target intrinsics as a parameter block (optimize_intrinsics): (records (n_blocks, 44)
    float64 = [r | J_host | J_target | J_rho | J_intr (2×8)], valid).  Projection with intr_state (n_cams × 8), host
    unprojection with pb.intrinsics."""
    L = lib()
    keep = _Keep()
    s = make_problem_struct(pb, keep)
    poses = keep(pb.poses if poses is None else poses, np.float64)
    rho = keep(pb.rho if rho is None else rho, np.float64)
    ks = keep(intr_state, np.float64)
    out = np.zeros((pb.n_blocks, 44), np.float64)
    valid = np.zeros(pb.n_blocks, np.uint8)
    rc = L.orc_evaluate_intrinsics(C.byref(s), _ptr(poses), _ptr(rho), _ptr(ks), int(bool(want_jac)), _ptr(out),
                                   _ptr(valid))
    if rc != 0:
        raise RuntimeError(f"orc_evaluate_intrinsics failed ({rc})")
    return out, valid


def sample(img: np.ndarray, uv: np.ndarray, interp: int = 0) -> np.ndarray:
    """The oracle's interpolator (0 bilinear, 1 Ceres' bicubic) of a u8 image at (column, row) positions:
    (n, 3) float64 [I, ∂I/∂u, ∂I/∂v]."""
    L = lib()
    img = np.ascontiguousarray(img, np.uint8)
    uv = np.asarray(uv, np.float64).reshape(-1, 2)
    out = np.zeros((uv.shape[0], 3))
    f3 = np.zeros(3)
    for i, (u, v) in enumerate(uv):
        L.orc_sample(int(interp), _ptr(img), img.shape[1], img.shape[0], float(u), float(v), _ptr(f3))
        out[i] = f3
    return out


def split_record(out: np.ndarray, R: int):
    """(r, J_host, J_target, J_rho) views of a record array."""
    n = out.shape[0]
    r = out[:, :R]
    Jh = out[:, R:7 * R].reshape(n, R, 6)
    Jt = out[:, 7 * R:13 * R].reshape(n, R, 6)
    Jr = out[:, 13 * R:14 * R]
    return r, Jh, Jt, Jr


def huber_block(r: np.ndarray, a: float):
    L = lib()
    r = np.ascontiguousarray(r, np.float64)
    sc = C.c_double()
    cost = L.orc_huber_block(_ptr(r), r.shape[0], a, C.byref(sc))
    return cost, sc.value


def _call(name, outn, *arrs):
    L = lib()
    arrs = [np.ascontiguousarray(a, np.float64) for a in arrs]
    out = np.zeros(outn)
    getattr(L, name)(*[_ptr(a) for a in arrs], _ptr(out))
    return out


def se3_exp(d):
    return _call("orc_se3_exp", 7, d)


def se3_mul(a, b):
    return _call("orc_se3_mul", 7, a, b)


def se3_plus(T, d):
    return _call("orc_se3_plus", 7, T, d)


def se3_plus_jacobian(T):
    return _call("orc_se3_plus_jacobian", 42, T).reshape(7, 6)


def se3_act(T, p):
    return _call("orc_se3_act", 3, T, p)


def se3_inverse(T):
    return _call("orc_se3_inverse", 7, T)


def compute_projections(pb, poses, rho, obs_point, obs_frame, obs_uv, obs_is_outlier=None,
                        thresholds=(3.0, 40.0, 0.1, 0.05)) -> dict:
    """compute_projections + set_outlier_flags (src/sfm.cpp:1928-2008) in double, per observation."""
    k = np.ascontiguousarray(pb.intrinsics, np.float64)
    fc = np.ascontiguousarray(pb.frame_cam, np.int32)
    P = np.ascontiguousarray(poses, np.float64)
    ph = np.ascontiguousarray(pb.point_host, np.int32)
    ur = np.ascontiguousarray(pb.u_ref, np.float64)
    rh = np.ascontiguousarray(rho, np.float64)
    op = np.ascontiguousarray(obs_point, np.int32)
    of = np.ascontiguousarray(obs_frame, np.int32)
    uv = np.ascontiguousarray(obs_uv, np.float64)
    oo = None if obs_is_outlier is None else np.ascontiguousarray(obs_is_outlier, np.uint8)
    th = np.ascontiguousarray(thresholds, np.float64)
    n = op.shape[0]
    out = {"reprojected": np.zeros((n, 2)), "point_c": np.zeros((n, 3)), "error": np.zeros(n),
           "flags": np.zeros(n, np.uint32)}
    lib().orc_compute_projections(pb.model, _ptr(k), _ptr(fc), _ptr(P), _ptr(ph), _ptr(ur), _ptr(rh), n, _ptr(op),
                                  _ptr(of), _ptr(uv), _ptr(oo), _ptr(th), _ptr(out["reprojected"]),
                                  _ptr(out["point_c"]), _ptr(out["error"]), _ptr(out["flags"]))
    return out


def outlier_landmarks(n_points, obs_point, obs_frame, flags, obs_is_outlier=None):
    """remove_outlier_landmarks (src/sfm.cpp:2028-2114) over map<track, map<frame, flags>>."""
    op = np.ascontiguousarray(obs_point, np.int32)
    of = np.ascontiguousarray(obs_frame, np.int32)
    fl = np.ascontiguousarray(flags, np.uint32)
    oo = None if obs_is_outlier is None else np.ascontiguousarray(obs_is_outlier, np.uint8)
    rm = np.zeros(n_points, np.uint8)
    counts = np.zeros(5, np.int32)
    lib().orc_outlier_landmarks(n_points, op.shape[0], _ptr(op), _ptr(of), _ptr(fl), _ptr(oo), _ptr(rm), _ptr(counts))
    return rm.astype(bool), dict(zip(("huge", "normal", "camera_distance", "z", "any_severe"), counts.tolist()))
