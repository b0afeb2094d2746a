"""Python binding of the C ABI in include/pba.h (ctypes over csrc/libpba.so).

This is the host-side mirror used by the tests and bench; the C++ Ceres-style adapter for the reference's
own code lives in include/pba_ceres.h.  There is no CPU fallback: if libpba.so is
missing or the device call fails, every method raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_PATH = os.environ.get("PBA_LIBRARY") or os.path.join(CSRC, "libpba.so")  # override: A/B builds (tools/)
# the library's test build (PBA_TEST_HOOKS: forced decision mismatch, host delay, λ-specific path, 14-column A/B
# lineariser — pba_internal.h test_hook); only the GPU tests that need those hooks load it (Engine(library=…))
TEST_LIB_PATH = os.path.join(CSRC, "libpba_test.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "pba.h")

PBA_OK = 0
_LIBS = {}


class Options(C.Structure):
    _fields_ = [("device", C.c_int32), ("residual_kind", C.c_int32), ("camera_model", C.c_int32),
                ("huber_width", C.c_float)]


class OutlierThresholds(C.Structure):
    """pba_outlier_thresholds (defaults: src/sfm.cpp:254-261)."""
    _fields_ = [("reprojection_error_normal_px", C.c_double), ("reprojection_error_huge_px", C.c_double),
                ("camera_center_distance_m", C.c_double), ("z_coordinate_m", C.c_double)]


OUTLIER_HUGE, OUTLIER_NORMAL, OUTLIER_DISTANCE, OUTLIER_Z = 1, 2, 4, 8
RECORD_F32, RECORD_F16 = 0, 1
INTERP_BILINEAR, INTERP_BICUBIC = 0, 1  # pba_set_interpolator


class MapInfo(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("n_points", C.c_int32), ("n_blocks", C.c_int32), ("n_cams", C.c_int32),
                ("camera_model", C.c_int32), ("n_outlier_obs", C.c_int32), ("width", C.c_int32), ("height", C.c_int32)]


class SolverOptions(C.Structure):
    """pba_solver_options (Ceres' Solver::Options defaults, solver.h:278-322)."""
    _fields_ = [("max_iterations", C.c_int32), ("max_num_consecutive_invalid_steps", C.c_int32),
                ("initial_trust_region_radius", C.c_double), ("function_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double), ("min_relative_decrease", C.c_double),
                ("gradient_tolerance", C.c_double), ("max_trust_region_radius", C.c_double),
                ("min_trust_region_radius", C.c_double)]


def solver_options(max_iterations=20, initial_trust_region_radius=1e4, function_tolerance=1e-6,
                   min_relative_decrease=1e-3, parameter_tolerance=1e-8, gradient_tolerance=1e-10,
                   max_trust_region_radius=1e16, min_trust_region_radius=1e-32, max_num_consecutive_invalid_steps=5):
    return SolverOptions(max_iterations, max_num_consecutive_invalid_steps, initial_trust_region_radius,
                         function_tolerance, parameter_tolerance, min_relative_decrease, gradient_tolerance,
                         max_trust_region_radius, min_trust_region_radius)


TERMINATION_CONVERGENCE, TERMINATION_MAX_ITERATIONS, TERMINATION_FAILURE = 0, 1, 2
STOP_REASONS = ("max_iterations", "function_tolerance", "parameter_tolerance", "gradient_tolerance",
                "min_trust_region_radius", "invalid_steps")


class SolverSummary(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("successful_steps", C.c_int32), ("unsuccessful_steps", C.c_int32),
                ("termination", C.c_int32), ("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("total_ms", C.c_double), ("linearize_ms", C.c_double), ("solve_ms", C.c_double),
                ("cost_ms", C.c_double), ("gradient_max_norm", C.c_double), ("stop_reason_code", C.c_int32),
                ("pad_", C.c_int32)]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_ if f != "pad_"}
        d["stop_reason"] = STOP_REASONS[self.stop_reason_code]
        return d


class IterationSummary(C.Structure):
    """pba_iteration_summary (Ceres' IterationSummary fields, iteration_callback.h)."""
    _fields_ = [("iteration", C.c_int32), ("step_is_successful", C.c_int32), ("step_is_valid", C.c_int32),
                ("pad_", C.c_int32), ("cost", C.c_double), ("cost_change", C.c_double),
                ("relative_decrease", C.c_double), ("trust_region_radius", C.c_double), ("step_norm", C.c_double),
                ("gradient_max_norm", C.c_double)]


# int (*pba_allreduce_fn)(void* user, double* d_buf, int64_t count)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64)


def build(force: bool = False) -> str:
    """Compile csrc/libpba.so for gfx950 with hipcc (in-tree)."""
    args = ["make", "-s", "-j", str(min(8, os.cpu_count() or 1)), "-C", CSRC]
    if force:
        args.append("-B")
    subprocess.run(args + ["libpba.so"], check=True)
    return LIB_PATH


def header_functions() -> list[str]:
    """Every function declared in include/pba.h."""
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|void)\s+(pba_\w+)\s*\(", src, re.M)))


def lib(path: Optional[str] = None):
    """The engine library at `path` (default LIB_PATH: csrc/libpba.so), loaded once per path."""
    path = path or LIB_PATH
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise RuntimeError(f"HIP engine library missing: {path} (run __graft_entry__.build())")
    # torch bundles its own HIP runtime under the same soname: load it first so the engine binds to that one.
    # Loaded the other way round (engine first), torch's runtime later finds no devices in this process.
    try:
        import torch  # noqa: F401  (loads libraries only; no GPU initialisation)
    except ImportError:
        pass
    L = C.CDLL(path)
    vp, i32 = C.c_void_p, C.c_int32
    sig = {
        "pba_create": ([C.POINTER(Options), C.POINTER(vp)], C.c_int),
        "pba_destroy": ([vp], C.c_int),
        "pba_status_string": ([C.c_int], C.c_char_p),
        "pba_last_error": ([], C.c_char_p),
        "pba_version": ([], C.c_int),
        "pba_set_cameras": ([vp, i32, vp], C.c_int),
        "pba_set_frames": ([vp, i32, vp, i32, i32, vp], C.c_int),
        "pba_set_frames_device": ([vp, i32, vp, i32, i32, vp], C.c_int),
        "pba_set_pattern": ([vp, i32, vp], C.c_int),
        "pba_set_points": ([vp, i32, vp, vp, vp], C.c_int),
        "pba_set_blocks": ([vp, i32, vp, vp, vp], C.c_int),
        "pba_set_state": ([vp, vp, vp], C.c_int),
        "pba_set_state_device": ([vp, vp, vp], C.c_int),
        "pba_evaluate": ([vp, i32], C.c_int),
        "pba_evaluate_state_device": ([vp, vp, vp, i32], C.c_int),
        "pba_evaluate_states_device": ([vp, i32, vp, vp, i32], C.c_int),
        "pba_synchronize": ([vp], C.c_int),
        "pba_record_floats": ([vp], C.c_int),
        "pba_residuals_per_block": ([vp], C.c_int),
        "pba_num_blocks": ([vp], C.c_int),
        "pba_num_points": ([vp], C.c_int),
        "pba_num_frames": ([vp], C.c_int),
        "pba_get_records": ([vp, vp, vp], C.c_int),
        "pba_get_block_costs": ([vp, vp], C.c_int),
        "pba_get_residuals": ([vp, vp, vp], C.c_int),
        "pba_host_alloc": ([C.c_size_t, C.POINTER(vp)], C.c_int),
        "pba_host_free": ([vp], C.c_int),
        "pba_set_interpolator": ([vp, i32], C.c_int),
        "pba_set_solver_timing": ([vp, i32], C.c_int),
        "pba_solver_iterations": ([vp, i32, vp, C.POINTER(i32)], C.c_int),
        "pba_interpolator": ([vp], C.c_int),
        "pba_sample_image": ([vp, i32, i32, vp, vp], C.c_int),
        "pba_get_cost": ([vp, C.POINTER(C.c_double), C.POINTER(i32)], C.c_int),
        "pba_set_stream": ([vp, vp], C.c_int),
        "pba_get_stream": ([vp, C.POINTER(vp)], C.c_int),
        "pba_device_records": ([vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)], C.c_int),
        "pba_enable_kernel_timing": ([vp, i32], C.c_int),
        "pba_get_kernel_timing": ([vp, C.POINTER(C.c_double), C.POINTER(i32)], C.c_int),
        "pba_set_fixed_frames": ([vp, i32, vp], C.c_int),
        "pba_gn_linearize": ([vp, C.POINTER(C.c_double)], C.c_int),
        "pba_gn_step": ([vp, C.c_double, C.POINTER(C.c_double), C.POINTER(i32)], C.c_int),
        "pba_gn_candidate_cost": ([vp, C.POINTER(C.c_double)], C.c_int),
        "pba_gn_accept": ([vp], C.c_int),
        "pba_solve": ([vp, C.POINTER(SolverOptions), C.POINTER(SolverSummary)], C.c_int),
        "pba_get_state": ([vp, vp, vp], C.c_int),
        "pba_gn_get_reduced_system": ([vp, vp, vp], C.c_int),
        "pba_gn_get_step": ([vp, vp, vp], C.c_int),
        "pba_gn_band": ([vp, C.POINTER(i32)], C.c_int),
        "pba_gn_exchange_size": ([vp, i32, C.POINTER(C.c_int64)], C.c_int),
        "pba_gn_step_export": ([vp, C.c_double, i32, vp], C.c_int),
        "pba_gn_step_import": ([vp, C.c_double, i32, vp, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                C.POINTER(i32)], C.c_int),
        "pba_solve_distributed": ([vp, C.POINTER(SolverOptions), i32, vp, ALLREDUCE_FN, vp,
                                   C.POINTER(SolverSummary)], C.c_int),
        "pba_solve_distributed_comm": ([vp, C.POINTER(SolverOptions), i32, vp, C.POINTER(SolverSummary)], C.c_int),
        "pba_comm_unique_id": ([vp], C.c_int),
        "pba_comm_init": ([vp, i32, i32, i32, C.POINTER(vp)], C.c_int),
        "pba_comm_init_local": ([i32, i32, vp], C.c_int),
        "pba_comm_destroy": ([vp], C.c_int),
        "pba_comm_rank": ([vp], C.c_int),
        "pba_comm_size": ([vp], C.c_int),
        "pba_comm_allreduce": ([vp, vp, C.c_int64, vp], C.c_int),
        "pba_set_optimize_intrinsics": ([vp, i32], C.c_int),
        "pba_set_intrinsics_state": ([vp, vp], C.c_int),
        "pba_get_intrinsics": ([vp, vp], C.c_int),
        "pba_gn_system_size": ([vp, C.POINTER(i32)], C.c_int),
        "pba_gn_set_rank": ([vp, i32], C.c_int),
        "pba_compute_projections": ([vp, i32, vp, vp, vp, vp, C.POINTER(OutlierThresholds), vp, vp, vp, vp], C.c_int),
        "pba_outlier_landmarks": ([i32, i32, vp, vp, vp, vp, vp, vp], C.c_int),
        "pba_set_record_format": ([vp, i32], C.c_int),
        "pba_record_format": ([vp], C.c_int),
        "pba_build_pyramid": ([vp, i32], C.c_int),
        "pba_num_levels": ([vp], C.c_int),
        "pba_set_level": ([vp, i32], C.c_int),
        "pba_get_level": ([vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "pba_get_host_intensities": ([vp, vp], C.c_int),
        "pba_solve_pyramid": ([vp, C.POINTER(SolverOptions), C.POINTER(SolverSummary)], C.c_int),
        "pba_map_load": ([C.c_char_p, C.c_char_p, C.POINTER(vp)], C.c_int),
        "pba_map_destroy": ([vp], C.c_int),
        "pba_map_get_info": ([vp, C.POINTER(MapInfo)], C.c_int),
        "pba_map_get_cameras": ([vp, vp, vp], C.c_int),
        "pba_map_get_frames": ([vp, vp, vp, vp], C.c_int),
        "pba_map_get_points": ([vp, vp, vp, vp, vp], C.c_int),
        "pba_map_get_blocks": ([vp, vp, vp, vp], C.c_int),
        "pba_map_get_outlier_obs": ([vp, vp, vp, vp], C.c_int),
    }
    for name, (argt, rest) in sig.items():
        f = getattr(L, name)
        f.argtypes = argt
        f.restype = rest
    _LIBS[path] = L
    return L


class PbaError(RuntimeError):
    pass


def _check(rc: int, what: str, L=None):
    if rc != PBA_OK:
        L = L or lib()
        raise PbaError(f"{what}: {L.pba_status_string(rc).decode()} — {L.pba_last_error().decode()}")


def _p(a: Optional[np.ndarray]):
    return None if a is None else C.c_void_p(a.ctypes.data)


class Engine:
    """One engine = one problem on one GPU (include/pba.h)."""

    def __init__(self, kind: int, model: int, device: int = 0, huber_width: float = 0.0, library: Optional[str] = None):
        L = lib(library)
        self._L = L
        self._h = C.c_void_p()
        opt = Options(device, kind, model, huber_width)
        _check(L.pba_create(C.byref(opt), C.byref(self._h)), "pba_create", L)
        self.kind, self.model = kind, model
        self.n_blocks = self.n_points = self.n_frames = self._n_cams = 0
        self._keep = []

    def _ck(self, rc: int, what: str):
        _check(rc, what, self._L)

    # -- problem -------------------------------------------------------------------------------
    def set_problem(self, pb, images_device_ptr: Optional[int] = None):
        L, h = self._L, self._h
        intr = np.ascontiguousarray(pb.intrinsics, np.float64)
        _check(L.pba_set_cameras(h, intr.shape[0], _p(intr)), "pba_set_cameras", L)
        self._n_cams = intr.shape[0]
        fc = np.ascontiguousarray(pb.frame_cam, np.int32)
        if images_device_ptr is not None:
            _check(L.pba_set_frames_device(h, fc.shape[0], _p(fc), pb.width, pb.height, C.c_void_p(images_device_ptr)),
                   "pba_set_frames_device", L)
        else:
            imgs = None if pb.images is None else np.ascontiguousarray(pb.images, np.uint8)
            _check(L.pba_set_frames(h, fc.shape[0], _p(fc), pb.width, pb.height, _p(imgs)), "pba_set_frames", L)
        if pb.kind == 0:
            pat = np.ascontiguousarray(pb.pattern, np.float32)
            _check(L.pba_set_pattern(h, pat.shape[0], _p(pat)), "pba_set_pattern", L)
            _check(L.pba_set_interpolator(h, int(getattr(pb, "interp", 0))), "pba_set_interpolator", L)
        ph = np.ascontiguousarray(pb.point_host, np.int32)
        ur = np.ascontiguousarray(pb.u_ref, np.float64)
        hi = None if (pb.kind != 0 or pb.host_intensity is None) else np.ascontiguousarray(pb.host_intensity, np.float32)
        _check(L.pba_set_points(h, ph.shape[0], _p(ph), _p(ur), _p(hi)), "pba_set_points", L)
        bp = np.ascontiguousarray(pb.block_point, np.int32)
        bt = np.ascontiguousarray(pb.block_target, np.int32)
        uo = None if pb.u_obs is None else np.ascontiguousarray(pb.u_obs, np.float64)
        _check(L.pba_set_blocks(h, bp.shape[0], _p(bp), _p(bt), _p(uo)), "pba_set_blocks", L)
        self.n_blocks, self.n_points, self.n_frames = bp.shape[0], ph.shape[0], fc.shape[0]
        self.R = L.pba_residuals_per_block(h)
        self.record = L.pba_record_floats(h)

    def set_state(self, poses: np.ndarray, rho: np.ndarray):
        poses = np.ascontiguousarray(poses, np.float64)
        rho = np.ascontiguousarray(rho, np.float64)
        if poses.size != 7 * self.n_frames or rho.size != self.n_points:
            raise ValueError("state shape mismatch")
        self._ck(self._L.pba_set_state(self._h, _p(poses), _p(rho)), "pba_set_state")

    def set_state_device(self, poses_ptr: int, rho_ptr: int):
        self._ck(self._L.pba_set_state_device(self._h, C.c_void_p(poses_ptr), C.c_void_p(rho_ptr)), "pba_set_state_device")

    # -- evaluation ------------------------------------------------------------------------------
    def evaluate(self, want_jacobians: bool = True, sync: bool = True):
        self._ck(self._L.pba_evaluate(self._h, int(bool(want_jacobians))), "pba_evaluate")
        if sync:
            self.synchronize()

    def evaluate_state_device(self, poses_ptr: int, rho_ptr: int, want_jacobians: bool = True, sync: bool = True):
        """Evaluate at a device-resident state and adopt it (Ceres Evaluator::Evaluate(state, …),
        program_evaluator.h:139-258): one launch for photometric engines."""
        self._ck(self._L.pba_evaluate_state_device(self._h, C.c_void_p(poses_ptr), C.c_void_p(rho_ptr),
                                                 int(bool(want_jacobians))), "pba_evaluate_state_device")
        if sync:
            self.synchronize()

    def evaluate_states_device(self, poses_ptrs, rho_ptrs, want_jacobians: bool = True, sync: bool = True):
        """n evaluations back to back, one per (poses, ρ) device-pointer pair, enqueued by one ABI call
        (pba_evaluate_states_device); each adopts its state, the records hold the last one's evaluation."""
        n = len(poses_ptrs)
        if len(rho_ptrs) != n:
            raise ValueError("one ρ array per pose array")
        pa = (C.c_void_p * max(n, 1))(*poses_ptrs)
        ra = (C.c_void_p * max(n, 1))(*rho_ptrs)
        self._ck(self._L.pba_evaluate_states_device(self._h, n, pa, ra, int(bool(want_jacobians))),
               "pba_evaluate_states_device")
        if sync:
            self.synchronize()

    def synchronize(self):
        self._ck(self._L.pba_synchronize(self._h), "pba_synchronize")

    # -- reprojections / outliers (src/sfm.cpp:1928-2008) --------------------------------------------
    def compute_projections(self, obs_point, obs_frame, obs_uv, obs_is_outlier=None, thresholds=None) -> dict:
        """Reprojection of every observation at the current state: dict(reprojected (n,2), point_c (n,3),
        error (n,), flags (n,) uint32)."""
        op = np.ascontiguousarray(obs_point, np.int32)
        of = np.ascontiguousarray(obs_frame, np.int32)
        uv = np.ascontiguousarray(obs_uv, np.float64).reshape(-1, 2)
        n = op.shape[0]
        oo = None if obs_is_outlier is None else np.ascontiguousarray(obs_is_outlier, np.uint8)
        th = None if thresholds is None else C.byref(OutlierThresholds(*thresholds))
        out = {"reprojected": np.zeros((n, 2)), "point_c": np.zeros((n, 3)), "error": np.zeros(n),
               "flags": np.zeros(n, np.uint32)}
        self._ck(self._L.pba_compute_projections(self._h, n, _p(op), _p(of), _p(uv), _p(oo), th, _p(out["reprojected"]),
                                               _p(out["point_c"]), _p(out["error"]), _p(out["flags"])),
               "pba_compute_projections")
        return out

    def set_record_format(self, fmt: int):
        """RECORD_F32 (default) or RECORD_F16 (records stored as IEEE halves; records() still returns floats)."""
        self._ck(self._L.pba_set_record_format(self._h, fmt), "pba_set_record_format")

    def records(self):
        rec = np.empty((self.n_blocks, self.record), np.float32)
        valid = np.empty(self.n_blocks, np.uint8)
        self._ck(self._L.pba_get_records(self._h, _p(rec), _p(valid)), "pba_get_records")
        return rec, valid

    def sample_image(self, frame: int, uv: np.ndarray) -> np.ndarray:
        """The engine's interpolator at (column, row) positions of one frame: (n, 3) float32 [I, ∂I/∂u, ∂I/∂v]."""
        uv = np.ascontiguousarray(uv, np.float64).reshape(-1, 2)
        out = np.empty((uv.shape[0], 3), np.float32)
        self._ck(self._L.pba_sample_image(self._h, frame, uv.shape[0], _p(uv), _p(out)), "pba_sample_image")
        return out

    def residuals(self):
        """Residuals only (after a residual-only evaluation one contiguous copy, else the first R values of every record)
        and the validity flags."""
        r = np.empty((self.n_blocks, self.R), np.float32)
        valid = np.empty(self.n_blocks, np.uint8)
        self._ck(self._L.pba_get_residuals(self._h, _p(r), _p(valid)), "pba_get_residuals")
        return r, valid

    def block_costs(self):
        c = np.empty(self.n_blocks, np.float32)
        self._ck(self._L.pba_get_block_costs(self._h, _p(c)), "pba_get_block_costs")
        return c

    def cost(self):
        tot, nv = C.c_double(), C.c_int32()
        self._ck(self._L.pba_get_cost(self._h, C.byref(tot), C.byref(nv)), "pba_get_cost")
        return tot.value, nv.value

    def stream(self) -> int:
        s = C.c_void_p()
        self._ck(self._L.pba_get_stream(self._h, C.byref(s)), "pba_get_stream")
        return s.value or 0

    def set_stream(self, stream_ptr: int):
        self._ck(self._L.pba_set_stream(self._h, C.c_void_p(stream_ptr)), "pba_set_stream")

    def device_records(self):
        r, v, c = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._ck(self._L.pba_device_records(self._h, C.byref(r), C.byref(v), C.byref(c)), "pba_device_records")
        return r.value, v.value, c.value

    def enable_kernel_timing(self, on: bool = True):
        self._ck(self._L.pba_enable_kernel_timing(self._h, int(on)), "pba_enable_kernel_timing")

    def kernel_timing(self):
        """(summed block-kernel ms, launches) since the last call (HIP events on the engine stream)."""
        ms, n = C.c_double(), C.c_int32()
        self._ck(self._L.pba_get_kernel_timing(self._h, C.byref(ms), C.byref(n)), "pba_get_kernel_timing")
        return ms.value, n.value

    # -- on-device Gauss-Newton / LM ---------------------------------------------------------------
    def set_fixed_frames(self, frames):
        f = np.ascontiguousarray(frames, np.int32)
        self._ck(self._L.pba_set_fixed_frames(self._h, f.shape[0], _p(f) if f.size else None), "pba_set_fixed_frames")

    def gn_linearize(self) -> float:
        c = C.c_double()
        self._ck(self._L.pba_gn_linearize(self._h, C.byref(c)), "pba_gn_linearize")
        return c.value

    def gn_step(self, lam: float):
        m, st = C.c_double(), C.c_int32()
        self._ck(self._L.pba_gn_step(self._h, lam, C.byref(m), C.byref(st)), "pba_gn_step")
        return m.value, st.value

    def gn_candidate_cost(self) -> float:
        c = C.c_double()
        self._ck(self._L.pba_gn_candidate_cost(self._h, C.byref(c)), "pba_gn_candidate_cost")
        return c.value

    def gn_accept(self):
        self._ck(self._L.pba_gn_accept(self._h), "pba_gn_accept")

    def set_solver_timing(self, enable: bool):
        """per-phase device timing of solve() (linearize_ms / solve_ms / cost_ms); off by default"""
        self._ck(self._L.pba_set_solver_timing(self._h, 1 if enable else 0), "pba_set_solver_timing")

    def solver_iterations(self) -> dict:
        """The last solve's trajectory (pba_solver_iterations: Ceres' Solver::Summary::iterations) as arrays."""
        n = C.c_int32()
        self._ck(self._L.pba_solver_iterations(self._h, 0, None, C.byref(n)), "pba_solver_iterations")
        arr = (IterationSummary * max(n.value, 1))()
        self._ck(self._L.pba_solver_iterations(self._h, n.value, arr, C.byref(n)), "pba_solver_iterations")
        rows = arr[:n.value]
        return {f: np.array([getattr(r, f) for r in rows], np.float64 if f not in (
            "iteration", "step_is_successful", "step_is_valid") else np.int64) for f, _ in IterationSummary._fields_
                if f != "pad_"}

    def solve(self, **options) -> dict:
        """pba_solve; options as solver_options() (Ceres' names and defaults, max_iterations 20)."""
        o = solver_options(**options)
        s = SolverSummary()
        self._ck(self._L.pba_solve(self._h, C.byref(o), C.byref(s)), "pba_solve")
        return s.as_dict()

    # -- image pyramid / coarse-to-fine (pba_pyramid.hip) ---------------------------------------------
    def build_pyramid(self, n_levels: int):
        self._ck(self._L.pba_build_pyramid(self._h, n_levels), "pba_build_pyramid")

    def set_level(self, level: int):
        self._ck(self._L.pba_set_level(self._h, level), "pba_set_level")

    def level(self):
        """(active level, its width, its height)"""
        l, w, h = C.c_int32(), C.c_int32(), C.c_int32()
        self._ck(self._L.pba_get_level(self._h, C.byref(l), C.byref(w), C.byref(h)), "pba_get_level")
        return l.value, w.value, h.value

    def host_intensities(self) -> np.ndarray:
        out = np.zeros((self.n_points, self._L.pba_residuals_per_block(self._h)), np.float32)
        self._ck(self._L.pba_get_host_intensities(self._h, _p(out)), "pba_get_host_intensities")
        return out

    def solve_pyramid(self, **options) -> dict:
        o = solver_options(**options)
        s = SolverSummary()
        self._ck(self._L.pba_solve_pyramid(self._h, C.byref(o), C.byref(s)), "pba_solve_pyramid")
        return s.as_dict()

    # -- multi-GPU Gauss-Newton (include/pba.h §8e; host driver in distributed.py) ------------------
    def gn_band(self) -> int:
        b = C.c_int32()
        self._ck(self._L.pba_gn_band(self._h, C.byref(b)), "pba_gn_band")
        return b.value

    def gn_exchange_size(self, band: int) -> int:
        n = C.c_int64()
        self._ck(self._L.pba_gn_exchange_size(self._h, band, C.byref(n)), "pba_gn_exchange_size")
        return n.value

    def gn_step_export(self, lam: float, band: int, exchange_ptr: int):
        self._ck(self._L.pba_gn_step_export(self._h, lam, band, C.c_void_p(exchange_ptr)), "pba_gn_step_export")

    def gn_step_import(self, lam: float, band: int, exchange_ptr: int):
        """(model decrease pose part, this rank's point part, solver status)"""
        mp, mq, st = C.c_double(), C.c_double(), C.c_int32()
        self._ck(self._L.pba_gn_step_import(self._h, lam, band, C.c_void_p(exchange_ptr), C.byref(mp), C.byref(mq),
                                          C.byref(st)), "pba_gn_step_import")
        return mp.value, mq.value, st.value

    def set_rank(self, rank: int):
        """this engine's rank in solve_distributed's host-callback collective (pba_gn_set_rank)"""
        self._ck(self._L.pba_gn_set_rank(self._h, int(rank)), "pba_gn_set_rank")

    def solve_distributed(self, band: int, exchange_ptr: int, allreduce, **options) -> dict:
        """pba_solve_distributed; `allreduce(ptr, count) -> None` sums `count` doubles at device address `ptr`
        over all ranks in place (collective, complete on return)."""
        err = []

        def cb(_user, ptr, count):
            try:
                allreduce(ptr, count)
                return 0
            except BaseException as ex:  # surfaced after the C call returns
                err.append(ex)
                return 1

        fn = ALLREDUCE_FN(cb)
        o = solver_options(**options)
        s = SolverSummary()
        rc = self._L.pba_solve_distributed(self._h, C.byref(o), band, C.c_void_p(exchange_ptr), fn, None, C.byref(s))
        if err:
            raise err[0]
        _check(rc, "pba_solve_distributed")
        return s.as_dict()

    def solve_distributed_comm(self, band: int, comm: "Comm", **options) -> dict:
        """pba_solve_distributed_comm: the collectives are enqueued on the engine stream (RCCL or an in-process
        group), the exchange buffer is the engine's own."""
        o = solver_options(**options)
        s = SolverSummary()
        self._ck(self._L.pba_solve_distributed_comm(self._h, C.byref(o), band, comm.handle, C.byref(s)),
               "pba_solve_distributed_comm")
        return s.as_dict()

    # -- target intrinsics (geometric, optimize_intrinsics) -----------------------------------------
    def set_optimize_intrinsics(self, enable: bool = True):
        self._ck(self._L.pba_set_optimize_intrinsics(self._h, int(bool(enable))), "pba_set_optimize_intrinsics")
        self.record = self._L.pba_record_floats(self._h)

    def set_intrinsics_state(self, intrinsics: np.ndarray):
        k = np.ascontiguousarray(intrinsics, np.float64)
        self._ck(self._L.pba_set_intrinsics_state(self._h, _p(k)), "pba_set_intrinsics_state")

    def get_state(self):
        poses = np.empty((self.n_frames, 7), np.float64)
        rho = np.empty(self.n_points, np.float64)
        self._ck(self._L.pba_get_state(self._h, _p(poses), _p(rho)), "pba_get_state")
        return poses, rho

    def get_intrinsics(self) -> np.ndarray:
        """the intrinsics state (n_cams × 8): the free intrinsics with set_optimize_intrinsics, else the cameras'"""
        k = np.empty((self._n_cams, 8), np.float64)
        self._ck(self._L.pba_get_intrinsics(self._h, _p(k)), "pba_get_intrinsics")
        return k

    def gn_system_size(self) -> int:
        n = C.c_int32()
        self._ck(self._L.pba_gn_system_size(self._h, C.byref(n)), "pba_gn_system_size")
        return n.value

    def gn_reduced_system(self):
        """(S, g) of the reduced camera system over pba_gn_system_size unknowns: 6 per keyframe, then — free intrinsics —
        12 per camera (its 8 intrinsics and 4 identity pads)."""
        n = self.gn_system_size()
        S = np.empty((n, n), np.float64)
        g = np.empty(n, np.float64)
        self._ck(self._L.pba_gn_get_reduced_system(self._h, _p(S), _p(g)), "pba_gn_get_reduced_system")
        return S, g

    def gn_last_step(self):
        dp = np.empty((self.n_frames, 6), np.float64)
        dr = np.empty(self.n_points, np.float64)
        self._ck(self._L.pba_gn_get_step(self._h, _p(dp), _p(dr)), "pba_gn_get_step")
        return dp, dr

    def close(self):
        if self._h:
            self._L.pba_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Comm:
    """pba_comm: an RCCL communicator (one process per GPU) or one rank of an in-process group."""

    def __init__(self, handle: C.c_void_p, library: Optional[str] = None):
        self.handle = handle
        self.library = library

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        _check(lib().pba_comm_unique_id(buf), "pba_comm_unique_id")
        return bytes(buf)

    @classmethod
    def rccl(cls, uid: bytes, n_ranks: int, rank: int, device: int = 0) -> "Comm":
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        _check(lib().pba_comm_init(buf, n_ranks, rank, device, C.byref(h)), "pba_comm_init")
        return cls(h)

    @classmethod
    def local_group(cls, n_ranks: int, device: int = 0, library: Optional[str] = None) -> list:
        """An in-process group of n_ranks (library: the engines' library — a communicator is used by the library that
        made it)."""
        hs = (C.c_void_p * n_ranks)()
        _check(lib(library).pba_comm_init_local(n_ranks, device, hs), "pba_comm_init_local", lib(library))
        return [cls(C.c_void_p(h), library) for h in hs]

    def allreduce(self, ptr: int, count: int, stream: int = 0):
        _check(lib(self.library).pba_comm_allreduce(self.handle, C.c_void_p(ptr), count, C.c_void_p(stream)),
               "pba_comm_allreduce", lib(self.library))

    @property
    def rank(self) -> int:
        return lib(self.library).pba_comm_rank(self.handle)

    @property
    def size(self) -> int:
        return lib(self.library).pba_comm_size(self.handle)

    def close(self):
        if self.handle:
            lib(self.library).pba_comm_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_map(map_path: str, calib_path: str):
    """map.cereal + opt_calib.json → (synth.Problem (geometric), extras dict) through pba_map_load (host-only C++)."""
    import importlib
    synth = importlib.import_module(__package__ + ".synth")
    L = lib()
    h = C.c_void_p()
    _check(L.pba_map_load(map_path.encode(), calib_path.encode(), C.byref(h)), "pba_map_load", L)
    try:
        info = MapInfo()
        _check(L.pba_map_get_info(h, C.byref(info)), "pba_map_get_info", L)
        nf, npt, nb, nc, no = info.n_frames, info.n_points, info.n_blocks, info.n_cams, info.n_outlier_obs
        intr, tic = np.zeros((nc, 8)), np.zeros((nc, 7))
        fid, fcam, poses = np.zeros(nf, np.int64), np.zeros(nf, np.int32), np.zeros((nf, 7))
        tid, host, uref, rho = np.zeros(npt, np.int64), np.zeros(npt, np.int32), np.zeros((npt, 2)), np.zeros(npt)
        bp, bt, uobs = np.zeros(nb, np.int32), np.zeros(nb, np.int32), np.zeros((nb, 2))
        op, of, ouv = np.zeros(no, np.int32), np.zeros(no, np.int32), np.zeros((no, 2))
        _check(L.pba_map_get_cameras(h, _p(intr), _p(tic)), "pba_map_get_cameras", L)
        _check(L.pba_map_get_frames(h, _p(fid), _p(fcam), _p(poses)), "pba_map_get_frames", L)
        _check(L.pba_map_get_points(h, _p(tid), _p(host), _p(uref), _p(rho)), "pba_map_get_points", L)
        _check(L.pba_map_get_blocks(h, _p(bp), _p(bt), _p(uobs)), "pba_map_get_blocks", L)
        _check(L.pba_map_get_outlier_obs(h, _p(op), _p(of), _p(ouv)), "pba_map_get_outlier_obs", L)
    finally:
        L.pba_map_destroy(h)
    pb = synth.Problem(kind=synth.GEOMETRIC, model=info.camera_model, width=info.width, height=info.height,
                       intrinsics=intr, frame_cam=fcam, images=None, pattern=np.zeros((0, 2), np.float32),
                       point_host=host, u_ref=uref, host_intensity=None, block_point=bp, block_target=bt, u_obs=uobs,
                       poses=poses, rho=rho)
    extras = {"T_i_c": tic, "frame_id": fid, "track_id": tid, "outlier_point": op, "outlier_frame": of,
              "outlier_uv": ouv}
    return pb, extras


def outlier_landmarks(n_points: int, obs_point, obs_frame, flags, obs_is_outlier=None):
    """remove_outlier_landmarks (src/sfm.cpp:2028-2114): (remove (n_points,) bool, counts dict)."""
    op = np.ascontiguousarray(obs_point, np.int32)
    of = np.ascontiguousarray(obs_frame, np.int32)
    fl = np.ascontiguousarray(flags, np.uint32)
    oo = None if obs_is_outlier is None else np.ascontiguousarray(obs_is_outlier, np.uint8)
    rm = np.zeros(n_points, np.uint8)
    counts = np.zeros(5, np.int32)
    _check(lib().pba_outlier_landmarks(n_points, op.shape[0], _p(op), _p(of), _p(fl), _p(oo), _p(rm), _p(counts)),
           "pba_outlier_landmarks")
    return rm.astype(bool), dict(zip(("huge", "normal", "camera_distance", "z", "any_severe"), counts.tolist()))


def split_record(rec: np.ndarray, R: int):
    n = rec.shape[0]
    return rec[:, :R], rec[:, R:7 * R].reshape(n, R, 6), rec[:, 7 * R:13 * R].reshape(n, R, 6), rec[:, 13 * R:14 * R]
