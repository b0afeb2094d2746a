"""TEST-ONLY: runs tests/cpp/ceres_lm_driver (the real Ceres 2.0.0 LM solve of map_utils.h:322-383, built by
oracle/ceres.mk into oracle/_ref/) on a synthetic problem, in its CPU (the reference's AutoDiff path) or GPU
(include/pba_ceres.h over the engine) mode, and returns the parsed JSON summary.  Used by tests/ and by bench.py's
cpu_baseline leg (Ceres' own "Jacobian & residual evaluation" timer)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ceres_lm_driver")
ADAPTER_DRIVER = os.path.join(ROOT, "oracle", "_ref", "adapter_driver")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def available() -> bool:
    return os.path.exists(DRIVER)


def run(mode: str, pb, iters: int = 20, huber: float = 1.0, threads: int = 8, fixed=(0, 1), ftol: float = 1e-6,
        timeout: float = 600.0, ptol: float = 1e-8, gtol: float = 1e-10, optimize_intrinsics: bool = False,
        pose_param: str = "ref", check: bool = True, teacher=None) -> dict:
    """mode: "cpu" (AutoDiff), "gpu" (the drop-in) or "floor" (constant cost functions: Ceres' own per-evaluation work).
    check: gpu mode with the evaluation-callback protocol checks (tests) or the plain adapter (timing).
    pose_param: "ref" — the reference's LocalParameterizationSE3 in both modes (the GPU adapter then emits 7-wide
    Jacobians J6·P⁺); "tangent" — the adapter's SE3TangentParameterization in gpu mode.  optimize_intrinsics: 0 constant
    intrinsics blocks, 1 free (the GPU evaluator is given them), 2 free but not given to the evaluator (refusal).
    teacher (cpu mode): a list of (poses, rho, radius) states — one LM iteration of the Solve from each, returned as
    out["teacher"] rows [cost at the state, cost after, step_is_successful, relative_decrease, radius after, step_norm,
    iterations pushed, gradient max norm at the state]."""
    from make_golden import write_problem
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.json")
        with open(fin, "wb") as f:
            write_problem(f, pb)
        fx = ",".join(str(int(i)) for i in fixed) if len(fixed) else "-"
        ft = "-"
        if teacher is not None:
            ft = os.path.join(td, "teacher.bin")
            with open(ft, "wb") as f:
                for poses, rho, radius in teacher:
                    np.concatenate([np.asarray(poses, np.float64).ravel(), np.asarray(rho, np.float64).ravel(),
                                    [float(radius)]]).tofile(f)
        subprocess.run([DRIVER, mode, fin, fout, str(iters), repr(float(huber)), str(threads), fx, repr(float(ftol)),
                        str(int(getattr(pb, "interp", 0))), repr(float(ptol)), repr(float(gtol)),
                        str(int(optimize_intrinsics)), pose_param, "1" if check else "0", ft], check=True, timeout=timeout)
        with open(fout) as f:
            out = json.load(f)
    out["poses"] = np.asarray(out["poses"]).reshape(-1, 7)
    out["rho"] = np.asarray(out["rho"])
    it = np.asarray(out["iterations"], np.float64).reshape(-1, 7)
    out["costs"] = it[:, 1]
    out["step_ok"] = it[:, 2].astype(bool)
    out["relative_decrease"] = it[:, 3]
    out["radius"] = it[:, 4]
    out["step_norm"] = it[:, 5]
    out["gradient_max_norm"] = it[:, 6]
    out["intrinsics"] = np.asarray(out["intrinsics"]).reshape(-1, 8)
    if out.get("teacher") is not None:
        out["teacher"] = np.asarray(out["teacher"], np.float64).reshape(-1, 8)
    return out
