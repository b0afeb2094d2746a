#!/usr/bin/env python3
"""bench.py — photometric residual+Jacobian blocks/s on MI355X (BASELINE.json metric; configs[3] workload).

Workload (BASELINE.json configs[3] / SURVEY.md §8d C4): ONE synthetic problem of 1000 host keyframes × 100k points,
8-pixel DSO pattern, every point observed by the 4 keyframes after its host → 400,000 residual blocks (3.2 M pixel
residuals), 1004 keyframes of 752×480 u8 images (361 MB), pinhole camera.  One step = one full evaluation of every
block's residuals and tangent Jacobians (Ceres-mode records, include/pba.h) at a new state already resident in HBM:
ONE launch (pba_evaluate_state_device — the blocks form their relative poses in the prologue and the launch adopts
the state).

Multi-GPU (torch.distributed.run, one rank per GPU): BASELINE.json configs[3] is ONE 1000-keyframe problem sharded by
host keyframe across the GPUs, so the headline scales strongly — rank r evaluates its host-keyframe shard of the one C4
problem (distributed.shard_problem: contiguous host ranges balanced by block count), with no data-path collective (the
evaluation has no exchange step) → `scaling: "strong"`, value = 400k blocks ÷ the max-over-ranks time of a
step.  The weak form (every rank a full C4-size shard of an N·1000-keyframe trajectory) is reported under "weak", and at
N = 1 the step of a 1/8 shard under "shard8" (the strong-scaling ceiling at N = 8).  Timing: a clock warm-up, W warmup
steps, then exactly K steps bracketed by barrier + synchronize.

Also reported: the block kernel's roofline position (algorithmic bytes ÷ HIP-event-timed kernel duration on the engine
stream); the CPU baseline — the reference's CPU path, real Ceres 2.0.0 (built from the reference's vendored sources
by oracle/ceres.mk) evaluating AutoDiff cost functions with its ProgramEvaluator on this host's cores, timed by its
own "Jacobian & residual evaluation" timer on a bounded sample of the same workload; ms per LM iteration of the
on-device Gauss-Newton (C4 on rendered images — the solve the GPU tests pin against real Ceres, whose trajectory on the
same problem is reported beside it — and C3 = configs[2] in "gn_c3"); and the C5-style 21-px / fp16 / pyramid leg.
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
engine_mod = importlib.import_module("photometric-bundle-adjustment_amd.engine")
D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes_per_block(P: int, K: int, n_frames: int, n_points: int, n_blocks: int, value_bytes: int = 4) -> float:
    """SURVEY.md §8d, Ceres mode, fp32 records, fused state (pba_evaluate_state_device): inputs + taps + outputs
    per block (formula in DESIGN.md §3)."""
    idx = 16.0                                 # block record {point, host, target, cameras} (int32 × 4)
    point = (16.0 + 8.0 + 4.0 * P) / K         # u_ref (2×f64) + ρ (f64) + I_h (P×f32), shared by the point's K blocks
    state = (56.0 * 2 * n_frames + 8.0 * n_points) / n_blocks  # pose reads (L2-shared) + adopted state written
    taps = 4.0 * P                             # 4 u8 bilinear taps per pixel (gradient from the same taps)
    out = value_bytes * 14.0 * P + 4.0 + 1.0   # record [r | J_h | J_t | J_ρ] (fp32, or fp16 for C5) + cost + valid
    return idx + point + state + taps + out


def host_cores():
    """Cores this process may use (affinity ∩ cgroup CPU quota), the machine's count and the CPU model."""
    n_all = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = n_all
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    usable = max(1, min(aff, int(quota + 0.5) if quota else aff))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "nproc": n_all, "affinity": aff, "cgroup_quota_cpus": quota, "cpu_model": model}


def c4_sample(pb, images_host, hosts: int = 250):
    """The points hosted by the first `hosts` keyframes of the C4 problem with all their blocks (100k blocks)."""
    sel_pts = np.nonzero(pb.point_host < hosts)[0]
    remap = np.full(pb.n_points, -1, np.int64)
    remap[sel_pts] = np.arange(len(sel_pts))
    sel_blk = np.nonzero(remap[pb.block_point] >= 0)[0]
    nfs = hosts + 4
    return synth.Problem(kind=pb.kind, model=pb.model, width=pb.width, height=pb.height, intrinsics=pb.intrinsics,
                         frame_cam=pb.frame_cam[:nfs], images=images_host[:nfs], pattern=pb.pattern,
                         point_host=pb.point_host[sel_pts], u_ref=pb.u_ref[sel_pts],
                         host_intensity=pb.host_intensity[sel_pts], block_point=remap[pb.block_point[sel_blk]].astype(np.int32),
                         block_target=pb.block_target[sel_blk], u_obs=None, poses=pb.poses[:nfs], rho=pb.rho[sel_pts])


def per_call(r):
    """Ceres' own timers (Solver::Summary) per evaluation call."""
    return {"jacobian_evaluation_ms": 1e3 * r["jacobian_evaluation_s"] / max(r["jacobian_evaluations"], 1),
            "jacobian_evaluations": r["jacobian_evaluations"],
            "residual_evaluation_ms": 1e3 * r["residual_evaluation_s"] / max(r["residual_evaluations"], 1),
            "linear_solver_ms_per_iteration": 1e3 * r["linear_solver_s"] / max(len(r["costs"]) - 1, 1),
            "minimizer_s": r["minimizer_s"], "successful_steps": r["successful_steps"],
            "unsuccessful_steps": r["unsuccessful_steps"], "final_cost": r["final_cost"], "threads": r["threads"],
            **({"prepare_breakdown": r["prepare"]} if "prepare" in r else {})}


RUNS_PER_MODE = 7  # C2 / C4-sample Ceres runs per mode, interleaved; the median run of each is reported


def c2_dropin(pb_c4, images_host, threads: int):
    """BASELINE.json configs[1] (C2) — "Ceres LM + GPU EvaluationCallback": real Ceres 2.0.0 ceres::Solve (LM,
    SPARSE_SCHUR, Huber, the reference's LocalParameterizationSE3) over include/pba_ceres.h (GpuEvaluator + per-block
    CostFunctions, the engine's records read back in chunks that overlap Ceres' per-block work) against the same Solve
    over AutoDiff on the CPU.  Ceres' "Jacobian & residual evaluation" time per call (program_evaluator.h:139-258, with
    the Jacobian writer) is C2's metric; also on the 100k-block C4 sample of cpu_baseline."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ceres_runner as CR
    if not CR.available():
        return None
    pb = synth.c2_problem()
    pb.poses[:2] = pb.poses_gt[:2]
    out = {"config": f"C2: {pb.n_frames} keyframes of EuRoC V1 image content, {pb.n_blocks} blocks, 8-px pattern, "
                     f"double sphere, Huber 9, 10 LM iterations"}
    # the plain adapter (no protocol checks: the tests run those), its floor (the same Solve replayed over the drop-in's
    # recorded read-backs: Ceres' own work plus the adapter's per-block copy on the drop-in's own trajectory, i.e.
    # everything but the device's part), and the CPU AutoDiff path — same Solve options
    # each mode RUNS_PER_MODE times, interleaved, the median run of each reported (the box's host is shared: a 16-CPU
    # cgroup quota; single runs of these ~3-ms evaluations vary by ±10-30 %)
    # floor_cold: the floor with its staged read-backs flushed from the CPU caches before each evaluation
    # (PBA_FLOOR_COLD, tests/cpp/ceres_lm_driver.cpp) — the drop-in's records arrive by DMA into memory no core has cached
    runs = {m: [] for m in ("gpu", "cpu", "floor", "floor_cold")}
    for _ in range(RUNS_PER_MODE):
        runs["gpu"].append(CR.run("gpu", pb, iters=10, huber=9.0, threads=threads, check=False))
        runs["cpu"].append(CR.run("cpu", pb, iters=10, huber=9.0, threads=threads))
        runs["floor"].append(CR.run("floor", pb, iters=10, huber=9.0, threads=threads))
        os.environ["PBA_FLOOR_COLD"] = "1"
        try:
            runs["floor_cold"].append(CR.run("floor", pb, iters=10, huber=9.0, threads=threads))
        finally:
            os.environ.pop("PBA_FLOOR_COLD", None)
    best = {m: sorted(v, key=lambda r: r["jacobian_evaluation_s"] + r["residual_evaluation_s"])[len(v) // 2]
            for m, v in runs.items()}
    g, c, fl = best["gpu"], best["cpu"], best["floor"]
    out["gpu_dropin"], out["cpu_autodiff"], out["ceres_floor"] = per_call(g), per_call(c), per_call(fl)
    out["ceres_floor_cold"] = per_call(best["floor_cold"])
    out["runs_per_mode"] = RUNS_PER_MODE
    out["jacobian_evaluation_ms_runs"] = {m: [1e3 * r["jacobian_evaluation_s"] / max(r["jacobian_evaluations"], 1)
                                              for r in v] for m, v in runs.items()}
    out["blocks"] = pb.n_blocks
    out["speedup_jacobian_evaluation"] = out["cpu_autodiff"]["jacobian_evaluation_ms"] / out["gpu_dropin"]["jacobian_evaluation_ms"]
    out["speedup_residual_evaluation"] = out["cpu_autodiff"]["residual_evaluation_ms"] / out["gpu_dropin"]["residual_evaluation_ms"]
    out["jacobian_evaluation_vs_floor"] = out["gpu_dropin"]["jacobian_evaluation_ms"] / out["ceres_floor"]["jacobian_evaluation_ms"]
    jr = out["jacobian_evaluation_ms_runs"]
    out["jacobian_evaluation_vs_floor_min"] = min(jr["gpu"]) / min(jr["floor"])  # (the fastest run of each mode)
    out["jacobian_evaluation_vs_floor_cold"] = (out["gpu_dropin"]["jacobian_evaluation_ms"] /
                                                out["ceres_floor_cold"]["jacobian_evaluation_ms"])
    out["residual_evaluation_vs_floor"] = out["gpu_dropin"]["residual_evaluation_ms"] / out["ceres_floor"]["residual_evaluation_ms"]
    out["same_trajectory"] = bool(len(g["costs"]) == len(c["costs"]) and np.array_equal(g["step_ok"], c["step_ok"]))
    out["floor_replay_ok"] = bool(all(r["replay_ok"] == 1 for r in runs["floor"]))
    out["floor_same_evaluations"] = bool(fl["jacobian_evaluations"] == g["jacobian_evaluations"] and
                                         fl["residual_evaluations"] == g["residual_evaluations"])
    out["floor_note"] = ("ceres_floor: the same Solve over the same per-block CostFunctions, replaying the drop-in's "
                         "recorded read-backs (records / residuals, validity, P+) — the drop-in's trajectory and evaluation "
                         "counts with the device's part (state upload, launch, read-back) removed; ceres_floor_cold: the "
                         "same with the replayed records flushed from the CPU caches before each evaluation (the drop-in's "
                         "arrive by DMA)")
    # the C4 sample the same way: interleaved runs per mode, the median of each (single runs moved the floor's
    # evaluations and even Ceres' own linear solver by +30-60 % between neighbouring processes on the shared host)
    sample = c4_sample(pb_c4, images_host)
    sruns = {m: [] for m in ("gpu", "floor")}
    for _ in range(RUNS_PER_MODE):
        sruns["gpu"].append(CR.run("gpu", sample, iters=4, huber=9.0, threads=threads, ftol=0.0, check=False))
        sruns["floor"].append(CR.run("floor", sample, iters=4, huber=9.0, threads=threads, ftol=0.0))
    jpc = lambda r: r["jacobian_evaluation_s"] / max(r["jacobian_evaluations"], 1)  # noqa: E731
    gs, fs = (sorted(v, key=jpc)[len(v) // 2] for v in (sruns["gpu"], sruns["floor"]))
    out["c4_sample"] = dict(per_call(gs), blocks=sample.n_blocks, ceres_floor=per_call(fs), runs_per_mode=RUNS_PER_MODE,
                            jacobian_evaluation_vs_floor_min=min(map(jpc, sruns["gpu"])) / min(map(jpc, sruns["floor"])),
                            jacobian_evaluation_ms_runs={m: [1e3 * jpc(r) for r in v] for m, v in sruns.items()},
                            jacobian_evaluation_vs_floor=jpc(gs) / jpc(fs),
                            floor_same_evaluations=bool(fs["jacobian_evaluations"] == gs["jacobian_evaluations"]),
                            floor_replay_ok=bool(all(r["replay_ok"] == 1 for r in sruns["floor"])))
    return out


def cpu_baseline(pb, images_host, budget_s: float):
    """The reference's CPU path on a bounded sample of the same workload: real Ceres 2.0.0 (oracle/_ref, built from
    the reference's vendored sources) — ceres::Solve, LEVENBERG_MARQUARDT + SPARSE_SCHUR, one AutoDiffCostFunction per
    residual block over the restated PhotometricError functor (bilinear, pinhole), HuberLoss, the reference's
    LocalParameterizationSE3, num_threads = the usable host cores (map_utils.h:376-381) — timed by Ceres' own
    "Jacobian & residual evaluation" timer (Solver::Summary).  Sample: the points hosted by the first keyframes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ceres_runner as CR
    cores = host_cores()
    if not CR.available():
        return None
    hosts = 250
    nfs = hosts + 4
    sample = c4_sample(pb, images_host, hosts)
    t0 = time.perf_counter()
    r = CR.run("cpu", sample, iters=2, huber=9.0, threads=cores["usable"], fixed=(0, 1), ftol=0.0)
    per_eval = r["jacobian_evaluation_s"] / max(r["jacobian_evaluations"], 1)
    iters = int(min(60, max(2, budget_s / max(per_eval, 1e-3))))
    if iters > 2:
        r = CR.run("cpu", sample, iters=iters, huber=9.0, threads=cores["usable"], fixed=(0, 1), ftol=0.0)
    n_eval = r["jacobian_evaluations"]
    rate = sample.n_blocks * n_eval / r["jacobian_evaluation_s"]
    return {"value": rate, "unit": "blocks/s", "cores": r["threads"],
            "kind": "reference",
            "kind_detail": "Ceres 2.0.0 evaluator (ProgramEvaluator + AutoDiff) over the restated photometric functor",
            "per_core": rate / max(r["threads"], 1),
            "reference_functor_per_core": {
                "value": 43000.0, "unit": "blocks/s",
                "note": "SURVEY.md §6: the reference's own BundleAdjustmentReprojectionCostFunctor inside Ceres' evaluator "
                        "(per-call AbstractCamera::from_data heap allocation + string dispatch, camera_models.h:452-474) "
                        "measured in the survey container; the restated functor above avoids that overhead"},
            "host": cores,
            "sample": f"{sample.n_blocks} blocks (the points hosted by keyframes 0-{hosts - 1} of the same problem, "
                      f"{nfs} frames), {n_eval} Jacobian+residual evaluations timed by Ceres' Solver::Summary "
                      f"({r['jacobian_evaluation_s']:.1f} s of {time.perf_counter() - t0:.1f} s wall) in ceres::Solve "
                      f"(LM, SPARSE_SCHUR, {r['threads']} threads); real Ceres 2.0.0 ProgramEvaluator + AutoDiff over "
                      f"the restated photometric functor (the reference's own photometric functor is on its absent "
                      f"pba2 branch)",
            "residual_only_blocks_per_s": sample.n_blocks * r["residual_evaluations"] / max(r["residual_evaluation_s"], 1e-9),
            "linear_solver_s_per_iteration": r["linear_solver_s"] / max(len(r["costs"]) - 1, 1)}


def all_reduce_max(torch, dist, values, dev):
    """MAX over ranks of a few host scalars (on the device for RCCL, through the host for gloo)."""
    on_dev = dist is not None and dist.get_backend() == "nccl"
    t = torch.tensor(values, dtype=torch.float64, device=dev if on_dev else "cpu")
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu()


def ranks_agree(torch, dist, values, dev):
    """True when every rank holds bit-identical `values` (one MAX all-reduce of v and -v)."""
    m = all_reduce_max(torch, dist, list(values) + [-x for x in values], dev).tolist()
    return all(m[i] == -m[i + len(values)] for i in range(len(values)))


def make_states(pb, torch, dev, seed):
    rng = np.random.default_rng(seed)
    states = []
    for _ in range(2):  # alternate two perturbed states so every step evaluates a new point
        poses = synth.se3_plus(pb.poses, 1e-3 * rng.normal(0, 1, (pb.n_frames, 6)))
        rho = pb.rho * (1 + 0.01 * rng.normal(0, 1, pb.n_points))
        states.append((torch.from_numpy(poses).to(dev), torch.from_numpy(rho).to(dev)))
    return states


def time_evaluation(eng, states, steps, warmup, clock_warmup_s, torch, dist, dev):
    """W warmup steps (after a clock warm-up), then K timed steps bracketed by barrier + synchronize (enqueued by one
    pba_evaluate_states_device call: K launches, one per step, each at a new HBM-resident state); returns
    (max-over-ranks elapsed s, max-over-ranks average block-kernel µs, host diagnostics).  The kernel duration comes
    from two HIP events on the engine's stream around the K timed launches (elapsed ÷ K: each launch plus the
    dispatch gap to the next, so never below rocprof's kernel average); the launches themselves carry no events —
    a pair of timing events per launch idles the GPU ~4 µs per step (`host` reports that instrumented run too)."""
    def step(i):  # one launch: pairs formed in the block prologue, state adopted by the same launch
        p, r = states[i & 1]
        eng.evaluate_state_device(p.data_ptr(), r.data_ptr(), True, sync=False)

    # clock warm-up (untimed, on top of the W warmup steps): the GPU's clocks take ~0.1 s of load to ramp, and a short
    # run measured 70 µs per step cold against 54 µs warm (profiles/r1_bench_c4_v27.json)
    t_w = time.perf_counter()
    i = 0
    while time.perf_counter() - t_w < clock_warmup_s:
        for _ in range(20):
            step(i)
            i += 1
        eng.synchronize()
    for i in range(warmup):
        step(i)
    eng.synchronize()
    # diagnostic (not the metric): the same steps with a timing-event pair around every launch (the engine's
    # per-launch kernel timing: kernel-only durations)
    eng.enable_kernel_timing(True)
    eng.kernel_timing()  # reset
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    eng.synchronize()
    t_ev = time.perf_counter() - t0
    kern_only_ms, launches = eng.kernel_timing()
    eng.enable_kernel_timing(False)
    host_diag = {"us_per_step_with_per_launch_events": 1e6 * t_ev / steps,
                 "kernel_only_us_per_launch_events": 1e3 * kern_only_ms / max(launches, 1)}
    # the timed region
    stream = torch.cuda.ExternalStream(eng.stream(), device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the K steps enqueued by one ABI call (pba_evaluate_states_device: K launches, each at the next state and adopting
    # it) — per-step foreign calls from Python cost ~5 µs of host time each, more than a 1/8 shard's 8-µs kernel
    pp = [states[i & 1][0].data_ptr() for i in range(steps)]
    rr = [states[i & 1][1].data_ptr() for i in range(steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    eng.evaluate_states_device(pp, rr, True, sync=False)
    host_diag["enqueue_us_per_step"] = 1e6 * (time.perf_counter() - t0) / steps
    e1.record(stream)
    # completion: ONE device-wide synchronize (it covers the engine's stream).  Round 5 synchronized the engine stream
    # first and then the device: two wake-ups, ≈ 5 µs more per timed region (tools/probe/sync_probe.py,
    # profiles/r6_sync_probe.txt: 17-20 µs of fixed cost per region against 23-25)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    t = all_reduce_max(torch, dist, [t1 - t0, 1e3 * e0.elapsed_time(e1) / steps], dev)
    return float(t[0]), float(t[1]), host_diag


def gn_benchmark(eng, pb, iters, torch, dist, dev, world, ceres_problem=None, threads=1):
    """ms per Levenberg-Marquardt iteration (BASELINE.json metric, part 2) on the C4 problem with rendered images (the
    problem test_c4_engine_lm_matches_ceres_cpu pins against real Ceres), through the engine's own LM loop (pba_solve;
    pba_solve_distributed with an all-reduce of the banded reduced system for N>1).  An iteration = Schur complement +
    reduced-system solve + candidate linearisation (its cost) + the decision; function_tolerance = 0 so exactly `iters`
    iterations run.  Two keyframes are held constant (the reference's fixed cameras).  ceres_problem (N = 1): the same
    problem with host images — real Ceres 2.0.0 LM over the AutoDiff functor runs the same 20 iterations on the CPU and its
    trajectory is reported beside the engine's."""
    eng.set_fixed_frames(np.array([0, 1], np.int32))
    eng.gn_linearize()  # symbolic analysis (once per problem structure), outside the timed region
    opts = dict(max_iterations=iters, function_tolerance=0.0)
    agree = None
    traj = None
    device_steered = world > 1 and dist.get_backend() == "nccl" and os.environ.get("PBA_BENCH_GN_COMM", "0") == "1"
    if world > 1:
        band = D.global_band(eng, None, dev)
        # Default: the host-callback loop (pba_solve_distributed: torch.distributed's all_reduce — RCCL under "nccl" —
        # between trials, host decisions from the all-reduced sums).  PBA_BENCH_GN_COMM=1 selects the device-steered
        # loop (pba_solve_distributed_comm: both all-reduces of every trial on the engine stream through the engine's
        # own RCCL communicator, the next trial enqueued ahead of the decision, every trial's scalar all-reduce checking
        # that the ranks took the same previous decision).  That loop has run with one RCCL rank and with in-process
        # groups only (no multi-GPU box in the build pipeline), so the unattended N > 1 bench uses torch's collective,
        # whose only failure mode is an error, not a hang on mismatched stream-ordered collectives.
        comm = None if device_steered else False
        D.solve_distributed(eng, device=dev, comm=comm, max_iterations=1)  # warm-up (sets the RCCL communicator up)
        eng.set_state(pb.poses, pb.rho)
        dist.barrier()
        torch.cuda.synchronize()
        s = D.solve_distributed(eng, device=dev, comm=comm, **opts)
        exchange_mb = 8.0 * eng.gn_exchange_size(band) / 1e6
        # every rank must have taken the same decisions: the global costs and step counts agree bit for bit
        agree = ranks_agree(torch, dist, [s["initial_cost"], s["final_cost"], float(s["iterations"]),
                                          float(s["successful_steps"])], dev)
    else:
        eng.solve(max_iterations=1)  # warm-up
        eng.set_state(pb.poses, pb.rho)
        torch.cuda.synchronize()
        s = eng.solve(**opts)
        traj = eng.solver_iterations()
        exchange_mb = None
        # the per-phase breakdown comes from a second, event-instrumented solve (events idle the GPU a few µs each,
        # so the timed solve above runs without them) from the same initial state: the same work per iteration
        eng.set_state(pb.poses, pb.rho)
        eng.set_solver_timing(True)
        sb = eng.solve(**opts)
        eng.set_solver_timing(False)
        s = dict(s, linearize_ms=sb["linearize_ms"], solve_ms=sb["solve_ms"], cost_ms=sb["cost_ms"])
    t = all_reduce_max(torch, dist, [s["total_ms"], s["linearize_ms"], s["solve_ms"], s["cost_ms"]], dev)
    n = max(s["iterations"], 1)
    out = {"ms_per_iteration": float(t[0]) / n, "iterations": s["iterations"], "accepted": s["successful_steps"],
           "initial_cost": s["initial_cost"], "final_cost": s["final_cost"],
           "breakdown_ms_per_iteration": {"linearize_ms": float(t[1]) / n, "step_ms": float(t[2]) / n,
                                          "cost_ms": float(t[3]) / n},
           "exchange_mb_per_iteration": exchange_mb, "ranks_agree": agree,
           "note": "host wall clock of the engine's LM loop (pba_solve" + (
               "_distributed_comm: the device-steered loop with two RCCL all-reduces per trial on the engine stream "
               "(the banded reduced camera system, then 16 scalars)" if device_steered
               else f"_distributed: {dist.get_backend()} all-reduces through a host callback" if world > 1 else "") +
                   ") on the C4 problem with rendered images (one textured plane seen by every keyframe), from its "
                   "perturbed initial state"}
    if ceres_problem is not None and traj is not None:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import ceres_runner as CR
        if CR.available():
            t0 = time.perf_counter()
            ref = CR.run("cpu", ceres_problem, iters=iters, huber=9.0, threads=threads, ftol=0.0, timeout=900)
            m = min(len(traj["cost"]), len(ref["costs"]))
            rel = np.abs(traj["cost"][:m] - ref["costs"][:m]) / np.abs(ref["costs"][:m])
            e_ok = traj["step_is_successful"][:m].astype(bool)
            c_ok = np.asarray(ref["step_ok"][:m]).astype(bool)
            within = np.flatnonzero((rel > 1e-5) | (e_ok != c_ok))
            out["ceres"] = {
                # the iterations before the first one whose cost differs by more than the north star's 1e-5 (or whose
                # accept flag differs): the solves part once λ is tiny (test_c4_engine_lm_matches_ceres_cpu_free_running)
                "iterations_within_1e-5": int(within[0]) if within.size else int(m),
                "same_steps_through": int(np.flatnonzero(e_ok != c_ok)[0]) if (e_ok != c_ok).any() else int(m),
                "rel_cost_difference_per_iteration": [float(f"{x:.3g}") for x in rel],
                "final_cost": ref["final_cost"], "successful_steps": ref["successful_steps"] - 1,
                "unsuccessful_steps": ref["unsuccessful_steps"], "message": ref["message"],
                "same_steps": bool(len(traj["cost"]) == len(ref["costs"]) and
                                   np.array_equal(traj["step_is_successful"].astype(bool), ref["step_ok"])),
                "max_rel_cost_difference_per_iteration": float(rel.max()),
                "final_cost_rel_difference": abs(s["final_cost"] - ref["final_cost"]) / abs(ref["final_cost"]),
                "minimizer_s": ref["minimizer_s"], "linear_solver_s_per_iteration": ref["linear_solver_s"] / max(m - 1, 1),
                "threads": ref["threads"], "wall_s": time.perf_counter() - t0,
                "note": "real Ceres 2.0.0 LM (SPARSE_SCHUR, AutoDiff over the restated photometric functor, the reference's "
                        "LocalParameterizationSE3, the same options) on the same problem on this host's cores: the "
                        "trajectory the engine's timed solve is compared with, iteration by iteration"}
    return out


def gn_c3(iters, torch, dev_index, dev):
    """BASELINE.json configs[2] (C3): synthetic 200 keyframes × 20k points × 8-px patch (80k blocks) with
    rendered (smooth, textured) images, so LM actually converges; on-device JᵀJ/Jᵀr + Schur GN through the
    engine's LM loop (pba_solve).  One GPU (rank 0 at N = 1 only)."""
    t0 = time.perf_counter()
    pb = synth.make_problem(n_frames=200, n_points=20000, K=4, kind="photometric", model="pinhole", seed=42)
    gen_s = time.perf_counter() - t0
    eng = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=dev_index, huber_width=9.0)
    try:
        images = torch.from_numpy(pb.images).to(dev)
        eng.set_problem(pb, images_device_ptr=images.data_ptr())
        eng.set_fixed_frames(np.array([0, 1], np.int32))
        eng.set_state(pb.poses, pb.rho)
        eng.gn_linearize()  # symbolic analysis, outside the timed region
        eng.solve(max_iterations=1)  # warm-up
        eng.set_state(pb.poses, pb.rho)
        torch.cuda.synchronize()
        s = eng.solve(max_iterations=iters, function_tolerance=0.0)
        eng.set_state(pb.poses, pb.rho)  # the breakdown: the same solve again, with per-phase events
        eng.set_solver_timing(True)
        sb = eng.solve(max_iterations=iters, function_tolerance=0.0)
        s = dict(s, linearize_ms=sb["linearize_ms"], solve_ms=sb["solve_ms"], cost_ms=sb["cost_ms"])
    finally:
        eng.close()
    n = max(s["iterations"], 1)
    return {"config": "C3: synthetic 200 keyframes x 20000 points x 8-px patch x 4 targets = 80000 blocks, 752x480 "
                      "rendered images, pinhole, 2 fixed keyframes",
            "ms_per_iteration": s["total_ms"] / n, "iterations": s["iterations"], "accepted": s["successful_steps"],
            "initial_cost": s["initial_cost"], "final_cost": s["final_cost"],
            "breakdown_ms_per_iteration": {"linearize_ms": s["linearize_ms"] / n, "step_ms": s["solve_ms"] / n,
                                           "cost_ms": s["cost_ms"] / n},
            "problem_generation_s": gen_s,
            "note": "host wall clock of pba_solve (Ceres LM logic on the host, every kernel on the device); the breakdown "
                    "is device time between stream events of a second, instrumented run of the same solve"}


DISK21 = np.array([(dx, dy) for dy in range(-2, 3) for dx in range(-2, 3) if dx * dx + dy * dy <= 5], np.float32)


def c5_eval(pb, images, states, steps, warmup, clock_warmup_s, torch, dev_index, dev, gn_iterations=0):
    """BASELINE.json configs[4] (C5) on the C4 problem: 21-pixel pattern (the radius-√5 disk), records stored as
    fp16 (PBA_RECORD_F16), and a 3-level image pyramid built on the device.  Same one-launch step and the same clock
    warm-up / warmup count as the headline; the full EuRoC sequence is not in the container, so the images are the
    synthetic ones."""
    import copy
    pb5 = copy.copy(pb)
    pb5.pattern = DISK21
    host = torch.from_numpy(pb.point_host.astype(np.int64)).to(dev)
    uu = torch.from_numpy(pb.u_ref[:, 0].astype(np.int64)).to(dev)[:, None] + torch.from_numpy(DISK21[:, 0].astype(np.int64)).to(dev)
    vv = torch.from_numpy(pb.u_ref[:, 1].astype(np.int64)).to(dev)[:, None] + torch.from_numpy(DISK21[:, 1].astype(np.int64)).to(dev)
    pb5.host_intensity = images[host[:, None], vv, uu].float().cpu().numpy()
    eng = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=dev_index, huber_width=9.0)
    try:
        eng.set_problem(pb5, images_device_ptr=images.data_ptr())
        eng.set_record_format(engine_mod.RECORD_F16)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.build_pyramid(3)
        eng.synchronize()
        pyr_ms = 1e3 * (time.perf_counter() - t0)
        el, kern_us, _ = time_evaluation(eng, states, steps, warmup, clock_warmup_s, torch, None, dev)
        gn = None
        if gn_iterations > 0:
            # on-device GN at the 21-px pattern (the finest level; BASELINE C5's "fp32 jacobian accumulate": the rows go
            # through the fp32 matrix cores into JᵀJ, nothing is stored): the LM loop as in the C4 GN leg
            eng.set_fixed_frames(np.array([0, 1], np.int32))
            eng.set_state(pb5.poses, pb5.rho)
            eng.gn_linearize()
            eng.solve(max_iterations=1)  # warm-up
            torch.cuda.synchronize()
            sg = eng.solve(max_iterations=gn_iterations, function_tolerance=0.0)
            gn = {"ms_per_iteration": sg["total_ms"] / max(sg["iterations"], 1), "iterations": sg["iterations"],
                  "accepted": sg["successful_steps"]}
    finally:
        eng.close()
    P = DISK21.shape[0]
    bpb = algorithmic_bytes_per_block(P, pb.n_blocks // max(pb.n_points, 1), pb.n_frames, pb.n_points, pb.n_blocks, 2)
    gbs = bpb * pb.n_blocks / (kern_us * 1e-6) / 1e9
    return {"config": f"C5-style: the C4 problem with a {P}-px pattern, fp16 records, 3-level pyramid (synthetic images)",
            "blocks_per_s": pb.n_blocks * steps / el, "ms_per_step": 1e3 * el / steps, "kernel_avg_us": kern_us,
            "bytes_per_block_alg": bpb, "achieved_gbs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS,
            "record_format": "f16", "P": P, "record_bytes_per_block": 2 * 14 * P, "pyramid_levels": 3,
            "pyramid_build_ms": pyr_ms, "gn": gn}


HEADLINE_KERNEL = "photometric_block_kernel<0, 8, 1, float>"


def traffic_probe(args):
    """--traffic-probe (a child of measure_traffic under rocprofv3 --pmc): the headline launch at 5 HBM-resident
    states of the same C4 problem, nothing else."""
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pb, images = synth.c4_shard(dev, n_frames=args.frames, n_points=args.points, K=args.targets,
                                block_order=args.block_order)
    eng = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=0, huber_width=9.0)
    eng.set_problem(pb, images_device_ptr=images.data_ptr())
    states = make_states(pb, torch, dev, 7)
    for i in range(5):
        eng.evaluate_state_device(states[i % len(states)][0].data_ptr(), states[i % len(states)][1].data_ptr(), True)
    eng.synchronize()
    eng.close()
    print(json.dumps({"probe": "ok", "n_blocks": pb.n_blocks}), flush=True)


def counter_bytes_per_launch(rows, ctr, kernel):
    """Mean bytes per dispatch of `kernel` from rocprofv3 counter_collection rows of counter `ctr` (KB): the rows of
    one dispatch (one per XCD / instance dimension) are summed, the dispatches averaged, KB x 1024.  None: no sample."""
    per = {}
    for x in rows:
        if x["Counter_Name"] == ctr and kernel in x["Kernel_Name"]:
            per[x["Dispatch_Id"]] = per.get(x["Dispatch_Id"], 0.0) + float(x["Counter_Value"])
    return sum(per.values()) / len(per) * 1024.0 if per else None


def measure_traffic(args, n_blocks, timeout_s=150):
    """HBM bytes per headline launch, measured in this run: two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE —
    separate passes, MI355X_MICROARCH.md: the two do not fit one pass) over a child process running --traffic-probe,
    raw KB x 1024 (the guide's 2x FETCH correction is calibrated for 16-B streaming reads; these are byte gathers of
    tiled image lines and the corrected total would exceed the chip's achievable 6.3 TB/s at the measured launch time,
    DESIGN.md §5).  Returns (bytes, source) or (None, reason)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    vals = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory(dir="/tmp") as d:
            cmd = [prof, "--pmc", ctr, "--kernel-include-regex", HEADLINE_KERNEL,
                   "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable, os.path.abspath(__file__),
                   "--traffic-probe", "--frames", str(args.frames), "--points", str(args.points),
                   "--targets", str(args.targets)]
            try:
                r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout_s)
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 --pmc {ctr} pass timed out"
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {ctr} pass failed (rc {r.returncode})"
            rows = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                rows += list(csv.DictReader(open(f)))
            v = counter_bytes_per_launch(rows, ctr, HEADLINE_KERNEL)
            if v is None:
                return None, f"no {ctr} samples for {HEADLINE_KERNEL}"
            vals[ctr] = v
    return vals["FETCH_SIZE"] + vals["WRITE_SIZE"], {
        "source": "measured in this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (child processes), raw KB x 1024",
        "fetch_bytes": vals["FETCH_SIZE"], "write_bytes": vals["WRITE_SIZE"]}


def stream_copy_peak(torch, dev, achieved):
    """a measured streaming rate beside the 8 TB/s spec.  The reference point is hand-written float4 copy
    kernels (tools/micro/stream_copy.hip: 16-B loads and stores, 1-4 moves per lane, default or non-temporal policies,
    1 GiB, the best launch over forms and grid sizes) — MI355X_MICROARCH.md's "float4 copy" measurement (6.29 TB/s
    there), taken on this box; a torch device copy of the same size is reported beside it."""
    import ctypes
    out = {}
    so = os.path.join(ROOT, "tools", "micro", "libstream_copy.so")
    try:
        lib = ctypes.CDLL(so)
        lib.stream_copy_gbs.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int)]
        g, grid = ctypes.c_double(0.0), ctypes.c_int(0)
        torch.cuda.synchronize()
        rc = lib.stream_copy_gbs(1 << 30, 5, ctypes.byref(g), ctypes.byref(grid))
        if rc == 0 and g.value > 0:
            out = {"stream_copy_gbs": g.value, "frac_of_stream_copy": achieved / g.value,
                   "stream_copy_note": f"hand-written float4 copy kernels (16-B loads / stores, 1-4 moves per lane, "
                                       f"default or non-temporal policies), 1 GiB (2 GiB of traffic per copy), best of "
                                       f"5 launches x 7 forms x 4 grids (form {grid.value % 100}, "
                                       f"{grid.value // 100} workgroups; tools/micro/stream_copy.hip)"}
        else:
            out = {"stream_copy_error": f"stream_copy_gbs returned {rc}"}
    except OSError as ex:
        out = {"stream_copy_error": f"{so}: {ex}"[:200]}
    try:
        a = torch.empty(1 << 28, dtype=torch.float32, device=dev).fill_(1.0)
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        best = None
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b.copy_(a)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        out["torch_copy_gbs"] = 2.0 * a.numel() * 4 / (best * 1e-3) / 1e9
        del a, b
    except Exception as ex:  # diagnostic only
        out["torch_copy_error"] = f"{type(ex).__name__}: {ex}"[:200]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--clock-warmup-s", type=float, default=0.3)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--points", type=int, default=100000)
    ap.add_argument("--targets", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # a bundle adjustment of the reference runs 20 LM iterations (sfm.cpp:1910, map_utils.h:318)
    ap.add_argument("--gn-iterations", type=int, default=20)
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 Gauss-Newton measurement (configs[2])")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5-style 21-px / fp16 / pyramid measurement")
    ap.add_argument("--no-shard-leg", action="store_true", help="N = 1: skip the 1/8-shard step leg")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 Ceres drop-in measurement (configs[1])")
    ap.add_argument("--no-live-traffic", action="store_true",
                    help="take roofline.traffic from the committed profiles/ file instead of two rocprofv3 --pmc passes")
    ap.add_argument("--traffic-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--block-order", default="point", help=argparse.SUPPRESS)  # traffic probe: "point" | "morton"
    args = ap.parse_args()
    if args.traffic_probe:
        traffic_probe(args)
        return

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run")
    # PBA_BENCH_BACKEND=gloo rehearses the N>1 path with several ranks on fewer GPUs (ranks share devices)
    backend = os.environ.get("PBA_BENCH_BACKEND", "nccl")
    dev_index = local_rank % max(torch.cuda.device_count(), 1) if backend != "nccl" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    dd = None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        dd = dist

    # ---- the headline: the one C4 problem (BASELINE.json configs[3]); N > 1 — split by host keyframe, strong scaling ------
    # (the evaluation partitions by host keyframe with no exchange step, SURVEY.md §8e: rank r evaluates the points
    # hosted by its contiguous range of host keyframes, with all their blocks; every rank holds all poses and images)
    K, F, Np = args.targets, args.frames, args.points
    full, images = synth.c4_shard(dev, n_frames=F, n_points=Np, K=K)  # identical on every rank (same seeds)
    pb = D.shard_problem(full, world, rank)[0] if world > 1 else full
    eng = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=dev_index, huber_width=9.0)
    eng.set_problem(pb, images_device_ptr=images.data_ptr())
    states = make_states(pb, torch, dev, 7)
    eng.set_state_device(states[0][0].data_ptr(), states[0][1].data_ptr())
    eng.evaluate(True)
    _, valid = eng.records()
    elapsed, kern_us, host_diag = time_evaluation(eng, states, args.steps, args.warmup, args.clock_warmup_s, torch, dd, dev)
    eng.close()
    kern_us_max = float(all_reduce_max(torch, dd, [kern_us], dev)[0])

    # ---- N > 1: the weak form beside it — every rank a full C4-size shard of one N·F-keyframe trajectory ---------------
    weak = None
    if world > 1:
        pw, images_w = synth.c4_shard(dev, rank=rank, world=world, n_frames=F, n_points=Np, K=K)
        ew = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=dev_index, huber_width=9.0)
        ew.set_problem(pw, images_device_ptr=images_w.data_ptr())
        sw = make_states(pw, torch, dev, 7 + rank)
        el_w, kern_w, _ = time_evaluation(ew, sw, args.steps, args.warmup, args.clock_warmup_s, torch, dd, dev)
        ew.close()
        del images_w
        weak = {"value": world * pw.n_blocks * args.steps / el_w, "unit": "blocks/s", "ms_per_step": 1e3 * el_w / args.steps,
                "blocks_per_rank": pw.n_blocks, "kernel_avg_us_rank0": kern_w,
                "note": f"weak scaling: rank r evaluates host keyframes [r*{F}, (r+1)*{F}) of one {world * F + K}-keyframe "
                        f"trajectory ({pw.n_blocks} blocks per GPU), no data-path collective"}
    shard8 = None
    if world == 1 and not args.no_shard_leg:  # one rank's step of the C4 problem split 8 ways, on this GPU
        p8, _, _ = D.shard_problem(full, 8, 0)
        e8 = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=dev_index, huber_width=9.0)
        e8.set_problem(p8, images_device_ptr=images.data_ptr())
        st8 = make_states(p8, torch, dev, 7)
        el8, k8, _ = time_evaluation(e8, st8, args.steps, args.warmup, args.clock_warmup_s, torch, None, dev)
        e8.close()
        bpb8 = algorithmic_bytes_per_block(p8.P, K, p8.n_frames, p8.n_points, p8.n_blocks)
        shard8 = {"blocks": p8.n_blocks, "ms_per_step": 1e3 * el8 / args.steps, "kernel_avg_us": k8,
                  "hbm_frac": bpb8 * p8.n_blocks / (k8 * 1e-6) / 1e9 / HBM_PEAK_GBS,
                  "strong_scaling_ceiling_n8": (elapsed / args.steps) / (el8 / args.steps),
                  "note": "a 1/8 host-keyframe shard of the C4 problem (rank 0's share at N = 8) timed on one GPU: the "
                          "strong-scaling ceiling at N = 8 is the full problem's step over this step"}

    # ---- the Gauss-Newton leg: the C4 problem with rendered images (the solve the GPU tests pin against real Ceres) ----
    gn = None
    if args.gn_iterations > 0:
        gfull, gimages = synth.c4_shard(dev, n_frames=F, n_points=Np, K=K, texture="render")
        gpb = D.shard_problem(gfull, world, rank)[0] if world > 1 else gfull
        eng = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=dev_index, huber_width=9.0)
        eng.set_problem(gpb, images_device_ptr=gimages.data_ptr())
        eng.set_state(gpb.poses, gpb.rho)
        cp = None
        if world == 1 and not args.no_cpu_baseline:
            cp = synth.Problem(**{**gfull.__dict__, "images": gimages.cpu().numpy()})
        try:
            gn = gn_benchmark(eng, gpb, args.gn_iterations, torch, dd, dev, world, cp, host_cores()["usable"])
        except Exception as ex:  # a secondary leg: report it, keep the headline line (every rank raises alike)
            if world == 1:
                raise
            gn = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        eng.close()
        del gimages

    c3 = None
    if world == 1 and not args.no_c3 and args.gn_iterations > 0:
        c3 = gn_c3(args.gn_iterations, torch, dev_index, dev)
    c5 = None
    if world == 1 and not args.no_c5:
        c5 = c5_eval(full, images, states, args.steps, args.warmup, args.clock_warmup_s, torch, dev_index, dev,
                     args.gn_iterations)

    if rank == 0:
        total_blocks = full.n_blocks
        ms_per_step = 1e3 * elapsed / args.steps
        value = total_blocks * args.steps / elapsed
        bpb = algorithmic_bytes_per_block(pb.P, K, pb.n_frames, pb.n_points, pb.n_blocks)
        achieved = bpb * pb.n_blocks / (kern_us * 1e-6) / 1e9
        traffic, traffic_info = None, None
        if world == 1 and not args.no_live_traffic:
            traffic, traffic_info = measure_traffic(args, pb.n_blocks)
        if traffic is None:  # fall back to the committed profile of the same workload
            reason = traffic_info
            tf = os.path.join(ROOT, "profiles", "traffic_photometric_block_kernel.json")
            if os.path.exists(tf):
                try:
                    tj = json.load(open(tf))
                    if tj.get("n_blocks") == pb.n_blocks and tj.get("P") == pb.P:
                        traffic = tj.get("hbm_bytes_per_launch")
                        traffic_info = {"source": "profiles/traffic_photometric_block_kernel.json (committed rocprofv3 passes)",
                                        "live_measurement": reason}
                except Exception:
                    traffic = None
        cpu = None
        c2 = None
        if world == 1 and not args.no_cpu_baseline:
            images_host = images.cpu().numpy()
            cpu = cpu_baseline(full, images_host, args.cpu_seconds)
            if not args.no_c2:
                try:
                    c2 = c2_dropin(full, images_host, host_cores()["usable"])
                except Exception as ex:  # a secondary leg: report it, keep the headline line
                    c2 = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        stream_peak = stream_copy_peak(torch, dev, achieved)
        # the GN leg's collective, as the leg chooses it (torch.distributed between trials unless PBA_BENCH_GN_COMM=1)
        gn_comm = ("device-steered RCCL loop" if world > 1 and dist.get_backend() == "nccl"
                   and os.environ.get("PBA_BENCH_GN_COMM", "0") == "1" else "torch.distributed between trials")
        out = {
            "metric": "photometric residual+jacobian blocks/sec",
            "value": value,
            "unit": "blocks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"C4: one synthetic problem of {F} host keyframes x {Np} points x {pb.P}-px patch x {K} "
                            f"targets = {total_blocks} residual blocks, {full.width}x{full.height} u8 images, pinhole" +
                            (f", split by host keyframe over {world} GPUs (rank 0: {pb.n_blocks} blocks)" if world > 1 else "") +
                            "; one step = full r + tangent-J evaluation (Ceres-mode records) at a new HBM-resident state",
                "keyframes": F, "points": Np, "patch": pb.P, "targets_per_point": K,
                "blocks_total": total_blocks, "blocks_rank0": pb.n_blocks, "valid_blocks_rank0": int(valid.sum()),
                "parallelism": f"host-keyframe shards x{world} (evaluation: no data-path collective; "
                               + (f"GN: all-reduce of the reduced camera system — {gn_comm})" if world > 1
                                  else "GN: one GPU)"),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "photometric_block_kernel<pinhole,8>",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_detail": traffic_info,
                "bytes_per_block_alg": bpb,
                "kernel_avg_us": kern_us,
                "kernel_avg_us_max_over_ranks": kern_us_max,
                **stream_peak,
                **({"note": "rank 0's shard: its algorithmic bytes over its launch duration"} if world > 1 else {}),
            },
            "cpu_baseline": cpu,
            "c2": c2,
            "gn": gn,
            "gn_c3": c3,
            "c5": c5,
            "weak": weak,
            "shard8": shard8,
            "host": {k: round(v, 2) for k, v in host_diag.items()},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
