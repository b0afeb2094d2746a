#!/usr/bin/env python3
"""bench.py — photometric residual+Jacobian blocks/s on MI355X (BASELINE.json metric, configs[3] workload).

Workload per GPU (BASELINE.json configs[3] / SURVEY.md §8d C4): a synthetic 1000-keyframe × 100k-point problem,
8-pixel DSO pattern, every point observed by the 4 keyframes after its host → 400,000 residual blocks
(3.2 M pixel residuals), 752×480 u8 images (361 MB), pinhole camera.  One step = one full evaluation of
every block's residuals and tangent Jacobians (Ceres-mode records, include/pba.h) at a new state that is
already resident in HBM: state copy + pair kernel + block kernel, all on the engine stream.

Multi-GPU (launched by torch.distributed.run): residual blocks shard by host keyframe — each rank owns its
own 1000-host-keyframe shard (weak scaling) and evaluates it with no data-path collective (the Ceres-mode
evaluation has no exchange step).  Timing: W warmup steps, then exactly K steps bracketed by
barrier + synchronize; the MAX over ranks is reported; value = all ranks' blocks ÷ that time.

Also reported: the block kernel's roofline position (algorithmic bytes ÷ HIP-event-timed kernel duration,
on the engine stream) and a CPU baseline (the oracle's dual-number AutoDiff evaluation — the reference's
Ceres AutoDiff arithmetic restated — timed on a bounded sample of the same workload on this host).
"""
from __future__ import annotations

import argparse
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def gpu_noise_images(torch, n, H, W, seed, device):
    """Independent smooth random u8 textures, generated on the GPU (content irrelevant for throughput)."""
    import torch.nn.functional as F
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty((n, H, W), dtype=torch.uint8, device=device)
    chunk = 100
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        coarse = torch.rand((m, 1, H // 8 + 2, W // 8 + 2), generator=g, device=device) * 215 + 20
        img = F.interpolate(coarse, size=(H + 16, W + 16), mode="bilinear", align_corners=False)[:, 0, :H, :W]
        img = img + torch.randn((m, H, W), generator=g, device=device) * 2.0
        out[s:s + m] = img.round().clamp(0, 255).to(torch.uint8)
    return out


def algorithmic_bytes_per_block(P: int, K: int, n_frames: int, n_points: int, n_blocks: int) -> float:
    """SURVEY.md §8d, Ceres mode, fp32 records, fused state (pba_evaluate_state_device): inputs + taps + outputs
    per block (formula in DESIGN.md §3)."""
    idx = 16.0                                 # block record {point, host, target, cameras} (int32 × 4)
    point = (16.0 + 8.0 + 4.0 * P) / K         # u_ref (2×f64) + ρ (f64) + I_h (P×f32), shared by the point's K blocks
    state = (56.0 * 2 * n_frames + 8.0 * n_points) / n_blocks  # pose reads (L2-shared) + adopted state written
    taps = 4.0 * P                             # 4 u8 bilinear taps per pixel (gradient from the same taps)
    out = 4.0 * 14 * P + 4.0 + 1.0             # record [r | J_h | J_t | J_ρ] + cost + valid
    return idx + point + state + taps + out


def cpu_baseline(pb, images_host, budget_s: float, threads: int):
    """Oracle (dual-number AutoDiff, as Ceres' AutoDiffCostFunction) on a bounded sample of the workload:
    repeated passes over a block sample until ~budget_s of CPU work has been timed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes
    import oracle as O
    pbc = synth.Problem(**{**pb.__dict__, "images": images_host})
    L = O.lib()
    keep = O._Keep()
    s = O.make_problem_struct(pbc, keep)
    poses = keep(pbc.poses, np.float64)
    rho = keep(pbc.rho, np.float64)
    out = np.zeros((pbc.n_blocks, 14 * pbc.P), np.float64)
    valid = np.zeros(pbc.n_blocks, np.uint8)

    def run(n):
        s.n_blocks = n
        t0 = time.perf_counter()
        rc = L.orc_evaluate(ctypes.byref(s), poses.ctypes.data, rho.ctypes.data, 1, out.ctypes.data,
                            valid.ctypes.data, threads)
        assert rc == 0
        return time.perf_counter() - t0

    n = min(pbc.n_blocks, 20000)
    rate = n / max(run(n), 1e-9)
    n = int(min(pbc.n_blocks, max(20000, rate * budget_s)))
    passes, total, done = 0, 0.0, 0
    while total < budget_s and passes < 1000:
        total += run(n)
        done += n
        passes += 1
    return {"value": done / total, "unit": "blocks/s", "cores": threads, "kind": "port",
            "sample": f"{passes} pass(es) over the first {n} of the {pbc.n_blocks} blocks of the same problem "
                      f"(r + tangent J, P={pbc.P}), {total:.1f} s on {threads} host threads; oracle/oracle.cpp "
                      f"Jet<15> dual-number AutoDiff (the reference's Ceres AutoDiff arithmetic, restated)"}


def all_reduce_max(torch, dist, values, dev):
    """MAX over ranks of a few host scalars (on the device for RCCL, through the host for gloo)."""
    on_dev = dist is not None and dist.get_backend() == "nccl"
    t = torch.tensor(values, dtype=torch.float64, device=dev if on_dev else "cpu")
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu()


def gn_benchmark(eng, iters, torch, dist, dev, world):
    """ms per Levenberg-Marquardt iteration (BASELINE.json metric, part 2) on the same problem, through the
    engine's own LM loop (pba_solve; pba_solve_distributed with an RCCL all-reduce of the banded reduced
    system for N>1).  An iteration = Schur complement + reduced-system solve + candidate cost, plus the
    next linearisation (r, J, Huber, JᵀJ/Jᵀr partials) after an accepted step; function_tolerance = 0 so
    exactly `iters` iterations run.  Two keyframes are held constant (the reference's fixed cameras)."""
    D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")
    eng.set_fixed_frames(np.array([0, 1], np.int32))
    eng.gn_linearize()  # symbolic analysis (once per problem structure), outside the timed region
    opts = dict(max_iterations=iters, function_tolerance=0.0)
    if world > 1:
        band = D.global_band(eng, None, dev)
        ar = D.TorchAllReduce(eng.gn_exchange_size(band), dev)
        eng.solve_distributed(band, ar.ptr, ar, max_iterations=1)  # warm-up
        dist.barrier()
        torch.cuda.synchronize()
        s = eng.solve_distributed(band, ar.ptr, ar, **opts)
        exchange_mb = 8.0 * eng.gn_exchange_size(band) / 1e6
    else:
        eng.solve(max_iterations=1)  # warm-up
        torch.cuda.synchronize()
        s = eng.solve(**opts)
        exchange_mb = None
    t = all_reduce_max(torch, dist, [s["total_ms"], s["linearize_ms"], s["solve_ms"], s["cost_ms"]], dev)
    n = max(s["iterations"], 1)
    return {"ms_per_iteration": float(t[0]) / n, "iterations": s["iterations"], "accepted": s["successful_steps"],
            "breakdown_ms_per_iteration": {"linearize_ms": float(t[1]) / n, "step_ms": float(t[2]) / n,
                                           "cost_ms": float(t[3]) / n},
            "exchange_mb_per_iteration": exchange_mb,
            "note": "host wall clock of the engine's LM loop (pba_solve" + (f"_distributed, {dist.get_backend()} all-reduce "
                    "(nccl = RCCL) of the banded reduced camera system + 3 scalars per iteration" if world > 1 else "") +
                    "); noise-textured images, so the steps are not expected to converge — timing only"}


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
            "note": "host wall clock of pba_solve (Ceres LM logic on the host, every kernel on the device)"}


DISK21 = np.array([(dx, dy) for dy in range(-2, 3) for dx in range(-2, 3) if dx * dx + dy * dy <= 5], np.float32)


def c5_eval(pb, images, states, steps, torch, dev_index, dev):
    """BASELINE.json configs[4] (C5) on this GPU's synthetic C4 shard: 21-pixel pattern (the radius-√5 disk), records
    stored as fp16 (PBA_RECORD_F16), and a 3-level image pyramid built on the device.  Same one-launch step as the
    headline (evaluate at a new HBM-resident state); the full EuRoC sequence is not in the container, so the
    images are the shard's synthetic ones."""
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

        def step(i):
            p, r = states[i & 1]
            eng.evaluate_state_device(p.data_ptr(), r.data_ptr(), True, sync=False)

        for i in range(max(steps // 4, 5)):
            step(i)
        eng.synchronize()
        eng.enable_kernel_timing(True)
        eng.kernel_timing()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        eng.synchronize()
        el = time.perf_counter() - t0
        kern_ms, launches = eng.kernel_timing()
    finally:
        eng.close()
    P = DISK21.shape[0]
    return {"config": f"C5-style: the C4 shard with a {P}-px pattern, fp16 records, 3-level pyramid (synthetic images)",
            "blocks_per_s": pb.n_blocks * steps / el, "ms_per_step": 1e3 * el / steps,
            "kernel_avg_us": 1e3 * kern_ms / max(launches, 1), "record_format": "f16", "P": P,
            "record_bytes_per_block": 2 * 14 * P, "pyramid_levels": 3, "pyramid_build_ms": pyr_ms}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--clock-warmup-s", type=float, default=0.3)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--points", type=int, default=100000)
    ap.add_argument("--targets", type=int, default=4)
    ap.add_argument("--width", type=int, default=752)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gn-iterations", type=int, default=10)
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 Gauss-Newton measurement (configs[2])")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5-style 21-px / fp16 / pyramid measurement")
    args = ap.parse_args()

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
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    # ---- problem shard of this rank --------------------------------------------------------------------
    # Global keyframe indexing: rank r hosts keyframes [r·F, (r+1)·F); its points are observed by the K
    # keyframes after their host, so the last K hosts of a shard reach into the next shard (coupled
    # reduced system for the multi-GPU Gauss-Newton).  Every rank holds all NF = world·F + K poses.
    K, F, Np = args.targets, args.frames, args.points
    NF = world * F + K
    pb = synth.make_problem(n_frames=F + K, n_points=Np, K=K, width=args.width, height=args.height, kind="photometric",
                            model="pinhole", texture="noise", with_images=False, seed=42 + rank)
    off = rank * F
    pb.point_host = (pb.point_host + off).astype(np.int32)
    pb.block_target = (pb.block_target + off).astype(np.int32)
    pb.frame_cam = np.zeros(NF, np.int32)
    prng = np.random.default_rng(99)  # same global poses on every rank
    pb.poses_gt = synth.trajectory(NF)
    pb.poses = synth.se3_plus(pb.poses_gt, 3e-3 * prng.normal(0, 1, (NF, 6)))
    images = torch.zeros((NF, args.height, args.width), dtype=torch.uint8, device=dev)
    images[off:off + F + K] = gpu_noise_images(torch, F + K, args.height, args.width, 1234 + rank, dev)
    host = torch.from_numpy(pb.point_host.astype(np.int64)).to(dev)
    uu = torch.from_numpy(pb.u_ref[:, 0].astype(np.int64)).to(dev)[:, None] + torch.from_numpy(pb.pattern[:, 0].astype(np.int64)).to(dev)
    vv = torch.from_numpy(pb.u_ref[:, 1].astype(np.int64)).to(dev)[:, None] + torch.from_numpy(pb.pattern[:, 1].astype(np.int64)).to(dev)
    # integer u_ref and integer pattern → the bilinear host sample is exactly the pixel value
    pb.host_intensity = images[host[:, None], vv, uu].float().cpu().numpy()

    eng = engine_mod.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=dev_index, huber_width=9.0)
    eng.set_problem(pb, images_device_ptr=images.data_ptr())
    n_blocks = pb.n_blocks
    rng = np.random.default_rng(7 + rank)
    states = []
    for _ in range(2):  # alternate two perturbed states so every step evaluates a new point
        poses = synth.se3_plus(pb.poses, 1e-3 * rng.normal(0, 1, (NF, 6)))
        rho = pb.rho * (1 + 0.01 * rng.normal(0, 1, Np))
        states.append((torch.from_numpy(poses).to(dev), torch.from_numpy(rho).to(dev)))
    eng.set_state_device(states[0][0].data_ptr(), states[0][1].data_ptr())
    eng.evaluate(True)
    _, valid = eng.records()

    def step(i):  # one launch: pairs formed in the block prologue, state adopted by the same launch
        p, r = states[i & 1]
        eng.evaluate_state_device(p.data_ptr(), r.data_ptr(), True, sync=False)

    # clock warm-up (untimed, on top of the W warmup steps): the GPU's clocks take ~0.1 s of load to ramp, and
    # a short run measured 70 µs per step cold against 54 µs warm (profiles/r1_bench_c4_v27.json)
    t_w = time.perf_counter()
    i = 0
    while time.perf_counter() - t_w < args.clock_warmup_s:
        for _ in range(20):
            step(i)
            i += 1
        eng.synchronize()
    for i in range(args.warmup):
        step(i)
    eng.synchronize()
    # diagnostic (not the metric): the same steps without the per-launch timing events, and the host's enqueue rate
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    t_enq = time.perf_counter()
    eng.synchronize()
    host_diag = {"us_per_step_without_events": 1e6 * (time.perf_counter() - t0) / args.steps,
                 "enqueue_us_per_step_without_events": 1e6 * (t_enq - t0) / args.steps}
    eng.enable_kernel_timing(True)
    eng.kernel_timing()  # reset
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    host_diag["enqueue_us_per_step"] = 1e6 * (time.perf_counter() - t0) / args.steps
    eng.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kern_ms, launches = eng.kernel_timing()
    t = all_reduce_max(torch, dist if world > 1 else None, [elapsed, kern_ms / max(launches, 1)], dev)
    elapsed_max, kern_avg_ms = float(t[0]), float(t[1])

    gn = None
    if args.gn_iterations > 0:
        eng.set_state(pb.poses, pb.rho)
        gn = gn_benchmark(eng, args.gn_iterations, torch, dist if world > 1 else None, dev, world)
    c3 = None
    if world == 1 and not args.no_c3 and args.gn_iterations > 0:
        c3 = gn_c3(args.gn_iterations, torch, dev_index, dev)
    c5 = None
    if world == 1 and not args.no_c5:
        eng.close()  # the headline engine's buffers are not needed any more
        c5 = c5_eval(pb, images, states, args.steps, torch, dev_index, dev)

    if rank == 0:
        ms_per_step = 1e3 * elapsed_max / args.steps
        total_blocks = n_blocks * world * args.steps
        value = total_blocks / elapsed_max
        bpb = algorithmic_bytes_per_block(pb.P, K, NF, Np, n_blocks)
        achieved = bpb * n_blocks / (kern_avg_ms * 1e-3) / 1e9
        traffic = None
        tf = os.path.join(ROOT, "profiles", "traffic_photometric_block_kernel.json")
        if os.path.exists(tf):
            try:
                tj = json.load(open(tf))
                if tj.get("n_blocks") == n_blocks and tj.get("P") == pb.P:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            threads = max(1, min(16, os.cpu_count() or 1))
            cpu = cpu_baseline(pb, images.cpu().numpy(), args.cpu_seconds, threads)  # N=1: all NF frames local
        out = {
            "metric": "photometric residual+jacobian blocks/sec",
            "value": value,
            "unit": "blocks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"C4 shard per GPU: synthetic {F} host keyframes x {Np} points x {pb.P}-px patch x {K} targets "
                            f"= {n_blocks} residual blocks, {args.width}x{args.height} u8 images, pinhole; one step = "
                            f"full r + tangent-J evaluation (Ceres-mode records) at a new HBM-resident state",
                "keyframes": F, "keyframes_global": NF, "points": Np, "patch": pb.P, "targets_per_point": K, "blocks_per_gpu": n_blocks,
                "valid_blocks": int(valid.sum()), "parallelism": f"host-keyframe shards x{world} (evaluation: no data-path collective; "
                                               f"GN: RCCL all-reduce of the reduced camera system)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "photometric_block_kernel<pinhole,8>",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "bytes_per_block_alg": bpb,
                "kernel_avg_us": kern_avg_ms * 1e3,
            },
            "cpu_baseline": cpu,
            "gn": gn,
            "gn_c3": c3,
            "c5": c5,
            "host": {k: round(v, 2) for k, v in host_diag.items()},
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
