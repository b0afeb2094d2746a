"""Worker bodies of the multi-process (gloo) tests; a module of its own so spawned ranks can import it."""
from __future__ import annotations

import importlib
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def exchange_worker(rank: int, world: int, port: int, case: dict, out):
    """Rank body: shard, per-rank partial reduced system (dense restatement of the engine's export), the
    exchange through distributed.TorchAllReduce over gloo, finalisation; reports max errors vs the
    single-process reference."""
    try:
        import numpy as np
        import torch.distributed as dist

        import gn_reference as GR
        synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
        D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if case.get("backend", "gloo") == "nccl":  # RCCL: one rank per device
            torch.cuda.set_device(0)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        pb = synth.make_problem(kind=case["kind"], n_frames=case["n_frames"], n_points=case["n_points"],
                                width=376, height=240, seed=case["seed"], border=12, obs_sigma=0.3)
        lam, huber, fixed = case["lam"], case["huber"], tuple(case["fixed"])
        sub, pids, bids = D.shard_problem(pb, world, rank)
        S, gS, gd, dA, obs = GR.partial_system(sub, sub.poses, sub.rho, huber, lam)
        _, _, cost = GR.linearize(sub, sub.poses, sub.rho, huber, ())
        n = 6 * pb.n_frames
        body = np.concatenate([S.ravel(), gS, gd, dA, obs])
        ar = D.TorchAllReduce(body.size + 8, "cpu")
        ar.buf[:body.size] = ar.torch.from_numpy(body)
        ar.buf[body.size] = cost
        ar(ar.ptr, body.size)                       # the system
        ar(ar.ptr + 8 * body.size, 1)               # a scalar slot (offset path of the callback)
        tot = ar.buf.numpy()
        S_sum = tot[:n * n].reshape(n, n)
        o = n * n
        gS_sum, dA_sum, obs_sum = tot[o:o + n], tot[o + 2 * n:o + 3 * n], tot[o + 3 * n:o + 3 * n + pb.n_frames]
        S_fin, gS_fin = GR.finalize_system(S_sum, gS_sum, dA_sum, obs_sum, lam, fixed)
        H, g, cost_full = GR.linearize(pb, pb.poses, pb.rho, huber, fixed)
        S_ref, gS_ref, dp_ref, dl_ref, _ = GR.schur_step(H, g, pb.n_frames, lam, fixed)
        dp = np.linalg.solve(S_fin, -gS_fin)
        out.put((rank, {
            "S": float(np.abs(S_fin - S_ref).max() / np.abs(S_ref).max()),
            "g": float(np.abs(gS_fin - gS_ref).max() / (np.abs(gS_ref).max() + 1e-300)),
            "dp": float(np.linalg.norm(dp - dp_ref.ravel()) / np.linalg.norm(dp_ref)),
            "cost": float(abs(tot[body.size] - cost_full) / cost_full),
            "n_points": int(len(pids)), "n_blocks": int(len(bids)),
        }))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        out.put((rank, traceback.format_exc()))
        raise


def solve_worker(rank: int, world: int, port: int, case: dict, out):
    """GPU rank body (one process per rank, all on cuda:0, gloo group): the rank's host-keyframe shard in its own
    engine, the LM loop of pba_solve_distributed with the reduced camera system summed by
    distributed.solve_distributed (TorchAllReduce over torch.distributed, staged through the host for gloo) — the
    path bench.py --gpus N runs with RCCL.  Reports the summary and the shard's final state."""
    try:
        import numpy as np
        import torch
        import torch.distributed as dist

        synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
        E = importlib.import_module("photometric-bundle-adjustment_amd.engine")
        D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if case.get("backend", "gloo") == "nccl":  # RCCL: one rank per device
            torch.cuda.set_device(0)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        pb = synth.make_problem(kind=case["kind"], n_frames=case["n_frames"], n_points=case["n_points"],
                                width=376, height=240, seed=case["seed"], border=12, obs_sigma=0.3)
        pb.poses[:2] = pb.poses_gt[:2]
        sub, pids, _ = D.shard_problem(pb, world, rank)
        eng = E.Engine(pb.kind, pb.model, device=0, huber_width=case["huber"])
        try:
            eng.set_problem(sub)
            eng.set_fixed_frames(np.array(case["fixed"], np.int32))
            eng.set_state(sub.poses, sub.rho)
            # comm False: the host-callback loop (TorchAllReduce); None: the RCCL communicator for an nccl group
            s = D.solve_distributed(eng, device=torch.device("cuda", 0), comm=case.get("comm"),
                                    max_iterations=case["iters"])
            poses, rho = eng.get_state()
        finally:
            eng.close()
        out.put((rank, {"summary": s, "poses": poses, "rho": rho, "pids": pids}))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        out.put((rank, traceback.format_exc()))
        raise


def agree_worker(rank: int, world: int, port: int, values_by_rank: list, out):
    """Rank body of bench.ranks_agree over gloo: each rank contributes its own values."""
    try:
        import torch
        import torch.distributed as dist
        bench = importlib.import_module("bench")
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out.put((rank, bench.ranks_agree(torch, dist, values_by_rank[rank], "cpu")))
        dist.destroy_process_group()
    except BaseException:
        out.put((rank, traceback.format_exc()))
