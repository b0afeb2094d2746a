"""GPU parity of the multi-GPU Gauss-Newton path (include/pba.h §8e) with shard engines on one device:
the summed exchange of two/three host-keyframe shards must reproduce the single-engine step
(pba_gn_step on the whole problem) and pba_solve_distributed must take the same LM decisions as pba_solve.

Tolerances: identical arithmetic up to the order of the fp64 sums (per-rank sums, then across ranks), so
steps agree to 1e-6 relative, model decreases and costs to 1e-8 relative; LM runs to 1e-6 in final cost
and 1e-6 in poses."""
import importlib
import threading

import numpy as np
import pytest

import gn_reference as GR
from helpers import engine_module, synth

pytestmark = pytest.mark.gpu
E = engine_module()
D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")


def engine_for(pb, huber, fixed):
    eng = E.Engine(pb.kind, pb.model, huber_width=huber)
    eng.set_problem(pb)
    eng.set_fixed_frames(np.array(fixed, np.int32))
    eng.set_state(pb.poses, pb.rho)
    return eng


def shards(pb, world, huber, fixed):
    out = []
    for r in range(world):
        sub, pids, bids = D.shard_problem(pb, world, r)
        out.append((engine_for(sub, huber, fixed), pids))
    return out


@pytest.mark.parametrize("kind,model,huber,world", [(0, 0, 9.0, 2), (1, 0, 1.0, 2), (0, 1, 9.0, 3), (1, 1, 1.0, 3)])
@pytest.mark.parametrize("lam", [1e-4, 1e-1])
def test_exchange_matches_single_engine_step(kind, model, huber, world, lam):
    import torch
    pb = synth.make_problem(kind=kind, model=model, n_frames=14, n_points=140, width=376, height=240,
                            seed=71 + model, border=12, obs_sigma=0.3)
    fixed = (0,)
    with engine_for(pb, huber, fixed) as full:
        c_full = full.gn_linearize()
        m_full, st_full = full.gn_step(lam)
        dp_full, dr_full = full.gn_last_step()
    assert st_full == 0
    sh = shards(pb, world, huber, fixed)
    try:
        costs = [e.gn_linearize() for e, _ in sh]
        assert abs(sum(costs) - c_full) <= 1e-8 * c_full
        band = max(e.gn_band() for e, _ in sh)
        n = sh[0][0].gn_exchange_size(band)
        bufs = [torch.zeros(n, dtype=torch.float64, device="cuda") for _ in sh]
        for (e, _), b in zip(sh, bufs):
            e.gn_step_export(lam, band, b.data_ptr())
        tot = bufs[0].clone()
        for b in bufs[1:]:
            tot += b
        torch.cuda.synchronize()
        model_pts, dr = 0.0, np.zeros(pb.n_points)
        mps = []
        for e, pids in sh:
            mp, mq, st = e.gn_step_import(lam, band, tot.data_ptr())
            assert st == 0
            mps.append(mp)
            model_pts += mq
            dp, drs = e.gn_last_step()
            assert np.linalg.norm(dp - dp_full) <= 1e-6 * np.linalg.norm(dp_full)
            dr[pids] = drs
        assert max(mps) - min(mps) <= 1e-12 * abs(mps[0])  # identical pose step on every rank
        assert abs(mps[0] + model_pts - m_full) <= 1e-8 * abs(m_full)
        np.testing.assert_allclose(dr, dr_full, rtol=1e-6, atol=1e-12 * np.abs(dr_full).max())
    finally:
        for e, _ in sh:
            e.close()
    # and against the dense reference
    H, g, _ = GR.linearize(pb, pb.poses, pb.rho, huber, fixed)
    _, _, dp_ref, _, _ = GR.schur_step(H, g, pb.n_frames, lam, fixed)
    assert np.linalg.norm(dp_full - dp_ref) <= 1e-3 * np.linalg.norm(dp_ref)


@pytest.mark.parametrize("kind,model,huber", [(0, 0, 9.0), (1, 0, 1.0)])
def test_solve_distributed_matches_solve(kind, model, huber):
    """Three shard engines in three threads, summed in-process: same LM trajectory as one engine."""
    import torch
    pb = synth.make_problem(kind=kind, model=model, n_frames=16, n_points=400, width=376, height=240, seed=81,
                            border=12, obs_sigma=0.3)
    pb.poses[:2] = pb.poses_gt[:2]
    fixed = (0, 1)
    with engine_for(pb, huber, fixed) as full:
        ref = full.solve(max_iterations=12)
        poses_ref, rho_ref = full.get_state()
    world = 3
    sh = shards(pb, world, huber, fixed)
    try:
        band = max(e.gn_band() for e, _ in sh)
        n = sh[0][0].gn_exchange_size(band)
        bufs = [torch.zeros(n, dtype=torch.float64, device="cuda") for _ in sh]
        comm = D.InProcessAllReduce(bufs, timeout=120)
        res, errs = [None] * world, []

        def run(r):
            try:
                res[r] = sh[r][0].solve_distributed(band, bufs[r].data_ptr(), comm.rank(r), max_iterations=12)
            except BaseException as ex:
                errs.append(ex)
                comm.barrier.abort()

        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(300)
        assert not errs, errs
        rho = np.zeros(pb.n_points)
        for r, (e, pids) in enumerate(sh):
            s = res[r]
            assert s["iterations"] == ref["iterations"] and s["successful_steps"] == ref["successful_steps"], (s, ref)
            assert abs(s["initial_cost"] - ref["initial_cost"]) <= 1e-8 * ref["initial_cost"]
            assert abs(s["final_cost"] - ref["final_cost"]) <= 1e-6 * ref["final_cost"], (s, ref)
            poses, rr = e.get_state()
            np.testing.assert_allclose(poses, poses_ref, atol=1e-6)
            rho[pids] = rr
        np.testing.assert_allclose(rho, rho_ref, rtol=1e-6)
        assert ref["final_cost"] < ref["initial_cost"]
    finally:
        for e, _ in sh:
            e.close()


@pytest.mark.parametrize("kind,huber", [(0, 9.0), (1, 1.0)])
def test_two_process_gloo_solve_matches_solve(kind, huber):
    """Two processes, one engine each (both on cuda:0), a world-size-2 gloo group: distributed.solve_distributed
    (the engine's export → torch.distributed all-reduce → import, every scalar of the LM decision all-reduced) takes
    the same LM trajectory as one engine on the whole problem — the bench's multi-GPU GN path with gloo standing in
    for RCCL (two ranks cannot share a device under RCCL)."""
    import socket

    import torch.multiprocessing as mp

    import dist_workers
    case = dict(kind=kind, n_frames=16, n_points=400, seed=83, huber=huber, fixed=[0, 1], iters=10)
    pb = synth.make_problem(kind=kind, n_frames=16, n_points=400, width=376, height=240, seed=83, border=12,
                            obs_sigma=0.3)
    pb.poses[:2] = pb.poses_gt[:2]
    with engine_for(pb, huber, (0, 1)) as full:
        ref = full.solve(max_iterations=10)
        poses_ref, rho_ref = full.get_state()
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=dist_workers.solve_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = {}
        for _ in range(2):
            r, v = q.get(timeout=240)
            res[r] = v
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    rho = np.zeros(pb.n_points)
    for r in range(2):
        assert isinstance(res[r], dict), res[r]
        s = res[r]["summary"]
        assert s["iterations"] == ref["iterations"] and s["successful_steps"] == ref["successful_steps"], (s, ref)
        assert abs(s["initial_cost"] - ref["initial_cost"]) <= 1e-8 * ref["initial_cost"]
        assert abs(s["final_cost"] - ref["final_cost"]) <= 1e-6 * ref["final_cost"], (s, ref)
        np.testing.assert_allclose(res[r]["poses"], poses_ref, atol=1e-6)
        rho[res[r]["pids"]] = res[r]["rho"]
    np.testing.assert_allclose(rho, rho_ref, rtol=1e-6)
    assert ref["final_cost"] < ref["initial_cost"]


def test_band_too_small_is_rejected():
    import torch
    pb = synth.make_problem(kind="geometric", n_frames=12, n_points=60, seed=5)
    with engine_for(pb, 1.0, (0,)) as e:
        e.gn_linearize()
        b = e.gn_band()
        with pytest.raises(E.PbaError, match="band"):
            e.gn_exchange_size(b - 1)
        n = e.gn_exchange_size(b)
        assert n == 12 * ((E_band(b) + 1) * 36 + 24) + 8


def E_band(b):
    return 4 if b <= 4 else (8 if b <= 8 else 16)
