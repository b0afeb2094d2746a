"""GPU parity: the HIP engine (through the C ABI) against the oracle and the reference-compiled fixtures.

Tolerances (fp32 device vs double oracle; rationale in tests/helpers.compare_records and DESIGN.md §Parity):
  photometric residual |Δr| ≤ 1e-4 intensity units, geometric ≤ 1e-5 px (tests/helpers.py)
  Jacobians            per block and parameter block, max|ΔJ| ≤ 1e-5 × max|J_ref| (BASELINE north star: 1e-5 relative)
                       (photometric pixels within 2e-3 px of a bilinear cell edge excluded)
  validity flags       identical
"""
import numpy as np
import pytest

import oracle as O
from helpers import R_ATOL_GEOMETRIC, R_ATOL_PHOTOMETRIC, BLOCK_FIXTURES, compare_records, engine_module, load_golden, projected_uv, synth

pytestmark = pytest.mark.gpu
E = engine_module()


def run_engine(pb, jac=True, huber=0.0, poses=None, rho=None):
    with E.Engine(pb.kind, pb.model, huber_width=huber) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses if poses is None else poses, pb.rho if rho is None else rho)
        eng.evaluate(jac)
        rec, valid = eng.records()
        costs = eng.block_costs()
    return rec, valid, costs


@pytest.mark.parametrize("name", BLOCK_FIXTURES)
def test_golden_fixture_parity(name):
    pb, z = load_golden(name)
    rec, valid, _ = run_engine(pb)
    uv = projected_uv(pb) if pb.kind == 0 else None
    ref, vref = O.evaluate(pb)
    st = compare_records(pb.kind, pb.R, rec, ref, valid, vref, uv)
    # and directly against the Sophus-harness expectations
    compare_records(pb.kind, pb.R, rec, z["expect_record"], valid, z["expect_valid"], uv)
    print(name, st)


CASES = [(k, m, s) for k in (0, 1) for m in (0, 1, 2, 3) for s in (1, 2)]


@pytest.mark.parametrize("kind,model,seed", CASES)
def test_random_problem_parity(kind, model, seed):
    pb = synth.make_problem(n_frames=9, n_points=300, width=376, height=240, kind=kind, model=model, seed=100 + seed,
                            texture="render" if seed == 1 else "noise", border=10)
    rec, valid, _ = run_engine(pb)
    ref, vref = O.evaluate(pb, n_threads=4)
    compare_records(kind, pb.R, rec, ref, valid, vref, projected_uv(pb) if kind == 0 else None)


@pytest.mark.parametrize("kind", [0, 1])
def test_residual_only_mode(kind):
    pb = synth.make_problem(n_frames=8, n_points=200, width=376, height=240, kind=kind, seed=7, border=10)
    full, v1, c1 = run_engine(pb, jac=True)
    ronly, v2, c2 = run_engine(pb, jac=False)
    assert np.array_equal(v1, v2)
    # separate kernel instantiations: the compiler may contract differently, so compare within tolerance
    np.testing.assert_allclose(full[:, :pb.R], ronly[:, :pb.R], atol=R_ATOL_PHOTOMETRIC if kind == 0 else R_ATOL_GEOMETRIC)
    np.testing.assert_allclose(c1, c2, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("kind,P", [(0, 8), (0, 21), (1, 2)])
def test_residual_read_back_paths(kind, P):
    """pba_get_residuals after a residual-only evaluation (the contiguous copy the Ceres adapter's LM candidates use) is
    bit-identical to the residual part of that evaluation's records; after a Jacobian evaluation it reads the records
    (pitched copy).  An asynchronous read-back of an earlier evaluation is not reported as arrived after a new one."""
    import ctypes as C
    pb = synth.make_problem(n_frames=8, n_points=200, width=376, height=240, kind=kind, seed=7, border=10)
    if kind == 0 and P != 8:
        disk = np.array([(dx, dy) for dy in range(-2, 3) for dx in range(-2, 3) if dx * dx + dy * dy <= 5], np.float32)
        pb = synth.Problem(**{**pb.__dict__, "pattern": disk, "host_intensity": None})
    with E.Engine(pb.kind, pb.model) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        for jac in (False, True):
            eng.evaluate(jac)
            rec, v_rec = eng.records()
            res, v_res = eng.residuals()
            assert np.array_equal(v_rec, v_res)
            assert np.array_equal(rec[:, :pb.R].view(np.uint32), res.reshape(pb.n_blocks, pb.R).view(np.uint32)), jac
        L, h = eng._L, eng._h
        L.pba_get_records_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
        L.pba_wait_records.argtypes = [C.c_void_p, C.c_int32]
        buf = C.c_void_p()
        assert L.pba_host_alloc(C.c_size_t(rec.nbytes + pb.n_blocks), C.byref(buf)) == 0
        try:
            assert L.pba_get_records_async(h, buf, C.c_void_p(buf.value + rec.nbytes), 64) == 0
            assert L.pba_wait_records(h, pb.n_blocks - 1) == 0
            got = np.frombuffer((C.c_float * rec.size).from_address(buf.value), np.float32).reshape(rec.shape)
            assert np.array_equal(got.view(np.uint32), rec.view(np.uint32))
            eng.evaluate(True)  # a new evaluation: the earlier read-back no longer describes the records
            assert L.pba_wait_records(h, 0) == -4  # PBA_ERR_NOT_READY
        finally:
            L.pba_host_free(buf)


@pytest.mark.parametrize("kind,huber", [(0, 0.0), (0, 9.0), (1, 1.0)])
def test_block_costs_match_oracle_huber(kind, huber):
    pb = synth.make_problem(n_frames=8, n_points=200, width=376, height=240, kind=kind, seed=8, border=10)
    rec, valid, costs = run_engine(pb, huber=huber)
    ref, vref = O.evaluate(pb, want_jac=False)
    for b in range(pb.n_blocks):
        if not vref[b]:
            assert costs[b] == 0
            continue
        c_ref, _ = O.huber_block(ref[b, :pb.R], huber)
        # bound implied by the residual tolerance: |Δ½Σr²| ≤ Σ|r|·δr (+ fp32 summation)
        r_tol = R_ATOL_PHOTOMETRIC if kind == 0 else R_ATOL_GEOMETRIC
        tol = r_tol * np.abs(ref[b, :pb.R]).sum() + 1e-5 * abs(c_ref) + 1e-5
        assert abs(costs[b] - c_ref) <= tol, (b, costs[b], c_ref)


def test_deterministic_and_state_update():
    pb = synth.make_problem(n_frames=10, n_points=500, width=376, height=240, seed=31, border=10)
    with E.Engine(0, 0) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        eng.evaluate()
        a, va = eng.records()
        eng.evaluate()
        b, vb = eng.records()
        np.testing.assert_array_equal(a, b)
        # new state on the same engine → matches a fresh oracle evaluation at that state
        eng.set_state(pb.poses_gt, pb.rho_gt)
        eng.evaluate()
        c, vc = eng.records()
    ref, vref = O.evaluate(pb, poses=pb.poses_gt, rho=pb.rho_gt)
    pb_gt = synth.Problem(**{**pb.__dict__, "poses": pb.poses_gt, "rho": pb.rho_gt})
    compare_records(0, pb.R, c, ref, vc, vref, projected_uv(pb_gt))


@pytest.mark.parametrize("kind", [0, 1])
def test_evaluate_states_device_batch(kind):
    """pba_evaluate_states_device: n evaluations enqueued by one call equal n pba_evaluate_state_device calls — the
    engine ends at the last state, its records are that state's, and an empty batch is a no-op."""
    import torch

    pb = synth.make_problem(kind=kind, n_frames=8, n_points=300, width=376, height=240, seed=43, border=10)
    dev = torch.device("cuda", 0)
    states = [(torch.from_numpy(np.ascontiguousarray(p)).to(dev), torch.from_numpy(np.ascontiguousarray(r)).to(dev))
              for p, r in ((pb.poses, pb.rho), (pb.poses_gt, pb.rho_gt), (pb.poses, pb.rho_gt))]
    with E.Engine(kind, 0) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        eng.evaluate_states_device([], [], True)
        eng.evaluate_states_device([p.data_ptr() for p, _ in states], [r.data_ptr() for _, r in states], True)
        a, va = eng.records()
        poses, rho = eng.get_state()
        np.testing.assert_array_equal(poses, pb.poses)
        np.testing.assert_array_equal(rho, pb.rho_gt)
        eng.evaluate_state_device(states[-1][0].data_ptr(), states[-1][1].data_ptr(), True)
        b, vb = eng.records()
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(va, vb)


@pytest.mark.parametrize("kind,model,extra_points", [(0, 0, 0), (0, 3, 0), (1, 0, 0), (0, 0, 40000)])
def test_evaluate_state_device_adopts(kind, model, extra_points):
    """pba_evaluate_state_device (one launch for photometric engines: pairs formed in the block prologue, state
    copied by the same launch) equals set_state + evaluate, matches the oracle at that state, and leaves the state
    adopted.  extra_points > 0 appends points without blocks (more state than lanes: the copy-first path)."""
    import torch

    pb = synth.make_problem(kind=kind, model=model, n_frames=8, n_points=300, width=376, height=240, seed=41,
                            border=10)
    if extra_points:
        rng = np.random.default_rng(3)
        n = extra_points
        pb = synth.Problem(**{**pb.__dict__,
                              "u_ref": np.concatenate([pb.u_ref, pb.u_ref[rng.integers(0, pb.n_points, n)]]),
                              "point_host": np.concatenate([pb.point_host, np.zeros(n, pb.point_host.dtype)]),
                              "rho": np.concatenate([pb.rho, np.full(n, 0.5)]),
                              "rho_gt": np.concatenate([pb.rho_gt, np.full(n, 0.6)]),
                              "host_intensity": (np.concatenate([pb.host_intensity, np.zeros((n, pb.P), np.float32)])
                                                 if pb.host_intensity is not None else None)})
    dev = torch.device("cuda", 0)
    poses_d = torch.from_numpy(np.ascontiguousarray(pb.poses_gt)).to(dev)
    rho_d = torch.from_numpy(np.ascontiguousarray(pb.rho_gt)).to(dev)
    with E.Engine(kind, model) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        eng.evaluate_state_device(poses_d.data_ptr(), rho_d.data_ptr(), True)
        a, va = eng.records()
        ca = eng.block_costs()
        poses, rho = eng.get_state()
        np.testing.assert_array_equal(poses, pb.poses_gt)
        np.testing.assert_array_equal(rho, pb.rho_gt)
        eng.evaluate(True)  # at the adopted state
        b, vb = eng.records()
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(va, vb)
        eng.set_state(pb.poses_gt, pb.rho_gt)
        eng.evaluate(True)
        c, _ = eng.records()
        np.testing.assert_array_equal(a, c)
        np.testing.assert_array_equal(ca, eng.block_costs())
    ref, vref = O.evaluate(pb, poses=pb.poses_gt, rho=pb.rho_gt)
    pb_gt = synth.Problem(**{**pb.__dict__, "poses": pb.poses_gt, "rho": pb.rho_gt})
    compare_records(kind, pb.R, a, ref, va, vref, projected_uv(pb_gt))


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("n_blocks", [1, 31, 33])
def test_ragged_block_counts(kind, n_blocks):
    """Block counts that leave the last workgroup partly empty (32 blocks per photometric workgroup, 256 per geometric
    one) and a single block: records, validity and costs against the oracle, fused-state launch included."""
    import torch
    pb = synth.make_problem(kind=kind, n_frames=6, n_points=40, width=376, height=240, seed=90 + n_blocks, border=12)
    keep = np.arange(n_blocks)
    pb = synth.Problem(**{**pb.__dict__, "block_point": pb.block_point[keep], "block_target": pb.block_target[keep],
                          "u_obs": None if pb.u_obs is None else pb.u_obs[keep]})
    rec, valid, costs = run_engine(pb, huber=9.0 if kind == 0 else 1.0)
    assert rec.shape[0] == n_blocks
    ref, vref = O.evaluate(pb)
    compare_records(kind, pb.R, rec, ref, valid, vref, projected_uv(pb) if kind == 0 else None)
    with E.Engine(pb.kind, pb.model, huber_width=9.0 if kind == 0 else 1.0) as eng:
        eng.set_problem(pb)
        eng.set_state(pb.poses, pb.rho)
        dev = torch.device("cuda", 0)
        poses_d, rho_d = torch.from_numpy(pb.poses).to(dev), torch.from_numpy(pb.rho).to(dev)  # alive for the launch
        eng.evaluate_state_device(poses_d.data_ptr(), rho_d.data_ptr(), True)
        a, va = eng.records()
        np.testing.assert_array_equal(va, valid)
        np.testing.assert_array_equal(a.view(np.uint32), rec.view(np.uint32))
        np.testing.assert_array_equal(eng.block_costs(), costs)


@pytest.mark.parametrize("kind,model", [(0, 0), (0, 1), (0, 2), (0, 3), (1, 0), (1, 3)])
def test_non_finite_state_gives_invalid_blocks(kind, model):
    """A NaN inverse distance or a NaN pose makes the blocks that use it invalid (validity 0, zero record, zero cost;
    Ceres' Evaluate returning false) and leaves every other block exactly as at the finite state: the branch-free row
    clamps any position to an in-bounds read."""
    pb = synth.make_problem(kind=kind, model=model, n_frames=6, n_points=120, width=376, height=240, seed=95, border=12)
    rec0, valid0, _ = run_engine(pb)
    rho = pb.rho.copy()
    rho[5] = np.nan
    poses = pb.poses.copy()
    poses[3, 4] = np.nan
    rec, valid, costs = run_engine(pb, poses=poses, rho=rho)
    hit = (pb.block_point == 5) | (pb.block_target == 3) | (pb.point_host[pb.block_point] == 3)
    assert hit.any() and (~hit).any()
    assert not valid[hit].any()
    assert (rec[hit] == 0).all() and (costs[hit] == 0).all()
    np.testing.assert_array_equal(valid[~hit], valid0[~hit])
    np.testing.assert_array_equal(rec[~hit].view(np.uint32), rec0[~hit].view(np.uint32))


def test_invalid_inputs_raise():
    pb = synth.make_problem(n_frames=6, n_points=20, width=64, height=48, seed=1, border=6)
    with E.Engine(0, 0) as eng:
        with pytest.raises(E.PbaError):
            eng.evaluate()  # nothing set
        bad = synth.Problem(**{**pb.__dict__, "block_target": pb.point_host[pb.block_point].copy()})
        with pytest.raises(E.PbaError, match="host"):
            eng.set_problem(bad)
        bad = synth.Problem(**{**pb.__dict__, "block_point": pb.block_point + 1000})
        with pytest.raises(E.PbaError, match="range"):
            eng.set_problem(bad)


def test_large_problem_sampled_parity():
    """C3-sized problem (200 KF × 20k points × 4 targets = 80k blocks): sampled blocks vs the oracle, plus
    size-independent properties (all valid, finite, per-block costs consistent with the records)."""
    pb = synth.make_problem(n_frames=200, n_points=20000, texture="noise", seed=42)
    rec, valid, costs = run_engine(pb)
    assert valid.all() and np.isfinite(rec).all()
    s = (rec[:, :pb.R].astype(np.float64) ** 2).sum(1)
    np.testing.assert_allclose(costs, 0.5 * s, rtol=1e-5, atol=1e-4)
    idx = np.random.default_rng(0).choice(pb.n_blocks, 2000, replace=False)
    idx.sort()
    sub = synth.Problem(**{**pb.__dict__, "block_point": pb.block_point[idx], "block_target": pb.block_target[idx]})
    ref, vref = O.evaluate(sub, n_threads=8)
    compare_records(0, pb.R, rec[idx], ref, valid[idx], vref, projected_uv(sub))


def test_pattern_sizes():
    """Patterns of 1…32 pixels (C5's 21-px pattern; PBA_MAX_PATTERN = 32): one pixel per lane up to 8, then the
    multi-pixel kernel with ⌈P/8⌉ = 2, 3, 4 pixels per lane (P = 32 in fp32 runs 128-thread workgroups), records,
    residual-only records and block costs against the oracle."""
    rng = np.random.default_rng(5)
    for P in (1, 5, 8, 9, 12, 16, 17, 21, 24, 27, 32):
        pat = rng.integers(-3, 4, (P, 2)).astype(np.float32)
        pb = synth.make_problem(n_frames=7, n_points=100, width=376, height=240, pattern=pat, seed=P, border=12)
        rec, valid, costs = run_engine(pb, huber=9.0)
        ref, vref = O.evaluate(pb)
        compare_records(0, P, rec, ref, valid, vref, projected_uv(pb))
        res_only, valid_r, _ = run_engine(pb, jac=False)
        assert np.array_equal(valid_r, valid)
        np.testing.assert_allclose(res_only[:, :P], rec[:, :P], atol=R_ATOL_PHOTOMETRIC)  # separate instantiations
        for b in np.flatnonzero(vref):
            c_ref, _ = O.huber_block(ref[b, :P], 9.0)
            tol = R_ATOL_PHOTOMETRIC * np.abs(ref[b, :P]).sum() + 1e-5 * abs(c_ref) + 1e-5
            assert abs(costs[b] - c_ref) <= tol, (P, b, costs[b], c_ref)
