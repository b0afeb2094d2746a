"""Multi-GPU host driver: host-keyframe sharding and the collective of pba_solve_distributed.

The reference runs one Ceres problem on one machine (map_utils.h:322-399); its evaluation is a ParallelFor
over residual blocks (program_evaluator.h:187-258) and the points are eliminated per point in the Schur
eliminator.  Both properties make the host keyframe the natural shard unit: a point and all of its blocks
live on the rank that owns the point's host keyframe, so

* evaluation (the headline metric) needs no collective at all — each rank evaluates its own blocks;
* Gauss-Newton needs exactly one exchange per LM iteration: the sum of the per-rank reduced camera systems
  (banded, (K+1)·36 + 24 doubles per keyframe) plus three scalars (cost, candidate cost, point part of the
  model decrease).  Every rank then solves the same system and back-substitutes its own points.

Every rank holds all keyframe poses (7 doubles each) and the images of the keyframes its blocks target.
The collective is `torch.distributed.all_reduce` (RCCL on ROCm for the "nccl" backend; "gloo" stages
through the host) on a device buffer the engine writes into; `pba_solve_distributed` calls back into
`TorchAllReduce` whenever it needs a sum.
"""
from __future__ import annotations

import dataclasses
import threading
from typing import Optional

import numpy as np


# ------------------------------------------------------------------------------------------------
# Sharding
# ------------------------------------------------------------------------------------------------
def host_ranges(point_host: np.ndarray, block_point: np.ndarray, n_frames: int, world: int) -> np.ndarray:
    """Contiguous host-keyframe ranges [b[r], b[r+1]) with about equal residual-block counts per rank."""
    per_frame = np.bincount(point_host[block_point], minlength=n_frames).astype(np.int64)
    cum = np.concatenate([[0], np.cumsum(per_frame)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        f = int(np.searchsorted(cum, total * r / world, side="left"))
        bounds.append(min(max(f, bounds[-1]), n_frames))
    bounds.append(n_frames)
    return np.asarray(bounds, np.int64)


def shard_problem(pb, world: int, rank: int, bounds: Optional[np.ndarray] = None):
    """The shard of rank `rank`: all keyframes (global indices, same poses), the points hosted in its
    keyframe range (renumbered 0..n−1, original order kept) and all their blocks (original order kept).
    Returns (problem, point_ids, block_ids) with the global indices of the shard's points and blocks."""
    if bounds is None:
        bounds = host_ranges(pb.point_host, pb.block_point, len(pb.frame_cam), world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    point_ids = np.nonzero((pb.point_host >= lo) & (pb.point_host < hi))[0]
    remap = np.full(len(pb.point_host), -1, np.int64)
    remap[point_ids] = np.arange(len(point_ids))
    block_ids = np.nonzero(remap[pb.block_point] >= 0)[0]
    sub = dict(pb.__dict__)
    sub.update(point_host=pb.point_host[point_ids], u_ref=pb.u_ref[point_ids],
               host_intensity=None if pb.host_intensity is None else pb.host_intensity[point_ids],
               block_point=remap[pb.block_point[block_ids]].astype(np.int32),
               block_target=pb.block_target[block_ids],
               u_obs=None if pb.u_obs is None else pb.u_obs[block_ids],
               rho=pb.rho[point_ids],
               rho_gt=None if getattr(pb, "rho_gt", None) is None else pb.rho_gt[point_ids])
    return dataclasses.replace(pb, **sub), point_ids, block_ids


# ------------------------------------------------------------------------------------------------
# Collectives
# ------------------------------------------------------------------------------------------------
class TorchAllReduce:
    """Exchange buffer + the `allreduce(ptr, count)` callback of pba_solve_distributed over a
    torch.distributed process group.  The engine writes the buffer on its own stream and synchronises
    before calling back; the callback returns once the sum is in place."""

    def __init__(self, count: int, device, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.buf = torch.zeros(count, dtype=torch.float64, device=device)
        self.device = self.buf.device
        self.staged = self.device.type == "cuda" and dist.get_backend(group) != "nccl"

    @property
    def ptr(self) -> int:
        return self.buf.data_ptr()

    def __call__(self, ptr: int, count: int):
        off = (ptr - self.buf.data_ptr()) // 8
        if off < 0 or off + count > self.buf.numel():
            raise ValueError("allreduce range outside the exchange buffer")
        view = self.buf[off:off + count]
        if self.staged:  # gloo on a GPU buffer: through the host
            host = view.cpu()
            self.dist.all_reduce(host, group=self.group)
            view.copy_(host)
        else:
            self.dist.all_reduce(view, group=self.group)
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)


class InProcessAllReduce:
    """Several engines of one process (one thread each) standing in for ranks: sums the ranks' exchange
    buffers in fixed rank order.  Test / single-GPU rehearsal helper."""

    def __init__(self, buffers, timeout: float = 300.0):
        self.bufs = buffers
        self.barrier = threading.Barrier(len(buffers), timeout=timeout)

    def rank(self, r: int):
        def fn(ptr: int, count: int):
            import torch
            off = (ptr - self.bufs[r].data_ptr()) // 8
            self.barrier.wait()
            if r == 0:
                tot = self.bufs[0][off:off + count].clone()
                for b in self.bufs[1:]:
                    tot += b[off:off + count]
                for b in self.bufs:
                    b[off:off + count].copy_(tot)
                if tot.is_cuda:
                    torch.cuda.synchronize(tot.device)
            self.barrier.wait()
        return fn


def global_band(engine, group=None, device=None) -> int:
    """max over ranks of the local reduced-system bandwidth (the exchange layout must agree)."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None and dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([engine.gn_band()], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def solve_distributed(engine, group=None, device=None, **options) -> dict:
    """LM over all ranks of `group` (pba_solve_distributed): collective, every rank calls it."""
    band = global_band(engine, group, device)
    ar = TorchAllReduce(engine.gn_exchange_size(band), device if device is not None else "cpu", group)
    return engine.solve_distributed(band, ar.ptr, ar, **options)
