"""Multi-GPU host driver: host-keyframe sharding and the collective of pba_solve_distributed.

The reference runs one Ceres problem on one machine (map_utils.h:322-399); its evaluation is a ParallelFor
over residual blocks (program_evaluator.h:187-258) and the points are eliminated per point in the Schur
eliminator.  Both properties make the host keyframe the natural shard unit: a point and all of its blocks
live on the rank that owns the point's host keyframe, so

* evaluation (the headline metric) needs no collective at all — each rank evaluates its own blocks;
* Gauss-Newton needs two sums per LM trial: the per-rank reduced camera systems (banded, (K+1)·36 + 24 doubles per
  keyframe), then 8 point-part scalars of the trial (model decrease, candidate cost and valid blocks, step and state
  norms, points above the gradient tolerance).  Every rank solves the same system, back-substitutes its own points and
  takes the same LM decision on the device.

Every rank holds all keyframe poses (7 doubles each) and the images of the keyframes its blocks target.
With the "nccl" backend (RCCL on ROCm) the engine gets its own RCCL communicator (`rccl_comm`: rank 0's id broadcast
through the process group) and enqueues both sums on its stream (`pba_solve_distributed_comm`: the host never waits
inside a trial).  Other backends ("gloo", CPU tests) go through `TorchAllReduce`, a host callback the engine calls once
its stream has drained.
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


_RCCL = {}


def rccl_comm(group=None, device_index: int = 0):
    """The engine's RCCL communicator over the ranks of `group` (collective on first use, then cached): rank 0's
    ncclUniqueId is broadcast through the torch.distributed group, every rank calls pba_comm_init."""
    import torch.distributed as dist
    key = (id(group), device_index)
    if key not in _RCCL:
        import importlib
        E = importlib.import_module(__package__ + ".engine")
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [E.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        _RCCL[key] = E.Comm.rccl(obj[0], world, rank, device_index)
    return _RCCL[key]


def solve_distributed(engine, group=None, device=None, comm=None, **options) -> dict:
    """LM over all ranks of `group`: collective, every rank calls it.  comm (an engine.Comm) or, for the "nccl" backend
    on a GPU, the cached RCCL communicator: stream-ordered pba_solve_distributed_comm; otherwise (or comm=False) the
    TorchAllReduce callback of pba_solve_distributed."""
    import torch.distributed as dist
    import torch
    if device is not None:
        device = torch.device(device)  # "cuda", "cuda:1", torch.device(...) alike
    band = global_band(engine, group, device)
    if comm is None and device is not None and device.type == "cuda" and dist.get_backend(group) == "nccl":
        comm = rccl_comm(group, device.index if device.index is not None else torch.cuda.current_device())
    if comm is not None and comm is not False:
        return engine.solve_distributed_comm(band, comm, **options)
    ar = TorchAllReduce(engine.gn_exchange_size(band), device if device is not None else "cpu", group)
    engine.set_rank(dist.get_rank(group))  # rank 0's pose part decides on every rank (pba_gn_set_rank)
    return engine.solve_distributed(band, ar.ptr, ar, **options)
