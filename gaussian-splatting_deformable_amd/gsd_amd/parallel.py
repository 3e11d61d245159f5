"""Data parallelism over views: one process per GPU, RCCL all-reduce of the
per-Gaussian gradients.

The reference is single-GPU (train.py:106-112, utils/general_utils.py:133).
Views are independent given replicated Gaussian parameters, so each rank
renders its own view forward+backward with no communication, then ONE
collective sums the gradients.  Every parameter's ``.grad`` is a view into one
flat, contiguous slab, so the reduction is a single large all-reduce with no
pack/unpack copies (xGMI rings are per-link bound: few, large collectives).
Densification statistics (visibility counts, |dL/dmean2D| sums, max radii)
are per-view quantities and must be taken before the reduction; see
``view_stats_allreduce``.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
    """torchrun-style env (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) -> (rank, local_rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, local, world


class FlatGrads:
    """Owns one contiguous gradient slab; each parameter's .grad is a view of it."""

    def __init__(self, params, device=None):
        self.params = [p for p in params if p is not None]
        dev = device or self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.slab = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        self.views = []
        for p in self.params:
            v = self.slab[off:off + p.numel()].view_as(p)
            self.views.append(v)
            off += p.numel()
        self.attach()

    def attach(self):
        for p, v in zip(self.params, self.views):
            p.grad = v
            p._gsd_inplace_grad = True  # fused HIP backwards may add into this .grad directly

    def zero(self):
        self.slab.zero_()
        self.attach()

    def collect(self):
        """Copy any .grad autograd replaced (instead of accumulating in place) back into the slab."""
        for p, v in zip(self.params, self.views):
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v

    def allreduce(self, op=None, async_op=False):
        """Sum the slab across ranks (no-op for world size 1)."""
        self.collect()
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return None
        return dist.all_reduce(self.slab, op=op or dist.ReduceOp.SUM, async_op=async_op)


def view_stats_allreduce(visible_count: torch.Tensor, grad2d_norm_sum: torch.Tensor, max_radii: torch.Tensor):
    """Per-view densification statistics (gaussian_model.py:1252-1257, train.py:613),
    combined across ranks after each rank has accumulated its own view: sums for
    the counts / norm sums, max for the radii."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(visible_count, op=dist.ReduceOp.SUM)
        dist.all_reduce(grad2d_norm_sum, op=dist.ReduceOp.SUM)
        dist.all_reduce(max_radii, op=dist.ReduceOp.MAX)
    return visible_count, grad2d_norm_sum, max_radii
