"""Multi-GPU modes around the rasterizer, one process per GPU.

1. Chunk-per-GPU (the product's only mode, mirroring scripts/full_train.py:171-232 and the
   Slurm fan-out of scripts/train_chunk.slurm): chunks are independent units, assigned to
   ranks round-robin; no data-path collective.  Only timing uses a MAX reduction.

2. Optional image-batch data parallelism inside one chunk (new; not in the reference): every
   rank holds the same Gaussians, rasterizes a different camera, and the Gaussian gradients are
   summed with ONE flat all-reduce per step (RCCL over xGMI on MI355X, gloo on CPU).  The
   densification statistics of scene/gaussian_model.py:780-793 are reduced with MAX
   (max_radii2D, xyz_gradient_accum) and SUM (denom).

Works with any torch.distributed backend ("nccl" == RCCL on ROCm, "gloo" for CPU tests).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def chunk_assignment(n_chunks: int, world_size: int, rank_id: int) -> List[int]:
    """Round-robin chunk -> rank map (chunk c runs on rank c % world_size)."""
    return [c for c in range(n_chunks) if c % world_size == rank_id]


def max_over_ranks(x: float, device=None) -> float:
    if world() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_gaussian_grads(params: Sequence[torch.Tensor], average: bool = False) -> None:
    """Sum the .grad of every Gaussian parameter tensor across ranks with one flat bucket.

    One large all-reduce instead of one per tensor: on MI355X the ring is per-xGMI-link bound,
    so a single ~P*59*4-byte bucket amortises the per-collective latency."""
    if world() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    if average:
        flat /= world()
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


def allreduce_densify_stats(max_radii2D: torch.Tensor, xyz_gradient_accum: torch.Tensor,
                            denom: torch.Tensor) -> None:
    """MAX of the per-Gaussian screen radius and accumulated screen-space gradient norm, SUM
    of the visibility counts (the statistics densify_and_prune consumes)."""
    if world() == 1:
        return
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX)
    dist.all_reduce(xyz_gradient_accum, op=dist.ReduceOp.MAX)
    dist.all_reduce(denom, op=dist.ReduceOp.SUM)


def run_chunks(chunks: Iterable[int], fn) -> Dict[int, object]:
    """Run fn(chunk_id) for this rank's chunks; returns {chunk_id: result}."""
    return {c: fn(c) for c in chunks}
