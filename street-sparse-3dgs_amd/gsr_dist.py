"""Multi-GPU modes around the rasterizer, one process per GPU.

1. Chunk-per-GPU (the product's only mode, mirroring scripts/full_train.py:171-232 and the
   Slurm fan-out of scripts/train_chunk.slurm): chunks are independent units, assigned to
   ranks round-robin; no data-path collective.  Only timing uses a MAX reduction.

2. Optional image-batch data parallelism inside one chunk (new; not in the reference): every
   rank holds the same Gaussians, rasterizes a different camera, and the Gaussian gradients are
   summed with ONE flat all-reduce per step (RCCL over xGMI on MI355X, gloo on CPU).  The
   densification statistics of scene/gaussian_model.py:780-793 are reduced with MAX
   (max_radii2D, xyz_gradient_accum) and SUM (denom).

   GradBucket keeps that flat buffer persistent: while it captures a backward, the kernels that
   produce the Gaussian parameters' gradients (the rasterizer's dL/dmeans3D and dL/dshs, the
   activations' dL/d(raw scaling, rotation, opacity)) write straight into views of it, autograd
   stores those views as the parameters' .grad without a copy, and the all-reduce runs in place:
   no torch.cat and no copy back (2 x 236 MB of HBM traffic less per step at 1M Gaussians).

Works with any torch.distributed backend ("nccl" == RCCL on ROCm, "gloo" for CPU tests).
"""
from __future__ import annotations

import threading
from typing import Dict, Iterable, List, Sequence, Tuple

import torch
import torch.distributed as dist

# The capturing bucket: process-wide, because torch runs a CUDA backward on its own device thread.
_ACTIVE = None
_LOCK = threading.Lock()
# called with the capturing bucket on capture entry and with None on exit (the rasterizer's C++
# backward registers one: it then asks grad_out for its leaf gradients' outputs)
_LISTENERS = []


def add_capture_listener(fn) -> None:
    if fn not in _LISTENERS:
        _LISTENERS.append(fn)


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
    """Sum the .grad of every Gaussian parameter tensor across ranks with one flat bucket
    (a temporary one: cat + copy back; GradBucket avoids both).

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


class GradBucket:
    """One flat fp32 buffer for the gradients of a set of parameters (name -> parameter).

        bucket = GradBucket({"xyz": g._xyz, "features": g._features, "opacity": g._opacity,
                             "scaling": g._scaling, "rotation": g._rotation})
        with bucket.capture(g):          # zeroes nothing: every view is written whole
            loss.backward()
        bucket.allreduce()               # in place; the parameters' .grad are views of it

    During capture, grad_out(param.data_ptr(), shape) hands the producing kernel the view of that
    parameter (once per capture); a second request, or one for an unknown tensor, gets a fresh
    tensor and autograd accumulates it into the view as usual.  Views are keyed by the
    parameter's storage address: rebuild the bucket after densification replaces parameters."""

    def __init__(self, params: Dict[str, torch.Tensor]):
        self.names = list(params)
        self.params = [params[n] for n in self.names]
        dev = self.params[0].device
        self.sizes = [p.numel() for p in self.params]
        self.flat = torch.empty(sum(self.sizes), dtype=torch.float32, device=dev)
        # (offset, shape) per parameter address: the views are made when handed out, so the bucket
        # holds no reference to them and autograd's AccumulateGrad adopts them as .grad (a
        # gradient tensor referenced elsewhere would be copied instead)
        self.slots = {}
        off = 0
        for p, n in zip(self.params, self.sizes):
            self.slots[p.data_ptr()] = (off, tuple(p.shape))
            off += n
        self._handed = set()

    def _view(self, key):
        off, shape = self.slots[key]
        n = 1
        for d in shape:
            n *= d
        return self.flat[off:off + n].view(shape)

    def capture(self, *_):
        bucket = self

        class _Ctx:
            def __enter__(self_):
                global _ACTIVE
                for p in bucket.params:
                    if p.grad is not None:
                        raise RuntimeError("GradBucket.capture: clear the parameters' .grad first "
                                           "(zero_grad(set_to_none=True))")
                with _LOCK:
                    if _ACTIVE is not None:
                        raise RuntimeError("GradBucket.capture: another bucket is capturing")
                    bucket._handed = set()
                    _ACTIVE = bucket
                for f in _LISTENERS:
                    f(bucket)
                return bucket

            def __exit__(self_, *exc):
                global _ACTIVE
                with _LOCK:
                    _ACTIVE = None
                for f in _LISTENERS:
                    f(None)
                return False
        return _Ctx()

    def view_for(self, key: int, shape: Tuple[int, ...]):
        with _LOCK:
            slot = self.slots.get(key)
            if slot is None or slot[1] != tuple(shape) or key in self._handed:
                return None
            self._handed.add(key)
        return self._view(key)

    def owns(self, param: torch.Tensor) -> bool:
        g = param.grad
        if g is None:
            return False
        base = self.flat.data_ptr()
        return base <= g.data_ptr() < base + 4 * self.flat.numel()

    def allreduce(self, average: bool = False) -> None:
        """Sum the bucket across ranks in place.  Every parameter must hold its view as .grad
        (a parameter without a gradient this step contributes zeros)."""
        for p in self.params:
            if p.grad is None:
                v = self._view(p.data_ptr())
                v.zero_()
                p.grad = v
            elif not self.owns(p):
                v = self._view(p.data_ptr())
                v.copy_(p.grad)
                p.grad = v
        if world() == 1:
            return
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
        if average:
            self.flat /= world()


def grad_out(key: int | None, shape, device, dtype=torch.float32) -> torch.Tensor:
    """Output tensor for the gradient of the parameter stored at address `key` (its data_ptr()):
    its GradBucket view when a bucket is capturing and owns it, a fresh tensor otherwise (the
    kernel wrappers call this for the leaf gradients they produce; the kernels write every row)."""
    b = _ACTIVE
    if b is not None and key is not None and dtype == torch.float32:
        v = b.view_for(key, tuple(shape))
        if v is not None:
            return v
    return torch.empty(tuple(shape), dtype=dtype, device=device)


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
