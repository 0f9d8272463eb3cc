"""Densification statistics in one launch (train_single.py:193-194 +
scene/gaussian_model.py:780-793): for Gaussians with radius > 0,
max_radii2D = max(max_radii2D, radii), xyz_gradient_accum = max(||dL/dmeans2D[:, :2]||, accum),
denom += 1.  The reference builds visibility_filter with nonzero() (a host sync) and runs three
indexed torch updates; here the radius test happens per row on the device."""
from __future__ import annotations

import torch

from ._native import check, lib, ptr, require_gpu, stream


def add_densification_stats(radii: torch.Tensor, means2D_grad: torch.Tensor, max_radii2D: torch.Tensor,
                            xyz_gradient_accum: torch.Tensor, denom: torch.Tensor) -> None:
    require_gpu(radii, means2D_grad, max_radii2D, xyz_gradient_accum, denom)
    P = radii.shape[0]
    for name, t, n in (("means2D_grad", means2D_grad, 3 * P), ("max_radii2D", max_radii2D, P),
                       ("xyz_gradient_accum", xyz_gradient_accum, P), ("denom", denom, P)):
        if t.numel() != n or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"{name}: expected {n} contiguous float32 values")
    if radii.dtype != torch.int32 or not radii.is_contiguous():
        raise ValueError("radii: expected contiguous int32")
    check(lib().gsr_densify_stats(P, ptr(radii), ptr(means2D_grad), ptr(max_radii2D), ptr(xyz_gradient_accum),
                                  ptr(denom), stream(radii.device)), "gsr_densify_stats")
