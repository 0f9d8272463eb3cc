"""Densification on the device (csrc/train.hip, csrc/densify.hip).

add_densification_stats: one launch (train_single.py:193-194 + scene/gaussian_model.py:780-793):
for Gaussians with radius > 0, max_radii2D = max(max_radii2D, radii), xyz_gradient_accum =
max(||dL/dmeans2D[:, :2]||, accum), denom += 1.  The reference builds visibility_filter with
nonzero() (a host sync) and runs three indexed torch updates; here the radius test happens per
row on the device.

densify_and_prune: GaussianModel.densify_and_prune (scene/gaussian_model.py:733-778, clone +
split + opacity prune, gt_point_cloud_constraints off) as one planned gather over every
parameter and Adam moment (include/gsr_densify.h): one host read of four counts, the split
samples drawn exactly as the reference's torch.normal draws them, one launch writing the new
arrays."""
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


def densify_and_prune(g, optimizer, max_grad: float, min_opacity: float, extent: float, percent_dense: float,
                      first_row: int = 0, normals: torch.Tensor = None) -> dict:
    """g: a joined-layout gs_train.harness.GaussianSet; optimizer: its gs_train.optim.Adam.  Replaces
    the parameters (and their optimizer state) with the densified / pruned rows and resets the
    densification statistics, as the reference does.  first_row: scaffold_points (rows never
    densified or pruned).  normals: the (2 n_split, 3) standard-normal draws behind the split
    samples, if given (parity tests inject the reference's own; a callable gets n_split and returns
    them); drawn here otherwise.  Returns the plan's counts."""
    from diff_gaussian_rasterization._lib import RowGroup
    if not getattr(g, "joined", False):
        raise ValueError("densify_and_prune works on the joined (P,16,3) SH layout")
    dev = g._xyz.device
    require_gpu(g._xyz)
    P0 = g.P
    names = ["_xyz", "_features", "_opacity", "_scaling", "_rotation"]
    params = [getattr(g, n) for n in names]
    L = lib()
    s = stream(dev)
    scratch = torch.empty(max(1, L.gsr_densify_scratch_bytes(P0)), dtype=torch.uint8, device=dev)
    counts = torch.zeros(4, dtype=torch.int64, device=dev)
    acc = g.xyz_gradient_accum.reshape(-1).contiguous()
    check(L.gsr_densify_plan(P0, int(first_row), ptr(acc), ptr(g.max_radii2D.contiguous()), ptr(g._opacity.detach()),
                             ptr(g._scaling.detach()), float(max_grad), float(min_opacity),
                             float(percent_dense * extent), ptr(scratch), ptr(counts), s), "gsr_densify_plan")
    n_old, n_clone, n_split, total = (int(v) for v in counts.cpu())
    # the reference's torch.normal(mean=zeros, std=stds) draws normal_(0, 1) on a (2 n_split, 3)
    # tensor and scales it: the same generator stream
    if callable(normals):
        normals = normals(n_split)
    if normals is None:
        normals = torch.empty((2 * n_split, 3), device=dev).normal_() if n_split else None
    else:
        if tuple(normals.shape) != (2 * n_split, 3):
            raise ValueError(f"normals: expected shape {(2 * n_split, 3)}, got {tuple(normals.shape)}")
        normals = normals.to(device=dev, dtype=torch.float32).contiguous() if n_split else None
    src = (RowGroup * len(names))()
    dst = (RowGroup * len(names))()
    new = []
    for k, p in enumerate(params):
        w = p[0].numel() if P0 else p.numel() // max(p.shape[0], 1)
        st = optimizer.state.get(p)
        np_ = torch.empty((total,) + tuple(p.shape[1:]), device=dev)
        m = v = None
        if st and "exp_avg" in st:
            m = torch.empty_like(np_)
            v = torch.empty_like(np_)
        new.append((np_, m, v))
        src[k] = RowGroup(p.data_ptr(), st["exp_avg"].data_ptr() if m is not None else None,
                          st["exp_avg_sq"].data_ptr() if m is not None else None, w)
        dst[k] = RowGroup(np_.data_ptr(), m.data_ptr() if m is not None else None,
                          v.data_ptr() if v is not None else None, w)
    check(L.gsr_densify_apply(P0, len(names), src, dst, 0, 3, 4, ptr(normals), n_split, ptr(scratch), total, s),
          "gsr_densify_apply")
    for (name, p, (np_, m, v)) in zip(names, params, new):
        newp = torch.nn.Parameter(np_)
        st = optimizer.state.pop(p, None)
        if st is not None:
            if m is not None:
                st["exp_avg"], st["exp_avg_sq"] = m, v
            optimizer.state[newp] = st
        for group in optimizer.param_groups:
            group["params"] = [newp if q is p else q for q in group["params"]]
        setattr(g, name, newp)
    g.xyz_gradient_accum = torch.zeros((total, 1), device=dev)
    g.denom = torch.zeros((total, 1), device=dev)
    g.max_radii2D = torch.zeros((total,), device=dev)
    return dict(kept=n_old, cloned=n_clone, split=n_split, total=total)
