"""Fused hierarchy-cut interpolation (include/gsr_hier.h): the LOD blend render_post performs in
Python before rasterizing (gaussian_renderer/__init__.py:200-243; train_post.py:119,
render_hierarchy.py:88), as one gfx950 launch each way.

    means3D, scales, rotations, opacities, shs = interpolate_cut(
        pc.get_xyz, pc.get_scaling, pc.get_rotation, pc.get_opacity, pc.get_features,
        render_indices, parent_indices, interpolation_weights, pc.skybox_points)

returns the R + S rows render_post hands to GaussianRasterizer (R rendered nodes blended with
their parents, then the S skybox Gaussians), differentiable w.r.t. the five float inputs.
"""
from __future__ import annotations

import torch

from ._native import check, lib, ptr, require_gpu, stream


def _f32(t):
    return t.detach().float().contiguous()


class _InterpolateCut(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, scales, rotations, opacities, shs, render_indices, parent_indices, weights, skybox):
        require_gpu(means3D, scales, rotations, opacities, shs, render_indices, parent_indices, weights)
        N = means3D.shape[0]
        M = shs.shape[1]
        R = render_indices.shape[0]
        S = int(skybox)
        if parent_indices.shape[0] < R or weights.shape[0] < R:
            raise ValueError("parent_indices / interpolation_weights shorter than render_indices")
        ri = render_indices.to(torch.int32).contiguous()
        pi = parent_indices[:R].to(torch.int32).contiguous()
        w = _f32(weights)
        ins = [_f32(t) for t in (means3D, scales, rotations, opacities, shs)]
        dev = means3D.device
        rows = R + S
        outs = [torch.empty((rows,) + tuple(t.shape[1:]), dtype=torch.float32, device=dev) for t in ins]
        check(lib().gsr_interpolate_cut_forward(N, M, R, S, ptr(ri), ptr(pi), ptr(w), *[ptr(t) for t in ins],
                                                *[ptr(t) for t in outs], stream(dev)), "gsr_interpolate_cut_forward")
        ctx.save_for_backward(ri, pi, w, ins[2])
        ctx.meta = (N, M, R, S, [tuple(t.shape) for t in ins])
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        ri, pi, w, rots = ctx.saved_tensors
        N, M, R, S, shapes = ctx.meta
        dev = rots.device
        rows = R + S
        g = [(go if go is not None else torch.zeros((rows,) + shapes[k][1:], device=dev)).float().contiguous()
             for k, go in enumerate(gouts)]
        grads = [torch.zeros(s, dtype=torch.float32, device=dev) for s in shapes]
        check(lib().gsr_interpolate_cut_backward(N, M, R, S, ptr(ri), ptr(pi), ptr(w), ptr(rots),
                                                 *[ptr(t) for t in g], *[ptr(t) for t in grads], stream(dev)),
              "gsr_interpolate_cut_backward")
        return (*grads, None, None, None, None)


def interpolate_cut(means3D, scales, rotations, opacities, shs, render_indices, parent_indices,
                    interpolation_weights, skybox_points=0):
    return _InterpolateCut.apply(means3D, scales, rotations, opacities, shs, render_indices, parent_indices,
                                 interpolation_weights, int(skybox_points))
