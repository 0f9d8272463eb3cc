"""Parameter activations and the per-step scale shrink in one launch each (csrc/train.hip):

  activate(scaling, rotation, opacity) -> (exp(scaling), normalize(rotation), sigmoid(opacity))
      the getters of scene/gaussian_model.py:125-156 with the activations of :39-47; the backward
      is one launch with torch autograd's formulas (exp: g*y, sigmoid: g*(1-y)*y, normalize:
      g/d - x * sum(g * x/d/d) / n)
  shrink_scales(scaling, limit, first_row)
      train_single.py:235-241: rows whose largest exp(scaling) exceeds `limit` get
      scaling = log(exp(scaling) * 0.8), in place, without the max / compare / index kernels
"""
from __future__ import annotations

import torch

from ._native import check, lib, ptr, require_gpu, stream


def _rows(t: torch.Tensor, width: int, name: str) -> torch.Tensor:
    if t.dtype != torch.float32 or t.numel() != t.shape[0] * width:
        raise ValueError(f"{name}: expected (P, {width}) float32")
    return t.contiguous()


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, scaling, rotation, opacity):
        require_gpu(scaling, rotation, opacity)
        P = scaling.shape[0]
        s, q, o = _rows(scaling, 3, "scaling"), _rows(rotation, 4, "rotation"), _rows(opacity, 1, "opacity")
        if q.shape[0] != P or o.shape[0] != P:
            raise ValueError("scaling, rotation and opacity must have the same number of rows")
        scales, rots, opac = torch.empty_like(s), torch.empty_like(q), torch.empty_like(o)
        check(lib().gsr_activate_forward(P, ptr(s), ptr(q), ptr(o), ptr(scales), ptr(rots), ptr(opac),
                                         stream(s.device)), "gsr_activate_forward")
        ctx.save_for_backward(q, scales, opac)
        ctx.keys = (scaling.data_ptr(), rotation.data_ptr(), opacity.data_ptr())  # gsr_dist.GradBucket views
        return scales, rots, opac

    @staticmethod
    def backward(ctx, g_s, g_q, g_o):
        q, scales, opac = ctx.saved_tensors
        P = q.shape[0]
        z = lambda g, like: torch.zeros_like(like) if g is None else g.float().contiguous()
        g_s, g_q, g_o = z(g_s, scales), z(g_q, q), z(g_o, opac)
        from gsr_dist import grad_out
        ks, kq, ko = ctx.keys
        d_s, d_q, d_o = (grad_out(ks, scales.shape, q.device), grad_out(kq, q.shape, q.device),
                         grad_out(ko, opac.shape, q.device))
        check(lib().gsr_activate_backward(P, ptr(q), ptr(scales), ptr(opac), ptr(g_s), ptr(g_q), ptr(g_o),
                                          ptr(d_s), ptr(d_q), ptr(d_o), stream(q.device)), "gsr_activate_backward")
        return d_s, d_q, d_o


def activate(scaling: torch.Tensor, rotation: torch.Tensor, opacity: torch.Tensor):
    """(exp(scaling), F.normalize(rotation), sigmoid(opacity)), differentiable."""
    return _Activate.apply(scaling, rotation, opacity)


@torch.no_grad()
def shrink_scales(scaling: torch.Tensor, limit: float, first_row: int = 0) -> None:
    require_gpu(scaling)
    if scaling.dtype != torch.float32 or not scaling.is_contiguous() or scaling.numel() != 3 * scaling.shape[0]:
        raise ValueError("scaling: expected contiguous (P, 3) float32")
    check(lib().gsr_shrink_scales(scaling.shape[0], int(first_row), ptr(scaling), float(limit),
                                  stream(scaling.device)), "gsr_shrink_scales")
