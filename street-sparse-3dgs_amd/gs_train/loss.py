"""Fused photometric loss: mean |img - gt| and mean SSIM (11x11 Gaussian window, sigma 1.5) in one
gfx950 launch each way (in training the forward also stores the SSIM gradient field and the
backward is elementwise) (csrc/train.hip), replacing utils/loss_utils.py:17-18 (l1_loss) and
:33-63 (ssim: five depthwise conv2d + elementwise ops) as combined at train_single.py:121-123.

Gradients flow only to `img` (the rendered image); `gt` is a constant, as in the reference.
"""
from __future__ import annotations

import torch

from ._native import check, lib, ptr, require_gpu, stream


def _planes(img: torch.Tensor):
    if img.dim() == 3:
        return img.shape[0], img.shape[1], img.shape[2]
    if img.dim() == 4:
        return img.shape[0] * img.shape[1], img.shape[2], img.shape[3]
    raise ValueError("expected a (C, H, W) or (B, C, H, W) image")


class _L1SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, gt):
        require_gpu(img, gt)
        if img.shape != gt.shape:
            raise ValueError(f"image shapes differ: {tuple(img.shape)} vs {tuple(gt.shape)}")
        img = img.detach().float().contiguous()
        gt = gt.detach().float().contiguous()
        C, H, W = _planes(img)
        L = lib()
        out = torch.empty(2, dtype=torch.float32, device=img.device)
        scratch = torch.empty(max(1, L.gsr_l1_ssim_scratch_bytes(C, H, W)), dtype=torch.uint8, device=img.device)
        s = stream(img.device)
        if ctx.needs_input_grad[0]:
            # training: the forward also stores the SSIM gradient field, the backward is elementwise
            gmap = torch.empty_like(img)
            check(L.gsr_l1_ssim_forward_with_map(ptr(img), ptr(gt), C, H, W, ptr(scratch), ptr(out), ptr(gmap), s),
                  "gsr_l1_ssim_forward_with_map")
            ctx.save_for_backward(img, gt, gmap)
        else:
            check(L.gsr_l1_ssim_forward(ptr(img), ptr(gt), C, H, W, ptr(scratch), ptr(out), s), "gsr_l1_ssim_forward")
            ctx.save_for_backward(img, gt)
        ctx.dims = (C, H, W)
        return out

    @staticmethod
    def backward(ctx, gout):
        saved = ctx.saved_tensors
        img, gt = saved[0], saved[1]
        C, H, W = ctx.dims
        gout = gout.float().contiguous()
        dimg = torch.empty_like(img)
        s = stream(img.device)
        if len(saved) == 3:
            check(lib().gsr_l1_ssim_backward_from_map(ptr(img), ptr(gt), ptr(saved[2]), C, H, W, ptr(gout), ptr(dimg),
                                                      s), "gsr_l1_ssim_backward_from_map")
        else:
            check(lib().gsr_l1_ssim_backward(ptr(img), ptr(gt), C, H, W, ptr(gout), ptr(dimg), s),
                  "gsr_l1_ssim_backward")
        return dimg, None


def l1_ssim(img: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """Returns the 2-vector [mean |img - gt|, mean SSIM(img, gt)], differentiable w.r.t. img."""
    return _L1SSIM.apply(img, gt)


class _PhotoLoss(torch.autograd.Function):
    """loss = (1 - lambda) L1 + lambda (1 - SSIM) as ONE node (include/gsr_train.h
    gsr_photo_loss_*): the same values and gradient bits as composing l1_ssim with torch's scalar
    ops, without their one-element launches.  L1 and SSIM come back as non-differentiable
    by-products (the reference uses Ll1 only for its progress bar)."""

    @staticmethod
    def forward(ctx, img, gt, lambda_dssim):
        require_gpu(img, gt)
        if img.shape != gt.shape:
            raise ValueError(f"image shapes differ: {tuple(img.shape)} vs {tuple(gt.shape)}")
        img = img.detach().float().contiguous()
        gt = gt.detach().float().contiguous()
        C, H, W = _planes(img)
        L = lib()
        out = torch.empty(3, dtype=torch.float32, device=img.device)
        scratch = torch.empty(max(1, L.gsr_l1_ssim_scratch_bytes(C, H, W)), dtype=torch.uint8, device=img.device)
        gmap = torch.empty_like(img)
        check(L.gsr_photo_loss_forward(ptr(img), ptr(gt), C, H, W, float(lambda_dssim), ptr(scratch), ptr(out),
                                       ptr(gmap), stream(img.device)), "gsr_photo_loss_forward")
        ctx.save_for_backward(img, gt, gmap)
        ctx.dims = (C, H, W)
        ctx.lambda_dssim = float(lambda_dssim)
        ctx.set_materialize_grads(False)
        loss, l1, s = out[2], out[0], out[1]
        ctx.mark_non_differentiable(l1, s)
        return loss, l1, s

    @staticmethod
    def backward(ctx, gloss, _gl1, _gs):
        if gloss is None:
            return None, None, None
        img, gt, gmap = ctx.saved_tensors
        C, H, W = ctx.dims
        gloss = gloss.float().contiguous()
        dimg = torch.empty_like(img)
        check(lib().gsr_photo_loss_backward(ptr(img), ptr(gt), ptr(gmap), C, H, W, ctx.lambda_dssim, ptr(gloss),
                                            ptr(dimg), stream(img.device)), "gsr_photo_loss_backward")
        return dimg, None, None


def photo_loss(img: torch.Tensor, gt: torch.Tensor, lambda_dssim: float = 0.2):
    """(1 - lambda) L1 + lambda (1 - SSIM)  (train_single.py:121-123); returns (loss, l1, ssim).
    With a gradient wanted for img: one fused node (_PhotoLoss); otherwise l1_ssim's forward and
    the same expression."""
    if torch.is_grad_enabled() and img.requires_grad:
        return _PhotoLoss.apply(img, gt, lambda_dssim)
    v = l1_ssim(img, gt)
    l1, s = v[0], v[1]
    return (1.0 - lambda_dssim) * l1 + lambda_dssim * (1.0 - s), l1, s


class _DepthL1(torch.autograd.Function):
    """w * mean(|(invdepth - mono) * mask|) as one node (include/gsr_train.h gsr_depth_l1_*):
    train_single.py:138-140's Ll1depth.  The gradient w.r.t. invdepth is bit-identical to torch's
    autograd through the reference's expression; the value is the fp64-accumulated mean (torch
    sums in fp32: they agree to fp32 rounding)."""

    @staticmethod
    def forward(ctx, invd, mono, mask, weight):
        require_gpu(invd, mono, mask)
        if invd.shape != mono.shape or (mask is not None and mask.shape != invd.shape):
            raise ValueError("invdepth, mono_invdepth and depth_mask must have one shape")
        x = invd.detach().float().contiguous()
        y = mono.detach().float().contiguous()
        m = mask.detach().float().contiguous() if mask is not None else None
        n = x.numel()
        L = lib()
        out = torch.empty(2, dtype=torch.float32, device=x.device)
        scratch = torch.empty(max(8, int(L.gsr_depth_l1_scratch_bytes(n))), dtype=torch.uint8, device=x.device)
        check(L.gsr_depth_l1_forward(ptr(x), ptr(y), ptr(m), n, float(weight), ptr(scratch), ptr(out),
                                     stream(x.device)), "gsr_depth_l1_forward")
        ctx.save_for_backward(x, y, m)
        ctx.weight = float(weight)
        ctx.set_materialize_grads(False)
        loss, pure = out[1], out[0]
        ctx.mark_non_differentiable(pure)
        return loss, pure

    @staticmethod
    def backward(ctx, gloss, _gpure):
        if gloss is None:
            return None, None, None, None
        x, y, m = ctx.saved_tensors
        d = torch.empty_like(x)
        check(lib().gsr_depth_l1_backward(ptr(x), ptr(y), ptr(m), x.numel(), ctx.weight,
                                          ptr(gloss.float().contiguous()), ptr(d), stream(x.device)),
              "gsr_depth_l1_backward")
        return d, None, None, None


def depth_l1_loss(invd: torch.Tensor, mono: torch.Tensor, mask: torch.Tensor | None, weight: float):
    """depth_l1_weight * |(invDepth - mono_invdepth) * depth_mask|.mean()  (train_single.py:138-140),
    differentiable w.r.t. invd.  Returns the weighted loss (a 0-dim tensor)."""
    return _DepthL1.apply(invd, mono, mask, weight)[0]


class _DepthOnlyLoss(torch.autograd.Function):
    """A depth-only view's loss (include/gsr_train.h gsr_depth_only_loss_*), train_single.py:152-156:
    w * (a * mean(clamp(mono - invD, min=0)) + (1 - a) * mean(|(invD - mono) * mask|)), a =
    additional_depth_maps_weight.  Gradient bit-identical to torch's autograd through that
    expression; the means are fp64-accumulated (fp32 rounding from torch's)."""

    @staticmethod
    def forward(ctx, invd, mono, mask, weight, dens_weight):
        require_gpu(invd, mono, mask)
        if invd.shape != mono.shape or (mask is not None and mask.shape != invd.shape):
            raise ValueError("invdepth, mono_invdepth and depth_mask must have one shape")
        x = invd.detach().float().contiguous()
        y = mono.detach().float().contiguous()
        m = mask.detach().float().contiguous() if mask is not None else None
        n = x.numel()
        L = lib()
        out = torch.empty(3, dtype=torch.float32, device=x.device)
        scratch = torch.empty(max(16, int(L.gsr_depth_only_scratch_bytes(n))), dtype=torch.uint8, device=x.device)
        check(L.gsr_depth_only_loss_forward(ptr(x), ptr(y), ptr(m), n, float(weight), float(dens_weight),
                                            ptr(scratch), ptr(out), stream(x.device)), "gsr_depth_only_loss_forward")
        ctx.save_for_backward(x, y, m)
        ctx.weight = float(weight)
        ctx.dens_weight = float(dens_weight)
        ctx.set_materialize_grads(False)
        loss, pure, dens = out[2], out[0], out[1]
        ctx.mark_non_differentiable(pure, dens)
        return loss, pure, dens

    @staticmethod
    def backward(ctx, gloss, _gpure, _gdens):
        if gloss is None:
            return None, None, None, None, None
        x, y, m = ctx.saved_tensors
        d = torch.empty_like(x)
        check(lib().gsr_depth_only_loss_backward(ptr(x), ptr(y), ptr(m), x.numel(), ctx.weight, ctx.dens_weight,
                                                 ptr(gloss.float().contiguous()), ptr(d), stream(x.device)),
              "gsr_depth_only_loss_backward")
        return d, None, None, None, None


def depth_only_loss(invd: torch.Tensor, mono: torch.Tensor, mask: torch.Tensor | None, weight: float,
                    dens_weight: float = 0.9):
    """depth_l1_weight * (a * Ll1depth_dens + (1 - a) * Ll1depth_pure) for a depth-only view
    (train_single.py:152-156), differentiable w.r.t. invd.  Returns (loss, pure, dens)."""
    return _DepthOnlyLoss.apply(invd, mono, mask, weight, dens_weight)
