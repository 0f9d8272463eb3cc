"""The reference's own torch formulation of the train-step pieces, run on the GPU for the
side-by-side "train-step ms" number (harness.TrainStep(fused=False)).  Not the product path and
not a fallback: the fused kernels never route here.

  photo_loss           utils/loss_utils.py:17-63 (five depthwise 11x11 conv2d) as combined at
                       train_single.py:121-123
  OurAdamTorch         scene/OurAdam.py:249-337: per-group gather of the relevant rows, the
                       update as separate torch ops, scatter back; dense when nothing is relevant
  densification_stats  train_single.py:193-194 + scene/gaussian_model.py:780-793 with the
                       nonzero()-built visibility filter of gaussian_renderer/__init__.py:124-135
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

_windows = {}


def _window(C, device):
    key = (C, device)
    w = _windows.get(key)
    if w is None:
        g = torch.tensor([math.exp(-((i - 5) ** 2) / (2.0 * 1.5 ** 2)) for i in range(11)], dtype=torch.float32)
        g = g / g.sum()
        w = torch.outer(g, g).expand(C, 1, 11, 11).contiguous().to(device)
        _windows[key] = w
    return w


def ssim(img, gt):
    C = img.shape[-3]
    w = _window(C, img.device)
    blur = lambda t: F.conv2d(t, w, padding=5, groups=C)
    mu1, mu2 = blur(img), blur(gt)
    mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = blur(img * img) - mu1_sq
    s2 = blur(gt * gt) - mu2_sq
    s12 = blur(img * gt) - mu12
    m = ((2 * mu12 + 0.01 ** 2) * (2 * s12 + 0.03 ** 2)) / ((mu1_sq + mu2_sq + 0.01 ** 2) * (s1 + s2 + 0.03 ** 2))
    return m.mean()


def photo_loss(img, gt, lambda_dssim=0.2):
    return (1.0 - lambda_dssim) * torch.abs(img - gt).mean() + lambda_dssim * (1.0 - ssim(img, gt))


class OurAdamTorch(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, relevant):
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                step = st["step"].item()
                sparse = relevant.numel() > 0
                idx = relevant if sparse else slice(None)
                grad, m, v, param = p.grad[idx], st["exp_avg"][idx], st["exp_avg_sq"][idx], p[idx]
                m.mul_(b1).add_(grad, alpha=1 - b1)
                v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
                step_size = group["lr"] / (1 - b1 ** step)
                denom = (v.sqrt() / math.sqrt(1 - b2 ** step)).add_(group["eps"])
                param.addcdiv_(m, denom, value=-step_size)
                if sparse:
                    st["exp_avg"][idx] = m
                    st["exp_avg_sq"][idx] = v
                    p[idx] = param


def densification_stats(g, radii, grad2d):
    vis = (radii > 0).nonzero().flatten().long()
    g.max_radii2D[vis] = torch.max(g.max_radii2D[vis], radii[vis].float())
    n = torch.norm(grad2d[vis, :2], dim=-1, keepdim=True)
    g.xyz_gradient_accum[vis] = torch.max(n, g.xyz_gradient_accum[vis])
    g.denom[vis] += 1
