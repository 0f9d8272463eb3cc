"""Fused sparse Adam: a drop-in for scene/OurAdam.Adam (scene/OurAdam.py:80-175) as the Gaussian
model uses it (scene/gaussian_model.py:286-296, train_single.py:224-231).

Same constructor, `param_groups` and per-parameter state keys ('step', 'exp_avg',
'exp_avg_sq'), so GaussianModel's learning-rate schedule and its densification bookkeeping
(which edits optimizer.state directly) keep working.  A group may also carry
`column_lrs = [(start, stop, lr), ...]`: column blocks of each row of its parameter, each with its
own learning rate, so the DC and rest SH coefficients can live in one (P, 16, 3) tensor (no
torch.cat / split per step) and still get f_dc's and f_rest's rates.  `step(relevant)` accepts the reference's
index tensor; `step(relevance=opacity.grad)` skips the host-synchronising nonzero() and tests
relevance per row on the device.  Either way all groups are updated by ONE gfx950 launch
(csrc/train.hip) that reads (param, grad, m, v) and writes (param, m, v) once for the relevant
rows; with no relevant row every row is updated (OurAdam's _single_tensor_adam2 branch).

Arithmetic follows _single_tensor_adam (scene/OurAdam.py:249-337): step counters are host
floats, bias corrections are computed in double on the host, and the row update is
m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps).
"""
from __future__ import annotations

import math

import torch

from diff_gaussian_rasterization._lib import AdamGroup

from ._native import check, lib, ptr, require_gpu, stream


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 foreach=None, maximize=False, capturable=False):
        if not 0.0 <= lr:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if not 0.0 <= eps:
            raise ValueError("Invalid epsilon value: {}".format(eps))
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError("Invalid beta parameter at index 0: {}".format(betas[0]))
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError("Invalid beta parameter at index 1: {}".format(betas[1]))
        if not 0.0 <= weight_decay:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        if weight_decay != 0 or amsgrad or maximize:
            raise NotImplementedError("fused sparse Adam: weight_decay / amsgrad / maximize are not used by the "
                                      "reference and not implemented")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable)
        super().__init__(params, defaults)
        self._flag = {}

    def _flag_for(self, device):
        f = self._flag.get(device)
        if f is None:
            f = torch.zeros(1, dtype=torch.int32, device=device)
            self._flag[device] = f
        return f

    @torch.no_grad()
    def step(self, relevant=None, closure=None, *, relevance=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        entries = []
        betas = None
        eps = None
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            if betas is not None and (betas != (beta1, beta2) or eps != group["eps"]):
                raise NotImplementedError("fused sparse Adam needs the same betas / eps in every group")
            betas, eps = (beta1, beta2), group["eps"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients, please consider SparseAdam instead")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state["step"] += 1
                st = state["step"].item()
                for start, stop, lr in group.get("column_lrs", [(None, None, group["lr"])]):
                    entries.append((p, state, lr / (1 - beta1 ** st), math.sqrt(1 - beta2 ** st), start, stop))
        if not entries:
            return loss
        P = entries[0][0].shape[0]
        dev = entries[0][0].device
        groups = (AdamGroup * len(entries))()
        keep = []
        for k, (p, state, step_size, bc2s, start, stop) in enumerate(entries):
            require_gpu(p)
            if p.shape[0] != P or p.device != dev:
                raise ValueError("fused sparse Adam: every parameter must have the same number of rows")
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("fused sparse Adam: parameters must be contiguous float32")
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            m, v = state["exp_avg"], state["exp_avg_sq"]
            if not (m.is_contiguous() and v.is_contiguous()):
                raise ValueError("fused sparse Adam: moment buffers must be contiguous")
            keep.append(g)
            row = p.numel() // max(P, 1)
            if start is None:
                start, stop = 0, row
            if not 0 <= start < stop <= row:
                raise ValueError(f"column_lrs block ({start}, {stop}) outside a row of {row} values")
            off = 4 * start  # bytes
            groups[k] = AdamGroup(p.data_ptr() + off, g.data_ptr() + off, m.data_ptr() + off, v.data_ptr() + off,
                                  stop - start, step_size, bc2s, row)
        if relevance is not None:
            rel = relevance.detach().reshape(-1)
            if rel.numel() != P:
                raise ValueError("relevance must have one value per row")
            rel = rel.float().contiguous()
        elif relevant is not None and relevant.numel() > 0:
            rel = torch.zeros(P, dtype=torch.float32, device=dev)
            rel.index_fill_(0, relevant.to(dev).flatten().long(), 1.0)
        else:
            rel = None  # no relevant row given: the dense update, as OurAdam's fallback branch
        check(lib().gsr_sparse_adam_step(len(entries), groups, P, ptr(rel), betas[0], betas[1], eps,
                                         ptr(self._flag_for(dev)), stream(dev)), "gsr_sparse_adam_step")
        return loss
