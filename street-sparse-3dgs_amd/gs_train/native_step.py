"""NativeTrainStep: TrainStep.step (harness.py) as ONE native call, gsr_train_step
(include/gsr_train.h, csrc/train_step.hip).

The Python step issues ~45 launches through autograd nodes, tensor allocations and ctypes
marshalling, and the host takes about as long to do so as the GPU takes to run them.  Here the
host keeps only the schedule arithmetic of train_single.py (learning rates, Adam step counters and
bias corrections, the depth-loss weight, the random background) and hands the rest to the
executor, which runs the same arithmetic in the same order with several launches fused -- same
results as TrainStep (bit for bit with the deterministic backward; tests/test_gpu_train.py).

The parameters, the Adam moments (the optimizer's own state tensors, so densification and
checkpoint code keep working on them) and the densification statistics stay the Python
objects'.  The gradients land in persistent buffers (`grads`) instead of `.grad`, which stays None
as after TrainStep's zero_grad(set_to_none=True).  `grads` is sparse by default: the opacity
gradient is written for every row each step, the other rows only for the Gaussians the backward
reached this step (every other row's gradient is zero by definition and its buffer row keeps an
older value; the buffers start zeroed).  GSR_STEP_DENSE_ROWS=1 writes every row.
"""
from __future__ import annotations

import ctypes
import math

import torch

from diff_gaussian_rasterization._lib import AdamGroup, TrainStepArgs

from ._native import check, lib, require_gpu, stream
from .harness import LR, TrainStep

_PARAMS = ("_xyz", "_features", "_opacity", "_scaling", "_rotation")


class NativeTrainStep(TrainStep):
    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self._ctx = None
        self._key = None
        ctx = lib().gsr_train_ctx_create()
        if not ctx:
            raise RuntimeError("gsr_train_ctx_create failed")
        self._ctx = ctypes.c_void_p(ctx)

    def ctx_stats(self) -> dict:
        """The executor's grow-only buffers: growths since creation, bytes held, stream-ordered
        growth (gsr_train_ctx_stats)."""
        buf = (ctypes.c_int64 * 3)()
        lib().gsr_train_ctx_stats(self._ctx, buf, 3)
        return {"growths": int(buf[0]), "bytes": int(buf[1]), "stream_ordered": bool(buf[2])}

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            try:
                lib().gsr_train_ctx_destroy(ctx)
            except Exception:  # interpreter shutdown
                pass
            self._ctx = None

    # ---- set-up (again whenever the parameter tensors change, e.g. after densification) ----
    def _state(self, opt, p):
        st = opt.state[p]
        if len(st) == 0:  # Adam.step's lazy initialisation
            st["step"] = torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    def _entries(self, opt, grads):
        """Adam.step's group entries (optim.py), with the gradient pointers of `grads`."""
        out = []
        for group in opt.param_groups:
            for p in group["params"]:
                st = self._state(opt, p)
                row = p.numel() // max(p.shape[0], 1)
                for start, stop, _ in group.get("column_lrs", [(None, None, None)]):
                    start, stop = (0, row) if start is None else (start, stop)
                    off = 4 * start
                    g = grads[id(p)]
                    out.append((group, p, st, start, stop, AdamGroup(
                        p.data_ptr() + off, g.data_ptr() + off, st["exp_avg"].data_ptr() + off,
                        st["exp_avg_sq"].data_ptr() + off, stop - start, 0.0, 0.0, row)))
        return out

    def _setup(self):
        g = self.g
        require_gpu(g._xyz)
        for n in _PARAMS:
            t = getattr(g, n)
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"{n}: the native step needs contiguous float32 parameters")
        dev = g._xyz.device
        self.grads = {n: torch.zeros_like(getattr(g, n)) for n in _PARAMS}
        self.grads["_exposure"] = torch.zeros_like(g._exposure)
        by_id = {id(getattr(g, n)): self.grads[n] for n in _PARAMS + ("_exposure",)}
        self._main = self._entries(self.optimizer, by_id)
        self._expo = self._entries(self.exposure_optimizer, by_id)
        if len(self._expo) != 1:
            raise ValueError("the exposure optimizer must hold the one exposure tensor")
        b = {tuple(gr["betas"]) + (gr["eps"],) for gr in self.optimizer.param_groups}
        if len(b) != 1:
            raise NotImplementedError("fused sparse Adam needs the same betas / eps in every group")
        (b1, b2, eps), = b
        eg = self.exposure_optimizer.param_groups[0]
        self._groups = (AdamGroup * len(self._main))(*[e[5] for e in self._main])
        self._egroup = (AdamGroup * 1)(self._expo[0][5])
        a = TrainStepArgs()
        a.P, a.D, a.M = g.P, g.active_sh_degree, g._features.shape[1]
        a.width, a.height = self.W, self.H
        for n, f in zip(_PARAMS, ("xyz", "features", "opacity", "scaling", "rotation")):
            setattr(a, f, getattr(g, n).data_ptr())
            setattr(a, f + "_grad", self.grads[n].data_ptr())
        a.exposure, a.exposure_grad = g._exposure.data_ptr(), self.grads["_exposure"].data_ptr()
        a.n_images = g._exposure.shape[0]
        a.lambda_dssim = LR["lambda_dssim"]
        a.max_radii2D, a.xyz_gradient_accum, a.denom = (g.max_radii2D.data_ptr(), g.xyz_gradient_accum.data_ptr(),
                                                        g.denom.data_ptr())
        a.n_groups = len(self._main)
        a.groups = self._groups
        a.beta1, a.beta2, a.eps = b1, b2, eps
        a.exposure_group = self._egroup
        a.exposure_beta1, a.exposure_beta2 = eg["betas"]
        a.exposure_eps = eg["eps"]
        a.skybox_rows, a.scaffold_rows = self.skybox, self.scaffold
        a.max_scale = self.extent * 0.02
        self._args = a
        self._key = self._params_key()

    def _params_key(self):
        """Everything the cached argument block points at: the parameters, the statistics and the
        optimizers' moment tensors (load_state_dict or a cleared state swaps those in without
        touching the parameters)."""
        g = self.g
        moments = tuple(
            (id(st), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()) if "exp_avg" in st else (id(st),)
            for opt in (self.optimizer, self.exposure_optimizer) for group in opt.param_groups
            for p in group["params"] for st in (opt.state.get(p, {}),))
        return tuple((getattr(g, n).data_ptr(), tuple(getattr(g, n).shape)) for n in _PARAMS) + \
            (g._exposure.data_ptr(), g.max_radii2D.data_ptr(), g.xyz_gradient_accum.data_ptr(), g.denom.data_ptr(),
             g.active_sh_degree) + moments

    @staticmethod
    def _advance(entries, carr):
        """Adam.step's bookkeeping: one step per parameter, bias corrections in double."""
        seen = {}
        for i, (group, p, st, _start, _stop, _grp) in enumerate(entries):
            if id(p) not in seen:
                st["step"] += 1
                seen[id(p)] = st["step"].item()
            s = seen[id(p)]
            b1, b2 = group["betas"]
            lr = group["lr"]
            if "column_lrs" in group:
                lr = next(l for a0, a1, l in group["column_lrs"] if a0 == _start)
            carr[i].step_size = lr / (1 - b1 ** s)
            carr[i].bias_correction2_sqrt = math.sqrt(1 - b2 ** s)

    def step(self, cam_idx=None, between=None):
        """One iteration through gsr_train_step; returns the loss tensor (no host synchronisation
        unless `between` is given).  between: as TrainStep.step -- the native step stops after the
        exposure step, `between` replaces the parameters, and the scale shrink runs on the new ones
        (no Gaussian Adam step in such an iteration, as in train_single.py)."""
        if self._key is None or self._key != self._params_key():
            self._setup()
        g = self.g
        it = self.iteration
        k = self._view(cam_idx)
        depth_only = self.depth_only[k]
        for pg in self.optimizer.param_groups:
            if pg["name"] == "xyz":
                pg["lr"] = self.xyz_lr(it)
        for pg in self.exposure_optimizer.param_groups:
            pg["lr"] = self.exposure_lr(it)
        if between is None:
            self._advance(self._main, self._groups)
        if not depth_only:
            self._advance(self._expo, self._egroup)
        dev = g._xyz.device
        bg = torch.rand(3, device=dev)
        c = self.cams[k]
        a = self._args
        a.image_index = k
        a.viewmatrix, a.projmatrix, a.campos = c["view"].data_ptr(), c["proj"].data_ptr(), c["campos"].data_ptr()
        a.tan_fovx, a.tan_fovy = c["tx"], c["ty"]
        a.background = bg.data_ptr()
        a.gt = self.gts[k].data_ptr() if not depth_only else None
        am = self.amask[k]
        a.alpha_mask = am.data_ptr() if (am is not None and not depth_only) else None
        w = self.depth_weight(it)
        mono = self.mono[k]
        depth = mono is not None and w > 0
        if depth_only and not depth:
            raise ValueError("a depth-only iteration with no depth weight has no loss (train_single.py:158-161)")
        a.mono_invdepth = mono.data_ptr() if depth else None
        dm = self.dmask[k]
        a.depth_mask = dm.data_ptr() if (depth and dm is not None) else None
        a.depth_weight = w if depth else 0.0
        a.depth_only = int(depth_only)
        a.depth_dens_weight = self.dens_weight
        a.skip_gaussian_step = int(between is not None)
        losses = torch.empty(6, dtype=torch.float32, device=dev)  # a fresh tensor per step, as TrainStep's
        a.losses = losses.data_ptr()
        a.stream = stream(dev).value
        K = ctypes.c_int64(0)
        check(lib().gsr_train_step(self._ctx, ctypes.byref(a), ctypes.byref(K)), "gsr_train_step")
        self.last_K = K.value
        self._bg = bg  # keep the background alive until the stream has used it
        if between is not None:
            with torch.no_grad():
                between()
                self._shrink()
        self.iteration += 1
        return losses[5]
