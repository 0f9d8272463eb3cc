"""Per-image exposure affine + clamp of render() (gaussian_renderer/__init__.py:115-120) as one
gfx950 launch each way (csrc/train.hip).  The reference runs a (H*W, 3) x (3, 3) GEMM, a
broadcast add and a clamp, and autograd adds two more GEMMs and a spatial reduction in backward;
at 1080p that GEMM shape alone costs milliseconds on a BLAS library, while the whole op is a
~50 MB streaming pass."""
from __future__ import annotations

import torch

from ._native import check, lib, ptr, require_gpu, stream


class _Exposure(torch.autograd.Function):
    @staticmethod
    def forward(ctx, color, E):
        require_gpu(color, E)
        if color.dim() != 3 or color.shape[0] != 3 or tuple(E.shape) != (3, 4):
            raise ValueError("expected color (3, H, W) and exposure (3, 4)")
        color = color.detach().float().contiguous()
        E = E.detach().float().contiguous()
        out = torch.empty_like(color)
        n = color.shape[1] * color.shape[2]
        check(lib().gsr_exposure_forward(ptr(color), ptr(E), n, ptr(out), stream(color.device)),
              "gsr_exposure_forward")
        ctx.save_for_backward(color, E)
        return out

    @staticmethod
    def backward(ctx, gout):
        color, E = ctx.saved_tensors
        n = color.shape[1] * color.shape[2]
        gout = gout.float().contiguous()
        L = lib()
        dcolor = torch.empty_like(color)
        dE = torch.empty(3, 4, dtype=torch.float32, device=color.device)
        scratch = torch.empty(max(4, L.gsr_exposure_scratch_bytes(n)), dtype=torch.uint8, device=color.device)
        check(L.gsr_exposure_backward(ptr(color), ptr(E), n, ptr(gout), ptr(dcolor), ptr(dE), ptr(scratch),
                                      stream(color.device)), "gsr_exposure_backward")
        return dcolor, dE


def apply_exposure(color: torch.Tensor, exposure: torch.Tensor) -> torch.Tensor:
    """clamp(matmul(color.permute(1, 2, 0), E[:3, :3]).permute(2, 0, 1) + E[:3, 3, None, None], 0, 1)."""
    return _Exposure.apply(color, exposure)
