"""The forward queues its binning and render before reading K when it has a capacity hint from the
previous frame (csrc/rasterizer.hip, GSR_DEFER_K).  A frame whose K exceeds that capacity is
binned and rendered again at K: its outputs and gradients must equal those of the same frame
rendered with enough capacity, bit for bit."""
from __future__ import annotations

import pytest
import torch

from helpers import settings, torch_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _frame(scene, deg=3):
    from diff_gaussian_rasterization import GaussianRasterizer
    inp = torch_inputs(scene, DEV)
    for v in inp.values():
        v.requires_grad_(True)
    color, radii, invd = GaussianRasterizer(settings(scene, DEV, deg))(**inp)
    g = torch.Generator(device=DEV).manual_seed(3)
    (color * torch.randn(color.shape, generator=g, device=DEV)).sum().backward()
    torch.cuda.synchronize()
    return [color.detach(), radii, invd.detach()] + [inp[k].grad for k in ("means3D", "shs", "opacities", "scales",
                                                                            "rotations", "means2D")]


def test_capacity_overflow_rerun_matches():
    import gs_oracle as O
    small = O.synthetic_scene(200, 160, 120, seed=31, sh_degree=3, log_scale_mean=-3.0)
    big = O.synthetic_scene(20000, 480, 320, seed=32, sh_degree=3, log_scale_mean=-2.0)
    _frame(small)          # leaves a small capacity hint
    a = _frame(big)        # K far above the hint: binned and rendered twice
    b = _frame(big)        # the hint now covers K: one pass
    c = _frame(small)      # large hint, small frame
    d = _frame(small)
    for x, y in zip(a + c, b + d):
        assert torch.equal(x, y)
