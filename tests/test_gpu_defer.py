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


def _frame(scene, deg=3, debug=False):
    from diff_gaussian_rasterization import GaussianRasterizer
    inp = torch_inputs(scene, DEV)
    for v in inp.values():
        v.requires_grad_(True)
    color, radii, invd = GaussianRasterizer(settings(scene, DEV, deg, debug=debug))(**inp)
    g = torch.Generator(device=DEV).manual_seed(3)
    (color * torch.randn(color.shape, generator=g, device=DEV)).sum().backward()
    torch.cuda.synchronize()
    return [color.detach(), radii, invd.detach()] + [inp[k].grad for k in ("means3D", "shs", "opacities", "scales",
                                                                            "rotations", "means2D")]


def test_capacity_overflow_rerun_matches():
    from helpers import deterministic
    with deterministic():
        _capacity_overflow_rerun_matches()


def _capacity_overflow_rerun_matches():
    import gs_oracle as O
    small = O.synthetic_scene(200, 160, 120, seed=31, sh_degree=3, log_scale_mean=-3.0)
    big = O.synthetic_scene(20000, 480, 320, seed=32, sh_degree=3, log_scale_mean=-2.0)
    from diff_gaussian_rasterization import _C
    reruns = lambda: _C.forward_stats()["reruns"]
    _C.reset_capacity_hint()  # the hint is the largest K of the last 256 frames: start from a small one
    for _ in range(3):
        _frame(small)
    r0 = reruns()
    a = _frame(big)        # K far above the hint: binned and rendered twice
    r1 = reruns()
    b = _frame(big)        # the hint now covers K: one pass
    r2 = reruns()
    c = _frame(small)      # large hint, small frame
    d = _frame(small)
    r3 = reruns()
    e = _frame(big, debug=True)  # debug mode reads K first and never defers
    assert (r1 - r0, r2 - r1, r3 - r2, reruns() - r3) == (1, 0, 0, 0)
    for x, y in zip(a + c + a, b + d + e):
        assert torch.equal(x, y)
