"""Debug mode at render_coarse's shape (gaussian_renderer/__init__.py:306-417: debug forced on at
:341, SH degree 1 so shs is (P, 4, 3), train_coarse.py:31), at a realistic size: a debug-mode frame
(device-side input snapshots, a synchronize + error check after every stage) returns exactly what
the same frame returns with debug off, forward and backward."""
from __future__ import annotations

import pytest
import torch

from helpers import deterministic, settings, torch_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _frame(scene, debug):
    from diff_gaussian_rasterization import GaussianRasterizer
    inp = torch_inputs(scene, DEV)
    for v in inp.values():
        v.requires_grad_(True)
    color, radii, invd = GaussianRasterizer(settings(scene, DEV, 1, debug=debug))(**inp)
    g = torch.Generator(device=DEV).manual_seed(5)
    loss = (color * torch.randn(color.shape, generator=g, device=DEV)).sum() + \
        (invd * torch.randn(invd.shape, generator=g, device=DEV)).sum()
    loss.backward()
    torch.cuda.synchronize()
    return [color.detach(), radii, invd.detach()] + [inp[k].grad for k in ("means3D", "shs", "opacities", "scales",
                                                                            "rotations", "means2D")]


@pytest.mark.parametrize("host_snapshot", [False, True])
def test_coarse_debug_frame_equals_non_debug(monkeypatch, host_snapshot):
    import gs_oracle as O
    if host_snapshot:
        monkeypatch.setenv("GSR_DEBUG_HOST_SNAPSHOT", "1")
    scene = O.synthetic_scene(200_000, 1920, 1080, seed=41, sh_degree=1, log_scale_mean=-4.5)
    assert scene["shs"].shape[1] == 4
    with deterministic():
        ref = _frame(scene, debug=False)
        got = _frame(scene, debug=True)
    assert int((ref[1] > 0).sum()) > 100_000
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
