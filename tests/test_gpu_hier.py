"""GPU parity of the fused hierarchy-cut interpolation (csrc/hier.hip, include/gsr_hier.h) with the
reference's render_post blend: the reference-generated fixture (tests/golden/render_post.npz),
the numpy restatement (oracle/hier_ref.py) on a larger random cut, and the gradient against
torch autograd through the reference's own formulation in float64 (tolerance 1e-5 relative; the
kernel accumulates shared parents with float atomics)."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

import hier_ref

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"
KEYS = ("means3D", "scales", "rotations", "opacities", "shs")


def _run(f, ri, pi, w, sky, requires_grad=False):
    from gs_train.hier import interpolate_cut
    ts = [torch.tensor(f[k], device=DEV, requires_grad=requires_grad) for k in ("xyz", "scaling", "rotation",
                                                                              "opacity", "features")]
    out = interpolate_cut(*ts, torch.tensor(ri, device=DEV), torch.tensor(pi, device=DEV),
                          torch.tensor(w, device=DEV), sky)
    return ts, out


def test_cut_matches_reference_fixture():
    f = np.load(os.path.join(GOLD, "render_post.npz"))
    _, out = _run(f, f["render_indices"], f["parent_indices"], f["interpolation_weights"], int(f["skybox"]))
    for k, o in zip(KEYS, out):
        np.testing.assert_allclose(o.cpu().numpy(), f["out_" + k], rtol=0, atol=1e-6, err_msg=k)


def _random_cut(N=60_000, R=40_000, S=500, seed=0):
    rng = np.random.default_rng(seed)
    q = rng.normal(size=(N, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    f = dict(xyz=rng.normal(size=(N, 3)).astype(np.float32), scaling=rng.random((N, 3)).astype(np.float32),
             rotation=q, opacity=rng.random((N, 1)).astype(np.float32),
             features=rng.normal(size=(N, 16, 3)).astype(np.float32))
    ri = rng.permutation(N - S)[:R].astype(np.int32)
    pi = rng.integers(0, N - S, R).astype(np.int32)  # parents shared by several rendered nodes
    w = rng.random(N).astype(np.float32)
    return f, ri, pi, w, S


def test_cut_matches_oracle_on_random_cut():
    f, ri, pi, w, S = _random_cut()
    _, out = _run(f, ri, pi, w, S)
    ref = hier_ref.interpolate_cut(f["xyz"], f["scaling"], f["rotation"], f["opacity"], f["features"], ri, pi, w, S)
    for k, o in zip(KEYS, out):
        np.testing.assert_allclose(o.cpu().numpy(), ref[k], rtol=0, atol=2e-6, err_msg=k)


def test_cut_gradient_matches_torch_autograd():
    f, ri, pi, w, S = _random_cut(N=20_000, R=12_000, S=300, seed=1)
    ts, out = _run(f, ri, pi, w, S, requires_grad=True)
    g = torch.Generator().manual_seed(2)
    ups = [torch.randn(o.shape, generator=g).to(DEV) for o in out]
    sum((o * u).sum() for o, u in zip(out, ups)).backward()
    # the reference's formulation (gaussian_renderer/__init__.py:204-229) in float64
    x = [torch.tensor(f[k], dtype=torch.float64, requires_grad=True) for k in ("xyz", "scaling", "rotation",
                                                                             "opacity", "features")]
    r, p = torch.tensor(ri).long(), torch.tensor(pi).long()
    t = torch.tensor(w[:len(ri)], dtype=torch.float64)[:, None]
    sk = torch.arange(f["xyz"].shape[0] - S, f["xyz"].shape[0])
    par = x[2][p]
    sign = torch.where((x[2][r] * par).sum(1, keepdim=True) < 0, -1.0, 1.0).double()
    outs = [t * x[0][r] + (1 - t) * x[0][p], t * x[1][r] + (1 - t) * x[1][p], t * x[2][r] + (1 - t) * par * sign,
            t * x[3][r] + (1 - t) * x[3][p], t[:, :, None] * x[4][r] + (1 - t[:, :, None]) * x[4][p]]
    outs = [torch.cat([o, xx[sk]]) for o, xx in zip(outs, x)]
    sum((o * u.double().cpu()).sum() for o, u in zip(outs, ups)).backward()
    for k, a, b in zip(KEYS, ts, x):
        ga, gb = a.grad.double().cpu().numpy(), b.grad.numpy()
        assert np.abs(ga - gb).max() <= 1e-5 * max(1.0, np.abs(gb).max()), k


def test_cut_then_rasterize_runs_like_render_post():
    """render_post's flow: blend the cut, then rasterize the R + S rows (forward only, as
    render_hierarchy.py runs it)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gs_train.hier import interpolate_cut
    from gs_train.synthetic import synthetic_scene
    s = synthetic_scene(30_000, 320, 240, seed=5)
    N, S = 30_000, 200
    rng = np.random.default_rng(6)
    ri = torch.tensor(rng.permutation(N - S)[:20_000].astype(np.int32), device=DEV)
    pi = torch.tensor(rng.integers(0, N - S, 20_000).astype(np.int32), device=DEV)
    w = torch.tensor(rng.random(N).astype(np.float32), device=DEV)
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=DEV)
    with torch.no_grad():
        m, sc, rot, op, sh = interpolate_cut(t(s["means3D"]), t(s["scales"]), t(s["rotations"]), t(s["opacities"]),
                                             t(s["shs"]), ri, pi, w, S)
        rs = GaussianRasterizationSettings(
            image_height=240, image_width=320, tanfovx=float(s["tanfovx"]), tanfovy=float(s["tanfovy"]),
            bg=t(s["bg"]), scale_modifier=1.0, viewmatrix=t(s["view"]), projmatrix=t(s["proj"]), sh_degree=3,
            campos=t(s["campos"]), prefiltered=False, debug=False, do_depth=True,
            render_indices=torch.empty(0, dtype=torch.int32), parent_indices=torch.empty(0, dtype=torch.int32),
            interpolation_weights=w, num_node_kids=torch.ones(N, dtype=torch.int32, device=DEV))
        color, radii, invd = GaussianRasterizer(rs)(means3D=m, means2D=torch.zeros_like(m), shs=sh,
                                                    colors_precomp=None, opacities=op, scales=sc, rotations=rot,
                                                    cov3D_precomp=None)
    assert color.shape == (3, 240, 320) and radii.shape == (20_200,)
    assert torch.isfinite(color).all() and (radii > 0).sum() > 10_000
