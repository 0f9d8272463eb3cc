"""GPU parity of the hierarchy LOD cut (csrc/lod.hip through the gaussian_hierarchy drop-in) with its
C restatement (oracle/gs_oracle.c; parity unpinned against the un-vendored gaussianhierarchy
extension -- see tests/test_lod_cpu.py for what pins the restatement), and config 5 end to end:
render_hierarchy.py's per-frame work -- expand_to_size at a tau threshold, get_interpolation_weights,
render_post's blend, the forward render at 1080p -- on a synthetic 10M-node hierarchy, against the
oracle on the same rows (bit-exact cut, weights, radii, K and tile lists; PSNR >= 80 dB)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import hier_ref
from helpers import psnr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cut_hip(h, thr, vp=None):
    from gaussian_hierarchy._C import expand_to_size, get_interpolation_weights
    N = h["nodes"].shape[0]
    ri, pi, ni = (torch.zeros(N, dtype=torch.int32, device=DEV) for _ in range(3))
    w = torch.zeros(N, device=DEV)
    k = torch.zeros(N, dtype=torch.int32, device=DEV)
    cam = torch.tensor(h["campos"] if vp is None else vp, device=DEV)
    n = expand_to_size(h["nodes"], h["boxes"], thr, cam, torch.zeros(3), ri, pi, ni)
    get_interpolation_weights(ni[:n], thr, h["nodes"], h["boxes"], cam.cpu(), torch.zeros(3), w, k)
    return n, ri, pi, ni, w, k


@pytest.mark.parametrize("tau,vp", [(3.0, None), (15.0, None), (60.0, (0.3, 0.1, 4.0)), (6.0, (0.0, 0.0, -50.0))])
def test_lod_cut_matches_oracle(tau, vp):
    import gs_oracle as O
    from gs_train.synthetic import synthetic_lod_hierarchy, tau_threshold
    h = synthetic_lod_hierarchy(400_000, 1920, 1080, DEV, seed=7, zmin=1.0, zmax=30.0, log_scale_mean=-3.5)
    thr = float(np.float32(tau_threshold(tau, h["tanfovx"], 1920)))
    n, ri, pi, ni, w, k = _cut_hip(h, thr, vp)
    nodes, boxes = h["nodes"].cpu().numpy(), h["boxes"].cpu().numpy()
    v = np.asarray(h["campos"] if vp is None else vp, np.float32)
    ori, opi, oni = O.expand_to_size(nodes, boxes, np.float32(thr), v)
    ow, ok = O.interpolation_weights(oni, np.float32(thr), nodes, boxes, v)
    assert n == len(ori) and n > 0
    np.testing.assert_array_equal(ri[:n].cpu().numpy(), ori)
    np.testing.assert_array_equal(pi[:n].cpu().numpy(), opi)
    np.testing.assert_array_equal(ni[:n].cpu().numpy(), oni)
    np.testing.assert_array_equal(w[:n].cpu().numpy(), ow)
    np.testing.assert_array_equal(k[:n].cpu().numpy(), ok)
    # outputs beyond the cut are untouched (the reference slices [:to_render])
    assert int(ri[n:].abs().sum()) == 0 and float(w[n:].abs().sum()) == 0.0


def test_config5_end_to_end_vs_oracle():
    """Config 5: a 10M-node hierarchy (7.5M leaves), the cut at tau = 3 px seen from the camera,
    blended with the parents and rendered at 1920x1080 (forward, do_depth), against the oracle."""
    import gs_oracle as O
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gs_train.hier import interpolate_cut
    from gs_train.synthetic import synthetic_lod_hierarchy, tau_threshold
    W, H = 1920, 1080
    h = synthetic_lod_hierarchy(7_500_000, W, H, DEV, seed=5, skybox=20_000)
    N = h["nodes"].shape[0]
    assert N >= 10_000_000
    thr = float(np.float32(tau_threshold(3.0, h["tanfovx"], W)))
    n, ri, pi, ni, w, k = _cut_hip(h, thr)
    assert 1_000_000 < n < N
    # the cut against the oracle
    ori, opi, oni = O.expand_to_size(h["nodes"].cpu().numpy(), h["boxes"].cpu().numpy(), np.float32(thr),
                                     h["campos"])
    np.testing.assert_array_equal(ri[:n].cpu().numpy(), ori)
    np.testing.assert_array_equal(pi[:n].cpu().numpy(), opi)
    S = h["skybox"]
    with torch.no_grad():
        m, sc, rot, op, sh = interpolate_cut(h["means3D"], h["scales"], h["rotations"], h["opacities"], h["shs"],
                                             ri[:n], pi, w, S)
    rows = n + S
    # blended rows vs the numpy restatement of render_post on a sample of rows
    smp = np.random.default_rng(0).choice(n, 20_000, replace=False)
    idx = np.concatenate([ori[smp], opi[smp][opi[smp] >= 0]])
    uniq, inv = np.unique(idx, return_inverse=True)
    take = lambda t: t[torch.tensor(uniq, device=DEV)].cpu().numpy()
    f = dict(xyz=take(h["means3D"]), scaling=take(h["scales"]), rotation=take(h["rotations"]),
             opacity=take(h["opacities"]), features=take(h["shs"]))
    loc_c = inv[:len(smp)]
    loc_p = np.where(opi[smp] >= 0, 0, -1)
    loc_p[opi[smp] >= 0] = inv[len(smp):]
    ref = hier_ref.interpolate_cut(f["xyz"], f["scaling"], f["rotation"], f["opacity"], f["features"], loc_c,
                                   np.where(loc_p < 0, loc_c, loc_p), w[:n].cpu().numpy()[smp], 0)
    for name, got in (("means3D", m), ("scales", sc), ("rotations", rot), ("opacities", op), ("shs", sh)):
        np.testing.assert_array_equal(got[torch.tensor(smp, device=DEV)].cpu().numpy(), ref[name], err_msg=name)
    # forward render of the cut vs the oracle
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=DEV)
    bg = np.array([0.1, 0.2, 0.3], np.float32)
    rs = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=float(h["tanfovx"]), tanfovy=float(h["tanfovy"]), bg=t(bg),
        scale_modifier=1.0, viewmatrix=t(h["view"]).reshape(4, 4), projmatrix=t(h["proj"]).reshape(4, 4),
        sh_degree=3, campos=t(h["campos"]), prefiltered=False, debug=False, do_depth=True,
        render_indices=torch.empty(0, dtype=torch.int32), parent_indices=torch.empty(0, dtype=torch.int32),
        interpolation_weights=w, num_node_kids=k)
    with torch.no_grad():
        color, radii, invd = GaussianRasterizer(rs)(means3D=m, means2D=torch.zeros_like(m), shs=sh, opacities=op,
                                                    scales=sc, rotations=rot)
    torch.cuda.synchronize()
    cpu = lambda x: x.cpu().numpy()
    st = O.forward(cpu(m), cpu(op), h["view"], h["proj"], h["campos"], bg, W, H, h["tanfovx"], h["tanfovy"],
                   sh_degree=3, shs=cpu(sh), scales=cpu(sc), rotations=cpu(rot))
    np.testing.assert_array_equal(cpu(radii), st["radii"])
    assert int((radii > 0).sum()) > 1_000_000 and rows == m.shape[0]
    p = psnr(cpu(color), st["color"])
    assert p >= 80.0, p
    assert float(np.mean(np.abs(cpu(color) - st["color"]) > 1e-4)) <= 1e-3


def test_rasterizer_render_indices_equal_render_post_blend():
    """Non-empty render_indices in the rasterizer (the blend done inside gsr_rasterize_forward)
    against render_post's order of work (interpolate_cut, then the rasterizer on the R rows):
    identical image / radii / K; gradients of the N hierarchy rows equal up to the order of the
    float atomics that sum shared parents; means2D's gradient in rows [0, R)."""
    from helpers import deterministic
    with deterministic():
        _render_indices_equal_render_post_blend()


def _render_indices_equal_render_post_blend():
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gs_train.hier import interpolate_cut
    from gs_train.synthetic import synthetic_lod_hierarchy, tau_threshold
    W, H = 640, 360
    h = synthetic_lod_hierarchy(60_000, W, H, DEV, seed=9, zmin=1.0, zmax=12.0, log_scale_mean=-3.5)
    thr = tau_threshold(20.0, h["tanfovx"], W)
    n, ri, pi, ni, w, k = _cut_hip(h, thr)
    N = h["means3D"].shape[0]
    assert 0 < n < N
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(1)
    gc = torch.randn(3, H, W, generator=g, device=DEV)
    gd = torch.randn(1, H, W, generator=g, device=DEV)

    def settings(ri_, pi_, w_):
        return GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=float(h["tanfovx"]), tanfovy=float(h["tanfovy"]),
            bg=t([0.3, 0.2, 0.1]), scale_modifier=1.0, viewmatrix=t(h["view"]).reshape(4, 4),
            projmatrix=t(h["proj"]).reshape(4, 4), sh_degree=3, campos=t(h["campos"]), prefiltered=False,
            debug=False, do_depth=True, render_indices=ri_, parent_indices=pi_, interpolation_weights=w_,
            num_node_kids=k)

    def leaves():
        return [h[x].detach().clone().requires_grad_(True) for x in ("means3D", "scales", "rotations", "opacities",
                                                                      "shs")]

    # (a) inside the rasterizer
    m, sc, rot, op, sh = leaves()
    m2a = torch.zeros(N, 3, device=DEV, requires_grad=True)
    ca, ra, da = GaussianRasterizer(settings(ri[:n], pi, w))(means3D=m, means2D=m2a, shs=sh, opacities=op,
                                                             scales=sc, rotations=rot)
    ((ca * gc).sum() + (da * gd).sum()).backward()
    ga = [x.grad for x in (m, sc, rot, op, sh)]
    # (b) render_post's order: blend, then rasterize the R rows
    m, sc, rot, op, sh = leaves()
    bm, bs, br, bo, bsh = interpolate_cut(m, sc, rot, op, sh, ri[:n], pi, w, 0)
    m2b = torch.zeros(n, 3, device=DEV, requires_grad=True)
    e = torch.empty(0, dtype=torch.int32)
    cb, rb, db = GaussianRasterizer(settings(e, e, torch.empty(0, device=DEV)))(
        means3D=bm, means2D=m2b, shs=bsh, opacities=bo, scales=bs, rotations=br)
    ((cb * gc).sum() + (db * gd).sum()).backward()
    gb = [x.grad for x in (m, sc, rot, op, sh)]
    assert torch.equal(ca, cb) and torch.equal(da, db) and torch.equal(ra, rb)
    assert ra.shape[0] == n
    for name, x, y in zip(("means3D", "scales", "rotations", "opacities", "shs"), ga, gb):
        err = float((x - y).norm() / y.norm().clamp_min(1e-30))
        assert err <= 1e-6, (name, err)
    assert torch.equal(m2a.grad[:n], m2b.grad) and int(m2a.grad[n:].abs().sum()) == 0
