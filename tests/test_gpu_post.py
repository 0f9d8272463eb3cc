"""GPU tests of the train_post.py iteration (gs_train.post.PostTrainStep, train_post.py:69-198):

* the activation-fused LOD blend (gsr_interpolate_cut_*_act: exp / normalize / abs applied to the
  gathered rows) against the reference's formulation (getters, then render_post's gather,
  gaussian_renderer/__init__.py:200-243) in float64 autograd -- forward and the gradients of the raw
  parameters -- on a random cut and at >= 1M cut rows;
* the skybox / anchor gradient zeroing (train_post.py:167-181) against indexing;
* whole iterations against the reference's torch formulation (oracle/train_torch_ref.
  ReferencePostStep: conv2d SSIM, matmul exposure, torch.optim.Adam over split SH groups) on the
  same cut: losses to fp32 rounding, parameters within an fp32 tolerance after 1 and 3 steps.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _raw_cut(N, R, S, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    raw = dict(xyz=torch.randn(N, 3, generator=g, device=DEV), s=-4 + 0.5 * torch.randn(N, 3, generator=g, device=DEV),
               q=torch.randn(N, 4, generator=g, device=DEV), o=torch.randn(N, 1, generator=g, device=DEV),
               sh=torch.randn(N, 16, 3, generator=g, device=DEV))
    ri = torch.randperm(N - S, generator=g, device=DEV)[:R].int()
    pi = torch.randint(0, N - S, (R,), generator=g, device=DEV).int()
    pi[:7] = -1  # roots: the parent reads the last row with weight 0 (hier.hip cut_row)
    w = torch.rand(N, generator=g, device=DEV)
    w[:7] = 1.0
    return raw, ri, pi, w


def _reference_blend(x, ri, pi, w, S, act):
    """render_post's gather (interp_python=True) over the getters' outputs, float64."""
    means, scales, rots, shs = x[0], torch.exp(x[1]), F.normalize(x[2]), x[4]
    opac = torch.abs(x[3]) if act == 2 else torch.sigmoid(x[3])
    r, p = ri.long(), pi.long() % means.shape[0]
    t = w[:len(ri)].double()[:, None]
    par = rots[p]
    sign = torch.where((rots[r] * par).sum(1, keepdim=True) < 0, -1.0, 1.0).double()
    outs = [t * means[r] + (1 - t) * means[p], t * scales[r] + (1 - t) * scales[p], t * rots[r] + (1 - t) * par * sign,
            t * opac[r] + (1 - t) * opac[p], t[:, :, None] * shs[r] + (1 - t[:, :, None]) * shs[p]]
    sk = torch.arange(means.shape[0] - S, means.shape[0], device=means.device)
    full = [means, scales, rots, opac, shs]
    return [torch.cat([o, f[sk]]) for o, f in zip(outs, full)]


@pytest.mark.parametrize("N,R,S,act", [(30_000, 20_000, 300, 2), (30_000, 20_000, 0, 1), (1_500_000, 1_100_000, 10_000, 2)])
def test_cut_act_matches_reference_formulation(N, R, S, act):
    from gs_train.post import interpolate_cut_act
    raw, ri, pi, w = _raw_cut(N, R, S, seed=N % 97 + act)
    xs = [raw[k].clone().requires_grad_(True) for k in ("xyz", "s", "q", "o", "sh")]
    out = interpolate_cut_act(*xs, ri, pi, w, S, opacity_act=act)
    xd = [raw[k].double().clone().requires_grad_(True) for k in ("xyz", "s", "q", "o", "sh")]
    ref = _reference_blend(xd, ri, pi, w, S, act)
    for name, o, r_ in zip(("means", "scales", "rotations", "opacities", "shs"), out, ref):
        assert o.shape == r_.shape, name
        err = (o.double() - r_).abs().max().item()
        assert err <= 2e-6 * max(1.0, r_.abs().max().item()), (name, err)
    g = torch.Generator(device=DEV).manual_seed(11)
    ups = [torch.randn(o.shape, generator=g, device=DEV) for o in out]
    sum((o * u).sum() for o, u in zip(out, ups)).backward()
    sum((o * u.double()).sum() for o, u in zip(ref, ups)).backward()
    for name, a, b in zip(("xyz", "scaling", "rotation", "opacity", "features"), xs, xd):
        ga, gb = a.grad.double(), b.grad
        err = (ga - gb).abs().max().item()
        assert err <= 2e-5 * max(1.0, gb.abs().max().item()), (name, err)


def test_zero_grad_rows_matches_indexing():
    from gs_train.post import zero_grad_rows
    N, S = 50_000, 700
    g = torch.Generator(device=DEV).manual_seed(4)
    ts = [torch.randn(N, w_, generator=g, device=DEV) for w_ in (3, 4, 48, 1, 3)]
    anchors = torch.randint(0, N, (5000,), generator=g, device=DEV)  # repeats allowed
    ref = [t.clone() for t in ts]
    for t in ref:
        t[-S:] = 0
        t[anchors] = 0
    zero_grad_rows(ts, S, anchors)
    for a, b in zip(ts, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("steps", [1, 3])
def test_post_step_matches_reference_formulation(steps):
    """PostTrainStep vs ReferencePostStep on the same views and the same cut limits."""
    from gs_train.post import POST_LR, synthetic_post_problem
    from helpers import assert_adam_trajectories_close, record_margins
    from train_torch_ref import ReferencePostStep
    torch.manual_seed(0)
    post = synthetic_post_problem(60_000, 320, 240, n_views=3, skybox=2000, n_anchors=500, seed=2)
    ref = ReferencePostStep(post)
    limits = [0.004, 0.02, 0.05]
    post.limit_fn = lambda it: limits[(it - 1) % 3]
    m = post.m
    init = [t.detach().clone() for t in (m._xyz, m._features, m._opacity, m._scaling, m._rotation)]
    la, lb = [], []
    for i in range(steps):
        la.append(post.step().item())
        lb.append(ref.step(i % 3, limits[i % 3]).item())
        assert post.last_cut > 1000
    np.testing.assert_allclose(la, lb, rtol=2e-5, atol=1e-7)
    got = (m._xyz, m._features, m._opacity, m._scaling, m._rotation)
    want = (ref._xyz, ref.features(), ref._opacity, ref._scaling, ref._rotation)
    # per-element Adam travel bound; the bulk within 1e-3 of the largest move (an fp32-noise gradient
    # may take an element the other way: Adam's first steps move it by ~lr * sign(grad))
    col_lr = torch.full((1, m._features.shape[1], 1), POST_LR["feature_lr"] / 20.0, device=DEV)
    col_lr[:, 0] = POST_LR["feature_lr"]
    lrs = dict(xyz=max(post.xyz_lr(it) for it in range(0, steps + 2)), features=col_lr,
               opacity=POST_LR["opacity_lr"], scaling=POST_LR["scaling_lr"], rotation=POST_LR["rotation_lr"])
    for name, x, y, x0 in zip(("xyz", "features", "opacity", "scaling", "rotation"), got, want, init):
        x, y = x.detach(), y.detach()
        atol = 2e-6 + 1e-3 * (x - x0).abs().max().item()
        worst, close = assert_adam_trajectories_close(name, x, y, x0, lrs[name], steps, atol)
        record_margins(f"post_step{steps}_{name}", travel_frac=worst, close=close)
    # the locked rows never move: the skybox (last rows) and the anchors
    S = m.skybox_points
    for x, x0 in zip(got, init):
        assert torch.equal(x.detach()[-S:], x0[-S:])
        assert torch.equal(x.detach()[m.anchors], x0[m.anchors])


@pytest.mark.parametrize("limit", [0.004, 0.02, 0.08])
def test_cut_unique_children_writes_match_accumulation(limit):
    """A real cut (expand_to_size over a synthetic hierarchy): the backward that writes the child
    rows (GSR_CUT_UNIQUE_CHILDREN) equals the accumulating one -- child rows exactly (an atomic add
    into a zero row is the value), parent rows to fp32 summation order -- and the reference
    formulation (float64 autograd of the getters + render_post's gather)."""
    from gs_train.post import interpolate_cut_act, synthetic_post_problem
    post = synthetic_post_problem(60_000, 320, 240, n_views=2, skybox=2000, n_anchors=100, seed=5)
    m = post.m
    n = post.cut(0, limit)
    ri, pi, w = post.ri[:n], post.pi, post.w
    assert n > 1000 and torch.unique(ri).numel() == n
    S = m.skybox_points
    raw = [m._xyz, m._scaling, m._rotation, m._opacity, m._features]
    g = torch.Generator(device=DEV).manual_seed(3)
    grads = {}
    for uniq in (False, True):
        xs = [t.detach().clone().requires_grad_(True) for t in raw]
        out = interpolate_cut_act(*xs, ri, pi, w, S, unique_children=uniq)
        if not grads:
            ups = [torch.randn(o.shape, generator=g, device=DEV) for o in out]
        sum((o * u).sum() for o, u in zip(out, ups)).backward()
        grads[uniq] = [x.grad.detach() for x in xs]
    child = ri.long()
    for a, b in zip(grads[True], grads[False]):
        assert torch.equal(a[child], b[child])
        err = (a - b).abs().max().item()
        assert err <= 1e-5 * max(1.0, b.abs().max().item()), err
    xd = [t.detach().double().clone().requires_grad_(True) for t in raw]
    ref = _reference_blend(xd, ri, pi[:n], w, S, 2)
    sum((o * u.double()).sum() for o, u in zip(ref, ups)).backward()
    for a, b in zip(grads[True], xd):
        err = (a.double() - b.grad).abs().max().item()
        assert err <= 2e-5 * max(1.0, b.grad.abs().max().item()), err
