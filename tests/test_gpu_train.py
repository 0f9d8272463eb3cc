"""GPU parity of the train-step kernels (csrc/train.hip) through their C ABI (include/gsr_train.h)
against the reference-generated fixtures and the CPU oracle (oracle/train_ref.py), and the
train-step harness end to end.

Tolerances (fp32 kernels vs fp32/fp64 references):
  loss values  |diff| <= 2e-6 (L1, SSIM means of O(1) quantities)
  loss grad    max |diff| <= 1e-5 * max|grad| (separable vs 2-D window rounding)
  Adam         atol 5e-7 on params (a few fp32 ulps after three steps), moments rtol 1e-6
  densify      exact (max / +1) and 1 ulp for the 2-norm
"""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

import train_ref as TR

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
DEV = "cuda"


def test_l1_ssim_matches_reference_fixtures():
    from gs_train import l1_ssim
    d = np.load(os.path.join(GOLD, "loss.npz"))
    for k in range(int(d["n"])):
        img = torch.tensor(d[f"img_{k}"], device=DEV, requires_grad=True)
        gt = torch.tensor(d[f"gt_{k}"], device=DEV)
        v = l1_ssim(img, gt)
        loss = 0.8 * v[0] + 0.2 * (1 - v[1])
        loss.backward()
        assert abs(v[0].item() - float(d[f"l1_{k}"])) <= 2e-6, k
        assert abs(v[1].item() - float(d[f"ssim_{k}"])) <= 2e-6, k
        ref = d[f"grad_{k}"]
        err = np.abs(img.grad.cpu().numpy() - ref).max()
        assert err <= 1e-5 * np.abs(ref).max(), (k, err)


@pytest.mark.parametrize("shape", [(3, 270, 480), (3, 1080, 1920), (2, 3, 65, 130)])
def test_l1_ssim_matches_oracle_fp64(shape):
    from gs_train import l1_ssim
    g = torch.Generator().manual_seed(sum(shape))
    img = torch.rand(shape, generator=g)
    gt = (img + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1)
    x = img.double().requires_grad_(True)
    flat = lambda t: t.reshape(-1, *t.shape[-2:]) if t.dim() == 4 else t
    l1, s = TR.l1(flat(x), flat(gt.double())), TR.ssim(flat(x), flat(gt.double()))
    (0.8 * l1 + 0.2 * (1 - s)).backward()
    xi = img.to(DEV).requires_grad_(True)
    v = l1_ssim(xi, gt.to(DEV))
    (0.8 * v[0] + 0.2 * (1 - v[1])).backward()
    assert abs(v[0].item() - l1.item()) <= 2e-6
    assert abs(v[1].item() - s.item()) <= 2e-6
    ref = x.grad.float().numpy()
    got = xi.grad.cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_l1_ssim_is_deterministic_and_gt_gets_no_grad():
    from gs_train import l1_ssim
    img = torch.rand(3, 200, 333, device=DEV, requires_grad=True)
    gt = torch.rand(3, 200, 333, device=DEV, requires_grad=True)
    a = l1_ssim(img, gt)
    b = l1_ssim(img, gt)
    assert torch.equal(a, b)
    a.sum().backward()
    g1 = img.grad.clone()
    img.grad = None
    b.sum().backward()
    assert torch.equal(g1, img.grad)
    assert gt.grad is None


@pytest.mark.parametrize("shape", [(3, 1080, 1920), (3, 77, 131)])
def test_l1_ssim_map_path_equals_direct_backward(shape):
    """Training runs gsr_l1_ssim_forward_with_map + the elementwise backward; the gradient must be
    bit-identical to gsr_l1_ssim_backward's and the loss equal to the plain forward's (up to the
    order of the per-block sums)."""
    from gs_train import l1_ssim
    from gs_train._native import lib, ptr, stream
    g = torch.Generator().manual_seed(7)
    img = torch.rand(shape, generator=g).to(DEV).requires_grad_(True)
    gt = torch.rand(shape, generator=g).to(DEV)
    v = l1_ssim(img, gt)
    up = torch.tensor([0.8, -0.2], device=DEV)
    (v * up).sum().backward()
    with torch.no_grad():
        v0 = l1_ssim(img, gt)
    assert torch.allclose(v, v0, rtol=0, atol=1e-6)
    direct = torch.empty_like(img)
    C, H, W = shape
    assert lib().gsr_l1_ssim_backward(ptr(img.detach()), ptr(gt), C, H, W, ptr(up), ptr(direct), stream(img.device)) == 0
    torch.cuda.synchronize()
    assert torch.equal(img.grad, direct)


@pytest.mark.parametrize("shape", [(3, 1080, 1920), (3, 77, 131), (1, 200, 64), (2, 64, 63), (1, 5, 9)])
def test_l1_ssim_streaming_equals_tiled(shape, monkeypatch):
    """The streaming gradient kernel (64 x 64 strips, LDS rings) and the 64 x 16 tile kernel form
    every value with the same fmaf order: G and dx must agree bit for bit (GSR_SSIM_TILED=1
    selects the tile kernel)."""
    from gs_train._native import lib, ptr, stream
    g = torch.Generator().manual_seed(11)
    img = torch.rand(shape, generator=g).to(DEV)
    gt = torch.rand(shape, generator=g).to(DEV)
    C, H, W = shape
    up = torch.tensor([0.8, -0.2], device=DEV)
    L = lib()
    scratch = torch.empty(L.gsr_l1_ssim_scratch_bytes(C, H, W), dtype=torch.uint8, device=DEV)
    res = {}
    for tiled in ("0", "1"):
        monkeypatch.setenv("GSR_SSIM_TILED", tiled)
        dx = torch.empty_like(img)
        gmap = torch.empty_like(img)
        out = torch.empty(2, device=DEV)
        s = stream(img.device)
        assert L.gsr_l1_ssim_backward(ptr(img), ptr(gt), C, H, W, ptr(up), ptr(dx), s) == 0
        assert L.gsr_l1_ssim_forward_with_map(ptr(img), ptr(gt), C, H, W, ptr(scratch), ptr(out), ptr(gmap), s) == 0
        torch.cuda.synchronize()
        res[tiled] = (dx, gmap, out)
    assert torch.equal(res["0"][0], res["1"][0])
    assert torch.equal(res["0"][1], res["1"][1])
    assert torch.allclose(res["0"][2], res["1"][2], rtol=0, atol=1e-6)


def _adam_from_fixture(use_index):
    from gs_train import Adam
    d = np.load(os.path.join(GOLD, "adam.npz"))
    params = [torch.nn.Parameter(torch.tensor(d[f"init_{n}"], device=DEV)) for n in NAMES]
    opt = Adam([{"params": [p], "lr": float(lr), "name": n} for p, lr, n in zip(params, d["lrs"], NAMES)],
               lr=0.0, eps=1e-15)
    for it in range(3):
        for j, n in enumerate(NAMES):
            params[j].grad = torch.tensor(d[f"grad{it}_{n}"], device=DEV)
        if use_index:
            opt.step((params[3].grad.flatten() != 0).nonzero().flatten().long())
        else:
            opt.step(relevance=params[3].grad)
        for j, n in enumerate(NAMES):
            st = opt.state[params[j]]
            np.testing.assert_allclose(params[j].detach().cpu().numpy(), d[f"after{it}_{n}"], rtol=0, atol=5e-7,
                                       err_msg=f"{n} step {it}")
            np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), d[f"m{it}_{n}"], rtol=0, atol=2e-7)
            np.testing.assert_allclose(st["exp_avg_sq"].cpu().numpy(), d[f"v{it}_{n}"], rtol=1e-6, atol=1e-9)
    return [p.detach().cpu() for p in params]


def test_sparse_adam_matches_reference_ouradam():
    a = _adam_from_fixture(use_index=False)
    b = _adam_from_fixture(use_index=True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_sparse_adam_coarse_pair_index_quirk():
    """train_coarse.py:133-134 hands OurAdam `(opacity.grad != 0).nonzero()` of the (P, 1) gradient:
    an (R, 2) index whose second column is 0.  OurAdam's gather / scatter
    (scene/OurAdam.py:267-270,334-337) then also updates row 0 once per step (its copies are all
    updated alike).  gs_train.optim.Adam.step(relevant) flattens the index, which marks the same
    rows: bit for bit (within fp32 ulps) the reference run in tests/golden/adam_coarse.npz, where
    row 0 is never relevant by itself."""
    from gs_train import Adam
    d = np.load(os.path.join(GOLD, "adam_coarse.npz"))
    params = [torch.nn.Parameter(torch.tensor(d[f"init_{n}"], device=DEV)) for n in NAMES]
    opt = Adam([{"params": [p], "lr": float(lr), "name": n} for p, lr, n in zip(params, d["lrs"], NAMES)],
               lr=0.0, eps=1e-15)
    for it in range(2):
        for j, n in enumerate(NAMES):
            params[j].grad = torch.tensor(d[f"grad{it}_{n}"], device=DEV)
        relevant = (params[3].grad != 0).nonzero()
        assert tuple(relevant.shape) == tuple(d[f"relevant{it}"].shape)
        opt.step(relevant)
        for j, n in enumerate(NAMES):
            got = params[j].detach().cpu().numpy()
            np.testing.assert_allclose(got, d[f"after{it}_{n}"], rtol=0, atol=5e-7, err_msg=f"{n} step {it}")
            # row 0 moved although its opacity gradient is zero (the quirk); its opacity (zero gradient,
            # zero moments at the first step) cannot move
            if it == 0 and n != "opacity":
                assert not np.array_equal(got[0], d[f"init_{n}"][0]), n
            np.testing.assert_allclose(opt.state[params[j]]["exp_avg"].cpu().numpy(), d[f"m{it}_{n}"], rtol=0,
                                       atol=2e-7)


def test_sparse_adam_large_matches_oracle():
    from gs_train import Adam
    P = 300_001
    g = torch.Generator().manual_seed(3)
    shapes = [(3,), (1, 3), (15, 3), (1,), (3,), (4,)]
    lrs = [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3]
    host = [torch.randn((P,) + s, generator=g) for s in shapes]
    params = [torch.nn.Parameter(h.to(DEV)) for h in host]
    opt = Adam([{"params": [p], "lr": lr} for p, lr in zip(params, lrs)], lr=0.0, eps=1e-15)
    m = [torch.zeros_like(h) for h in host]
    v = [torch.zeros_like(h) for h in host]
    steps = [0] * 6
    for it in range(2):
        grads = [torch.randn((P,) + s, generator=g) for s in shapes]
        grads[3][torch.rand(P, generator=g) < 0.3] = 0.0
        for p, gr in zip(params, grads):
            p.grad = gr.to(DEV)
        opt.step(relevance=params[3].grad)
        steps = TR.sparse_adam(host, grads, m, v, steps, lrs, grads[3])
    for p, h in zip(params, host):
        np.testing.assert_allclose(p.detach().cpu().numpy(), h.numpy(), rtol=0, atol=5e-7)


def test_densify_stats_matches_reference():
    from gs_train import add_densification_stats
    d = np.load(os.path.join(GOLD, "densify.npz"))
    t = lambda k: torch.tensor(d[k], device=DEV).contiguous()
    mr, acc, den = t("max_r"), t("accum"), t("denom")
    add_densification_stats(t("radii"), t("grad2d"), mr, acc, den)
    np.testing.assert_array_equal(mr.cpu().numpy(), d["max_r_after"])
    np.testing.assert_allclose(acc.cpu().numpy(), d["accum_after"], rtol=2e-7, atol=0)
    np.testing.assert_array_equal(den.cpu().numpy(), d["denom_after"])


@pytest.mark.parametrize("depth,alpha,skybox,scaffold", [(False, False, 0, 0), (True, True, 500, 0),
                                                          (True, False, 300, 2000)])
def test_train_step_fused_matches_reference_structured_step(depth, alpha, skybox, scaffold):
    """The fused Street-sparse iteration against the reference's torch formulation of it
    (oracle/train_torch_ref.ReferenceTrainStep): with and without the masked inverse-depth L1,
    the alpha mask and a locked skybox."""
    from gs_train.harness import LR, make_problem
    from helpers import assert_adam_trajectories_close, record_margins
    from train_torch_ref import ReferenceTrainStep
    names = ("_xyz", "_features_dc", "_opacity", "_scaling", "_rotation")
    steps, n_steps = {}, 3
    for fused in (True, False):
        torch.manual_seed(0)
        ts = make_problem(20_000, 256, 192, n_views=3, seed=1, step_cls=None if fused else ReferenceTrainStep,
                          depth=depth, alpha=alpha, skybox_points=skybox, scaffold_points=scaffold)
        if scaffold:  # some over-large Gaussians on both sides of the scaffold boundary: the shrink runs
            with torch.no_grad():
                ts.g._scaling[scaffold - 50:scaffold + 50] += 3.0
        init = [getattr(ts.g, n).detach().clone() for n in names]
        xyz_lr = max(ts.xyz_lr(it) for it in range(0, n_steps + 2))
        losses = [ts.step().item() for _ in range(n_steps)]
        steps[fused] = (losses, [getattr(ts.g, n).detach().clone() for n in names], ts.g.xyz_gradient_accum.clone(),
                        ts.g.denom.clone(), init)
    (la, pa, aa, da, ia), (lb, pb, ab, db, _) = steps[True], steps[False]
    np.testing.assert_allclose(la, lb, rtol=1e-5, atol=1e-6)
    # Adam's first steps move each element by ~lr * sign(grad): an element whose gradient is fp32
    # noise around zero may legitimately go the other way, so the bulk is compared within atol and
    # EVERY element within twice the Adam travel (helpers.assert_adam_trajectories_close; a
    # mis-indexed row fails it: profiles/r06_mutation_check.txt).
    lrs = dict(_xyz=xyz_lr, _features_dc=LR["feature_lr"], _opacity=LR["opacity_lr"], _scaling=LR["scaling_lr"],
               _rotation=LR["rotation_lr"])
    for n, x, y, x0 in zip(names, pa, pb, ia):
        worst, close = assert_adam_trajectories_close(n, x, y, x0, lrs[n], n_steps, atol=1e-5)
        record_margins(f"fused_vs_reference_step_{depth}_{alpha}_{skybox}_{scaffold}{n}", travel_frac=worst,
                       close=close)
    assert torch.equal(da, db)
    assert torch.isclose(aa, ab, rtol=1e-3, atol=1e-9).float().mean().item() >= 0.999
    if scaffold:  # the scaffold rows are never shrunk; the big rows after them are
        s0, s1 = ia[names.index("_scaling")], pa[names.index("_scaling")]
        assert torch.all(s1[scaffold - 50:scaffold] > s0[scaffold - 50:scaffold] - 0.05)
        assert torch.all(s1[scaffold:scaffold + 50] < s0[scaffold:scaffold + 50] - 0.2)
    if skybox:  # the locked rows never move (the scale shrink aside, which the reference applies to them too)
        for x, x0, name in zip(pa, ia, names):
            if name != "_scaling":
                assert torch.equal(x[:skybox], x0[:skybox]), name


@pytest.mark.parametrize("depth,alpha,skybox,scaffold", [(True, False, 0, 0), (False, True, 300, 0),
                                                          (True, True, 300, 2000)])
def test_native_step_equals_python_step(depth, alpha, skybox, scaffold):
    """gsr_train_step (gs_train.native_step.NativeTrainStep) against the Python-driven fused step
    (harness.TrainStep): the same entry points in the same order, so with the deterministic
    backward every parameter, Adam moment, exposure, densification statistic and loss value is
    bit-identical after several steps over cycled views."""
    from helpers import deterministic
    from gs_train.harness import make_problem
    from gs_train.native_step import NativeTrainStep
    names = ("_xyz", "_features", "_opacity", "_scaling", "_rotation", "_exposure")
    out = {}
    with deterministic():
        for native in (False, True):
            torch.manual_seed(0)
            ts = make_problem(20_000, 256, 192, n_views=3, seed=1, step_cls=NativeTrainStep if native else None,
                              depth=depth, alpha=alpha, skybox_points=skybox, scaffold_points=scaffold)
            if scaffold:
                with torch.no_grad():
                    ts.g._scaling[scaffold - 50:scaffold + 50] += 3.0
            torch.manual_seed(3)  # the random backgrounds
            losses = [ts.step().clone() for _ in range(4)]
            params = [getattr(ts.g, n).detach().clone() for n in names]
            moments = [torch.cat([ts.optimizer.state[getattr(ts.g, n)][k].reshape(-1)
                                  for n in names[:-1]]) for k in ("exp_avg", "exp_avg_sq")]
            moments += [ts.exposure_optimizer.state[ts.g._exposure][k].clone() for k in ("exp_avg", "exp_avg_sq")]
            steps = [float(ts.optimizer.state[getattr(ts.g, n)]["step"]) for n in names[:-1]]
            stats = [ts.g.max_radii2D.clone(), ts.g.xyz_gradient_accum.clone(), ts.g.denom.clone()]
            out[native] = (torch.stack(losses), params, moments, steps, stats)
    (la, pa, ma, sa, ta), (lb, pb, mb, sb, tb) = out[False], out[True]
    assert torch.equal(la, lb), (la, lb)
    for n, x, y in zip(names, pa, pb):
        assert torch.equal(x, y), n
    for x, y in zip(ma, mb):
        assert torch.equal(x, y)
    assert sa == sb == [4.0] * 5
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)


@pytest.mark.parametrize("dense_rows", ["0", "1"])
def test_native_step_sparse_rows_and_dense_fallback(dense_rows, monkeypatch):
    """The native step's sparse gradient rows (gradient rows of Gaussians no pixel's backward
    reached are not written: GSR_STEP_DENSE_ROWS unset) and its dense rows give the Python-driven
    step's bits, including the sparse Adam's dense fallback: after two ordinary steps every opacity
    is pushed to ~0, no pixel blends, no row is relevant and OurAdam updates every row with zero
    gradients (train_single.py:226-231, OurAdam.py:214) -- the skybox rows' six gradients zeroed
    by the lock (:217-223), the never-written rows read as zero."""
    from helpers import deterministic
    from gs_train.harness import make_problem
    from gs_train.native_step import NativeTrainStep
    monkeypatch.setenv("GSR_STEP_DENSE_ROWS", dense_rows)
    names = ("_xyz", "_features", "_opacity", "_scaling", "_rotation")
    out = {}
    with deterministic():
        for native in (False, True):
            torch.manual_seed(0)
            ts = make_problem(20_000, 256, 192, n_views=2, seed=4, step_cls=NativeTrainStep if native else None,
                              depth=True, skybox_points=300)
            torch.manual_seed(3)
            ts.step()
            ts.step()
            with torch.no_grad():
                ts.g._opacity.fill_(-30.0)
            before = [getattr(ts.g, n).detach().clone() for n in names]
            ts.step()
            params = [getattr(ts.g, n).detach().clone() for n in names]
            moments = [ts.optimizer.state[getattr(ts.g, n)][k].clone() for n in names for k in ("exp_avg", "exp_avg_sq")]
            out[native] = (before, params, moments)
    (b0, pa, ma), (b1, pb, mb) = out[False], out[True]
    for n, x, y in zip(names, b0, b1):
        assert torch.equal(x, y), n
    for n, x, y, x0 in zip(names, pa, pb, b0):
        assert torch.equal(x, y), n
        if n != "_opacity":
            assert not torch.equal(x[300:], x0[300:]), n  # the fallback moved the rows (momentum)
    for x, y in zip(ma, mb):
        assert torch.equal(x, y)


def test_native_step_follows_densification():
    """The executor re-reads the parameter tensors when densification replaces them."""
    from gs_train.harness import make_problem
    from gs_train.native_step import NativeTrainStep
    from gs_train.densify import densify_and_prune
    torch.manual_seed(0)
    ts = make_problem(20_000, 256, 192, n_views=2, seed=2, perturb=0.05, step_cls=NativeTrainStep)
    for _ in range(3):
        ts.step()
    # the executor's gradients stand in for the .grad fields densification statistics came from
    P0 = ts.g.P
    densify_and_prune(ts.g, ts.optimizer, 1e-6, 0.005, 10.0, 0.01)
    assert ts.g.P != P0
    first = ts.step().item()
    for _ in range(10):
        ts.step()
    assert np.isfinite(first) and ts.last_K > 0 and ts._args.P == ts.g.P


def test_depth_l1_node_matches_torch_expression():
    """gs_train.loss.depth_l1_loss vs train_single.py:138-140 through torch autograd: value to fp32
    rounding (fp64 accumulation here), dL/dinvdepth bit-identical (including sgn(0) = 0 where the
    mask or the difference is zero)."""
    from gs_train.loss import depth_l1_loss
    g = torch.Generator(device=DEV).manual_seed(5)
    for H, W in ((1080, 1920), (37, 53)):
        invd = torch.rand(1, H, W, generator=g, device=DEV)
        mono = invd * (1 + 0.1 * torch.randn(1, H, W, generator=g, device=DEV))
        mono[:, :3] = invd[:, :3]  # exact zeros of the difference
        mask = (torch.rand(1, H, W, generator=g, device=DEV) < 0.8).float()
        w = 0.73
        a = invd.clone().requires_grad_(True)
        la = depth_l1_loss(a, mono, mask, w)
        la.backward()
        b = invd.clone().requires_grad_(True)
        lb = w * torch.abs((b - mono) * mask).mean()
        lb.backward()
        assert abs(la.item() - lb.item()) <= 2e-6 * abs(lb.item())
        assert torch.equal(a.grad, b.grad)
        c = invd.clone().requires_grad_(True)
        depth_l1_loss(c, mono, None, w).backward()
        d = invd.clone().requires_grad_(True)
        (w * torch.abs(d - mono).mean()).backward()
        assert torch.equal(c.grad, d.grad)


def test_train_step_reduces_loss():
    from gs_train.harness import make_problem
    torch.manual_seed(0)
    ts = make_problem(20_000, 256, 192, n_views=2, seed=2, perturb=0.05)
    first = [ts.step().item() for _ in range(2)]
    for _ in range(40):
        ts.step()
    last = [ts.step().item() for _ in range(2)]
    assert np.mean(last) < 0.9 * np.mean(first), (first, last)


def test_exposure_matches_torch_reference_formula():
    from gs_train import apply_exposure
    g = torch.Generator().manual_seed(9)
    color = (torch.rand(3, 97, 203, generator=g) * 1.4 - 0.2).to(DEV).requires_grad_(True)
    E = (torch.eye(3, 4) + 0.1 * torch.randn(3, 4, generator=g)).to(DEV).requires_grad_(True)
    up = torch.randn(3, 97, 203, generator=g).to(DEV)
    out = apply_exposure(color, E)
    (out * up).sum().backward()
    c64 = color.detach().double().requires_grad_(True)
    e64 = E.detach().double().requires_grad_(True)
    ref = (torch.matmul(c64.permute(1, 2, 0), e64[:3, :3]).permute(2, 0, 1) + e64[:3, 3, None, None]).clamp(0, 1)
    (ref * up.double()).sum().backward()
    assert (out.double() - ref).abs().max().item() <= 1e-6
    assert (color.grad.double() - c64.grad).abs().max().item() <= 1e-6
    assert (E.grad.double() - e64.grad).abs().max().item() <= 1e-4 * e64.grad.abs().max().item()


def test_activate_matches_torch_getters_and_autograd():
    """gsr_activate_forward/_backward against scene/gaussian_model.py's getters (exp, normalize,
    sigmoid) and torch autograd through them."""
    from gs_train import activate
    g = torch.Generator().manual_seed(11)
    P = 100_003
    s = (torch.randn(P, 3, generator=g) - 3).to(DEV).requires_grad_(True)
    q = torch.randn(P, 4, generator=g)
    q[:5] = 0.0  # zero quaternions: normalize's eps clamp
    q = q.to(DEV).requires_grad_(True)
    o = torch.randn(P, 1, generator=g).to(DEV).requires_grad_(True)
    ups = [torch.randn(P, k, generator=g).to(DEV) for k in (3, 4, 1)]
    outs = activate(s, q, o)
    sum((a * u).sum() for a, u in zip(outs, ups)).backward()
    s2, q2, o2 = (t.detach().clone().requires_grad_(True) for t in (s, q, o))
    refs = (torch.exp(s2), torch.nn.functional.normalize(q2), torch.sigmoid(o2))
    sum((a * u).sum() for a, u in zip(refs, ups)).backward()
    for a, b in zip(outs, refs):
        torch.testing.assert_close(a, b, rtol=2e-7, atol=1e-7)
    for a, b in ((s, s2), (o, o2)):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-7)
    # normalize's gradient g/d - x (g.x)/d^3 cancels: bound the error by the size of its terms
    d = q.detach().norm(dim=1, keepdim=True).clamp_min(1e-12)
    scale = ups[1].norm(dim=1, keepdim=True) / d
    assert ((q.grad - q2.grad).abs() <= 4e-7 * scale + 1e-7).all()


def test_shrink_scales_matches_reference_indexing():
    from gs_train import shrink_scales
    g = torch.Generator().manual_seed(12)
    s = (torch.randn(50_000, 3, generator=g) * 2 - 3).to(DEV)
    ref = s.clone()
    limit, first = 0.2, 100
    sc = torch.exp(ref)
    bad = sc.max(dim=1).values > limit
    bad[:first] = False  # scaffold points
    ref[bad] = torch.log(sc[bad] * 0.8)
    shrink_scales(s, limit, first_row=first)
    assert bad.sum() > 1000
    torch.testing.assert_close(s, ref, rtol=0, atol=0)


def test_adam_column_blocks_equal_separate_groups():
    """One (P,16,3) SH tensor with column_lrs == the reference's f_dc / f_rest groups, bitwise."""
    from gs_train import Adam
    g = torch.Generator().manual_seed(13)
    P = 30_000
    base = torch.randn(P, 16, 3, generator=g).to(DEV)
    grads = [torch.randn(P, 16, 3, generator=g).to(DEV) for _ in range(3)]
    rel = (torch.rand(P, generator=g) < 0.7).float().to(DEV)
    joined = torch.nn.Parameter(base.clone())
    dc = torch.nn.Parameter(base[:, :1].clone())
    rest = torch.nn.Parameter(base[:, 1:].clone())
    oj = Adam([{"params": [joined], "lr": 0.0025, "column_lrs": [(0, 3, 0.0025), (3, 48, 0.0025 / 20.0)]}], eps=1e-15)
    os_ = Adam([{"params": [dc], "lr": 0.0025}, {"params": [rest], "lr": 0.0025 / 20.0}], eps=1e-15)
    for gr in grads:
        joined.grad = gr.clone()
        dc.grad, rest.grad = gr[:, :1].contiguous(), gr[:, 1:].contiguous()
        oj.step(relevance=rel)
        os_.step(relevance=rel)
    assert torch.equal(joined.detach()[:, :1], dc.detach())
    assert torch.equal(joined.detach()[:, 1:], rest.detach())
    assert torch.equal(oj.state[joined]["exp_avg_sq"][:, 1:], os_.state[rest]["exp_avg_sq"])


@pytest.mark.parametrize("frac", [0.12, 0.9, 0.0, 1.0])
def test_sparse_adam_row_blocks_equal_elementwise(frac, monkeypatch):
    """The row-block Adam kernel (one wave per 64 rows) and the element-per-thread kernel apply
    the same per-element arithmetic: parameters and moments bit-identical, for sparse and dense
    relevance (frac 0: no relevant row, the dense fallback; frac 1: every wave fully relevant, the
    joined (P,16,3) column blocks then updated as whole float4 rows) and joined column blocks."""
    from gs_train import Adam
    P = 70_001
    g = torch.Generator().manual_seed(5)
    shapes = [(3,), (16, 3), (1,), (3,), (4,)]
    init = [torch.randn((P,) + s, generator=g) for s in shapes]
    grads = [[torch.randn((P,) + s, generator=g) for s in shapes] for _ in range(2)]
    for gr in grads:
        gr[2][torch.rand(P, generator=g) >= frac] = 0.0
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("GSR_ADAM_ELEMENTWISE", mode)
        params = [torch.nn.Parameter(h.to(DEV)) for h in init]
        groups = [{"params": [params[0]], "lr": 1.6e-4},
                  {"params": [params[1]], "lr": 2.5e-3, "column_lrs": [(0, 3, 2.5e-3), (3, 48, 1.25e-4)]},
                  {"params": [params[2]], "lr": 5e-2}, {"params": [params[3]], "lr": 5e-3},
                  {"params": [params[4]], "lr": 1e-3}]
        opt = Adam(groups, lr=0.0, eps=1e-15)
        for gr in grads:
            for p, x in zip(params, gr):
                p.grad = x.to(DEV)
            opt.step(relevance=params[2].grad)
        torch.cuda.synchronize()
        out[mode] = [t.detach().clone() for p in params
                     for t in (p, opt.state[p]["exp_avg"], opt.state[p]["exp_avg_sq"])]
    for a, b in zip(out["0"], out["1"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("P", [70_001, 1])
def test_dense_adam_flat_runs_equal_row_blocks(P, monkeypatch):
    """The dense step (no relevance: torch.optim.Adam over every element, train_post's optimizer)
    streams each group as one flat float4 run and merges a column-split pair into whole rows.
    Parameters and moments are bit-identical to the row-block and element-per-thread kernels, for
    float4 runs ((P,16,3) pair, (P,4)), scalar runs ((P,3), (P,1), a 4-B-offset (P,4) view) and a
    column split that does not cover the row (that group alone goes to the row-block kernel)."""
    from gs_train import Adam
    g = torch.Generator().manual_seed(9)
    shapes = [(3,), (16, 3), (1,), (4,), (8,), (6,)]
    init = [torch.randn((P,) + s, generator=g) for s in shapes]
    grads = [[torch.randn((P,) + s, generator=g) for s in shapes] for _ in range(3)]
    out = {}
    for mode in ("flat", "rows", "elementwise"):
        monkeypatch.setenv("GSR_ADAM_DENSE_ROWS", "1" if mode == "rows" else "0")
        monkeypatch.setenv("GSR_ADAM_ELEMENTWISE", "1" if mode == "elementwise" else "0")
        params = [torch.nn.Parameter(h.to(DEV)) for h in init]
        # an (P, 4) parameter whose storage starts 4 B past a 16-B boundary: the scalar run
        store = torch.zeros(P * 4 + 1, device=DEV)
        odd = torch.nn.Parameter(store[1:].view(P, 4))
        with torch.no_grad():
            odd.copy_(init[5][:, :4].to(DEV))
        groups = [{"params": [params[0]], "lr": 1.6e-4},
                  {"params": [params[1]], "lr": 2.5e-3, "column_lrs": [(0, 3, 2.5e-3), (3, 48, 1.25e-4)]},
                  {"params": [params[2]], "lr": 5e-2}, {"params": [params[3]], "lr": 1e-3},
                  {"params": [params[4]], "lr": 7e-3, "column_lrs": [(0, 2, 7e-3), (2, 6, 3e-3)]},
                  {"params": [odd], "lr": 4e-3}]
        opt = Adam(groups, lr=0.0, eps=1e-15)
        for gr in grads:
            for p, x in zip(params[:5], gr[:5]):
                p.grad = x.to(DEV)
            odd.grad = gr[5][:, :4].contiguous().to(DEV)
            opt.step()
        torch.cuda.synchronize()
        out[mode] = [t.detach().clone() for p in params[:5] + [odd]
                     for t in (p, opt.state[p]["exp_avg"], opt.state[p]["exp_avg_sq"])]
    for name in ("rows", "elementwise"):
        for a, b in zip(out["flat"], out[name]):
            assert torch.equal(a, b), name
    # and it moved every element of every run
    assert not torch.equal(out["flat"][3], init[1].to(DEV))


@pytest.mark.parametrize("lam,scale", [(0.2, 1.0), (0.35, 2.5)])
def test_photo_loss_fused_equals_composed(lam, scale):
    """gsr_photo_loss_* (one autograd node) against l1_ssim composed with torch's scalar ops as
    train_single.py:121-123 writes it: loss, L1, SSIM and the image gradient bit for bit, also
    for an upstream dL/dloss != 1."""
    from gs_train import l1_ssim, photo_loss
    g = torch.Generator().manual_seed(17)
    img = torch.rand(3, 211, 333, generator=g).to(DEV)
    gt = torch.rand(3, 211, 333, generator=g).to(DEV)
    x1 = img.clone().requires_grad_(True)
    loss, l1, s = photo_loss(x1, gt, lam)
    (scale * loss).backward()
    x2 = img.clone().requires_grad_(True)
    v = l1_ssim(x2, gt)
    loss2 = (1.0 - lam) * v[0] + lam * (1.0 - v[1])
    (scale * loss2).backward()
    assert torch.equal(loss, loss2) and torch.equal(l1, v[0].detach()) and torch.equal(s, v[1].detach())
    assert torch.equal(x1.grad, x2.grad)
    assert not l1.requires_grad and not s.requires_grad


def test_grad_bucket_captures_rasterizer_gradients():
    """Data-parallel flat bucket (gsr_dist.GradBucket) on the real kernels: inside a capture the
    rasterizer's dL/dmeans3D, dL/dshs and the activations' raw gradients are written straight into
    the bucket (the parameters' .grad are views of it) and equal the gradients of an uncaptured
    backward bit for bit; the world-size-1 all-reduce keeps them in place."""
    import gsr_dist
    from gs_train.harness import make_problem
    ts = make_problem(20_000, 256, 192, n_views=1, seed=3)
    g = ts.g
    params = {"xyz": g._xyz, "features": g._features, "opacity": g._opacity, "scaling": g._scaling,
              "rotation": g._rotation}
    bg = torch.zeros(3, device=DEV)

    def backward():
        for p in params.values():
            p.grad = None
        image, invd, _, _ = ts.render(0, bg)
        loss = ts._photo_loss(image, ts.gts[0]) + ts._depth_loss(invd, ts.mono[0], ts.dmask[0], 0.5)
        loss.backward()

    from helpers import deterministic
    with deterministic():  # two backward passes compared bit for bit
        backward()
        ref = {k: p.grad.clone() for k, p in params.items()}
        bucket = gsr_dist.GradBucket(params)
        for p in params.values():
            p.grad = None
        with bucket.capture():
            backward()
    for k, p in params.items():
        assert bucket.owns(p), k
        assert torch.equal(p.grad, ref[k]), k
    bucket.allreduce()
    for k, p in params.items():
        assert bucket.owns(p) and torch.equal(p.grad, ref[k]), k
