"""GPU tests of the Street-sparse per-chunk loop (gs_train.chunk.TrainChunk: train_single.py:65-247)
and of its depth-only iterations (train_single.py:69-72,145-161,203-214).

* the depth-only loss node vs torch's autograd through the reference's expression: gradient bit
  for bit, value to fp32 rounding;
* the native step (gsr_train_step) vs the Python-driven step over a view cycle mixing photometric
  and depth-only views: bit-identical with the deterministic backward;
* the whole chunk loop -- densify / prune events, opacity resets, SH-degree increments, lr and depth
  weight schedules -- native vs Python-driven: bit-identical, P identical after every event; and
  vs the reference's torch formulation (oracle/train_torch_ref.ReferenceTrainStep, its own
  densify_and_prune / reset_opacity) on the same generator stream: P identical after every event,
  parameters within an fp32 tolerance;
* checkpoint / resume (capture + restore, which swaps every parameter and moment tensor) is
  bit-identical to the uninterrupted run;
* the native step's dense-rows fallback zeroes the locked skybox rows' six gradients.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
NAMES = ("_xyz", "_features", "_opacity", "_scaling", "_rotation", "_exposure")


def _snapshot(ts):
    g = ts.g
    return ([getattr(g, n).detach().clone() for n in NAMES],
            [ts.optimizer.state[getattr(g, n)][k].clone() for n in NAMES[:-1] for k in ("exp_avg", "exp_avg_sq")],
            [float(ts.optimizer.state[getattr(g, n)]["step"]) for n in NAMES[:-1]],
            [g.max_radii2D.clone(), g.xyz_gradient_accum.clone(), g.denom.clone()], g.active_sh_degree)


def _assert_equal_snapshots(a, b):
    (pa, ma, sa, ta, da), (pb, mb, sb, tb, db) = a, b
    for n, x, y in zip(NAMES, pa, pb):
        assert x.shape == y.shape and torch.equal(x, y), n
    for x, y in zip(ma, mb):
        assert torch.equal(x, y)
    assert sa == sb and da == db
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)


def test_depth_only_loss_matches_torch_expression():
    """gs_train.loss.depth_only_loss vs train_single.py:152-156 through torch autograd: dL/dinvdepth
    bit-identical (the clamp passes the gradient at mono == invD, sgn(0) = 0), the value to fp32
    rounding; with a mask and without."""
    from gs_train.loss import depth_only_loss
    g = torch.Generator(device=DEV).manual_seed(9)
    for H, W in ((1536, 1536), (37, 53)):
        invd = torch.rand(1, H, W, generator=g, device=DEV)
        mono = invd * (1 + 0.1 * torch.randn(1, H, W, generator=g, device=DEV))
        mono *= (torch.rand(1, H, W, generator=g, device=DEV) < 0.4).float()  # sparse LiDAR-like map
        mono[:, :3] = invd[:, :3]  # exact ties of the clamp and of sgn
        mask = (torch.rand(1, H, W, generator=g, device=DEV) < 0.9).float()
        for m in (mask, None):
            w, a = 0.61, 0.9
            x = invd.clone().requires_grad_(True)
            lx, pure, dens = depth_only_loss(x, mono, m, w, a)
            lx.backward()
            y = invd.clone().requires_grad_(True)
            mm = m if m is not None else torch.ones_like(invd)
            p_ref = torch.abs((y - mono) * mm).mean()
            d_ref = (mono - y).clamp(min=0).mean()
            ly = (w * (a * d_ref + (1 - a) * p_ref)).clone()
            ly.backward()
            assert torch.equal(x.grad, y.grad)
            assert abs(lx.item() - ly.item()) <= 2e-6 * abs(ly.item())
            assert abs(pure.item() - p_ref.item()) <= 2e-6 * abs(p_ref.item())
            assert abs(dens.item() - d_ref.item()) <= 2e-6 * abs(d_ref.item())


@pytest.mark.parametrize("skybox,alpha", [(0, False), (300, True)])
def test_native_step_with_depth_only_views_equals_python_step(skybox, alpha):
    """A view cycle of three photometric and two depth-only views: the native step (depth-only
    branch: no SSIM / exposure pass, zero colour gradient, exposure gradient zeroed, no exposure
    step) is bit-identical to the Python-driven step, which zeroes the SH gradients explicitly."""
    from helpers import deterministic
    from gs_train.harness import make_problem
    from gs_train.native_step import NativeTrainStep
    out = {}
    with deterministic():
        for native in (False, True):
            torch.manual_seed(0)
            ts = make_problem(20_000, 256, 192, n_views=5, seed=1, step_cls=NativeTrainStep if native else None,
                              depth=True, alpha=alpha, skybox_points=skybox, depth_only=2)
            torch.manual_seed(3)
            losses = torch.stack([ts.step().clone() for _ in range(7)])
            out[native] = (losses, _snapshot(ts),
                           [ts.exposure_optimizer.state[ts.g._exposure][k].clone() for k in ("exp_avg", "exp_avg_sq")],
                           float(ts.exposure_optimizer.state[ts.g._exposure]["step"]))
    (la, sa, ea, esa), (lb, sb, eb, esb) = out[False], out[True]
    assert torch.equal(la, lb), (la, lb)
    _assert_equal_snapshots(sa, sb)
    for x, y in zip(ea, eb):
        assert torch.equal(x, y)
    # 7 steps over [p, p, p, d, d, p, p]: the exposure optimizer stepped on the 5 photometric ones
    assert esa == esb == 5.0
    assert sa[2] == [7.0] * 5


def test_depth_only_step_matches_reference_structured_step():
    """The depth-only iteration against the reference's torch formulation (ReferenceTrainStep: the
    torch expression of :152-156, SH and exposure gradients zeroed, no exposure step).  Every element
    within Adam's travel bound (helpers.assert_adam_trajectories_close), the bulk within 1e-5, and
    the locked skybox rows unmoved on both sides."""
    from gs_train.harness import LR, make_problem
    from helpers import assert_adam_trajectories_close, record_margins
    from train_torch_ref import ReferenceTrainStep
    names = ("_xyz", "_features_dc", "_opacity", "_scaling", "_rotation")
    steps, sky = 4, 300
    res = {}
    for fused in (True, False):
        torch.manual_seed(0)
        ts = make_problem(20_000, 256, 192, n_views=2, seed=2, depth=True, depth_only=2, skybox_points=sky,
                          step_cls=None if fused else ReferenceTrainStep)
        init = [getattr(ts.g, n).detach().clone() for n in names]
        xyz_lr = max(ts.xyz_lr(it) for it in range(0, steps + 2))
        losses = [ts.step().item() for _ in range(steps)]
        res[fused] = (losses, [getattr(ts.g, n).detach().clone() for n in names], init,
                      ts.g._exposure.detach().clone())
    (la, pa, ia, ea), (lb, pb, _, eb) = res[True], res[False]
    np.testing.assert_allclose(la, lb, rtol=1e-5, atol=1e-7)
    lrs = dict(_xyz=xyz_lr, _features_dc=LR["feature_lr"], _opacity=LR["opacity_lr"], _scaling=LR["scaling_lr"],
               _rotation=LR["rotation_lr"])
    for n, x, y, x0 in zip(names, pa, pb, ia):
        # the skybox rows: all six gradients zeroed (train_single.py:217-223), so Adam never moves them
        assert torch.equal(x[:sky], x0[:sky]) and torch.equal(y[:sky], x0[:sky]), n
        if n == "_features_dc":  # a depth-only view zeroes the SH gradients: momentum only
            assert torch.isclose(x, y, rtol=0, atol=1e-5).float().mean().item() >= 0.999
            continue
        worst, close = assert_adam_trajectories_close(n, x, y, x0, lrs[n], steps, atol=1e-5)
        record_margins(f"depth_only_step{n}", travel_frac=worst, close=close)
    assert torch.equal(ea, eb) and torch.equal(ea, torch.eye(3, 4, device=DEV)[None].expand_as(ea))


def _small_schedule(iterations):
    from gs_train.chunk import ChunkSchedule
    # train_single.py's loop on a scaled schedule: densify every 60 iterations in (60, 300), an opacity
    # reset at 180 (with a densify, as every reset of the default schedule), SH increments every 100
    return ChunkSchedule(iterations=iterations, densification_interval=60, opacity_reset_interval=180,
                         densify_from_iter=60, densify_until_iter=300, sh_interval=100,
                         densify_grad_threshold=0.0008, percent_dense=0.01)


def _chunk_problem(step_cls, iterations, seed=3):
    from gs_train.harness import make_problem
    ts = make_problem(30_000, 192, 160, n_views=6, seed=seed, step_cls=step_cls, depth=True, alpha=True,
                      skybox_points=200, scaffold_points=1000, depth_only=2, perturb=0.05, iterations=iterations)
    with torch.no_grad():
        ts.g.active_sh_degree = 0  # create_from_pcd's GaussianModel starts at degree 0
    return ts


@pytest.fixture
def live_list_restored():
    from diff_gaussian_rasterization import _C
    prev = _C.set_live_list(False)
    yield
    _C.set_live_list(prev)


@pytest.mark.parametrize("spatial", [False, True], ids=["index_order", "spatial_order"])
def test_chunk_loop_native_equals_python(spatial, live_list_restored):
    """train_single.py's loop with 4 densify / prune events, an opacity reset, SH increments and
    depth-only views: native executor vs Python-driven step, bit for bit (deterministic backward),
    P after every event identical, the Adam step counts showing the skipped Gaussian updates.
    spatial: the rows kept in spatial order (TrainChunk(spatial=True): reorder_rows after every
    densification, the backward's live-row list walk) on both sides."""
    from helpers import deterministic
    from diff_gaussian_rasterization import _C
    from gs_train.chunk import TrainChunk
    from gs_train.native_step import NativeTrainStep
    iters = 320
    out = {}
    with deterministic():
        for native in (False, True):
            torch.manual_seed(0)
            ts = _chunk_problem(NativeTrainStep if native else None, iters)
            torch.manual_seed(5)
            tc = TrainChunk(ts, _small_schedule(iters), spatial=spatial)
            tc.run()
            # run() restores the process-wide live-list knob it sets for spatial rows
            assert _C.set_live_list(False) is False
            out[native] = ([(e["iteration"], e["P_before"], e["P_after"]) for e in tc.events], _snapshot(ts))
    (ea, sa), (eb, sb) = out[False], out[True]
    assert ea == eb
    assert [e[0] for e in ea] == [120, 180, 240]  # > densify_from_iter, < densify_until_iter
    assert any(e[2] != e[1] for e in ea)
    _assert_equal_snapshots(sa, sb)
    assert sa[4] == 3  # degree 0 -> 3 at iterations 100, 200, 300
    # Gaussian Adam steps: iterations 1..319 minus the 3 event iterations
    assert sa[2] == [316.0] * 5


def test_spatial_order_is_a_row_permutation(live_list_restored):
    """TrainChunk(spatial=True) without densification (an opacity reset, SH increments, depth-only
    views): the rows after the skybox / scaffold prefix permuted once by Morton code, and after 240
    iterations every parameter, moment and statistic is the index-order run's, permuted -- up to the
    rounding of exactly equal depths, whose blending order follows the row index (upstream's (depth
    bits, index) key): the first such frame here is iteration 41, and from there the two runs drift
    apart by fp32 noise, relative to each tensor's travel ~7e-5 (r05ao), bar 1e-3."""
    from helpers import deterministic, record_margins
    from gs_train.chunk import ChunkSchedule, TrainChunk, spatial_order
    from gs_train.native_step import NativeTrainStep
    iters = 240
    sched = ChunkSchedule(iterations=iters, densification_interval=60, opacity_reset_interval=120,
                          densify_from_iter=iters, densify_until_iter=iters, sh_interval=60)
    out = {}
    with deterministic():
        for spatial in (False, True):
            torch.manual_seed(0)
            ts = _chunk_problem(NativeTrainStep, iters)
            first = max(ts.skybox, ts.scaffold)
            xyz0 = ts.g._xyz.detach().clone()
            init = [getattr(ts.g, n).detach().clone() for n in NAMES]
            torch.manual_seed(5)
            tc = TrainChunk(ts, sched, spatial=spatial)
            tc.run()
            assert [e["iteration"] for e in tc.events] == [120]
            out[spatial] = _snapshot(ts)
    perm = torch.cat((torch.arange(first, device=DEV), spatial_order(xyz0[first:]) + first))
    assert not torch.equal(perm, torch.arange(perm.numel(), device=DEV))
    (pa, ma, sa, ta, da), (pb, mb, sb, tb, db) = out[False], out[True]
    assert sa == sb and da == db
    for n, x, y, x0 in zip(NAMES, pa, pb, init):
        if n == "_exposure":
            torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-6)
            continue
        d = ((x[perm] - y).norm() / (x - x0).norm().clamp_min(1e-30)).item()
        record_margins(f"spatial_order_drift{n}", drift=d)
        print(f"spatial-order drift {n}: {d:.3g}")
        assert d <= 1e-3, (n, d)
    # the densification statistics: the same rows saw the same views
    assert torch.equal(ta[2][perm], tb[2])


def _split_params(ts):
    g = ts.g
    f = g._features.detach()
    return [g._xyz.detach(), f[:, :1], f[:, 1:], g._opacity.detach(), g._scaling.detach(), g._rotation.detach()]


def _split_state(ts):
    """(params, moments, stats) of a step in the reference's split layout (f_dc | f_rest)."""
    g = ts.g
    if g.joined:
        f = g._features.detach()
        params = [g._xyz.detach(), f[:, :1], f[:, 1:], g._opacity.detach(), g._scaling.detach(), g._rotation.detach()]
        st = [ts.optimizer.state[p] for p in (g._xyz, g._features, g._opacity, g._scaling, g._rotation)]
        mom = [(st[0]["exp_avg"], st[0]["exp_avg_sq"]), (st[1]["exp_avg"][:, :1], st[1]["exp_avg_sq"][:, :1]),
               (st[1]["exp_avg"][:, 1:], st[1]["exp_avg_sq"][:, 1:])] + [(x["exp_avg"], x["exp_avg_sq"]) for x in st[2:]]
    else:
        ps = (g._xyz, g._features_dc, g._features_rest, g._opacity, g._scaling, g._rotation)
        params = [p.detach() for p in ps]
        mom = [(ts.optimizer.state[p]["exp_avg"], ts.optimizer.state[p]["exp_avg_sq"]) for p in ps]
    return params, mom, [g.max_radii2D, g.xyz_gradient_accum, g.denom]


def test_chunk_loop_matches_reference_structured_loop():
    """~700 iterations of the loop, fused step vs the reference's torch formulation
    (ReferenceTrainStep: OurAdam-style gather / scatter, conv2d SSIM, the torch depth expressions,
    the reference's own densify_and_prune and reset_opacity), run in lockstep on one generator
    stream (the random backgrounds, the split draws).  Between events the two trajectories drift by
    fp32 noise (different SSIM / Adam rounding), which can move a Gaussian across the densification
    threshold; so at every event the reference side is re-seeded with the fused side's
    pre-event state (parameters, moments, statistics) -- after checking that state agrees within
    tolerance -- and both then run their own densify / prune / reset: P identical after every
    event, every parameter and moment identical after it (the split children's xyz, formed with
    torch.bmm by the reference, within 1e-6), and the densify / reset iterations skip the Gaussian
    Adam step on both sides (equal step counts at the end)."""
    from gs_train.chunk import ChunkSchedule, TrainChunk
    from train_torch_ref import ReferenceTrainStep
    iters = 700
    sched = ChunkSchedule(iterations=iters, densification_interval=100, opacity_reset_interval=300,
                          densify_from_iter=100, densify_until_iter=600, sh_interval=200,
                          densify_grad_threshold=0.0008, percent_dense=0.01)
    torch.manual_seed(0)
    ta = _chunk_problem(None, iters)
    torch.manual_seed(0)
    tb = _chunk_problem(ReferenceTrainStep, iters)
    ca, cb = TrainChunk(ta, sched), TrainChunk(tb, sched)
    pre = {}
    checks = []
    # drift is measured against how far the parameters moved since the last re-seed (or the start)
    since = [[x.clone() for x in _split_params(ta)]]

    def drift(x, y, x0):
        return ((x - y).norm() / (x - x0).norm().clamp_min(1e-30)).item()

    orig_a, orig_b = ca._between, cb._between

    def between_a(it, dens, reset):
        run = orig_a(it, dens, reset)

        def wrapped():
            p, m, st = _split_state(ta)
            pre[it] = ([x.clone() for x in p], [(u.clone(), v.clone()) for u, v in m], [x.clone() for x in st])
            run()
        return wrapped

    def between_b(it, dens, reset):
        run = orig_b(it, dens, reset)

        def wrapped():
            pa, ma, sa = pre[it]
            pb, mb, sb = _split_state(tb)
            # the trajectories agree within fp32 drift before the re-seed ...
            for k, (x, y, x0) in enumerate(zip(pa, pb, since[-1])):
                checks.append((it, k, drift(x, y, x0)))
            # ... then the reference side takes the fused side's exact state
            for x, y in zip(pa, pb):
                y.copy_(x)
            for (u, v), (uu, vv) in zip(ma, mb):
                uu.copy_(u)
                vv.copy_(v)
            for x, y in zip(sa, sb):
                y.copy_(x)
            run()
        return wrapped
    ca._between, cb._between = between_a, between_b
    torch.manual_seed(5)
    while ta.iteration <= iters - 1:
        it = ta.iteration
        state = torch.cuda.get_rng_state()
        ca.iteration()
        after_a = torch.cuda.get_rng_state()
        torch.cuda.set_rng_state(state)
        cb.iteration()
        assert torch.equal(torch.cuda.get_rng_state(), after_a), it  # same draws on both sides
        if it in pre:
            pa, ma, sa = _split_state(ta)
            pb, mb, sb = _split_state(tb)
            assert ta.g.P == tb.g.P, (it, ta.g.P, tb.g.P)
            n_old = pre[it][0][0].shape[0]
            for k, (x, y) in enumerate(zip(pa, pb)):
                if k == 0:  # xyz: the split children's positions come from torch.bmm on the reference side
                    torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-6)
                elif k == 4:  # scaling: log(exp(s) / 1.6) of the split children, a few ulps
                    torch.testing.assert_close(x, y, rtol=4e-7, atol=0)
                else:
                    assert torch.equal(x, y), (it, k)
            for (u, v), (uu, vv) in zip(ma, mb):
                assert torch.equal(u, uu) and torch.equal(v, vv), it
            since.append([x.clone() for x in pa])
    ev_a = [(e["iteration"], e["P_before"], e["P_after"]) for e in ca.events]
    ev_b = [(e["iteration"], e["P_before"], e["P_after"]) for e in cb.events]
    assert [e[0] for e in ev_a] == [200, 300, 400, 500]
    assert ev_a == ev_b, (ev_a, ev_b)
    assert any(e[2] > e[1] for e in ev_a) and n_old > 0
    # fp32 drift over an interval of ~100 iterations: a few percent of the interval's own update
    # (Adam's normalised steps let rounding flip the sign of near-zero-gradient updates)
    pa, _, _ = _split_state(ta)
    pb, _, _ = _split_state(tb)
    for k, (x, y, x0) in enumerate(zip(pa, pb, since[-1])):
        checks.append(("end", k, drift(x, y, x0)))
    print("drift / update per interval and parameter:", [(it, k, round(d, 4)) for it, k, d in checks])
    from helpers import record_margins
    for it, k, d in checks:
        record_margins(f"chunk_lockstep_drift_{it}_{k}", drift=d)
    # bars ~5x the recorded drift (profiles/r05_parity_margins.jsonl: <= 0.0117 over the 100-iteration
    # intervals between events, <= 0.043 over the last ~200 iterations, which the bar of 0.1 keeps)
    for it, k, d in checks:
        assert d <= (0.06 if it != "end" else 0.1), (it, k, d)
    # the same number of Gaussian Adam steps on both sides
    steps_a = [float(ta.optimizer.state[p]["step"]) for p in (ta.g._xyz, ta.g._opacity)]
    steps_b = [float(tb.optimizer.state[p]["step"]) for p in (tb.g._xyz, tb.g._opacity)]
    assert steps_a == steps_b == [iters - 1 - 4] * 2


def test_checkpoint_resume_is_bit_identical():
    """capture() at an iteration and restore() into a fresh native step (new parameter and moment
    tensors: the executor must re-read them) continues exactly as the uninterrupted run."""
    from helpers import deterministic
    from gs_train.chunk import TrainChunk, capture, restore
    from gs_train.native_step import NativeTrainStep
    iters = 260
    with deterministic():
        torch.manual_seed(0)
        ts = _chunk_problem(NativeTrainStep, iters)
        torch.manual_seed(5)
        saved = {}
        sched = _small_schedule(iters)
        sched.checkpoint_iterations = (150,)
        tc = TrainChunk(ts, sched, on_checkpoint=lambda it, st: saved.setdefault(it, st))
        tc.run()
        full = _snapshot(ts)
        assert 150 in saved
        torch.manual_seed(0)
        ts2 = _chunk_problem(NativeTrainStep, iters)
        ts2.step()  # the executor caches its argument block for the old tensors
        restore(ts2, saved[150])
        assert ts2.iteration == 151
        TrainChunk(ts2, _small_schedule(iters)).run()
        _assert_equal_snapshots(full, _snapshot(ts2))


def test_native_step_after_optimizer_load_state_dict():
    """optimizer.load_state_dict between native steps swaps in new moment tensors with the same
    parameters (a checkpoint resume): the executor follows them, bit-identical to the Python step."""
    from helpers import deterministic
    from gs_train.harness import make_problem
    from gs_train.native_step import NativeTrainStep
    out = {}
    with deterministic():
        for native in (False, True):
            torch.manual_seed(0)
            ts = make_problem(20_000, 256, 192, n_views=3, seed=1, step_cls=NativeTrainStep if native else None)
            torch.manual_seed(3)
            ts.step()
            ts.step()
            sd = ts.optimizer.state_dict()
            sd = {"state": {k: {kk: (vv.clone() if torch.is_tensor(vv) else vv) for kk, vv in v.items()}
                            for k, v in sd["state"].items()}, "param_groups": sd["param_groups"]}
            ts.step()
            ts.optimizer.load_state_dict(sd)  # back to the moments after two steps, new tensors
            ts.step()
            out[native] = _snapshot(ts)
    _assert_equal_snapshots(out[False], out[True])


def test_native_dense_fallback_zeroes_skybox_rows(monkeypatch):
    """GSR_STEP_DENSE_ROWS=1 and only the locked skybox rows blending: their opacity gradient is
    locked at zero, no row is relevant and OurAdam's dense fallback updates every row -- with all six
    of the skybox rows' gradients zero (train_single.py:217-223), as the Python step has them."""
    from helpers import deterministic
    from gs_train.harness import make_problem
    from gs_train.native_step import NativeTrainStep
    monkeypatch.setenv("GSR_STEP_DENSE_ROWS", "1")
    S = 2000
    out = {}
    with deterministic():
        for native in (False, True):
            torch.manual_seed(0)
            ts = make_problem(20_000, 256, 192, n_views=2, seed=4, step_cls=NativeTrainStep if native else None,
                              depth=True, skybox_points=S)
            torch.manual_seed(3)
            ts.step()
            with torch.no_grad():
                ts.g._opacity[S:] = -30.0
            ts.step()
            out[native] = _snapshot(ts)
    _assert_equal_snapshots(out[False], out[True])


@pytest.mark.timeout(240)
def test_street_chunk_full_size_through_densify_and_reset():
    """The config-3 stand-in at full size in the suite (not only in bench): street_chunk's 1536^2 cube
    faces (48 stations, 1M-Gaussian truth street, 330k initial rows) through train_single.py's loop on a
    compressed schedule -- two densify events, an opacity reset (after which nothing saturates and the
    vanishing-point tiles hold 100k+ instances) and SH increments.  Properties: every loss finite, P
    grows, no NaN pixel in the views afterwards, capacity re-runs bounded, and the long-list paths
    (the forward split and the tile binning's superblock split) armed after the reset."""
    from diff_gaussian_rasterization import _C
    from gs_train.chunk import ChunkSchedule, TrainChunk, street_chunk
    from gs_train.native_step import NativeTrainStep
    n_it = 400
    torch.manual_seed(0)
    ts, info = street_chunk(NativeTrainStep, iterations=n_it, device=DEV)
    assert (info["W"], info["H"]) == (1536, 1536)
    sched = ChunkSchedule(iterations=n_it, densification_interval=100, opacity_reset_interval=200,
                          densify_from_iter=100, densify_until_iter=n_it, sh_interval=100)
    P0 = ts.g.P
    r0 = _C.forward_stats()
    losses = []
    tc = TrainChunk(ts, sched)
    tc.run(callback=lambda it, loss: losses.append(loss.detach().reshape(-1)[:1]))
    torch.cuda.synchronize()
    r1 = _C.forward_stats()
    assert torch.isfinite(torch.cat(losses)).all()
    ev = tc.events
    assert sum(1 for e in ev if "total" in e) >= 2 and any(e.get("reset") for e in ev), ev
    assert max(e["P_after"] for e in ev) > P0
    for k in range(0, len(ts.cams), 9):
        img, invd, _, _ = ts.render(k, torch.zeros(3, device=DEV))
        assert torch.isfinite(img).all() and torch.isfinite(invd).all(), k
    d = {k: r1[k] - r0[k] for k in r1}
    print("street chunk, full size:", {k: d[k] for k in ("frames", "reruns", "fwd_split_frames", "tb_split_frames",
                                                          "fwd_worker_giveups")}, "P", P0, "->", ts.g.P)
    assert d["reruns"] <= 0.1 * d["frames"], d
    assert d["fwd_split_frames"] > 0 and d["tb_split_frames"] > 0, d
    assert d["fwd_worker_giveups"] == 0, d
