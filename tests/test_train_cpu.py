"""CPU tests of the train-step row: the oracle
(oracle/train_ref.py) and the reference-structured baseline (oracle/train_torch_ref.py) are pinned to
the fixtures the reference's own loss_utils / OurAdam / get_expon_lr_func produced
(tests/golden/make_train_golden.py); host logic of gs_train is checked without a GPU."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

import train_ref as TR

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]


def _gold(name):
    return np.load(os.path.join(GOLD, name))


@pytest.mark.parametrize("mod", ["oracle", "baseline"])
def test_loss_matches_reference_fixtures(mod):
    import train_torch_ref as baseline
    d = _gold("loss.npz")
    for k in range(int(d["n"])):
        img = torch.tensor(d[f"img_{k}"], requires_grad=True)
        gt = torch.tensor(d[f"gt_{k}"])
        if mod == "oracle":
            l1, s = TR.l1(img, gt), TR.ssim(img, gt)
            loss = 0.8 * l1 + 0.2 * (1 - s)
            assert abs(l1.item() - float(d[f"l1_{k}"])) <= 1e-6
            assert abs(s.item() - float(d[f"ssim_{k}"])) <= 1e-6
        else:
            loss = baseline.photo_loss(img, gt)
        assert abs(loss.item() - float(d[f"loss_{k}"])) <= 1e-6
        loss.backward()
        g = img.grad.numpy()
        ref = d[f"grad_{k}"]
        assert np.abs(g - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max()) + 1e-9


def _run_adam(step_fn):
    d = _gold("adam.npz")
    params = [torch.tensor(d[f"init_{n}"]) for n in NAMES]
    m = [torch.zeros_like(p) for p in params]
    v = [torch.zeros_like(p) for p in params]
    steps = [0] * len(NAMES)
    for it in range(3):
        grads = [torch.tensor(d[f"grad{it}_{n}"]) for n in NAMES]
        steps = step_fn(params, grads, m, v, steps, list(d["lrs"]), grads[3])
        for j, n in enumerate(NAMES):
            np.testing.assert_allclose(params[j].numpy(), d[f"after{it}_{n}"], rtol=0, atol=2e-7)
            np.testing.assert_allclose(m[j].numpy(), d[f"m{it}_{n}"], rtol=0, atol=1e-7)
            np.testing.assert_allclose(v[j].numpy(), d[f"v{it}_{n}"], rtol=1e-6, atol=1e-9)


def test_oracle_sparse_adam_matches_reference_ouradam():
    _run_adam(TR.sparse_adam)


def test_baseline_ouradam_matches_reference_ouradam():
    import train_torch_ref as baseline
    d = _gold("adam.npz")
    params = [torch.nn.Parameter(torch.tensor(d[f"init_{n}"])) for n in NAMES]
    opt = baseline.OurAdamTorch([{"params": [p], "lr": float(lr), "name": n}
                                 for p, lr, n in zip(params, d["lrs"], NAMES)], lr=0.0, eps=1e-15)
    for it in range(3):
        for j, n in enumerate(NAMES):
            params[j].grad = torch.tensor(d[f"grad{it}_{n}"])
        opt.step((params[3].grad.flatten() != 0).nonzero().flatten().long())
        for j, n in enumerate(NAMES):
            np.testing.assert_allclose(params[j].detach().numpy(), d[f"after{it}_{n}"], rtol=0, atol=2e-7)


def test_oracle_densify_matches_reference():
    d = _gold("densify.npz")
    radii = torch.tensor(d["radii"])
    mr, acc, den = (torch.tensor(d[k]).clone() for k in ("max_r", "accum", "denom"))
    TR.densify_stats(radii, torch.tensor(d["grad2d"]), mr, acc, den)
    np.testing.assert_array_equal(mr.numpy(), d["max_r_after"])
    np.testing.assert_array_equal(acc.numpy(), d["accum_after"])
    np.testing.assert_array_equal(den.numpy(), d["denom_after"])


def test_lr_schedule_matches_reference():
    from gs_train.harness import expon_lr
    d = _gold("lr.npz")
    for s, xyz, ex in zip(d["steps"], d["xyz"], d["exposure"]):
        assert expon_lr(int(s), 0.00002 * 3.5, 0.0000002 * 3.5, lr_delay_mult=0.01, max_steps=30_000) == \
            pytest.approx(float(xyz), rel=1e-12, abs=0)
        assert expon_lr(int(s), 0.001, 0.0001, lr_delay_steps=5000, lr_delay_mult=0.001, max_steps=30_000) == \
            pytest.approx(float(ex), rel=1e-12, abs=0)


def test_synthetic_scene_matches_oracle_generator():
    import gs_oracle as O
    from gs_train import synthetic
    a = synthetic.synthetic_scene(500, 320, 240, seed=3)
    b = O.synthetic_scene(500, 320, 240, seed=3)
    for k in ("means3D", "scales", "rotations", "opacities", "shs", "view", "proj", "campos", "bg"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert a["tanfovx"] == b["tanfovx"] and a["tanfovy"] == b["tanfovy"]


def test_train_kernels_refuse_cpu_tensors():
    from gs_train import add_densification_stats, l1_ssim
    x = torch.rand(3, 8, 8)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        l1_ssim(x, x)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        add_densification_stats(torch.zeros(4, dtype=torch.int32), torch.zeros(4, 3), torch.zeros(4),
                                torch.zeros(4, 1), torch.zeros(4, 1))


def test_fused_adam_validation_on_host():
    from gs_train import Adam
    p = torch.nn.Parameter(torch.zeros(4, 3))
    with pytest.raises(ValueError):
        Adam([p], lr=-1.0)
    with pytest.raises(NotImplementedError):
        Adam([p], amsgrad=True)
    opt = Adam([{"params": [p], "lr": 0.1, "name": "xyz"}], lr=0.0, eps=1e-15)
    assert opt.param_groups[0]["name"] == "xyz" and opt.param_groups[0]["eps"] == 1e-15
    opt.step(torch.zeros(0, dtype=torch.long))  # no grads: nothing to do, no device call
    p.grad = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        opt.step(relevance=torch.zeros(4))


@pytest.mark.parametrize("case", ["plain", "scaffold"])
def test_torch_ref_densify_matches_reference_run(case):
    """oracle/train_torch_ref.densify_and_prune (the larger-size checker of test_gpu_densify.py) on
    CPU against the reference's own densify_and_prune run (tests/golden/densify_prune_*.npz), with
    the reference's standard-normal split draws injected: bit-exact."""
    import train_torch_ref as R
    from gs_train.harness import GaussianSet
    d = _gold(f"densify_prune_{case}.npz")
    P = d["in_xyz"].shape[0]
    g = GaussianSet(means3D=d["in_xyz"], shs=np.concatenate([d["in_f_dc"], d["in_f_rest"]], 1),
                    opacities=np.full((P, 1), 0.5, np.float32), scales=np.ones((P, 3), np.float32),
                    rotations=d["in_rotation"], device="cpu", joined_features=False)
    with torch.no_grad():
        g._opacity.copy_(torch.tensor(d["in_opacity"]))
        g._scaling.copy_(torch.tensor(d["in_scaling"]))
    g.xyz_gradient_accum = torch.tensor(d["in_accum"])
    g.max_radii2D = torch.tensor(d["in_max_radii2D"])
    g.denom = torch.tensor(d["in_denom"])
    opt = R.OurAdamTorch(g.param_groups(), lr=0.0, eps=1e-15)
    keys = {"_xyz": "xyz", "_features_dc": "f_dc", "_features_rest": "f_rest", "_opacity": "opacity",
            "_scaling": "scaling", "_rotation": "rotation"}
    for attr, k in keys.items():
        opt.state[getattr(g, attr)] = {"step": torch.tensor(7.0), "exp_avg": torch.tensor(d["in_m_" + k]),
                                       "exp_avg_sq": torch.tensor(d["in_v_" + k])}
    z = torch.tensor(d["normals"])
    real = torch.normal
    torch.normal = lambda mean, std: z * std
    try:
        R.densify_and_prune(g, opt, float(d["max_grad"]), float(d["min_opacity"]), float(d["extent"]),
                            float(d["percent_dense"]), first_row=int(d["scaffold"]))
    finally:
        torch.normal = real
    for attr, k in keys.items():
        p = getattr(g, attr)
        np.testing.assert_array_equal(p.detach().numpy(), d["out_" + k], err_msg=k)
        np.testing.assert_array_equal(opt.state[p]["exp_avg"].numpy(), d["out_m_" + k])
        np.testing.assert_array_equal(opt.state[p]["exp_avg_sq"].numpy(), d["out_v_" + k])
    np.testing.assert_array_equal(g.denom.numpy(), d["out_denom"])
    np.testing.assert_array_equal(g.max_radii2D.numpy(), d["out_max_radii2D"])


def test_chunk_schedule_events_follow_train_single():
    """gs_train.chunk.ChunkSchedule.events on the default OptimizationParams: densify every 300
    iterations after 500 and before 15000, a reset every 3000 (each on a densify iteration), none from
    densify_until_iter on (train_single.py:191-201, arguments/__init__.py:103-107)."""
    from gs_train.chunk import ChunkSchedule
    s = ChunkSchedule()
    ev = {it: s.events(it) for it in range(1, s.iterations + 1)}
    dens = [it for it, (d, _) in ev.items() if d]
    resets = [it for it, (_, r) in ev.items() if r]
    assert dens == list(range(600, 15000, 300))
    assert resets == [3000, 6000, 9000, 12000]
    assert set(resets) <= set(dens)
    w = ChunkSchedule(white_background=True)
    assert w.events(500) == (False, True)


def test_spatial_reorder_is_a_row_permutation():
    """gs_train.chunk.reorder_rows: the rows after the fixed prefix are permuted by Morton code --
    every parameter, both Adam moments and the densification statistics by the same permutation,
    the optimizer's groups and state re-keyed to the new parameters, the prefix rows untouched --
    and spatial_order is stable and groups nearby points."""
    import types
    from gs_train.chunk import reorder_rows, spatial_order
    from gs_train.harness import GaussianSet
    from gs_train.optim import Adam
    rng = np.random.default_rng(3)
    P, first = 500, 37
    g = GaussianSet(rng.normal(size=(P, 3)) * 5, rng.normal(size=(P, 16, 3)), rng.uniform(0.1, 0.9, (P, 1)),
                    np.exp(rng.normal(-3, 0.3, (P, 3))), rng.normal(size=(P, 4)), device="cpu", joined_features=True)
    opt = Adam(g.param_groups(), lr=0.0, eps=1e-15)
    names = ("_xyz", "_features", "_opacity", "_scaling", "_rotation")
    for n in names:
        p = getattr(g, n)
        opt.state[p] = {"step": torch.tensor(3.0), "exp_avg": torch.randn_like(p), "exp_avg_sq": torch.rand_like(p)}
    g.max_radii2D = torch.arange(P, dtype=torch.float32)
    g.xyz_gradient_accum = torch.rand(P, 1)
    g.denom = torch.rand(P, 1)
    before = {n: (getattr(g, n).detach().clone(), opt.state[getattr(g, n)]["exp_avg"].clone(),
                  opt.state[getattr(g, n)]["exp_avg_sq"].clone()) for n in names}
    stats = {n: getattr(g, n).clone() for n in ("max_radii2D", "xyz_gradient_accum", "denom")}
    reorder_rows(types.SimpleNamespace(g=g, optimizer=opt), first)
    perm = g.max_radii2D.long()  # the statistics carried the row numbers
    assert torch.equal(perm[:first], torch.arange(first))
    assert sorted(perm.tolist()) == list(range(P))
    want = torch.cat((torch.arange(first), spatial_order(before["_xyz"][0][first:]) + first))
    assert torch.equal(perm, want)
    for n in names:
        p = getattr(g, n)
        st = opt.state[p]
        p0, m0, v0 = before[n]
        assert torch.equal(p.detach(), p0[perm])
        assert torch.equal(st["exp_avg"], m0[perm]) and torch.equal(st["exp_avg_sq"], v0[perm])
        assert float(st["step"]) == 3.0
        assert sum(q is p for grp in opt.param_groups for q in grp["params"]) == 1
    assert len(opt.state) == len(names)
    for n in ("xyz_gradient_accum", "denom"):
        assert torch.equal(getattr(g, n), stats[n][perm])
    # stable, and nearby points adjacent: two tight clusters come out as two runs
    pts = torch.cat((torch.full((5, 3), 1.0), torch.full((5, 3), -1.0), torch.full((5, 3), 1.0)))
    o = spatial_order(pts)
    assert o.tolist() == [5, 6, 7, 8, 9, 0, 1, 2, 3, 4, 10, 11, 12, 13, 14]
