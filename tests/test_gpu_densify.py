"""GPU parity of the fused densify-and-prune (csrc/densify.hip, include/gsr_densify.h):

* against the reference itself: tests/golden/densify_prune_*.npz hold the inputs and outputs of
  the reference's own GaussianModel.densify_and_prune (scene/gaussian_model.py:672-778, run by
  tests/golden/make_train_golden.py in the build container) and the standard-normal draws behind
  its split samples, which are injected here -- row order, counts, every parameter, both Adam
  moments and the statistics bit-exact, except the split children's xyz, which the reference
  forms with torch.bmm (library summation order; 1e-6), and their scaling log(exp(s) / 1.6)
  (CPU exp / log / true division in the fixture run; a few ulps);
* at larger sizes against the torch restatement (oracle/train_torch_ref.densify_and_prune) on the
  same generator stream."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _state(P, seed):
    from gs_train.harness import GaussianSet
    rng = np.random.default_rng(seed)
    q = rng.normal(size=(P, 4)).astype(np.float32)
    kw = dict(means3D=rng.normal(size=(P, 3)).astype(np.float32) * 5,
              shs=rng.normal(size=(P, 16, 3)).astype(np.float32),
              opacities=rng.uniform(0.01, 0.99, (P, 1)).astype(np.float32),
              scales=np.exp(rng.normal(-4.0, 0.5, (P, 3))).astype(np.float32), rotations=q, device=DEV)
    a = GaussianSet(joined_features=True, **kw)
    b = GaussianSet(joined_features=False, **kw)
    acc = rng.uniform(0, 0.001, (P, 1)).astype(np.float32)
    acc[::97] = np.nan  # NaN accumulators are zeroed first
    maxr = rng.uniform(0, 20, P).astype(np.float32)
    for g in (a, b):
        g.xyz_gradient_accum = torch.tensor(acc, device=DEV)
        g.max_radii2D = torch.tensor(maxr, device=DEV)
    return a, b, rng


def _optimizers(a, b, rng):
    from gs_train import Adam
    from train_torch_ref import OurAdamTorch
    oa = Adam(a.param_groups(), lr=0.0, eps=1e-15)
    ob = OurAdamTorch(b.param_groups(), lr=0.0, eps=1e-15)
    mom = {}
    for name in ("_xyz", "_features", "_opacity", "_scaling", "_rotation"):
        p = getattr(a, name)
        m = torch.tensor(rng.normal(size=p.shape).astype(np.float32), device=DEV)
        v = torch.tensor(rng.uniform(0, 1, p.shape).astype(np.float32), device=DEV)
        oa.state[p] = {"step": torch.tensor(7.0), "exp_avg": m.clone(), "exp_avg_sq": v.clone()}
        mom[name] = (m, v)
    for name, attr in (("_xyz", "_xyz"), ("_opacity", "_opacity"), ("_scaling", "_scaling"),
                       ("_rotation", "_rotation")):
        m, v = mom[name]
        ob.state[getattr(b, attr)] = {"step": torch.tensor(7.0), "exp_avg": m.clone(), "exp_avg_sq": v.clone()}
    m, v = mom["_features"]
    ob.state[b._features_dc] = {"step": torch.tensor(7.0), "exp_avg": m[:, :1].clone(), "exp_avg_sq": v[:, :1].clone()}
    ob.state[b._features_rest] = {"step": torch.tensor(7.0), "exp_avg": m[:, 1:].clone(),
                                  "exp_avg_sq": v[:, 1:].clone()}
    return oa, ob


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("case", ["plain", "scaffold"])
def test_densify_and_prune_matches_reference_run(case):
    from gs_train import Adam
    from gs_train.densify import densify_and_prune
    from gs_train.harness import GaussianSet
    d = np.load(os.path.join(GOLD, f"densify_prune_{case}.npz"))
    t = lambda k: torch.tensor(d[k], device=DEV).contiguous()
    P = d["in_xyz"].shape[0]
    g = GaussianSet(means3D=np.zeros((P, 3), np.float32), shs=np.zeros((P, 16, 3), np.float32),
                    opacities=np.full((P, 1), 0.5, np.float32), scales=np.ones((P, 3), np.float32),
                    rotations=np.zeros((P, 4), np.float32), device=DEV, joined_features=True)
    with torch.no_grad():  # the raw parameters exactly as the reference held them
        g._xyz.copy_(t("in_xyz"))
        g._features.copy_(torch.cat((t("in_f_dc"), t("in_f_rest")), 1))
        g._opacity.copy_(t("in_opacity"))
        g._scaling.copy_(t("in_scaling"))
        g._rotation.copy_(t("in_rotation"))
    g.xyz_gradient_accum, g.max_radii2D, g.denom = t("in_accum"), t("in_max_radii2D"), t("in_denom")
    opt = Adam(g.param_groups(), lr=0.0, eps=1e-15)
    mom = {"_xyz": ("xyz",), "_features": ("f_dc", "f_rest"), "_opacity": ("opacity",), "_scaling": ("scaling",),
           "_rotation": ("rotation",)}
    for name, keys in mom.items():
        opt.state[getattr(g, name)] = {"step": torch.tensor(7.0),
                                       "exp_avg": torch.cat([t("in_m_" + k) for k in keys], 1),
                                       "exp_avg_sq": torch.cat([t("in_v_" + k) for k in keys], 1)}
    c = densify_and_prune(g, opt, float(d["max_grad"]), float(d["min_opacity"]), float(d["extent"]),
                          float(d["percent_dense"]), first_row=int(d["scaffold"]), normals=t("normals"))
    n = d["out_xyz"].shape[0]
    assert c["total"] == n and c["cloned"] > 0 and c["split"] > 0 and c["kept"] < P
    assert 2 * c["split"] == d["normals"].shape[0]
    got = {"f_dc": g._features[:, :1], "f_rest": g._features[:, 1:], "opacity": g._opacity, "rotation": g._rotation}
    for k, v in got.items():
        np.testing.assert_array_equal(v.detach().cpu().numpy(), d["out_" + k], err_msg=k)
    old = c["kept"] + c["cloned"]  # rows before the split children: copies
    # the split children's log(exp(s) / 1.6): the reference ran on the CPU here (true division and
    # CPU exp / log); on its own CUDA device torch divides by a scalar as a multiply by its
    # reciprocal, as the kernel does -- an ulp apart at most
    sc = g._scaling.detach().cpu().numpy()
    np.testing.assert_array_equal(sc[:old], d["out_scaling"][:old])
    np.testing.assert_allclose(sc, d["out_scaling"], rtol=4e-7, atol=0)
    xyz = g._xyz.detach().cpu().numpy()
    np.testing.assert_array_equal(xyz[:old], d["out_xyz"][:old])
    np.testing.assert_allclose(xyz, d["out_xyz"], rtol=1e-6, atol=1e-6)
    for name, keys in mom.items():
        st = opt.state[getattr(g, name)]
        for sk, pre in (("exp_avg", "out_m_"), ("exp_avg_sq", "out_v_")):
            want = np.concatenate([d[pre + k] for k in keys], 1)
            np.testing.assert_array_equal(st[sk].cpu().numpy(), want, err_msg=f"{name} {sk}")
        assert float(st["step"]) == 7.0
    np.testing.assert_array_equal(g.xyz_gradient_accum.cpu().numpy(), d["out_accum"])
    np.testing.assert_array_equal(g.denom.cpu().numpy(), d["out_denom"])
    np.testing.assert_array_equal(g.max_radii2D.cpu().numpy(), d["out_max_radii2D"])


@pytest.mark.parametrize("P,first_row", [(50_000, 0), (20_011, 300)])
def test_densify_and_prune_matches_reference(P, first_row):
    from train_torch_ref import densify_and_prune as ref
    from gs_train.densify import densify_and_prune
    a, b, rng = _state(P, 3)
    oa, ob = _optimizers(a, b, rng)
    args = dict(max_grad=0.005, min_opacity=0.05, extent=200.0, percent_dense=0.0001, first_row=first_row)
    torch.manual_seed(11)
    c = densify_and_prune(a, oa, **args)
    torch.manual_seed(11)
    ref(b, ob, **args)
    n = b._xyz.shape[0]
    assert c["total"] == n and c["cloned"] > 100 and c["split"] > 100 and c["kept"] < P
    feats = torch.cat((b._features_dc, b._features_rest), 1)
    for x, y in ((a._features, feats), (a._opacity, b._opacity), (a._scaling, b._scaling),
                 (a._rotation, b._rotation)):
        assert torch.equal(x.detach(), y.detach())
    old = c["kept"] + c["cloned"]  # rows before the split children: copied xyz
    assert torch.equal(a._xyz.detach()[:old], b._xyz.detach()[:old])
    torch.testing.assert_close(a._xyz.detach(), b._xyz.detach(), rtol=1e-6, atol=1e-6)
    for name, pa, pb in (("xyz", a._xyz, b._xyz), ("rot", a._rotation, b._rotation)):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(oa.state[pa][k], ob.state[pb][k]), (name, k)
    fm = torch.cat((ob.state[b._features_dc]["exp_avg_sq"], ob.state[b._features_rest]["exp_avg_sq"]), 1)
    assert torch.equal(oa.state[a._features]["exp_avg_sq"], fm)
    assert float(oa.state[a._xyz]["step"]) == 7.0
    for x, y in ((a.xyz_gradient_accum, b.xyz_gradient_accum), (a.denom, b.denom), (a.max_radii2D, b.max_radii2D)):
        assert torch.equal(x, y)


def test_densify_then_train_step_runs():
    """The densified set keeps training: the optimizer's groups point at the new parameters."""
    from gs_train.densify import densify_and_prune
    from gs_train.harness import make_problem
    ts = make_problem(20_000, 256, 192, n_views=2, seed=4)
    for _ in range(3):
        ts.step()
    g = ts.g
    g.xyz_gradient_accum.fill_(0.01)
    c = densify_and_prune(g, ts.optimizer, 0.0001, 0.005, 10.0, 0.0001)
    assert g.P == c["total"] and c["total"] > 20_000
    loss = [ts.step().item() for _ in range(3)]
    assert np.isfinite(loss).all()
    assert all(p.shape[0] == g.P for grp in ts.optimizer.param_groups for p in grp["params"])
