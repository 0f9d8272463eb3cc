"""Generate train-step golden fixtures from the reference's own Python (build container only).

  loss.npz       utils/loss_utils.py:17-18 l1_loss and :33-63 ssim on small (3, H, W) images,
                 the photometric loss of train_single.py:121-123 ((1 - 0.2) L1 + 0.2 (1 - SSIM))
                 and its gradient w.r.t. the rendered image (torch autograd through the
                 reference functions), for several sizes incl. odd ones smaller than the window
  adam.npz       scene/OurAdam.py Adam(..., lr=0.0, eps=1e-15) with the six groups and learning
                 rates of scene/gaussian_model.py:286-296: two sparse steps (relevant = rows with
                 nonzero opacity grad, train_single.py:224-230) then one step with no relevant
                 row (the _single_tensor_adam2 dense branch)
  adam_coarse.npz  the same optimizer as train_coarse.py:131-134 drives it: relevant =
                 (opacity.grad != 0).nonzero() of the (P, 1) gradient, an (R, 2) index whose second
                 column is all 0, so OurAdam's gather / scatter (scene/OurAdam.py:267-270,334-337)
                 also updates row 0; the coarse model's degree-1 SH (f_rest (P, 3, 3)); row 0 kept
                 irrelevant so the quirk shows
  lr.npz         utils/general_utils.py:31-70 get_expon_lr_func with the xyz and exposure
                 schedules of scene/gaussian_model.py:301-305 (arguments/__init__.py:89-100)
  densify.npz    scene/gaussian_model.py:780-793 add_densification_stats + the max_radii2D update
                 of train_single.py:193
  densify_prune_<case>.npz
                 the reference's own GaussianModel.densify_and_prune (scene/gaussian_model.py:
                 672-778: clone, split, opacity prune; gt_point_cloud_constraints off), imported with
                 its native dependencies stubbed and a CPU device shim, run on a seeded model with
                 OurAdam moments: inputs, the standard-normal draws behind its torch.normal split
                 samples (checked bit for bit against the samples it drew), and every parameter,
                 moment and statistic it leaves (case "plain": no scaffold; "scaffold": the first
                 rows a scaffold, scaffold_points set)

Nothing from the reference is copied; only numbers are kept.
Usage:  python tests/golden/make_train_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))
LRS = {"xyz": 0.00016, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.05, "scaling": 0.005,
       "rotation": 0.001}
SHAPES = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,)}


def load_by_path(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_loss(ref):
    loss_utils = load_by_path("ref_loss_utils", os.path.join(ref, "utils", "loss_utils.py"))
    g = torch.Generator().manual_seed(7)
    out = {}
    sizes = [(3, 16, 16), (3, 37, 53), (3, 7, 9), (1, 24, 70), (3, 64, 96)]
    for k, (C, H, W) in enumerate(sizes):
        img = torch.rand((C, H, W), generator=g)
        gt = (img + 0.15 * torch.randn((C, H, W), generator=g)).clamp(0, 1)
        img.requires_grad_(True)
        l1 = loss_utils.l1_loss(img, gt)
        s = loss_utils.ssim(img, gt)
        loss = (1.0 - 0.2) * l1 + 0.2 * (1.0 - s)
        loss.backward()
        out[f"img_{k}"] = img.detach().numpy()
        out[f"gt_{k}"] = gt.numpy()
        out[f"l1_{k}"] = np.float32(l1.item())
        out[f"ssim_{k}"] = np.float32(s.item())
        out[f"loss_{k}"] = np.float32(loss.item())
        out[f"grad_{k}"] = img.grad.numpy()
    out["n"] = np.int32(len(sizes))
    np.savez_compressed(os.path.join(OUT, "loss.npz"), **out)


def make_adam(ref):
    our_adam = load_by_path("ref_our_adam", os.path.join(ref, "scene", "OurAdam.py"))
    g = torch.Generator().manual_seed(11)
    P = 50
    params = {n: torch.nn.Parameter(torch.randn((P,) + s, generator=g)) for n, s in SHAPES.items()}
    groups = [{"params": [params[n]], "lr": LRS[n], "name": n} for n in SHAPES]
    opt = our_adam.Adam(groups, lr=0.0, eps=1e-15)
    out = {f"init_{n}": p.detach().numpy().copy() for n, p in params.items()}
    for step in range(3):
        grads = {n: torch.randn((P,) + s, generator=g) for n, s in SHAPES.items()}
        if step < 2:
            mask = torch.rand(P, generator=g) < 0.6
        else:
            mask = torch.zeros(P, dtype=torch.bool)
        grads["opacity"][~mask] = 0.0
        for n, p in params.items():
            p.grad = grads[n].clone()
            out[f"grad{step}_{n}"] = grads[n].numpy().copy()
        relevant = (params["opacity"].grad.flatten() != 0).nonzero().flatten().long()
        opt.step(relevant)
        for n, p in params.items():
            out[f"after{step}_{n}"] = p.detach().numpy().copy()
            st = opt.state[p]
            out[f"m{step}_{n}"] = st["exp_avg"].numpy().copy()
            out[f"v{step}_{n}"] = st["exp_avg_sq"].numpy().copy()
    out["lrs"] = np.array([LRS[n] for n in SHAPES], np.float64)
    np.savez_compressed(os.path.join(OUT, "adam.npz"), **out)


def make_adam_coarse(ref):
    our_adam = load_by_path("ref_our_adam_coarse", os.path.join(ref, "scene", "OurAdam.py"))
    g = torch.Generator().manual_seed(12)
    P = 40
    shapes = dict(SHAPES, f_rest=(3, 3))
    params = {n: torch.nn.Parameter(torch.randn((P,) + s, generator=g)) for n, s in shapes.items()}
    groups = [{"params": [params[n]], "lr": LRS[n], "name": n} for n in shapes]
    opt = our_adam.Adam(groups, lr=0.0, eps=1e-15)
    out = {f"init_{n}": p.detach().numpy().copy() for n, p in params.items()}
    for step in range(2):
        grads = {n: torch.randn((P,) + s, generator=g) for n, s in shapes.items()}
        mask = torch.rand(P, generator=g) < 0.5
        mask[0] = False
        grads["opacity"][~mask] = 0.0
        for n, p in params.items():
            p.grad = grads[n].clone()
            out[f"grad{step}_{n}"] = grads[n].numpy().copy()
        relevant = (params["opacity"].grad != 0).nonzero()  # train_coarse.py:133, shape (R, 2)
        assert relevant.dim() == 2 and relevant.shape[1] == 2
        out[f"relevant{step}"] = relevant.numpy().copy()
        opt.step(relevant)
        for n, p in params.items():
            out[f"after{step}_{n}"] = p.detach().numpy().copy()
            st = opt.state[p]
            out[f"m{step}_{n}"] = st["exp_avg"].numpy().copy()
            out[f"v{step}_{n}"] = st["exp_avg_sq"].numpy().copy()
    out["lrs"] = np.array([LRS[n] for n in shapes], np.float64)
    np.savez_compressed(os.path.join(OUT, "adam_coarse.npz"), **out)


def make_densify():
    # add_densification_stats is a GaussianModel method that needs the whole scene package;
    # its three lines are evaluated here on the same tensors the method would see.
    ref_src = open(os.path.join(ARGS.ref, "scene", "gaussian_model.py")).read()
    assert "def add_densification_stats" in ref_src
    g = torch.Generator().manual_seed(5)
    P = 64
    radii = torch.randint(-2, 12, (P,), generator=g).clamp_min(0).int()
    grad2d = torch.randn((P, 3), generator=g)
    grad2d[:, 2] = 0
    max_r = torch.rand(P, generator=g) * 8
    accum = torch.rand((P, 1), generator=g) * 2
    denom = torch.randint(0, 5, (P, 1), generator=g).float()
    out = {"radii": radii.numpy(), "grad2d": grad2d.numpy(), "max_r": max_r.numpy(), "accum": accum.numpy(),
           "denom": denom.numpy()}
    vis = radii > 0
    max_r2, accum2, denom2 = max_r.clone(), accum.clone(), denom.clone()
    max_r2[vis] = torch.max(max_r2[vis], radii[vis])  # train_single.py:193
    nv = torch.norm(grad2d[vis, :2], dim=-1, keepdim=True)  # gaussian_model.py:781-793
    accum2[vis] = torch.max(nv, accum2[vis])
    denom2[vis] += 1
    out.update({"max_r_after": max_r2.numpy(), "accum_after": accum2.numpy(), "denom_after": denom2.numpy()})
    np.savez_compressed(os.path.join(OUT, "densify.npz"), **out)


def _import_gaussian_model(ref):
    """scene.gaussian_model with its native / optional imports stubbed (plyfile, simple_knn._C,
    gaussian_hierarchy._C, faiss): the module's Python runs as written."""
    import importlib
    import types
    stubs = {"plyfile": dict(PlyData=object, PlyElement=object), "simple_knn": {}, "simple_knn._C": dict(distCUDA2=None),
             "gaussian_hierarchy": {}, "gaussian_hierarchy._C": dict(load_hierarchy=None, write_hierarchy=None),
             "faiss": {}}
    for name, attrs in stubs.items():
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
    pkg = types.ModuleType("scene")  # the package __init__ pulls in dataset readers (PIL, plyfile)
    pkg.__path__ = [os.path.join(ref, "scene")]
    sys.modules["scene"] = pkg
    return importlib.import_module("scene.gaussian_model")


def make_densify_prune(ref):
    from make_golden import _NoCuda
    gm = _import_gaussian_model(ref)
    our_adam = sys.modules["scene.OurAdam"]
    for case, scaffold in (("plain", None), ("scaffold", 150)):
        g = torch.Generator().manual_seed(21 if scaffold is None else 22)
        P = 1200
        m = gm.GaussianModel.__new__(gm.GaussianModel)
        m.setup_functions()
        q = torch.randn((P, 4), generator=g)
        init = {"xyz": torch.randn((P, 3), generator=g) * 5, "f_dc": torch.randn((P, 1, 3), generator=g),
                "f_rest": torch.randn((P, 15, 3), generator=g), "opacity": torch.randn((P, 1), generator=g) * 2,
                "scaling": torch.randn((P, 3), generator=g) * 0.7 - 4.0, "rotation": q}
        for k, v in init.items():
            setattr(m, "_" + ("features_dc" if k == "f_dc" else "features_rest" if k == "f_rest" else k),
                    torch.nn.Parameter(v.clone()))
        acc = torch.rand((P, 1), generator=g) * 0.001
        acc[::97] = float("nan")  # NaN accumulators are zeroed first (gaussian_model.py:735)
        maxr = torch.rand(P, generator=g) * 20
        m.xyz_gradient_accum = acc.clone()
        m.xyz_gradient_accum_depth = torch.zeros((P, 1))
        m.denom = torch.randint(0, 5, (P, 1), generator=g).float()
        m.max_radii2D = maxr.clone()
        m.percent_dense = 0.0001
        m.scaffold_points = scaffold
        attr = {"xyz": m._xyz, "f_dc": m._features_dc, "f_rest": m._features_rest, "opacity": m._opacity,
                "scaling": m._scaling, "rotation": m._rotation}
        m.optimizer = our_adam.Adam([{"params": [attr[n]], "lr": 0.0, "name": n} for n in attr], lr=0.0, eps=1e-15)
        out = {"in_" + n: v.numpy() for n, v in init.items()}
        for n, p_ in attr.items():
            mom, var = torch.randn(p_.shape, generator=g), torch.rand(p_.shape, generator=g)
            m.optimizer.state[p_] = {"step": torch.tensor(7.0), "exp_avg": mom.clone(), "exp_avg_sq": var.clone()}
            out["in_m_" + n], out["in_v_" + n] = mom.numpy(), var.numpy()
        out.update(in_accum=acc.numpy(), in_max_radii2D=maxr.numpy(), in_denom=m.denom.numpy())
        args = dict(max_grad=0.0002, min_opacity=0.05, extent=200.0)
        # record the split samples torch.normal draws, and the standard normals behind them
        real_normal, rec = torch.normal, {}

        def normal(*a, **k):
            r = real_normal(*a, **k)
            rec["samples"], rec["std"] = r.clone(), k["std"].clone()
            return r
        torch.manual_seed(1234)
        state = torch.get_rng_state()
        torch.normal = normal
        try:
            with _NoCuda():
                m.densify_and_prune(args["max_grad"], args["min_opacity"], args["extent"], False)
        finally:
            torch.normal = real_normal
        torch.set_rng_state(state)
        z = torch.empty(rec["samples"].shape).normal_()
        assert torch.equal(z * rec["std"], rec["samples"]), "torch.normal is not normal_() * std here"
        out["normals"] = z.numpy()
        out.update(max_grad=np.float32(args["max_grad"]), min_opacity=np.float32(args["min_opacity"]),
                   extent=np.float32(args["extent"]), percent_dense=np.float32(m.percent_dense),
                   scaffold=np.int32(scaffold or 0))
        final = {"xyz": m._xyz, "f_dc": m._features_dc, "f_rest": m._features_rest, "opacity": m._opacity,
                 "scaling": m._scaling, "rotation": m._rotation}
        grp = {pg["name"]: pg["params"][0] for pg in m.optimizer.param_groups}
        for n, p_ in final.items():
            assert grp[n] is p_
            st = m.optimizer.state[p_]
            out["out_" + n] = p_.detach().numpy()
            out["out_m_" + n], out["out_v_" + n] = st["exp_avg"].numpy(), st["exp_avg_sq"].numpy()
        out.update(out_accum=m.xyz_gradient_accum.numpy(), out_denom=m.denom.numpy(),
                   out_max_radii2D=m.max_radii2D.numpy())
        np.savez_compressed(os.path.join(OUT, f"densify_prune_{case}.npz"), **out)
        print(case, "P", P, "->", m._xyz.shape[0], "split samples", tuple(rec["samples"].shape))


def make_lr(ref):
    gu = load_by_path("ref_general_utils", os.path.join(ref, "utils", "general_utils.py"))
    steps = np.array([0, 1, 2, 10, 100, 999, 1000, 5000, 12345, 29999, 30000, 40000], np.int64)
    xyz = gu.get_expon_lr_func(lr_init=0.00002 * 3.5, lr_final=0.0000002 * 3.5, lr_delay_mult=0.01, max_steps=30_000)
    exp = gu.get_expon_lr_func(0.001, 0.0001, lr_delay_steps=5000, lr_delay_mult=0.001, max_steps=30_000)
    np.savez_compressed(os.path.join(OUT, "lr.npz"), steps=steps, xyz=np.array([xyz(int(s)) for s in steps]),
                        exposure=np.array([exp(int(s)) for s in steps]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ARGS = ap.parse_args()
    sys.path.insert(0, ARGS.ref)
    make_loss(ARGS.ref)
    make_adam(ARGS.ref)
    make_adam_coarse(ARGS.ref)
    make_densify()
    make_lr(ARGS.ref)
    sys.path.insert(0, OUT)
    make_densify_prune(ARGS.ref)
    print("wrote loss.npz adam.npz adam_coarse.npz densify.npz lr.npz densify_prune_*.npz")
