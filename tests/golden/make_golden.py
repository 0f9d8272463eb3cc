"""Generate golden fixtures from the reference's own Python (run in the build container only).

The rasterizer's CUDA source is not vendored in the reference, but the
reference holds pure-torch twins of the in-kernel maths and the callers of the boundary.
This script imports them from /root/reference and records inputs + outputs as small .npz /
.json fixtures.  Nothing from the reference is copied; only numbers are kept.

  sh_eval.npz        utils/sh_utils.py:57-112 eval_sh, degrees 0..3, and the +0.5/clamp_min
                     colour path of gaussian_renderer/__init__.py:85-89
  covariance.npz     scene/gaussian_model.py:33-37 build_covariance_from_scaling_rotation
                     (utils/general_utils.py:68-114), incl. scaling_modifier != 1
  cameras.npz        scene/cameras.py:96-99 (getWorld2View2 / getProjectionMatrix from
                     utils/graphics_utils.py:38-77): world_view_transform,
                     full_proj_transform, camera_center, tanfov
  boundary.json      keyword names / shapes / dtypes / devices the reference's render(),
                     render_post() and render_coarse() hand to GaussianRasterizer
  render_post.npz    tensors render_post()'s Python LOD interpolation
                     (gaussian_renderer/__init__.py:200-243) passes to the rasterizer

Usage:  python tests/golden/make_golden.py  [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import types

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))


class _NoCuda:
    """Device shim: the reference hardcodes device='cuda' / .cuda() (utils/general_utils.py:69,87,
    106; gaussian_renderer/__init__.py:29,39-42).  Strip it so the code runs on CPU."""

    def __enter__(self):
        self.saved = {}
        for name in ["zeros", "zeros_like", "empty", "ones", "range", "tensor"]:
            fn = getattr(torch, name)
            self.saved[name] = fn

            def wrap(*a, __fn=fn, **k):
                k.pop("device", None)
                return __fn(*a, **k)
            setattr(torch, name, wrap)
        self.saved_cuda = torch.Tensor.cuda
        torch.Tensor.cuda = lambda self, *a, **k: self
        return self

    def __exit__(self, *exc):
        for name, fn in self.saved.items():
            setattr(torch, name, fn)
        torch.Tensor.cuda = self.saved_cuda


def gen_sh(ref):
    import utils.sh_utils as shu
    g = torch.Generator().manual_seed(11)
    P = 64
    sh = torch.randn(P, 16, 3, generator=g) * 0.5
    dirs = torch.nn.functional.normalize(torch.randn(P, 3, generator=g), dim=1)
    out = {"sh": sh.numpy(), "dirs": dirs.numpy()}
    for deg in range(4):
        M = (deg + 1) ** 2
        shs_view = sh[:, :M, :].transpose(1, 2)  # (P, 3, M) as render() builds it
        r = shu.eval_sh(deg, shs_view, dirs)
        out[f"eval_deg{deg}"] = r.numpy()
        out[f"rgb_deg{deg}"] = torch.clamp_min(r + 0.5, 0.0).numpy()
    rgb = torch.rand(8, 3, generator=g)
    out["rgb_in"] = rgb.numpy()
    out["RGB2SH"] = shu.RGB2SH(rgb).numpy()
    np.savez_compressed(os.path.join(OUT, "sh_eval.npz"), **out)


def gen_cov(ref):
    import utils.general_utils as gu
    g = torch.Generator().manual_seed(12)
    P = 64
    scales = torch.exp(torch.randn(P, 3, generator=g) * 0.7 - 3.0)
    rot_raw = torch.randn(P, 4, generator=g)
    out = {"scales": scales.numpy(), "rot_raw": rot_raw.numpy(),
           "rot_normalized": torch.nn.functional.normalize(rot_raw).numpy()}
    with _NoCuda():
        for mod in (1.0, 0.5, 2.0):
            L = gu.build_scaling_rotation(mod * scales, rot_raw)
            cov = gu.strip_symmetric(L @ L.transpose(1, 2))
            out[f"cov_mod{mod}"] = cov.numpy()
        out["R"] = gu.build_rotation(rot_raw).numpy()
    np.savez_compressed(os.path.join(OUT, "covariance.npz"), **out)


def gen_cameras(ref):
    from utils.graphics_utils import getWorld2View2, getProjectionMatrix, focal2fov
    rng = np.random.default_rng(13)
    rows = []
    cams = [
        (64, 48, 60.0, np.eye(3), np.zeros(3), 0.5, 0.5),
        (96, 64, 50.0, None, np.array([0.3, -0.2, 1.5]), 0.45, 0.55),
        (1920, 1080, 60.0, None, np.array([-1.0, 0.5, 2.0]), 0.5, 0.5),
        (1536, 1536, 90.0, None, np.array([0.0, 0.0, 0.0]), 0.5, 0.5),
    ]
    out = {}
    for i, (W, H, fovx_deg, R, T, px, py) in enumerate(cams):
        if R is None:
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            r, x, y, z = q
            R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)],
                          [2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)],
                          [2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)]])
        FoVx = math.radians(fovx_deg)
        fx = W / (2 * math.tan(FoVx / 2))
        FoVy = focal2fov(fx, H)
        # scene/cameras.py:96-99
        wvt = torch.tensor(getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
        pm = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=FoVx, fovY=FoVy, primx=px, primy=py).transpose(0, 1)
        fpt = (wvt.unsqueeze(0).bmm(pm.unsqueeze(0))).squeeze(0)
        cc = wvt.inverse()[3, :3]
        out[f"cam{i}_W"] = np.int32(W)
        out[f"cam{i}_H"] = np.int32(H)
        out[f"cam{i}_R"] = np.asarray(R, np.float64)
        out[f"cam{i}_T"] = np.asarray(T, np.float64)
        out[f"cam{i}_FoVx"] = np.float64(FoVx)
        out[f"cam{i}_FoVy"] = np.float64(FoVy)
        out[f"cam{i}_primx"] = np.float64(px)
        out[f"cam{i}_primy"] = np.float64(py)
        out[f"cam{i}_viewmatrix"] = wvt.numpy()
        out[f"cam{i}_projmatrix"] = fpt.numpy()
        out[f"cam{i}_campos"] = cc.numpy()
        out[f"cam{i}_tanfovx"] = np.float64(math.tan(FoVx * 0.5))
        out[f"cam{i}_tanfovy"] = np.float64(math.tan(FoVy * 0.5))
    out["n"] = np.int32(len(cams))
    np.savez_compressed(os.path.join(OUT, "cameras.npz"), **out)


class _Recorder:
    calls = []


def _fake_rasterizer_module():
    mod = types.ModuleType("diff_gaussian_rasterization")
    from typing import NamedTuple

    class GaussianRasterizationSettings(NamedTuple):
        image_height: int
        image_width: int
        tanfovx: float
        tanfovy: float
        bg: torch.Tensor
        scale_modifier: float
        viewmatrix: torch.Tensor
        projmatrix: torch.Tensor
        sh_degree: int
        campos: torch.Tensor
        prefiltered: bool
        debug: bool
        do_depth: bool
        render_indices: torch.Tensor
        parent_indices: torch.Tensor
        interpolation_weights: torch.Tensor
        num_node_kids: torch.Tensor

    def describe(v):
        if isinstance(v, torch.Tensor):
            return {"type": "tensor", "shape": list(v.shape), "dtype": str(v.dtype).replace("torch.", ""),
                    "requires_grad": bool(v.requires_grad)}
        if v is None:
            return {"type": "None"}
        return {"type": type(v).__name__, "value": v if isinstance(v, (int, float, bool)) else str(v)}

    class GaussianRasterizer(torch.nn.Module):
        def __init__(self, raster_settings):
            super().__init__()
            self.raster_settings = raster_settings

        def forward(self, **kw):
            s = self.raster_settings
            rec = {"settings": {f: describe(getattr(s, f)) for f in s._fields},
                   "settings_order": list(s._fields), "kwargs": {k: describe(v) for k, v in kw.items()},
                   "kwargs_order": list(kw.keys())}
            rec["_tensors"] = {k: v.detach().clone() for k, v in kw.items() if isinstance(v, torch.Tensor)}
            _Recorder.calls.append(rec)
            P = kw["means3D"].shape[0]
            H, W = s.image_height, s.image_width
            color = torch.zeros(3, H, W) + 0 * kw["means3D"].sum()
            return color, torch.ones(P, dtype=torch.int32), torch.zeros(1, H, W)

    mod.GaussianRasterizationSettings = GaussianRasterizationSettings
    mod.GaussianRasterizer = GaussianRasterizer
    mod._C = types.ModuleType("diff_gaussian_rasterization._C")
    return mod


class _FakePC:
    """The attributes of scene/gaussian_model.py:125-156 that the renderer reads."""

    def __init__(self, P, deg=3, seed=0, skybox=0):
        g = torch.Generator().manual_seed(seed)
        self.max_sh_degree = deg
        self.active_sh_degree = deg
        self._xyz = torch.randn(P, 3, generator=g)
        self._features_dc = torch.randn(P, 1, 3, generator=g)
        self._features_rest = torch.randn(P, (deg + 1) ** 2 - 1, 3, generator=g) * 0.1
        self._scaling = torch.randn(P, 3, generator=g) - 3
        self._rotation = torch.randn(P, 4, generator=g)
        self._opacity = torch.randn(P, 1, generator=g)
        self.skybox_points = skybox
        self.pretrained_exposures = None
        self._exposure = torch.eye(3, 4)[None].repeat(1, 1, 1)

    get_xyz = property(lambda s: s._xyz)
    get_scaling = property(lambda s: torch.exp(s._scaling))
    get_rotation = property(lambda s: torch.nn.functional.normalize(s._rotation))
    get_opacity = property(lambda s: torch.sigmoid(s._opacity))
    get_features = property(lambda s: torch.cat((s._features_dc, s._features_rest), dim=1))

    def get_exposure_from_name(self, name):
        return self._exposure[0]

    def get_covariance(self, mod=1.0):
        import utils.general_utils as gu
        L = gu.build_scaling_rotation(mod * self.get_scaling, self._rotation)
        return gu.strip_symmetric(L @ L.transpose(1, 2))


def gen_boundary(ref):
    stubs = {}
    for name in ["plyfile", "simple_knn", "simple_knn._C", "gaussian_hierarchy", "gaussian_hierarchy._C", "faiss",
                 "cv2", "scene", "scene.gaussian_model"]:
        stubs[name] = sys.modules.get(name)
        m = types.ModuleType(name)
        sys.modules[name] = m
    sys.modules["scene.gaussian_model"].GaussianModel = object
    sys.modules["diff_gaussian_rasterization"] = _fake_rasterizer_module()
    sys.modules["diff_gaussian_rasterization._C"] = sys.modules["diff_gaussian_rasterization"]._C
    import importlib
    gr = importlib.import_module("gaussian_renderer")

    cams = np.load(os.path.join(OUT, "cameras.npz"))
    cam = types.SimpleNamespace(
        image_height=int(cams["cam1_H"]), image_width=int(cams["cam1_W"]), FoVx=float(cams["cam1_FoVx"]),
        FoVy=float(cams["cam1_FoVy"]), world_view_transform=torch.tensor(cams["cam1_viewmatrix"]),
        full_proj_transform=torch.tensor(cams["cam1_projmatrix"]), camera_center=torch.tensor(cams["cam1_campos"]),
        image_name="img0")
    pipes = {
        "default": types.SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=False),
        "python_paths": types.SimpleNamespace(debug=False, compute_cov3D_python=True, convert_SHs_python=True),
    }
    result = {}
    bg = torch.rand(3)
    with _NoCuda():
        for pname, pipe in pipes.items():
            pc = _FakePC(50, 3, seed=1)
            _Recorder.calls.clear()
            gr.render(cam, pc, pipe, bg, use_trained_exp=True)
            r = _Recorder.calls[-1]
            r.pop("_tensors")
            result[f"render/{pname}"] = r
            _Recorder.calls.clear()
            gr.render_coarse(cam, _FakePC(50, 1, seed=2), pipe, bg)
            r = _Recorder.calls[-1]
            r.pop("_tensors")
            result[f"render_coarse/{pname}"] = r

        # render_post with a toy hierarchy cut: 40 nodes, 12 rendered, 2 skybox points
        N, n_render, sky = 40, 12, 2
        pc = _FakePC(N, 3, seed=3, skybox=sky)
        g = torch.Generator().manual_seed(4)
        render_indices = torch.randperm(N - sky, generator=g)[:n_render].int()
        parent_indices = torch.randint(0, N - sky, (n_render,), generator=g).int()
        weights = torch.rand(N, generator=g)
        kids = torch.randint(1, 4, (N,), generator=g).int()
        _Recorder.calls.clear()
        gr.render_post(cam, pc, pipes["default"], bg, render_indices=render_indices, parent_indices=parent_indices,
                       interpolation_weights=weights, num_node_kids=kids, use_trained_exp=False, do_depth=True)
        r = _Recorder.calls[-1]
        tens = r.pop("_tensors")
        result["render_post/default"] = r
        np.savez_compressed(
            os.path.join(OUT, "render_post.npz"),
            xyz=pc.get_xyz.numpy(), scaling=pc.get_scaling.numpy(), rotation=pc.get_rotation.numpy(),
            opacity=pc.get_opacity.numpy(), features=pc.get_features.numpy(), skybox=np.int32(sky),
            render_indices=render_indices.numpy(), parent_indices=parent_indices.numpy(),
            interpolation_weights=weights.numpy(), num_node_kids=kids.numpy(),
            **{"out_" + k: v.numpy() for k, v in tens.items()})
    with open(os.path.join(OUT, "boundary.json"), "w") as f:
        json.dump(result, f, indent=1, sort_keys=True)
    for name, m in stubs.items():
        if m is None:
            sys.modules.pop(name, None)
        else:
            sys.modules[name] = m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    sys.path.insert(0, a.ref)
    torch.manual_seed(0)
    gen_sh(a.ref)
    gen_cov(a.ref)
    gen_cameras(a.ref)
    gen_boundary(a.ref)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
