"""Seeded synthetic workloads: cameras in the rasterizer's matrix convention and
Gaussian scenes in the camera frustum.  numpy only; the same seeds give the same arrays as the
oracle's generator (tests/test_train_cpu.py checks this), so bench numbers and parity tests refer
to the same scenes.
"""
from __future__ import annotations

import math

import numpy as np


def projection_matrix(znear, zfar, fovX, fovY, primx=0.5, primy=0.5):
    """utils/graphics_utils.py:51-77 (row-major, not transposed), principal point included."""
    tan_y, tan_x = math.tan(fovY / 2), math.tan(fovX / 2)
    top = tan_y * znear
    bottom = (1 - primy) * 2 * -top
    top = primy * 2 * top
    right = tan_x * znear
    left = (1 - primx) * 2 * -right
    right = primx * 2 * right
    P = np.zeros((4, 4), np.float32)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def camera(W, H, fovx_deg=60.0, R=None, t=None, znear=0.01, zfar=100.0, primx=0.5, primy=0.5):
    """(viewmatrix, projmatrix, campos, tanfovx, tanfovy): viewmatrix = W2C^T and
    projmatrix = (P W2C)^T as row-major fp32 (scene/cameras.py:96-99).  R is the world->camera
    rotation's transpose as the reference stores it, t the world->camera translation."""
    fovx = math.radians(fovx_deg)
    fx = W / (2 * math.tan(fovx / 2))
    fovy = 2 * math.atan(H / (2 * fx))
    R = np.eye(3) if R is None else np.asarray(R, np.float64)
    t = np.zeros(3) if t is None else np.asarray(t, np.float64)
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.T
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    view = Rt.astype(np.float32).T.copy()
    Pm = projection_matrix(znear, zfar, fovx, fovy, primx, primy)
    proj = (view @ Pm.T.astype(np.float32)).astype(np.float32)
    campos = np.linalg.inv(view.astype(np.float64))[3, :3].astype(np.float32)
    return view, proj, campos, math.tan(fovx * 0.5), math.tan(fovy * 0.5)


def synthetic_scene(P, W, H, seed=0, sh_degree=3, fovx_deg=60.0, zmin=2.0, zmax=20.0, log_scale_mean=-4.0,
                    log_scale_std=0.5, primx=0.5, primy=0.5):
    """P Gaussians uniform in the frustum at z ~ U[zmin, zmax], log-scales ~ N(-4, 0.5),
    normalised random quaternions, opacity ~ U[0.05, 0.99], SH DC ~ N(0, 0.5), rest ~ N(0, 0.05)."""
    rng = np.random.default_rng(seed)
    view, proj, campos, tx, ty = camera(W, H, fovx_deg, primx=primx, primy=primy)
    z = rng.uniform(zmin, zmax, P)
    x = rng.uniform(-0.95, 0.95, P) * tx * z
    y = rng.uniform(-0.95, 0.95, P) * ty * z
    means = np.stack([x, y, z], 1).astype(np.float32)
    scales = np.exp(rng.normal(log_scale_mean, log_scale_std, (P, 3))).astype(np.float32)
    q = rng.normal(size=(P, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    opac = rng.uniform(0.05, 0.99, (P, 1)).astype(np.float32)
    M = max((sh_degree + 1) ** 2, 1)
    shs = np.zeros((P, 16 if sh_degree == 3 else M, 3), np.float32)
    shs[:, 0, :] = rng.normal(0, 0.5, (P, 3))
    shs[:, 1:, :] = rng.normal(0, 0.05, (P, shs.shape[1] - 1, 3))
    bg = rng.uniform(0, 1, 3).astype(np.float32)
    return dict(means3D=means, scales=scales, rotations=q.astype(np.float32), opacities=opac, shs=shs, view=view,
                proj=proj, campos=campos, tanfovx=tx, tanfovy=ty, bg=bg, W=W, H=H, sh_degree=sh_degree)


def orbit_cameras(n, W, H, fovx_deg=60.0, radius_deg=4.0, shift=0.3):
    """n cameras looking roughly down +z with small yaw/pitch and translation offsets (training
    views for the train-step harness)."""
    cams = []
    for k in range(n):
        a = math.radians(radius_deg) * math.sin(2 * math.pi * k / max(n, 1))
        b = math.radians(radius_deg) * math.cos(2 * math.pi * k / max(n, 1))
        Ry = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        Rx = np.array([[1, 0, 0], [0, math.cos(b), -math.sin(b)], [0, math.sin(b), math.cos(b)]])
        Rw2c = Rx @ Ry
        t = np.array([shift * math.sin(a * 7), shift * math.cos(b * 7) - shift, 0.0])
        cams.append(camera(W, H, fovx_deg, R=Rw2c.T, t=t))
    return cams


def synthetic_hierarchy(N, R, S, W, H, device, seed=0, sh_degree=3, fovx_deg=60.0, zmin=2.0, zmax=40.0,
                        log_scale_mean=-4.5, log_scale_std=0.5):
    """Config-5 stand-in: N hierarchy nodes generated on the device (torch), a cut
    of R rendered nodes with random parents and blend weights, and S skybox Gaussians at the end.
    The node attributes are *activated* tensors, as render_post reads them (pc.get_xyz, ...).
    The merged .hier files and expand_to_size are not available here, so the cut
    is random: what it stresses is the size of the gather and of the rendered set."""
    import torch
    g = torch.Generator(device=device).manual_seed(seed)
    view, proj, campos, tx, ty = camera(W, H, fovx_deg)
    u = lambda *s: torch.rand(*s, generator=g, device=device)
    z = zmin + (zmax - zmin) * u(N)
    means = torch.stack([(u(N) * 1.9 - 0.95) * tx * z, (u(N) * 1.9 - 0.95) * ty * z, z], 1)
    scales = torch.exp(log_scale_mean + log_scale_std * torch.randn(N, 3, generator=g, device=device))
    q = torch.randn(N, 4, generator=g, device=device)
    q = q / q.norm(dim=1, keepdim=True)
    opac = 0.05 + 0.94 * u(N, 1)
    M = 16 if sh_degree == 3 else max((sh_degree + 1) ** 2, 1)
    shs = 0.05 * torch.randn(N, M, 3, generator=g, device=device)
    shs[:, 0, :] = 0.5 * torch.randn(N, 3, generator=g, device=device)
    ri = torch.randperm(N - S, generator=g, device=device)[:R].int()
    pi = torch.randint(0, N - S, (R,), generator=g, device=device).int()
    w = u(N)
    return dict(means3D=means, scales=scales, rotations=q, opacities=opac, shs=shs, render_indices=ri,
                parent_indices=pi, interpolation_weights=w, skybox=S, view=view, proj=proj, campos=campos,
                tanfovx=tx, tanfovy=ty, W=W, H=H, sh_degree=sh_degree)
