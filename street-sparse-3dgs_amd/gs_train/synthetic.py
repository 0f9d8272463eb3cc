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


def _morton3(q):
    """30-bit... 60-bit Morton code of int64 coordinates q (n, 3) in [0, 2^20)."""
    def spread(x):
        x = x & 0xFFFFF
        x = (x | (x << 32)) & 0x1F00000000FFFF
        x = (x | (x << 16)) & 0x1F0000FF0000FF
        x = (x | (x << 8)) & 0x100F00F00F00F00F
        x = (x | (x << 4)) & 0x10C30C30C30C30C3
        x = (x | (x << 2)) & 0x1249249249249249
        return x
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def synthetic_lod_hierarchy(L, W, H, device, seed=0, branching=4, skybox=0, sh_degree=3, fovx_deg=60.0, zmin=2.0,
                            zmax=40.0, log_scale_mean=-4.5, log_scale_std=0.5):
    """Config-5 stand-in with a real tree: L leaf Gaussians in the
    frustum, grouped bottom-up in Morton order, `branching` consecutive nodes per parent, up to one
    root.  Every node holds one Gaussian (leaf: count_leafs = 1; interior: count_merged = 1, the
    children's mean position, SH and opacity, a scale covering their box).  Nodes are stored root
    first, level by level (children of a node are contiguous), Gaussian i belongs to node i, and
    `skybox` far Gaussians follow the N node Gaussians.  nodes (N, 7) int32 {depth, parent, start,
    count_leafs, count_merged, start_children, count_children}, boxes (N, 2, 4) float32
    {minn.xyz, size | maxx.xyz, 0} with size = the box's largest extent -- the gaussianhierarchy
    layout (scene/gaussian_model.py:345, 424-425).  Gaussian attributes are *activated*, as
    render_post reads them.  Works on any torch device."""
    import torch
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    view, proj, campos, tx, ty = camera(W, H, fovx_deg)
    u = lambda *s: torch.rand(*s, generator=g, device=dev)
    z = zmin + (zmax - zmin) * u(L)
    means = torch.stack([(u(L) * 1.9 - 0.95) * tx * z, (u(L) * 1.9 - 0.95) * ty * z, z], 1)
    scales = torch.exp(log_scale_mean + log_scale_std * torch.randn(L, 3, generator=g, device=dev))
    q = torch.randn(L, 4, generator=g, device=dev)
    rots = q / q.norm(dim=1, keepdim=True)
    opac = 0.05 + 0.94 * u(L, 1)
    M = 16 if sh_degree == 3 else max((sh_degree + 1) ** 2, 1)
    shs = 0.05 * torch.randn(L, M, 3, generator=g, device=dev)
    shs[:, 0, :] = 0.5 * torch.randn(L, 3, generator=g, device=dev)
    # Morton order of the leaves: consecutive groups are spatially compact
    lo, hi = means.min(0).values, means.max(0).values
    qc = ((means - lo) / (hi - lo).clamp_min(1e-12) * (2 ** 20 - 1)).long()
    order = torch.argsort(_morton3(qc))
    means, scales, rots, opac, shs = means[order], scales[order], rots[order], opac[order], shs[order]
    ext = 3.0 * scales.max(1, keepdim=True).values
    levels = [dict(means=means, scales=scales, rots=rots, opac=opac, shs=shs, bmin=means - ext, bmax=means + ext)]
    while levels[-1]["means"].shape[0] > 1:
        c = levels[-1]
        n = c["means"].shape[0]
        m = (n + branching - 1) // branching
        grp = torch.arange(n, device=dev) // branching
        cnt = torch.bincount(grp, minlength=m).to(torch.float32)[:, None]
        mean_of = lambda x: torch.zeros((m,) + x.shape[1:], device=dev, dtype=x.dtype).index_add_(0, grp, x) / (
            cnt.view((m,) + (1,) * (x.dim() - 1)))
        bmin = torch.full((m, 3), float("inf"), device=dev).scatter_reduce(0, grp[:, None].expand(n, 3), c["bmin"],
                                                                           "amin")
        bmax = torch.full((m, 3), float("-inf"), device=dev).scatter_reduce(0, grp[:, None].expand(n, 3), c["bmax"],
                                                                            "amax")
        pr = torch.zeros(m, 4, device=dev)
        pr[:, 0] = 1.0
        levels.append(dict(means=mean_of(c["means"]), scales=(bmax - bmin) / 6.0, rots=pr, opac=mean_of(c["opac"]),
                           shs=mean_of(c["shs"]), bmin=bmin, bmax=bmax))
    levels = levels[::-1]  # root first
    sizes = [lv["means"].shape[0] for lv in levels]
    offs = [0]
    for s_ in sizes:
        offs.append(offs[-1] + s_)
    N = offs[-1]
    nodes = torch.zeros(N, 7, dtype=torch.int32, device=dev)
    for d, lv in enumerate(levels):
        n = sizes[d]
        j = torch.arange(n, device=dev, dtype=torch.int64)
        rows = slice(offs[d], offs[d] + n)
        nodes[rows, 0] = d
        nodes[rows, 1] = (offs[d - 1] + j // branching).int() if d > 0 else -1
        nodes[rows, 2] = (offs[d] + j).int()
        leaf = d == len(levels) - 1
        nodes[rows, 3] = 1 if leaf else 0
        nodes[rows, 4] = 0 if leaf else 1
        if not leaf:
            nc = sizes[d + 1]
            nodes[rows, 5] = (offs[d + 1] + j * branching).int()
            nodes[rows, 6] = torch.clamp(nc - j * branching, max=branching).int()
        else:
            nodes[rows, 5] = -1
            nodes[rows, 6] = 0
    cat = lambda k: torch.cat([lv[k] for lv in levels])
    bmin, bmax = cat("bmin"), cat("bmax")
    size = (bmax - bmin).max(1).values
    boxes = torch.zeros(N, 2, 4, device=dev)
    boxes[:, 0, :3], boxes[:, 0, 3], boxes[:, 1, :3] = bmin, size, bmax
    out = dict(means3D=cat("means"), scales=cat("scales"), rotations=cat("rots"), opacities=cat("opac"),
               shs=cat("shs"))
    if skybox:
        r = 200.0
        d = torch.randn(skybox, 3, generator=g, device=dev)
        d[:, 2] = d[:, 2].abs() + 0.5
        d = d / d.norm(dim=1, keepdim=True)
        sk = dict(means3D=r * d, scales=torch.full((skybox, 3), 2.0, device=dev),
                  rotations=torch.tensor([[1.0, 0, 0, 0]], device=dev).expand(skybox, 4),
                  opacities=0.5 + 0.4 * u(skybox, 1), shs=0.05 * torch.randn(skybox, M, 3, generator=g, device=dev))
        sk["shs"][:, 0, :] = 0.5 * torch.randn(skybox, 3, generator=g, device=dev)
        out = {k: torch.cat([out[k], sk[k]]).contiguous() for k in out}
    out.update(nodes=nodes, boxes=boxes, skybox=skybox, view=view, proj=proj, campos=campos, tanfovx=tx, tanfovy=ty,
               W=W, H=H, sh_degree=sh_degree, levels=len(levels))
    return out


def tau_threshold(tau, tanfovx, W):
    """render_hierarchy.py:61: the target size for a tau (in pixels)."""
    return (2 * (tau + 0.5)) * tanfovx / (0.5 * W)
