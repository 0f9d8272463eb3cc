"""Naive vectorised PyTorch-CPU Gaussian splat -- the CPU baseline of SURVEY.md 8(d).

TEST / BASELINE INFRASTRUCTURE ONLY: imported by tests/ and by bench.py's cpu_baseline leg,
never by the product package.  It is the "naive PyTorch-CPU splat" BASELINE.json's north_star
times next to the HIP path: plain fp32 torch ops on the host cores, differentiated by
torch.autograd, no hand-written kernels.

Algorithm (the published 3DGS rasterizer, SURVEY.md 8(a) A4-A10, restated with tensor ops):
  * preprocess over all P at once: view / projection (`scene/cameras.py:96-99` conventions),
    cov3D = (R S)(R S)^T (`utils/general_utils.py:68-114`), EWA cov2D with the 1.3 tanfov clamp
    and the +0.3 low-pass, conic, radius ceil(3 sqrt(lambda_max)), tile rect, SH colour
    (`utils/sh_utils.py:57-112`, +0.5, clamp at 0);
  * duplicate-with-keys: one (tile << 32 | depth bits) key per tile instance, a stable torch.sort,
    per-tile ranges from a bincount;
  * per 16x16 tile: the (256 pixels x tile list) alpha matrix, alpha < 1/255 and power > 0
    skipped, transmittance by cumprod, the T < 1e-4 stop as a monotone mask (T is
    non-increasing, so "stop at the first instance whose T(1 - alpha) < 1e-4" is "keep the
    prefix where the inclusive product stays >= 1e-4"), colour / inverse depth as matrix products;
  * backward: torch.autograd through all of it (alpha's 0.99 clamp passes the gradient, as
    upstream does).
"""
from __future__ import annotations

import time

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)
TILE = 16


def _sh(deg, sh, d):
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C0 * sh[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
             + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r


def _rot(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)


def render(means3D, scales, rotations, opacities, shs, view, proj, campos, bg, W, H, tanfovx, tanfovy, sh_degree,
           scale_modifier=1.0):
    """Forward render; every argument a CPU fp32 torch tensor (or number).  Returns
    (color (3,H,W), invdepth (1,H,W), radii (P,) int32)."""
    P = means3D.shape[0]
    fx, fy = W / (2.0 * tanfovx), H / (2.0 * tanfovy)
    gx, gy = (W + TILE - 1) // TILE, (H + TILE - 1) // TILE
    V, Pm = view.reshape(4, 4), proj.reshape(4, 4)

    # ---- preprocess ----
    t = means3D @ V[:3, :3] + V[3, :3]
    ph = means3D @ Pm[:3, :] + Pm[3, :]
    pw = 1.0 / (ph[:, 3] + 1e-7)
    xy = torch.stack([((ph[:, 0] * pw + 1) * W - 1) * 0.5, ((ph[:, 1] * pw + 1) * H - 1) * 0.5], 1)
    L = _rot(rotations) * (scale_modifier * scales)[:, None, :]
    S3 = L @ L.transpose(1, 2)
    tz = t[:, 2]
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    txc = torch.clamp(t[:, 0] / tz, -limx, limx) * tz
    tyc = torch.clamp(t[:, 1] / tz, -limy, limy) * tz
    Wr = V[:3, :3].T
    m0 = (fx / tz)[:, None] * Wr[0] + (-(fx * txc) / (tz * tz))[:, None] * Wr[2]
    m1 = (fy / tz)[:, None] * Wr[1] + (-(fy * tyc) / (tz * tz))[:, None] * Wr[2]
    a = torch.einsum("pi,pij,pj->p", m0, S3, m0) + 0.3
    b = torch.einsum("pi,pij,pj->p", m0, S3, m1)
    c = torch.einsum("pi,pij,pj->p", m1, S3, m1) + 0.3
    det = a * c - b * b
    with torch.no_grad():
        mid = 0.5 * (a + c)
        lam = mid + torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
        radius = torch.ceil(3.0 * torch.sqrt(lam))
        x0 = torch.clamp(((xy[:, 0] - radius) / TILE).int(), 0, gx)
        y0 = torch.clamp(((xy[:, 1] - radius) / TILE).int(), 0, gy)
        x1 = torch.clamp(((xy[:, 0] + radius + TILE - 1) / TILE).int(), 0, gx)
        y1 = torch.clamp(((xy[:, 1] + radius + TILE - 1) / TILE).int(), 0, gy)
        touched = (x1 - x0) * (y1 - y0)
        vis = (tz > 0.2) & (det != 0) & (touched > 0)
        radii = torch.where(vis, radius, torch.zeros_like(radius)).int()
    det_s = torch.where(vis, det, torch.ones_like(det))
    ca, cb, cc = c / det_s, -b / det_s, a / det_s
    d = means3D - campos
    d = d / d.norm(dim=1, keepdim=True)
    rgb = torch.clamp_min(_sh(sh_degree, shs, d) + 0.5, 0.0)
    invz = 1.0 / tz

    # ---- duplicate with keys, sort, tile ranges ----
    with torch.no_grad():
        ids = torch.nonzero(vis).squeeze(1)
        n = touched[ids].long()
        gid = torch.repeat_interleave(ids, n)
        first = torch.repeat_interleave(torch.cumsum(n, 0) - n, n)
        local = torch.arange(gid.numel()) - first
        w = (x1 - x0)[gid].long()
        tile = (y0[gid].long() + local // w) * gx + x0[gid].long() + local % w
        dbits = tz.detach().contiguous().view(torch.int32)[gid].long() & 0xFFFFFFFF
        order = torch.sort((tile << 32) | dbits, stable=True).indices
        plist = gid[order]
        counts = torch.bincount(tile, minlength=gx * gy)
        ends = torch.cumsum(counts, 0)

    # ---- per-tile blend ----
    lx = torch.arange(TILE, dtype=torch.float32).repeat(TILE)
    ly = torch.arange(TILE, dtype=torch.float32).repeat_interleave(TILE)
    cols, deps = [], []
    bgc = bg.reshape(3)
    for tt in range(gx * gy):
        e = int(ends[tt])
        g = plist[e - int(counts[tt]):e]
        px = (tt % gx) * TILE + lx
        py = (tt // gx) * TILE + ly
        if g.numel() == 0:
            cols.append(bgc[None, :].expand(TILE * TILE, 3))
            deps.append(torch.zeros(TILE * TILE))
            continue
        dx = xy[g, 0][None, :] - px[:, None]
        dy = xy[g, 1][None, :] - py[:, None]
        power = -0.5 * (ca[g][None] * dx * dx + cc[g][None] * dy * dy) - cb[g][None] * dx * dy
        oG = opacities[g, 0][None] * torch.exp(power)
        alpha = oG - torch.clamp_min(oG - 0.99, 0.0).detach()
        alpha = alpha * ((power <= 0) & (alpha >= 1.0 / 255.0)).float()
        one_m = 1.0 - alpha
        Tinc = torch.cumprod(one_m, 1)
        keep = (Tinc >= 1e-4).float()
        Tex = torch.cat([torch.ones(TILE * TILE, 1), Tinc[:, :-1]], 1)
        wgt = alpha * Tex * keep
        Tfin = torch.cumprod(one_m * keep + (1.0 - keep), 1)[:, -1]
        cols.append(wgt @ rgb[g] + Tfin[:, None] * bgc[None, :])
        deps.append(wgt @ invz[g])
    col = torch.stack(cols).reshape(gy, gx, TILE, TILE, 3).permute(4, 0, 2, 1, 3).reshape(3, gy * TILE, gx * TILE)
    dep = torch.stack(deps).reshape(gy, gx, TILE, TILE).permute(0, 2, 1, 3).reshape(1, gy * TILE, gx * TILE)
    return col[:, :H, :W], dep[:, :H, :W], radii


def scene_tensors(s, requires_grad=True):
    """torch CPU leaves + camera tensors from a gs_oracle.synthetic_scene dict."""
    f = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32)
    leaves = {k: f(s[k]).requires_grad_(requires_grad) for k in ("means3D", "scales", "rotations", "opacities", "shs")}
    cam = dict(view=f(s["view"]), proj=f(s["proj"]), campos=f(s["campos"]), bg=f(s["bg"]), W=int(s["W"]),
               H=int(s["H"]), tanfovx=float(s["tanfovx"]), tanfovy=float(s["tanfovy"]),
               sh_degree=int(s["sh_degree"]))
    return leaves, cam


def fwd_bwd(s, dcol, dinv):
    """One forward + autograd backward of scene dict `s`; returns (color, invdepth, radii, grads)."""
    leaves, cam = scene_tensors(s)
    color, invd, radii = render(**leaves, **cam)
    loss = (color * torch.as_tensor(dcol)).sum() + (invd * torch.as_tensor(dinv)).sum()
    loss.backward()
    return color.detach(), invd.detach(), radii, {k: v.grad for k, v in leaves.items()}


def time_fwd_bwd(s, dcol, dinv, min_seconds=2.0, max_frames=20):
    """Frames of fwd+bwd until ~min_seconds: (Mpix/s, frames, seconds, threads)."""
    frames = 0
    t0 = time.perf_counter()
    while frames < max_frames and (frames == 0 or time.perf_counter() - t0 < min_seconds):
        fwd_bwd(s, dcol, dinv)
        frames += 1
    dt = time.perf_counter() - t0
    return s["W"] * s["H"] * frames / dt / 1e6, frames, dt, torch.get_num_threads()
