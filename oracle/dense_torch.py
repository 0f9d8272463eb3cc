"""Dense fp64 autograd restatement of the rasterizer -- cross-checks the hand-derived
backward of oracle/gs_oracle.c (and through it the HIP kernels).

TEST INFRASTRUCTURE ONLY (see oracle/gs_oracle.py).

The discrete decisions of the tile renderer -- which Gaussians are visible (radii > 0),
each tile's depth-sorted instance list, each pixel's last contributor (n_contrib) and the
alpha < 1/255 / power > 0 skips -- are taken from the fp32 oracle forward; everything
continuous is recomputed here in float64 and differentiated by torch.autograd.  Two
upstream conventions are reproduced on purpose:
  * alpha = min(0.99, o*G) passes the gradient straight through the clamp;
  * the 1.3*tanfov clamp of the view-space mean zeroes d/dtx (d/dty) when active and keeps
    the clamped value fixed in d/dtz.
Small problems only (pure-Python loop over tiles).
"""
from __future__ import annotations

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def eval_sh_t(deg, sh, dirs):
    """sh: (P, M, 3) coefficient-major; dirs: (P, 3) unit.  utils/sh_utils.py:57-112."""
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
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


def quat_to_R(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)
    return R


def _mask_fp32(st, pix_x, pix_y, gids):
    """fp32 replica of the renderer's skip test for pixel coordinate arrays x gaussian ids."""
    xy = st["xy"][gids]
    co = st["conic_opacity"][gids]
    dx = (xy[None, :, 0] - pix_x[:, None].astype(np.float32)).astype(np.float32)
    dy = (xy[None, :, 1] - pix_y[:, None].astype(np.float32)).astype(np.float32)
    a, b, c, o = (co[None, :, k] for k in range(4))
    power = np.float32(-0.5) * (a * dx * dx + c * dy * dy) - b * dx * dy
    alpha = np.minimum(np.float32(0.99), o * np.exp(power))
    return (power <= 0) & (alpha >= np.float32(1.0 / 255.0))


def dense_grads(st, dL_dcolor, dL_dinvdepth=None):
    dt = torch.float64
    P, W, H = st["P"], st["W"], st["H"]
    V = torch.tensor(st["view"].reshape(4, 4), dtype=dt)
    Pm = torch.tensor(st["proj"].reshape(4, 4), dtype=dt)
    campos = torch.tensor(st["campos"], dtype=dt)
    bg = torch.tensor(st["bg"], dtype=dt)
    mod = float(st["scale_modifier"])
    tanx, tany = float(st["tanfovx"]), float(st["tanfovy"])
    fx = W / (2.0 * tanx)
    fy = H / (2.0 * tany)

    means = torch.tensor(st["means3D"], dtype=dt, requires_grad=True)
    opac = torch.tensor(st["opacities"].reshape(P, 1), dtype=dt, requires_grad=True)
    leaves = {"means3D": means, "opacities": opac}
    if st["cov3D_precomp"] is None:
        scales = torch.tensor(st["scales"], dtype=dt, requires_grad=True)
        rots = torch.tensor(st["rotations"], dtype=dt, requires_grad=True)
        leaves.update(scales=scales, rotations=rots)
        Lm = quat_to_R(rots) * (mod * scales)[:, None, :]
        S3 = Lm @ Lm.transpose(1, 2)
    else:
        c6 = torch.tensor(st["cov3D_precomp"], dtype=dt, requires_grad=True)
        leaves.update(cov3D=c6)
        S3 = torch.stack([torch.stack([c6[:, 0], c6[:, 1], c6[:, 2]], -1),
                          torch.stack([c6[:, 1], c6[:, 3], c6[:, 4]], -1),
                          torch.stack([c6[:, 2], c6[:, 4], c6[:, 5]], -1)], -2)
    if st["shs"] is None:
        cp = torch.tensor(st["colors_precomp"], dtype=dt, requires_grad=True)
        leaves.update(colors=cp)
        rgb = cp
    else:
        sh = torch.tensor(st["shs"], dtype=dt, requires_grad=True)
        leaves.update(shs=sh)
        d = means - campos
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(eval_sh_t(st["sh_degree"], sh, d) + 0.5, 0.0)

    t = means @ V[:3, :3] + V[3, :3]
    ph = means @ Pm[:3, :] + Pm[3, :]
    pw = 1.0 / (ph[:, 3] + 1e-7)
    ndc = ph[:, :2] * pw[:, None]
    ndc.retain_grad()
    xy = torch.stack([((ndc[:, 0] + 1) * W - 1) * 0.5, ((ndc[:, 1] + 1) * H - 1) * 0.5], 1)

    limx, limy = 1.3 * tanx, 1.3 * tany
    tx, ty, tz = t[:, 0], t[:, 1], t[:, 2]
    txtz, tytz = tx / tz, ty / tz
    cx = (txtz < -limx) | (txtz > limx)
    cy = (tytz < -limy) | (tytz > limy)
    txc = torch.where(cx, (torch.sign(txtz) * limx * tz).detach(), tx)
    tyc = torch.where(cy, (torch.sign(tytz) * limy * tz).detach(), ty)
    Wr = V[:3, :3].T  # Wr[r] = view rotation row r
    j00, j02 = fx / tz, -(fx * txc) / (tz * tz)
    j11, j12 = fy / tz, -(fy * tyc) / (tz * tz)
    m0 = j00[:, None] * Wr[0] + j02[:, None] * Wr[2]
    m1 = j11[:, None] * Wr[1] + j12[:, None] * Wr[2]
    A = torch.einsum("pi,pij,pj->p", m0, S3, m0) + 0.3
    B = torch.einsum("pi,pij,pj->p", m0, S3, m1)
    C = torch.einsum("pi,pij,pj->p", m1, S3, m1) + 0.3
    det = A * C - B * B
    ca, cb, cc = C / det, -B / det, A / det
    invd = 1.0 / t[:, 2]

    img = torch.zeros(3, H, W, dtype=dt)
    dimg = torch.zeros(H, W, dtype=dt)
    gx = (W + 15) // 16
    ranges, plist, ncon = st["ranges"], st["point_list"], st["n_contrib"]
    img_rows, dimg_rows = [], []
    for tile in range(st["T"]):
        tx0, ty0 = (tile % gx) * 16, (tile // gx) * 16
        xs = np.arange(tx0, min(tx0 + 16, W))
        ys = np.arange(ty0, min(ty0 + 16, H))
        if len(xs) == 0 or len(ys) == 0:
            continue
        PX, PY = np.meshgrid(xs, ys)
        PX, PY = PX.ravel(), PY.ravel()
        r0, r1 = int(ranges[tile, 0]), int(ranges[tile, 1])
        gids = plist[r0:r1].astype(np.int64)
        n = ncon[PY, PX].astype(np.int64)
        if len(gids) == 0:
            col = bg[:, None].expand(3, len(PX))
            img_rows.append((PY, PX, col))
            dimg_rows.append((PY, PX, torch.zeros(len(PX), dtype=dt)))
            continue
        mask = _mask_fp32(st, PX, PY, gids) & (np.arange(len(gids))[None, :] < n[:, None])
        mk = torch.tensor(mask, dtype=dt)
        g = torch.as_tensor(gids)
        dx = xy[g, 0][None, :] - torch.tensor(PX, dtype=dt)[:, None]
        dy = xy[g, 1][None, :] - torch.tensor(PY, dtype=dt)[:, None]
        power = -0.5 * (ca[g][None] * dx * dx + cc[g][None] * dy * dy) - cb[g][None] * dx * dy
        oG = opac[g, 0][None] * torch.exp(power)
        alpha = oG - torch.clamp_min(oG - 0.99, 0.0).detach()
        alpha = alpha * mk
        one_m = 1 - alpha
        Tcum = torch.cumprod(torch.cat([torch.ones(len(PX), 1, dtype=dt), one_m], 1), 1)
        Tex = Tcum[:, :-1]
        Tfin = Tcum[:, -1]
        w = alpha * Tex
        col = (w @ rgb[g]).T + Tfin[None] * bg[:, None]
        dep = w @ invd[g]
        img_rows.append((PY, PX, col))
        dimg_rows.append((PY, PX, dep))
    for PY, PX, col in img_rows:
        img = img.index_put((torch.arange(3)[:, None], torch.as_tensor(PY)[None], torch.as_tensor(PX)[None]), col)
    for PY, PX, dep in dimg_rows:
        dimg = dimg.index_put((torch.as_tensor(PY), torch.as_tensor(PX)), dep)
    loss = (img * torch.tensor(np.asarray(dL_dcolor, np.float64).reshape(3, H, W))).sum()
    if st["do_depth"] and dL_dinvdepth is not None:
        loss = loss + (dimg * torch.tensor(np.asarray(dL_dinvdepth, np.float64).reshape(H, W))).sum()
    loss.backward()
    vis = torch.tensor(st["radii"] > 0)
    out = {"color": img.detach().numpy(), "invdepth": dimg.detach().numpy()[None]}
    for k, v in leaves.items():
        gr = v.grad if v.grad is not None else torch.zeros_like(v)
        gr = gr * vis.reshape(-1, *([1] * (gr.dim() - 1)))
        out["dL_d" + k] = gr.numpy()
    dm2 = torch.zeros(P, 3, dtype=dt)
    dm2[:, :2] = ndc.grad * vis[:, None]
    out["dL_dmeans2D"] = dm2.numpy()
    return out
