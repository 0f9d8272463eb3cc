"""Python driver for the CPU oracle (oracle/gs_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package (street-sparse-3dgs_amd/).

`forward()` / `backward()` chain the C restatement's stages exactly as the upstream
rasterizer chains its kernels and return every
intermediate (radii, keys, sorted point list, tile ranges, n_contrib, ...) so tests can
compare the HIP path bit-exactly on integer outputs.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "gs_oracle.c")
LIB = os.path.join(HERE, "build", "libgs_oracle.so")
BLOCK = 16

_lib = None


def build(force: bool = False) -> str:
    """Compile the C restatement with gcc (fp-contract off, OpenMP for the CPU baseline)."""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        cmd = ["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
               "-fopenmp", SRC, "-o", LIB + ".tmp", "-lm"]
        subprocess.check_call(cmd)
        os.replace(LIB + ".tmp", LIB)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.gso_scan.restype = ctypes.c_ulonglong
        _lib.gso_num_threads.restype = ctypes.c_int
    return _lib


def _p(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    if a is None:
        return None
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def num_threads() -> int:
    return int(lib().gso_num_threads())


def forward(means3D, opacities, view, proj, campos, bg, W, H, tanfovx, tanfovy, sh_degree=0,
            shs=None, colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
            scale_modifier=1.0, do_depth=True):
    """Full forward.  Arrays are numpy (any float dtype; cast to fp32).  Returns a dict."""
    L = lib()
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    opacities = _f32(opacities).reshape(P)
    view = _f32(view).reshape(16)
    proj = _f32(proj).reshape(16)
    campos = _f32(campos).reshape(3)
    bg = _f32(bg).reshape(3)
    shs = _f32(shs)
    M = 0 if shs is None or shs.size == 0 else shs.reshape(P, -1, 3).shape[1]
    if M == 0:
        shs = None
    colors_precomp = _f32(colors_precomp)
    if colors_precomp is not None and colors_precomp.size == 0:
        colors_precomp = None
    cov3D_precomp = _f32(cov3D_precomp)
    if cov3D_precomp is not None and cov3D_precomp.size == 0:
        cov3D_precomp = None
    scales = _f32(scales)
    rotations = _f32(rotations)
    tx = np.float32(tanfovx)
    ty = np.float32(tanfovy)
    gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
    T = gx * gy
    radii = np.zeros(P, np.int32)
    depths = np.zeros(P, np.float32)
    xy = np.zeros((P, 2), np.float32)
    conic = np.zeros((P, 4), np.float32)
    rgb = np.zeros((P, 3), np.float32)
    clamped = np.zeros((P, 3), np.uint8)
    cov3D = np.zeros((P, 6), np.float32)
    tiles = np.zeros(P, np.uint32)
    L.gso_preprocess(ctypes.c_int(P), ctypes.c_int(sh_degree), ctypes.c_int(M), _p(means3D), _p(scales),
                     ctypes.c_float(scale_modifier), _p(rotations), _p(opacities), _p(shs), _p(colors_precomp),
                     _p(cov3D_precomp), _p(view), _p(proj), _p(campos), ctypes.c_int(W), ctypes.c_int(H),
                     ctypes.c_float(tx), ctypes.c_float(ty), _p(radii), _p(depths), _p(xy), _p(conic), _p(rgb),
                     _p(clamped), _p(cov3D), _p(tiles))
    offsets = np.zeros(P, np.uint32)
    K = int(L.gso_scan(ctypes.c_int(P), _p(tiles), _p(offsets)))
    keys = np.zeros(max(K, 1), np.uint64)
    vals = np.zeros(max(K, 1), np.uint32)
    L.gso_duplicate(ctypes.c_int(P), _p(xy), _p(radii), _p(depths), _p(offsets), ctypes.c_int(W), ctypes.c_int(H),
                    _p(keys), _p(vals))
    keys_unsorted, vals_unsorted = keys[:K].copy(), vals[:K].copy()
    L.gso_sort(ctypes.c_ulonglong(K), _p(keys), _p(vals))
    ranges = np.zeros((T, 2), np.uint32)
    L.gso_ranges(ctypes.c_ulonglong(K), _p(keys), ctypes.c_int(T), _p(ranges))
    color = np.zeros((3, H, W), np.float32)
    invdepth = np.zeros((1, H, W), np.float32)
    final_T = np.zeros((H, W), np.float32)
    n_contrib = np.zeros((H, W), np.uint32)
    L.gso_render_fwd(ctypes.c_int(W), ctypes.c_int(H), _p(ranges), _p(vals), _p(xy), _p(conic), _p(rgb), _p(depths),
                     _p(bg), ctypes.c_int(1 if do_depth else 0), _p(color), _p(invdepth), _p(final_T), _p(n_contrib))
    return dict(
        P=P, M=M, K=K, W=W, H=H, T=T, sh_degree=sh_degree, tanfovx=tx, tanfovy=ty, scale_modifier=scale_modifier,
        do_depth=do_depth, means3D=means3D, opacities=opacities, view=view, proj=proj, campos=campos, bg=bg,
        shs=shs, colors_precomp=colors_precomp, cov3D_precomp=cov3D_precomp, scales=scales, rotations=rotations,
        radii=radii, depths=depths, xy=xy, conic_opacity=conic, rgb=rgb, clamped=clamped, cov3D=cov3D,
        tiles_touched=tiles, offsets=offsets, keys_unsorted=keys_unsorted, vals_unsorted=vals_unsorted,
        keys=keys[:K], point_list=vals[:K], ranges=ranges, color=color, invdepth=invdepth, final_T=final_T,
        n_contrib=n_contrib)


def backward(st, dL_dcolor, dL_dinvdepth=None, true_scale_grad=False):
    """Backward from a forward() state.  Returns grads named as the _C backward returns them.

    dL/dscales follows upstream by default: the gradient with respect to the modified scale
    (scale_modifier * s), reported as dL/ds.  true_scale_grad=True multiplies in scale_modifier
    (the exact derivative; what fp64 autograd in dense_torch.py computes)."""
    L = lib()
    P, M, K, W, H = st["P"], st["M"], st["K"], st["W"], st["H"]
    dL_dcolor = _f32(dL_dcolor).reshape(3, H, W)
    dinv = None
    if st["do_depth"] and dL_dinvdepth is not None:
        dinv = _f32(dL_dinvdepth).reshape(H, W)
    inst = np.zeros((max(K, 1), 10), np.float32)
    L.gso_render_bwd(ctypes.c_int(W), ctypes.c_int(H), _p(st["ranges"]), _p(st["point_list"]), _p(st["xy"]),
                     _p(st["conic_opacity"]), _p(st["rgb"]), _p(st["depths"]), _p(st["bg"]), _p(st["final_T"]),
                     _p(st["n_contrib"]), _p(dL_dcolor), _p(dinv), _p(inst))
    g10 = np.zeros((P, 10), np.float32)
    L.gso_reduce_instances(ctypes.c_int(P), ctypes.c_ulonglong(K), _p(st["point_list"]), _p(inst), _p(g10))
    has_shs = st["shs"] is not None
    has_scales = st["cov3D_precomp"] is None
    dm3 = np.zeros((P, 3), np.float32)
    dm2 = np.zeros((P, 3), np.float32)
    dcol = np.zeros((P, 3), np.float32)
    dop = np.zeros((P, 1), np.float32)
    dcov = np.zeros((P, 6), np.float32)
    dsh = np.zeros((P, max(M, 1), 3), np.float32)
    dsc = np.zeros((P, 3), np.float32)
    drot = np.zeros((P, 4), np.float32)
    L.gso_preprocess_bwd(ctypes.c_int(P), ctypes.c_int(st["sh_degree"]), ctypes.c_int(M), _p(st["means3D"]),
                         _p(st["radii"]), _p(st["shs"]), _p(st["clamped"]), _p(st["scales"]), _p(st["rotations"]),
                         ctypes.c_float(st["scale_modifier"]), _p(st["cov3D"]), _p(st["view"]), _p(st["proj"]),
                         _p(st["campos"]), ctypes.c_int(W), ctypes.c_int(H), ctypes.c_float(st["tanfovx"]),
                         ctypes.c_float(st["tanfovy"]), _p(g10), ctypes.c_int(int(has_shs)),
                         ctypes.c_int(int(has_scales)), ctypes.c_int(int(true_scale_grad)), _p(dm3), _p(dm2), _p(dcol), _p(dop), _p(dcov), _p(dsh),
                         _p(dsc), _p(drot))
    return dict(dL_dmeans3D=dm3, dL_dmeans2D=dm2, dL_dcolors=dcol, dL_dopacity=dop, dL_dcov3D=dcov,
                dL_dsh=dsh if has_shs else np.zeros((0,), np.float32), dL_dscales=dsc, dL_drotations=drot,
                inst=inst[:K], g10=g10)


def expand_to_size(nodes, boxes, target, viewpoint):
    """C restatement of gaussian_hierarchy expand_to_size -> (render_indices, parent_indices,
    nodes_for_render_indices), each int32 of the cut's length."""
    nodes = np.ascontiguousarray(nodes, np.int32).reshape(-1, 7)
    boxes = _f32(boxes).reshape(-1, 8)
    N = nodes.shape[0]
    cap = int(nodes[:, 3].astype(np.int64).sum() + nodes[:, 4].astype(np.int64).sum())
    ri, pi, ni = (np.zeros(max(cap, 1), np.int32) for _ in range(3))
    L = lib()
    L.gso_expand_to_size.restype = ctypes.c_longlong
    n = L.gso_expand_to_size(ctypes.c_longlong(N), _p(nodes), _p(boxes), ctypes.c_float(target),
                             _p(_f32(viewpoint).reshape(3)), _p(ri), _p(pi), _p(ni))
    return ri[:n].copy(), pi[:n].copy(), ni[:n].copy()


def interpolation_weights(node_indices, target, nodes, boxes, viewpoint):
    """C restatement of gaussian_hierarchy get_interpolation_weights -> (weights f32, num_kids i32)."""
    node_indices = np.ascontiguousarray(node_indices, np.int32)
    n = node_indices.shape[0]
    w = np.zeros(max(n, 1), np.float32)
    k = np.zeros(max(n, 1), np.int32)
    lib().gso_interpolation_weights(ctypes.c_longlong(n), _p(node_indices), ctypes.c_float(target),
                                    _p(np.ascontiguousarray(nodes, np.int32)), _p(_f32(boxes)),
                                    _p(_f32(viewpoint).reshape(3)), _p(w), _p(k))
    return w[:n], k[:n]


class upstream_exponent:
    """Context manager: the oracle's render fwd/bwd evaluate the Gaussian as upstream writes it
    (power = -0.5 (a dx^2 + c dy^2) - b dx dy, expf) instead of the kernels' exp2 order."""

    def __enter__(self):
        lib().gso_set_upstream_exponent(ctypes.c_int(1))
        return self

    def __exit__(self, *exc):
        lib().gso_set_upstream_exponent(ctypes.c_int(0))
        return False


def mark_visible(means3D, view, proj):
    L = lib()
    means3D = _f32(means3D).reshape(-1, 3)
    out = np.zeros(means3D.shape[0], np.uint8)
    L.gso_mark_visible(ctypes.c_int(means3D.shape[0]), _p(means3D), _p(_f32(view).reshape(16)),
                       _p(_f32(proj).reshape(16)), _p(out))
    return out.astype(bool)


# -----------------------------------------------------------------------------------------
# Camera helpers (restating utils/graphics_utils.py:38-83 and scene/cameras.py:96-99)
# -----------------------------------------------------------------------------------------
def projection_matrix(znear, zfar, fovX, fovY, primx=0.5, primy=0.5):
    """utils/graphics_utils.py:51-77 (row-major P, not transposed)."""
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
    """Returns (viewmatrix, projmatrix, campos, tanfovx, tanfovy) in the rasterizer's
    convention: viewmatrix = W2C^T, projmatrix = (P W2C)^T as row-major fp32 arrays
    (scene/cameras.py:96-99)."""
    fovx = math.radians(fovx_deg)
    fx = W / (2 * math.tan(fovx / 2))
    fovy = 2 * math.atan(H / (2 * fx))
    R = np.eye(3) if R is None else np.asarray(R, np.float64)
    t = np.zeros(3) if t is None else np.asarray(t, np.float64)
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.T
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    w2c = Rt.astype(np.float32)
    view = w2c.T.copy()
    Pm = projection_matrix(znear, zfar, fovx, fovy, primx, primy)
    proj = (view.astype(np.float32) @ Pm.T.astype(np.float32)).astype(np.float32)
    campos = np.linalg.inv(view.astype(np.float64))[3, :3].astype(np.float32)
    return view, proj, campos, math.tan(fovx * 0.5), math.tan(fovy * 0.5)


def camera_from(W, H, R, T, FoVx, FoVy, primx=0.5, primy=0.5, znear=0.01, zfar=100.0):
    """scene/cameras.py:96-99 restated: (viewmatrix, projmatrix, campos, tanfovx, tanfovy)
    for a COLMAP-style camera (R = camera-to-world rotation as stored by the reference, T =
    world-to-camera translation)."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = np.asarray(R, np.float64).T
    Rt[:3, 3] = T
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    Rt = np.linalg.inv(C2W)  # getWorld2View2 round trip (trans = 0, scale = 1)
    view = np.float32(Rt).T.copy()
    Pm = projection_matrix(znear, zfar, FoVx, FoVy, primx, primy)
    proj = (view.astype(np.float32) @ Pm.T.astype(np.float32)).astype(np.float32)
    campos = np.linalg.inv(view.astype(np.float64))[3, :3].astype(np.float32)
    return view, proj, campos, math.tan(FoVx * 0.5), math.tan(FoVy * 0.5)


def eval_sh(deg, shs, dirs):
    """C restatement of the SH colour (utils/sh_utils.py:57-112 + the +0.5 / clamp_min(0) of
    gaussian_renderer/__init__.py:89): shs (n, M, 3), dirs (n, 3) -> rgb (n, 3), clamped."""
    shs = _f32(shs)
    n, M = shs.shape[0], shs.shape[1]
    dirs = _f32(dirs).reshape(n, 3)
    rgb = np.zeros((n, 3), np.float32)
    cl = np.zeros((n, 3), np.uint8)
    lib().gso_eval_sh(ctypes.c_int(n), ctypes.c_int(deg), ctypes.c_int(M), _p(shs), _p(dirs), _p(rgb), _p(cl))
    return rgb, cl.astype(bool)


def cov3d(scales, rotations, scale_modifier=1.0):
    """C restatement of cov3D = (R S)(R S)^T as 6 floats (scene/gaussian_model.py:33-37)."""
    scales = _f32(scales).reshape(-1, 3)
    rotations = _f32(rotations).reshape(-1, 4)
    out = np.zeros((scales.shape[0], 6), np.float32)
    lib().gso_cov3d(ctypes.c_int(scales.shape[0]), _p(scales), ctypes.c_float(scale_modifier), _p(rotations),
                    _p(out))
    return out


def synthetic_scene(P, W, H, seed=0, sh_degree=3, fovx_deg=60.0, zmin=2.0, zmax=20.0, log_scale_mean=-4.0,
                    log_scale_std=0.5, primx=0.5, primy=0.5):
    """Seeded synthetic Gaussians as SURVEY.md section 8(d) defines them."""
    rng = np.random.default_rng(seed)
    view, proj, campos, tx, ty = camera(W, H, fovx_deg, primx=primx, primy=primy)
    z = rng.uniform(zmin, zmax, P)
    x = rng.uniform(-0.95, 0.95, P) * tx * z
    y = rng.uniform(-0.95, 0.95, P) * ty * z
    means = np.stack([x, y, z], 1).astype(np.float32)
    scales = np.exp(rng.normal(log_scale_mean, log_scale_std, (P, 3))).astype(np.float32)
    q = rng.normal(size=(P, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    rots = q.astype(np.float32)
    opac = rng.uniform(0.05, 0.99, (P, 1)).astype(np.float32)
    M = (sh_degree + 1) ** 2 if sh_degree >= 0 else 1
    M = max(M, 1)
    shs = np.zeros((P, 16 if sh_degree == 3 else M, 3), np.float32)
    shs[:, 0, :] = rng.normal(0, 0.5, (P, 3))
    shs[:, 1:, :] = rng.normal(0, 0.05, (P, shs.shape[1] - 1, 3))
    bg = rng.uniform(0, 1, 3).astype(np.float32)
    return dict(means3D=means, scales=scales, rotations=rots, opacities=opac, shs=shs.astype(np.float32),
                view=view, proj=proj, campos=campos, tanfovx=tx, tanfovy=ty, bg=bg, W=W, H=H,
                sh_degree=sh_degree)


def knn_mean_dist2(points) -> np.ndarray:
    """simple_knn distCUDA2 restated (gso_knn_mean_dist2): exact brute force, parity unpinned
    against the real extension (not vendored; see gs_oracle.c)."""
    p = _f32(points).reshape(-1, 3)
    out = np.empty(p.shape[0], np.float32)
    lib().gso_knn_mean_dist2(ctypes.c_longlong(p.shape[0]), _p(p), _p(out))
    return out


def knn_mean_dist2_at(points, queries) -> np.ndarray:
    """knn_mean_dist2 for the given query indices only (all N points are candidates)."""
    p = _f32(points).reshape(-1, 3)
    q = np.ascontiguousarray(np.asarray(queries, dtype=np.int64))
    out = np.empty(q.shape[0], np.float32)
    lib().gso_knn_mean_dist2_at(ctypes.c_longlong(p.shape[0]), _p(p), ctypes.c_longlong(q.shape[0]), _p(q), _p(out))
    return out
