"""Shared test helpers: scene construction, running the HIP path through the public API, and
decoding the scratch buffers (GeomState / BinningState / ImageState carve order of
csrc/rasterizer.hip) so integer intermediates can be compared bit-exactly with the oracle."""
from __future__ import annotations

import contextlib

import math

import numpy as np

ALIGN = 256


def _align(x):
    return (x + ALIGN - 1) // ALIGN * ALIGN


def carve(sizes):
    """sizes: list of (name, nbytes) in carve order -> {name: (offset, nbytes)}."""
    off, out = 0, {}
    for name, nb in sizes:
        off = _align(off)
        out[name] = (off, nb)
        off += nb
    return out


def geom_layout(P):
    return carve([("rec", 64 * P), ("tiles", 4 * P), ("dkey", 4 * P), ("dkey_sorted", 4 * P), ("ids", 4 * P),
                  ("order", 4 * P), ("offsets", 4 * P), ("clamped", P)])


def binning_layout(K, T):
    # point_list first (csrc/rasterizer.hip carve_binning): the forward may carve a larger capacity
    return carve([("point_list", 4 * K), ("sblist", 16 * K)])


def image_layout(T, npix):
    return carve([("ranges", 8 * T), ("boundary", 8 * T), ("final_T", 4 * npix), ("n_contrib", 4 * npix),
                  ("tile_work", 4 * T), ("tile_ids", 4 * T), ("tile_order", 4 * T)])


def view(buf_np, layout, name, dtype, shape=None):
    off, nb = layout[name]
    a = buf_np[off:off + nb].view(dtype)
    return a if shape is None else a.reshape(shape)


def decode_state(geom, binning, image, P, K, W, H):
    """Decode the HIP scratch state.  The HIP binning lays tiles out superblock-major
    (binning.hip); `point_list` / `ranges` / `keys` are re-expressed in upstream's row-major tile
    order (each tile's list unchanged) so they compare bit-exactly with the oracle, and the raw
    layout is returned as `ranges_raw` / `point_list_raw`."""
    g = geom.cpu().numpy()
    b = binning.cpu().numpy()
    im = image.cpu().numpy()
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    gl, bl = geom_layout(P), binning_layout(K, T)
    il = image_layout(T, W * H)
    rec = view(g, gl, "rec", np.float32, (P, 16))
    pl_raw = view(b, bl, "point_list", np.uint32)
    r_raw = view(im, il, "ranges", np.uint32, (T, 2))
    lens = (r_raw[:, 1].astype(np.int64) - r_raw[:, 0].astype(np.int64))
    point_list = np.concatenate([pl_raw[r_raw[t, 0]:r_raw[t, 1]] for t in range(T)]) if K > 0 else \
        np.zeros(0, np.uint32)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint32)
    ranges = np.zeros((T, 2), np.uint32)
    nz = lens > 0
    ranges[nz, 0] = starts[nz]
    ranges[nz, 1] = starts[nz] + lens[nz].astype(np.uint32)
    dbits = rec[:, 14].view(np.uint32)
    tile_of = np.repeat(np.arange(T, dtype=np.uint64), np.maximum(lens, 0))
    # the 64-bit (tile << 32 | depth bits) keys upstream sorts, rebuilt from the per-tile lists
    keys = (tile_of << np.uint64(32)) | dbits[point_list].astype(np.uint64)
    return dict(
        rec=rec, depths=dbits.view(np.float32).copy(), xy=rec[:, 0:2], conic_opacity=rec[:, 2:6],
        rgbd=rec[:, 8:12], tiles_touched=view(g, gl, "tiles", np.uint32), offsets=view(g, gl, "offsets", np.uint32),
        order=view(g, gl, "order", np.uint32), clamped=view(g, gl, "clamped", np.uint8),
        keys=keys, point_list=point_list, ranges=ranges, ranges_raw=r_raw, point_list_raw=pl_raw,
        final_T=view(im, il, "final_T", np.float32, (H, W)), n_contrib=view(im, il, "n_contrib", np.uint32, (H, W)))


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def psnr(a, b, peak=1.0):
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    return float("inf") if mse == 0 else 10 * math.log10(peak * peak / mse)


def torch_inputs(scene, device, sh_degree=None, use_precomp_colors=False, use_precomp_cov=False,
                 requires_grad=True, colors_precomp=None, cov3D_precomp=None):
    """numpy synthetic scene (oracle.gs_oracle.synthetic_scene) -> torch tensors on device."""
    import torch
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=device)
    P = scene["means3D"].shape[0]
    d = dict(means3D=t(scene["means3D"]), opacities=t(scene["opacities"]).reshape(P, 1),
             means2D=torch.zeros(P, 3, device=device))
    if use_precomp_colors:
        d["colors_precomp"] = t(colors_precomp)
    else:
        d["shs"] = t(scene["shs"])
    if use_precomp_cov:
        d["cov3D_precomp"] = t(cov3D_precomp)
    else:
        d["scales"] = t(scene["scales"])
        d["rotations"] = t(scene["rotations"])
    if requires_grad:
        for k, v in d.items():
            v.requires_grad_(True)
    return d


def settings(scene, device, sh_degree, scale_modifier=1.0, do_depth=True, debug=False, bg=None):
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=device)
    return GaussianRasterizationSettings(
        image_height=int(scene["H"]), image_width=int(scene["W"]), tanfovx=float(scene["tanfovx"]),
        tanfovy=float(scene["tanfovy"]), bg=t(scene["bg"] if bg is None else bg), scale_modifier=scale_modifier,
        viewmatrix=t(scene["view"]).reshape(4, 4), projmatrix=t(scene["proj"]).reshape(4, 4), sh_degree=sh_degree,
        campos=t(scene["campos"]), prefiltered=False, debug=debug, do_depth=do_depth,
        render_indices=torch.empty(0, dtype=torch.int32), parent_indices=torch.empty(0, dtype=torch.int32),
        interpolation_weights=torch.empty(0, dtype=torch.float32, device=device),
        num_node_kids=torch.empty(0, dtype=torch.int32, device=device))


@contextlib.contextmanager
def deterministic():
    """Backward in the record mode (gsr_set_deterministic(1)): bitwise reproducible gradients, for
    tests that compare two runs bit for bit; the default atomic mode differs in summation order."""
    from diff_gaussian_rasterization import _C
    prev = _C.set_deterministic(True)
    try:
        yield
    finally:
        _C.set_deterministic(prev)


def record_margins(name, **values):
    """Observed parity margins of a GPU test (PSNR, n_contrib mismatch, gradient errors), appended as
    one JSON line to $GSR_PARITY_RECORD when set: the bars in the tests are set from these
    (profiles/r04_parity_margins.jsonl)."""
    import json
    import os
    path = os.environ.get("GSR_PARITY_RECORD")
    if not path:
        return
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(dict(case=name, **{k: (float(v) if v is not None else None) for k, v in values.items()}))
                + "\n")


def assert_adam_trajectories_close(name, x, y, x0, lr, steps, atol, frac=0.999, margin=1.1):
    """Two trajectories of one parameter under Adam from the same start x0 (a fused step and the
    reference's formulation), after `steps` updates of learning rate <= lr (a number, or a tensor
    broadcastable to x for per-column rates).

    Every element: |x - y| <= 2 * margin * lr * steps + atol.  Each side's Adam update of an element
    is at most ~lr in magnitude per step over these few steps (|m_hat / sqrt(v_hat)| <= 1 for
    consistent gradients, less otherwise), so even an element whose near-zero gradient flipped sign
    in fp32 on one side ends within twice the travel; anything further off is an indexing or
    arithmetic error, not rounding.  The bulk (>= frac of the elements) agrees within atol.
    Returns the measured margins (max |x - y| over the travel bound, the close fraction)."""
    import torch
    x, y, x0 = x.detach(), y.detach(), x0.detach()
    d = (x - y).abs()
    travel = torch.as_tensor(lr, dtype=d.dtype, device=d.device) * float(steps)
    bound = 2.0 * margin * travel + atol
    over = d > bound
    assert not bool(over.any()), (name, "elements beyond the Adam travel bound", int(over.sum()),
                                  float((d - bound).max()))
    close = float(torch.isclose(x, y, rtol=0, atol=atol).float().mean())
    assert close >= frac, (name, close)
    assert not torch.equal(x, x0), (name, "did not move")
    return float((d / (2.0 * travel).clamp_min(1e-30)).max()), close
