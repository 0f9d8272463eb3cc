"""`diff_gaussian_rasterization._C` -- the operator surface the reference's autograd Function
binds (imported at gaussian_renderer/__init__.py:17 of Street-sparse-3DGS), implemented over
the gfx950 C ABI (include/gsr.h) instead of a CUDA torch extension.

Same function names, positional argument order, return tuples and error behaviour as the
upstream extension:

  rasterize_gaussians(bg, means3D, colors, opacity, scales, rotations, scale_modifier,
      cov3D_precomp, viewmatrix, projmatrix, tanfovx, tanfovy, image_height, image_width, sh,
      degree, campos, prefiltered, debug, render_indices, parent_indices,
      interpolation_weights, num_node_kids, do_depth)
    -> (num_rendered, color, invdepth, radii, geomBuffer, binningBuffer, imgBuffer)

  rasterize_gaussians_backward(bg, means3D, radii, colors, scales, rotations, scale_modifier,
      cov3D_precomp, viewmatrix, projmatrix, tanfovx, tanfovy, dL_dout_color,
      dL_dout_invdepth, sh, degree, campos, geomBuffer, num_rendered, binningBuffer,
      imgBuffer, render_indices, parent_indices, interpolation_weights, num_node_kids, debug)
    -> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
        dL_drotations)

  mark_visible(means3D, viewmatrix, projmatrix) -> bool tensor (P,)

Scratch buffers are torch uint8 tensors created by resize callbacks, so they come from the
torch caching allocator and are freed with the autograd graph, as upstream's are.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading

import torch

from . import _lib

_L = _lib.load()
_FWD_NO_BACKWARD = 1  # GSR_FWD_NO_BACKWARD (include/gsr.h)


def _ptr(t):
    """A tensor's device address as a plain int (the argtypes are c_void_p: ctypes converts it
    without a c_void_p object per argument), or None (NULL) for an absent or empty tensor."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def _dev_f32(t, name, device):
    if t is None or t.numel() == 0:
        return None
    if t.get_device() != device.index:
        raise RuntimeError(f"{name} must be on {device} (got {t.device})")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    return t if t.is_contiguous() else t.contiguous()


def _saved(t):
    """A tensor the forward already validated (the autograd Function saved it): contiguous, or
    None when absent / empty."""
    if t is None or t.numel() == 0:
        return None
    return t if t.is_contiguous() else t.contiguous()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device):
    """The current HIP stream of `device` (the raw handle, without building a torch Stream object
    per call when torch exposes it)."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def _on(device):
    """torch.cuda.device(device), or nothing when it is already the current device (the library
    works on the current HIP device; the usual single-device caller pays no device switch)."""
    if device.index is None or device.index == torch.cuda.current_device():
        return contextlib.nullcontext()
    return torch.cuda.device(device)


class _Resizer:
    """Holds the uint8 tensors the library asks for through gsr_resize_fn callbacks.

    The ctypes thunks are built once per process (one per buffer name, module level) and find
    the resizer of the call in progress through a thread-local slot, so a call builds no
    CFUNCTYPE objects (three per frame cost measurable host time on slow hosts).  `release()`
    empties the slot: the tensors are owned by `bufs` alone, and every frame's scratch returns
    to the caching allocator as soon as autograd releases it."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}
        _TLS.current = self

    def fn(self, name):
        return _THUNKS[name]

    def release(self):
        _TLS.current = None

    def get(self, name):
        return self.bufs.get(name, torch.empty(0, dtype=torch.uint8, device=self.device))


_TLS = threading.local()


def _make_thunk(name):
    def cb(_ctx, nbytes):
        r = _TLS.current
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=r.device)
        r.bufs[name] = t
        return t.data_ptr()
    return _lib.RESIZE_FN(cb)


_THUNKS = {n: _make_thunk(n) for n in ("geom", "binning", "image", "scratch")}


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_lib.last_error()}")


def _require_gpu(t):
    if not t.is_cuda:
        raise RuntimeError("diff_gaussian_rasterization (gfx950) requires tensors on a ROCm GPU device; "
                           "there is no CPU path")


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug, render_indices=None, parent_indices=None, interpolation_weights=None,
                        num_node_kids=None, do_depth=True, need_backward=True):
    """need_backward=False (an extension; upstream has no such argument): no backward will use
    this frame's buffers -- the autograd Function passes it for frames autograd does not record
    (torch.no_grad evaluation), which then skip the backward's accumulator clear
    (GSR_FWD_NO_BACKWARD, include/gsr.h)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    M = sh.size(1) if (sh is not None and sh.numel() != 0) else 0
    means3D_c = _dev_f32(means3D, "means3D", dev)
    sh_c = _dev_f32(sh, "sh", dev)
    colors_c = _dev_f32(colors, "colors_precomp", dev)
    opac_c = _dev_f32(opacity, "opacities", dev)
    scales_c = _dev_f32(scales, "scales", dev)
    rots_c = _dev_f32(rotations, "rotations", dev)
    cov_c = _dev_f32(cov3D_precomp, "cov3D_precomp", dev)
    view_c = _dev_f32(viewmatrix, "viewmatrix", dev)
    proj_c = _dev_f32(projmatrix, "projmatrix", dev)
    campos_c = _dev_f32(campos, "campos", dev)
    bg_c = _dev_f32(background, "bg", dev)
    if P > 0 and opac_c is None:
        raise RuntimeError("opacities must be provided")
    n_render, ri_c, pi_c, w_c, kids_c = _cut_args(render_indices, parent_indices, interpolation_weights,
                                                  num_node_kids, dev)

    out_color = torch.empty(3, H, W, dtype=torch.float32, device=dev)
    # written for every pixel when do_depth; zeros otherwise (callers ignore it)
    out_invdepth = (torch.empty if do_depth else torch.zeros)(1, H, W, dtype=torch.float32, device=dev)
    radii = torch.empty(n_render if n_render > 0 else P, dtype=torch.int32, device=dev)
    res = _Resizer(dev)
    K = ctypes.c_int64(0)
    with _on(dev):
        rc = _L.gsr_rasterize_forward_ex(
            res.fn("geom"), res.fn("binning"), res.fn("image"), None, P, int(degree), M, _ptr(bg_c), W, H,
            _ptr(means3D_c), _ptr(sh_c), _ptr(colors_c), _ptr(opac_c), _ptr(scales_c), float(scale_modifier),
            _ptr(rots_c), _ptr(cov_c), _ptr(view_c), _ptr(proj_c), _ptr(campos_c), float(tan_fovx),
            float(tan_fovy), int(bool(prefiltered)), _ptr(out_color), _ptr(out_invdepth) if do_depth else None,
            _ptr(radii), _ptr(ri_c), _ptr(pi_c), _ptr(w_c), _ptr(kids_c), n_render, int(bool(debug)), _stream(dev),
            ctypes.byref(K), 0 if need_backward else _FWD_NO_BACKWARD)
    res.release()
    _check(rc, "rasterize_gaussians")
    return int(K.value), out_color, out_invdepth, radii, res.get("geom"), res.get("binning"), res.get("image")


def _cut_args(render_indices, parent_indices, interpolation_weights, num_node_kids, dev):
    """The hierarchy-cut fields: empty render_indices (every reference caller) -> nothing is
    passed; non-empty ones must come with parent_indices / interpolation_weights of at least as
    many entries, on the device (include/gsr.h)."""
    n = 0 if render_indices is None else int(render_indices.numel())
    if n == 0:
        return 0, None, None, None, None
    if parent_indices is None or interpolation_weights is None or parent_indices.numel() < n or \
            interpolation_weights.numel() < n:
        raise RuntimeError("render_indices needs parent_indices and interpolation_weights of at least as many entries")
    i32 = lambda t: t.to(device=dev, dtype=torch.int32).contiguous()
    kids = i32(num_node_kids) if num_node_kids is not None and num_node_kids.numel() else None
    return n, i32(render_indices), i32(parent_indices), \
        interpolation_weights.to(device=dev, dtype=torch.float32).contiguous(), kids


_GSR_DIST = []


def _leaf_grad(t, shape, dev):
    """Output for the gradient of input `t`: a view of the capturing gsr_dist.GradBucket when
    one owns t (data-parallel training: the all-reduce then needs no cat / copy), else new."""
    if not _GSR_DIST:
        try:
            import gsr_dist
            _GSR_DIST.append(gsr_dist)
        except ImportError:  # the package used without the repo's multi-GPU helpers
            _GSR_DIST.append(None)
    gd = _GSR_DIST[0]
    if gd is None:
        return torch.empty(shape, dtype=torch.float32, device=dev)
    return gd.grad_out(t.data_ptr() if t is not None else None, shape, dev)


_ZEROS = {}


def _zero(dev):
    """One cached zero per device: the source of the zero-stride gradient views below."""
    z = _ZEROS.get(dev)
    if z is None:
        z = _ZEROS[dev] = torch.zeros(1, dtype=torch.float32, device=dev)
    return z


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color,
                                 dL_dout_invdepth, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                                 render_indices=None, parent_indices=None, interpolation_weights=None,
                                 num_node_kids=None, debug=False, validated=False):
    """validated=True (an extension; the autograd Function passes it): the forward's inputs were
    checked by rasterize_gaussians, so only the incoming gradients are checked again."""
    _require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    H, W = dL_dout_color.size(1), dL_dout_color.size(2)
    M = sh.size(1) if (sh is not None and sh.numel() != 0) else 0
    f = lambda t, n: _dev_f32(t, n, dev)
    if validated:  # the autograd Function's own forward checked these tensors
        means3D_c, sh_c, colors_c = _saved(means3D), _saved(sh), _saved(colors)
        scales_c, rots_c, cov_c = _saved(scales), _saved(rotations), _saved(cov3D_precomp)
        view_c, proj_c, campos_c, bg_c = _saved(viewmatrix), _saved(projmatrix), _saved(campos), _saved(background)
    else:
        means3D_c, sh_c, colors_c = f(means3D, "means3D"), f(sh, "sh"), f(colors, "colors_precomp")
        scales_c, rots_c, cov_c = f(scales, "scales"), f(rotations, "rotations"), f(cov3D_precomp, "cov3D_precomp")
        view_c, proj_c, campos_c, bg_c = f(viewmatrix, "viewmatrix"), f(projmatrix, "projmatrix"), f(campos, "campos"), \
            f(background, "bg")
    dpix = f(dL_dout_color, "dL_dout_color")
    dinv = f(dL_dout_invdepth, "dL_dout_invdepth") if dL_dout_invdepth is not None else None
    radii_c = radii.contiguous()
    n_render, ri_c, pi_c, w_c, kids_c = _cut_args(render_indices, parent_indices, interpolation_weights,
                                                  num_node_kids, dev)

    e = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)
    # gradients of inputs that were not given are identically zero: returned as zero-stride views
    # (upstream's shapes, no memory traffic) and not computed by the kernels
    z = lambda *shape: _zero(dev).expand(*shape)
    dL_dmeans2D, dL_dopacity = e(P, 3), e(P, 1)
    dL_dmeans3D = _leaf_grad(means3D, (P, 3), dev)
    dL_dcolors = e(P, 3) if sh_c is None else z(P, 3)
    dL_dcov3D = e(P, 6) if cov_c is not None else z(P, 6)
    dL_dsh = _leaf_grad(sh, (P, M, 3), dev) if sh_c is not None else torch.zeros(P, 0, 3, device=dev)
    if cov_c is None:
        dL_dscales, dL_drotations = e(P, 3), e(P, 4)
    else:
        dL_dscales, dL_drotations = z(P, 3), z(P, 4)
    res = _Resizer(dev)
    with _on(dev):
        rc = _L.gsr_rasterize_backward(
            res.fn("scratch"), None, P, int(degree), M, int(R), _ptr(bg_c), W, H, _ptr(means3D_c), _ptr(sh_c),
            _ptr(colors_c), _ptr(scales_c), float(scale_modifier), _ptr(rots_c), _ptr(cov_c), _ptr(view_c),
            _ptr(proj_c), _ptr(campos_c), float(tan_fovx), float(tan_fovy), _ptr(radii_c), _ptr(geomBuffer),
            _ptr(binningBuffer), _ptr(imageBuffer), _ptr(dpix), _ptr(dinv), _ptr(dL_dmeans2D),
            _ptr(dL_dcolors) if sh_c is None else None, _ptr(dL_dopacity), _ptr(dL_dmeans3D),
            _ptr(dL_dcov3D) if cov_c is not None else None, _ptr(dL_dsh) if sh_c is not None else None,
            _ptr(dL_dscales) if cov_c is None else None, _ptr(dL_drotations) if cov_c is None else None,
            _ptr(ri_c), _ptr(pi_c), _ptr(w_c), _ptr(kids_c), n_render, int(bool(debug)), _stream(dev))
    res.release()
    _check(rc, "rasterize_gaussians_backward")
    return dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations


def mark_visible(means3D, viewmatrix, projmatrix):
    _require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    present = torch.empty(P, dtype=torch.uint8, device=dev)
    m = _dev_f32(means3D, "means3D", dev)
    v = _dev_f32(viewmatrix, "viewmatrix", dev)
    p = _dev_f32(projmatrix, "projmatrix", dev)
    with torch.cuda.device(dev):
        rc = _L.gsr_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), _stream(dev))
    _check(rc, "mark_visible")
    return present.bool()


def set_true_scale_gradient(enable: bool) -> bool:
    """dL/dscales as the exact derivative (times scale_modifier) instead of upstream's dL/d(mod*s).
    Process-wide; returns the previous setting.  Only differs when scale_modifier != 1."""
    return bool(_L.gsr_set_true_scale_gradient(int(bool(enable))))


def set_deterministic(enable: bool) -> bool:
    """Backward accumulation: False (default) = hardware float atomics into per-Gaussian rows
    (upstream's scheme, last-bit run-to-run variation); True = per-instance records summed in a
    fixed order (bitwise reproducible, slower).  Process-wide; returns the previous setting."""
    return bool(_L.gsr_set_deterministic(int(bool(enable))))


def set_binning(mode: int) -> int:
    """Depth-order strategy (gsr_set_binning): 0 = local per-superblock sort where it applies,
    1 = always the global depth sort (default).  Process-wide; returns the previous mode."""
    r = _L.gsr_set_binning(int(mode))
    _check(0 if r >= 0 else r, "set_binning")
    return r


def set_bwd_segment(length: int) -> int:
    """Backward work split (gsr_set_bwd_segment): 0 = one workgroup per tile, L = a multiple of
    64 >= 512 (default 512) = heavy tiles replayed as segments of L list positions.  Process-wide;
    returns the previous length."""
    r = _L.gsr_set_bwd_segment(int(length))
    _check(0 if r >= 0 else r, "set_bwd_segment")
    return r


def set_fwd_segment(length: int) -> int:
    """Forward work split (gsr_set_fwd_segment): 0 = one workgroup per tile, L = a multiple of 64
    >= 4096 (default 4096, behind the split gate) = tiles with lists longer than 4 L blended as
    segments of L positions by a worker pool.  Process-wide; returns the previous length."""
    r = _L.gsr_set_fwd_segment(int(length))
    _check(0 if r >= 0 else r, "set_fwd_segment")
    return r


def set_fwd_split_min(length: int) -> int:
    """gsr_set_fwd_split_min: the shortest tile list the forward split takes (0 = 4 segments, the
    default).  Process-wide; returns the previous setting."""
    r = _L.gsr_set_fwd_split_min(int(length))
    _check(0 if r >= 0 else r, "set_fwd_split_min")
    return r


def set_split_gate(enable: bool) -> bool:
    """gsr_set_split_gate: True (default) arms the forward split and the tile binning's superblock
    split only for the 256 frames after one whose lists called for them; False arms them on every
    frame.  Process-wide; returns the previous setting."""
    return bool(_L.gsr_set_split_gate(int(bool(enable))))


def reset_capacity_hint() -> None:
    """Forget this thread's point-list capacity hint (gsr_reset_capacity_hint)."""
    _L.gsr_reset_capacity_hint()


def forward_stats() -> dict:
    """Frames rasterized since load, how many re-ran their binning at K, how many were binned by
    the local sort and how many of those fell back to the global sort (gsr_forward_stats)."""
    buf = (ctypes.c_int64 * 4)()
    n = _L.gsr_forward_stats(buf, 4)
    keys = ("frames", "reruns", "local_sort", "fallbacks")
    return {k: (int(buf[i]) if n > i else 0) for i, k in enumerate(keys)}


def frame_stats(geomBuffer, P, image_height, image_width) -> dict:
    """Level-1 binning entries, tile instances, tile_bin split items and the longest superblock
    list of the frame whose geometry buffer this is (gsr_frame_stats; one device sync)."""
    buf = (ctypes.c_int64 * 4)()
    with torch.cuda.device(geomBuffer.device):
        n = _L.gsr_frame_stats(_ptr(geomBuffer), int(P), int(image_width), int(image_height), buf, 4)
    if n < 0:
        _check(n, "frame_stats")
    return {"level1_entries": int(buf[0]), "tile_instances": int(buf[1]), "tb_split_items": int(buf[2]),
            "max_sb_list": int(buf[3])}


def set_profiling(enable: bool) -> None:
    _L.gsr_set_profiling(int(bool(enable)))


STAGES = ("preprocess", "depth_sort_scan", "bin_superblocks", "bin_tiles", "tile_order", "render_fwd", "render_bwd",
          "preprocess_bwd", "sh_color", "tile_order_bwd")


def stage_times_ms() -> dict:
    buf = (ctypes.c_float * len(STAGES))()
    n = _L.gsr_stage_times_ms(buf, len(STAGES))
    return {STAGES[i]: float(buf[i]) for i in range(n)}
