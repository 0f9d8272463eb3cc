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

The three calls are implemented in C++ (host/rasterize_host.cpp, built as _gsr_host.so): validation,
output allocation, the scratch buffers' resize callbacks (torch uint8 tensors from the caching
allocator, freed with the autograd graph, as upstream's are) and the C ABI call.  GaussianRasterizer's
autograd Function is a C++ one too (_gsr_host.rasterize; __init__.py).  The process-wide settings and
statistics below go through ctypes (_lib).
"""
from __future__ import annotations

import ctypes

import torch  # noqa: F401  (the host extension needs torch's libraries loaded first)

from . import _lib

_L = _lib.load()
try:
    from . import _gsr_host as _host
except ImportError as e:  # no fallback: a missing or stale extension fails the import
    raise _lib.RasterizerLibraryError(
        f"the rasterizer's host extension _gsr_host.so is missing or stale ({e}); build it with "
        f"`python street-sparse-3dgs_amd/build_hip.py` (or __graft_entry__.build())") from e
_host.bind(_lib.LIB_PATH)  # the same library file ctypes loaded (GSR_LIBRARY variants included)

# (bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
#  projmatrix, tanfovx, tanfovy, image_height, image_width, sh, degree, campos, prefiltered, debug,
#  render_indices=None, parent_indices=None, interpolation_weights=None, num_node_kids=None,
#  do_depth=True, need_backward=True) -> (num_rendered, color, invdepth, radii, geomBuffer,
#  binningBuffer, imgBuffer).  need_backward=False (an extension; upstream has no such argument): no
#  backward will use this frame's buffers (torch.no_grad evaluation), which then skip the backward's
#  accumulator clear (GSR_FWD_NO_BACKWARD, include/gsr.h).
rasterize_gaussians = _host.rasterize_gaussians
# (..., debug=False, validated=False): validated=True (the autograd Function passes it) skips
# re-checking the forward's own inputs; only the incoming gradients are checked.
rasterize_gaussians_backward = _host.rasterize_gaussians_backward
mark_visible = _host.mark_visible


def _capture_listener(bucket):
    """gsr_dist.GradBucket capture on / off: while one captures, the C++ backward asks
    gsr_dist.grad_out for the leaf gradients' outputs (views of the bucket: no cat, no copy)."""
    import gsr_dist
    _host.set_grad_provider(gsr_dist.grad_out if bucket is not None else None)


try:
    import gsr_dist as _gsr_dist
    _gsr_dist.add_capture_listener(_capture_listener)
except ImportError:  # the package used without the repo's multi-GPU helpers
    pass


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_lib.last_error()}")


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
    >= 1024 (default 2048, behind the split gate) = tiles with lists longer than the split minimum
    (6 L by default, gsr_set_fwd_split_min) blended as segments of L positions by a worker pool.
    Process-wide; returns the previous length."""
    r = _L.gsr_set_fwd_segment(int(length))
    _check(0 if r >= 0 else r, "set_fwd_segment")
    return r


def set_fwd_split_min(length: int) -> int:
    """gsr_set_fwd_split_min: the shortest tile list the forward split takes (0 = 6 segments of the
    forward segment length, the default).  Process-wide; returns the previous setting."""
    r = _L.gsr_set_fwd_split_min(int(length))
    _check(0 if r >= 0 else r, "set_fwd_split_min")
    return r


def set_live_list(enable: bool) -> bool:
    """gsr_set_live_list: True walks the backward's live rows through one list spread over the chip
    (rows in spatial order: gs_train.chunk.reorder_rows); False (default) per 2048-row range.  Same
    gradients either way.  Returns the previous setting."""
    return bool(_L.gsr_set_live_list(int(bool(enable))))


def set_split_gate(enable: bool) -> bool:
    """gsr_set_split_gate: True (default) arms the forward split and the tile binning's superblock
    split only for the 256 frames after one whose lists called for them; False arms them on every
    frame.  Process-wide; returns the previous setting."""
    return bool(_L.gsr_set_split_gate(int(bool(enable))))


def set_fwd_spin_limits(ready: int = 0, flag: int = 0) -> None:
    """gsr_set_fwd_spin_limits: the forward-split workers' spin bounds (0 = default; tests)."""
    _check(_L.gsr_set_fwd_spin_limits(int(ready), int(flag)), "set_fwd_spin_limits")


def reset_capacity_hint() -> None:
    """Forget this thread's point-list capacity hint (gsr_reset_capacity_hint)."""
    _L.gsr_reset_capacity_hint()


def forward_stats() -> dict:
    """Frames rasterized since load, how many re-ran their binning at K, how many were binned by
    the local sort and how many of those fell back to the global sort, forward-split workers that
    gave up waiting for tile_order (their frames completed by the pool's second launch) and the host
    nanoseconds spent waiting for K (gsr_forward_stats)."""
    buf = (ctypes.c_int64 * 8)()
    n = _L.gsr_forward_stats(buf, 8)
    keys = ("frames", "reruns", "local_sort", "fallbacks", "fwd_worker_giveups", "k_wait_ns", "fwd_split_frames",
            "tb_split_frames")
    return {k: (int(buf[i]) if n > i else 0) for i, k in enumerate(keys)}


def fwd_pool_stats(reset: bool = False) -> dict:
    """The forward-split worker pool's time (gsr_fwd_pool_stats; synchronises the device): seconds
    its workgroups spent waiting for tile_order's release of the queue (ready), waiting for
    predecessor segments (flags), in total, the workgroup count and the busy fraction."""
    buf = (ctypes.c_int64 * 4)()
    n = _L.gsr_fwd_pool_stats(buf, 4, 1 if reset else 0)
    if n < 4:
        raise RuntimeError(f"gsr_fwd_pool_stats failed ({n})")
    ready, flags, total = (buf[i] * 1e-8 for i in range(3))
    return {"ready_wait_s": ready, "flag_wait_s": flags, "total_s": total, "workgroups": int(buf[3]),
            "busy_frac": (1.0 - (ready + flags) / total) if total > 0 else None}


def frame_stats(geomBuffer, P, image_height, image_width) -> dict:
    """Level-1 binning entries, tile instances, tile_bin split items and the longest superblock
    list of the frame whose geometry buffer this is (gsr_frame_stats; one device sync)."""
    buf = (ctypes.c_int64 * 4)()
    with torch.cuda.device(geomBuffer.device):
        n = _L.gsr_frame_stats((geomBuffer.data_ptr() if geomBuffer.numel() else None), int(P), int(image_width), int(image_height), buf, 4)
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
