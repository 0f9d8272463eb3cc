"""diff_gaussian_rasterization -- MI355X (gfx950) drop-in for the differentiable Gaussian-splat
rasterizer Street-sparse-3DGS imports at gaussian_renderer/__init__.py:14,17:

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from diff_gaussian_rasterization import _C

Public surface: the 17-field settings NamedTuple, the nn.Module whose forward
takes means3D / means2D / opacities / shs | colors_precomp / scales+rotations | cov3D_precomp
by keyword and returns (color (3,H,W), radii (P,) int32, invdepth (1,H,W)), markVisible, and
the autograd Function that routes gradients to means3D, means2D (screen-space, NDC-scaled),
shs, colors_precomp, opacities, scales, rotations and cov3D_precomp.  Compute runs in the
hand-written HIP kernels of libgsr_hip.so (street-sparse-3dgs_amd/csrc), called from the C++ host
extension _gsr_host.so (street-sparse-3dgs_amd/host); there is no CPU path.
"""
from __future__ import annotations

import os
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_C"]


def _snapshot(args):
    """Debug mode: copies of the call's tensors, kept so a failing call can be replayed.

    Upstream deep-copies every tensor to the host before each debug-mode call
    (diff_gaussian_rasterization/__init__.py:26-28,53-54,90-91), which render_coarse pays on every
    frame (gaussian_renderer/__init__.py:341 forces debug).  Here the copies stay on the device (one
    device-to-device clone per tensor, at HBM rate) and move to the host only when the call fails --
    the dump the caller sees is the same host tuple.  A failure that leaves the device unusable
    aborts the process on ROCm before any Python handler runs, so a host copy would not survive it
    either.  GSR_DEBUG_HOST_SNAPSHOT=1 takes upstream's host copies instead (read per call)."""
    host = os.environ.get("GSR_DEBUG_HOST_SNAPSHOT") == "1"
    return tuple((a.cpu().clone() if host else a.clone()) if isinstance(a, torch.Tensor) else a for a in args)


def _dump(saved, path):
    torch.save(tuple(a.cpu() if isinstance(a, torch.Tensor) else a for a in saved), path)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    """The autograd call.  Normally the C++ autograd Function of the host extension (_C._host.rasterize:
    settings read, validation, buffers and both library calls in C++, the backward on autograd's
    device thread without the GIL); debug mode keeps the Python Function below, whose input
    snapshots and dumps are upstream's debug behaviour."""
    if not raster_settings.debug:
        return _C._host.rasterize(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                                  raster_settings)
    # a frame autograd will not record (torch.no_grad evaluation, or no input that requires grad)
    # can never reach the backward: it skips the backward's accumulator clear
    need_backward = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad
        for t in (means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp))
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings, need_backward)


def _hier(rs, name):
    t = getattr(rs, name, None)
    return torch.empty(0) if t is None else t


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, need_backward=True):
        rs = raster_settings
        do_depth = bool(getattr(rs, "do_depth", True))
        args = (rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, sh,
                rs.sh_degree, rs.campos, rs.prefiltered, rs.debug, _hier(rs, "render_indices"),
                _hier(rs, "parent_indices"), _hier(rs, "interpolation_weights"), _hier(rs, "num_node_kids"),
                do_depth)
        if rs.debug:
            saved = _snapshot(args)
            try:
                num_rendered, color, invdepth, radii, geomBuffer, binningBuffer, imgBuffer = \
                    _C.rasterize_gaussians(*args, need_backward=need_backward)
            except Exception:
                _dump(saved, "snapshot_fw.dump")
                print("\n[diff_gaussian_rasterization] forward failed in debug mode; its inputs are in "
                      "snapshot_fw.dump (torch.load it and call _C.rasterize_gaussians(*args) to replay)")
                raise
        else:
            num_rendered, color, invdepth, radii, geomBuffer, binningBuffer, imgBuffer = \
                _C.rasterize_gaussians(*args, need_backward=need_backward)

        ctx.raster_settings = rs
        # an output no loss uses (the inverse depth, in most training steps) arrives as None, not
        # as a materialised zero image: no fill launch, and the backward skips its depth term
        ctx.set_materialize_grads(False)
        ctx.num_rendered = num_rendered
        ctx.do_depth = do_depth
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer,
                              binningBuffer, imgBuffer)
        ctx.mark_non_differentiable(radii)
        return color, radii, invdepth

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, grad_out_depth):
        rs = ctx.raster_settings
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer, \
            imgBuffer = ctx.saved_tensors
        if grad_out_color is None:
            grad_out_color = torch.zeros(3, rs.image_height, rs.image_width, device=means3D.device)
        dinv = grad_out_depth if (ctx.do_depth and grad_out_depth is not None) else None
        args = (rs.bg, means3D, radii, colors_precomp, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color.contiguous(),
                dinv.contiguous() if dinv is not None else None, sh, rs.sh_degree, rs.campos, geomBuffer,
                ctx.num_rendered, binningBuffer, imgBuffer, _hier(rs, "render_indices"), _hier(rs, "parent_indices"),
                _hier(rs, "interpolation_weights"), _hier(rs, "num_node_kids"), rs.debug)
        if rs.debug:
            saved = _snapshot(args)
            try:
                grads = _C.rasterize_gaussians_backward(*args, validated=True)
            except Exception:
                _dump(saved, "snapshot_bw.dump")
                print("\n[diff_gaussian_rasterization] backward failed in debug mode; its inputs are in "
                      "snapshot_bw.dump (replay with _C.rasterize_gaussians_backward(*args))")
                raise
        else:
            grads = _C.rasterize_gaussians_backward(*args, validated=True)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh, grad_scales,
         grad_rotations) = grads

        def keep(g, inp):
            return g if (inp is not None and inp.numel() != 0) else None

        return (grad_means3D, grad_means2D, keep(grad_sh, sh), keep(grad_colors_precomp, colors_precomp),
                grad_opacities, keep(grad_scales, scales), keep(grad_rotations, rotations),
                keep(grad_cov3Ds_precomp, cov3Ds_precomp), None, None)


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
    do_depth: bool = True
    render_indices: torch.Tensor = None
    parent_indices: torch.Tensor = None
    interpolation_weights: torch.Tensor = None
    num_node_kids: torch.Tensor = None


_EMPTY = torch.empty(0)  # the stand-in for an absent input (upstream builds torch.Tensor([]) per call)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        """Boolean mask of the positions in front of the camera's near plane (view z > 0.2)."""
        with torch.no_grad():
            rs = self.raster_settings
            visible = _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = _EMPTY
        if shs is None:
            shs = empty
        if colors_precomp is None:
            colors_precomp = empty
        if scales is None:
            scales = empty
        if rotations is None:
            rotations = empty
        if cov3D_precomp is None:
            cov3D_precomp = empty
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                   rs)
