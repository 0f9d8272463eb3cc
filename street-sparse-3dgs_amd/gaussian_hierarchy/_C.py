"""`gaussian_hierarchy._C` -- expand_to_size / get_interpolation_weights over the C ABI of
include/gsr_hier.h (csrc/lod.hip), with the argument order and in-place outputs the reference's
callers use:

    to_render = expand_to_size(nodes, boxes, threshold, camera_center, viewdir,
                               render_indices, parent_indices, nodes_for_render_indices)
    get_interpolation_weights(node_indices, threshold, nodes, boxes, camera_center.cpu(), viewdir,
                              interpolation_weights, num_siblings)

(render_hierarchy.py:63-85, train_post.py:91-113).  nodes (N, 7) int32 and boxes (N, 2, 4) float32
on the GPU, as the reference keeps them (scene/gaussian_model.py:424-425).  `viewdir` is accepted
and unused, as in the published cut (the reference passes zeros).  The outputs are written in
place; expand_to_size returns the cut length (one host read, as upstream).

The .hier file I/O of the extension (load_hierarchy / write_hierarchy) is not part of the
rasterizer's hot path and its binary format is not vendored here: both raise.
"""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _lib

_L = _lib.load()


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_lib.last_error()}")


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else None


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _need(t, name, dtype, dev):
    if not t.is_cuda or t.device != dev:
        raise RuntimeError(f"{name} must be on {dev}")
    if t.dtype != dtype:
        raise RuntimeError(f"{name} must be {dtype}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous (written in place)")
    return t


def expand_to_size(nodes, boxes, size, viewpoint, viewdir, render_indices, parent_indices,
                   nodes_for_render_indices):
    dev = nodes.device
    if not nodes.is_cuda:
        raise RuntimeError("expand_to_size: nodes must be on a ROCm GPU device")
    N = nodes.shape[0]
    nodes_c = nodes.to(torch.int32).contiguous()
    boxes_c = boxes.to(torch.float32).contiguous()
    if nodes_c.numel() != 7 * N or boxes_c.numel() != 8 * N:
        raise RuntimeError("expand_to_size: nodes must be (N, 7) int32 and boxes (N, 2, 4) float32")
    for t, n in ((render_indices, "render_indices"), (parent_indices, "parent_indices"),
                 (nodes_for_render_indices, "nodes_for_render_indices")):
        _need(t, n, torch.int32, dev)
    # the device writes at most `cap` entries and the call fails when the cut is longer (a node can
    # hold several Gaussians, so the cut can exceed N)
    cap = min(render_indices.numel(), parent_indices.numel(), nodes_for_render_indices.numel())
    vp = viewpoint.to(device=dev, dtype=torch.float32).contiguous().reshape(3)
    scratch = torch.empty(int(_L.gsr_expand_to_size_scratch_bytes(N)), dtype=torch.uint8, device=dev)
    out = ctypes.c_int64(0)
    with torch.cuda.device(dev):
        rc = _L.gsr_expand_to_size(N, _p(nodes_c), _p(boxes_c), float(size), _p(vp), _p(render_indices),
                                   _p(parent_indices), _p(nodes_for_render_indices), cap, _p(scratch),
                                   scratch.numel(), ctypes.byref(out), _stream(dev))
    _check(rc, "expand_to_size")
    return int(out.value)


def get_interpolation_weights(node_indices, size, nodes, boxes, viewpoint, viewdir, out_weights, out_num_kids):
    dev = nodes.device
    n = node_indices.shape[0]
    idx = node_indices.to(device=dev, dtype=torch.int32).contiguous()
    nodes_c = nodes.to(torch.int32).contiguous()
    boxes_c = boxes.to(torch.float32).contiguous()
    _need(out_weights, "interpolation_weights", torch.float32, dev)
    _need(out_num_kids, "num_node_kids", torch.int32, dev)
    if out_weights.numel() < n or out_num_kids.numel() < n:
        raise RuntimeError("get_interpolation_weights: output arrays shorter than node_indices")
    vx, vy, vz = (float(v) for v in viewpoint.detach().reshape(3).cpu().tolist())
    with torch.cuda.device(dev):
        rc = _L.gsr_interpolation_weights(n, _p(idx), float(size), _p(nodes_c), _p(boxes_c), vx, vy, vz,
                                          _p(out_weights), _p(out_num_kids), _stream(dev))
    _check(rc, "get_interpolation_weights")


# The .hier file (gaussian_hierarchy's writer / loader; the submodule is not vendored in the
# reference, so this layout is restated from the upstream project's uncompressed format and is
# parity-unpinned: no file written by the reference's tools is available here):
#   int32 P; float32 positions[P][3]; float32 rotations[P][4]; float32 log_scales[P][3];
#   float32 opacities[P]; float32 shs[P][48] (16 coefficients x RGB, coefficient-major);
#   int32 N; int32 nodes[N][7] (depth, parent, start, count_leafs, count_merged, start_children,
#   count_children); float32 boxes[N][2][4] (min xyz w, max xyz w).
# A negative P marks the half-precision "compressed" variant, which is not supported (loud).
_HIER_FIELDS = (("positions", 3), ("rotations", 4), ("log_scales", 3), ("opacities", 1), ("shs", 48))


def load_hierarchy(path):
    """(xyz (P,3), shs (P,16,3), alpha (P,1), log-scales (P,3), rotations (P,4), nodes (N,7) int32,
    boxes (N,2,4)) as CPU tensors -- what scene/gaussian_model.py:347 unpacks."""
    import numpy as np
    import torch
    with open(path, "rb") as f:
        data = f.read()
    off = 0

    def take(dtype, count):
        nonlocal off
        a = np.frombuffer(data, dtype=dtype, count=count, offset=off)
        off += a.nbytes
        return a

    P = int(take(np.int32, 1)[0])
    if P < 0:
        raise NotImplementedError("gaussian_hierarchy.load_hierarchy: compressed (half precision) .hier files are "
                                  "not supported")
    arrs = {name: take(np.float32, P * w).reshape(P, w) for name, w in _HIER_FIELDS}
    N = int(take(np.int32, 1)[0])
    nodes = take(np.int32, N * 7).reshape(N, 7)
    boxes = take(np.float32, N * 8).reshape(N, 2, 4)
    if off != len(data):
        raise ValueError(f"gaussian_hierarchy.load_hierarchy: {len(data) - off} trailing bytes in {path}")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    return (t(arrs["positions"]), t(arrs["shs"]).reshape(P, 16, 3), t(arrs["opacities"]), t(arrs["log_scales"]),
            t(arrs["rotations"]), t(nodes), t(boxes))


def write_hierarchy(path, xyz, shs, opacities, scales, rotations, nodes, boxes):
    """The inverse of load_hierarchy (scene/gaussian_model.py:437-445 save_hier): log-scales and
    activated opacities as the caller passes them, any device."""
    import numpy as np
    f32 = lambda x, w: np.ascontiguousarray(x.detach().float().cpu().numpy().reshape(-1, w), dtype=np.float32)
    pos = f32(xyz, 3)
    P = pos.shape[0]
    fields = {"positions": pos, "rotations": f32(rotations, 4), "log_scales": f32(scales, 3),
              "opacities": f32(opacities, 1), "shs": f32(shs, 48)}
    for name, w in _HIER_FIELDS:
        if fields[name].shape != (P, w):
            raise ValueError(f"gaussian_hierarchy.write_hierarchy: {name} has {fields[name].shape[0]} rows, not {P}")
    nd = np.ascontiguousarray(nodes.detach().cpu().numpy().reshape(-1, 7), dtype=np.int32)
    bx = np.ascontiguousarray(boxes.detach().float().cpu().numpy().reshape(-1, 2, 4), dtype=np.float32)
    if bx.shape[0] != nd.shape[0]:
        raise ValueError("gaussian_hierarchy.write_hierarchy: nodes and boxes differ in length")
    with open(path, "wb") as f:
        f.write(np.int32(P).tobytes())
        for name, _ in _HIER_FIELDS:
            f.write(fields[name].tobytes())
        f.write(np.int32(nd.shape[0]).tobytes())
        f.write(nd.tobytes())
        f.write(bx.tobytes())
