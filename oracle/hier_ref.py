"""TEST INFRASTRUCTURE ONLY -- numpy restatement of render_post's hierarchy-cut interpolation
(gaussian_renderer/__init__.py:200-243, interp_python=True), pinned by tests/golden/render_post.npz
(the tensors the reference's own render_post handed to the rasterizer).  Only tests/ import it.
"""
from __future__ import annotations

import numpy as np


def interpolate_cut(xyz, scaling, rotation, opacity, features, render_indices, parent_indices, weights, skybox):
    ri = np.asarray(render_indices, np.int64)
    n = len(ri)
    pi = np.asarray(parent_indices, np.int64)[:n]
    t = np.asarray(weights, np.float32)[:n, None]
    u = (np.float32(1) - np.asarray(weights, np.float32)[:n])[:, None]
    N = xyz.shape[0]
    sk = np.arange(N - skybox, N)
    means = t * xyz[ri] + u * xyz[pi]
    scal = t * scaling[ri] + u * scaling[pi]
    shs = t[:, :, None] * features[ri] + u[:, :, None] * features[pi]
    par = rotation[pi].copy()
    rot = rotation[ri]
    par[(rot * par).sum(1) < 0] *= -1
    rots = t * rot + u * par
    op = t * opacity[ri] + u * opacity[pi]
    cat = lambda a, full: np.concatenate([a, full[sk]]).astype(np.float32)
    return dict(means3D=cat(means, xyz), scales=cat(scal, scaling), rotations=cat(rots, rotation),
                opacities=cat(op, opacity), shs=cat(shs, features))
