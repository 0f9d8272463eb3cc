"""simple_knn._C.distCUDA2 on the gfx950 kernel (csrc/knn.hip, include/gsr_knn.h).

distCUDA2(points) -> (N,) float32: the mean of the squared distances from each point to its three
nearest other points (exact, self excluded by index), as scene/gaussian_model.py:207 consumes it:
    dist2 = torch.clamp_min(distCUDA2(fused_point_cloud), 0.0000001)
"""
from __future__ import annotations

import torch

from gs_train._native import check, lib, ptr, require_gpu, stream


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    require_gpu(points)
    if points.dim() != 2 or points.shape[1] != 3:
        raise ValueError(f"distCUDA2 expects (N, 3) points, got {tuple(points.shape)}")
    pts = points.detach().float().contiguous()
    N = pts.shape[0]
    out = torch.empty(N, dtype=torch.float32, device=pts.device)
    if N == 0:
        return out
    L = lib()
    scratch = torch.empty(L.gsr_knn_scratch_bytes(N), dtype=torch.uint8, device=pts.device)
    check(L.gsr_knn_mean_dist2(N, ptr(pts), ptr(out), ptr(scratch), stream(pts.device)), "gsr_knn_mean_dist2")
    return out
