"""expand_to_size / get_interpolation_weights alone on config 5's synthetic hierarchy (bench.py
config5: 37.5M leaves, ~50M nodes, tau 15 px at 1080p), HIP events around each call (measurement
tool, run on the GPU box; GSR_LIBRARY picks a variant library).  Output: one JSON line."""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "street-sparse-3dgs_amd"))


def main():
    import numpy as np
    import torch
    from gaussian_hierarchy._C import expand_to_size, get_interpolation_weights
    from gs_train.synthetic import synthetic_lod_hierarchy, tau_threshold
    dev = torch.device("cuda:0")
    h = synthetic_lod_hierarchy(37_500_000, 1920, 1080, dev, seed=5, skybox=100_000, log_scale_mean=-6.0)
    N = h["nodes"].shape[0]
    thr = tau_threshold(15.0, h["tanfovx"], 1920)
    ri, pi, ni = (torch.zeros(N, dtype=torch.int32, device=dev) for _ in range(3))
    w = torch.zeros(N, device=dev)
    k = torch.zeros(N, dtype=torch.int32, device=dev)
    cam = torch.tensor(h["campos"], dtype=torch.float32, device=dev)
    cam_cpu, z3 = cam.cpu(), torch.zeros(3)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    t_cut, t_w = [], []
    for it in range(25):
        e0, e1, e2 = ev(), ev(), ev()
        e0.record()
        n = expand_to_size(h["nodes"], h["boxes"], thr, cam, z3, ri, pi, ni)
        e1.record()
        get_interpolation_weights(ni[:n], thr, h["nodes"], h["boxes"], cam_cpu, z3, w, k)
        e2.record()
        torch.cuda.synchronize()
        if it >= 5:
            t_cut.append(e0.elapsed_time(e1))
            t_w.append(e1.elapsed_time(e2))
    print(json.dumps({"lib": os.environ.get("GSR_LIBRARY", "default"), "nodes": N, "cut": n,
                      "expand_ms_median": round(float(np.median(t_cut)), 4),
                      "weights_ms_median": round(float(np.median(t_w)), 4),
                      "checksum": int(ri[:n].long().sum().item()) ^ int(pi[:n].long().sum().item())}))


if __name__ == "__main__":
    main()
