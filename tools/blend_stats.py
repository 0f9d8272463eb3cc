"""Lane-liveness statistics of the blend kernels on the bench frame (run ON the GPU box with a
stats variant library):
    python3 street-sparse-3dgs_amd/build_hip.py --define GSR_BLEND_STATS=1 --out vlibs/stats.so
    GSR_LIBRARY=vlibs/stats.so python3 tools/blend_stats.py [--gaussians N --width W --height H]
One fwd+bwd step of bench.py's workload; prints the counters of gsr_blend_stats as fractions."""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "street-sparse-3dgs_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--fovx", type=float, default=60.0)
    a = ap.parse_args()
    import torch
    from diff_gaussian_rasterization import _C
    dev = torch.device("cuda:0")
    s, inp, gcol, ginv = bench.make_inputs(a.gaussians, a.width, a.height, 3, 0, dev, fovx_deg=a.fovx)
    rs, raster = bench.rasterizer_for(s, a.width, a.height, 3, dev)
    step = bench.fwd_bwd_step(raster, inp, gcol, ginv)
    step()
    torch.cuda.synchronize()
    buf = (ctypes.c_int64 * 16)()
    _C._L.gsr_blend_stats(buf, 16, 1)  # reset
    step()
    torch.cuda.synchronize()
    n = _C._L.gsr_blend_stats(buf, 16, 1)
    v = [int(buf[i]) for i in range(n)]
    bp, bl, bh, br, bq, bi, bb, fp, fl, fh, fr, fq, fa, bt = v[:14]
    out = {"frame": f"{a.gaussians} Gaussians {a.width}x{a.height}",
           "bwd": {"pairs": bp, "live_lane_frac": bl / max(1, 64 * bp), "live_half_frac": bh / max(1, 2 * bp),
                   "live_row_frac": br / max(1, 4 * bp), "live_quad_frac": bq / max(1, 4 * bp),
                   "staged_instances": bi, "batches": bb, "tiles": bt, "pairs_per_instance": bp / max(1, bi)},
           "fwd": {"pairs": fp, "alpha_lane_frac": fl / max(1, 64 * fp), "accepted_lane_frac": fa / max(1, 64 * fp),
                   "live_half_frac": fh / max(1, 2 * fp), "live_row_frac": fr / max(1, 4 * fp),
                   "live_quad_frac": fq / max(1, 4 * fp)},
           "raw": v}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
