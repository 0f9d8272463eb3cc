"""Per-tile work of a trained synthetic street chunk (measurement tool, run on the GPU box):
trains gs_train.chunk.street_chunk for --iters iterations of the default schedule with the native
step, then for --views photometric views reports the tile list lengths (ranges), the per-tile
backward work (tile_work: the last contributor any pixel of the tile uses) and the rasterizer's
stage times, to see whether the render / binning kernels are tail-bound on street views (cube
faces looking down a corridor collect its far Gaussians in the tiles around the vanishing point).

    python tools/street_tiles.py --iters 12000 --views 8 > gpurun_out/street_tiles.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "street-sparse-3dgs_amd"), os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12000)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--size", type=int, default=1536)
    a = ap.parse_args()
    import torch
    from diff_gaussian_rasterization import _C
    from gs_train.chunk import ChunkSchedule, TrainChunk, street_chunk
    from gs_train.native_step import NativeTrainStep
    from helpers import image_layout, view
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    ts, info = street_chunk(NativeTrainStep, W=a.size, H=a.size, iterations=30_000, device=dev)
    tc = TrainChunk(ts, ChunkSchedule())
    t0 = time.perf_counter()
    tc.run(until=a.iters)
    torch.cuda.synchronize()
    print(f"trained {a.iters} iterations in {time.perf_counter() - t0:.1f} s, P = {ts.g.P}", file=sys.stderr)
    W = H = a.size
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    out = {"iters": a.iters, "P": ts.g.P, "views": []}
    g = ts.g
    k = 0
    done = 0
    while done < a.views and k < len(ts.cams):
        if ts.depth_only[k]:
            k += 1
            continue
        c = ts.cams[k]
        e = torch.empty(0, device=dev)
        with torch.no_grad():
            scales, rots, opac = torch.exp(g._scaling), torch.nn.functional.normalize(g._rotation), torch.sigmoid(g._opacity)
            _C.set_profiling(True)
            raw = _C.rasterize_gaussians(torch.zeros(3, device=dev), g._xyz.detach(), e, opac, scales, rots, 1.0, e,
                                         c["view"], c["proj"], c["tx"], c["ty"], H, W, g._features.detach(),
                                         g.active_sh_degree, c["campos"], False, False, ts.empty_i, ts.empty_i,
                                         ts.empty_f, ts.empty_id, True)
            torch.cuda.synchronize()
            st = _C.stage_times_ms()
            _C.set_profiling(False)
        im = raw[6].cpu().numpy()
        il = image_layout(T, W * H)
        rg = view(im, il, "ranges", np.uint32, (T, 2)).astype(np.int64)
        lens = rg[:, 1] - rg[:, 0]
        work = view(im, il, "tile_work", np.uint32).astype(np.int64)
        ls, ws = np.sort(lens)[::-1], np.sort(work)[::-1]
        out["views"].append({
            "view": k, "K": int(raw[0]), "fwd_stages_ms": {kk: round(v, 4) for kk, v in st.items() if v > 0},
            "list_len": {"mean": float(lens.mean()), "p50": float(np.median(lens)), "p99": float(np.percentile(lens, 99)),
                         "max": int(ls[0]), "top8": ls[:8].tolist(), "top1pct_share": float(ls[:T // 100].sum() / max(1, ls.sum()))},
            "bwd_work": {"mean": float(work.mean()), "p50": float(np.median(work)), "p99": float(np.percentile(work, 99)),
                         "max": int(ws[0]), "top8": ws[:8].tolist(), "sum": int(work.sum()),
                         "top1pct_share": float(ws[:T // 100].sum() / max(1, ws.sum()))}})
        done += 1
        k += 1
    print(json.dumps(out))


if __name__ == "__main__":
    main()
