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
    ap.add_argument("--segs", default="0:0,0:512,4096:512,8192:512",
                    help="forward:backward[:fwd split minimum] segment lengths to time (A/B), comma separated")
    ap.add_argument("--no-gate", action="store_true", help="arm the splits on every frame (gsr_set_split_gate off)")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from diff_gaussian_rasterization import _C
    from gs_train.chunk import ChunkSchedule, TrainChunk, street_chunk
    from gs_train.native_step import NativeTrainStep
    from helpers import image_layout, view
    dev = torch.device("cuda:0")
    if a.no_gate:
        _C.set_split_gate(False)
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
        out["views"][-1]["bwd_ms_by_seg"] = time_segments(g, c, H, W, a.segs.split(","), a.reps)
        done += 1
        k += 1
    print(json.dumps(out))


def time_segments(g, c, H, W, segs, reps):
    """fwd+bwd of one view through the public rasterizer per backward segment length: the stage
    times (render_bwd, render_fwd) and the fwd+bwd wall time, medians over reps."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, _C
    dev = g._xyz.device
    rs = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=float(c["tx"]), tanfovy=float(c["ty"]),
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=c["view"], projmatrix=c["proj"],
        sh_degree=g.active_sh_degree, campos=c["campos"], prefiltered=False, debug=False, do_depth=True,
        render_indices=torch.empty(0, dtype=torch.int32), parent_indices=torch.empty(0, dtype=torch.int32),
        interpolation_weights=torch.empty(0, dtype=torch.float32, device=dev),
        num_node_kids=torch.empty(0, dtype=torch.int32, device=dev))
    gen = torch.Generator(device=dev).manual_seed(5)
    up_c = torch.randn(3, H, W, generator=gen, device=dev) * 1e-3
    up_d = torch.randn(1, H, W, generator=gen, device=dev) * 1e-3
    res = {}
    ref = ref_det = ref_col = None

    def det_grads():
        prev_det = _C.set_deterministic(True)
        xs = [t.detach().clone().requires_grad_(True) for t in
              (g._xyz, g._features, torch.sigmoid(g._opacity), torch.exp(g._scaling),
               torch.nn.functional.normalize(g._rotation))]
        col, _, invd = GaussianRasterizer(rs)(means3D=xs[0], means2D=torch.zeros_like(g._xyz, requires_grad=True),
                                              shs=xs[1], opacities=xs[2], scales=xs[3], rotations=xs[4])
        ((col * up_c).sum() + (invd * up_d).sum()).backward()
        _C.set_deterministic(prev_det)
        return [x.grad for x in xs]

    rel = lambda ga, gb: max(float((a - b).norm() / b.norm().clamp_min(1e-30)) for a, b in zip(ga, gb))
    for cfg in segs:
        parts = [int(x) for x in cfg.split(":")]
        fL, L = parts[:2]
        prev, fprev = _C.set_bwd_segment(L), _C.set_fwd_segment(fL)
        mprev = _C.set_fwd_split_min(parts[2] if len(parts) > 2 else 0)
        st_all, wall, last2 = [], [], []
        for r in range(reps + 2):
            xs = [t.detach().clone().requires_grad_(True) for t in
                  (g._xyz, g._features, torch.sigmoid(g._opacity), torch.exp(g._scaling),
                   torch.nn.functional.normalize(g._rotation))]
            m2 = torch.zeros_like(g._xyz, requires_grad=True)
            _C.set_profiling(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            col, _, invd = GaussianRasterizer(rs)(means3D=xs[0], means2D=m2, shs=xs[1], opacities=xs[2],
                                                  scales=xs[3], rotations=xs[4])
            ((col * up_c).sum() + (invd * up_d).sum()).backward()
            e1.record()
            torch.cuda.synchronize()
            st = _C.stage_times_ms()
            _C.set_profiling(False)
            if r >= 2:
                st_all.append(st)
                wall.append(e0.elapsed_time(e1))
            last2 = (last2 + [[x.grad for x in xs]])[-2:]
            col_last = col.detach()
        grads = last2[-1]
        if ref is None:
            ref, ref_col = grads, col_last
        gd = det_grads()
        if ref_det is None:
            ref_det = gd
        _C.set_bwd_segment(prev)
        _C.set_fwd_segment(fprev)
        _C.set_fwd_split_min(mprev)
        med = lambda k: float(np.median([s_[k] for s_ in st_all]))
        # grad errors (max over tensors of relative L2): atomic vs the first length's atomic run, the
        # run-to-run atomic noise at this length, and record mode (bitwise ordered sums) vs the first
        # length's record mode -- the split's own rounding
        res[cfg] = {"render_bwd": round(med("render_bwd"), 4), "render_fwd": round(med("render_fwd"), 4),
                       "fwd_bwd_wall": round(float(np.median(wall)), 4), "grad_rel_l2_vs_first": rel(grads, ref),
                       "atomic_noise": rel(last2[0], last2[1]), "det_grad_rel_l2_vs_first": rel(gd, ref_det),
                       "color_maxabs_vs_first": float((col_last - ref_col).abs().max())}
    return res


if __name__ == "__main__":
    main()
