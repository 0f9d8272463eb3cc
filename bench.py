"""bench.py -- fwd+bwd Mpix/s of the gfx950 Gaussian-splat rasterizer (BASELINE.json metric).

One step = one forward + backward of GaussianRasterizer through its public API (autograd) on a
1920x1080 frame of 1M synthetic Gaussians (SH degree 3), inputs resident in HBM, upstream
gradients dL/dcolor and dL/dinvdepth ~ N(0,1)/Npix.  Multi-GPU (driver-launched
via torch.distributed.run): one process per GPU, each rank rasterizes its own synthetic chunk
(seed = rank) -- the product's one-chunk-per-GPU sharding, no data-path collective -- and
`value` is the aggregate Mpix/s over all ranks (weak scaling).

Prints ONE JSON line on rank 0.  Extras: "roofline" for the dominant kernel (algorithmic bytes
per launch from SURVEY.md 8(d) / its HIP-event-measured average duration on the rasterizer's
stream), "stages_ms" for every kernel, "cpu_baseline" (the C oracle, timed on the host cores on
full-size fwd+bwd frames, rank 0 at N=1 only) and "cpu_baseline_torch" (the naive PyTorch-CPU
splat of SURVEY.md 8(d) on config 1).
"""
from __future__ import annotations

import argparse
import contextlib
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "street-sparse-3dgs_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--profile-steps", type=int, default=5, help="extra steps with per-stage HIP events")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--diag", action="store_true", help="print synced per-step fwd/bwd wall times to stderr")
    ap.add_argument("--train-steps", type=int, default=20, help="timed train-step harness iterations (0 = skip)")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip config 5 (hierarchy cut + blend + forward render of the cut at 1080p; on by default)")
    ap.add_argument("--config5", action="store_true", help=argparse.SUPPRESS)  # round-2 spelling: now the default
    ap.add_argument("--no-street", action="store_true",
                    help="skip the street-frame point (1536x1536 cube face, 90 deg fov: fwd+bwd and train step)")
    ap.add_argument("--no-coarse-debug", action="store_true", help="skip the render_coarse debug-mode timing")
    ap.add_argument("--no-config4", action="store_true",
                    help="skip config 4 (500k-Gaussian chunk per rank, seed = chunk id: fwd+bwd and train step)")
    ap.add_argument("--metric-only", action="store_true",
                    help="only the metric line's own work (profiling runs): no train step, configs 4/5, street "
                         "frame or CPU baselines")
    ap.add_argument("--c5-leaves", type=int, default=37_500_000, help="leaves of the config-5 tree (~4/3 as many nodes)")
    ap.add_argument("--c5-tau", type=float, default=15.0,
                    help="render_hierarchy.py tau in pixels (its default list: 0, 3, 6, 15)")
    ap.add_argument("--c5-log-scale", type=float, default=-6.0,
                    help="mean log leaf scale of the config-5 tree (-6: ~7.4M-node cut of 50M at tau 15)")
    ap.add_argument("--no-config3", action="store_true",
                    help="skip the config-3 stand-in (train_single.py's whole loop on a synthetic street chunk)")
    ap.add_argument("--chunk-iterations", type=int, default=30_000)
    ap.add_argument("--chunk-size", type=int, default=1536, help="cube-face width = height of the chunk's views")
    ap.add_argument("--chunk-positions", type=int, default=48, help="camera stations (4 cube faces each)")
    ap.add_argument("--chunk-truth", type=int, default=1_000_000, help="Gaussians of the synthetic truth street")
    ap.add_argument("--chunk-init", type=int, default=300_000, help="LiDAR-like initial points")
    ap.add_argument("--chunk-spatial", type=int, default=0,
                    help="row order of the headline config-3 run: 0 (default) the reference's row order; 1 the rows "
                         "in spatial (Morton) order (TrainChunk(spatial=True): gs_train.chunk.reorder_rows after every "
                         "densification -- a permutation the reference does not make, DESIGN.md 10.9)")
    ap.add_argument("--no-chunk-spatial-variant", action="store_true",
                    help="skip the second config-3 run in the other row order (reported as config3_proxy.variant)")
    ap.add_argument("--prewarm-s", type=float, default=0.6,
                    help="cap of the time-based pre-warm before the counted warm-ups (fwd+bwd steps until the shader "
                         "clock settles; 0 = none)")
    ap.add_argument("--detail-out", default=os.environ.get("GSR_BENCH_DETAIL_OUT") or None,
                    help="also write the long diagnostics the line summarises (config 3's per-iteration record, the "
                         "clock samples) to this JSON file")
    ap.add_argument("--post-leaves", type=int, default=3_000_000,
                    help="leaves of the train_post step's synthetic hierarchy (0 = skip that step)")
    ap.add_argument("--bwd-seg", type=int, default=None,
                    help="backward segment length (gsr_set_bwd_segment; default: the library's setting)")
    ap.add_argument("--fwd-seg", type=int, default=None,
                    help="forward segment length (gsr_set_fwd_segment; default: the library's setting)")
    ap.add_argument("--train-baseline", action="store_true",
                    help="also time the reference-structured torch train step (oracle/train_torch_ref.py: conv2d "
                         "SSIM, OurAdam gather/scatter) -- a baseline leg, like cpu_baseline")
    return ap.parse_args()


OVERLAPPED_STAGES = ("sh_color",)


def algorithmic_bytes(P, Pv, K, T, npix, P1, M=16, Pl=None):
    """Per-launch algorithmic bytes per stage.  SURVEY.md 8(d) figures (M=16 constants; the SH
    term scales with M) for the stages it defines; the binning stages follow this build's
    algorithm: a 32-bit depth sort of P ids (4 LSD passes, 16 B/elem/pass) + the
    gathered scan; level-1 binning reads (order, tiles, rect) twice per Gaussian and writes the
    superblock lists (P1 entries of 8 B, measured per frame: gsr_frame_stats); level 2 re-reads
    them with the rects twice and writes the K-entry point list + ranges.  Upstream's 64-bit
    6-pass key sort alone would be 24*K*6.  The dense gradient outputs (56 + 12 M B per Gaussian:
    means2D 12, opacity 4, means3D 12, SH, scales 12, rotations 16) are zeroed by render_bwd's
    waves after their replay (counted under preprocess_bwd, as 8(d) counts every gradient row there, so
    render_bwd's figure is 8(d)'s own 44 K + 24 Npix + 40 Pv); preprocess_bwd reads every row's live
    stamp (4 B), and for the Pl live rows the accumulator (48 B), parameters (40 B) and SH row in and
    the full gradient row out."""
    sh = 12 * M
    grad_row = 56 + sh
    Pl = Pv if Pl is None else Pl
    return {
        # geometry: 44 B of inputs, the GRec minus its colour (48 B) and 4 x 4 B of per-Gaussian
        # outputs; the SH colour pass (side stream, overlapped): SH rows + means + radii in,
        # colour (16 B) + clamp bits out
        "preprocess": 44 * P + 64 * P,
        "sh_color": (sh + 12 + 4) * P + 17 * P,
        "depth_sort_scan": 16 * P * 4 + 12 * P,
        # sb_count reads each visible Gaussian's 4-B depth-ordered tile rect; sb_scatter its order
        # entry and rect again and writes the P1 8-B list entries (id, SB-local footprint)
        "bin_superblocks": 4 * Pv + 8 * Pv + 8 * P1,
        # tile_bin reads the level-1 lists (once, ideally: its second pass should hit L2) and
        # writes the K-entry point list and the ranges
        "bin_tiles": 8 * P1 + 4 * K + 8 * T,
        "tile_order": 16 * T,
        "tile_order_bwd": 12 * T,
        "render_fwd": 44 * K + 24 * npix,
        # SURVEY.md 8(d)'s render-bwd term exactly; the dense zero gradient rows render_bwd's waves
        # also write are booked where 8(d) books every gradient row, under preprocess-bwd
        "render_bwd": 44 * K + 24 * npix + 40 * Pv,
        "preprocess_bwd": 4 * P + (48 + 40 + sh + 12 + grad_row) * Pl + grad_row * P,
    }


def make_inputs(P, W, H, deg, seed, device, fovx_deg=60.0):
    import numpy as np
    import torch
    from gs_train.synthetic import synthetic_scene
    s = synthetic_scene(P, W, H, seed=seed, sh_degree=deg, fovx_deg=fovx_deg)
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=device)
    inp = dict(means3D=t(s["means3D"]), means2D=torch.zeros(P, 3, device=device), opacities=t(s["opacities"]),
               shs=t(s["shs"]), scales=t(s["scales"]), rotations=t(s["rotations"]))
    for v in inp.values():
        v.requires_grad_(True)
    rng = np.random.default_rng(seed + 1000)
    gcol = t(rng.normal(size=(3, H, W)) / (W * H))
    ginv = t(rng.normal(size=(1, H, W)) / (W * H))
    return s, inp, gcol, ginv


def cpu_baseline(s, P, W, H, deg, min_seconds=10.0, max_frames=8):
    """The C oracle (oracle/gs_oracle.c, OpenMP) on full-size fwd+bwd frames of the bench
    workload, repeated until ~min_seconds of CPU work (a bounded sample)."""
    import numpy as np
    import gs_oracle as O
    rng = np.random.default_rng(7)
    dcol = (rng.normal(size=(3, H, W)) / (W * H)).astype(np.float32)
    dinv = (rng.normal(size=(1, H, W)) / (W * H)).astype(np.float32)
    frames = 0
    t0 = time.perf_counter()
    while frames < max_frames and (frames == 0 or time.perf_counter() - t0 < min_seconds):
        st = O.forward(s["means3D"], s["opacities"], s["view"], s["proj"], s["campos"], s["bg"], W, H, s["tanfovx"],
                       s["tanfovy"], sh_degree=deg, shs=s["shs"], scales=s["scales"], rotations=s["rotations"])
        O.backward(st, dcol, dinv)
        frames += 1
    dt = time.perf_counter() - t0
    return {"value": round(frames * W * H / dt / 1e6, 4), "unit": "Mpix/s", "cores": O.num_threads(), "kind": "port",
            "sample": f"{frames} fwd+bwd frames of the bench workload ({P} Gaussians, {W}x{H}, SH deg {deg}) "
                      f"through the C oracle, {dt:.2f} s"}, st


def cpu_baseline_torch(min_seconds=3.0):
    """SURVEY.md 8(d) / north_star: the naive vectorised PyTorch-CPU splat (oracle/torch_splat.py:
    tensor-op preprocess, key sort, per-tile alpha matrices with cumprod transmittance, autograd
    backward) timed on the host cores on config 1 (10k Gaussians at 256x256, SH degree 3), in full."""
    import numpy as np
    import gs_oracle as O
    import torch_splat as TS
    W = H = 256
    s = O.synthetic_scene(10_000, W, H, seed=0, sh_degree=3)
    rng = np.random.default_rng(7)
    dcol = (rng.normal(size=(3, H, W)) / (W * H)).astype(np.float32)
    dinv = (rng.normal(size=(1, H, W)) / (W * H)).astype(np.float32)
    v, frames, dt, threads = TS.time_fwd_bwd(s, dcol, dinv, min_seconds=min_seconds)
    return {"value": round(v, 5), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"config 1 in full: {frames} fwd+bwd frames of 10000 Gaussians at {W}x{H} (SH deg 3) through the "
                      f"naive PyTorch-CPU splat (oracle/torch_splat.py, torch.autograd backward), {dt:.2f} s"}


def psnr_vs_oracle(gpu_color, gpu_invd, st):
    """BASELINE.json metric part 3: PSNR of the bench frame rendered by the HIP path against the
    same frame rendered by the CPU oracle (peak 1.0; colour and inverse depth), plus the fraction
    of pixels off by more than 1e-4."""
    import numpy as np
    c = gpu_color.detach().float().cpu().numpy()
    d = gpu_invd.detach().float().cpu().numpy()
    mse = float(np.mean((c.astype(np.float64) - st["color"]) ** 2))
    out = {"psnr_db": round(10 * np.log10(1.0 / mse), 2) if mse > 0 else None,  # None: bit-identical
           "max_abs_err": float(np.max(np.abs(c - st["color"]))),
           "frac_pixels_off_1e-4": float(np.mean(np.abs(c - st["color"]) > 1e-4)),
           "invdepth_rel_l2": float(np.linalg.norm(d - st["invdepth"]) / max(np.linalg.norm(st["invdepth"]), 1e-30)),
           "reference": "oracle/gs_oracle.c forward of the bench frame (fp32, upstream algorithm restated)"}
    return out


def train_step_ms(P, W, H, steps, warmup, dev, street=True, reference=False, seed=0, fovx_deg=60.0, native=True,
                  depth_only=False):
    """one train_single.py iteration on the bench scene (1M Gaussians at
    1080p, perturbed), wall time per step between synchronisations (the fused step never syncs).
    street=True: the Street-sparse iteration -- 4 training views cycled, the masked inverse-depth
    L1 (train_single.py:133-141, weight schedule 1.0 -> 0.01), the first 10k rows a locked skybox
    (:217-223), exposure and xyz lr schedules.  street=False: photometric loss only, one fixed
    view (round 1's number, kept as a labelled variant).  reference=True: the same step in the
    reference's torch formulation (oracle/train_torch_ref.py, a baseline leg).  native=True: the
    step as one gsr_train_step call (gs_train.native_step); False: issued from Python through the
    autograd API (gs_train.harness.TrainStep) -- the same kernels in the same order.  depth_only:
    every view a depth-only view (train_single.py:145-161: the depth-only loss, no photometric
    term, no exposure step)."""
    import torch
    from gs_train.harness import make_problem
    step_cls = None
    if native and not reference:
        from gs_train.native_step import NativeTrainStep as step_cls
    if reference:
        from train_torch_ref import ReferenceTrainStep as step_cls
    ts = make_problem(P, W, H, n_views=4 if street else 1, seed=seed, step_cls=step_cls, depth=street,
                      skybox_points=10_000 if street else 0, fovx_deg=fovx_deg, depth_only=4 if depth_only else 0)
    settle()
    for _ in range(warmup):
        ts.step()
    torch.cuda.synchronize()
    with quiet_gc():
        t0 = time.perf_counter()
        for _ in range(steps):
            ts.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
    del ts
    torch.cuda.empty_cache()
    return ms


def config3(a, dev, seed=0, ranks=None, spatial=False):
    """The config-3 stand-in (BASELINE.json configs[2]: train_single.py's whole loop per chunk; the
    example_dataset is absent): gs_train.chunk.TrainChunk over a synthetic Street-sparse chunk
    (street_chunk: cube faces along a street, LiDAR-like initial points, skybox + scaffold rows,
    depth-only views) with the native step, the default OptimizationParams schedule (densify /
    prune, opacity resets, SH increments, lr / depth-weight schedules) scaled to --chunk-iterations.
    Per-iteration device time from HIP events between iterations; the chunk's wall clock from
    after set-up to the last iteration."""
    import torch
    from diff_gaussian_rasterization import _C
    from gs_train.chunk import ChunkSchedule, TrainChunk, street_chunk
    from gs_train.native_step import NativeTrainStep
    n_it = a.chunk_iterations
    f = n_it / 30_000
    sched = ChunkSchedule(iterations=n_it)
    if n_it != 30_000:  # the same schedule compressed in time
        sched = ChunkSchedule(iterations=n_it, densification_interval=max(1, round(300 * f)),
                              opacity_reset_interval=max(1, round(3000 * f)), densify_from_iter=round(500 * f),
                              densify_until_iter=round(15_000 * f), sh_interval=max(1, round(1000 * f)))
    t_set = time.perf_counter()
    torch.manual_seed(seed)
    ts, info = street_chunk(NativeTrainStep, W=a.chunk_size, H=a.chunk_size, positions=a.chunk_positions,
                            n_truth=a.chunk_truth, n_init=a.chunk_init, iterations=n_it, device=dev)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_set

    from gs_train.chunk import view_psnr
    psnr0 = view_psnr(ts)
    tc = TrainChunk(ts, sched, spatial=bool(spatial))
    settle()
    evs, losses = [], {}
    # per iteration, for the attribution of the slowest ones: binning re-runs (capacity short), the
    # executor's buffer growths, the torch caching allocator's reserved bytes
    marks = []

    def cb(it, loss):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        evs.append(e)
        fs = _C.forward_stats()
        marks.append((it, fs["reruns"], ts.ctx_stats()["growths"], torch.cuda.memory_reserved(dev),
                      fs["fwd_split_frames"], fs["tb_split_frames"], fs["fwd_worker_giveups"],
                      int(getattr(getattr(ts, "_args", None), "image_index", -1)), int(getattr(ts, "last_K", 0))))
        if it % 1000 == 0 or it == 1:
            losses[it] = loss
    r0 = _C.forward_stats()
    torch.cuda.synchronize()
    _C.fwd_pool_stats(reset=True)
    if ranks is not None:
        ranks.barrier()
        torch.cuda.synchronize()
    with quiet_gc():
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        t0 = time.perf_counter()
        tc.run(callback=cb)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if ranks is not None:  # the job ends when the last rank's chunk does
            ranks.barrier()
            torch.cuda.synchronize()
            job_wall = time.perf_counter() - t0
    r1 = _C.forward_stats()
    pool = _C.fwd_pool_stats()
    per = np.array([start.elapsed_time(evs[0])] + [evs[i].elapsed_time(evs[i + 1]) for i in range(len(evs) - 1)])
    psnr1 = view_psnr(ts)
    # where a late iteration's time goes: the rasterizer's stages (HIP events) over 32 more steps
    # of the trained chunk (the view cycle continues; these steps are outside the timed run)
    _C.set_profiling(True)
    acc, nprof = {}, 32
    rel = []
    for _ in range(nprof):
        ts.step()
        for k_, v_ in _C.stage_times_ms().items():
            acc[k_] = acc.get(k_, 0.0) + v_ / nprof
        # the sparse Adam's relevant rows (nonzero opacity gradient, train_single.py:226)
        og = ts.grads["_opacity"] if hasattr(ts, "grads") else ts.g._opacity.grad
        if og is not None:
            rel.append((og != 0).float().mean())
    _C.set_profiling(False)
    relevant_frac = round(float(torch.stack(rel).mean()), 4) if rel else None
    late_K = int(ts.last_K)
    ev = tc.events
    # the slowest iterations and what ran in them (verdict r04: the 28-127 ms spike)
    ev_at = {e["iteration"]: e for e in ev}
    slow = []
    for i in np.argsort(per)[::-1][:10]:
        it, rr, gr, res, fsf, tbf, gup, view_k, kk = marks[i]
        prev = marks[i - 1] if i > 0 else (it - 1, r0["reruns"], 0, res, r0["fwd_split_frames"],
                                           r0["tb_split_frames"], r0["fwd_worker_giveups"], -1, 0)
        e = ev_at.get(it, {})
        # the view, its instance count and whether the frame's forward / tile-binning splits were armed
        # (the split gate arms them for 256 frames after a frame with long lists)
        slow.append({"iteration": int(it), "ms": round(float(per[i]), 3), "densify": "total" in e,
                     "reset": bool(e.get("reset")), "after_event": (it - 1) in ev_at,
                     "sh_increment": it % sched.sh_interval == 0,
                     "binning_rerun": rr > prev[1], "buffer_growths": gr - prev[2],
                     "torch_reserved_growth_mb": round((res - prev[3]) / 2 ** 20, 1),
                     "view": view_k, "K": kk, "fwd_split_armed": fsf > prev[4], "tb_split_armed": tbf > prev[5],
                     "fwd_worker_giveups": gup - prev[6], "event_ms": e.get("ms"), "event_densify_ms": e.get("ms_densify")})
    detail = {"slowest_iterations": slow, "iteration_ms_per_1000": [round(float(per[i:i + 1000].mean()), 3)
                                                                    for i in range(0, len(per), 1000)],
              "loss": {str(k): round(float(v), 5) for k, v in sorted(losses.items())},
              "P_trace": [[e["iteration"], e["P_after"]] for e in ev],
              "late_raster_stages_ms": {k_: round(v_, 4) for k_, v_ in acc.items()},
              "fwd_pool": pool, "executor_buffers": ts.ctx_stats()}
    blk = detail["iteration_ms_per_1000"]
    # the line keeps a summary (the driver's record holds only the tail of stdout); --detail-out the rest
    out = {"workload": f"train_single.py loop, synthetic Street-sparse chunk: {info['views']} views "
                       f"({info['depth_only_views']} depth-only) of {info['W']}x{info['H']}, {info['P_init']} initial "
                       f"Gaussians, {n_it} iterations, default schedule" + ("" if n_it == 30_000 else " compressed"),
           "spatial_rows": bool(spatial), "chunk_wall_s": round(wall, 3),
           "chunk_iterations_per_s": round(n_it / wall, 2), "setup_s": round(setup_s, 2),
           "iteration_ms": {"mean": round(float(per.mean()), 4), "median": round(float(np.median(per)), 4),
                            "p90": round(float(np.percentile(per, 90)), 4), "max": round(float(per.max()), 3),
                            "first_1000_mean": blk[0] if blk else None, "last_1000_mean": blk[-1] if blk else None},
           # [iteration, ms, events in it: d(ensify) r(eset) s(h increment)]
           # [iteration, ms, events in it: d(ensify) r(eset) s(h increment), host ms of its densify / reset]
           "slowest3": [[e["iteration"], e["ms"], ("d" if e["densify"] else "") + ("r" if e["reset"] else "") +
                         ("s" if e["sh_increment"] else ""), e["event_ms"]] for e in slow[:3]],
           "P_init": info["P_init"], "P_final": ts.g.P, "P_max": max([e["P_after"] for e in ev] + [info["P_init"]]),
           "densify_events": sum(1 for e in ev if "total" in e), "opacity_resets": sum(1 for e in ev if e.get("reset")),
           "event_s": round(tc.event_s, 3), "capacity_reruns": int(r1["reruns"] - r0["reruns"]),
           "final_sh_degree": ts.g.active_sh_degree,
           "loss_first_last": [round(float(losses[min(losses)]), 5), round(float(losses[max(losses)]), 5)] if losses else None,
           "train_view_psnr_db": {"before": psnr0, "after": psnr1},
           "late_frame_ms": {k_: round(v_, 3) for k_, v_ in acc.items() if v_ > 0},
           "late_tile_instances": late_K, "late_relevant_row_frac": relevant_frac,
           "fwd_pool_busy_frac": round(pool.get("busy_frac", 0.0), 4) if isinstance(pool.get("busy_frac"), float) else None,
           "seed": seed}
    if ranks is not None:
        out["job_wall_s"] = round(ranks.max(job_wall), 3)
    del ts, tc
    torch.cuda.empty_cache()
    return out, detail


def train_post_ms(a, dev):
    """One train_post.py iteration (train_post.py:69-198, gs_train.post.PostTrainStep): a random LOD
    limit, expand_to_size + get_interpolation_weights, the activation-fused render_post blend,
    rasterizer fwd+bwd of the cut at the chunk's view size, pretrained exposure, L1 + SSIM on
    image * alpha, skybox / anchor gradient zeroing, dense Adam -- on a synthetic hierarchy of
    --post-leaves leaves (~4/3 as many nodes).  Wall time per iteration between synchronisations
    (the cut length is read by the host every iteration, as in the reference)."""
    import torch
    from gs_train.post import synthetic_post_problem
    W = H = a.chunk_size
    torch.manual_seed(0)
    post = synthetic_post_problem(a.post_leaves, W, H, n_views=4, skybox=10_000, n_anchors=10_000, seed=1, device=dev)
    settle()
    for _ in range(5):
        post.step()
    torch.cuda.synchronize()
    cuts = []
    steps = max(10, a.train_steps)
    with quiet_gc():
        t0 = time.perf_counter()
        for _ in range(steps):
            post.step()
            cuts.append(post.last_cut)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
    out = {"ms": round(ms, 4), "steps": steps, "nodes": post.m.N, "cut_rows_mean": int(np.mean(cuts)),
           "cut_rows_max": int(np.max(cuts)), "width": W, "height": H,
           "workload": "train_post.py iteration on a synthetic hierarchy (Morton-grouped tree, 10k skybox rows last, "
                       "10k anchors): random LOD limit in [0.005, 0.1], cut + weights, fused blend over raw "
                       "parameters, rasterizer fwd+bwd, pretrained exposure, L1 + SSIM, locked-row zeroing, dense Adam"}
    del post
    torch.cuda.empty_cache()
    return out


def config5(a, dev):
    """render_hierarchy.py's per-frame work on a synthetic merged
    hierarchy (a real tree: Morton-grouped leaves, one Gaussian per node, ~50M nodes) --
    expand_to_size at the tau threshold (render_hierarchy.py:61-72), get_interpolation_weights
    (:76-85), render_post's LOD blend (fused kernel) and the forward render of the cut at 1080p
    (no_grad, do_depth), timed together per frame."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gaussian_hierarchy._C import expand_to_size, get_interpolation_weights
    from gs_train.hier import interpolate_cut
    from gs_train.synthetic import synthetic_lod_hierarchy, tau_threshold
    W, H = a.width, a.height
    h = synthetic_lod_hierarchy(a.c5_leaves, W, H, dev, seed=5, skybox=100_000, log_scale_mean=a.c5_log_scale)
    N = h["nodes"].shape[0]
    thr = tau_threshold(a.c5_tau, h["tanfovx"], W)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
    ri, pi, ni = (torch.zeros(N, dtype=torch.int32, device=dev) for _ in range(3))
    wts = torch.zeros(N, device=dev)
    kids = torch.zeros(N, dtype=torch.int32, device=dev)
    cam = t(h["campos"])
    cam_cpu = cam.cpu()
    zero3 = torch.zeros(3)
    rs = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=float(h["tanfovx"]), tanfovy=float(h["tanfovy"]), bg=t([0, 0, 0]),
        scale_modifier=1.0, viewmatrix=t(h["view"]).reshape(4, 4), projmatrix=t(h["proj"]).reshape(4, 4),
        sh_degree=3, campos=cam, prefiltered=False, debug=False, do_depth=True,
        render_indices=torch.empty(0, dtype=torch.int32), parent_indices=torch.empty(0, dtype=torch.int32),
        interpolation_weights=wts, num_node_kids=kids)
    raster = GaussianRasterizer(rs)

    def frame(split=None):
        with torch.no_grad():
            n = expand_to_size(h["nodes"], h["boxes"], thr, cam, zero3, ri, pi, ni)
            get_interpolation_weights(ni[:n], thr, h["nodes"], h["boxes"], cam_cpu, zero3, wts, kids)
            if split is not None:
                torch.cuda.synchronize()
                split.append(time.perf_counter())
            m, sc, rot, op, sh = interpolate_cut(h["means3D"], h["scales"], h["rotations"], h["opacities"], h["shs"],
                                                 ri[:n], pi, wts, h["skybox"])
            if split is not None:
                torch.cuda.synchronize()
                split.append(time.perf_counter())
            out = raster(means3D=m, means2D=torch.zeros_like(m), shs=sh, colors_precomp=None, opacities=op,
                         scales=sc, rotations=rot, cov3D_precomp=None)
            if split is not None:
                torch.cuda.synchronize()
                split.append(time.perf_counter())
            return n, out

    # the same frame through the rasterizer's own cut (non-empty render_indices: render_post's blend
    # fused into its preprocess and SH colour pass, the cut's rows read in place); the skybox rows
    # ride in render_indices with weight 1, as render_post blends them
    S = h["skybox"]
    sky = torch.arange(N - S, N, dtype=torch.int32, device=dev)
    ri2, pi2 = (torch.zeros(N + S, dtype=torch.int32, device=dev) for _ in range(2))
    w2 = torch.ones(N + S, device=dev)
    zero2 = torch.zeros(N + S, 3, device=dev)

    def frame_fused(split=None):
        with torch.no_grad():
            n = expand_to_size(h["nodes"], h["boxes"], thr, cam, zero3, ri2, pi2, ni)
            get_interpolation_weights(ni[:n], thr, h["nodes"], h["boxes"], cam_cpu, zero3, w2, kids)
            ri2[n:n + S] = sky
            pi2[n:n + S] = sky
            w2[n:n + S] = 1.0
            if split is not None:
                torch.cuda.synchronize()
                split.append(time.perf_counter())
                split.append(split[-1])  # no blend pass of its own
            rsf = rs._replace(render_indices=ri2[:n + S], parent_indices=pi2, interpolation_weights=w2)
            out = GaussianRasterizer(rsf)(means3D=h["means3D"], means2D=zero2[:N], shs=h["shs"], colors_precomp=None,
                                          opacities=h["opacities"], scales=h["scales"], rotations=h["rotations"],
                                          cov3D_precomp=None)
            if split is not None:
                torch.cuda.synchronize()
                split.append(time.perf_counter())
            return n, out

    from diff_gaussian_rasterization import _C

    def measure(fr):
        for _ in range(3):
            fr()
        torch.cuda.synchronize()
        nf = 10
        t0 = time.perf_counter()
        for _ in range(nf):
            n, (color, radii, _) = fr()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / nf * 1e3
        parts = []
        for _ in range(3):  # synced split, separate from the timed frames
            sp = [time.perf_counter()]
            fr(sp)
            parts.append([1e3 * (sp[i + 1] - sp[i]) for i in range(3)])
        parts = np.median(np.array(parts), 0)
        # the rasterizer's own stages for one more frame (HIP events on its stream)
        _C.set_profiling(True)
        fr()
        stages = {k: round(v, 4) for k, v in _C.stage_times_ms().items()}
        _C.set_profiling(False)
        return ms, n, radii, parts, stages

    ms, n, radii, parts, stages = measure(frame)
    fms, fn, fradii, fparts, fstages = measure(frame_fused)
    out = {"ms_per_frame": round(fms, 3), "raster_stages_ms": fstages, "fwd_mpix_s": round(W * H / fms / 1e3, 1),
           "nodes": N, "leaves": a.c5_leaves, "tau": a.c5_tau, "leaf_log_scale": a.c5_log_scale, "cut": fn,
           "rendered": fn + S, "visible": int((fradii > 0).sum().item()), "width": W, "height": H,
           "split_ms": {"cut_and_weights": round(float(fparts[0]), 3), "raster_fwd": round(float(fparts[2]), 3)},
           "workload": "expand_to_size + get_interpolation_weights + the rasterizer's own cut (render_indices / "
                       "parent_indices / interpolation_weights: the LOD blend fused into its preprocess and SH colour "
                       "pass), no_grad, do_depth",
           "render_post_order": {
               "ms_per_frame": round(ms, 3), "raster_stages_ms": stages, "cut": n,
               "split_ms": {"cut_and_weights": round(float(parts[0]), 3), "blend": round(float(parts[1]), 3),
                            "raster_fwd": round(float(parts[2]), 3)},
               "workload": "the same frame in render_post's order: expand_to_size + get_interpolation_weights + the "
                           "materialised LOD blend (interpolate_cut, one fused kernel) + the rasterizer forward of the "
                           "blended rows"},
           "data": "synthetic hierarchy generated on the device (Morton-grouped tree, branching 4, 100k skybox)"}
    del h, raster
    torch.cuda.empty_cache()
    return out


def kernel_source_sha():
    """Content hash of the kernel sources (csrc/, include/, the build flags): profiles/*_pmc.json
    record it (tools/pmc_summary.py), so a profile taken before the kernels changed is flagged
    stale instead of being reported as if it described the code that ran."""
    import hashlib
    h = hashlib.sha256()
    pkg = os.path.join(REPO, "street-sparse-3dgs_amd")
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.h")) +
                   glob.glob(os.path.join(REPO, "include", "*.h"))) + [os.path.join(pkg, "build_hip.py")]
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


_PROFILES = None


def _profiles():
    """Committed PMC summaries, newest first (profiles/r<round><letter>_pmc.json), each with
    whether it was taken from the kernel sources in this tree."""
    global _PROFILES
    if _PROFILES is None:
        sha = kernel_source_sha()
        _PROFILES = []
        for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")), reverse=True):
            try:
                d = json.load(open(f))
            except Exception:
                continue
            _PROFILES.append((os.path.basename(f), d, d.get("source_sha") == sha))
    return _PROFILES


def latest_profile_entry(kernel, field):
    """`field` of `kernel` (a stage name: render_bwd is the depth-gradient variant the bench runs)
    from the newest committed PMC summary that has it -- one taken from the current kernel
    sources if any -- as (value, file, current)."""
    found = None
    for name, d, cur in _profiles():
        e = d.get("kernels", {}).get(kernel, {})
        v = e.get(field) if "." not in field else e.get(field.split(".")[0], {}).get(field.split(".")[1])
        if v is None:
            continue
        if cur:
            return v, name, True
        if found is None:
            found = (v, name, False)
    return found if found else (None, None, False)


def latest_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary of the current sources
    (None when only a profile of older kernels exists)."""
    v, src, cur = latest_profile_entry(kernel, "hbm_bytes_per_launch")
    return (v if cur else None), src, cur


# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every 2 cycles at the
# 2.4 GHz engine clock (MI355X_MICROARCH.md, v_fma_f32 row)
VALU_PEAK_INSTR_S = 256 * 4 * 2.4e9 / 2
# Sustained issue rate of independent v_fma_f32 on the box, 8 waves per SIMD
# (tools/valu_bench.hip, profiles/r02e_valu_bench.txt): 947 G wave-instr/s -- the clock under full
# VALU load sits near 1.85 GHz, so 77% of the nominal figure above is the practical ceiling
# (v_exp_f32 / v_rcp_f32 issue at about a quarter of that rate; v_pk_fma_f32 adds only ~10% of
# fp32 throughput, so packed math is no lever)
VALU_SUSTAINED_INSTR_S = 947e9


def valu_roofline(kernel, ms):
    """Second roofline for the blend kernels, which are VALU-issue bound: wave-level VALU
    instructions per launch (SQ_INSTS_VALU from the committed rocprofv3 summary of the same
    kernel variant) over the live-measured launch time, against the issue peak."""
    instr, src, cur = latest_profile_entry(kernel, "sq.SQ_INSTS_VALU")
    if not instr or not ms or not cur:  # an instruction count of other kernel code says nothing
        return None
    ach = instr / (ms * 1e-3)
    return {"kernel": kernel, "bound": "valu-issue", "achieved": round(ach / 1e9, 2), "peak": VALU_PEAK_INSTR_S / 1e9,
            "unit": "G wave-instr/s", "frac": round(ach / VALU_PEAK_INSTR_S, 4),
            "sustained_peak": VALU_SUSTAINED_INSTR_S / 1e9, "frac_of_sustained": round(ach / VALU_SUSTAINED_INSTR_S, 4),
            "valu_instr_per_launch": instr, "avg_ms": round(ms, 5), "instr_source": src,
            "rocprof_avg_ms": rocprof_ms(kernel)}


def rocprof_ms(kernel):
    """The kernel's average duration in the committed rocprofv3 summary (the same command,
    --profile-steps).  The VALU-bound blend kernels run ~8% longer under the profiler than the
    same launches timed with HIP events here; the memory-bound kernels agree within ~2%
    (DESIGN.md section 4)."""
    us, _, cur = latest_profile_entry(kernel, "avg_us")
    return round(us / 1e3, 5) if us and cur else None


def log(msg):
    """Progress on stderr (a long default run keeps writing while it works)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def spawn_ranks(a):
    """bench.py --gpus N run directly (no WORLD_SIZE): start N fresh rank processes through
    torch.distributed.run -- one process per GPU, as the driver launches it -- before this process
    touches the GPU, and exit with their status.  Mirrors the reference's one-process-per-chunk
    fan-out (scripts/full_train.py:171-232, scripts/train_chunk.slurm:5-7)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


class Ranks:
    """Process-group helpers: barrier, MAX / gather of host floats (gloo on CPU tensors when the
    ranks share one GPU, RCCL otherwise)."""

    def __init__(self, world, rank, share, dev, pg=None):
        self.world, self.rank, self.share, self.dev = world, rank, share, dev
        self.pg = world > 1 if pg is None else pg  # a process group exists (GSR_BENCH_FORCE_PG: also at N = 1)

    def barrier(self):
        if self.pg:
            import torch.distributed as dist
            dist.barrier()

    def gather(self, x):
        if not self.pg:
            return [float(x)]
        import torch
        import torch.distributed as dist
        d = "cpu" if self.share else self.dev
        t = torch.zeros(self.world, dtype=torch.float64, device=d)
        t[self.rank] = float(x)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return [float(v) for v in t.cpu()]

    def max(self, x):
        return max(self.gather(x))


def rasterizer_for(s, W, H, deg, dev, debug=False):
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
    rs = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=float(s["tanfovx"]), tanfovy=float(s["tanfovy"]), bg=t(s["bg"]),
        scale_modifier=1.0, viewmatrix=t(s["view"]).reshape(4, 4), projmatrix=t(s["proj"]).reshape(4, 4),
        sh_degree=deg, campos=t(s["campos"]), prefiltered=False, debug=debug, do_depth=True,
        render_indices=torch.empty(0, dtype=torch.int32), parent_indices=torch.empty(0, dtype=torch.int32),
        interpolation_weights=torch.empty(0, device=dev), num_node_kids=torch.empty(0, dtype=torch.int32, device=dev))
    return rs, GaussianRasterizer(rs)


def fwd_bwd_step(raster, inp, gcol, ginv):
    import torch
    leaves = list(inp.values())

    def step():
        for v in leaves:
            v.grad = None
        color, radii, invd = raster(**inp)
        torch.autograd.backward([color, invd], [gcol, ginv])
        return radii
    return step


@contextlib.contextmanager
def quiet_gc():
    """Python's cyclic collector kept out of a timed region: every object alive is frozen (gc.freeze),
    so a generation-2 pass over the interpreter's ~10^5 long-lived objects (torch's modules, the
    synthetic scene's builders) cannot land inside the timed steps -- a few-ms host stall that showed
    up as a 10% low sample now and then.  No gc.collect() here: a collection right before the timed
    steps made the next ~20 steps 7% slower on the GPU (0.66 -> 0.71 ms per step, tools/timing_ab.py
    r06i: the buffers it frees change where the steps' allocations land); settle() collects once,
    before the pre-warm.  Collection stays enabled; the objects the steps create are collected as usual."""
    import gc
    gc.freeze()
    try:
        yield
    finally:
        gc.unfreeze()


def settle():
    """One full collection after the set-up, before any warm-up (see quiet_gc)."""
    import gc
    gc.collect()


def timed(step, steps, warmup, ranks, per_step=None, host=None, per_call=None):
    """W untimed steps, then exactly `steps` steps bracketed by barrier + synchronize on both sides;
    the MAX over ranks of the elapsed seconds.  per_step (a list): receives each timed step's device
    duration in ms -- HIP events recorded on the current stream between consecutive steps (no
    synchronisation inside the timed region).  host (a dict): the host's side of the same steps --
    the time each step() call took to return (perf_counter, ms) and the part of it the forward spent
    waiting for K (gsr_forward_stats' k_wait_ns), so a line shows whether the host or the GPU bounds
    the step."""
    import torch
    from diff_gaussian_rasterization import _C
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ranks.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if per_step is not None else None
    ht = [0.0] * (steps + 1)
    with quiet_gc():
        k0 = _C.forward_stats()["k_wait_ns"] if host is not None else 0
        t0 = time.perf_counter()
        if ev is not None:
            ev[0].record()
        ht[0] = time.perf_counter()
        for i in range(steps):
            step()
            ht[i + 1] = time.perf_counter()
            if ev is not None:
                ev[i + 1].record()
        k1 = _C.forward_stats()["k_wait_ns"] if host is not None else 0
        torch.cuda.synchronize()
        ranks.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    if ev is not None:
        per_step.extend(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
    if per_call is not None:  # the timed steps' own host call times (ms)
        per_call.extend(float(v) for v in np.diff(np.asarray(ht)) * 1e3)
    if host is not None:
        call = np.diff(np.asarray(ht)) * 1e3
        kw = (k1 - k0) / max(1, steps) * 1e-6
        host.update({"step_call_ms_median": round(float(np.median(call)), 5),
                     "step_call_ms_mean": round(float(call.mean()), 5),
                     "step_call_ms_max": round(float(call.max()), 5),
                     "k_wait_ms_mean": round(kw, 5),
                     "busy_ms_mean": round(float(call.mean()) - kw, 5),
                     "source": "perf_counter around each timed step() call; k_wait from gsr_forward_stats[5] "
                               "(the forward's wait for num_rendered); busy = call - k_wait"})
    return ranks.max(el)


def dispersion(ms):
    """Median / p10 / p90 / min / max of the timed steps' per-step times (ms): SURVEY.md 8(d) asks for
    the median; the mean comes from the wall clock.  The times are each step() call's host duration:
    the step is GPU-bound (the forward waits for its frame's K, which the GPU produces one frame after
    the previous), so in steady state the calls follow the GPU's frames; per-step HIP events would
    put a marker packet (~7 us) between every two steps."""
    if not ms:
        return None
    a = np.asarray(ms, np.float64)
    return {"median_ms": round(float(np.median(a)), 5), "p10_ms": round(float(np.percentile(a, 10)), 5),
            "p90_ms": round(float(np.percentile(a, 90)), 5), "min_ms": round(float(a.min()), 5),
            "max_ms": round(float(a.max()), 5), "n": int(a.size),
            "source": "perf_counter around each timed step() call (GPU-bound steps: the host waits for each frame's K)"}


class ClockProbe:
    """Shader clock, power and temperature of the bench's GPU (amdsmi GPU metrics; None where the
    library or the metric is unavailable): the blend kernels are VALU-issue bound, so their times
    scale with the clock the box runs at, and a line without it cannot be compared with another
    box's.  read() is one sample; sample_while(fn) samples every ~10 ms on a thread while fn runs
    (used around untimed steps only)."""
    KEYS = ("current_gfxclk", "average_gfxclk_frequency", "current_uclk", "current_socket_power",
            "average_socket_power", "temperature_hotspot", "gfx_activity")

    def __init__(self, dev):
        self.h = None
        self.err = None
        if os.environ.get("GSR_BENCH_NO_SMI") == "1":  # A/B: the bench without amdsmi in the process
            self.err = "disabled (GSR_BENCH_NO_SMI=1)"
            return
        try:
            import amdsmi
            import torch
            amdsmi.amdsmi_init()
            pr = torch.cuda.get_device_properties(dev)
            want = (int(pr.pci_domain_id), int(pr.pci_bus_id), int(pr.pci_device_id))
            for h in amdsmi.amdsmi_get_processor_handles():
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
                dom, bus, rest = bdf.split(":")
                if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                    self.h = h
                    break
            if self.h is None:
                self.err = "no amdsmi handle with the device's PCI address"
            self.amdsmi = amdsmi
        except Exception as e:  # pragma: no cover - depends on the box
            self.err = f"{type(e).__name__}: {e}"[:160]

    def read(self):
        if self.h is None:
            return None
        try:
            m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        except Exception as e:  # pragma: no cover
            self.err = f"{type(e).__name__}: {e}"[:160]
            return None
        out = {}
        for k in self.KEYS:
            v = m.get(k)
            if isinstance(v, (list, tuple)):  # per-XCD clocks on some parts
                v = [x for x in v if isinstance(x, (int, float)) and x < 0xFFFF]
                v = max(v) if v else None
            if isinstance(v, (int, float)) and v < 0xFFFFFFFF:
                out[k] = v
        clks = m.get("current_gfxclks")
        if isinstance(clks, (list, tuple)):
            c = [x for x in clks if isinstance(x, (int, float)) and 0 < x < 0xFFFF]
            if c:
                out["current_gfxclks_min_max"] = [min(c), max(c)]
        return out

    def sample_while(self, fn):
        import threading
        samples, stop = [], threading.Event()

        def loop():
            while not stop.is_set():
                r = self.read()
                if r:
                    samples.append(r)
                stop.wait(0.01)
        th = threading.Thread(target=loop, daemon=True)
        if self.h is not None:
            th.start()
        try:
            fn()
        finally:
            stop.set()
            if self.h is not None:
                th.join()
        if not samples:
            return None
        summ = {"samples": len(samples)}
        for k in ("current_gfxclk", "current_socket_power", "temperature_hotspot"):
            v = [x[k] for x in samples if k in x]
            if v:
                summ[k + "_median"] = float(np.median(v))
                summ[k + "_max"] = float(np.max(v))
        return summ


SECONDARY_LEGS = ("train_step", "config4", "street_frame", "coarse_debug", "train_post_step", "config3_proxy",
                  "config5", "cpu_baseline_torch", "psnr_vs_oracle")
PROSE_KEYS = ("workload", "data", "source", "collectives", "reference")
MOVED_KEYS = {
    "config3_proxy": ("setup_s", "P_init", "P_max", "capacity_reruns", "final_sh_degree", "loss_first_last",
                      "train_view_psnr_db", "late_tile_instances", "late_relevant_row_frac", "seed",
                      "variant.iteration_ms", "variant.slowest3", "variant.P_final", "variant.train_view_psnr_db"),
    "config5": ("nodes", "leaves", "tau", "leaf_log_scale", "width", "height", "visible", "rendered", "fwd_mpix_s",
                "render_post_order.cut", "render_post_order.split_ms"),
    "street_frame": ("stages_ms", "tiles", "level1_entries"),
    "cpu_baseline_torch": ("sample",),
    "config4": ("visible_rank0", "tile_instances_rank0"),
}


def compact_legs(out, detail):
    """Keep the line short (the driver's record holds only the last ~8 kB of stdout, and the metric's
    diagnostics come last): the secondary legs' prose fields (workload descriptions, data and source
    notes) move to the detail file, keyed by their path; the numbers stay in the line."""
    prose = detail.setdefault("prose", {})

    def strip(d, path):
        for k in list(d):
            if k in PROSE_KEYS and isinstance(d[k], str):
                prose[path + "." + k] = d.pop(k)
            elif isinstance(d[k], dict):
                strip(d[k], path + "." + k)
    for leg in SECONDARY_LEGS:
        if isinstance(out.get(leg), dict):
            strip(out[leg], leg)
    c5 = out.get("config5")
    if isinstance(c5, dict) and isinstance(c5.get("render_post_order"), dict):
        detail["config5_render_post_order_stages_ms"] = c5["render_post_order"].pop("raster_stages_ms", None)
    # descriptive numbers of the secondary legs (sizes, schedules, per-stage splits) to the detail file
    # too: the line stays under ~5 kB with the metric's diagnostics last
    if isinstance(c5, dict) and isinstance(c5.get("raster_stages_ms"), dict):  # a forward-only frame's zero stages
        c5["raster_stages_ms"] = {k: v for k, v in c5["raster_stages_ms"].items() if v}
    moved = detail.setdefault("moved", {})
    for leg, keys in MOVED_KEYS.items():
        d = out.get(leg)
        if not isinstance(d, dict):
            continue
        for k in keys:
            sub = d
            path = k.split(".")
            for part in path[:-1]:
                sub = sub.get(part) if isinstance(sub, dict) else None
            if isinstance(sub, dict) and path[-1] in sub:
                moved[leg + "." + k] = sub.pop(path[-1])


def prewarm(step, probe, max_s=0.6, min_s=0.25, tol=0.03, burst=20):
    """Time-based pre-warm before the counted warm-ups: one step (the process's first-call set-up:
    code objects, buffers), then the bench's own fwd+bwd step in bursts of `burst` steps
    (synchronised), the shader clock read after each, for at least `min_s` and until the clock has
    settled -- the last two readings within `tol` of each other and of the highest seen -- or `max_s`
    has passed.  Measured on one box (tools/kstamp.py, r06e): after 5 warm-up steps the next 20 steps
    average 0.707 ms, after 50 or more 0.664-0.668 ms -- the driver's 20 timed steps after its 5
    warm-ups sat on that ramp.  Returns what it did, for the line."""
    import torch
    if max_s <= 0:
        return {"ms": 0.0, "steps": 0}
    t_init = time.perf_counter()
    step()
    torch.cuda.synchronize()
    init_ms = (time.perf_counter() - t_init) * 1e3
    clks, n = [], 1
    t0 = time.perf_counter()
    settled = False
    while True:
        for _ in range(burst):
            step()
        torch.cuda.synchronize()
        n += burst
        r = probe.read()
        if r and r.get("current_gfxclk"):
            clks.append(float(r["current_gfxclk"]))
        el = time.perf_counter() - t0
        if el >= max_s:
            break
        if el >= min_s:
            hi = max(clks) if clks else 0.0
            settled = len(clks) < 2 or (clks[-1] >= (1 - tol) * hi and abs(clks[-1] - clks[-2]) <= tol * hi)
            if settled:
                break
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "first_step_ms": round(init_ms, 1), "steps": n,
            "settled": settled, "gfxclk_samples_mhz": clks[-3:],
            "rule": f"one set-up step, then bursts of {burst} steps for >= {min_s} s until two clock readings are "
                    f"within {tol:.0%} of each other and of the highest seen, cap {max_s} s"}


def stage_profile(step, n):
    """Per-stage device time (HIP events on the rasterizer's stream) averaged over n extra steps."""
    from diff_gaussian_rasterization import _C
    _C.set_profiling(True)
    acc = {}
    for _ in range(max(1, n)):
        step()
        for k, v in _C.stage_times_ms().items():
            acc[k] = acc.get(k, 0.0) + v
    _C.set_profiling(False)
    return {k: v / max(1, n) for k, v in acc.items()}


def frame_workload(rs, inp, W, H, deg, dev):
    """Pv, K and the level-1 entry count P1 of the frame (one raw forward, no_grad)."""
    import torch
    from diff_gaussian_rasterization import _C
    with torch.no_grad():
        raw = _C.rasterize_gaussians(rs.bg, inp["means3D"], torch.empty(0, device=dev), inp["opacities"],
                                     inp["scales"], inp["rotations"], 1.0, torch.empty(0, device=dev), rs.viewmatrix,
                                     rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W, inp["shs"], deg, rs.campos, False,
                                     False, rs.render_indices, rs.parent_indices, rs.interpolation_weights,
                                     rs.num_node_kids, True)
        fs = _C.frame_stats(raw[4], inp["means3D"].shape[0], H, W)
    return dict(K=int(raw[0]), Pv=int((raw[3] > 0).sum().item()), P1=fs["level1_entries"],
                tb_split_items=fs["tb_split_items"], max_sb_list=fs["max_sb_list"])


def config4(a, ranks, dev):
    """one synthetic 500k-Gaussian chunk per rank (seed = chunk id =
    rank), rasterized at 1080p -- the product's one-chunk-per-GPU sharding, no data-path
    collective -- and the Street-sparse train step on that chunk.  Aggregate Mpix/s over all ranks
    and every rank's train-step ms (at N = 1 this is config 2's train step)."""
    import torch
    P4, W, H, deg = 500_000, a.width, a.height, a.sh_degree
    s, inp, gcol, ginv = make_inputs(P4, W, H, deg, seed=ranks.rank, device=dev)
    rs, raster = rasterizer_for(s, W, H, deg, dev)
    el = timed(fwd_bwd_step(raster, inp, gcol, ginv), a.steps, a.warmup, ranks)
    wl = frame_workload(rs, inp, W, H, deg, dev)
    del inp, raster
    torch.cuda.empty_cache()
    tr = train_step_ms(P4, W, H, a.train_steps, 5, dev, seed=ranks.rank) if a.train_steps > 0 else None
    per_rank = ranks.gather(tr) if tr is not None else None
    return {"workload": f"{ranks.world} chunk(s) of {P4} Gaussians (seed = chunk id), one per rank, fwd+bwd at "
                        f"{W}x{H} SH degree {deg} do_depth; train step = the Street-sparse iteration on the chunk",
            "value": round(ranks.world * W * H * a.steps / el / 1e6, 3), "unit": "Mpix/s", "n_gpus": ranks.world,
            "ms_per_step": round(el / a.steps * 1e3, 4), "visible_rank0": wl["Pv"], "tile_instances_rank0": wl["K"],
            "train_step_ms_per_rank": [round(v, 4) for v in per_rank] if per_rank else None,
            "train_step_ms_max": round(max(per_rank), 4) if per_rank else None,
            "scaling": "weak", "collectives": "none on the data path (barrier + MAX of the elapsed time only)"}


def street_frame(a, dev):
    """The Street-sparse training frame: a 1536x1536 cube face with a 90 deg field of view
    (ss_utils/generate_colmap_calibration.py:306-308,476-479,572: SIMPLE_PINHOLE, f = size / 2;
    below the 1600-px rescale of utils/camera_utils.py:64-81), 1M synthetic Gaussians: fwd+bwd
    Mpix/s with its stage split, and the train step with 4 cycled views of that size."""
    import torch
    W = H = 1536
    P, deg = a.gaussians, a.sh_degree
    s, inp, gcol, ginv = make_inputs(P, W, H, deg, seed=0, device=dev, fovx_deg=90.0)
    rs, raster = rasterizer_for(s, W, H, deg, dev)
    step = fwd_bwd_step(raster, inp, gcol, ginv)
    el = timed(step, a.steps, a.warmup, Ranks(1, 0, False, dev))
    stages = stage_profile(step, 3)
    wl = frame_workload(rs, inp, W, H, deg, dev)
    del inp, raster
    torch.cuda.empty_cache()
    out = {"workload": f"rasterizer fwd+bwd, {P} Gaussians, SH degree {deg}, {W}x{H} (90 deg fov), do_depth",
           "value": round(W * H * a.steps / el / 1e6, 3), "unit": "Mpix/s", "ms_per_step": round(el / a.steps * 1e3, 4),
           "visible": wl["Pv"], "tile_instances": wl["K"], "level1_entries": wl["P1"],
           "tiles": ((W + 15) // 16) * ((H + 15) // 16), "stages_ms": {k: round(v, 5) for k, v in stages.items()}}
    if a.train_steps > 0:
        out["train_step_ms"] = round(train_step_ms(P, W, H, a.train_steps, 5, dev, fovx_deg=90.0), 4)
    return out


def coarse_debug(a, dev):
    """render_coarse's frames: debug forced on (gaussian_renderer/__init__.py:341), SH degree 1
    (shs (P, 4, 3), train_coarse.py:31), 500k Gaussians at 1080p.  fwd+bwd ms with debug off, with
    debug on (device-side input snapshots and a synchronize + error check after every stage), and
    with upstream's host snapshots (GSR_DEBUG_HOST_SNAPSHOT=1: every input deep-copied to the host
    before each forward and backward, diff_gaussian_rasterization/__init__.py:26-28,53-54,90-91)."""
    import torch
    P, W, H, deg = 500_000, a.width, a.height, 1
    s, inp, gcol, ginv = make_inputs(P, W, H, deg, seed=0, device=dev)
    one = Ranks(1, 0, False, dev)
    out = {"workload": f"render_coarse frame: {P} Gaussians, SH degree 1 (M = 4), {W}x{H}, fwd+bwd, do_depth"}
    steps = max(5, a.steps // 2)
    for name, debug, host in (("debug_off_ms", False, False), ("debug_ms", True, False),
                              ("debug_host_snapshot_ms", True, True)):
        if host:
            os.environ["GSR_DEBUG_HOST_SNAPSHOT"] = "1"
        try:
            _, raster = rasterizer_for(s, W, H, deg, dev, debug=debug)
            el = timed(fwd_bwd_step(raster, inp, gcol, ginv), steps, 3, one)
        finally:
            os.environ.pop("GSR_DEBUG_HOST_SNAPSHOT", None)
        out[name] = round(el / steps * 1e3, 4)
    del inp
    torch.cuda.empty_cache()
    return out


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a))
    if a.metric_only:
        a.train_steps, a.no_config5, a.no_street, a.no_config4, a.no_cpu_baseline = 0, True, True, True, True
        a.no_coarse_debug = a.no_config3 = True
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GSR_BENCH_SHARE_GPU=1 (rehearsal of the multi-rank path on a one-GPU box): every rank on
    # device 0 and gloo for the barriers / timing reduction (RCCL refuses two ranks on one device).
    # The driver's runs use one GPU per rank and RCCL.
    share = os.environ.get("GSR_BENCH_SHARE_GPU") == "1"
    # GSR_BENCH_FORCE_PG=1 (launched by torch.distributed.run): the RCCL process group, barriers and
    # timing all-reduce even for one rank -- the collective path the driver's multi-GPU runs take,
    # exercised on a one-GPU box (RCCL refuses two ranks on one device)
    use_pg = world > 1 or (os.environ.get("GSR_BENCH_FORCE_PG") == "1" and "RANK" in os.environ)
    if use_pg:
        torch.cuda.set_device(0 if share else local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", 0 if share or world == 1 else local)
    ranks = Ranks(world, rank, share, dev, pg=use_pg)

    from diff_gaussian_rasterization import _C as _gsr
    if a.bwd_seg is not None:
        _gsr.set_bwd_segment(a.bwd_seg)
    if a.fwd_seg is not None:
        _gsr.set_fwd_segment(a.fwd_seg)
    bwd_seg = _gsr.set_bwd_segment(0)
    _gsr.set_bwd_segment(bwd_seg)
    fwd_seg = _gsr.set_fwd_segment(0)
    _gsr.set_fwd_segment(fwd_seg)
    P, W, H, deg = a.gaussians, a.width, a.height, a.sh_degree
    s, inp, gcol, ginv = make_inputs(P, W, H, deg, seed=rank, device=dev)
    rs, raster = rasterizer_for(s, W, H, deg, dev)
    step = fwd_bwd_step(raster, inp, gcol, ginv)
    leaves = list(inp.values())

    if a.diag:
        for _ in range(a.warmup):
            step()
        for it in range(5):
            for v in leaves:
                v.grad = None
            torch.cuda.synchronize()
            t_a = time.perf_counter()
            color, radii, invd = raster(**inp)
            torch.cuda.synchronize()
            t_b = time.perf_counter()
            torch.autograd.backward([color, invd], [gcol, ginv])
            torch.cuda.synchronize()
            t_c = time.perf_counter()
            print(f"diag step {it}: fwd {1e3 * (t_b - t_a):.3f} ms  bwd {1e3 * (t_c - t_b):.3f} ms", file=sys.stderr)
        ms = torch.cuda.memory_stats(dev)
        print("diag alloc:", {k: ms.get(k) for k in ("num_alloc_retries", "num_device_alloc", "num_device_free",
                                                      "reserved_bytes.all.current", "allocated_bytes.all.peak")},
              file=sys.stderr)
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(18)
    log("metric: timing")
    settle()
    probe = ClockProbe(dev)
    per_step = []
    host_side = {}
    clk_idle = probe.read()
    pw = prewarm(step, probe, max_s=a.prewarm_s, min_s=min(0.25, a.prewarm_s))
    clk_before = probe.read()
    pw["gfxclk_at_timed_start"] = (clk_before or {}).get("current_gfxclk")
    # the timed region carries no per-step event records: each is a marker packet on the stream, and
    # a marker costs ~7 us of idle between the kernels around it (tools/kstamp.py, r06e)
    elapsed = timed(step, a.steps, a.warmup, ranks, host=host_side, per_call=per_step)
    clk_after = probe.read()

    # the clock under the bench's load: sampled over ~400 more (untimed) steps
    def burst():
        for _ in range(400):
            step()
        torch.cuda.synchronize()
    clk_load = probe.sample_while(burst)

    # per-stage device time with HIP events on the rasterizer's stream (separate, untimed steps)
    stages = stage_profile(step, a.profile_steps)

    # workload statistics for the algorithmic-bytes model (P1 measured: gsr_frame_stats)
    wl = frame_workload(rs, inp, W, H, deg, dev)
    K, Pv, P1 = wl["K"], wl["Pv"], wl["P1"]
    # live rows (nonzero accumulated sums) of the frame: the rows whose means3D gradient is nonzero
    # after the last step
    g3 = inp["means3D"].grad
    Pl = int((g3 != 0).any(dim=1).sum().item()) if g3 is not None else None
    T = ((W + 15) // 16) * ((H + 15) // 16)
    npix = W * H
    abytes = algorithmic_bytes(P, Pv, K, T, npix, P1, M=inp["shs"].shape[1], Pl=Pl)
    strict_8d = 44 * K + 24 * npix + 40 * Pv
    serial_ms = sum(v for k, v in stages.items() if k not in OVERLAPPED_STAGES)
    dom = max(stages, key=lambda k: stages[k]) if stages else "render_bwd"
    dom_ms = stages.get(dom, 0.0)
    achieved = abytes[dom] / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    traffic, traffic_src, traffic_cur = latest_traffic(dom)
    rp_ms = rocprof_ms(dom)

    ms_per_step = elapsed / a.steps * 1e3
    value = world * npix * a.steps / elapsed / 1e6
    strict_frac = strict_8d / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if dom == "render_bwd" and dom_ms > 0 else None
    zero_rows = (56 + 12 * inp["shs"].shape[1]) * P
    out = {
        "metric": "fwd+bwd Mpix/s at 1080p (1M Gaussians)",  # + "train_step" ms below
        "value": round(value, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded Gaussians in the frustum, SURVEY.md 8(d); one chunk per rank, seed = rank)",
        "config": {"workload": f"rasterizer fwd+bwd, {P} Gaussians, SH degree {deg}, {W}x{H}, do_depth",
                   "gaussians": P, "width": W, "height": H, "sh_degree": deg, "visible": Pv, "tile_instances": K,
                   "level1_entries": P1, "max_sb_list": wl["max_sb_list"],
                   "tb_split_items": wl["tb_split_items"], "live_rows": Pl, "tiles": T, "bwd_segment": bwd_seg, "fwd_segment": fwd_seg,
                   "parallelism": f"chunk-per-gpu x{world}"},
        # frac: SURVEY.md 8(d)'s algorithmic bytes of the dominant kernel (render_bwd: 44 K + 24 Npix +
        # 40 Pv) / its HIP-event time measured here; frac_rocprof: the same bytes / the average duration
        # in the committed rocprofv3 summary of these kernel sources (profiles/, null when no summary
        # of the current sources is committed); frac_with_zero_rows: also counting the dense zero
        # gradient rows render_bwd's waves write (8(d) books them under preprocess-bwd)
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "algorithmic_bytes": abytes[dom], "avg_ms": round(dom_ms, 5),
                     "traffic_source": traffic_src, "profile_is_current": traffic_cur, "rocprof_avg_ms": rp_ms,
                     "frac_rocprof": round(abytes[dom] / (rp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if rp_ms else None,
                     "kernel_source_sha": kernel_source_sha(),
                     "frac_strict_8d": round(strict_frac, 5) if strict_frac is not None else None,
                     "frac_with_zero_rows": round((abytes[dom] + zero_rows) / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                     if dom == "render_bwd" and dom_ms > 0 else None},
    }
    diag = {
        "valu_roofline": [{k_: r[k_] for k_ in ("kernel", "achieved", "unit", "frac_of_sustained",
                                                 "valu_instr_per_launch", "avg_ms", "rocprof_avg_ms")}
                          for r in (valu_roofline(k, stages.get(k)) for k in ("render_bwd", "render_fwd")) if r],
        "stage_bytes": {k: int(v) for k, v in abytes.items()},
        # stages on the main stream (sh_color overlaps the sort / binning on a side stream)
        "pipeline_roofline": {"algorithmic_bytes": sum(abytes.values()),
                              "frac": round(sum(abytes.values()) / (serial_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                              if serial_ms > 0 else None},
        "stages_ms": {k: round(v, 5) for k, v in stages.items()},
        "step_dispersion": dispersion(per_step),
        "host_issue": host_side,
        "gpu_clock": {"idle_mhz": (clk_idle or {}).get("current_gfxclk"),
                      "timed_start_mhz": (clk_before or {}).get("current_gfxclk"),
                      "timed_end_mhz": (clk_after or {}).get("current_gfxclk"),
                      "under_load_median_mhz": (clk_load or {}).get("current_gfxclk_median"),
                      "under_load_power_w": (clk_load or {}).get("current_socket_power_median"),
                      "under_load_hotspot_c_max": (clk_load or {}).get("temperature_hotspot_max"),
                      "source": "amdsmi GPU metrics", "error": probe.err},
        "prewarm": pw,
    }
    detail = {"gpu_clock": {"idle": clk_idle, "before": clk_before, "after": clk_after, "under_load": clk_load}}
    del step, raster
    if a.train_steps > 0:
        log("train step")
        from diff_gaussian_rasterization import _C as _Cstats
        r0 = _Cstats.forward_stats()
        tr = {"ms": round(train_step_ms(P, W, H, a.train_steps, 5, dev, seed=rank), 4),
              "workload": f"Street-sparse train_single.py iteration on the bench scene ({P} Gaussians, {W}x{H}, 4 views "
                          f"cycled): render, exposure, 0.8 L1 + 0.2 (1 - SSIM) + masked inverse-depth L1, backward "
                          f"(depth gradient on), densify stats, exposure Adam, skybox lock (10k rows), sparse Adam, "
                          f"scale clamp; one native gsr_train_step call per step (python_driven_ms: the same step "
                          f"issued from Python through the autograd API)",
              "steps": a.train_steps}
        r1 = _Cstats.forward_stats()
        tr["binning_reruns"] = r1["reruns"] - r0["reruns"]
        tr["python_driven_ms"] = round(train_step_ms(P, W, H, a.train_steps, 5, dev, seed=rank, native=False), 4)
        tr["photo_only_fixed_view_ms"] = round(train_step_ms(P, W, H, a.train_steps, 5, dev, street=False), 4)
        tr["depth_only_view_ms"] = round(train_step_ms(P, W, H, a.train_steps, 5, dev, seed=rank, depth_only=True), 4)
        if a.train_baseline:
            tr["reference_structured_ms"] = round(train_step_ms(P, W, H, a.train_steps, 5, dev, reference=True), 4)
        out["train_step"] = tr
    if not a.no_config4:
        log("config 4")
        out["config4"] = config4(a, ranks, dev)
        if world == 1 and out["config4"]["train_step_ms_max"] is not None and "train_step" in out:
            out["train_step"]["config2_500k_ms"] = out["config4"]["train_step_ms_max"]
    if world == 1 and not a.no_street:
        log("street frame")
        out["street_frame"] = street_frame(a, dev)
    if world == 1 and not a.no_coarse_debug:
        log("render_coarse debug mode")
        out["coarse_debug"] = coarse_debug(a, dev)
    if world == 1 and a.train_steps > 0 and a.post_leaves > 0:
        log("train_post step")
        out["train_post_step"] = train_post_ms(a, dev)
    if world == 1 and not a.no_config3:
        log("config 3 stand-in: train_single.py loop on a synthetic street chunk")
        out["config3_proxy"], detail["config3"] = config3(a, dev, spatial=bool(a.chunk_spatial))
        if not a.no_chunk_spatial_variant:
            log("config 3 stand-in, rows in the other order")
            v, detail["config3_variant"] = config3(a, dev, spatial=not a.chunk_spatial)
            out["config3_proxy"]["variant"] = {k_: v[k_] for k_ in ("spatial_rows", "chunk_wall_s", "iteration_ms",
                                                                      "slowest3", "P_final", "train_view_psnr_db")}
    if not a.no_config4 and not a.no_config3:
        # config 4 as the product runs it (scripts/full_train.py:171-232): one whole chunk per GPU --
        # every rank trains its own synthetic street chunk (seed = chunk id = rank) through the
        # train_single.py loop, no collective on the data path.  At N = 1 the chunk is config 3's run.
        log("config 4: one whole chunk per rank")
        one = out.get("config3_proxy") if world == 1 else config3(a, dev, seed=rank, ranks=ranks,
                                                                   spatial=bool(a.chunk_spatial))[0]
        if one is not None:
            walls = ranks.gather(one["chunk_wall_s"])
            job = one.get("job_wall_s", one["chunk_wall_s"])
            out["config4"]["chunks"] = {
                "workload": f"{world} synthetic street chunk(s), one per rank (seed = rank), {a.chunk_iterations} "
                            f"train_single.py iterations each ({one['workload']})",
                "chunk_iterations_per_s": round(world * a.chunk_iterations / job, 2), "unit": "chunk-iterations/s",
                "job_wall_s": job, "chunk_wall_s_per_rank": walls, "n_gpus": world, "scaling": "weak",
                "P_final_rank0": one["P_final"], "collectives": "none on the data path (barriers + MAX of the walls)"}
    if world == 1 and not a.no_config5:
        log("config 5")
        out["config5"] = config5(a, dev)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        log("cpu baselines")
        out["cpu_baseline"], st = cpu_baseline(s, P, W, H, deg)
        out["cpu_baseline_torch"] = cpu_baseline_torch()
        with torch.no_grad():
            color, _, invd = raster_again(s, inp, W, H, deg, dev)
        out["psnr_vs_oracle"] = psnr_vs_oracle(color, invd, st)
    out["process_group"] = dist.get_backend() if use_pg else None
    # the metric's own diagnostics last: the driver's record keeps only the tail of stdout
    compact_legs(out, detail)
    for k_ in ("step_dispersion", "host_issue", "prewarm"):
        for p_ in ("source", "rule"):
            if isinstance(diag.get(k_), dict) and p_ in diag[k_]:
                detail.setdefault("prose", {})[k_ + "." + p_] = diag[k_].pop(p_)
    out.update(diag)
    if rank == 0:
        if a.detail_out:
            with open(a.detail_out, "w") as f:
                json.dump(detail, f)
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()


def raster_again(s, inp, W, H, deg, dev):
    _, raster = rasterizer_for(s, W, H, deg, dev)
    return raster(**inp)


if __name__ == "__main__":
    main()
