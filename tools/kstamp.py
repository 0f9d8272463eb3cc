"""The bench step's kernels on the GPU's own clock, no profiler (measurement tool, run on the GPU box
with a GSR_KSTAMP=1 library):

    python street-sparse-3dgs_amd/build_hip.py --define GSR_KSTAMP=1 --out vlibs/kstamp.so   # here
    GSR_LIBRARY=vlibs/kstamp.so python tools/kstamp.py [--steps 40] [--sync-every 0]          # on the box

Runs the bench's fwd+bwd step (bench.py's metric workload) back to back, then reads the instrumented
kernels' start / end stamps of the last 3 steps (gsr_kstamp_read: block 0's start, the last wave's
end, s_memrealtime at 100 MHz) and prints per kernel the mean start offset from the step's preprocess, the mean duration
and the mean idle gap since the previous main-stream kernel ended, plus the step period and its
busy / idle split.  Output: JSON.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "street-sparse-3dgs_amd"))

NAMES = ["preprocess", "sh_color", "upsweep", "pass0", "pass1", "pass2", "pass3", "sb_count", "sb_colscan",
         "sb_scatter", "tile_bin", "tile_order", "render_fwd", "render_bwd", "grad_range", "fwd_seg", "live_list",
         "grad_live"]
SIDE = {"sh_color", "fwd_seg"}
RING, PER = 4, 9


def read(lib):
    buf = (ctypes.c_uint64 * (24 * PER))()
    rc = lib.gsr_kstamp_read(buf, 24 * PER)
    if rc != 0:
        raise RuntimeError("gsr_kstamp_read failed (not a GSR_KSTAMP library?)")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(24, PER).astype(np.int64)
    out = {}
    for i, n in enumerate(NAMES):
        cnt = int(a[i, 0])
        if cnt == 0:
            continue
        k = min(cnt, RING)
        idx = [(cnt - k + j) % RING for j in range(k)]  # oldest first
        out[n] = [(int(a[i, 1 + r]), int(a[i, 1 + RING + r])) for r in idx]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    import bench
    from diff_gaussian_rasterization import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    P, W, H, deg = a.gaussians, 1920, 1080, 3
    s, inp, gcol, ginv = bench.make_inputs(P, W, H, deg, seed=0, device=dev)
    _, raster = bench.rasterizer_for(s, W, H, deg, dev)
    step = bench.fwd_bwd_step(raster, inp, gcol, ginv)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    ev_ms = e0.elapsed_time(e1) / a.steps
    try:
        st = read(lib)
    except RuntimeError as e:  # a normal library: the event time only
        print(json.dumps({"event_ms_per_step": round(ev_ms, 4), "stamps": str(e)}))
        return
    pre = st["preprocess"]
    steps = []
    for j in range(len(pre) - 1):
        t0, t1 = pre[j][0], pre[j + 1][0]
        rec = {}
        for n, v in st.items():
            for (b, e) in v:
                if t0 <= b < t1:
                    rec[n] = (b - t0, e - t0)
        steps.append((t1 - t0, rec))
    steps = steps[-min(len(steps), a.steps - 1):]
    period = np.array([p for p, _ in steps], np.float64) * 10.0 / 1e3  # ticks -> us
    order = [n for n in NAMES if n in steps[-1][1]]
    main_seq = sorted([n for n in order if n not in SIDE], key=lambda n: steps[-1][1][n][0])
    rows = {}
    idle = []
    for _, rec in steps:
        prev_end = 0
        busy_end = 0
        gaps = 0
        for n in main_seq:
            if n not in rec:
                continue
            b, e = rec[n]
            r = rows.setdefault(n, {"start": [], "dur": [], "gap": []})
            r["start"].append(b)
            r["dur"].append(e - b)
            r["gap"].append(max(0, b - prev_end))
            gaps += max(0, b - prev_end)
            prev_end = max(prev_end, e)
            busy_end = prev_end
        idle.append(gaps)
        for n in SIDE:
            if n in rec:
                b, e = rec[n]
                r = rows.setdefault(n, {"start": [], "dur": [], "gap": []})
                r["start"].append(b)
                r["dur"].append(e - b)
    us = lambda x: round(float(np.mean(x)) * 10.0 / 1e3, 2)
    out = {"event_ms_per_step": round(ev_ms, 4), "steps": len(steps), "period_us_mean": round(float(period.mean()), 2),
           "period_us_median": round(float(np.median(period)), 2),
           "main_stream_idle_us_mean": us(idle),
           "kernels": {n: {"start_us": us(r["start"]), "dur_us": us(r["dur"]),
                           **({"idle_before_us": us(r["gap"])} if r["gap"] else {})} for n, r in rows.items()},
           "note": "start / idle relative to the step's preprocess start; idle_before = gap since the previous "
                   "main-stream kernel's last wave ended (s_memrealtime, 100 MHz); the last main-stream gap "
                   "(grad_range -> next preprocess) is period - (grad_range end)"}
    last = steps[-1][1]
    if "grad_range" in rows:
        out["tail_idle_us_mean"] = round(float(period.mean()) - us(rows["grad_range"]["start"]) -
                                         us(rows["grad_range"]["dur"]), 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
