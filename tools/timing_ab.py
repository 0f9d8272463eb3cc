"""Why bench.py's timed steps and a plain event-bracketed loop of the same steps disagree
(measurement tool, run on the GPU box): one process, the bench's metric workload, then in turn

  plain   W warm-ups, synchronize, event, N steps, event, synchronize (GPU time of N steps)
  timed   bench.timed(): W warm-ups, synchronize, gc settled, perf_counter around N steps + synchronize
  wall    synchronize, perf_counter, N steps, synchronize (no gc handling)

each `--rounds` times, printing ms per step for every variant as JSON.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "street-sparse-3dgs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda:0")
    s, inp, gcol, ginv = bench.make_inputs(1_000_000, 1920, 1080, 3, seed=0, device=dev)
    _, raster = bench.rasterizer_for(s, 1920, 1080, 3, dev)
    step = bench.fwd_bwd_step(raster, inp, gcol, ginv)
    for _ in range(300):
        step()
    torch.cuda.synchronize()
    one = bench.Ranks(1, 0, False, dev)
    out = {"plain": [], "timed": [], "wall": [], "plain_long": []}
    for _ in range(a.rounds):
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        out["plain"].append(round(e0.elapsed_time(e1) / a.steps, 4))
        out["timed"].append(round(bench.timed(step, a.steps, a.warmup, one) / a.steps * 1e3, 4))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        out["wall"].append(round((time.perf_counter() - t0) / a.steps * 1e3, 4))
        import gc
        for name, pre in (("collect", lambda: gc.collect()), ("freeze", lambda: gc.freeze()),
                          ("collect_freeze", lambda: (gc.collect(), gc.freeze()))):
            torch.cuda.synchronize()
            pre()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            out.setdefault("wall_after_" + name, []).append(round((time.perf_counter() - t0) / a.steps * 1e3, 4))
            gc.unfreeze()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            out.setdefault("wall_next_" + name, []).append(round((time.perf_counter() - t0) / a.steps * 1e3, 4))
        e0.record()
        for _ in range(10 * a.steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        out["plain_long"].append(round(e0.elapsed_time(e1) / (10 * a.steps), 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
