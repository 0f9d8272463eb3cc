"""Where the library's host time goes (run ON the GPU box, with a GSR_HOST_TRACE build):

    python street-sparse-3dgs_amd/build_hip.py --define GSR_HOST_TRACE=1 --out vlibs/htrace.so
    GSR_LIBRARY=vlibs/htrace.so python tools/host_trace.py [--gaussians N] [--size S] [--iters I]

Runs fwd+bwd steps through the public API and prints the host microseconds per call spent issuing
each stage (StageTimer scopes in rasterizer.hip), the whole forward / backward calls and the K wait.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "street-sparse-3dgs_amd"), os.path.join(REPO, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--size", type=str, default="1920x1080")
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    import torch
    import bench
    from diff_gaussian_rasterization import _C
    W, H = (int(v) for v in a.size.split("x"))
    dev = torch.device("cuda", 0)
    s, inp, gcol, ginv = bench.make_inputs(a.gaussians, W, H, 3, 0, dev)
    _, raster = bench.rasterizer_for(s, W, H, 3, dev)
    step = bench.fwd_bwd_step(raster, inp, gcol, ginv)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    buf = (ctypes.c_int64 * 24)()
    _C._L.gsr_debug_trace(buf, 24, 1)
    k0 = _C.forward_stats()["k_wait_ns"]
    for _ in range(a.iters):
        step()
    torch.cuda.synchronize()
    k1 = _C.forward_stats()["k_wait_ns"]
    _C._L.gsr_debug_trace(buf, 24, 1)
    names = list(_C.STAGES) + ["forward_call", "backward_call"]
    out = {n: round(buf[i] / max(1, buf[12 + i]) * 1e-3, 2) for i, n in enumerate(names) if buf[12 + i]}
    out["calls"] = {n: buf[12 + i] for i, n in enumerate(names) if buf[12 + i]}
    out["k_wait_us_per_forward"] = round((k1 - k0) / a.iters * 1e-3, 2)
    print({"frame": f"{a.gaussians} at {W}x{H}", "host_us_per_call": out})


if __name__ == "__main__":
    main()
