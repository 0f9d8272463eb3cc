"""Host-side cost of one fwd+bwd step through the public autograd API (run ON the GPU box).

    python tools/host_overhead.py [--gaussians N] [--size S] [--iters I]

A tiny frame (the GPU finishes its work long before the host queues the next step), timed as:
  step_enqueue_us      the whole step through GaussianRasterizer + torch.autograd.backward (the C++
                       autograd Function of the host extension), host time per step;
  k_wait_us            of that, the host's wait for K (num_rendered) inside the forward
                       (gsr_forward_stats[5]): time the host is stalled on the GPU, not busy;
  host_busy_us         step_enqueue_us - k_wait_us;
  python_fn_step_us    the same step through the Python autograd Function (the debug-mode path,
                       with debug off: what round 4 ran for every frame, minus its ctypes marshalling);
  fwd_call_us / bwd_call_us   the two _C entry points called directly (no autograd);
  trivial_autograd_step_us    a do-nothing autograd Function's step, for scale;
and the frame's per-stage GPU time.  The bench frame's step is host-bound when host_busy_us
approaches its GPU time.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "street-sparse-3dgs_amd"), os.path.join(REPO, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=2000)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    dev = torch.device("cuda", 0)
    s, inp, gcol, ginv = bench.make_inputs(a.gaussians, a.size, a.size, 3, 0, dev)
    rs, raster = bench.rasterizer_for(s, a.size, a.size, 3, dev)
    step = bench.fwd_bwd_step(raster, inp, gcol, ginv)
    leaves = list(inp.values())

    def per_iter(fn, n):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        k0 = _C.forward_stats()["k_wait_ns"]
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        k1 = _C.forward_stats()["k_wait_ns"]
        return (t1 - t0) / n * 1e6, (k1 - k0) / n * 1e-3

    out = {}
    with bench.quiet_gc():
        out["step_enqueue_us"], out["k_wait_us"] = per_iter(step, a.iters)
        out["host_busy_us"] = out["step_enqueue_us"] - out["k_wait_us"]

        def fwd():
            with torch.no_grad():
                raster(**inp)
        out["fwd_nograd_enqueue_us"], _ = per_iter(fwd, a.iters)

        # the Python autograd Function (debug-mode path) with debug off
        def python_fn_step():
            for v in leaves:
                v.grad = None
            color, radii, invd = dgr._RasterizeGaussians.apply(
                inp["means3D"], inp["means2D"], inp["shs"], dgr._EMPTY, inp["opacities"], inp["scales"],
                inp["rotations"], dgr._EMPTY, rs, True)
            torch.autograd.backward([color, invd], [gcol, ginv])
        out["python_fn_step_us"], _ = per_iter(python_fn_step, a.iters)
        # interleaved A/B of the two autograd paths (5 rounds), medians
        ab = {"cpp": [], "python": []}
        for _ in range(5):
            ab["cpp"].append(per_iter(step, 100)[0])
            ab["python"].append(per_iter(python_fn_step, 100)[0])
        out["ab_cpp_fn_step_us"] = float(np.median(ab["cpp"]))
        out["ab_python_fn_step_us"] = float(np.median(ab["python"]))

        # the two entry points directly
        e = torch.empty(0, device=dev)
        args = (rs.bg, inp["means3D"], e, inp["opacities"], inp["scales"], inp["rotations"], 1.0, e, rs.viewmatrix,
                rs.projmatrix, rs.tanfovx, rs.tanfovy, a.size, a.size, inp["shs"], 3, rs.campos, False, False)
        last = {}

        def fcall():
            last["f"] = _C.rasterize_gaussians(*args)
        out["fwd_call_us"], _ = per_iter(fcall, a.iters)
        K, _col, _inv, radii, gb, bb, ib = last["f"]

        def bcall():
            _C.rasterize_gaussians_backward(rs.bg, inp["means3D"], radii, e, inp["scales"], inp["rotations"], 1.0, e,
                                            rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, gcol, ginv,
                                            inp["shs"], 3, rs.campos, gb, K, bb, ib)
        out["bwd_call_us"], _ = per_iter(bcall, a.iters)

        z = torch.zeros(4, device=dev, requires_grad=True)

        class Nop(torch.autograd.Function):
            @staticmethod
            def forward(ctx, x):
                return x * 1.0

            @staticmethod
            def backward(ctx, g):
                return g

        def nop():
            z.grad = None
            Nop.apply(z).sum().backward()
        out["trivial_autograd_step_us"], _ = per_iter(nop, a.iters)
    if os.environ.get("HOST_PROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(200):
            step()
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(30)
    out["stages_ms"] = bench.stage_profile(step, 5)
    out = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}
    print(out)
    for v in leaves:
        v.grad = None


if __name__ == "__main__":
    main()
