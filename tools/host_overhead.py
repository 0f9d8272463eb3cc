"""Host-side cost of one fwd+bwd step through the public autograd API (run ON the GPU box).

    python tools/host_overhead.py [--gaussians N] [--size S] [--iters I]

A tiny frame (the GPU finishes its work long before the host queues the next step) timed four ways:
the whole step; the Python around the two library calls (the ctypes entry points replaced by a stub
that returns 0, so no kernel runs); the library calls themselves; and, from the stage profile, the
GPU time.  The bench frame's step is host-bound when the host part approaches its GPU time.
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
    import torch
    import bench
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
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        return (t1 - t0) / n * 1e6, (time.perf_counter() - t0) / n * 1e6

    out = {}
    out["step_enqueue_us"], out["step_wall_us"] = per_iter(step, a.iters)

    def fwd():
        with torch.no_grad():
            raster(**inp)
    out["fwd_nograd_enqueue_us"], out["fwd_nograd_wall_us"] = per_iter(fwd, a.iters)

    # the Python around the library: every ctypes entry point the two calls use answers 0 at once
    real = _C._L

    class Stub:
        def __getattr__(self, name):
            f = getattr(real, name)
            if name in ("gsr_rasterize_forward_ex", "gsr_rasterize_backward"):
                return lambda *args: 0
            return f
    _C._L = Stub()
    try:
        out["python_only_step_us"], _ = per_iter(step, a.iters)
        # its parts: the forward call, then the backward alone (through autograd's device thread)
        import torch.autograd as ag

        def parts(n):
            tf = tb = 0.0
            for _ in range(n):
                for v in leaves:
                    v.grad = None
                t0 = time.perf_counter()
                color, radii, invd = raster(**inp)
                t1 = time.perf_counter()
                ag.backward([color, invd], [gcol, ginv])
                tb += time.perf_counter() - t1
                tf += t1 - t0
            return tf / n * 1e6, tb / n * 1e6
        parts(20)
        out["python_only_fwd_us"], out["python_only_bwd_us"] = parts(a.iters)
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
    finally:
        _C._L = real

    t0 = time.perf_counter()
    for _ in range(a.iters * 10):
        real.gsr_abi_version()
    out["ctypes_noarg_call_us"] = (time.perf_counter() - t0) / (a.iters * 10) * 1e6
    out["stages_ms"] = bench.stage_profile(step, 5)
    print(out)
    for v in leaves:
        v.grad = None


if __name__ == "__main__":
    main()
