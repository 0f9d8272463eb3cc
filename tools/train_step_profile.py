"""Time the train-step harness alone (for rocprofv3 kernel traces of row H).

    python tools/train_step_profile.py [--steps 10] [--baseline] [--gaussians 1000000]

Prints wall ms/step (synchronised around the timed loop) and the host-side ms/step spent issuing
the step (no synchronisation inside), which tells launch-bound from device-bound.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "street-sparse-3dgs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--baseline", action="store_true")
    ap.add_argument("--python", action="store_true", help="the Python-driven step (default: gsr_train_step)")
    a = ap.parse_args()
    import torch
    from gs_train.harness import make_problem
    step_cls = None
    if not a.python:
        from gs_train.native_step import NativeTrainStep as step_cls
    if a.baseline:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
        from train_torch_ref import ReferenceTrainStep as step_cls
    ts = make_problem(a.gaussians, a.width, a.height, n_views=4, seed=0, step_cls=step_cls, skybox_points=10_000)
    for _ in range(a.warmup):
        ts.step()
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        ts.step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"train step ({'baseline' if a.baseline else ('python' if a.python else 'native')}): wall {wall:.3f} ms/step, "
          f"host issue {host / a.steps * 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
