"""Host cost of the FIRST call of each torch op an opacity reset / densify event issues, in a fresh
process, against the second call (measurement tool, run on the GPU box).  torch's ROCm kernels
load their code objects on first use; an op first seen mid-run (config 3's first opacity reset at
iteration 3000) pays that inside the iteration.

    python tools/first_call_cost.py [rows]
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "street-sparse-3dgs_amd"))


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) * 1e3, 3)


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 700_000
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)  # context
    op = torch.randn(P, 1, device=dev)
    ops = {
        "sigmoid": lambda: torch.sigmoid(op[10_000:]),
        "ones_like_mul": lambda: torch.ones_like(op) * 0.01,
        "min": lambda: torch.min(op, torch.ones_like(op) * 0.01),
        "inverse_sigmoid": lambda: torch.log(op.clamp(0.01, 0.99) / (1 - op.clamp(0.01, 0.99))),
        "cat": lambda: torch.cat((op[:10], op[10:]), 0),
        "zeros_like": lambda: torch.zeros_like(op),
        "contiguous_param": lambda: torch.nn.Parameter(op.contiguous()),
    }
    out = {}
    for k, f in ops.items():
        out[k] = [timed(f), timed(f)]
    from gs_train.chunk import reset_opacity
    print(json.dumps({"rows": P, "first_vs_second_ms": out}))


if __name__ == "__main__":
    main()
