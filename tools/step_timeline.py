"""One bench step's kernels on the GPU's clock, from a rocprofv3 kernel trace (measurement tool, run
on the GPU box after `rocprofv3 --kernel-trace --output-format csv` of a short bench run):

    python tools/step_timeline.py <run_kernel_trace.csv> [--anchor preprocess_kernel] [--steps 3]

Takes the last `steps` complete steps (a step starts at a dispatch whose name contains --anchor) and
prints, per step, every dispatch's start offset from the step's start, its duration and the idle gap
since the previous dispatch on ANY queue ended (the chip's own idle time between kernels), then the
step's busy / idle split.  Output: JSON.
"""
from __future__ import annotations

import argparse
import csv
import json


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("gsr::", "")
    return n.split("(")[0][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="preprocess_kernel<true, true>")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--skip-last", type=int, default=2, help="steps at the end not taken (profiling / workload legs)")
    a = ap.parse_args()
    rows = []
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.anchor in r[2]]
    out = []
    pick = starts[-(a.steps + a.skip_last + 1):len(starts) - a.skip_last] if len(starts) > a.steps + a.skip_last else starts
    for s0, s1 in zip(pick[:-1], pick[1:]):
        seq = rows[s0:s1]
        t0 = seq[0][0]
        end = t0
        busy = 0
        items = []
        for st, en, name, q in seq:
            gap = max(0, st - end)
            items.append({"k": short(name), "q": q, "start_us": round((st - t0) / 1e3, 2),
                          "dur_us": round((en - st) / 1e3, 2), "idle_before_us": round(gap / 1e3, 2)})
            busy += max(0, en - max(st, end))
            end = max(end, en)
        total = rows[s1][0] - t0
        out.append({"step_us": round(total / 1e3, 2), "busy_us": round(busy / 1e3, 2),
                    "idle_us": round((total - busy) / 1e3, 2), "dispatches": len(seq), "kernels": items})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
