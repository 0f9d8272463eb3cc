"""The longest kernel dispatches of a rocprofv3 kernel trace and everything that overlapped them
(measurement tool, run on the GPU box after a `rocprofv3 --kernel-trace` of a long run, whose
trace CSV is too large to copy back):

    python tools/trace_spikes.py <run_kernel_trace.csv> [--top 5] > spikes.json

Streams the CSV once for the top dispatches by duration (name filter optional), then again for
the dispatches that overlap each of them (queue / stream ids, names, start / end relative to the
spike's start, in microseconds), plus the dispatches just before and after on every queue.
"""
from __future__ import annotations

import argparse
import csv
import heapq
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--context", type=int, default=3, help="dispatches kept before / after each spike per queue")
    a = ap.parse_args()
    top = []
    n = 0
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            n += 1
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            item = (d, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90], r["Queue_Id"],
                    r["Stream_Id"], int(r["Dispatch_Id"]))
            if len(top) < a.top:
                heapq.heappush(top, item)
            elif d > top[0][0]:
                heapq.heapreplace(top, item)
    top.sort(reverse=True)
    spikes = [{"dur_us": t[0] / 1e3, "start": t[1], "end": t[2], "name": t[3], "queue": t[4], "stream": t[5],
               "dispatch": t[6], "overlap": [], "before": {}, "after": {}} for t in top]
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            s0, s1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            q = r["Queue_Id"]
            for sp in spikes:
                rec = {"name": r["Kernel_Name"][:90], "queue": q, "stream": r["Stream_Id"],
                       "dispatch": int(r["Dispatch_Id"]), "start_us": (s0 - sp["start"]) / 1e3,
                       "end_us": (s1 - sp["start"]) / 1e3, "grid": int(r["Grid_Size_X"]),
                       "wg": int(r["Workgroup_Size_X"]), "lds": int(r["LDS_Block_Size"])}
                if s0 < sp["end"] and s1 > sp["start"]:
                    if len(sp["overlap"]) < 200:
                        sp["overlap"].append(rec)
                elif s1 <= sp["start"]:
                    b = sp["before"].setdefault(q, [])
                    b.append(rec)
                    if len(b) > a.context:
                        b.pop(0)
                elif s0 >= sp["end"]:
                    aft = sp["after"].setdefault(q, [])
                    if len(aft) < a.context:
                        aft.append(rec)
    print(json.dumps({"dispatches": n, "spikes": spikes}, indent=1))


if __name__ == "__main__":
    main()
