"""Compact view of a rocprofv3 kernel_stats.csv: short kernel name, calls, average / total us."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    m = re.search(r"(rocprim|gsr)::[^(<]*?(\w+)(<[^>]*>)?\(", n)
    short = n[:70]
    if "rocprim" in n:
        k = next((s for s in ("onesweep_iteration", "global_offsets", "histogram", "scan_impl", "init_lookback") if s in n), n[:60])
        short = "rocprim:" + k
    elif m:
        short = re.sub(r"\(.*", "", n.replace("void ", ""))[:70]
    print(f"{short:72s} {r['Calls']:>5} {float(r['AverageNs']) / 1000:9.2f}us {float(r['TotalDurationNs']) / 1000:10.1f}us")
