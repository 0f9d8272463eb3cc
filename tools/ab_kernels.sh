#!/bin/bash
# Per-kernel A/B of measurement-variant libraries (vlibs/*.so) under rocprofv3 kernel-trace stats,
# run ON the GPU box:  bash tools/ab_kernels.sh <tag>
# Prints, per kernel, the average duration (us) of the in-tree library ("base") and every variant.
set -uo pipefail
TAG=${1:-abk}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/abk_$TAG; mkdir -p "$OUT"
ARGS="--steps 20 --warmup 5 --profile-steps 1 --metric-only"
# AB_SCRIPT / AB_ARGS: profile another program (e.g. tools/train_step_profile.py --steps 20)
SCRIPT=${AB_SCRIPT:-bench.py}
[ -n "${AB_ARGS:-}" ] && ARGS=$AB_ARGS
export TMPDIR=/tmp
run() {  # name, library ("" = in-tree)
  ( cd /tmp && GSR_LIBRARY="$2" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/$1" -o run -- python3 "$ROOT/$SCRIPT" $ARGS > "$OUT/$1.log" 2>&1 )
}
run base "" || exit 1
for lib in vlibs/*.so; do
  n=$(basename "$lib" .so)
  run "$n" "$ROOT/$lib" || exit 1
done
python3 - "$OUT" <<'PY'
import csv, glob, os, re, sys
out = sys.argv[1]
def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = n.replace("gsr::", "")
    return n[:40]
tab, names = {}, []
for d in sorted(glob.glob(os.path.join(out, "*/"))):
    v = os.path.basename(d.rstrip("/"))
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        continue
    names.append(v)
    for r in csv.DictReader(open(f[0])):
        tab.setdefault(short(r["Name"]), {})[v] = float(r["AverageNs"]) / 1000
names.sort(key=lambda s: (s != "base", s))
print(f"{'kernel':40s} " + " ".join(f"{n[:12]:>12s}" for n in names))
for k, row in sorted(tab.items(), key=lambda kv: -max(kv[1].values())):
    if max(row.values()) < 1.0:
        continue
    print(f"{k:40s} " + " ".join(f"{row.get(n, float('nan')):12.2f}" for n in names))
PY
