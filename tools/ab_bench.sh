#!/bin/bash
# A/B of measurement-variant libraries (vlibs/*.so, built with build_hip.py --define ... --out) on the
# bench workload, interleaved, run ON the GPU box:  bash tools/ab_bench.sh <tag> [rounds]
set -uo pipefail
TAG=${1:-ab}; ROUNDS=${2:-2}
OUT=gpurun_out/ab_$TAG; mkdir -p "$OUT"
ARGS="--steps 50 --warmup 10 --metric-only"
for r in $(seq 1 "$ROUNDS"); do
  timeout -k 10 120 python3 bench.py $ARGS > "$OUT/base_$r.json" 2>/dev/null || exit 1
  for lib in ${AB_LIBS:-vlibs/*.so}; do
    n=$(basename "$lib" .so)
    GSR_LIBRARY="$lib" timeout -k 10 120 python3 bench.py $ARGS > "$OUT/${n}_$r.json" 2>/dev/null || exit 1
  done
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f)); n = os.path.basename(f).rsplit("_", 1)[0]
    acc[n].append((d["value"], d["stages_ms"]))
for n, v in acc.items():
    st = {k: round(sum(x[1][k] for x in v) / len(v), 4) for k in v[0][1]}
    print(f"{n:32s} Mpix/s {[x[0] for x in v]}  bwd {st.get('render_bwd')} fwd {st.get('render_fwd')} all {st}")
PY
