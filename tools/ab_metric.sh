#!/bin/bash
# Interleaved A/B of library variants on the metric line (ON the GPU box):
#   bash tools/ab_metric.sh <tag> <rounds> <variant>...   ("default" = the in-tree library, or a .so path)
set -u -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    if [ "$lib" = default ]; then
      timeout -k 10 300 python3 bench.py --metric-only --steps 50 --warmup 10 > "$O/$n.$r.json" 2> "$O/$n.$r.err" || exit 1
    else
      GSR_LIBRARY=$lib timeout -k 10 300 python3 bench.py --metric-only --steps 50 --warmup 10 > "$O/$n.$r.json" 2> "$O/$n.$r.err" || exit 1
    fi
  done
done
echo "ab_metric $TAG done"
