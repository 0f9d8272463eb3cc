#!/bin/bash
# Interleaved A/B of library variants on the metric line + config 5 (ON the GPU box):
#   bash tools/ab_c5.sh <tag> <rounds> <variant>...
# variant: "default" (the in-tree library), a library path, or NAME=VALUE[,NAME=VALUE]@<library or default>
# (environment settings for that run)
set -u -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
ARGS="--steps 20 --warmup 5 --train-steps 0 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --no-config3 --post-leaves 0"
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    envs=""; lib=$v
    case "$v" in *@*) envs=${v%@*}; lib=${v#*@} ;; esac
    n=$(basename "$lib" .so)${envs:+_$(echo "$envs" | tr ',=' '_-')}
    [ "$lib" != default ] && envs="GSR_LIBRARY=$lib${envs:+,$envs}"
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python3 bench.py $ARGS > "$O/$n.$r.json" 2> "$O/$n.$r.err" || exit 1
  done
done
echo "ab_c5 $TAG done"
