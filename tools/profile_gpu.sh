#!/bin/bash
# Run ON the GPU box (via gpurun) from the repo root: kernel-trace stats + two PMC passes of
# the bench workload, summarised into gpurun_out/prof_<tag>/summary.json.
#   usage: bash tools/profile_gpu.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS="--steps 3 --warmup 2 --profile-steps 1 --no-cpu-baseline $*"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/write.log" 2>&1
cd "$ROOT"
python3 tools/pmc_summary.py --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" --out "$OUT/summary.json" --note "$TAG: bench.py $ARGS" > /dev/null
echo "profile $TAG done"
