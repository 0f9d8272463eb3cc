#!/bin/bash
# GPU round check, run ON the GPU box from the repo root (via gpurun):
#   bash tools/gpu_check.sh <tag> [pytest -k expr]
# pytest -m gpu (each test under a thread timeout), then the default bench line, unless the tests
# ended in a fault / abort / timeout (exit status other than 0 or 1).
set -u
TAG=${1:-x}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" > "$OUT/gputest.log" 2>&1
rc=$?
tail -5 "$OUT/gputest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 600 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?
tail -c 600 "$OUT/bench.json"
echo "pytest rc $rc bench rc $brc"
exit $(( rc > brc ? rc : brc ))
