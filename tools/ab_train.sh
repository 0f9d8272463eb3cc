#!/bin/bash
# Run ON the GPU box: interleaved train-step A/B of an environment switch.
#   bash tools/ab_train.sh <tag> <VAR> <valueA> <valueB> [rounds]
set -u
TAG=$1; VAR=$2; A=$3; B=$4; N=${5:-3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$N"); do
  for v in "$A" "$B"; do
    n=$(echo "x$v" | tr '/.' '__')  # a file-name tag for the value (library paths allowed)
    env "$VAR=$v" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --train-steps 30 --no-config5 --no-street \
      --no-config4 --no-cpu-baseline > "$OUT/b_${n}_$r.json" 2> "$OUT/b_${n}_$r.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'train', d['train_step']['ms'], 'fwdbwd', d['ms_per_step'], 'pre_bwd', d['stages_ms']['preprocess_bwd'])" "$OUT/b_${n}_$r.json" "$VAR=$v" "$r" | tee -a "$OUT/ab.txt"
  done
done
