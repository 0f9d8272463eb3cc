#!/bin/bash
# SQ counter passes over the bench workload (run ON the GPU box from the repo root):
#   bash tools/sq_counters.sh <tag> [train]   -> gpurun_out/sq_<tag>/p{1,2,3}/...counter_collection.csv
# With "train" the program is tools/train_step_profile.py (the train-step kernels) instead of bench.py.
set -euo pipefail
TAG=${1:-x}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
PROG="$ROOT/bench.py"
ARGS="--steps 2 --warmup 1 --profile-steps 1 --metric-only"
if [ "${2:-}" = "train" ]; then
  PROG="$ROOT/tools/train_step_profile.py"
  ARGS="--steps 2 --warmup 1"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/p1" -o run -- python3 "$PROG" $ARGS > "$OUT/p1.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 "$PROG" $ARGS > "$OUT/p2.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_CVT --output-format csv -d "$OUT/p3" -o run -- python3 "$PROG" $ARGS > "$OUT/p3.log" 2>&1 || echo "pass 3 failed (counter names?)"
echo "sq $TAG done"
