#!/bin/bash
# Run ON the GPU box (via gpurun) from the repo root: kernel-trace stats + two PMC passes of
# the bench workload, summarised into gpurun_out/prof_<tag>/summary.json.
#   usage: bash tools/profile_gpu.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
# PROFILE_ARGS replaces the bench arguments (e.g. config 5 alone); default: the metric line only
ARGS=${PROFILE_ARGS:-"--steps 3 --warmup 2 --profile-steps 1 --metric-only $*"}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/sq1" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/sq1.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq2" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/sq2.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq3" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/sq3.log" 2>&1
SQ4=""
if [ -n "${PROFILE_CACHE:-}" ]; then  # L2 hit / miss and request counts (one more pass)
    timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/sq4" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/sq4.log" 2>&1
    SQ4="--sq $OUT/sq4"
fi
cd "$ROOT"
python3 tools/pmc_summary.py --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" --sq "$OUT/sq1" --sq "$OUT/sq2" --sq "$OUT/sq3" $SQ4 --out "$OUT/summary.json" --note "$TAG: bench.py $ARGS" > /dev/null
# keep the summary and the kernel stats; the raw traces and counter CSVs can exceed what gpurun copies back
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv" 2>/dev/null || true
if [ -z "${PROFILE_KEEP_RAW:-}" ]; then rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write" "$OUT/sq1" "$OUT/sq2" "$OUT/sq3" "$OUT/sq4"; fi
echo "profile $TAG done"
