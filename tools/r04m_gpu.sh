# split gate: tests, bench default vs splits off, config-3 with defaults
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for cfg in "on" "off" "on" "off"; do
  if [ $cfg = off ]; then X="GSR_TB_SPLIT=0"; F="--fwd-seg 0"; else X="GSR_TB_SPLIT=16384"; F=""; fi
  env $X timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 $F > $O/bench_$cfg.json 2>>$O/bench.err || exit 3
  cat $O/bench_$cfg.json >> $O/bench_all.jsonl
done
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
timeout -k 10 300 python3 -u bench.py $C3 > $O/c3.json 2>>$O/c3.err || exit 4
