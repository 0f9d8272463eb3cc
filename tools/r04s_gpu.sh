# render_bwd segment slots from history: tests, bench
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for k in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 > $O/bench_$k.json 2>>$O/bench.err || exit 3
  cat $O/bench_$k.json >> $O/bench_all.jsonl
done
