# armed-split overhead after merging tile_order's passes and the workers' early exit
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/street_tiles.py --iters 12000 --views 8 --segs 0:512,4096:512 --reps 7 > $O/street.json 2> $O/street.err || exit 5
for k in 1 2; do
  timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 > $O/bench_$k.json 2>>$O/bench.err || exit 3
  cat $O/bench_$k.json >> $O/bench_all.jsonl
done
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
timeout -k 10 300 python3 -u bench.py $C3 > $O/c3.json 2>>$O/c3.err || exit 4
