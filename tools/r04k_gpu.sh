# tile_bin split of long superblock lists: parity, bench and street / config-3 A/B (GSR_TB_SPLIT_OFF)
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for off in 1 0 1 0; do
  GSR_TB_SPLIT_OFF=$off timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 > $O/bench_off$off.json 2>>$O/bench.err || exit 3
  cat $O/bench_off$off.json >> $O/bench_all.jsonl
done
for off in 1 0; do
  GSR_TB_SPLIT_OFF=$off timeout -k 10 300 python3 -u tools/street_tiles.py --iters 12000 --views 6 --segs 0:512 --reps 5 > $O/street_off$off.json 2> $O/street_off$off.err || exit 5
done
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
timeout -k 10 300 python3 -u bench.py $C3 > $O/c3.json 2>>$O/c3.err || exit 4
