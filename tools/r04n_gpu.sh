# forward split: item 0 blends first; split factor A/B (GSR_FSEG_FACTOR) on street views; config-3
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for fac in 2 4; do
  GSR_FSEG_FACTOR=$fac timeout -k 10 300 python3 -u tools/street_tiles.py --iters 12000 --views 8 --segs 0:512,4096:512 --reps 5 > $O/street_f$fac.json 2> $O/street_f$fac.err || exit 5
done
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
timeout -k 10 300 python3 -u bench.py $C3 > $O/c3.json 2>>$O/c3.err || exit 4
timeout -k 10 300 python3 -u bench.py $C3 --fwd-seg 0 > $O/c3_nofwd.json 2>>$O/c3.err || exit 4
