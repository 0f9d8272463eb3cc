# forward-split follow-up: repeatability fix, side-stream workers; bench / street / config-3 A/B
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_segments.py -v -s --timeout 120 --timeout-method thread > $O/segtest.log 2>&1
rc=$?
echo "segtest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "0 512" "4096 512" "0 512" "4096 512"; do
  set -- $cfg
  timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 --fwd-seg $1 --bwd-seg $2 > $O/bench_$1_$2.json 2>>$O/bench.err || exit 3
  cat $O/bench_$1_$2.json >> $O/bench_all.jsonl
done
timeout -k 10 300 python3 -u tools/street_tiles.py --iters 12000 --views 6 --segs 0:512,4096:512,8192:512 > $O/street_tiles.json 2> $O/street_tiles.err || exit 5
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
for cfg in "0 512" "4096 512"; do
  set -- $cfg
  timeout -k 10 300 python3 -u bench.py $C3 --fwd-seg $1 --bwd-seg $2 > $O/c3_$1_$2.json 2>>$O/c3.err || exit 4
done
