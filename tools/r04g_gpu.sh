set -o pipefail
mkdir -p gpurun_out/r04g
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_segments.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r04g/segtest.log 2>&1
rc=$?
echo "segtest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "0 0" "0 512" "4096 512" "0 0" "0 512" "4096 512"; do
  set -- $cfg
  timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 --fwd-seg $1 --bwd-seg $2 > gpurun_out/r04g/bench_$1_$2.json 2>>gpurun_out/r04g/bench.err || exit 3
  cat gpurun_out/r04g/bench_$1_$2.json >> gpurun_out/r04g/bench_all.jsonl
done
timeout -k 10 500 python3 -u tools/street_tiles.py --iters 12000 --views 6 --segs 0:0,0:512,4096:512,8192:512 > gpurun_out/r04g/street_tiles.json 2> gpurun_out/r04g/street_tiles.err
