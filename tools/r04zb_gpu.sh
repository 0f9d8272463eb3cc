# forward workers launched ahead of tile_order: segment parity tests, then the street-view A/B
set -o pipefail
O=gpurun_out/r04zb
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for e in 1 0; do
  GSR_FWD_EARLY_WORKERS=$e timeout -k 10 600 python3 -u tools/street_tiles.py --iters 12000 --views 8 --reps 8 --no-gate \
    --segs 0:512,4096:512,4096:512:16384,4096:512:32768 > $O/street_early$e.json 2> $O/street_early$e.err || exit 2
done
