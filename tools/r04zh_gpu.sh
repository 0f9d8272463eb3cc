# ready word in the depth-sort control words (no memset): segment tests, then light/heavy street views
set -o pipefail
O=gpurun_out/r04zh
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 600 python3 -u tools/street_tiles.py --iters 12000 --views 8 --reps 8 --no-gate \
    --segs 0:512,4096:512 > $O/street.json 2> $O/street.err || exit 2
