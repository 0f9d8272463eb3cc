# forward split minimum with the early 512-workgroup pool: 16384 (default) vs 12288 vs 8192
set -o pipefail
O=gpurun_out/r04ze
mkdir -p $O
timeout -k 10 600 python3 -u tools/street_tiles.py --iters 12000 --views 8 --reps 8 --no-gate \
    --segs 0:512,4096:512,4096:512:12288,4096:512:8192 > $O/street_min.json 2> $O/street_min.err || exit 2
