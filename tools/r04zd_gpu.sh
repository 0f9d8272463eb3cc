# forward worker pool size A/B on street views (early workers, 4-segment minimum)
set -o pipefail
O=gpurun_out/r04zd
mkdir -p $O
for w in 256 512 1024; do
  GSR_FWD_WORKERS=$w timeout -k 10 600 python3 -u tools/street_tiles.py --iters 12000 --views 4 --reps 8 --no-gate \
    --segs 0:512,4096:512 > $O/street_w$w.json 2> $O/street_w$w.err || exit 2
done
