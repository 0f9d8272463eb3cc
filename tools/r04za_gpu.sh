# forward split minimum A/B on street views (split gate off so every frame is armed)
set -o pipefail
O=gpurun_out/r04za
mkdir -p $O
timeout -k 10 900 python3 -u tools/street_tiles.py --iters 12000 --views 8 --reps 8 --no-gate \
  --segs 0:512,4096:512,4096:512:8192,4096:512:16384,4096:512:32768 > $O/street_fmin.json 2> $O/street_fmin.err
