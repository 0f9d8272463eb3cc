# config-3 A/B: forward workers ahead of tile_order (early) x split minimum (GSR_FSEG_FACTOR x 4096)
set -o pipefail
O=gpurun_out/r04zc
mkdir -p $O
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
for v in 1:4 1:16 0:16 1:4; do
  e=${v%%:*}; f=${v##*:}
  GSR_FWD_EARLY_WORKERS=$e GSR_FSEG_FACTOR=$f timeout -k 10 300 python3 -u bench.py $C3 >> $O/c3_e${e}_f$f.json 2>>$O/c3.err || exit 4
done
