set -u -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06zy; mkdir -p $O
C5="--steps 3 --warmup 2 --train-steps 0 --no-config3 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0 --prewarm-s 0"
for round in 1 2; do
  for b in 0 192 232 256; do
    if [ $b = 0 ]; then unset GSR_COLOR_BIG_BLOCKS; else export GSR_COLOR_BIG_BLOCKS=$b; fi
    timeout -k 10 300 python3 $R/bench.py $C5 > $O/t.json 2> $O/t.err || exit 1
    python3 -c "
import json;d=json.loads(open('$O/t.json').read().strip().splitlines()[-1]);c=d['config5']
print('blocks $b', $round, c['ms_per_frame'], c['raster_stages_ms'].get('sh_color'), c['raster_stages_ms'].get('depth_sort_scan'), c['split_ms'])" >> $O/ab.log
  done
done
cat $O/ab.log
