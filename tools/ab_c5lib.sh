# config 5 under each vlibs/c5_*.so and the default library, interleaved twice (measurement script):
# bench.py's config-5 leg only -> gpurun_out/<AB_TAG>/c5ab.log (ms_per_frame, sh_color, split)
set -u -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${AB_TAG:-r06zk}; mkdir -p $O
C5="--steps 3 --warmup 2 --train-steps 0 --no-config3 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0 --prewarm-s 0"
for round in 1 2; do
  for L in default $(ls $R/vlibs/c5_*.so); do
    if [ $L = default ]; then unset GSR_LIBRARY; else export GSR_LIBRARY=$L; fi
    timeout -k 10 300 python3 $R/bench.py $C5 > $O/c5_tmp.json 2> $O/c5_tmp.err || exit 1
    python3 -c "
import json;d=json.loads(open('$O/c5_tmp.json').read().strip().splitlines()[-1]);c=d['config5']
print('$(basename $L .so)', $round, c['ms_per_frame'], c['raster_stages_ms']['sh_color'], c['raster_stages_ms']['depth_sort_scan'], c['split_ms'])" >> $O/c5ab.log
  done
done
cat $O/c5ab.log
