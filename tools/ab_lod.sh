# expand_to_size variants A/B on the GPU box (measurement script): tools/lod_bench.py under a
# kernel trace for the default library and each vlibs/cut_*.so -> gpurun_out/r06za/ab.log
set -u -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${AB_TAG:-r06za}; mkdir -p $O
for L in default $(ls $R/vlibs/cut_*.so); do
  n=$(basename $L .so)
  cd /tmp && export TMPDIR=/tmp
  if [ $L = default ]; then unset GSR_LIBRARY; else export GSR_LIBRARY=$L; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$n -o run -- python3 $R/tools/lod_bench.py > $O/$n.log 2>&1 || exit 1
  cd $R
  grep -h '"lib"' $O/$n.log >> $O/ab.log
  (grep -h "lod_cut_stats" $O/$n.log || true) | tail -1 >> $O/ab.log
  python3 -c "
import csv,glob,sys
for r in csv.DictReader(open(glob.glob('$O/tr_$n/**/*kernel_stats.csv',recursive=True)[0])):
    if 'lod' in r['Name'] or 'fill' in r['Name']: print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
" >> $O/ab.log
  rm -rf $O/tr_$n
done
cat $O/ab.log
