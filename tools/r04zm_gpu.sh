# split gate's pinned host words: their cost in tile_order / sb_colscan (vlibs/nohost.so stores none)
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04zm_seg.log 2>&1 || exit 9
O=$(pwd)/gpurun_out/r04zm
mkdir -p $O
bash tools/ab_bench.sh hostwords2 2 > $O/ab.txt 2>&1 || exit 1
A="--steps 20 --warmup 5 --metric-only --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_base -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > /dev/null 2>>$O/err.log || exit 3
GSR_LIBRARY=$GRAFT_REPO_ROOT/vlibs/nohost.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_nohost -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > /dev/null 2>>$O/err.log || exit 4
GSR_LIBRARY=$GRAFT_REPO_ROOT/vlibs/fwdstore.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_fwdstore -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > /dev/null 2>>$O/err.log
