# kernel time shares of the config-3 chunk (30k iterations): rocprofv3 stats only (trace deleted: too large)
set -o pipefail
O=$(pwd)/gpurun_out/r04zp
mkdir -p $O
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py $C3 > $O/c3.json 2> $O/c3.err
rc=$?
rm -f $O/tr/run_kernel_trace.csv
exit $rc
