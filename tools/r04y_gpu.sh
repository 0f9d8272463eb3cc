# kernel stats of the bench's train-step leg (plus the metric)
set -o pipefail
O=$(pwd)/gpurun_out/r04y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --train-steps 40 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --no-config3 --post-leaves 0 > $O/bench.json 2> $O/bench.err
