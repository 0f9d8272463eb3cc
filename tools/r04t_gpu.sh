# kernel stats of the train_post step (bench's train_post leg only)
set -o pipefail
O=$(pwd)/gpurun_out/r04t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --train-steps 3 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --no-config3 > $O/bench.json 2> $O/bench.err
