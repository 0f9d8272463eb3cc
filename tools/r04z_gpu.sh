# dense Adam flat runs: parity tests, then the train_post leg under kernel-trace stats
set -o pipefail
O=$(pwd)/gpurun_out/r04z
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_post.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --train-steps 3 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --no-config3 > $O/bench.json 2> $O/bench.err
