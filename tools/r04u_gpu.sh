set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_post.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --train-steps 3 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --no-config3 > $O/bench.json 2> $O/bench.err || exit 2
