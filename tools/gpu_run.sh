#!/bin/bash
# One parameterised GPU run, ON the GPU box from the repo root (via gpurun):
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]
# steps, run in order, each under its own time limit; the run stops at the first step that fails:
#   tests            pytest -m gpu (thread timeout per test)       -> gpurun_out/<tag>/gputest.log
#   tests=<k expr>   the same, only the tests matching -k <k expr>
#   smoke            __graft_entry__.smoke()                        -> smoke.log
#   host             tools/host_overhead.py (host cost of the API step)
#   metric           bench.py --metric-only (the headline line only) -> metric.json
#   bench            the full default bench line                    -> bench.json
#   driver           exactly the driver's command, `python3 bench.py --gpus 1 --steps 20 --warmup 5`
#                    (its long diagnostics via GSR_BENCH_DETAIL_OUT)  -> driver.json, driver_detail.json
#   profile          tools/profile_gpu.sh <tag> (rocprofv3 stats + PMC) -> gpurun_out/prof_<tag>/summary.json
#   c3               the config-3 stand-in only (bench.py, a 30k-iteration street chunk) -> c3.json
#   c5               config 5 only (bench.py: the LOD cut + fused frame at 1080p)  -> c5.json
#   py=<script args> python3 -u <script args>                       -> py.log (appended)
set -u -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
C5="--steps 3 --warmup 2 --train-steps 0 --no-config3 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0 --prewarm-s 0"
for st in "$@"; do
    echo "== $st" >&2
    case "$st" in
        tests) timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gputest.log" 2>&1 ;;
        tests=*) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${st#tests=}" > "$O/gputest.log" 2>&1 ;;
        smoke) timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
        host) timeout -k 10 300 python3 -u tools/host_overhead.py > "$O/host.log" 2>&1 ;;
        metric) timeout -k 10 300 python3 -u bench.py --metric-only > "$O/metric.json" 2> "$O/metric.err" ;;
        bench) timeout -k 10 900 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err" ;;
        driver) GSR_BENCH_DETAIL_OUT="$O/driver_detail.json" timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
                    > "$O/driver.json" 2> "$O/driver.err" ;;
        profile) bash tools/profile_gpu.sh "$TAG" ;;
        c3) timeout -k 10 600 python3 -u bench.py $C3 > "$O/c3.json" 2> "$O/c3.err" ;;
        c5) timeout -k 10 600 python3 -u bench.py $C5 > "$O/c5.json" 2> "$O/c5.err" ;;
        py=*) timeout -k 10 600 python3 -u ${st#py=} >> "$O/py.log" 2>&1 ;;
        *) echo "unknown step $st" >&2; exit 64 ;;
    esac
    rc=$?
    if [ $rc -ne 0 ]; then echo "step $st failed: rc $rc" >&2; exit $rc; fi
done
echo "gpu_run $TAG done" >&2
