# round-4 closing run at the final kernels: the whole -m gpu suite, smoke, the profile, the full bench
set -o pipefail
O=gpurun_out/r04zn
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
bash tools/profile_gpu.sh r04zn || exit 3
cp gpurun_out/prof_r04zn/summary.json profiles/r04zn_pmc.json
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err
