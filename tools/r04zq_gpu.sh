# sparse Adam: fully relevant waves update a column-split pair as whole float4 rows.  The whole
# -m gpu suite, smoke, a config-3 A/B (GSR_ADAM_NO_PAIRS=1 = the separate blocks), then the profile
# and the full bench at these kernels
set -o pipefail
O=gpurun_out/r04zq
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
C3="--steps 5 --warmup 2 --train-steps 40 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
GSR_ADAM_NO_PAIRS=1 timeout -k 10 300 python3 -u bench.py $C3 > $O/c3_nopairs.json 2>>$O/c3.err || exit 3
timeout -k 10 300 python3 -u bench.py $C3 > $O/c3_pairs.json 2>>$O/c3.err || exit 3
bash tools/profile_gpu.sh r04zq || exit 4
cp gpurun_out/prof_r04zq/summary.json profiles/r04zq_pmc.json
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err
