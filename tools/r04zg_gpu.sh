# final round-4 profile at the current kernels (kernel-trace stats + PMC passes), then the full bench
# (reading that profile: copied into profiles/ on the box first)
set -o pipefail
bash tools/profile_gpu.sh r04zg || exit 1
cp gpurun_out/prof_r04zg/summary.json profiles/r04zg_pmc.json
mkdir -p gpurun_out/r04zg
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04zg/bench.json 2> gpurun_out/r04zg/bench.err
