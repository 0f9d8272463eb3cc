set -uo pipefail
mkdir -p gpurun_out/c5ab
A="--steps 5 --warmup 2 --no-cpu-baseline --train-steps 0 --no-config4 --no-street"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > gpurun_out/c5ab/base_$r.json 2>/dev/null || exit 1
  GSR_LIBRARY=vlibs/cnt_plain.so timeout -k 10 200 python3 bench.py $A > gpurun_out/c5ab/plain_$r.json 2>/dev/null || exit 1
done
