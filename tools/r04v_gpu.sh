# config-3 A/B of the forward split's minimum list length (GSR_FSEG_FACTOR x 4096) and off
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
C3="--steps 5 --warmup 2 --train-steps 0 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --post-leaves 0"
for f in 4 8 16; do
  GSR_FSEG_FACTOR=$f timeout -k 10 300 python3 -u bench.py $C3 > $O/c3_f$f.json 2>>$O/c3.err || exit 4
done
timeout -k 10 300 python3 -u bench.py $C3 --fwd-seg 0 > $O/c3_off.json 2>>$O/c3.err || exit 4
