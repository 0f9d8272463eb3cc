# A/B: the zero gradient rows only on the workgroups from GSR_BWD_ZERO_FROM % of render_bwd's grid
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
for z in 0 25 50 75 90 0 25 50 75 90; do
  GSR_BWD_ZERO_FROM=$z timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 > $O/bench_$z.json 2>>$O/bench.err || exit 3
  echo "{\"z\": $z, \"line\": $(cat $O/bench_$z.json)}" >> $O/bench_all.jsonl
done
