# tile_bin split threshold A/B on the metric bench (GSR_TB_SPLIT env: 0 = off)
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
for t in 0 16384 32768 65536 0 16384 32768 65536; do
  GSR_TB_SPLIT=$t timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 > $O/bench_$t.json 2>>$O/bench.err || exit 3
  cat $O/bench_$t.json >> $O/bench_all.jsonl
done
