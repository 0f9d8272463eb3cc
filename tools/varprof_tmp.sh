set -e
ROOT=$(pwd)
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -1 gpurun_out/parity.log
cd /tmp && export TMPDIR=/tmp
for v in default; do
  rm -rf $ROOT/gpurun_out/vp_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/vp_$v -o run -- python3 $ROOT/bench.py --steps 5 --warmup 3 --profile-steps 1 --no-cpu-baseline --train-steps 0 > $ROOT/gpurun_out/vp_$v.log 2>&1
  python3 -c "
import csv
for r in csv.DictReader(open('$ROOT/gpurun_out/vp_$v/run_kernel_stats.csv')):
    n=r['Name']
    if 'gsr::' in n: print('$v', round(float(r['AverageNs'])/1e3,1), n.split('(')[0][-40:])
"
done
cd $ROOT && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --train-steps 0 > gpurun_out/var.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/var.json'));print(d['value'], d['ms_per_step'], d['stages_ms'])"
