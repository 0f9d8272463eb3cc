set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
for v in default default; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --train-steps 0 > gpurun_out/var.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/var.json'));print('$v', d['value'], d['ms_per_step'], d['stages_ms'])"
done
