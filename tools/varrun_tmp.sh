timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/parity.log 2>&1; tail -2 gpurun_out/parity.log
for v in default default; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --train-steps 5 > gpurun_out/var.json 2>gpurun_out/var.err || { echo "$v failed"; tail -3 gpurun_out/var.err; continue; }
  python -c "import json;d=json.load(open('gpurun_out/var.json'));print('$v', d['value'], d['stages_ms'], d['train_step']['ms'])"
done
