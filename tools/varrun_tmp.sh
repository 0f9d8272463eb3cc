set -e
for v in default variants/branch default variants/branch; do
  if [ "$v" = default ]; then unset GSR_LIBRARY; else export GSR_LIBRARY=$PWD/$v/libgsr_hip.so; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --train-steps 0 > gpurun_out/var.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/var.json'));print('$v', d['value'], d['stages_ms']['render_bwd'])"
done
