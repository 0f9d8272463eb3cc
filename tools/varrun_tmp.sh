timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/parity.log 2>&1; tail -2 gpurun_out/parity.log
for v in default variants/ec0 variants/ec1 variants/ec2 default variants/ec0; do
  if [ "$v" = default ]; then unset GSR_LIBRARY; else export GSR_LIBRARY=$PWD/$v/libgsr_hip.so; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --train-steps 0 > gpurun_out/var.json 2>gpurun_out/var.err || { echo "$v failed"; tail -3 gpurun_out/var.err; continue; }
  python -c "import json;d=json.load(open('gpurun_out/var.json'));print('$v', d['value'], d['stages_ms']['render_fwd'], d['stages_ms']['render_bwd'])"
done
