# forward-split worker pool: side stream (default build) vs inside render_fwd (abvar/libgsr_inkernel.so)
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
for lib in "" "abvar/libgsr_inkernel.so"; do
  tag=$([ -z "$lib" ] && echo side || echo inkernel)
  GSR_LIBRARY=$lib timeout -k 10 300 python3 -u tools/street_tiles.py --iters 12000 --views 8 --segs 0:512,4096:512 --reps 7 > $O/street_$tag.json 2> $O/street_$tag.err || exit 5
  for k in 1 2; do
    GSR_LIBRARY=$lib timeout -k 10 200 python3 -u bench.py --metric-only --steps 50 --warmup 10 > $O/bench_${tag}_$k.json 2>>$O/bench.err || exit 3
    cat $O/bench_${tag}_$k.json >> $O/bench_all.jsonl
  done
done
GSR_LIBRARY=abvar/libgsr_inkernel.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread > $O/gputest_inkernel.log 2>&1 || exit 1
