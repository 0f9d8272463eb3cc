# SSIM stream kernel, 8-row steps (vlibs/ssim8.so) vs 4-row steps: loss tests on the variant, train-step A/B, kernel times
set -o pipefail
O=$(pwd)/gpurun_out/r04zj
mkdir -p $O
GSR_LIBRARY=vlibs/ssim8.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
A="--steps 5 --warmup 2 --train-steps 40 --no-config5 --no-street --no-config4 --no-coarse-debug --no-cpu-baseline --no-config3 --post-leaves 0"
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py $A > $O/base_$r.json 2>>$O/err.log || exit 2
  GSR_LIBRARY=vlibs/ssim8.so timeout -k 10 300 python3 -u bench.py $A > $O/ssim8_$r.json 2>>$O/err.log || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_base -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > /dev/null 2>>$O/err.log || exit 3
GSR_LIBRARY=$GRAFT_REPO_ROOT/vlibs/ssim8.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_ssim8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > /dev/null 2>>$O/err.log
