# the whole -m gpu suite at the current kernels, then smoke
set -o pipefail
O=gpurun_out/r04zf
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
