# the GPU test suite into gpurun_out/<tag>/gpu_tests.log (one process, per-test time limit)
set -e
O=gpurun_out/${1:-suite}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
