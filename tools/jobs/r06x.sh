#!/bin/bash
# round 6: two-level heap sift (r_down2): tree tests, C1 latency against the previous final build, and the
# phase clock of the one-wave tree build (ZGPU_PLAN_ONEWAVE=1 on the clock build)
set -o pipefail
T=${1:-r06x}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_bigbuf.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for r in 1 2; do
  for L in ab/libzgpu_r06w.so zlib.wasm_amd/libzgpu.so; do
    timeout -k 10 300 python3 -u tools/c1_latency.py $L >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/c1_ab.log | grep -v "^stages"
ZGPU_PLAN_ONEWAVE=1 timeout -k 10 120 python3 -u tools/plan_clock.py ab/libzgpu_planclk.so > $O/plan_clock.log 2>&1 || { echo "clock failed"; tail -5 $O/plan_clock.log; exit 1; }
grep -v amdgpu.ids $O/plan_clock.log
