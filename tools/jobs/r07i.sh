#!/bin/bash
# round 6: DPP wave scan in k_enc_emit: deflate tests, C1 A/B against the
# previous library, the C4 encode stage
set -o pipefail
T=${1:-r07i}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_bigbuf.py tests/test_gpu_flush.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for r in 1 2; do
  for L in ab/libzgpu_base.so zlib.wasm_amd/libzgpu.so; do
    timeout -k 10 300 python3 -u tools/c1_latency.py $L >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/c1_ab.log
