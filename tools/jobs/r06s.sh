#!/bin/bash
# round 6: probe of the dictionary-header sessions that differ (Z_FILTERED), and the k_enc_emit batch change's tests
set -o pipefail
T=${1:-r06s}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/dict_header_probe.py > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_bigbuf.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so > $O/c1_latency.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_latency.log; exit 1; }
grep -v amdgpu.ids $O/c1_latency.log | grep -v "^stages"
for L in ab/libzgpu_r06head.so zlib.wasm_amd/libzgpu.so; do
  timeout -k 10 120 python3 -u tools/ab_match.py $L 2 >> $O/sub_ab.log 2>&1 || { echo "ab failed"; tail -5 $O/sub_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/sub_ab.log
