#!/bin/bash
# round 6: lone-buffer latency changes (64 B line caches in k_pbig1..3, k_pbig5 over all waves,
# batched table lookups in the block histogram): parity of the big-buffer paths first, then the
# C1 A/B against the round's HEAD build, with the one-lane tree build as a third arm
set -o pipefail
T=${1:-r06i}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bigbuf.py tests/test_gpu_stream.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for r in 1 2; do
  for L in ab/libzgpu_r06head.so zlib.wasm_amd/libzgpu.so; do
    timeout -k 10 300 python3 -u tools/c1_latency.py $L >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
  done
  echo "ZGPU_PLAN_LANE=1" >> $O/c1_ab.log
  ZGPU_PLAN_LANE=1 timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/c1_ab.log
for k in text mix; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$k -o run -- python3 tools/c1_trace.py $k > $O/k_$k.log 2>&1 || { echo "trace failed"; exit 1; }
  f=$(find $O/k_$k -name "*kernel_stats.csv" | head -1); cp $f $O/kstats_c1_$k.csv; head -14 $f | cut -c1-150
done
