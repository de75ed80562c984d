#!/bin/bash
# round 6: k_pbig1s (pass 1 of 256-byte segments from LDS copies of the records and bytes) and scan_tree counts
# by a whole wave (w_rle_count): the deflate suites, then C1 latency against ZGPU_PLAN_ONEWAVE=1
set -o pipefail
T=${1:-r06p}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_bigbuf.py tests/test_gpu_stream.py tests/test_gpu_zstream.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
  echo "ZGPU_PLAN_ONEWAVE=1" >> $O/c1_ab.log
  ZGPU_PLAN_ONEWAVE=1 timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/c1_ab.log | grep -v "^stages"
for k in text mix; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$k -o run -- python3 tools/c1_trace.py $k > $O/k_$k.log 2>&1 || { echo "trace failed"; exit 1; }
  f=$(find $O/k_$k -name "*kernel_stats.csv" | head -1); cp $f $O/kstats_c1_$k.csv; head -8 $f | cut -c1-110
done
