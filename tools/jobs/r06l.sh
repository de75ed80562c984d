#!/bin/bash
# round 6: k_enc_emit codes from LDS and arithmetic (no dependent c_ct loads per batch), k_links_seg1
# (one atomicMax pass over a segment's window), k_count's one-pass window for segments, and the phase
# clock of the wave tree build: per-position segment stages vs the oracle, the deflate
# suites, then C1 latency (with ZGPU_LINKS_SEG1=0 as the other arm) and the C4 sub-batch against HEAD
set -o pipefail
T=${1:-r06l}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_bigbuf.py tests/test_gpu_stream.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
  echo "ZGPU_LINKS_SEG1=0" >> $O/c1_ab.log
  ZGPU_LINKS_SEG1=0 timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/c1_ab.log | grep -v "^stages"
for L in ab/libzgpu_r06head.so zlib.wasm_amd/libzgpu.so ab/libzgpu_r06head.so zlib.wasm_amd/libzgpu.so; do
  timeout -k 10 120 python3 -u tools/ab_match.py $L 2 >> $O/sub_ab.log 2>&1 || { echo "ab failed"; tail -5 $O/sub_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/sub_ab.log
timeout -k 10 120 python3 -u tools/plan_clock.py ab/libzgpu_planclk.so > $O/plan_clock.log 2>&1 || { echo "clock failed"; tail -5 $O/plan_clock.log; exit 1; }
grep -v amdgpu.ids $O/plan_clock.log
for k in text mix; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$k -o run -- python3 tools/c1_trace.py $k > $O/k_$k.log 2>&1 || { echo "trace failed"; exit 1; }
  f=$(find $O/k_$k -name "*kernel_stats.csv" | head -1); cp $f $O/kstats_c1_$k.csv; head -14 $f | cut -c1-110
done
