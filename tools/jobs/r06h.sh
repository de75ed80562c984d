#!/bin/bash
# round 6: A/B of the packed records + one-shot segment staging against the round's previous commit:
# lone 64 KiB compress2 latency (C1 shape), the C4 sub-batch, and the current library's C1 kernel trace
set -o pipefail
T=${1:-r06h}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for L in ab/libzgpu_r06head.so zlib.wasm_amd/libzgpu.so; do
    timeout -k 10 300 python3 -u tools/c1_latency.py $L >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
    timeout -k 10 120 python3 -u tools/ab_match.py $L 2 >> $O/sub_ab.log 2>&1 || { echo "ab failed"; tail -5 $O/sub_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/c1_ab.log | grep -v "^stages"
grep -v amdgpu.ids $O/sub_ab.log
for k in text mix; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$k -o run -- python3 tools/c1_trace.py $k > $O/k_$k.log 2>&1 || { echo "trace failed"; exit 1; }
  f=$(find $O/k_$k -name "*kernel_stats.csv" | head -1); cp $f $O/kstats_c1_$k.csv; head -14 $f | cut -c1-150
done
