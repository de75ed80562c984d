#!/bin/bash
# round 6 final library: kernel statistics of a lone 64 KiB compress2 (text, byte runs)
set -o pipefail
T=${1:-r07h}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for k in text mix; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$k -o run -- python3 tools/c1_trace.py $k > $O/k_$k.log 2>&1 || { echo "trace failed"; exit 1; }
  f=$(find $O/k_$k -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_c1_lone64KiB_$k.csv; head -8 $f | cut -c1-100
done
