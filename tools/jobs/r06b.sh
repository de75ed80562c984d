#!/bin/bash
# round 6: k_lzp statistics build (priority on / off) and A/B of one 4096 x 1 MiB L6 sub-batch
set -o pipefail
T=${1:-r06d}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for f in 3 1; do
  ZGPU_LZP_FLAGS=$f timeout -k 10 120 python3 -u tools/lzp_stats.py > $O/stats_flags$f.log 2>&1 || { echo "stats failed"; tail -20 $O/stats_flags$f.log; exit 1; }
  echo "flags $f"; cat $O/stats_flags$f.log
done
for f in 3 1; do
  ZGPU_LZP_FLAGS=$f timeout -k 10 120 python3 -u tools/ab_match.py zlib.wasm_amd/libzgpu.so 2 > $O/ab_flags$f.log 2>&1 || { echo "ab failed"; tail -20 $O/ab_flags$f.log; exit 1; }
  echo "flags $f"; cat $O/ab_flags$f.log
done
true
true
