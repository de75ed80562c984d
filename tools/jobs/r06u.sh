#!/bin/bash
# round 6: stream trace of a diverging first-call-is-the-header session (995: L4) and a passing one (1443: L6)
set -o pipefail
T=${1:-r06u}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for k in 995 1443; do
  ZGPU_STREAM_TRACE=1 timeout -k 10 120 python3 -u tools/header_first_trace.py $k > $O/trace_$k.log 2>&1 || { echo "trace failed"; tail -20 $O/trace_$k.log; exit 1; }
  grep -v amdgpu.ids $O/trace_$k.log | head -60 | cut -c1-330
done
