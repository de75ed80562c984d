#!/bin/bash
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ck -o ck -- python3 tools/ck_trace.py > $O/ck_trace.log 2>&1 || { echo "ck trace failed"; tail -20 $O/ck_trace.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/c1 -o c1 -- python3 tools/c1_latency.py > $O/c1_trace.log 2>&1 || { echo "c1 trace failed"; tail -20 $O/c1_trace.log; exit 1; }
find $O -name "*stats.csv" | head
