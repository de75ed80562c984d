#!/bin/bash
# the GPU suite, then kernel traces of single checksum calls and the lone 64 KiB compress2
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ck -o ck -- python3 tools/ck_trace.py > $O/ck_trace.log 2>&1 || { echo "ck trace failed"; tail -20 $O/ck_trace.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/c1 -o c1 -- python3 tools/c1_latency.py > $O/c1_trace.log 2>&1 || { echo "c1 trace failed"; tail -20 $O/c1_trace.log; exit 1; }
find $O -name "*stats.csv"
