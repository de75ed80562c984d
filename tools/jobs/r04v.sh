#!/bin/bash
# randomized batches of the hot path against system zlib
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -v --timeout 280 --timeout-method thread -k batches > $O/batches.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/batches.log | tail -6
grep -n "AssertionError" $O/batches.log | head -2 | cut -c1-1500
exit $rc
