#!/bin/bash
# the header-fills-output rule: pending-flush sessions and every streaming deflate golden
set -o pipefail
O=gpurun_out/r04ze
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_stream.py tests/test_gpu_zstream.py tests/test_gpu_flush.py -m gpu -v -rxX --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|XPASS|XFAIL|passed|failed" $O/tests.log | tail -12
grep -n "AssertionError" $O/tests.log | head -2 | cut -c1-1500
exit $rc
