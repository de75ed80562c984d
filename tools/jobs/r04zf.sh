#!/bin/bash
# streaming inflate() consumption at output-limited stops: every inflate test
set -o pipefail
O=gpurun_out/r04zf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_zstream.py tests/test_gpu_inflate.py tests/test_gpu_inflate_par.py -m gpu -v --timeout 300 --timeout-method thread -k "inflate or zstream or isession or back or session" > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | tail -8
grep -n "AssertionError" $O/tests.log | head -2 | cut -c1-1800
exit $rc
