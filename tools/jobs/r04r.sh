#!/bin/bash
# randomized sessions + the inflate / z_stream goldens after the Z_BLOCK header fix
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_zstream.py -m gpu -v --timeout 280 --timeout-method thread > $O/fuzz.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/fuzz.log | tail -20
exit $rc
