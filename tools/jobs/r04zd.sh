#!/bin/bash
# deflate() sessions whose flushes end with output pending and are followed by more input
set -o pipefail
O=gpurun_out/r04zd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -v --timeout 280 --timeout-method thread -k "pending or header" > $O/pending.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pending.log | tail -4
grep -n "AssertionError" $O/pending.log | head -1 | cut -c1-2500
exit $rc
