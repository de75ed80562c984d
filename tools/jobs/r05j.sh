#!/bin/bash
# randomized Z_TREES sessions against system zlib, with the first differing calls
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/dbg/inflate_diff.py > $O/inflate_diff.log 2>&1; echo "inflate_diff rc $?"
grep -v amdgpu.ids $O/inflate_diff.log | cut -c1-400 | head -120
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fuzz.py -k "inflate" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/tests.log | head
exit $rc
