#!/bin/bash
# streaming inflate diffs, then the inflate-side tests
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/dbg/inflate_diff.py > $O/inflate_diff.log 2>&1; echo "inflate_diff rc $?"
grep -v amdgpu.ids $O/inflate_diff.log | cut -c1-400 | head -150
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_fuzz.py tests/test_gpu_inflate.py tests/test_gpu_flush.py tests/test_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/tests.log | head -20
exit $rc
