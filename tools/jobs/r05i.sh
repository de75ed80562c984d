#!/bin/bash
# streaming inflate diffs, then the zstream / fuzz / inflate / flush / batch tests
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/dbg/inflate_diff.py > $O/inflate_diff.log 2>&1; echo "inflate_diff rc $?"
grep -v amdgpu.ids $O/inflate_diff.log | cut -c1-400 | head -100
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_fuzz.py tests/test_gpu_inflate.py tests/test_gpu_flush.py tests/test_gpu.py tests/test_gpu_stream.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/tests.log | head -20
grep -E "^E  " $O/tests.log | cut -c1-600 | head -10
exit $rc
