#!/bin/bash
# streaming inflate accounting (reference sessions, randomized sessions vs
# system zlib), the inflate / flush tests, and the deflateParams
# fast <-> huff/rle sessions' first difference against the reference's bytes
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python3 -u tools/dbg/hrf_diff.py > $O/hrf_diff.log 2>&1; echo "hrf rc $?"
grep -v amdgpu.ids $O/hrf_diff.log | head -60
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_fuzz.py tests/test_gpu_inflate.py tests/test_gpu_flush.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|^E  " $O/tests.log | cut -c1-3000 | head -40
exit $rc
