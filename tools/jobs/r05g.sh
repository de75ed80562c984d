#!/bin/bash
# streaming inflate diffs (randomized small-output sessions, reference
# sessions incl. Z_TREES / sync-held), the deflateParams streams, then the
# whole GPU suite
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/dbg/inflate_diff.py > $O/inflate_diff.log 2>&1; echo "inflate_diff rc $?"
grep -v amdgpu.ids $O/inflate_diff.log | cut -c1-400 | head -150
timeout -k 10 240 python3 -u tools/dbg/hrf_diff.py > $O/hrf_diff.log 2>&1; echo "hrf rc $?"
grep -c OK $O/hrf_diff.log; grep BAD $O/hrf_diff.log | head
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/gpu_tests.log | head -20
exit $rc
