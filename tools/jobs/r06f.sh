#!/bin/bash
# round 6: the whole GPU suite on the product library after the hygiene changes
set -o pipefail
T=${1:-r06f}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/gpu_tests.log | head -20
exit $rc
