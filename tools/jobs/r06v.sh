#!/bin/bash
# round 6: a pause behind the resume point dropped from the next job's events -- every first-call-is-the-header
# session with the length guard off against the system zlib, then the stream suites
set -o pipefail
T=${1:-r06v}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
ZGPU_HEADER_FIRST_ANY=1 timeout -k 10 600 python3 -u tools/header_first_probe.py > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-400 | tail -20
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_zstream.py tests/test_gpu_flush.py tests/test_gpu_stream.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
