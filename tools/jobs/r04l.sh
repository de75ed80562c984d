#!/bin/bash
# round 4: deflateParams slow <-> huff/rle sessions against the compiled reference's
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/run_api_sessions.py > $O/api_diff.log 2>&1; echo "api diff rc $?"
tail -15 $O/api_diff.log | cut -c1-300
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_stream.py tests/test_gpu_flush.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
