#!/bin/bash
# the whole GPU suite on the final round-4 library, then the default bench line
set -o pipefail
O=gpurun_out/${RUN_TAG:-r04n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
