#!/bin/bash
# block-parallel lone-stream inflate: its tests and lone uncompress speed; then the randomized sessions
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_inflate_par.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/par_tests.log 2>&1 || { echo "par tests failed"; tail -50 $O/par_tests.log | cut -c1-3000; exit 1; }
tail -2 $O/par_tests.log
timeout -k 10 200 python3 -u tools/lone_inflate.py > $O/lone_inflate.log 2>&1 || { echo "lone failed"; tail -20 $O/lone_inflate.log; exit 1; }
cat $O/lone_inflate.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/fuzz.log 2>&1 || { echo "fuzz failed"; tail -60 $O/fuzz.log | cut -c1-3000; exit 1; }
tail -3 $O/fuzz.log
