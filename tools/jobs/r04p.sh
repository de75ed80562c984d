#!/bin/bash
# randomized deflate() sessions against the box's system zlib
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/fuzz.log 2>&1 || { echo "fuzz failed"; tail -60 $O/fuzz.log | cut -c1-3000; exit 1; }
tail -3 $O/fuzz.log
