#!/bin/bash
# round 6: Z_NO_FLUSH first calls whose output space is a preset dictionary's header, with the input in
# the dictionary: the dictionary-header tests against system zlib, then the z_stream and fuzz files
set -o pipefail
T=${1:-r07e}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_zstream.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
