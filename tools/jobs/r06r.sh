#!/bin/bash
# round 6: the first deflate() call whose output space is exactly a preset dictionary's header (modelled
# where the input's first string is not in the dictionary, refused before any output otherwise) against
# the system zlib, with the other stream / fuzz suites
set -o pipefail
T=${1:-r06r}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_zstream.py tests/test_gpu_flush.py tests/test_gpu_stream.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
