#!/bin/bash
# every inflate test with the parallel-decode threshold at 32 KiB
set -o pipefail
O=gpurun_out/r04y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_par.py tests/test_gpu.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log | cut -c1-1500; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 -u tools/lone_inflate.py > $O/lone.log 2>&1 && grep -v amdgpu.ids $O/lone.log
