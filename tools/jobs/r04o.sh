#!/bin/bash
# k_parse_fast LDS variant: its test, the L1-3 goldens, then lone-buffer speed with and without it
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fast_levels_lds or deflate_golden or random_sweep or wrappers_golden or dropin or wasm or strategies" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 -u tools/fast_lds_speed.py > $O/speed_lds.log 2>&1 || { echo "speed failed"; tail -20 $O/speed_lds.log; exit 1; }
ZGPU_FAST_LDS_MAX=0 timeout -k 10 300 python3 -u tools/fast_lds_speed.py > $O/speed_hbm.log 2>&1 || { echo "speed hbm failed"; tail -20 $O/speed_hbm.log; exit 1; }
paste -d'|' $O/speed_lds.log $O/speed_hbm.log
