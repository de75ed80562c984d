#!/bin/bash
# round 4: streaming jobs on the segmented parse + block encoder -- parity, then timing
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_zstream.py > $O/stream_tests.log 2>&1 || { echo "stream tests failed"; tail -30 $O/stream_tests.log; exit 1; }
timeout -k 10 300 python3 -u tools/stream_stages.py 256 > $O/stages_seg.log 2>&1 || { echo "stages failed"; tail -20 $O/stages_seg.log; exit 1; }
grep -v amdgpu.ids $O/stages_seg.log
timeout -k 10 500 python3 -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_gpu_bigbuf.py -k "over_4gib and 6" > $O/c2big.log 2>&1 || { echo "c2big failed"; tail -30 $O/c2big.log; exit 1; }
grep -E "zlib|libzgpu|passed|failed" $O/c2big.log
timeout -k 10 200 python3 -u tools/ck_latency.py 200 > $O/ck_latency.log 2>&1 || { echo "ck latency failed"; tail -5 $O/ck_latency.log; exit 1; }
grep -v amdgpu.ids $O/ck_latency.log
timeout -k 10 200 python3 -u tools/c1_latency.py > $O/c1_latency.log 2>&1 || { echo "c1 latency failed"; tail -5 $O/c1_latency.log; exit 1; }
grep -v amdgpu.ids $O/c1_latency.log
