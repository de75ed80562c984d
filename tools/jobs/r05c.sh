#!/bin/bash
# L1-3 from the sorted runs (ZGPU_FAST_SRT=1): lone-buffer speed and exactness
# against the one-wave k_parse_fast, the L1-3 goldens, the stream sessions and
# a 256 MiB L1 streaming job with it on
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
ZGPU_FAST_SRT=1 timeout -k 10 200 python3 -u tools/lone_fast.py 1,2,3 1,16 text,mix > $O/lone_srt.log 2>&1 || { echo "srt failed"; tail -20 $O/lone_srt.log; exit 1; }
grep -v amdgpu.ids $O/lone_srt.log
timeout -k 10 200 python3 -u tools/lone_fast.py 1,3 1 text,mix > $O/lone_fast.log 2>&1 || { echo "fast failed"; tail -20 $O/lone_fast.log; exit 1; }
grep -v amdgpu.ids $O/lone_fast.log
ZGPU_FAST_SRT=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "golden or fast or sweep or batch" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ZGPU_FAST_SRT=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/stream_tests.log 2>&1 || { echo "stream tests failed"; tail -30 $O/stream_tests.log; exit 1; }
tail -2 $O/stream_tests.log
ZGPU_FAST_SRT=1 timeout -k 10 300 python3 -u tools/stream_stages.py 256 1 > $O/stream256.log 2>&1 || { echo "stream256 failed"; tail -20 $O/stream256.log; exit 1; }
grep -v amdgpu.ids $O/stream256.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_zstream.py -x -q --timeout 300 --timeout-method thread > $O/zstream_tests.log 2>&1 || { echo "zstream tests failed"; tail -30 $O/zstream_tests.log; exit 1; }
tail -2 $O/zstream_tests.log
for m in 1 0; do
  ZGPU_FAST_SRT=$m timeout -k 10 300 python3 -u tools/ab_match.py zlib.wasm_amd/libzgpu.so 1 1 enwik 16384 >> $O/c3_ab.log 2>&1 || { echo "c3 ab failed"; tail -20 $O/c3_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/c3_ab.log
