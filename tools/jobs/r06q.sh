#!/bin/bash
# round 6: k_pbig3<true> (replays and run-ons of 256-byte segments from LDS copies): deflate suites and C1
# latency; then the C3 (no inflate leg: 64 GiB of inputs) and C5 bench lines of the round's library
set -o pipefail
T=${1:-r06q}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_bigbuf.py tests/test_gpu_stream.py tests/test_gpu_zstream.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so > $O/c1_latency.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_latency.log; exit 1; }
grep -v amdgpu.ids $O/c1_latency.log | grep -v "^stages"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_text -o run -- python3 tools/c1_trace.py text > $O/k_text.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find $O/k_text -name "*kernel_stats.csv" | head -1); cp $f $O/kstats_c1_text.csv; head -9 $f | cut -c1-110
timeout -k 10 300 python3 -u bench.py --level 1 --kind enwik --buffers 65536 --no-inflate > $O/bench_C3.json 2> $O/bench_C3.err || { echo "C3 failed"; tail -20 $O/bench_C3.err; exit 1; }
tail -c 300 $O/bench_C3.json
timeout -k 10 300 python3 -u bench.py --level 9 --kind vocab --buffers 256 --buffer-bytes 16777216 > $O/bench_C5.json 2> $O/bench_C5.err || { echo "C5 failed"; tail -20 $O/bench_C5.err; exit 1; }
tail -c 300 $O/bench_C5.json
