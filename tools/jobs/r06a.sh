#!/bin/bash
# round 6: first k_lzp run -- the deflate parity tests, then the default line with k_lzp and without (A/B)
set -o pipefail
T=${1:-r06a}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|Error" $O/gpu_tests.log | head -20
if [ $rc -ne 0 ]; then tail -40 $O/gpu_tests.log; exit $rc; fi
timeout -k 10 400 python3 -u bench.py --no-cpu --no-inflate > $O/bench_lzp.json 2> $O/bench_lzp.err || { echo "bench failed"; tail -20 $O/bench_lzp.err; exit 1; }
cut -c1-600 $O/bench_lzp.json
ZGPU_LZP=0 timeout -k 10 400 python3 -u bench.py --no-cpu --no-inflate > $O/bench_old.json 2> $O/bench_old.err || { echo "bench old failed"; tail -20 $O/bench_old.err; exit 1; }
cut -c1-600 $O/bench_old.json
