#!/bin/bash
# round 6: the product library after the k_lzp experiment moved to an A/B build -- deflate parity tests,
# the default line; then the A/B build's sub-batch beside the product's
set -o pipefail
T=${1:-r06e}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_bigbuf.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|Error" $O/gpu_tests.log | head -20
if [ $rc -ne 0 ]; then tail -40 $O/gpu_tests.log; exit $rc; fi
timeout -k 10 500 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
cut -c1-400 $O/bench_default.json
ZGPU_LZP=1 timeout -k 10 120 python3 -u tools/ab_match.py zlib.wasm_amd/libzgpu_lzp.so 2 > $O/ab_lzp.log 2>&1 || { echo "ab failed"; tail -20 $O/ab_lzp.log; exit 1; }
timeout -k 10 120 python3 -u tools/ab_match.py zlib.wasm_amd/libzgpu.so 2 > $O/ab_product.log 2>&1 || { echo "ab failed"; tail -20 $O/ab_product.log; exit 1; }
cat $O/ab_lzp.log $O/ab_product.log | grep -v amdgpu.ids
