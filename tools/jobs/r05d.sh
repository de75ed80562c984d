#!/bin/bash
# the whole GPU suite (exact streaming inflate accounting), then the C3 launch
# shape with L1 from the sorted runs (ZGPU_FAST_SRT=1) against k_parse_fast
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
tail -60 $O/gpu_tests.log
echo "tests rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in 1 0; do
  ZGPU_FAST_SRT=$m timeout -k 10 300 python3 -u tools/ab_match.py zlib.wasm_amd/libzgpu.so 1 1 enwik 16384 >> $O/c3_ab.log 2>&1 || { echo "c3 ab failed"; tail -20 $O/c3_ab.log; exit 1; }
done
grep -v amdgpu.ids $O/c3_ab.log
exit $rc
