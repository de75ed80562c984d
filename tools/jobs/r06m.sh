#!/bin/bash
# round 6 final library, part 1: the whole GPU suite, smoke(), and the C1 latency of the final library
set -o pipefail
T=${1:-r06m}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python3 -u tools/c1_latency.py zlib.wasm_amd/libzgpu.so > $O/c1_latency.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_latency.log; exit 1; }
grep -v amdgpu.ids $O/c1_latency.log | grep -v "^stages"
