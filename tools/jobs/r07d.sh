#!/bin/bash
# round 6 final library: the whole GPU suite, smoke(), C1 latency against the library before the batched
# result copies (ab/libzgpu_r07a.so), the default bench line and its rocprofv3 kernel statistics
set -o pipefail
T=${1:-r07d}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  for L in ab/libzgpu_r07a.so zlib.wasm_amd/libzgpu.so; do
    timeout -k 10 300 python3 -u tools/c1_latency.py $L >> $O/c1_ab.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/c1_ab.log | grep -v "^stages"
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
tail -c 300 $O/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-inflate > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_C4.csv; head -4 $f | cut -c1-120
