#!/bin/bash
# round 5 final (last library of the round): smoke(), the whole GPU suite, the default bench line and its
# kernel statistics
set -o pipefail
T=${1:-r05v3}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/gpu_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
cut -c1-700 $O/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kstats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/kstats_bench.json 2> $O/kstats.err || { echo "kstats failed"; tail -5 $O/kstats.err; exit 1; }
find $O/kstats -name "*stats.csv"
exit $rc
