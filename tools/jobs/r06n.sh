#!/bin/bash
# round 6 final library, part 2: the default bench line, its rocprofv3 kernel statistics, and the C3 / C5 lines
set -o pipefail
T=${1:-r06n}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
tail -c 600 $O/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-inflate > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_C4.csv; head -12 $f | cut -c1-120
timeout -k 10 300 python3 -u bench.py --level 1 --kind enwik --buffers 65536 > $O/bench_C3.json 2> $O/bench_C3.err || { echo "C3 failed"; tail -20 $O/bench_C3.err; exit 1; }
tail -c 300 $O/bench_C3.json
timeout -k 10 300 python3 -u bench.py --level 9 --kind vocab --buffers 256 --buffer-bytes 16777216 > $O/bench_C5.json 2> $O/bench_C5.err || { echo "C5 failed"; tail -20 $O/bench_C5.err; exit 1; }
tail -c 300 $O/bench_C5.json
