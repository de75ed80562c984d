#!/bin/bash
# round 4: checksum parity + call latency, PMC of the C4 launch shape, the
# default bench line and its kernel statistics
set -o pipefail
T=r04h
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -k "crc or adler or checksum" -x -q --timeout 200 --timeout-method thread > $O/ck_tests.log 2>&1 || { echo "checksum tests failed"; tail -30 $O/ck_tests.log; exit 1; }
tail -1 $O/ck_tests.log
timeout -k 10 120 python3 -u tools/ck_latency.py 200 > $O/ck_latency.log 2>&1 || { echo "ck latency failed"; exit 1; }
grep -v amdgpu.ids $O/ck_latency.log
A4="--steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
pick() { find "$1" -name "*counter_collection.csv" | head -1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4f -o run -- python3 bench.py $A4 > $O/c4f.json 2> $O/c4f.err || { echo "pmc fetch failed"; tail -5 $O/c4f.err; exit 1; }
cp "$(pick $O/c4f)" profiles/${T}_pmc_fetch_L6_4096x1048576.csv
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4w -o run -- python3 bench.py $A4 > $O/c4w.json 2> $O/c4w.err || { echo "pmc write failed"; tail -5 $O/c4w.err; exit 1; }
cp "$(pick $O/c4w)" profiles/${T}_pmc_write_L6_4096x1048576.csv
cp profiles/${T}_pmc_* $O/
timeout -k 10 500 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kstats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/kstats_bench.json 2> $O/kstats.err || { echo "kstats failed"; tail -5 $O/kstats.err; exit 1; }
find $O/kstats -name "*stats.csv"
