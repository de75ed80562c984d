#!/bin/bash
# round 6 final library: the C3 (L1, 65536 x 1 MiB enwik-style) and C5 (L9, 256 x 16 MiB) bench lines
set -o pipefail
T=${1:-r07g}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --level 1 --kind enwik --buffers 65536 --no-inflate > $O/bench_C3.json 2> $O/bench_C3.err || { echo "C3 failed"; tail -20 $O/bench_C3.err; exit 1; }
tail -c 200 $O/bench_C3.json
timeout -k 10 400 python3 -u bench.py --level 9 --kind vocab --buffers 256 --buffer-bytes 16777216 > $O/bench_C5.json 2> $O/bench_C5.err || { echo "C5 failed"; tail -20 $O/bench_C5.err; exit 1; }
tail -c 200 $O/bench_C5.json
