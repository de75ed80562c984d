#!/bin/bash
# round 5: the C3 and C5 bench lines (their roofline traffic from the r05y PMC passes)
set -o pipefail
T=${1:-r05x}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --level 1 --kind enwik --buffers 65536 --steps 3 --warmup 1 --no-inflate > $O/bench_C3_65536x1MiB_L1.json 2> $O/bench_C3.err || { echo "C3 bench failed"; tail -20 $O/bench_C3.err; exit 1; }
cut -c1-500 $O/bench_C3_65536x1MiB_L1.json
timeout -k 10 400 python3 -u bench.py --level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 3 --warmup 1 > $O/bench_C5_256x16MiB_L9.json 2> $O/bench_C5.err || { echo "C5 bench failed"; tail -20 $O/bench_C5.err; exit 1; }
cut -c1-500 $O/bench_C5_256x16MiB_L9.json
