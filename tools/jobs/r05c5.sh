#!/bin/bash
# the C5 and C3 lines with the final library, and the segmented-parse fallback counts on the C5 shape
set -o pipefail
O=gpurun_out/${R:-r05c5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 3 --warmup 1 > $O/bench_C5_256x16MiB_L9.json 2> $O/bench_C5.err || { echo "C5 bench failed"; tail -20 $O/bench_C5.err; exit 1; }
cut -c1-300 $O/bench_C5_256x16MiB_L9.json
timeout -k 10 400 python3 -u bench.py --level 1 --kind enwik --buffers 65536 --steps 3 --warmup 1 --no-inflate > $O/bench_C3_65536x1MiB_L1.json 2> $O/bench_C3.err || { echo "C3 bench failed"; tail -20 $O/bench_C3.err; exit 1; }
cut -c1-300 $O/bench_C3_65536x1MiB_L1.json
