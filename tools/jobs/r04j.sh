#!/bin/bash
# round 4: the C3 line (no inflate leg: the 64 GiB shard leaves no room for it),
# lone-buffer rates (uncompress, compress)
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/lone_inflate.py > $O/lone_inflate.log 2>&1 || { echo "lone inflate failed"; tail -5 $O/lone_inflate.log; exit 1; }
grep -v amdgpu.ids $O/lone_inflate.log
timeout -k 10 300 python3 -u tools/single_buffer.py > $O/single_buffer.log 2>&1 || { echo "single buffer failed"; tail -5 $O/single_buffer.log; exit 1; }
grep -v amdgpu.ids $O/single_buffer.log
timeout -k 10 500 python3 bench.py --level 1 --kind enwik --buffers 65536 --steps 3 --warmup 1 --no-inflate > $O/bench_C3_65536x1MiB_L1.json 2> $O/bench_C3.err || { echo "C3 failed"; tail -5 $O/bench_C3.err; exit 1; }
cut -c1-400 $O/bench_C3_65536x1MiB_L1.json
