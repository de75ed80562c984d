#!/bin/bash
# C4 sub-batch size A/B: 4 GiB (default) against 2 GiB in flight
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
A="--steps 3 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 --crc-buffers 4096"
for mb in 4096 2048 4096 2048; do
  timeout -k 10 400 python3 bench.py $A --inflight-mb $mb > $O/c4_$mb.json 2> $O/c4_$mb.err || { echo "c4 $mb failed"; tail -5 $O/c4_$mb.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$mb.json')); print('inflight $mb', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
