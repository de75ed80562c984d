#!/bin/bash
# A/B of the batched inflate decode at 5 waves per SIMD (96 VGPRs, ZGPU_INFL_W5=1) against 4 (125 VGPRs)
set -o pipefail
O=gpurun_out/${R:-r05y2}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for m in 1 0; do
    ZGPU_INFL_W5=$m timeout -k 10 400 python3 -u bench.py --no-cpu --steps 2 --warmup 1 --crc-buffers 4096 --adler-buffers 0 > $O/ab_$m.$k.json 2> $O/ab_$m.$k.err || { echo "bench failed"; tail -20 $O/ab_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$m.$k.json') if l.startswith('{')][-1]; i=d['inflate']; print('w5=$m', d['value'], i['value'], i['round_trip_bit_exact_all_buffers'], i['stage_ms_per_step'])"
  done
done
