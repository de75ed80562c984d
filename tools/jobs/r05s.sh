#!/bin/bash
# A/B on the C4 line: tails on their own stream (ZGPU_TAIL_STREAM=1), with and without the greatest priority for
# the walks' and tails' streams (ZGPU_AUX_PRIO=-1), against the default pipeline
set -o pipefail
O=gpurun_out/${R:-r05s}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for m in "0 0" "1 0" "1 -1"; do
    set -- $m
    ZGPU_TAIL_STREAM=$1 ZGPU_AUX_PRIO=$2 timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 --warmup 1 > $O/ab_$1_$2.$k.json 2> $O/ab_$1_$2.$k.err || { echo "bench failed"; tail -20 $O/ab_$1_$2.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$1_$2.$k.json') if l.startswith('{')][-1]; print('tailstream=$1 prio=$2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact'], d['stage_ms_per_step'])"
  done
done
