#!/bin/bash
# A/B of the L6 pipeline order: links and match in parallel streams (default)
# against links then match on one stream with the previous tail beside them
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for m in 0 2; do
    ZGPU_PIPE_SERIAL=$m timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 --warmup 1 > $O/ab_$m.$k.json 2> $O/ab_$m.$k.err || { echo "bench failed"; tail -20 $O/ab_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$m.$k.json') if l.startswith('{')][-1]; print('serial=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact'], d['stage_ms_per_step'])"
  done
done
