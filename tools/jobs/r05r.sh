#!/bin/bash
# A/B of the walks' stream priority (ZGPU_AUX_PRIO -1: greatest, 0: default, 1: least) on the C4 line
set -o pipefail
O=gpurun_out/${R:-r05r}
mkdir -p $O
export TMPDIR=/tmp
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream,'priority_range') else 'n/a')" || true
for k in 1 2; do
  for m in 0 -1 1; do
    ZGPU_AUX_PRIO=$m timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 --warmup 1 > $O/ab_$m.$k.json 2> $O/ab_$m.$k.err || { echo "bench failed"; tail -20 $O/ab_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$m.$k.json') if l.startswith('{')][-1]; print('prio=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact'], d['stage_ms_per_step'])"
  done
done
