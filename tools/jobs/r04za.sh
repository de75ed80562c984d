#!/bin/bash
# C4: tapered first / last sub-batches against uniform ones (ZGPU_NO_TAPER)
set -o pipefail
O=gpurun_out/r04za
mkdir -p $O
A="--steps 3 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 --crc-buffers 4096"
for v in taper flat taper flat; do
  if [ $v = flat ]; then export ZGPU_NO_TAPER=1; else unset ZGPU_NO_TAPER; fi
  timeout -k 10 400 python3 bench.py $A > $O/c4_$v.json 2> $O/c4_$v.err || { echo "c4 $v failed"; tail -5 $O/c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified'])"
done
