#!/bin/bash
# round 4: k_parse_fast's 16-byte first compare (A/B against 64), the C3 shard's
# in-flight budget, lone-buffer rates (compress, uncompress)
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test_gpu.log 2>&1 || { echo "test_gpu failed"; tail -30 $O/test_gpu.log; exit 1; }
tail -1 $O/test_gpu.log
C3="--level 1 --kind enwik --buffers 65536 --steps 2 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 --crc-buffers 4096"
for v in new old new old; do
  if [ $v = old ]; then export ZGPU_FAST_CMP64=1; else unset ZGPU_FAST_CMP64; fi
  timeout -k 10 300 python3 bench.py $C3 > $O/c3_$v.json 2> $O/c3_$v.err || { echo "c3 $v failed"; tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
unset ZGPU_FAST_CMP64
for mb in 2048 8192; do
  timeout -k 10 300 python3 bench.py $C3 --inflight-mb $mb > $O/c3_if$mb.json 2> $O/c3_if$mb.err || { echo "c3 inflight $mb failed"; tail -5 $O/c3_if$mb.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_if$mb.json')); print('inflight $mb', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python3 -u tools/lone_inflate.py > $O/lone_inflate.log 2>&1 || { echo "lone inflate failed"; tail -5 $O/lone_inflate.log; exit 1; }
grep -v amdgpu.ids $O/lone_inflate.log
timeout -k 10 300 python3 -u tools/single_buffer.py > $O/single_buffer.log 2>&1 || { echo "single buffer failed"; tail -5 $O/single_buffer.log; exit 1; }
grep -v amdgpu.ids $O/single_buffer.log
