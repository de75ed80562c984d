#!/bin/bash
# k_parse_fast with 16-bit swept head[] in HBM (kH16) against the 32-bit head: L1-3 tests, then the C3 shard A/B
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fast_levels or random_sweep or deflate_golden or batches or generator_kinds or bench_scale" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C3="--level 1 --kind enwik --buffers 65536 --steps 2 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 --crc-buffers 4096"
for v in h16 h32 h16 h32; do
  if [ $v = h32 ]; then export ZGPU_FAST_H16=0; else unset ZGPU_FAST_H16; fi
  timeout -k 10 300 python3 bench.py $C3 > $O/c3_$v.json 2> $O/c3_$v.err || { echo "c3 $v failed"; tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
