#!/bin/bash
# k_parse_seg with 32-byte lane windows against 16-byte: L4-9 tests, then the C4 A/B
set -o pipefail
O=gpurun_out/r04zc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "deflate_golden or random_sweep or pipeline or bench_scale or batches or literal or pathological or strategies or window_bits" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--steps 3 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 --crc-buffers 4096"
for v in w32 w16 w32 w16; do
  if [ $v = w16 ]; then export ZGPU_PARSE_WIN=16; else unset ZGPU_PARSE_WIN; fi
  timeout -k 10 400 python3 bench.py $A > $O/c4_$v.json 2> $O/c4_$v.err || { echo "c4 $v failed"; tail -5 $O/c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$v.json')); print('$v', d['value'], d['ms_per_step'], d['stage_ms_per_step']['parse_lazy'], d['verified']['all_status_ok'])"
done
