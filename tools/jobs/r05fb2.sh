#!/bin/bash
# A/B on the C4 line: the fallback parse launch after k_parse_seg with a 256-position tile (2.3 KiB of LDS, the
# default) against the 4096-position tile (36 KiB, ZGPU_FB_BIGTILE=1); then the deflate tests that force fallbacks
set -o pipefail
O=gpurun_out/${R:-r05fb2}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for m in 0 1; do
    ZGPU_FB_BIGTILE=$m timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 --warmup 1 > $O/ab_$m.$k.json 2> $O/ab_$m.$k.err || { echo "bench failed"; tail -20 $O/ab_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$m.$k.json') if l.startswith('{')][-1]; print('bigtile=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact'], d['stage_ms_per_step'])"
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_fuzz.py tests/test_gpu_bigbuf.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "golden or sweep or pipeline or random_batches or few or single or fallback" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
