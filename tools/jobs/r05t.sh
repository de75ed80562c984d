#!/bin/bash
# k_links_w (one wave per buffer, no LDS, beside k_match): deflate tests with it forced everywhere, then an A/B on
# the C4 line against the LDS k_links
set -o pipefail
O=gpurun_out/${R:-r05t}
mkdir -p $O
export TMPDIR=/tmp
ZGPU_LINKS_W=2 timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "stage_links or golden or sweep or pipeline or bench_scale or few" > $O/tests_w2.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_w2.log; exit 1; }
tail -2 $O/tests_w2.log
for k in 1 2; do
  for m in 1 0; do
    ZGPU_LINKS_W=$m timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 --warmup 1 > $O/ab_$m.$k.json 2> $O/ab_$m.$k.err || { echo "bench failed"; tail -20 $O/ab_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$m.$k.json') if l.startswith('{')][-1]; print('links_w=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact'], d['stage_ms_per_step'])"
  done
done
