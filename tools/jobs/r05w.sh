#!/bin/bash
# A/B on the C4 line: the pipeline's links on a third stream beside the tails (default) against links after the
# tail on the caller's stream (ZGPU_LINKS_STREAM=0); then the pipeline tests on the new order
set -o pipefail
O=gpurun_out/${R:-r05w}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for m in 1 0; do
    ZGPU_LINKS_STREAM=$m timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 --warmup 1 > $O/ab_$m.$k.json 2> $O/ab_$m.$k.err || { echo "bench failed"; tail -20 $O/ab_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$m.$k.json') if l.startswith('{')][-1]; print('links_stream=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact'], d['stage_ms_per_step'])"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_inflate.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "pipeline or many or bench_scale or golden" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
