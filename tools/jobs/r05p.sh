#!/bin/bash
# k_parse_fast on k_links' chains (kLk): L1-3 tests with every batch on the HBM variant, then an A/B on the C3 shard
set -o pipefail
O=gpurun_out/${R:-r05p}
mkdir -p $O
export TMPDIR=/tmp
ZGPU_FAST_LDS_MAX=0 timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_fuzz.py tests/test_gpu_bigbuf.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "golden or fast or random or sweep or few or single or wrappers" > $O/tests_lds0.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_lds0.log; exit 1; }
tail -2 $O/tests_lds0.log
for k in 1 2; do
  for m in 1 0; do
    ZGPU_FAST_LINKS=$m timeout -k 10 400 python3 -u bench.py --level 1 --kind enwik --buffers 65536 --steps 2 --warmup 1 --no-inflate --no-cpu > $O/c3_$m.$k.json 2> $O/c3_$m.$k.err || { echo "bench failed"; tail -20 $O/c3_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/c3_$m.$k.json') if l.startswith('{')][-1]; print('links=$m', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), d['verified'], d['stage_ms_per_step'])"
  done
done
