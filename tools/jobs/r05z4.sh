#!/bin/bash
# inflate with short matches copied one lane each (k_inflate_copy): the inflate-related GPU tests, then the C4 inflate leg (two runs) and a lone
# 1 MiB / 64 MiB uncompress
set -o pipefail
O=gpurun_out/${R:-r05z4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_par.py tests/test_gpu_fuzz.py tests/test_gpu_zstream.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --no-cpu --steps 2 --warmup 1 --crc-buffers 4096 --adler-buffers 0 > $O/b.$k.json 2> $O/b.$k.err || { echo "bench failed"; tail -20 $O/b.$k.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/b.$k.json') if l.startswith('{')][-1]; i=d['inflate']; print('lanecopy', d['value'], i['value'], i['round_trip_bit_exact_all_buffers'], i['stage_ms_per_step'])"
done
timeout -k 10 300 python3 -u tools/lone_inflate.py > $O/lone.log 2>&1 || { echo "lone failed"; tail -5 $O/lone.log; exit 1; }
cat $O/lone.log
