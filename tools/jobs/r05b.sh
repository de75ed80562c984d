#!/bin/bash
# sorted-run match (ZGPU_MATCH2=1) against the chain walk: interleaved A/B on
# the C4 launch shape, then the golden / sweep tests and the bench's full-shard
# reference check with it on
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
L=zlib.wasm_amd/libzgpu.so
for k in 1 2; do
  for m in 1 0; do
    ZGPU_MATCH2=$m timeout -k 10 120 python3 -u tools/ab_match.py $L 3 6 silesia 4096 >> $O/ab.log 2>&1 || { echo "ab failed"; tail -20 $O/ab.log; exit 1; }
  done
done
cat $O/ab.log | grep -v amdgpu.ids
ZGPU_MATCH2=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ZGPU_MATCH2=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=[json.loads(l) for l in open('$O/bench.log') if l.startswith('{')][-1]; print(d['value'], d['roofline']['avg_launch_ms'], d['stage_ms_per_step'], d['verified'])"
