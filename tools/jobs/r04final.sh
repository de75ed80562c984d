#!/bin/bash
# round-4 final: smoke(), the whole GPU suite, the default bench line
set -o pipefail
O=gpurun_out/r04final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=[json.loads(l) for l in open('$O/bench.log') if l.startswith('{')][-1]; print(d['value'], d['roofline']['avg_launch_ms'], d['crc32']['value'], d['inflate']['value'])"
