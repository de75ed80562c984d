#!/bin/bash
# kernel and runtime trace of a lone 1 MiB uncompress (10 calls)
set -o pipefail
O=gpurun_out/${R:-r05v}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --runtime-trace --stats --output-format csv -d $O/t -o run -- python3 tools/lone_inflate_one.py 1 10 > $O/calls.log 2> $O/err.log || { echo "trace failed"; tail -5 $O/err.log; exit 1; }
cat $O/calls.log
for f in $(find $O/t -name "*stats.csv"); do echo "== $f"; head -25 $f | cut -c1-150; done
