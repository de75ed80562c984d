#!/bin/bash
# C4 stages without the pipeline (each alone), then a kernel trace of the same
set -o pipefail
O=gpurun_out/r04zb
mkdir -p $O
A="--steps 2 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 --crc-buffers 4096"
ZGPU_NO_PIPELINE=1 timeout -k 10 400 python3 bench.py $A > $O/c4_nopipe.json 2> $O/c4_nopipe.err || { echo "failed"; tail -5 $O/c4_nopipe.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4_nopipe.json')); print(d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
cd /tmp && ZGPU_NO_PIPELINE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o np -- python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof failed"; tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
