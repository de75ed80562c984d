#!/bin/bash
# randomized sessions + z_stream goldens, then a kernel trace of the lone block-parallel uncompress
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_zstream.py -m gpu -v --timeout 280 --timeout-method thread > $O/fuzz.log 2>&1 || { grep -E "FAILED|passed|failed" $O/fuzz.log | tail; grep -n AssertionError $O/fuzz.log | head -3 | cut -c1-1500; exit 1; }
grep -E "passed|failed" $O/fuzz.log | tail -2
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o lone -- python3 $GRAFT_REPO_ROOT/tools/lone_inflate.py > $GRAFT_REPO_ROOT/$O/lone.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/$O/lone.log; exit 1; }
cd $GRAFT_REPO_ROOT && grep -v amdgpu.ids $O/lone.log | tail -4
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -14'
