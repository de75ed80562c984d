#!/bin/bash
# round 6: every first-call-is-the-header session that differs from the system zlib
set -o pipefail
T=${1:-r06t}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/header_first_probe.py > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | cut -c1-400
