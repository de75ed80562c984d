#!/bin/bash
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
ZGPU_PAR_INFLATE_MIN=0 timeout -k 10 200 python3 -u tools/par_threshold.py > $O/par.log 2>&1 || { tail -5 $O/par.log; exit 1; }
ZGPU_NO_PAR_INFLATE=1 timeout -k 10 200 python3 -u tools/par_threshold.py > $O/seq.log 2>&1 || { tail -5 $O/seq.log; exit 1; }
paste -d'|' <(grep KiB $O/par.log) <(grep KiB $O/seq.log)
