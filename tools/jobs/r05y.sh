#!/bin/bash
# round 5: PMC FETCH_SIZE / WRITE_SIZE passes (separate runs) of the C4, C3
# and C5 launch shapes, copied into profiles/ for bench.py's roofline, then
# (the C3 / C5 bench lines that read them: tools/jobs/r05x.sh)
set -o pipefail
T=${1:-r05y}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
A4="--steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
A3="--steps 1 --warmup 0 --level 1 --kind enwik --buffers 16384 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
A5="--level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 1 --warmup 0 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
pick() { find "$1" -name "*counter_collection.csv" | head -1; }
pass() {   # tag counter shape args...
  local tag=$1 ctr=$2 shape=$3; shift 3
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/$tag -o run -- python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "pmc $tag failed"; tail -5 $O/$tag.err; exit 1; }
  local lc=$(echo $ctr | sed 's/_SIZE//' | tr 'A-Z' 'a-z')
  cp "$(pick $O/$tag)" profiles/${T}_pmc_${lc}_${shape}.csv
  cp "$(pick $O/$tag)" $O/${T}_pmc_${lc}_${shape}.csv
  echo "pmc $tag ok"
}
pass c4f FETCH_SIZE L6_4096x1048576 $A4
pass c4w WRITE_SIZE L6_4096x1048576 $A4
pass c3f FETCH_SIZE L1_16384x1048576 $A3
pass c3w WRITE_SIZE L1_16384x1048576 $A3
pass c5f FETCH_SIZE L9_256x16777216 $A5
pass c5w WRITE_SIZE L9_256x16777216 $A5
