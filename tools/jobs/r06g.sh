#!/bin/bash
# round 6: k_match records packed (rquart only where it differs, a flag bit in rfull):
# deflate parity tests, sub-batch A/B timing, PMC FETCH/WRITE of the C4 and C5 launch shapes
set -o pipefail
T=${1:-r06g}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_bigbuf.py tests/test_gpu_flush.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|Error" $O/gpu_tests.log | head -20
if [ $rc -ne 0 ]; then tail -40 $O/gpu_tests.log; exit $rc; fi
timeout -k 10 120 python3 -u tools/ab_match.py zlib.wasm_amd/libzgpu.so 2 > $O/ab_packed.log 2>&1 || { echo "ab failed"; tail -20 $O/ab_packed.log; exit 1; }
grep -v amdgpu.ids $O/ab_packed.log
A4="--steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
A5="--level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 1 --warmup 0 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
pick() { find "$1" -name "*counter_collection.csv" | head -1; }
pass() {   # tag counter shape args...
  local tag=$1 ctr=$2 shape=$3; shift 3
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/$tag -o run -- python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "pmc $tag failed"; tail -5 $O/$tag.err; exit 1; }
  local lc=$(echo $ctr | sed 's/_SIZE//' | tr 'A-Z' 'a-z')
  cp "$(pick $O/$tag)" $O/${T}_pmc_${lc}_${shape}.csv
  echo "pmc $tag ok"
}
pass c4f FETCH_SIZE L6_4096x1048576 $A4
pass c4w WRITE_SIZE L6_4096x1048576 $A4
pass c5f FETCH_SIZE L9_256x16777216 $A5
pass c5w WRITE_SIZE L9_256x16777216 $A5
python3 tools/pmc_kernels.py $O/*_pmc_*.csv > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt | head -30
timeout -k 10 300 python3 -u tools/c1_latency.py > $O/c1_latency.log 2>&1 || { echo "c1 failed"; tail -5 $O/c1_latency.log; exit 1; }
grep -v amdgpu.ids $O/c1_latency.log
