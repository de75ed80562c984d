#!/bin/bash
# round 6: CRC-32 table copies A/B (16 copies, 2 blocks per CU, vs 32 copies, conflict-free under the
# ds_read_b32 32-lane-group bank rule, 1 block per CU) on the C2 shape, interleaved; then the C3
# launch-size A/B (k_parse_fast per buffer with 16384 / 4096 / 1024 buffers per launch)
set -o pipefail
T=${1:-r06j}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for L in zlib.wasm_amd/libzgpu.so ab/libzgpu_crc32c.so; do
    timeout -k 10 120 python3 -u tools/ab_crc.py $L >> $O/crc_ab.log 2>&1 || { echo "crc failed"; tail -5 $O/crc_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/crc_ab.log
for B in 16384 4096 1024; do
  timeout -k 10 300 python3 -u tools/ab_match.py zlib.wasm_amd/libzgpu.so 2 1 enwik $B >> $O/c3_launch.log 2>&1 || { echo "c3 failed"; tail -5 $O/c3_launch.log; exit 1; }
done
grep -v amdgpu.ids $O/c3_launch.log
