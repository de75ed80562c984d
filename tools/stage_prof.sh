# standalone (unpiped) stage times and rocprofv3 kernel statistics of one 4096 x 1 MiB L6 sub-batch
set -e
O=gpurun_out/${1:-stg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ab_match.py zlib.wasm_amd/libzgpu.so 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 tools/ab_match.py zlib.wasm_amd/libzgpu.so 2 > $O/run.log 2>&1
grep -E "zgpu" $O/stats/run_kernel_stats.csv | cut -c1-120
