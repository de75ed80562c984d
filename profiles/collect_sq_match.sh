# SQ counters for the deflate kernels at L6 (one 512 MiB sub-batch): issue mix,
# wait states and LDS-array activity (rocprofv3 --pmc, two passes)
set -e
mkdir -p gpurun_out/sqm
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU --output-format csv -d gpurun_out/sqm/a -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 512 --no-cpu --verify 1 --crc-buffers 4096 > gpurun_out/sqm/a.json 2> gpurun_out/sqm/a.err
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sqm/b -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 512 --no-cpu --verify 1 --crc-buffers 4096 > gpurun_out/sqm/b.json 2> gpurun_out/sqm/b.err
