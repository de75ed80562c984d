# SQ counter pass for the deflate kernels (one 512 MiB sub-batch, level 6)
set -e
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU --output-format csv -d gpurun_out/sq/a -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 512 --no-cpu --verify 1 --crc-buffers 4096 > gpurun_out/sq/a.json 2> gpurun_out/sq/a.err
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq/b -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 512 --no-cpu --verify 1 --crc-buffers 4096 > gpurun_out/sq/b.json 2> gpurun_out/sq/b.err
