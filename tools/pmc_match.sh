# SQ counters of k_match for two variants (rocprofv3 --pmc, one pass per counter set)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for V in "$@"; do
  export ZGPU_MATCH_VARIANT=$V
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc/v${V}a -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 512 --no-cpu --no-inflate --verify 1 --crc-buffers 4096 --adler-buffers 0 > gpurun_out/pmc/v${V}a.json 2> gpurun_out/pmc/v${V}a.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/v${V}b -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 512 --no-cpu --no-inflate --verify 1 --crc-buffers 4096 --adler-buffers 0 > gpurun_out/pmc/v${V}b.json 2> gpurun_out/pmc/v${V}b.err || exit 1
done
