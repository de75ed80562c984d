# SQ counters of k_parse_fast (level 1, 16384 x 1 MiB enwik-style), one pass per counter set
set -o pipefail
export TMPDIR=/tmp
T=${1:-pmc_fast}
mkdir -p gpurun_out/$T
ARGS="--steps 1 --warmup 0 --level 1 --kind enwik --buffers ${BUFS:-16384} --no-cpu --no-inflate --verify 1 --crc-buffers 4096 --adler-buffers 0"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/$T/a -o run -- python3 bench.py $ARGS > gpurun_out/$T/a.json 2> gpurun_out/$T/a.err
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/b -o run -- python3 bench.py $ARGS > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err
python3 tools/pmc_summary.py k_parse_fast $(find gpurun_out/$T -name "*counter_collection.csv")
