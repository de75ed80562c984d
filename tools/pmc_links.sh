# SQ counters of k_links and k_count (rocprofv3 --pmc, one pass per counter set): 512 x 1 MiB at L6
set -o pipefail
export TMPDIR=/tmp
T=${1:-pmc_links}
mkdir -p gpurun_out/$T
ARGS="--steps 1 --warmup 0 --buffers 512 --no-cpu --no-inflate --verify 1 --crc-buffers 4096 --adler-buffers 0"
export ZGPU_NO_PIPELINE=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/$T/a -o run -- python3 bench.py $ARGS > gpurun_out/$T/a.json 2> gpurun_out/$T/a.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/b -o run -- python3 bench.py $ARGS > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_BARRIER_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/c -o run -- python3 bench.py $ARGS > gpurun_out/$T/c.json 2> gpurun_out/$T/c.err || true
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/k -o run -- python3 bench.py $ARGS > gpurun_out/$T/k.json 2> gpurun_out/$T/k.err || exit 1
for k in k_links k_count k_match; do echo "== $k"; python3 tools/pmc_summary.py $k $(find gpurun_out/$T -name "*counter_collection.csv"); done
grep -E "k_links|k_count|k_match" $(find gpurun_out/$T/k -name "*kernel_stats.csv")
