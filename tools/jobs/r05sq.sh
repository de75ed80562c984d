#!/bin/bash
# SQ counters of k_match in the pipeline (8192 x 1 MiB: two sub-batches, links and tail beside the walks) and
# with the stages one after another (ZGPU_NO_PIPELINE=1): what the walks lose to their neighbours
set -o pipefail
O=gpurun_out/${R:-r05sq}
mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --buffers 8192 --no-cpu --no-inflate --verify 1 --crc-buffers 4096 --adler-buffers 0"
for mode in pipe alone; do
  if [ $mode = alone ]; then export ZGPU_NO_PIPELINE=1; else unset ZGPU_NO_PIPELINE; fi
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/$mode/a -o run -- python3 bench.py $ARGS > $O/$mode.a.json 2> $O/$mode.a.err || { echo "pass a failed"; tail -5 $O/$mode.a.err; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/$mode/b -o run -- python3 bench.py $ARGS > $O/$mode.b.json 2> $O/$mode.b.err || { echo "pass b failed"; tail -5 $O/$mode.b.err; exit 1; }
  echo "== k_match, $mode"
  python3 tools/pmc_summary.py "k_match<false, false>" $(find $O/$mode -name "*counter_collection.csv")
done
