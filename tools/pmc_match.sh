#!/bin/bash
# LDS-side PMC counters of k_match for the given variants (one 512 x 1 MiB L6
# sub-batch, no pipeline).  Usage: tools/pmc_match.sh V1 V2 ...
set -e
mkdir -p gpurun_out/pmcm
export TMPDIR=/tmp
for v in "$@"; do
  ZGPU_MATCH_VARIANT=$v ZGPU_NO_PIPELINE=1 timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE} \
     --kernel-include-regex k_match --output-format csv -d gpurun_out/pmcm/v$v -o run -- \
     python3 bench.py --steps 1 --warmup 0 --buffers 512 --no-cpu --no-inflate --verify 1 --crc-buffers 1024 > gpurun_out/pmcm/v$v.json 2> gpurun_out/pmcm/v$v.err
  python3 - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
f = glob.glob(f"gpurun_out/pmcm/v{v}/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if "k_match" in r["Kernel_Name"]:
        d[r["Counter_Name"]] += float(r["Counter_Value"])
print("variant", v, {k: f"{x:.4g}" for k, x in sorted(d.items())})
PY
done
