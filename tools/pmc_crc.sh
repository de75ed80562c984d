#!/bin/bash
# PMC counters of k_crc32 on the C2 workload (1 M x 4 KiB); PMC="..." selects the counters
set -e
mkdir -p gpurun_out/pmcc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc ${PMC} --kernel-include-regex k_crc32 --output-format csv -d gpurun_out/pmcc/r -o run -- \
   python3 bench.py --buffers 64 --no-cpu --no-inflate --verify 1 --steps 2 --warmup 1 > gpurun_out/pmcc/r.json 2> gpurun_out/pmcc/r.err
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmcc/r/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: f"{sum(v)/len(v):.4g}" for k, v in sorted(d.items())})
PY
