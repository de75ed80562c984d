#!/bin/bash
# rocprofv3 kernel stats of one L6 sub-batch (4096 x 1 MiB) per variant, no pipeline
set -e
mkdir -p gpurun_out/stats
export TMPDIR=/tmp
for v in "$@"; do
  ZGPU_MATCH_VARIANT=$v ZGPU_NO_PIPELINE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats/v$v -o run -- \
     python3 bench.py --steps 2 --warmup 1 --buffers 4096 --no-cpu --no-inflate --verify 2 --crc-buffers 1024 ${AB_ARGS} > gpurun_out/stats/v$v.json 2> gpurun_out/stats/v$v.err
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob(f"gpurun_out/stats/v{v}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("variant", v, r["Name"][:60], r["Calls"], "avg ms %.2f" % (float(r["AverageNs"]) / 1e6))
PY
done
