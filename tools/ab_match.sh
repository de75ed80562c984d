#!/bin/bash
# A/B of k_match variants on one L6 sub-batch (4096 x 1 MiB Silesia-style),
# no pipeline so per-stage times are clean.  Usage: tools/ab_match.sh V1 V2 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  ZGPU_MATCH_VARIANT=$v ZGPU_NO_PIPELINE=1 timeout -k 10 240 python bench.py --buffers 4096 --steps 2 --warmup 1 \
      --no-cpu --no-inflate --verify 4 --crc-buffers 1024 ${AB_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json"))
print("variant", sys.argv[1], "MB/s", d["value"], "stages", d["stage_ms_per_step"])
PY
done
