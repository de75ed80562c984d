# A/B of the k_parse_fast variants (ZGPU_FAST_VARIANT 0/1/2) on level-1
# workloads: C3-shaped enwik text and the Silesia-style mix, 16384 x 1 MiB.
# Usage (GPU box): bash tools/ab_fast.sh [tag]
set -e
T=${1:-ab_fast}
mkdir -p gpurun_out/$T
for kind in enwik silesia; do
  for v in ${VARIANTS:-0 1 2}; do
    ZGPU_FAST_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --level ${LEVEL:-1} --kind $kind \
      --buffers ${BUFS:-16384} --no-cpu --no-inflate --adler-buffers 0 --verify 4 \
      > gpurun_out/$T/${kind}_v$v.json 2> gpurun_out/$T/${kind}_v$v.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], 'MB/s', d['stage_ms_per_step'])" \
      gpurun_out/$T/${kind}_v$v.json $kind v$v
  done
done
