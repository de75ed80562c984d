# k_parse_fast rate vs buffers in flight (level 1, enwik-style 1 MiB): per-wave
# latency (few buffers) against contention (many)
set -e
T=${1:-ab_fast_occ}
mkdir -p gpurun_out/$T
for b in 256 2048 8192; do
  for v in ${VARIANTS:-0 3}; do
    ZGPU_FAST_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --level 1 --kind enwik \
      --buffers $b --inflight-mb 16384 --no-cpu --no-inflate --adler-buffers 0 --verify 1 --crc-buffers 4096 \
      > gpurun_out/$T/b${b}_v$v.json 2> gpurun_out/$T/b${b}_v$v.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], 'MB/s', d['stage_ms_per_step'])" \
      gpurun_out/$T/b${b}_v$v.json b$b v$v
  done
done
