# interleaved repeated A/B of k_match variants (bench 8192 x 1 MiB L6, 2 steps):
#   bash tools/ab_match_rep.sh "<variants>" <repeats>
set -o pipefail
mkdir -p gpurun_out/abr
for r in $(seq 1 ${2:-2}); do
  for W in $1; do
    ZGPU_MATCH_VARIANT=$W timeout -k 10 200 python bench.py --steps 2 --warmup 1 --buffers 8192 --no-cpu --no-inflate --crc-buffers 4096 --adler-buffers 0 --verify 1 > gpurun_out/abr/v${W}_r$r.json 2> gpurun_out/abr/v${W}_r$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['avg_launch_ms'])" gpurun_out/abr/v${W}_r$r.json $W $r
  done
done
