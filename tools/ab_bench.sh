# bench-only A/B of k_match variants: bash tools/ab_bench.sh 40 42 ...
set -o pipefail
for W in "$@"; do
  ZGPU_MATCH_VARIANT=$W timeout -k 10 200 python bench.py --steps 2 --warmup 1 --buffers 8192 --no-cpu --no-inflate --crc-buffers 4096 --adler-buffers 0 > gpurun_out/ab_v${W}.json 2> gpurun_out/ab_v${W}.err || exit 1
done
