# timing of k_match probe variants (wrong results; no verification): bash tools/ab_probe.sh 45 33 ...
set -o pipefail
for W in "$@"; do
  ZGPU_MATCH_VARIANT=$W timeout -k 10 200 python bench.py --steps 2 --warmup 1 --buffers 8192 --no-cpu --no-inflate --crc-buffers 4096 --adler-buffers 0 --verify 0 > gpurun_out/ab_v${W}.json 2> gpurun_out/ab_v${W}.err || exit 1
done
