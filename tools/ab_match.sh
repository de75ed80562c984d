# A/B of k_match variants (ZGPU_MATCH_VARIANT): parity tests, walk statistics, bench
set -o pipefail
V=${1:-40}
export ZGPU_MATCH_VARIANT=$V
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/v${V}_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/v${V}_tests.log
for S in 41 21; do
  ZGPU_MATCH_VARIANT=$S timeout -k 10 200 python bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --crc-buffers 4096 --adler-buffers 0 --verify 2 > gpurun_out/v${S}_stats.json 2> gpurun_out/v${S}_stats.err
done
for W in $V 19; do
  ZGPU_MATCH_VARIANT=$W timeout -k 10 200 python bench.py --steps 2 --warmup 1 --buffers 8192 --no-cpu --no-inflate --crc-buffers 4096 --adler-buffers 0 > gpurun_out/v${W}_bench.json 2> gpurun_out/v${W}_bench.err
done
