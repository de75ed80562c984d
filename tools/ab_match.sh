# A/B of k_match variants (ZGPU_MATCH_VARIANT):
#   bash tools/ab_match.sh <variant to test> "<stats variants>" "<bench variants>"
# parity tests (tests/test_gpu.py) of the first, walk statistics of the
# second list (4096 x 1 MiB, one launch), bench lines of the third
set -o pipefail
V=$1
ZGPU_MATCH_VARIANT=$V timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/v${V}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/v${V}_tests.log; [ $rc -eq 0 ] || exit $rc
for S in $2; do
  ZGPU_MATCH_VARIANT=$S timeout -k 10 200 python bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --crc-buffers 4096 --adler-buffers 0 --verify 2 > gpurun_out/v${S}_stats.json 2> gpurun_out/v${S}_stats.err || exit 1
done
for W in $3; do
  ZGPU_MATCH_VARIANT=$W timeout -k 10 200 python bench.py --steps 2 --warmup 1 --buffers 8192 --no-cpu --no-inflate --crc-buffers 4096 --adler-buffers 0 > gpurun_out/ab_v${W}.json 2> gpurun_out/ab_v${W}.err || exit 1
done
