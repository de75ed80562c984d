#!/bin/bash
# the k_links_gh parameter test, and PMC FETCH_SIZE / WRITE_SIZE of k_links_gh and k_count on one 4 GiB sub-batch
# with the stages one after another (ZGPU_NO_PIPELINE=1)
set -o pipefail
O=gpurun_out/${R:-r05x2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "links_head or stage_links" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ARGS="--buffers 4096 --steps 1 --warmup 0 --no-cpu --no-inflate --verify 1 --crc-buffers 4096 --adler-buffers 0"
export ZGPU_NO_PIPELINE=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 bench.py $ARGS > $O/f.json 2> $O/f.err || { echo "pmc fetch failed"; tail -5 $O/f.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 bench.py $ARGS > $O/w.json 2> $O/w.err || { echo "pmc write failed"; tail -5 $O/w.err; exit 1; }
for k in k_links_gh k_count k_match; do echo "== $k"; python3 tools/pmc_summary.py $k $(find $O/f $O/w -name "*counter_collection.csv"); done
