#!/bin/bash
# round 4: inflate decode registers back (codes_used in LDS), re-checked by the
# z_stream inflate sessions; C3 PMC passes of the current k_parse_fast; the
# default bench line
set -o pipefail
T=r04k
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A3="--steps 1 --warmup 0 --level 1 --kind enwik --buffers 16384 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
pick() { find "$1" -name "*counter_collection.csv" | head -1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3f -o run -- python3 bench.py $A3 > $O/c3f.json 2> $O/c3f.err || { echo "pmc fetch failed"; tail -5 $O/c3f.err; exit 1; }
cp "$(pick $O/c3f)" $O/${T}_pmc_fetch_L1_16384x1048576.csv
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3w -o run -- python3 bench.py $A3 > $O/c3w.json 2> $O/c3w.err || { echo "pmc write failed"; tail -5 $O/c3w.err; exit 1; }
cp "$(pick $O/c3w)" $O/${T}_pmc_write_L1_16384x1048576.csv
timeout -k 10 500 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['inflate']['value'], d['inflate'].get('stage_ms_per_step'))"
