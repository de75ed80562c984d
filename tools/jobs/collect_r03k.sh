# the rest of round 3's lines: C3 shard at L1 (no inflate leg: 64 GiB in + 64 GiB out), single-buffer rates,
# the 64 KiB latency
set -e
O=gpurun_out/${1:-r03k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py --kind enwik --level 1 --buffers 65536 --steps 2 --warmup 1 --no-inflate > $O/bench_C3.json 2> $O/bench_C3.err
python3 -c "import json; d=json.load(open('$O/bench_C3.json')); print('C3', d['value'], d['cpu_baseline']['value'])"
timeout -k 10 200 python3 -u tools/single_buffer.py > $O/single_buffer.log 2>&1
timeout -k 10 200 python3 -u tools/c1_latency.py > $O/c1_latency.log 2>&1
tail -3 $O/single_buffer.log; tail -4 $O/c1_latency.log
