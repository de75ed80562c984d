# round-3 measurement lines: default bench (C4 shard, CPU baselines), rocprofv3 kernel statistics of it, the C5
# shape (256 x 16 MiB L9: few large buffers -> k_pbig* / k_enc_*) with its kernel statistics, the C3 shard (L1),
# single-buffer rates and the 64 KiB latency
set -e
T=${1:-r03j}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['value'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
timeout -k 10 400 python3 -u bench.py --kind vocab --level 9 --buffer-bytes 16777216 --buffers 256 --steps 2 --warmup 1 > $O/bench_C5.json 2> $O/bench_C5.err
python3 -c "import json; d=json.load(open('$O/bench_C5.json')); print('C5', d['value'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5 -o run -- python3 bench.py --kind vocab --level 9 --buffer-bytes 16777216 --buffers 256 --steps 1 --warmup 1 --no-cpu --no-inflate > $O/bench_C5_under_rocprof.json 2> $O/bench_C5_under_rocprof.err
timeout -k 10 500 python3 -u bench.py --kind enwik --level 1 --buffers 65536 --steps 2 --warmup 1 > $O/bench_C3.json 2> $O/bench_C3.err
python3 -c "import json; d=json.load(open('$O/bench_C3.json')); print('C3', d['value'], d['cpu_baseline']['value'])"
timeout -k 10 200 python3 -u tools/single_buffer.py > $O/single_buffer.log 2>&1
timeout -k 10 200 python3 -u tools/c1_latency.py > $O/c1_latency.log 2>&1
tail -3 $O/single_buffer.log; tail -4 $O/c1_latency.log
