# round-3 lines: GPU suite (skipped with NO_SUITE=1), default bench (CPU baselines included), rocprofv3 kernel stats of the
# default bench, FETCH_SIZE / WRITE_SIZE passes (separate) of one 4 GiB L6 sub-batch + the C2 and
# A5 checksum legs (file names carry the launch shapes bench.py looks up)
set -e
T=${1:-r03b}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NO_SUITE" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -1 $O/gpu_tests.log
fi
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --verify 1 > $O/f.json 2> $O/f.err
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --verify 1 > $O/w.json 2> $O/w.err
for f in bench_default bench_under_rocprof; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['avg_launch_ms'], d['cpu_baseline'] and d['cpu_baseline']['value'])" $O/$f.json; done
grep -h "k_match\|k_links\|k_parse_seg\|k_encode" $O/stats/run_kernel_stats.csv | cut -c1-150
