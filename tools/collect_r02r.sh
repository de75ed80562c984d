# round-2 final lines (after the wave-wide tree build): rocprofv3 kernel stats of the default bench, the C3-shaped
# L1 leg and the C5-shaped L9 leg
set -e
mkdir -p gpurun_out/r02r
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/r02r/bench_default.json 2> gpurun_out/r02r/bench_default.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02r/stats -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r02r/bench_under_rocprof.json 2> gpurun_out/r02r/bench_under_rocprof.err
timeout -k 10 300 python3 bench.py --level 1 --kind enwik --buffers 65536 --steps 2 --warmup 1 --no-inflate --adler-buffers 0 > gpurun_out/r02r/bench_C3.json 2> gpurun_out/r02r/bench_C3.err
timeout -k 10 300 python3 bench.py --level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 2 --warmup 1 --no-inflate > gpurun_out/r02r/bench_C5.json 2> gpurun_out/r02r/bench_C5.err
for f in bench_default bench_under_rocprof bench_C3 bench_C5; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])" gpurun_out/r02r/$f.json; done
grep -i 'k_match\|k_parse' gpurun_out/r02r/stats/run_kernel_stats.csv | cut -c1-160
