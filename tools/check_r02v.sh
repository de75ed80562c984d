# hle as one OR + compare: GPU suite; lone 64 KiB compress2 (auto = wave build) vs lane build;
# default bench (auto = lane build) vs wave build; C5 shape (auto = wave) vs lane
set -e
mkdir -p gpurun_out/r02v
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02v/gpu_tests.log 2>&1
tail -2 gpurun_out/r02v/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 120 python3 tools/c1_latency.py > gpurun_out/r02v/c1_wave.log 2>&1
ZGPU_ENCODE_VARIANT=1 timeout -k 10 120 python3 tools/c1_latency.py > gpurun_out/r02v/c1_lane.log 2>&1
grep -h "GPU compress2" gpurun_out/r02v/c1_wave.log gpurun_out/r02v/c1_lane.log
for k in mix text; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02v/stats_wave_$k -o run -- python3 tools/c1_trace.py $k > /dev/null 2>&1
  ZGPU_ENCODE_VARIANT=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02v/stats_lane_$k -o run -- python3 tools/c1_trace.py $k > /dev/null 2>&1
done
grep -h k_encode gpurun_out/r02v/stats_*/run_kernel_stats.csv | cut -c1-90
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 > gpurun_out/r02v/bench_wave.json 2> gpurun_out/r02v/bench_wave.err
ZGPU_ENCODE_VARIANT=2 timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 > gpurun_out/r02v/bench_lane.json 2> gpurun_out/r02v/bench_lane.err
for f in wave lane; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d.get('stage_ms_per_step'))" gpurun_out/r02v/bench_$f.json; done
timeout -k 10 300 python3 bench.py --level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 2 --warmup 1 --no-inflate --no-cpu --adler-buffers 0 > gpurun_out/r02v/bench_C5_wave.json 2> gpurun_out/r02v/bench_C5_wave.err
ZGPU_ENCODE_VARIANT=1 timeout -k 10 300 python3 bench.py --level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 2 --warmup 1 --no-inflate --no-cpu --adler-buffers 0 > gpurun_out/r02v/bench_C5_lane.json 2> gpurun_out/r02v/bench_C5_lane.err
for f in C5_wave C5_lane; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d.get('stage_ms_per_step'))" gpurun_out/r02v/bench_$f.json; done
