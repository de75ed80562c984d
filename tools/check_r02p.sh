# k_encode with the wave-wide tree build (w_build): GPU suite, configs[0]-shaped
# latency and kernel stats against the one-lane build (ZGPU_ENCODE_VARIANT=1),
# and the batch encode stage of the default bench for both
set -e
mkdir -p gpurun_out/r02p
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02p/gpu_tests.log 2>&1
tail -2 gpurun_out/r02p/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 120 python3 tools/c1_latency.py > gpurun_out/r02p/c1_wave.log 2>&1
ZGPU_ENCODE_VARIANT=1 timeout -k 10 120 python3 tools/c1_latency.py > gpurun_out/r02p/c1_lane.log 2>&1
grep -h "GPU compress2" gpurun_out/r02p/c1_wave.log gpurun_out/r02p/c1_lane.log
for k in mix text; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02p/stats_wave_$k -o run -- python3 tools/c1_trace.py $k > /dev/null 2>&1
  ZGPU_ENCODE_VARIANT=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02p/stats_lane_$k -o run -- python3 tools/c1_trace.py $k > /dev/null 2>&1
done
grep -h k_encode gpurun_out/r02p/stats_*/run_kernel_stats.csv | cut -c1-90
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 > gpurun_out/r02p/bench_wave.json 2> gpurun_out/r02p/bench_wave.err
ZGPU_ENCODE_VARIANT=1 timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-inflate --adler-buffers 0 > gpurun_out/r02p/bench_lane.json 2> gpurun_out/r02p/bench_lane.err
for f in wave lane; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d.get('stage_ms_per_step'))" gpurun_out/r02p/bench_$f.json; done
