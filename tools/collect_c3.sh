# C3-shaped level-1 leg: rocprofv3 kernel stats of the full per-GPU shard
# (65536 x 1 MiB enwik-style), then FETCH_SIZE / WRITE_SIZE passes of one
# 16384 x 1 MiB launch (file names carry the launch shape bench.py looks up).
set -e
T=${1:-r02l}
mkdir -p gpurun_out/c3
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3/stats -o run -- python3 bench.py --level 1 --kind enwik --buffers 65536 --steps 2 --warmup 1 --no-inflate --adler-buffers 0 > gpurun_out/c3/bench_stats.json 2> gpurun_out/c3/bench_stats.err
timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c3/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --level 1 --kind enwik --buffers 16384 --no-cpu --no-inflate --verify 1 --adler-buffers 0 > gpurun_out/c3/f.json 2> gpurun_out/c3/f.err
timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c3/write -o run -- python3 bench.py --steps 1 --warmup 0 --level 1 --kind enwik --buffers 16384 --no-cpu --no-inflate --verify 1 --adler-buffers 0 > gpurun_out/c3/w.json 2> gpurun_out/c3/w.err
find gpurun_out/c3 -name "*.csv"
cat gpurun_out/c3/bench_stats.json
