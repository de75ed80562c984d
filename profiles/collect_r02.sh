# rocprofv3 collection for the round-2 profiles: kernel stats of the default
# bench (the line bench.py prints next to them), then FETCH_SIZE and WRITE_SIZE
# in separate passes on one 4 GiB L6 sub-batch + the C2 CRC-32 and C5-shaped
# Adler-32 legs (file names carry the launch shapes bench.py looks up).
set -e
T=${1:-r02g}
mkdir -p gpurun_out/p
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p/stats -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/p/bench_stats.json 2> gpurun_out/p/bench_stats.err
timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/p/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --verify 1 > gpurun_out/p/f.json 2> gpurun_out/p/f.err
timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/p/write -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --no-inflate --verify 1 > gpurun_out/p/w.json 2> gpurun_out/p/w.err
find gpurun_out/p -name "*.csv"
