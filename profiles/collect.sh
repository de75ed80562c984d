# rocprofv3 collection recipe for profiles/: kernel stats of the default bench,
# then FETCH_SIZE and WRITE_SIZE in separate passes on one 4 GiB sub-batch.
set -e
mkdir -p gpurun_out/p
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p/stats -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 6 > gpurun_out/p/bench_stats.json 2> gpurun_out/p/bench_stats.err
timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/p/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --verify 1 > gpurun_out/p/f.json 2> gpurun_out/p/f.err
timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/p/write -o run -- python3 bench.py --steps 1 --warmup 0 --buffers 4096 --no-cpu --verify 1 > gpurun_out/p/w.json 2> gpurun_out/p/w.err
find gpurun_out/p -name "*.csv" | head -20
