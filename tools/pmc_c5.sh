# FETCH_SIZE and WRITE_SIZE (separate passes) of the C5-shaped L9 leg's launch:
# 256 x 16 MiB small-vocabulary buffers (the shape bench.py looks up as L9_256x16777216)
set -e
mkdir -p gpurun_out/pmc5
export TMPDIR=/tmp
ARGS="--level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 1 --warmup 0 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc5/fetch -o run -- python3 bench.py $ARGS > gpurun_out/pmc5/f.json 2> gpurun_out/pmc5/f.err
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc5/write -o run -- python3 bench.py $ARGS > gpurun_out/pmc5/w.json 2> gpurun_out/pmc5/w.err
find gpurun_out/pmc5 -name "*.csv"
