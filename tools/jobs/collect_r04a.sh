# Round 4, first call: PMC FETCH/WRITE passes of the shipped kernels at the C5
# (256 x 16 MiB, L9) and C3 (16384 x 1 MiB launches, L1) shapes, copied into
# profiles/ so that the bench lines run after them read them; then the C3 and
# C5 bench lines; then the LDS access probe (tools/lds_probe.hip).
set -e
T=${1:-r04a}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
A5="--level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 1 --warmup 0 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
A3="--steps 1 --warmup 0 --level 1 --kind enwik --buffers 16384 --no-cpu --no-inflate --verify 1 --adler-buffers 0 --crc-buffers 4096"
pick() { find "$1" -name "*counter_collection.csv" | head -1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5f -o run -- python3 bench.py $A5 > $O/c5f.json 2> $O/c5f.err
cp "$(pick $O/c5f)" profiles/${T}_pmc_fetch_L9_256x16777216.csv
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5w -o run -- python3 bench.py $A5 > $O/c5w.json 2> $O/c5w.err
cp "$(pick $O/c5w)" profiles/${T}_pmc_write_L9_256x16777216.csv
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3f -o run -- python3 bench.py $A3 > $O/c3f.json 2> $O/c3f.err
cp "$(pick $O/c3f)" profiles/${T}_pmc_fetch_L1_16384x1048576.csv
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3w -o run -- python3 bench.py $A3 > $O/c3w.json 2> $O/c3w.err
cp "$(pick $O/c3w)" profiles/${T}_pmc_write_L1_16384x1048576.csv
cp profiles/${T}_pmc_* $O/
timeout -k 10 400 python3 bench.py --level 9 --kind vocab --buffer-bytes 16777216 --buffers 256 --steps 3 --warmup 1 > $O/bench_C5_256x16MiB_L9.json 2> $O/bench_C5.err
timeout -k 10 400 python3 bench.py --level 1 --kind enwik --buffers 65536 --steps 3 --warmup 1 > $O/bench_C3_65536x1MiB_L1.json 2> $O/bench_C3.err
timeout -k 10 60 tools/lds_probe > $O/lds_probe.log 2>&1
cat $O/lds_probe.log
