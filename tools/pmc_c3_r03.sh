# FETCH_SIZE / WRITE_SIZE passes (separate runs) of one 16384 x 1 MiB L1 launch (the C3 shape bench.py looks up)
set -e
O=gpurun_out/${1:-r03l}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --level 1 --kind enwik --buffers 16384 --no-cpu --no-inflate --verify 1 --adler-buffers 0 > $O/f.json 2> $O/f.err
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --level 1 --kind enwik --buffers 16384 --no-cpu --no-inflate --verify 1 --adler-buffers 0 > $O/w.json 2> $O/w.err
find $O -name "*counter_collection.csv"
