# Round 4, second call: the new zlib.h golden sessions and the big-buffer
# tests touched this round, then the C3 line (no inflate leg: the 64 GiB
# shard leaves no room for it) and the LDS access probe.
set -e
T=${1:-r04b}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_bigbuf.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 400 python3 bench.py --level 1 --kind enwik --buffers 65536 --steps 3 --warmup 1 --no-inflate > $O/bench_C3_65536x1MiB_L1.json 2> $O/bench_C3.err
timeout -k 10 60 tools/lds_probe > $O/lds_probe.log 2>&1
cat $O/lds_probe.log
