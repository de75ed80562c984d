# few-large-buffer parse/encode: GPU suite, single-buffer rates and the 64 KiB latency
set -e
O=gpurun_out/${1:-r03f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python3 -u tools/single_buffer.py > $O/single_buffer.log 2>&1
cat $O/single_buffer.log
timeout -k 10 200 python3 -u tools/c1_latency.py > $O/c1_latency.log 2>&1
cat $O/c1_latency.log
