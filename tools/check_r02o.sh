# fresh-build check of the current tree: GPU suite, smoke, default bench line
set -e
mkdir -p gpurun_out/r02o
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02o/gpu_tests.log 2>&1
tail -3 gpurun_out/r02o/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 python3 bench.py > gpurun_out/r02o/bench_default.json 2> gpurun_out/r02o/bench_default.err
cat gpurun_out/r02o/bench_default.json | cut -c1-400
