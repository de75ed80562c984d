# round-3 baseline on a fresh box: GPU suite, smoke, default bench without CPU legs
set -e
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03a/gpu_tests.log 2>&1
tail -2 gpurun_out/r03a/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-inflate > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline'], d.get('stage_ms_per_step'))" gpurun_out/r03a/bench.json
