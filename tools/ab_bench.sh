# interleaved A/B of libzgpu builds through the pipelined default bench (C4 shard, no CPU or inflate legs):
#   bash tools/ab_bench.sh libA.so libB.so ...   (runs on the GPU box's scratch copy: swaps the product .so in place)
set -e
cp zlib.wasm_amd/libzgpu.so /tmp/libzgpu_orig.so
for k in 1 2; do
  for L in "$@"; do
    cp $L zlib.wasm_amd/libzgpu.so
    timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-inflate > /tmp/ab_bench.json
    python3 -c "import json,sys; d=json.load(open('/tmp/ab_bench.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $L
  done
done
cp /tmp/libzgpu_orig.so zlib.wasm_amd/libzgpu.so
