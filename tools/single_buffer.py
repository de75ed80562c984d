# Single-buffer compression speed through the batch API (count = 1), L6 and L1.
import sys
import time

sys.path.insert(0, 'zlib.wasm_amd')
sys.path.insert(0, 'tests')
import datagen  # noqa: E402
import zgpu  # noqa: E402

zgpu.load()
assert zgpu.load().zgpu_init() == 0
for mb in (1, 16, 64):
    data = bytes(datagen.make("mix", mb << 20, 3))
    for level in (6, 9, 1):
        if level == 1 and mb > 16:
            continue
        zgpu.compress_batch([data], level=level)
        t = time.time()
        (st, z), = zgpu.compress_batch([data], level=level)
        el = time.time() - t
        print(f"single {mb} MiB L{level}: {el * 1e3:.1f} ms  {len(data) / el / 1e6:.1f} MB/s "
              f"ratio {len(data) / len(z):.2f}", flush=True)

# stage breakdown of one 64 MiB L6 buffer
data = bytes(datagen.make("mix", 64 << 20, 3))
zgpu.stage_timing(True)
zgpu.compress_batch([data], level=6)
print("stages 64 MiB L6:", zgpu.stage_timing_read(), flush=True)
zgpu.stage_timing(False)
