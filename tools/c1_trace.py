# Kernel trace helper for the configs[0] shape: compress2 of one 64 KiB buffer
# of each kind, 20 times (run under rocprofv3 --kernel-trace --stats).
import sys

sys.path.insert(0, 'zlib.wasm_amd')
sys.path.insert(0, 'tests')
import datagen  # noqa: E402
import zgpu  # noqa: E402

assert zgpu.load().zgpu_init() == 0
kind = sys.argv[1] if len(sys.argv) > 1 else "runs"   # datagen kind: text, mix, runs, ...
data = bytes(datagen.make(kind, 64 * 1024, 7))
for _ in range(20):
    rc, z = zgpu.compress2(data, level=6)
    assert rc == 0
print(kind, len(z), flush=True)
