# configs[0] shape on the GPU: one 64 KB text buffer through compress2 (host
# buffers in and out, so PCIe and launch latency included), level 6.  Reports
# the median wall time per call and checks the stream against Python's zlib
# (byte-identical to the reference on every survey probe).
import statistics
import sys
import time
import zlib

sys.path.insert(0, 'zlib.wasm_amd')
sys.path.insert(0, 'tests')
import datagen  # noqa: E402
import zgpu  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else None
assert (zgpu.load(lib) if lib else zgpu.load()).zgpu_init() == 0
print("library:", lib or "zlib.wasm_amd/libzgpu.so", flush=True)
for kind in ("text", "mix"):
    data = bytes(datagen.make(kind, 64 * 1024, 7))
    st, z = zgpu.compress2(data, level=6)
    assert st == 0 and z == zlib.compress(data, 6), "stream differs from zlib"
    ts = []
    for _ in range(200):
        t = time.perf_counter()
        zgpu.compress2(data, level=6)
        ts.append(time.perf_counter() - t)
    med = statistics.median(ts)
    t = time.perf_counter()
    for _ in range(200):
        zlib.compress(data, 6)
    cpu = (time.perf_counter() - t) / 200
    print(f"C1 64 KiB {kind} L6: GPU compress2 median {med * 1e3:.3f} ms ({len(data) / med / 1e6:.1f} MB/s), "
          f"host zlib 1 thread {cpu * 1e3:.3f} ms ({len(data) / cpu / 1e6:.1f} MB/s), ratio {len(data) / len(z):.2f}",
          flush=True)

for kind in ("text", "mix"):
    data = bytes(datagen.make(kind, 64 * 1024, 7))
    zgpu.stage_timing(True)
    zgpu.compress2(data, level=6)
    print(f"stages C1 64 KiB {kind} L6 (ms):", zgpu.stage_timing_read(), flush=True)
    zgpu.stage_timing(False)
