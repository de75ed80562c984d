"""A lone large uncompress (one zlib stream per call, the reference's
production shape) through libzgpu.so's uncompress2: 1, 16 and 64 MiB of the
generator's mix at L6, median of 3 calls, against system zlib on one host
thread; every output is checked."""
import os
import statistics
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
import zgpu  # noqa: E402

assert zgpu.load().zgpu_init() == 0
for mb in (1, 16, 64):
    data = bytes(datagen.make("mix", mb << 20, 3))
    z = zlib.compress(data, 6)
    ts, tz = [], []
    for _ in range(3):
        t = time.perf_counter()
        rc, out, used = zgpu.uncompress2(z, len(data))
        ts.append(time.perf_counter() - t)
        assert rc == 0 and out == data
        t = time.perf_counter()
        zlib.decompress(z)
        tz.append(time.perf_counter() - t)
    g, c = statistics.median(ts), statistics.median(tz)
    print(f"lone uncompress {mb} MiB (ratio {len(data) / len(z):.2f}): GPU {g * 1e3:.1f} ms "
          f"({len(data) / g / 1e6:.0f} MB/s), system zlib 1 thread {c * 1e3:.1f} ms ({len(data) / c / 1e6:.0f} MB/s)",
          flush=True)
