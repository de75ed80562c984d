"""One lone uncompress size, repeated (for a kernel / runtime trace): tools/lone_inflate_one.py <MiB> <calls>."""
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
import zgpu  # noqa: E402

mb, calls = int(sys.argv[1]), int(sys.argv[2])
assert zgpu.load().zgpu_init() == 0
data = bytes(datagen.make("mix", mb << 20, 3))
z = zlib.compress(data, 6)
for i in range(calls):
    t = time.perf_counter()
    rc, out, used = zgpu.uncompress2(z, len(data))
    dt = time.perf_counter() - t
    assert rc == 0 and out == data
    print(f"call {i}: {dt * 1e3:.2f} ms", flush=True)
