"""Lone uncompress2 time against stream size with the block-parallel decode
forced on (ZGPU_PAR_INFLATE_MIN=0) or off (ZGPU_NO_PAR_INFLATE=1): where the
parallel path starts to win (zgpu_api.cpp kParInflateMin).  Mix and text at L6."""
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
mode = "par" if os.environ.get("ZGPU_PAR_INFLATE_MIN") == "0" else "seq"
for kind in ("mix", "text"):
    for kb in (32, 64, 128, 256, 512):
        data = bytes(datagen.make(kind, kb << 10, 7))
        z = zlib.compress(data, 6)
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            rc, out, used = zgpu.uncompress2(z, len(data))
            ts.append(time.perf_counter() - t)
            assert rc == 0 and out == data
        print(f"{mode} {kind} {kb} KiB out, {len(z) >> 10} KiB in: {statistics.median(ts) * 1e3:.2f} ms", flush=True)
