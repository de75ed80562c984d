"""Lone-buffer L1-3 speed and exactness (batch API, count = 1) against the
system zlib: python3 tools/lone_fast.py [levels] [MiB sizes] [kinds]
The library reads ZGPU_FAST_SRT once: run it twice to compare the parses."""
import os
import sys
import time
import zlib

sys.path.insert(0, 'zlib.wasm_amd')
sys.path.insert(0, 'tests')
import datagen  # noqa: E402
import zgpu  # noqa: E402

levels = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3").split(",")]
sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,16").split(",")]
kinds = (sys.argv[3] if len(sys.argv) > 3 else "text,mix").split(",")
zgpu.load()
assert zgpu.load().zgpu_init() == 0
tag = "srt" if os.environ.get("ZGPU_FAST_SRT") == "1" else "fast"
for kind in kinds:
    for mb in sizes:
        data = bytes(datagen.make(kind, mb << 20, 3))
        for level in levels:
            zgpu.compress_batch([data[:65536]], level=level)
            zgpu.stage_timing(True)
            zgpu.stage_timing_read()
            t = time.perf_counter()
            (st, z), = zgpu.compress_batch([data], level=level)
            el = time.perf_counter() - t
            stg = zgpu.stage_timing_read()
            zgpu.stage_timing(False)
            ok = st == 0 and z == zlib.compress(data, level)
            st_s = ", ".join(f"{k} {v[0]:.1f}" for k, v in stg.items() if v[1])
            print(f"[{tag}] {kind} {mb} MiB L{level}: {el * 1e3:.1f} ms {len(data) / el / 1e6:.1f} MB/s "
                  f"{'identical' if ok else 'DIFFERS'} ({st_s})", flush=True)
