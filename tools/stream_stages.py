"""Where a large streaming deflate() job spends its time (one GPU): one
deflate(Z_NO_FLUSH) call with N MiB of input, then Z_FINISH, at levels 1/6/9,
with the library's per-stage HIP-event timing (zgpu_stage_timing) around it.
Usage: python tools/stream_stages.py [MiB] [levels, e.g. 1,6,9]"""
import faulthandler
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
import zgpu  # noqa: E402
from zhelpers import run_dsession  # noqa: E402

def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    data = datagen.make("mix", mib << 20, 5)
    faulthandler.enable()
    cap = len(data) + (len(data) >> 8) + (1 << 16)
    L = zgpu.load()
    levels = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 6, 9]
    for level in levels:
        print(f"L{level} {mib} MiB ...", flush=True)
        zgpu.compress2(data[:65536], level)
        zgpu.stage_timing(True)
        zgpu.stage_timing_read()
        t = time.perf_counter()
        recs, whole = run_dsession(L, data, [(len(data), 0, cap, True), (0, 4, cap, True)], level)
        dt = time.perf_counter() - t
        tm = zgpu.stage_timing_read()
        zgpu.stage_timing(False)
        st = ", ".join(f"{name} {m:.0f} ms ({k})" for name, (m, k) in tm.items() if k)
        c = zlib.compressobj(level)                 # the same two calls on the system zlib
        ok = whole == c.compress(data) + c.flush()
        print(f"L{level} {mib} MiB streaming job: {dt * 1e3:.0f} ms wall ({mib * 1.048576 / dt:.0f} MB/s); {st};"
              f" {'identical to' if ok else 'DIFFERS from'} the system zlib", flush=True)


if __name__ == "__main__":
    main()
