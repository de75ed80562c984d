"""Wall time of the streaming deflate() against compress2 on the same bytes
(one GPU): one call with all the input, zpipe.c-style 64 KiB chunks with a
16 KiB output buffer, and compress2.  Usage: python tools/stream_speed.py [MiB]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
import zgpu  # noqa: E402
from zhelpers import run_dsession  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    data = datagen.make("mix", mib << 20, 5)
    L = zgpu.load()
    for level in (1, 6, 9):
        zgpu.compress2(data[:65536], level)                        # warm up
        t = time.perf_counter()
        rc, z = zgpu.compress2(data, level)
        t_c2 = time.perf_counter() - t
        t = time.perf_counter()
        recs, whole = run_dsession(L, data, [(len(data), 0, 1 << 20, True), (0, 4, 1 << 20, True)], level)
        t_one = time.perf_counter() - t
        plan = [(65536, 0, 16384, True) for _ in range(0, len(data), 65536)] + [(0, 4, 16384, True)]
        t = time.perf_counter()
        recs2, whole2 = run_dsession(L, data, plan, level, max_calls=10 ** 6)
        t_pipe = time.perf_counter() - t
        ok = whole == z and whole2 == z
        print(f"L{level} {mib} MiB: compress2 {t_c2 * 1e3:.0f} ms, deflate() one call {t_one * 1e3:.0f} ms, "
              f"zpipe 64K/16K {t_pipe * 1e3:.0f} ms ({len(recs2)} calls), same stream: {ok}", flush=True)


if __name__ == "__main__":
    main()
