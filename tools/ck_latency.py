"""Latency of single crc32() / adler32() calls through libzgpu.so (the zlib.h
entry points, host buffers) at 16 B, 4 KiB, 64 KiB and 1 MiB, against system
zlib on one host thread; every GPU value is checked against system zlib.
Usage: python tools/ck_latency.py [calls]"""
import ctypes as C
import os
import statistics
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
import zgpu  # noqa: E402


def median_us(fn, calls):
    ts = []
    for _ in range(calls):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts) * 1e6


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    L = zgpu.load()
    for f in ("crc32_z", "adler32_z"):
        getattr(L, f).restype = C.c_ulong
        getattr(L, f).argtypes = [C.c_ulong, C.c_void_p, C.c_size_t]
    L.crc32_z(0, b"warm", 4)
    print(f"{'size':>8} {'call':>8} {'GPU us':>9} {'zlib us':>9}  check", flush=True)
    for n in (16, 4096, 65536, 1 << 20):
        data = os.urandom(n)
        buf = C.create_string_buffer(data, n)
        for name, ref in (("crc32", zlib.crc32), ("adler32", zlib.adler32)):
            fn = getattr(L, name + "_z")
            init = 0 if name == "crc32" else 1
            ok = fn(init, buf, n) == ref(data)
            g = median_us(lambda: fn(init, buf, n), calls)
            z = median_us(lambda: ref(data), calls)
            print(f"{n:>8} {name:>8} {g:>9.1f} {z:>9.1f}  {'ok' if ok else 'MISMATCH'}", flush=True)


if __name__ == "__main__":
    main()
