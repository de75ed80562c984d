"""crc32_z / adler32_z calls of 64 KiB and 1 MiB, 50 each, for rocprofv3's
kernel trace (which kernels a single checksum call runs, and for how long)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
import zgpu  # noqa: E402

L = zgpu.load()
for f in ("crc32_z", "adler32_z"):
    getattr(L, f).restype = C.c_ulong
    getattr(L, f).argtypes = [C.c_ulong, C.c_void_p, C.c_size_t]
for n in (65536, 1 << 20):
    buf = C.create_string_buffer(os.urandom(n), n)
    for _ in range(50):
        L.crc32_z(0, buf, n)
        L.adler32_z(1, buf, n)
print("done")
