# Lone-buffer L1-3 compression through the batch API and compress2 (the
# k_parse_fast LDS variant; ZGPU_FAST_LDS_MAX=0 runs the HBM variant), checked
# against system zlib.
import sys
import time
import zlib as pyzlib

sys.path.insert(0, 'zlib.wasm_amd')
sys.path.insert(0, 'tests')
import datagen  # noqa: E402
import zgpu  # noqa: E402

assert zgpu.load().zgpu_init() == 0
for kind in ("text", "mix"):
    for size in (64 << 10, 1 << 20, 16 << 20):
        data = bytes(datagen.make(kind, size, 5))
        for level in (1, 3):
            want = pyzlib.compress(data, level)
            t = time.perf_counter()
            for _ in range(3):
                pyzlib.compress(data, level)
            cpu = (time.perf_counter() - t) / 3
            (st, z), = zgpu.compress_batch([data], level=level)
            assert st == 0 and z == want, (kind, size, level)
            reps = 5 if size <= (1 << 20) else 2
            t = time.perf_counter()
            for _ in range(reps):
                zgpu.compress_batch([data], level=level)
            el = (time.perf_counter() - t) / reps
            print(f"{kind} {size >> 10} KiB L{level}: {el * 1e3:.2f} ms {size / el / 1e6:.1f} MB/s "
                  f"(one host thread {cpu * 1e3:.2f} ms)", flush=True)
