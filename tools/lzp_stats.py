"""Statistics of k_lzp on one 4096 x 1 MiB sub-batch (the bench's launch shape) from the statistics build
(make -C zlib.wasm_amd stats -> libzgpu_lzpstats.so, -DZGPU_LZP_STATS; never the product library):
    python3 tools/lzp_stats.py [lib] [level] [kind] [buffers]
Prints walks and steps per position, rounds per tile, full-walk requests, and where the parser wave's
clock goes."""
import ctypes as C
import os
import sys

os.environ.setdefault("ZGPU_LZP", "1")                 # the statistics build carries k_lzp

sys.path.insert(0, "zlib.wasm_amd")
import torch  # noqa: E402
import zgpu  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else "zlib.wasm_amd/libzgpu_lzpstats.so"
level = int(sys.argv[2]) if len(sys.argv) > 2 else 6
kind = {"silesia": zgpu.KIND_SILESIA, "enwik": zgpu.KIND_ENWIK, "vocab": zgpu.KIND_SMALLVOCAB}[
    sys.argv[3] if len(sys.argv) > 3 else "silesia"]
B = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
L = zgpu.load(lib)
n = 1 << 20
src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
zgpu.generate_dev(src, n, B, kind, seed=2025)
cap = (zgpu.compress_bound(n) + 15) // 16 * 16
off = torch.arange(B, dtype=torch.int64, device="cuda") * n
ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
dst = torch.empty(cap * B, dtype=torch.uint8, device="cuda")
doff = torch.arange(B, dtype=torch.int64, device="cuda") * cap
dcap = torch.full((B,), cap, dtype=torch.int64, device="cuda")
dlen = torch.zeros(B, dtype=torch.int64, device="cuda")
st = torch.zeros(B, dtype=torch.int32, device="cuda")
zgpu.set_inflight_bytes(n * B)
buf = (C.c_ulonglong * 32)()
zgpu.stage_timing(True)
L.zgpu_lzp_stats_read(buf, 1)
zgpu.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=level)
torch.cuda.synchronize()
L.zgpu_lzp_stats_read(buf, 1)
stg = zgpu.stage_timing_read()
v = list(buf)
N = n * B
tiles = max(v[0], 1)
print(f"level {level}, {B} x 1 MiB: match stage {stg['match'][0]:.1f} ms")
print(f"  quarter walks {v[3]} ({v[3] / N:.3f}/pos), steps {v[4] / N:.2f}/pos;"
      f" full walks {v[5]} ({v[5] / N:.4f}/pos), steps {v[6] / N:.2f}/pos; requests {v[2]} (dropped {v[7]})")
print(f"  tiles {v[0]}, rounds/tile {v[1] / tiles:.2f}, hist (1..7, 8+): {v[8:16]}")
tot = max(v[20], 1)
print(f"  parser clock/tile {v[20] / tiles:.0f}: passes 1-2 {100 * v[16] / tot:.1f}%, stitch+replay "
      f"{100 * v[17] / tot:.1f}%, waiting for full walks {100 * v[18] / tot:.1f}%, symbols {100 * v[19] / tot:.1f}%")
print(f"  step clock (wave 0) {v[21] / tiles:.0f}/tile; idle polls {v[22]}; speculative full walks {v[23]} "
      f"({v[23] / N:.4f}/pos)")
