"""Flush statistics of k_match on one 4096 x 1 MiB L6 sub-batch (the bench's launch shape), from a statistics
build of libzgpu (-DZGPU_MATCH_STATS; never the product library): python3 tools/match_stats.py lib.so"""
import ctypes as C
import sys

sys.path.insert(0, "zlib.wasm_amd")
import torch  # noqa: E402
import zgpu  # noqa: E402

lib = sys.argv[1]
L = zgpu.load(lib)
n, B = 1 << 20, 4096
src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
zgpu.generate_dev(src, n, B, zgpu.KIND_SILESIA, seed=2025)
cap = (zgpu.compress_bound(n) + 15) // 16 * 16
off = torch.arange(B, dtype=torch.int64, device="cuda") * n
ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
dst = torch.empty(cap * B, dtype=torch.uint8, device="cuda")
doff = torch.arange(B, dtype=torch.int64, device="cuda") * cap
dcap = torch.full((B,), cap, dtype=torch.int64, device="cuda")
dlen = torch.zeros(B, dtype=torch.int64, device="cuda")
st = torch.zeros(B, dtype=torch.int32, device="cuda")
zgpu.set_inflight_bytes(4 << 30)
buf = (C.c_ulonglong * 8)()
L.zgpu_match_stats_read(buf, 1)
zgpu.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=6)
torch.cuda.synchronize()
L.zgpu_match_stats_read(buf, 1)
v = list(buf)
names = ["wave_flushes", "wave_flush_rounds", "entries", "lane_flushes", "wave_walk_groups", "long_compares",
         "lane_walks", "unused"]
print({k: x for k, x in zip(names, v)})
print("rounds/flush %.2f  entries/round %.2f  entries/lane-flush %.2f  lanes/flush %.1f  flushes/walk-group %.2f"
      % (v[1] / v[0], v[2] / v[1], v[2] / v[3], v[3] / v[0], v[0] / v[4]))
