"""How many buffers of a bench-shaped sub-batch the segmented lazy parse hands
to the sequential one, by cause (zgpu_debug_parse_fallbacks): one deflate of
B x 1 MiB Silesia-style buffers at L6 through the device batch API.
  tools/parse_fallbacks.py [buffers] [level] [kind]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
import torch  # noqa: E402
import zgpu  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
level = int(sys.argv[2]) if len(sys.argv) > 2 else 6
kind = sys.argv[3] if len(sys.argv) > 3 else "silesia"
KIND_ID = {"random": 0, "silesia": 1, "enwik": 2, "vocab": 3, "four": 4, "runs": 5}   # bench.py
n = 1 << 20
L = zgpu.load()
L.zgpu_debug_parse_fallbacks.argtypes = [C.POINTER(C.c_uint64)]
src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
zgpu.generate_dev(src, n, B, KIND_ID[kind], seed=2025, first_index=0)
cap = (zgpu.compress_bound(n) + 15) // 16 * 16
off = torch.arange(B, dtype=torch.int64, device="cuda") * n
ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
dst = torch.empty(cap * B, dtype=torch.uint8, device="cuda")
doff = torch.arange(B, dtype=torch.int64, device="cuda") * cap
dcap = torch.full((B,), cap, dtype=torch.int64, device="cuda")
dlen = torch.zeros(B, dtype=torch.int64, device="cuda")
st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
before = (C.c_uint64 * 2)()
assert L.zgpu_debug_parse_fallbacks(before) == 0
zgpu.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=level)
torch.cuda.synchronize()
after = (C.c_uint64 * 2)()
assert L.zgpu_debug_parse_fallbacks(after) == 0
assert int((st != 0).sum().item()) == 0
print(f"{B} x 1 MiB {kind} L{level}: fallbacks no-meet {after[0] - before[0]}, run-on overflow {after[1] - before[1]}",
      flush=True)
