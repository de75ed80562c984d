"""A/B timing of one sub-batch on a given libzgpu build:
    python3 tools/ab_match.py path/to/libzgpu.so [launches] [level] [kind] [buffers]
(default: 3 launches of 4096 x 1 MiB Silesia-style at L6, the bench's launch shape; the C3 shape is
`... 2 1 enwik 16384`).  Prints the stage times per launch (library events) and checks the streams of
8 buffers against system zlib."""
import sys
import time
import zlib

sys.path.insert(0, "zlib.wasm_amd")
import torch  # noqa: E402  (before zgpu: torch bundles libamdhip64)
import zgpu  # noqa: E402

lib = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
level = int(sys.argv[3]) if len(sys.argv) > 3 else 6
kind = {"silesia": zgpu.KIND_SILESIA, "enwik": zgpu.KIND_ENWIK,
        "vocab": zgpu.KIND_SMALLVOCAB}[sys.argv[4] if len(sys.argv) > 4 else "silesia"]
zgpu.load(lib)
n, B = int(sys.argv[6]) if len(sys.argv) > 6 else 1 << 20, int(sys.argv[5]) if len(sys.argv) > 5 else 4096
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
zgpu.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=level)
torch.cuda.synchronize()
zgpu.stage_timing(True)
t = time.perf_counter()
for _ in range(reps):
    zgpu.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=level)
torch.cuda.synchronize()
el = (time.perf_counter() - t) / reps
stg = zgpu.stage_timing_read()
zgpu.stage_timing(False)
h_dst, dl = dst.cpu(), dlen.cpu()
ok = all(h_dst[i * cap:i * cap + int(dl[i])].numpy().tobytes() ==
         zlib.compress(src[i * n:(i + 1) * n].cpu().numpy().tobytes(), level) for i in range(0, B, B // 8))
key = "match" if level >= 4 else "parse_greedy"
import os  # noqa: E402
print(f"{lib} LZP={os.environ.get('ZGPU_LZP', '0')}: {key} {stg[key][0] / stg[key][1]:.1f} ms/launch, step {el * 1e3:.1f} ms, exact {ok}",
      flush=True)
print("  stages ms per launch:", {k: round(v[0] / max(v[1], 1) * (v[1] / reps), 2) for k, v in stg.items() if v[1]},
      flush=True)
