"""A/B timing of the batched CRC-32 on a given libzgpu build (the C2 shape by default):
    python3 tools/ab_crc.py path/to/libzgpu.so [buffers] [bytes] [reps]
Times zgpu_crc32_batch_dev with HIP events over `reps` launches on device-generated
Silesia-style buffers and checks 64 of the CRCs against zlib.crc32."""
import sys
import zlib

sys.path.insert(0, "zlib.wasm_amd")
import torch  # noqa: E402  (before zgpu: torch bundles libamdhip64)
import zgpu  # noqa: E402

lib = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
zgpu.load(lib)
src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
zgpu.generate_dev(src, n, B, zgpu.KIND_SILESIA, seed=7)
off = torch.arange(B, dtype=torch.int64, device="cuda") * n
ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
out = torch.zeros(B, dtype=torch.int32, device="cuda")
zgpu.crc32_batch_dev(src, off, ln, out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    zgpu.crc32_batch_dev(src, off, ln, out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
host = src[: 64 * n].cpu().numpy().tobytes()
got = out[:64].cpu().numpy().astype("uint32")
ok = all(int(got[i]) == zlib.crc32(host[i * n:(i + 1) * n]) for i in range(64))
print(f"{lib}: {B} x {n} B crc32 {ms:.3f} ms/launch, {B * (n + 4) / ms / 1e6:.1f} GB/s (alg), exact {ok}", flush=True)
