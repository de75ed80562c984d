"""Few large buffers per sub-batch (a lone compress2, a handful of big buffers):
k_links / k_count per segment, the lazy parse spread over many workgroups
(k_pbig1..6) and the per-block encoder (k_enc_plan / scan / emit).  Every stream
must equal the oracle's (our C restatement of deflate.c / trees.c, pinned to the
reference's golden vectors) byte for byte; the 64 MiB case is checked against
system zlib (bit-identical to the reference on the bench sample, BASELINE.md
section 3.1), which is fast enough at that size."""
import time
import zlib as pyzlib

import numpy as np
import pytest

import datagen

pytestmark = pytest.mark.gpu

KINDS = ["mix", "text", "runs", "random"]


def _bufs(kind, n, seed):
    return datagen.make(kind, n, seed)


@pytest.mark.parametrize("n", [5000, 65536, 200017, (1 << 20) + 3])
@pytest.mark.parametrize("kind", KINDS)
def test_single_buffer_levels_wraps(zg, oracle, kind, n):
    data = _bufs(kind, n, n % 97)
    for i, level in enumerate((4, 5, 6, 8, 9)):
        wrap = (i + n) % 3
        [(st, z)] = zg.compress_batch([data], level=level, wrap=wrap)
        rc, want = oracle.compress(data, level, wrap)
        assert rc == 0 and st == 0, (kind, n, level, wrap, st)
        assert z == want, (kind, n, level, wrap, len(z), len(want))


def test_few_buffers_one_subbatch(zg, oracle):
    """Several large buffers of different sizes in one call: lane groups and
    block plans of consecutive buffers must not mix."""
    sizes = [70001, 1 << 20, 333333, 4096 * 5 + 1, 2 * (1 << 20) + 77]
    bufs = [_bufs(KINDS[i % len(KINDS)], n, 11 + i) for i, n in enumerate(sizes)]
    for level in (4, 6, 9):
        res = zg.compress_batch(bufs, level=level)
        for b, (st, z) in zip(bufs, res):
            assert st == 0
            assert z == oracle.compress(b, level)[1], (len(b), level)


def test_short_output_prefix(zg, oracle):
    """compress2 into a buffer too small: Z_BUF_ERROR and the stream's prefix
    (the block-parallel encoder clips every write at the capacity)."""
    data = _bufs("mix", 1 << 20, 3)
    want = oracle.compress(data, 6)[1]
    for cap in (len(want) - 1, len(want) // 2 + 3, 1000, 7):
        [(st, z)] = zg.compress_batch([data], level=6, caps=[cap])
        assert st == -5, cap
        assert z == want[:cap], cap


def test_unaligned_device_offsets(zg, oracle):
    """Outputs at odd device offsets next to each other: the shared words at
    block and buffer edges are or-ed in, nothing outside a stream is touched."""
    import torch
    sizes = [300001, 1 << 20, 65537]
    bufs = [_bufs(k, n, 5 + i) for i, (k, n) in enumerate(zip(("text", "mix", "runs"), sizes))]
    wants = [oracle.compress(b, 6)[1] for b in bufs]
    src = torch.tensor(np.frombuffer(b"".join(bufs), dtype=np.uint8), device="cuda")
    offs = np.cumsum([0] + sizes[:-1])
    caps = [zg.compress_bound(n) for n in sizes]
    doffs, pos = [], 3
    for c in caps:
        doffs.append(pos)
        pos += c + 5                                   # odd gaps between the streams
    dst = torch.full((pos + 16,), 0xA5, dtype=torch.uint8, device="cuda")
    t64 = lambda v: torch.tensor(v, dtype=torch.int64, device="cuda")
    dlen = t64([0] * 3)
    st = torch.zeros(3, dtype=torch.int32, device="cuda")
    zg.deflate_batch_dev(src, t64(list(offs)), t64(sizes), dst, t64(doffs), t64(caps), dlen, st, level=6)
    torch.cuda.synchronize()
    h = dst.cpu().numpy()
    dl = dlen.cpu().numpy()
    assert list(st.cpu().numpy()) == [0, 0, 0]
    for i in range(3):
        assert h[doffs[i]:doffs[i] + dl[i]].tobytes() == wants[i], i
        # the bytes between this stream's end and the next one's start keep the fill
        end = doffs[i + 1] if i + 1 < 3 else pos
        assert (h[doffs[i] + dl[i]:end] == 0xA5).all(), i
    assert (h[:3] == 0xA5).all()


def test_lone_64mib_l6_vs_system_zlib(zg):
    """The VERDICT r2 #5 case: one 64 MiB buffer at level 6 through compress2,
    equal to system zlib's stream; the rate is printed."""
    import torch
    n = 64 << 20
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    zg.generate_dev(src, n, 1, zg.KIND_SILESIA, seed=9)
    data = src.cpu().numpy().tobytes()
    want = pyzlib.compress(data, 6)
    zg.compress2(data[:1 << 20], 6)                     # warm the context
    t = time.perf_counter()
    rc, z = zg.compress2(data, 6)
    dt = time.perf_counter() - t
    print(f"lone 64 MiB L6 compress2: {n / dt / 1e6:.0f} MB/s (host buffers in and out)")
    assert rc == 0 and z == want


def _over_4gib_input(zg):
    """> 4 GiB: runs of 256..4095 equal bytes, with 8 MiB of generated mixed
    text across the 1 GiB and 2 GiB marks and across 2^32 - 1 (the end of the
    reference's first deflate() piece, compress.c:44-54)."""
    import torch
    rng = np.random.default_rng(17)
    n = (4 << 30) + (96 << 20) + 12345
    lens = rng.integers(256, 4096, n // 2048 + 16)
    lens = lens[: np.searchsorted(np.cumsum(lens), n) + 1]
    data = np.repeat(rng.integers(0, 256, len(lens), dtype=np.uint8), lens)[:n].copy()
    text = torch.empty(8 << 20, dtype=torch.uint8, device="cuda")
    for k, at in enumerate((1 << 30, 2 << 30, (1 << 32) - 1)):
        zg.generate_dev(text, 8 << 20, 1, zg.KIND_SILESIA, seed=30 + k)
        data[at - (4 << 20):at + (4 << 20)] = text.cpu().numpy()
    return data.tobytes()


@pytest.mark.parametrize("level", [6, 0])
def test_compress2_over_4gib_vs_system_zlib(zg, level):
    """compress2 of a buffer over 4 GiB equals system zlib's
    compress2 (called through ctypes, so compress.c's own calls: one 2^32 - 1
    byte Z_NO_FLUSH piece, then Z_FINISH with the rest, the output space in
    pieces of at most 2^32 - 1 bytes).  Level 0's stored blocks follow those
    pieces; Python's zlib.compress grows its output buffer step by
    step, which cuts level-0 blocks differently, so it is not the oracle here."""
    import ctypes
    import ctypes.util
    import hashlib
    data = _over_4gib_input(zg)
    print(f"\n{len(data)} bytes generated", flush=True)
    libz = ctypes.CDLL(ctypes.util.find_library("z") or "libz.so.1")
    libz.compress2.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulong), ctypes.c_char_p, ctypes.c_ulong,
                               ctypes.c_int]
    libz.compressBound.restype = ctypes.c_ulong
    libz.compressBound.argtypes = [ctypes.c_ulong]
    t = time.perf_counter()
    wbuf = ctypes.create_string_buffer(libz.compressBound(len(data)))
    wlen = ctypes.c_ulong(len(wbuf))
    assert libz.compress2(wbuf, ctypes.byref(wlen), data, len(data), level) == 0
    want = bytes(memoryview(wbuf)[:wlen.value])
    del wbuf
    print(f"system zlib L{level}: {len(want)} bytes in {time.perf_counter() - t:.1f} s", flush=True)
    t = time.perf_counter()
    rc, z = zg.compress2(data, level)
    print(f"libzgpu compress2: rc {rc}, {len(z)} bytes in {time.perf_counter() - t:.1f} s", flush=True)
    assert rc == 0
    assert len(z) == len(want) and hashlib.sha256(z).digest() == hashlib.sha256(want).digest()


@pytest.mark.parametrize("limit_mb", [None, "1"])
def test_mem_level_1_large_buffer_plan_fallback(zg, monkeypatch, limit_mb):
    """at memLevel 1 a block holds at most 126 symbols, so the
    block-parallel encoder's plans (~1 KiB per possible block) of a large
    buffer are big.  When they cannot be allocated (forced here with
    ZGPU_EPLAN_LIMIT_MB) the job encodes with k_encode instead of failing;
    both paths give system zlib's stream (deflateInit2(6, 8, 15, 1))."""
    import torch
    if limit_mb:
        monkeypatch.setenv("ZGPU_EPLAN_LIMIT_MB", limit_mb)
    n = 24 << 20
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    zg.generate_dev(src, n, 1, zg.KIND_SILESIA, seed=21)
    data = src.cpu().numpy().tobytes()
    co = pyzlib.compressobj(6, pyzlib.DEFLATED, 15, 1)
    want = co.compress(data) + co.flush()
    [(st, z)] = zg.compress_batch2([data], level=6, window_bits=15, mem_level=1)
    assert st == 0 and z == want
