"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the
golden fixtures generated from the compiled reference.  Bit-exact everywhere:
deflate streams byte for byte, CRC-32 / Adler-32 values exactly."""
import ctypes as C
import hashlib
import os
import zlib as pyzlib

import numpy as np
import pytest

import datagen

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ----------------------------- checksums -----------------------------

def test_crc_adler_golden(zg, golden):
    bufs = [datagen.make(c["kind"], c["n"], c["seed"]) for c in golden["cases"]]
    crcs = zg.crc32_batch(bufs)
    adls = zg.adler32_batch(bufs)
    for c, cr, ad in zip(golden["cases"], crcs, adls):
        assert cr == c["crc32"], (c["kind"], c["n"])
        assert ad == c["adler32"], (c["kind"], c["n"])
    assert zg.crc32(b"123456789") == 0xCBF43926
    assert zg.adler32(b"123456789") == 0x091E01DE


def test_crc_adler_ragged_with_init(zg, oracle):
    rng = np.random.default_rng(5)
    lens = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 63, 64, 65, 1023, 1024, 1025, 4095, 4096, 4097]
    lens += [int(x) for x in rng.integers(0, 70000, 60)] + [1 << 20, (1 << 20) + 3, 3 * (1 << 20) + 5]
    bufs = [datagen.random_bytes(n, i) for i, n in enumerate(lens)]
    inits = [int(x) for x in rng.integers(0, 1 << 32, len(bufs), dtype=np.uint64)]
    ainit = [int(a) % 65521 | ((int(b) % 65521) << 16) for a, b in
             zip(rng.integers(0, 65521, len(bufs)), rng.integers(0, 65521, len(bufs)))]
    got_c = zg.crc32_batch(bufs, inits)
    got_a = zg.adler32_batch(bufs, ainit)
    for b, ic, ia, gc, ga in zip(bufs, inits, ainit, got_c, got_a):
        assert gc == oracle.crc32(b, ic), len(b)
        assert ga == oracle.adler32(b, ia), len(b)


def test_checksum_device_api_unaligned(zg, oracle):
    import torch
    rng = np.random.default_rng(7)
    lens = [int(x) for x in rng.integers(0, 9000, 500)]
    offs, pos = [], 3
    for n in lens:
        offs.append(pos)
        pos += n + int(rng.integers(0, 5))          # arbitrary alignment
    host = np.frombuffer(datagen.random_bytes(pos + 16, 1), dtype=np.uint8)
    src = torch.from_numpy(host.copy()).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor(lens, dtype=torch.int64).cuda()
    out = torch.zeros(len(lens), dtype=torch.int32).cuda()
    zg.crc32_batch_dev(src, off, ln, out)
    outa = torch.zeros(len(lens), dtype=torch.int32).cuda()
    zg.adler32_batch_dev(src, off, ln, outa)
    torch.cuda.synchronize()
    oc = out.cpu().numpy().view(np.uint32)
    oa = outa.cpu().numpy().view(np.uint32)
    for i, (o, n) in enumerate(zip(offs, lens)):
        b = host[o:o + n].tobytes()
        assert oc[i] == oracle.crc32(b), (i, n, o)
        assert oa[i] == oracle.adler32(b), (i, n, o)


# ----------------------------- deflate -----------------------------

@pytest.mark.parametrize("level", [4, 6, 9])
@pytest.mark.parametrize("kind,n", [("text", 16383), ("mix", 200000), ("runs", 70000),
                                    ("records", 100000), ("four", 50000),
                                    # >= 128 KiB: k_links keeps head[] in the key region (k_links_gh)
                                    ("text", 300001), ("runs", 131072)])
def test_stage_links_and_match_vs_oracle(zg, oracle, level, kind, n):
    """Per-position intermediates of the GPU pipeline == the oracle's
    position-parallel formulation (zo_pp_links / zo_pp_match)."""
    data = datagen.make(kind, n, 17)
    link, rf, rq = zg.debug_stages(data, level)
    olink = oracle.links(data)
    bad = np.nonzero(link != olink)[0]
    assert bad.size == 0, f"links differ at {bad[:10]}"
    of, oq = oracle.match(data, level, olink)
    bad = np.nonzero(rf != of)[0]
    assert bad.size == 0, f"rfull differ at {bad[:5]}: gpu {rf[bad[:5]]} oracle {of[bad[:5]]}"
    if level >= 5:
        bad = np.nonzero(rq != oq)[0]
        assert bad.size == 0, f"rquart differ at {bad[:5]}: gpu {rq[bad[:5]]} oracle {oq[bad[:5]]}"

@pytest.mark.parametrize("seg", [4096, 16384, 65536])
def test_stage_links_and_match_segments_vs_oracle(zg, oracle, seg, monkeypatch):
    """The per-segment stages of a sub-batch of few large buffers (k_links_seg1
    for segments up to 16 KiB: head[] at the segment start from one atomicMax
    pass over the window; k_links<kSegs> and k_match<kSegs> otherwise), per
    position against the oracle, across segment edges and ragged tails."""
    monkeypatch.setenv("ZGPU_DEBUG_SEG", str(seg))
    for kind, n, level in (("text", 70001, 6), ("mix", 150000, 9), ("runs", 65536, 4), ("records", 40000, 6)):
        data = datagen.make(kind, n, 23)
        link, rf, rq = zg.debug_stages(data, level)
        olink = oracle.links(data)
        bad = np.nonzero(link != olink)[0]
        assert bad.size == 0, f"{kind} seg {seg}: links differ at {bad[:10]}"
        of, oq = oracle.match(data, level, olink)
        bad = np.nonzero(rf != of)[0]
        assert bad.size == 0, f"{kind} seg {seg}: rfull differ at {bad[:5]}"
        if level >= 5:
            assert np.array_equal(rq, oq), f"{kind} seg {seg}: rquart differ"


@pytest.mark.parametrize("level", list(range(10)))
def test_deflate_golden(zg, golden, level):
    cases = [c for c in golden["cases"] if c["n"] <= (1 << 20)]
    bufs = [datagen.make(c["kind"], c["n"], c["seed"]) for c in cases]
    res = zg.compress_batch(bufs, level=level)
    for c, (st, z) in zip(cases, res):
        want = c["levels"][str(level)]
        assert st == 0
        assert len(z) == want["len"] and hashlib.sha256(z).hexdigest() == want["sha256"], \
            (c["kind"], c["n"], level)


def test_deflate_wrappers_golden(zg, golden):
    cases = [c for c in golden["cases"] if c["n"] <= 70000]
    bufs = [datagen.make(c["kind"], c["n"], c["seed"]) for c in cases]
    raw = zg.compress_batch(bufs, level=6, wrap=0)
    gz = zg.compress_batch(bufs, level=6, wrap=2)
    for c, (s1, r), (s2, g) in zip(cases, raw, gz):
        assert s1 == 0 and s2 == 0
        assert hashlib.sha256(r).hexdigest() == c["raw6"]["sha256"], (c["kind"], c["n"])
        assert hashlib.sha256(g).hexdigest() == c["gzip6"]["sha256"], (c["kind"], c["n"])


@pytest.mark.parametrize("level", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_deflate_random_sweep_vs_oracle(zg, oracle, level):
    rng = np.random.default_rng(100 + level)
    bufs = []
    for t in range(48):
        kind = ["text", "runs", "four", "random", "mix", "markup", "records"][t % 7]
        n = int(rng.choice([int(rng.integers(0, 700)), int(rng.integers(700, 70000)),
                            int(rng.integers(70000, 400000))]))
        bufs.append(datagen.make(kind, n, int(rng.integers(0, 1 << 30))))
    res = zg.compress_batch(bufs, level=level)
    for b, (st, z) in zip(bufs, res):
        rc, want = oracle.compress(b, level)
        assert st == 0 and z == want, (len(b), level)


def test_deflate_short_output(zg, oracle):
    data = datagen.mix(60000, 3)
    _, full = oracle.compress(data, 6)
    caps = [0, 1, 2, 9, len(full) // 2, len(full) - 1, len(full), len(full) + 100]
    res = zg.compress_batch([data] * len(caps), level=6, caps=caps)
    for cap, (st, z) in zip(caps, res):
        if cap < len(full):
            assert st == -5 and z == full[:cap], cap
        else:
            assert st == 0 and z == full


def test_deflate_device_generated_silesia(zg, oracle):
    """Device-generated benchmark input (Silesia-style mix): GPU vs oracle."""
    import torch
    n, count = 1 << 20, 6
    src = torch.empty(n * count, dtype=torch.uint8, device="cuda")
    zg.generate_dev(src, n, count, zg.KIND_SILESIA, seed=42)
    cap = zg.compress_bound(n)
    cap = (cap + 15) // 16 * 16
    off = torch.arange(count, dtype=torch.int64, device="cuda") * n
    ln = torch.full((count,), n, dtype=torch.int64, device="cuda")
    dst = torch.zeros(cap * count, dtype=torch.uint8, device="cuda")
    doff = torch.arange(count, dtype=torch.int64, device="cuda") * cap
    dcap = torch.full((count,), cap, dtype=torch.int64, device="cuda")
    dlen = torch.zeros(count, dtype=torch.int64, device="cuda")
    st = torch.zeros(count, dtype=torch.int32, device="cuda")
    zg.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=6)
    torch.cuda.synchronize()
    h_src, h_dst = src.cpu().numpy(), dst.cpu().numpy()
    dl, sts = dlen.cpu().numpy(), st.cpu().numpy()
    ratios = []
    for i in range(count):
        data = h_src[i * n:(i + 1) * n].tobytes()
        z = h_dst[i * cap: i * cap + dl[i]].tobytes()
        assert sts[i] == 0
        assert z == oracle.compress(data, 6)[1], i
        assert pyzlib.decompress(z) == data
        ratios.append(n / len(z))
    assert 2.0 < float(np.mean(ratios)) < 6.0, ratios


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_generator_kinds_roundtrip_l1_l9(zg, oracle, kind):
    import torch
    n, count = 300000, 2
    src = torch.empty(n * count, dtype=torch.uint8, device="cuda")
    zg.generate_dev(src, n, count, kind, seed=7)
    h = src.cpu().numpy()
    bufs = [h[i * n:(i + 1) * n].tobytes() for i in range(count)]
    for level in (1, 9):
        for b, (st, z) in zip(bufs, zg.compress_batch(bufs, level=level)):
            assert st == 0 and z == oracle.compress(b, level)[1]


def test_dropin_zlib_names(zg, oracle):
    L = zg.load()
    data = datagen.text(12345, 9)
    rc, z = zg.compress2(data, 9)
    assert rc == 0 and z == oracle.compress(data, 9)[1]
    # zlib_compress_simd: raw deflate (src/zlib_simd_optimized.c:365)
    out = C.create_string_buffer(zg.compress_bound(len(data)))
    olen = C.c_size_t(len(out))
    assert L.zlib_compress_simd(data, len(data), out, C.byref(olen), 6) == 0
    assert out.raw[:olen.value] == oracle.compress(data, 6, wrap=0)[1]
    # streaming deflate(): Z_NO_FLUSH chunks then Z_FINISH, drained 1000 B at a time
    from zhelpers import ZStream
    L.deflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_char_p, C.c_int]
    L.deflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.deflateEnd.argtypes = [C.POINTER(ZStream)]
    s = ZStream()
    assert L.deflateInit2_(C.byref(s), 6, 8, 31, 8, 0, b"1.3.1.1-motley", C.sizeof(ZStream)) == 0
    inbuf = C.create_string_buffer(data, len(data))
    outbuf = C.create_string_buffer(1000)
    got = b""
    for k in range(0, len(data), 4000):
        s.next_in = C.addressof(inbuf) + k
        s.avail_in = min(4000, len(data) - k)
        s.next_out, s.avail_out = C.addressof(outbuf), 1000
        assert L.deflate(C.byref(s), 0) == 0
        got += outbuf.raw[:1000 - s.avail_out]       # the header, then blocks as they complete
    while True:
        s.next_out, s.avail_out = C.addressof(outbuf), 1000
        rc = L.deflate(C.byref(s), 4)
        got += outbuf.raw[:1000 - s.avail_out]
        if rc == 1:
            break
        assert rc == 0
    assert L.deflateEnd(C.byref(s)) == 0
    assert got == oracle.compress(data, 6, wrap=2)[1]
    z = zg.Zlib().compress(data, level=6)
    assert z.data == oracle.compress(data, 6)[1] and z.originalSize == len(data)


def test_crc_adler_many_small_ragged(zg, oracle):
    """>= 16384 buffers selects the 16-lanes-per-buffer CRC kernel."""
    rng = np.random.default_rng(11)
    lens = [int(x) for x in rng.integers(0, 3000, 20000)]
    lens[:8] = [0, 1, 3, 4, 255, 256, 257, 4096]
    pool = datagen.random_bytes(sum(lens) + 16, 3)
    bufs, p = [], 0
    for n in lens:
        bufs.append(pool[p:p + n])
        p += n
    inits = [int(x) for x in rng.integers(0, 1 << 32, len(bufs), dtype=np.uint64)]
    got = zg.crc32_batch(bufs, inits)
    for b, ic, g in zip(bufs, inits, got):
        assert g == oracle.crc32(b, ic), len(b)
    got = zg.adler32_batch(bufs)
    for b, g in zip(bufs, got):
        assert g == oracle.adler32(b), len(b)


@pytest.mark.parametrize("level", [4, 6, 9])
def test_pipeline_many_subbatches(zg, oracle, level):
    """A small in-flight budget splits the batch into many sub-batches, so the
    two-stream L4-9 pipeline runs and reuses both workspace slots."""
    rng = np.random.default_rng(200 + level)
    bufs = []
    for t in range(40):
        kind = ["text", "runs", "four", "random", "mix", "markup", "records"][t % 7]
        n = int(rng.choice([0, 1, 300, int(rng.integers(300, 120000)), int(rng.integers(120000, 300000))]))
        bufs.append(datagen.make(kind, n, int(rng.integers(0, 1 << 30))))
    old = zg.set_inflight_bytes(300 * 1024)
    try:
        for wrap in (0, 1, 2):
            res = zg.compress_batch(bufs, level=level, wrap=wrap)
            for b, (st, z) in zip(bufs, res):
                assert st == 0 and z == oracle.compress(b, level, wrap=wrap)[1], (len(b), level, wrap)
    finally:
        zg.set_inflight_bytes(old)


def test_deflate_pathological_sync(zg, oracle):
    """Inputs where speculative lazy-parse segments may never meet (runs,
    short and long periods), plus the k_parse_slow fallback they can take."""
    n = 1 << 20
    pat3 = (b"abc" * (n // 3 + 1))[:n]
    pat257 = (bytes(range(256)) + b"!") * (n // 257 + 1)
    bufs = [bytes(n), pat3, pat257[:n], datagen.make("runs", n, 9), (b"\x00" * 258 + b"\x01") * 4000]
    for level in (4, 6, 9):
        for b, (st, z) in zip(bufs, zg.compress_batch(bufs, level=level)):
            assert st == 0 and z == oracle.compress(b, level)[1], (len(b), level)
            assert pyzlib.decompress(z) == b


def test_deflate_literal_tail_neighbours(zg, oracle):
    """All-literal buffers whose length is a multiple of 64 (the workspace
    rounding) packed between compressible ones: the lazy parse stages such a
    buffer's final pending literal at index n, which must stay inside its own
    workspace region (it once overwrote the neighbour's first staged symbol,
    depending on timing)."""
    bufs = []
    for t in range(96):
        n = 64 * int(np.random.default_rng(t).integers(1, 2048))
        bufs.append(datagen.make("random", n, 7000 + t))
        bufs.append(datagen.make("text", 65536, 8000 + t))
    for level in (4, 6, 9):
        for strategy in (0, 1):
            res = zg.compress_batch(bufs, level=level, strategy=strategy)
            for b, (st, z) in zip(bufs, res):
                assert st == 0 and z == oracle.compress(b, level, strategy=strategy)[1], (len(b), level, strategy)


@pytest.mark.parametrize("strategy", [1, 2, 3, 4], ids=["filtered", "huffman_only", "rle", "fixed"])
def test_deflate_strategies_golden(zg, golden, strategy):
    """deflateInit2_ strategies vs the compiled reference's outputs (fixtures)."""
    cases = [c for c in golden["cases"] if c["n"] <= (1 << 20)]
    bufs = [datagen.make(c["kind"], c["n"], c["seed"]) for c in cases]
    for level in (1, 4, 6, 9):
        res = zg.compress_batch(bufs, level=level, strategy=strategy)
        for c, (st, z) in zip(cases, res):
            want = c["strategies"][f"{strategy}/{level}"]
            assert st == 0 and len(z) == want["len"] and hashlib.sha256(z).hexdigest() == want["sha256"], \
                (c["kind"], c["n"], level, strategy)


@pytest.mark.parametrize("strategy", [1, 2, 3, 4])
def test_deflate_strategies_sweep_vs_oracle(zg, oracle, strategy):
    rng = np.random.default_rng(400 + strategy)
    bufs = [datagen.make(["runs", "text", "mix", "random", "records"][t % 5],
                         int(rng.choice([0, 5, 300, int(rng.integers(300, 300000))])),
                         int(rng.integers(0, 1 << 30))) for t in range(30)]
    old = zg.set_inflight_bytes(400 * 1024)            # several sub-batches (and the L4-9 pipeline)
    try:
        for level in (0, 2, 5, 8):
            for wrap in (0, 1, 2):
                for b, (st, z) in zip(bufs, zg.compress_batch(bufs, level=level, wrap=wrap, strategy=strategy)):
                    assert st == 0 and z == oracle.compress(b, level, wrap=wrap, strategy=strategy)[1], \
                        (len(b), level, wrap, strategy)
    finally:
        zg.set_inflight_bytes(old)


def test_deflateinit2_strategy_stream(zg, oracle):
    L = zg.load()
    from zhelpers import ZStream
    L.deflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_char_p, C.c_int]
    L.deflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.deflateEnd.argtypes = [C.POINTER(ZStream)]
    data = datagen.mix(150000, 4)
    for strategy in range(5):
        s = ZStream()
        assert L.deflateInit2_(C.byref(s), 6, 8, 15, 8, strategy, b"1.3.1.1-motley", C.sizeof(ZStream)) == 0
        inbuf = C.create_string_buffer(data, len(data))
        out = C.create_string_buffer(len(data) * 2 + 100)
        s.next_in, s.avail_in = C.addressof(inbuf), len(data)
        s.next_out, s.avail_out = C.addressof(out), len(out)
        assert L.deflate(C.byref(s), 4) == 1
        got = out.raw[:s.total_out]
        assert L.deflateEnd(C.byref(s)) == 0
        assert got == oracle.compress(data, 6, wrap=1, strategy=strategy)[1], strategy


def test_few_large_buffers_segmented_match(zg, oracle):
    """A sub-batch of few large buffers runs k_match per 256 KiB segment (each
    stages the 32 KiB before it): streams equal the oracle's at segment edges,
    ragged sizes and every lazy level."""
    bufs = [datagen.make("mix", (8 << 20) + 77, 61), datagen.make("text", (1 << 20) + 5, 62),
            datagen.make("runs", 700 * 1024 + 3, 63), datagen.make("records", (5 << 18) + 4095, 64)]
    for level in (4, 6, 9):
        got = zg.compress_batch(bufs, level=level)
        for b, (st, z) in zip(bufs, got):
            assert st == 0 and z == oracle.compress(b, level)[1], (len(b), level)


def test_small_single_buffers_tile_segments(zg, oracle):
    """A lone small buffer (C1's 64 KB compress2) walks k_match in segments as
    short as one 4 KiB tile, each staging the <= 32 KiB before it: streams equal
    the oracle's for one-tile, few-tile and ragged segments at every lazy level."""
    cases = [[datagen.make("text", 64 * 1024, 71)], [datagen.make("mix", 64 * 1024 + 1, 72)],
             [datagen.make("markup", 300 * 1024 + 9, 73)], [datagen.make("runs", 40 * 1024 - 1, 74)],
             [datagen.make("text", 5000, 75), datagen.make("records", 150 * 1024 + 3, 76)]]
    for bufs in cases:
        for level in (4, 6, 9):
            got = zg.compress_batch(bufs, level=level)
            for b, (st, z) in zip(bufs, got):
                assert st == 0 and z == oracle.compress(b, level)[1], (len(b), level)
        rc, z = zg.compress2(bufs[-1], level=6)
        assert rc == 0 and z == oracle.compress(bufs[-1], 6)[1]


def test_small_buffers_short_segments_chain(zg, oracle):
    """Sub-batches of few buffers of at most 64 KiB parse in 256-byte segments
    (k_pbig1..5), where a lane's run-on may cross up to 8 segments before it
    meets a later lane's pass 1 and k_pbig3 joins the chain of meets.  Runs
    of 300..600 bytes and periodic data make the meets skip segments; 64 KiB
    of zeros never meets within reach (the buffer falls back to k_parse_slow);
    tiny and ragged sizes give one- and two-lane buffers."""
    rng = np.random.default_rng(31)
    runs = bytes(np.repeat(rng.integers(0, 256, 200, dtype=np.uint8), rng.integers(300, 600, 200))[:65536])
    cases = [[bytes(65536)], [runs], [(b"\x00" * 258 + b"\x01") * 252], [(b"abc" * 21846)[:65536]],
             [datagen.make("text", 65536, 81)], [datagen.make("mix", 65535, 82)], [datagen.make("random", 65536, 83)],
             [datagen.make("markup", 40000, 84), datagen.make("records", 65536, 85), datagen.make("runs", 257, 86),
              datagen.make("text", 256, 87), datagen.make("text", 513, 88)],
             [datagen.make("runs", 65536, 89), runs[:4097], bytes(5000), datagen.make("text", 30001, 90)]]
    for bufs in cases:
        for level in (4, 5, 6, 9):
            for strategy in (0, 1):
                got = zg.compress_batch(bufs, level=level, strategy=strategy)
                for b, (st, z) in zip(bufs, got):
                    assert st == 0 and z == oracle.compress(b, level, strategy=strategy)[1], \
                        (len(b), level, strategy)
        rc, z = zg.compress2(bufs[0], level=6)
        assert rc == 0 and z == oracle.compress(bufs[0], 6)[1]


def _syszlib(b, level, wbits=15, mem_level=8):
    c = pyzlib.compressobj(level, pyzlib.DEFLATED, wbits, mem_level)
    return c.compress(bytes(b)) + c.flush()


@pytest.mark.parametrize("level", [1, 2, 3])
def test_fast_levels_lds_parse(zg, level):
    """Few buffers at L1-3.  Level 1 parses with head[], prev[] and the window
    in LDS (k_parse_fast<kLds>): 16-bit head entries swept every 16 Ki
    positions, a 32 Ki prev ring and a 32 Ki byte ring filled to p + 262.
    Levels 2-3 with at most 16 buffers take the sorted-run parse (k_parse_srt)
    by default; test_fast_levels_lds_parse_without_srt runs the same cases on
    k_parse_fast<kLds> there (the path a failed sorted-run allocation takes).
    Streams equal system zlib's for lone buffers across sweeps and ring wraps,
    tiny and empty buffers, smaller windows and memLevels, and a batch above the
    LDS variant's 256-buffer limit (the HBM variant) beside one below it."""
    cases = [[datagen.make("text", 64 * 1024, 81)], [datagen.make("mix", (3 << 20) + 17, 82)],
             [datagen.make("runs", 70000, 83)], [datagen.make("records", (1 << 20) + 1, 84)],
             [b"", b"a", b"ab", b"abc", bytes(300), datagen.make("markup", 32768 + 262, 85)]]
    for bufs in cases:
        got = zg.compress_batch(bufs, level=level)
        for b, (st, z) in zip(bufs, got):
            assert st == 0 and z == _syszlib(b, level), (len(b), level)
    b = datagen.make("mix", 200000, 86)
    for wb, ml in ((9, 8), (12, 5), (15, 1), (15, 9), (-13, 7)):
        (st, z), = zg.compress_batch2([b], level=level, window_bits=wb, mem_level=ml)
        assert st == 0 and z == _syszlib(b, level, wb, ml), (wb, ml)
    rng = np.random.default_rng(87)
    for count in (200, 300):
        bufs = [datagen.make(("text", "mix", "runs")[i % 3], int(rng.integers(1, 40000)), 900 + i)
                for i in range(count)]
        got = zg.compress_batch(bufs, level=level)
        for b, (st, z) in zip(bufs, got):
            assert st == 0 and z == _syszlib(b, level), (len(b), count)


def test_fast_levels_lds_parse_without_srt():
    """ZGPU_FAST_SRT is read once per process, so levels 2-3 with few buffers
    run k_parse_srt in the rest of the suite.  Here a child process with
    ZGPU_FAST_SRT=0 runs test_fast_levels_lds_parse's cases at levels 2 and 3
    on k_parse_fast<kLds>, against system zlib."""
    import subprocess
    import sys
    code = (
        "import sys, zlib; sys.path[:0] = [%r, %r]\n"
        "import torch, zgpu, datagen\n"
        "zgpu.load()\n"
        "for level in (2, 3):\n"
        "    cases = [[datagen.make('text', 64 * 1024, 81)], [datagen.make('mix', (3 << 20) + 17, 82)],\n"
        "             [datagen.make('runs', 70000, 83)], [datagen.make('records', (1 << 20) + 1, 84)],\n"
        "             [b'', b'a', b'ab', b'abc', bytes(300), datagen.make('markup', 32768 + 262, 85)]]\n"
        "    for bufs in cases:\n"
        "        for b, (st, z) in zip(bufs, zgpu.compress_batch(bufs, level=level)):\n"
        "            assert st == 0 and z == zlib.compress(b, level), (len(b), level)\n"
        "print('ok')\n" % (os.path.join(ROOT, "zlib.wasm_amd"), os.path.join(ROOT, "tests")))
    env = dict(os.environ, ZGPU_FAST_SRT="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("level", [5, 6, 9])
def test_links_head_in_key_region_params(zg, level):
    """k_links_gh (head[] as 32-bit positions in the key region, for batches
    whose buffers are all >= 128 KiB and whose stages run one after another)
    under other windowBits / memLevels: hash_bits 8..15 index the same table,
    memLevel 9 keeps the LDS kernel; streams equal system zlib's, beside a
    batch with one buffer under 128 KiB (the LDS kernel)."""
    bufs = [datagen.make("mix", 200000, 91), datagen.make("text", 300001, 92)]
    for wb, ml in ((9, 1), (10, 5), (13, 7), (15, 8), (15, 9)):
        got = zg.compress_batch2(bufs, level=level, window_bits=wb, mem_level=ml)
        for b, (st, z) in zip(bufs, got):
            assert st == 0 and z == _syszlib(b, level, wb, ml), (len(b), wb, ml)
    mixed = bufs + [datagen.make("records", 70000, 93)]
    got = zg.compress_batch(mixed, level=level)
    for b, (st, z) in zip(mixed, got):
        assert st == 0 and z == _syszlib(b, level), len(b)


def test_wasm_production_entry_points(zg, oracle):
    """The reference's production path: Zlib.compress -> zlib_compress_buffer,
    and the zlib_crc32 / zlib_adler32 exports (src/wasm_module.c:35,66,74),
    including their argument checks (null / zero length -> Z_STREAM_ERROR,
    level outside 0..9 -> the default level)."""
    L = zg.load()
    L.zlib_compress_buffer.restype = C.c_int
    L.zlib_compress_buffer.argtypes = [C.c_char_p, C.c_ulong, C.c_void_p, C.POINTER(C.c_ulong), C.c_int]
    L.zlib_crc32.restype = C.c_ulong
    L.zlib_crc32.argtypes = [C.c_ulong, C.c_char_p, C.c_uint]
    L.zlib_adler32.restype = C.c_ulong
    L.zlib_adler32.argtypes = [C.c_ulong, C.c_char_p, C.c_uint]
    for i, (kind, n) in enumerate([("text", 65536), ("mix", 300000), ("runs", 1000), ("random", 70000)]):
        data = datagen.make(kind, n, 40 + i)
        for level, want_level in ((1, 1), (6, 6), (9, 9), (-1, 6), (12, 6)):
            out = C.create_string_buffer(zg.compress_bound(n))
            olen = C.c_ulong(len(out))
            assert L.zlib_compress_buffer(data, n, out, C.byref(olen), level) == 0
            assert out.raw[:olen.value] == oracle.compress(data, want_level)[1], (kind, level)
        assert L.zlib_crc32(0, data, n) == oracle.crc32(data)
        assert L.zlib_crc32(0x12345678, data, n) == oracle.crc32(data, 0x12345678)
        assert L.zlib_adler32(1, data, n) == oracle.adler32(data)
    out = C.create_string_buffer(64)
    olen = C.c_ulong(64)
    assert L.zlib_compress_buffer(None, 10, out, C.byref(olen), 6) == -2
    assert L.zlib_compress_buffer(b"abc", 0, out, C.byref(olen), 6) == -2
    olen = C.c_ulong(5)                                   # short output: zlib's Z_BUF_ERROR
    assert L.zlib_compress_buffer(datagen.text(5000, 1), 5000, out, C.byref(olen), 6) == -5


def test_concurrent_host_threads(zg, oracle):
    """Host threads each lease their own context/stream (zlib.h:150-151): 8
    threads running compress2 / crc32 / uncompress side by side get the same
    results as one thread."""
    import concurrent.futures as cf
    datas = [datagen.make(k, 50000 + 7919 * i, 300 + i)
             for i, k in enumerate(["text", "mix", "runs", "four"] * 6)]
    want = [oracle.compress(d, 6)[1] for d in datas]

    def work(i):
        d = datas[i]
        rc, z = zg.compress2(d, 6)
        c = zg.crc32(d)
        u = zg.uncompress2(z, len(d))
        return rc, z, c, u

    with cf.ThreadPoolExecutor(8) as ex:
        res = list(ex.map(work, range(len(datas))))
    for d, w, (rc, z, c, u) in zip(datas, want, res):
        assert rc == 0 and z == w
        assert c == oracle.crc32(d)
        assert u[0] == 0 and u[1] == d


def test_bench_golden_device_generated(zg):
    """The benchmark's workloads end to end on the device: each golden case's
    input is generated in HBM by zgpu_generate_dev (its sha256 pins the device
    generator to the host build the fixtures came from), compressed by
    zgpu_deflate_batch_dev at the config's level, and the stream must equal
    the compiled reference's: C4 L6 (bench seed and indices up to 262143), C3
    L1, and C5's 16 MiB small-vocabulary / 4-letter / runs buffers at L9 with
    the Adler-32 trailer."""
    import hashlib
    import json
    import os
    import torch
    here = os.path.dirname(os.path.abspath(__file__))
    g = json.load(open(os.path.join(here, "golden", "bench_golden.json")))
    for c in g["cases"]:
        n = c["n"]
        src = torch.empty(n, dtype=torch.uint8, device="cuda")
        zg.generate_dev(src, n, 1, c["kind"], seed=c["seed"], first_index=c["index"])
        host = src.cpu().numpy().tobytes()
        assert hashlib.sha256(host).hexdigest() == c["input_sha256"], c["name"]
        cap = (zg.compress_bound(n) + 15) // 16 * 16
        dst = torch.empty(cap, dtype=torch.uint8, device="cuda")
        z64 = lambda v: torch.tensor([v], dtype=torch.int64, device="cuda")  # noqa: E731
        dlen, st = z64(0), torch.tensor([99], dtype=torch.int32, device="cuda")
        zg.deflate_batch_dev(src, z64(0), z64(n), dst, z64(0), z64(cap), dlen, st, level=c["level"])
        torch.cuda.synchronize()
        assert int(st.item()) == 0
        z = dst[:int(dlen.item())].cpu().numpy().tobytes()
        assert len(z) == c["len"] and hashlib.sha256(z).hexdigest() == c["sha256"], \
            (c["name"], c["kind"], c["index"])
        out = torch.zeros(2, dtype=torch.int32, device="cuda")
        zg.adler32_batch_dev(src, z64(0), z64(n), out[:1])
        zg.crc32_batch_dev(src, z64(0), z64(n), out[1:])
        a, cr = (int(x) & 0xffffffff for x in out.cpu().tolist())
        assert a == c["adler32"] and cr == c["crc32"], c["name"]


def test_literal_block_count_golden(zg):
    """All-literal inputs of 16383*k bytes (no 3-byte string repeats): blocks
    cut at exactly 16383 symbols (deflate.h:371), levels 1/6/9."""
    import hashlib
    import json
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    from make_bench_golden import literal_input
    g = json.load(open(os.path.join(here, "golden", "bench_golden.json")))
    for level in (1, 6, 9):
        bufs = [literal_input(e["n"]) for e in g["literal_blocks"]]
        res = zg.compress_batch(bufs, level=level)
        for e, (st, z) in zip(g["literal_blocks"], res):
            assert st == 0 and hashlib.sha256(z).hexdigest() == e["levels"][str(level)]["sha256"], (e["k"], level)


def test_checksum_split_few_large_buffers(zg, oracle):
    """Few large buffers take the split checksum kernels (row ranges per wave,
    joined per buffer): ragged lengths around the split boundaries, random
    inits, against the oracle."""
    import torch
    rng = np.random.default_rng(11)
    lens = [0, 1, 3, 4, 15, 16, 17, 4095, 4096, 4097, 65536 * 3 + 7, (1 << 20) + 1, 5 * (1 << 20) + 12345,
            16 << 20, (16 << 20) - 1]
    offs, pos = [], 0
    for n in lens:
        offs.append(pos)
        pos += n + 1 + int(rng.integers(0, 7))
    host = np.frombuffer(datagen.random_bytes(pos + 16, 2), dtype=np.uint8)
    src = torch.from_numpy(host.copy()).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor(lens, dtype=torch.int64).cuda()
    ci = [int(x) for x in rng.integers(0, 1 << 32, len(lens), dtype=np.uint64)]
    ai = [int(a) | (int(b) << 16) for a, b in zip(rng.integers(0, 65521, len(lens)), rng.integers(0, 65521, len(lens)))]
    cin = torch.tensor(np.array(ci, dtype=np.uint32).view(np.int32)).cuda()
    ain = torch.tensor(np.array(ai, dtype=np.uint32).view(np.int32)).cuda()
    oc = torch.zeros(len(lens), dtype=torch.int32).cuda()
    oa = torch.zeros(len(lens), dtype=torch.int32).cuda()
    zg.crc32_batch_dev(src, off, ln, oc, init=cin)
    zg.adler32_batch_dev(src, off, ln, oa, init=ain)
    torch.cuda.synchronize()
    gc, ga = oc.cpu().numpy().view(np.uint32), oa.cpu().numpy().view(np.uint32)
    for i, n in enumerate(lens):
        b = host[offs[i]:offs[i] + n].tobytes()
        assert int(gc[i]) == oracle.crc32(b, ci[i]), n
        assert int(ga[i]) == oracle.adler32(b, ai[i]), n


def test_window_bits_mem_level_golden(zg, golden):
    """deflateInit2_'s windowBits 8..15 (raw / gzip forms too) and memLevel 1..9
    at levels 0-9 and all strategies (hash_bits, hash_shift, lit_bufsize block
    cut, MAX_DIST, slide schedule, header): every stream equals the compiled
    reference's (tests/golden/params_golden.json)."""
    import hashlib
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "params_golden.json")))
    datas = [datagen.make(k, n, s) for k, n, s in g["inputs"]]
    for c in g["cases"]:
        res = zg.compress_batch2(datas, level=c["level"], window_bits=c["window_bits"], mem_level=c["mem_level"],
                                 strategy=c["strategy"])
        for (st, z), want, (k, n, _) in zip(res, c["streams"], g["inputs"]):
            assert st == 0 and len(z) == want["len"] and hashlib.sha256(z).hexdigest() == want["sha256"], \
                (c["level"], c["window_bits"], c["mem_level"], c["strategy"], k, n)


def test_deflateinit2_params_stream(zg):
    """The z_stream API with windowBits / memLevel: deflateInit2_ + deflate(Z_FINISH)
    equals the fixture for a sample of settings."""
    import hashlib
    import json
    import os
    from zhelpers import ZStream
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "params_golden.json")))
    L = zg.load()
    L.deflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_char_p, C.c_int]
    L.deflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.deflateEnd.argtypes = [C.POINTER(ZStream)]
    k, n, sd = g["inputs"][1]
    data = datagen.make(k, n, sd)
    for c in g["cases"][::9]:
        s = ZStream()
        assert L.deflateInit2_(C.byref(s), c["level"], 8, c["window_bits"], c["mem_level"], c["strategy"],
                               b"1.3.1.1-motley", C.sizeof(ZStream)) == 0
        inb = C.create_string_buffer(data, len(data))
        cap = len(data) * 2 + 1024
        out = C.create_string_buffer(cap)
        s.next_in, s.avail_in = C.addressof(inb), len(data)
        s.next_out, s.avail_out = C.addressof(out), cap
        assert L.deflate(C.byref(s), 4) == 1
        z = out.raw[:cap - s.avail_out]
        L.deflateEnd(C.byref(s))
        want = c["streams"][1]
        assert hashlib.sha256(z).hexdigest() == want["sha256"], (c["level"], c["window_bits"], c["mem_level"])


def test_huffman_length_overflow(zg, oracle):
    """Literal counts on a Fibonacci ladder (a 19-leaf tree 18 deep): gen_bitlen's
    overflow repair (trees.c:446-484) in the literal tree, and skewed code-length
    counts for the bit-length tree (max 7).  k_encode's wave-wide tree build
    (w_build, launches under 1024 buffers) and its one-lane build (t_build, a
    1026-buffer launch) against the oracle, Z_HUFFMAN_ONLY and level 1/6/9
    parses, one and several blocks."""
    fib = [1, 1]
    while len(fib) < 19:
        fib.append(fib[-1] + fib[-2])
    rng = np.random.default_rng(11)
    bufs = []
    for seed in range(6):
        syms = rng.permutation(256)[:19]
        parts = []
        for rep in range(1 + seed % 3):                  # 1..3 blocks of symbols
            a = np.repeat(syms, fib)
            parts.append(a[rng.permutation(len(a))])
        bufs.append(np.concatenate(parts).astype(np.uint8).tobytes())
    for level, strategy in ((6, 2), (1, 2), (6, 0), (9, 0)):
        res = zg.compress_batch(bufs, level=level, strategy=strategy)
        for b, (st, z) in zip(bufs, res):
            assert st == 0 and z == oracle.compress(b, level, strategy=strategy)[1], (len(b), level, strategy)
    # >= 1024 buffers in one launch: k_encode's one-lane build (t_build), same inputs
    many = bufs * 171
    for level, strategy in ((6, 2), (6, 0)):
        want = [oracle.compress(b, level, strategy=strategy)[1] for b in bufs]
        res = zg.compress_batch(many, level=level, strategy=strategy)
        for i, (st, z) in enumerate(res):
            assert st == 0 and z == want[i % len(bufs)], (i, level, strategy)


def test_bench_scale_subbatch_golden(zg):
    """Bench-scale parity: a whole sub-batch of the benchmark's
    shape -- 4096 x 1 MiB at L6 in one 4 GiB in-flight sub-batch (lane-built
    trees, the two-slot pipeline's slot 0), and 4096 x 1 MiB enwik-style at L1
    -- through zgpu_deflate_batch_dev; a strided sample of the streams equals
    the compiled reference's (tests/golden/batch_golden.json), every status is
    Z_OK and every stream inflates back to its input on the device."""
    import json
    import os
    import torch
    here = os.path.dirname(os.path.abspath(__file__))
    g = json.load(open(os.path.join(here, "golden", "batch_golden.json")))
    old = zg.set_inflight_bytes(4 << 30)
    try:
        for b in g["batches"]:
            n, B = b["n"], b["buffers"]
            cap = (zg.compress_bound(n) + 15) // 16 * 16
            src = torch.empty(n * B, dtype=torch.uint8, device="cuda")
            zg.generate_dev(src, n, B, b["kind"], seed=b["seed"], first_index=0)
            off = torch.arange(B, dtype=torch.int64, device="cuda") * n
            ln = torch.full((B,), n, dtype=torch.int64, device="cuda")
            dst = torch.empty(cap * B, dtype=torch.uint8, device="cuda")
            doff = torch.arange(B, dtype=torch.int64, device="cuda") * cap
            dcap = torch.full((B,), cap, dtype=torch.int64, device="cuda")
            dlen = torch.zeros(B, dtype=torch.int64, device="cuda")
            st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
            zg.deflate_batch_dev(src, off, ln, dst, doff, dcap, dlen, st, level=b["level"])
            torch.cuda.synchronize()
            assert int((st != 0).sum().item()) == 0, b["name"]
            lens = dlen.cpu().tolist()
            for c in b["cases"]:
                i = c["index"]
                raw = src[i * n:(i + 1) * n].cpu().numpy().tobytes()
                assert hashlib.sha256(raw).hexdigest() == c["input_sha256"], (b["name"], i)
                z = dst[i * cap:i * cap + lens[i]].cpu().numpy().tobytes()
                assert len(z) == c["len"] and hashlib.sha256(z).hexdigest() == c["sha256"], (b["name"], i)
            out = torch.empty(n * B, dtype=torch.uint8, device="cuda")
            olen = torch.zeros(B, dtype=torch.int64, device="cuda")
            ost = torch.full((B,), 99, dtype=torch.int32, device="cuda")
            zg.inflate_batch_dev(dst, doff, dlen, out, off, ln, olen, ost)
            torch.cuda.synchronize()
            assert int((ost != 0).sum().item()) == 0 and bool((olen == n).all().item())
            assert torch.equal(out, src), b["name"]
            del src, dst, out
            torch.cuda.empty_cache()
    finally:
        zg.set_inflight_bytes(old)


def test_bench_rccl_path_one_rank():
    """bench.py under torch.distributed.run with one rank on the GPU: the RCCL
    process group (nccl backend, device_id bound), its barrier, all_reduce and
    all_gather on device tensors -- the path every rank of an 8-GPU run takes --
    run on a one-GPU box, and the line reports them."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(root, "bench.py"), "--gpus", "1",
           "--steps", "1", "--warmup", "0", "--buffers", "64", "--no-cpu", "--no-inflate", "--crc-buffers", "4096",
           "--adler-buffers", "0", "--verify", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["config"]["collective_backend"] == "nccl" and line["config"]["world_size_seen"] == 1
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert len(line["per_rank"]) == 1 and line["per_rank"][0]["out_bytes"] > 0
