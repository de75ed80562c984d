"""GPU parity tests for batched inflate: the HIP path through
the C ABI against the reference's uncompress2 results frozen in
tests/golden/inflate_golden.json and against the oracle (oracle/zinflate.c).
Bit-exact: status, output bytes and input bytes consumed."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import datagen
import inflate_cases as ic
from zhelpers import ZStream

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def inflate_golden():
    with open(os.path.join(HERE, "golden", "inflate_golden.json")) as f:
        return json.load(f)


def _streams(cases, oracle):
    comp = lambda d, level, wrap, strategy: oracle.compress(d, level, wrap=wrap, strategy=strategy)[1]
    bases, out = {}, []
    for c in cases:
        if "hex" in c:
            out.append(bytes.fromhex(c["hex"]))
            continue
        key = (c["kind"], c["n"], c["seed"], c["level"], c["wrap"], c["strategy"])
        if key not in bases:
            bases[key] = ic.base_stream(c, comp)[1]
            assert ic.sha(bases[key]) == c["base_sha256"], key
        out.append(ic.mutate(bases[key], c["mut"]))
    return out


def test_inflate_golden(zg, oracle, inflate_golden):
    """All 2427 reference cases, one batch per decoder wrapper."""
    cases = inflate_golden["cases"]
    streams = _streams(cases, oracle)
    for wrap in (0, 1, 2, 3):
        idx = [i for i, c in enumerate(cases) if c["dwrap"] == wrap]
        res = zg.uncompress_batch([streams[i] for i in idx], [cases[i]["cap"] for i in idx], wrap=wrap)
        for i, (st, out, used) in zip(idx, res):
            e = cases[i]["expect"]
            assert (st, len(out), ic.sha(out), used) == (e["status"], e["len"], e["sha256"], e["consumed"]), \
                (i, cases[i])


def test_inflate_roundtrip_all_levels_strategies(zg, oracle):
    """GPU deflate -> GPU inflate over every level, strategy and wrapper."""
    rng = np.random.default_rng(5)
    bufs = [datagen.make(["text", "mix", "runs", "random", "records", "markup", "four"][t % 7],
                         int(rng.choice([0, 1, 100, 5000, 70000, 300000])), 900 + t) for t in range(28)]
    for level in range(10):
        for strategy in (0, 1, 2, 3, 4):
            if level == 0 and strategy:
                continue
            wrap = (level + strategy) % 3
            zs = zg.compress_batch(bufs, level=level, wrap=wrap, strategy=strategy)
            streams = [z for st, z in zs]
            assert all(st == 0 for st, _ in zs)
            res = zg.uncompress_batch(streams, [len(b) for b in bufs], wrap=wrap)
            for b, z, (st, out, used) in zip(bufs, streams, res):
                assert st == 0 and out == b and used == len(z), (len(b), level, strategy, wrap)


def test_inflate_large_many_subbatches(zg, oracle):
    """1 MiB streams across several sub-batches (small in-flight budget), with
    long matches, stored blocks and window-distance copies."""
    bufs = [datagen.make(["mix", "runs", "random", "text"][t % 4], 1 << 20, 40 + t) for t in range(12)]
    zs = [oracle.compress(b, [1, 6, 9][t % 3])[1] for t, b in enumerate(bufs)]
    old = zg.set_inflight_bytes(3 << 20)
    try:
        res = zg.uncompress_batch(zs, [len(b) for b in bufs])
    finally:
        zg.set_inflight_bytes(old)
    for b, z, (st, out, used) in zip(bufs, zs, res):
        assert st == 0 and used == len(z) and out == b


def test_inflate_fuzz_vs_oracle(zg, oracle):
    """Bit flips, truncations and short outputs of larger streams."""
    rng = np.random.default_rng(11)
    streams, caps, wraps = [], [], []
    for t in range(40):
        data = datagen.make(["text", "mix", "runs", "records"][t % 4], int(rng.integers(1000, 150000)), 300 + t)
        wrap = t % 3
        z = oracle.compress(data, int(rng.integers(1, 10)), wrap=wrap)[1]
        for _ in range(6):
            zz = bytearray(z)
            i = int(rng.integers(0, len(zz) * 8))
            zz[i >> 3] ^= 1 << (i & 7)
            streams.append(bytes(zz)); caps.append(len(data) + 10); wraps.append(wrap)
        cut = int(rng.integers(0, len(z)))
        streams.append(z[:cut]); caps.append(len(data)); wraps.append(wrap)
        streams.append(z); caps.append(int(rng.integers(0, len(data)))); wraps.append(wrap)
    for wrap in (0, 1, 2):
        idx = [i for i in range(len(streams)) if wraps[i] == wrap]
        res = zg.uncompress_batch([streams[i] for i in idx], [caps[i] for i in idx], wrap=wrap)
        for i, got in zip(idx, res):
            assert got == oracle.uncompress(streams[i], caps[i], wrap), i


def test_uncompress_dropin_names(zg, oracle):
    """uncompress / uncompress2 / zlib_decompress_buffer through the exported symbols."""
    L = zg.load()
    data = datagen.make("mix", 200000, 17)
    z = oracle.compress(data, 6)[1]
    assert zg.uncompress2(z, len(data)) == (0, data, len(z))
    assert zg.uncompress2(z + b"trailing", len(data) + 5) == (0, data, len(z))
    # truncated trailer: Z_BUF_ERROR when the output is exactly full, else Z_DATA_ERROR
    assert zg.uncompress2(z[:-3], len(data)) == oracle.uncompress(z[:-3], len(data))
    assert zg.uncompress2(z[:-3], len(data))[0] == -5
    assert zg.uncompress2(z[:-3], len(data) + 1) == oracle.uncompress(z[:-3], len(data) + 1)
    assert zg.uncompress2(z[:-3], len(data) + 1)[0] == -3
    assert zg.uncompress2(z, 1000) == oracle.uncompress(z, 1000)
    out = C.create_string_buffer(len(data))
    dl = C.c_ulong(len(data))
    assert L.uncompress(out, C.byref(dl), z, len(z)) == 0 and out.raw[: dl.value] == data
    L.zlib_decompress_buffer.argtypes = [C.c_char_p, C.c_ulong, C.c_void_p, C.POINTER(C.c_ulong)]
    dl = C.c_ulong(len(data))
    assert L.zlib_decompress_buffer(z, len(z), out, C.byref(dl)) == 0 and out.raw[: dl.value] == data
    assert L.zlib_decompress_buffer(z, 0, out, C.byref(dl)) == -2       # src_len == 0 -> Z_STREAM_ERROR


def test_inflate_stream_api(zg, oracle):
    """inflateInit2_ / inflate / inflateEnd with chunked input and small output
    windows, every wrapper, trailing data handed back, and a corrupt stream."""
    from zhelpers import ZStream
    L = zg.load()
    L.inflateInit2_.restype = C.c_int
    L.inflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_char_p, C.c_int]
    L.inflate.restype = C.c_int
    L.inflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.inflateEnd.argtypes = [C.POINTER(ZStream)]
    data = datagen.make("text", 300000, 3)
    for wrap, wbits in ((0, -15), (1, 15), (2, 31), (2, 47), (1, 47)):
        z = oracle.compress(data, 6, wrap=wrap)[1] + b"XYZ"
        s = ZStream()
        assert L.inflateInit2_(C.byref(s), wbits, b"1.3.1.1-motley", C.sizeof(ZStream)) == 0
        inbuf = C.create_string_buffer(z, len(z))
        outbuf = C.create_string_buffer(7000)
        got, pos, rc = bytearray(), 0, 0
        for _ in range(100000):
            if s.avail_in == 0 and pos < len(z):
                take = min(25000, len(z) - pos)
                s.next_in, s.avail_in = C.addressof(inbuf) + pos, take
                pos += take
            s.next_out, s.avail_out = C.addressof(outbuf), 7000
            rc = L.inflate(C.byref(s), 0)
            got += outbuf.raw[: 7000 - s.avail_out]
            if rc != 0:
                break
        assert rc == 1 and bytes(got) == data, (wrap, wbits, rc)
        assert s.total_in == len(z) - 3 and s.total_out == len(data)
        assert L.inflateEnd(C.byref(s)) == 0
    bad = bytearray(oracle.compress(data, 6)[1])
    bad[len(bad) // 2] ^= 0x40
    s = ZStream()
    assert L.inflateInit2_(C.byref(s), 15, b"1.3.1.1-motley", C.sizeof(ZStream)) == 0
    inbuf = C.create_string_buffer(bytes(bad), len(bad))
    outbuf = C.create_string_buffer(len(data) + 100)
    s.next_in, s.avail_in = C.addressof(inbuf), len(bad)
    s.next_out, s.avail_out = C.addressof(outbuf), len(data) + 100
    rc = L.inflate(C.byref(s), 4)
    want = oracle.uncompress(bytes(bad), len(data) + 100)
    assert rc == -3 and outbuf.raw[: s.total_out] == want[1]
    L.inflateEnd(C.byref(s))


def test_inflate_device_api(zg, oracle):
    """zgpu_inflate_batch_dev on HBM-resident streams (unaligned offsets)."""
    import torch
    bufs = [datagen.make("mix", n, 70 + n % 13) for n in (0, 1, 1000, 65536, 300001)]
    zs = [oracle.compress(b, 6)[1] for b in bufs]
    blob, offs = bytearray(), []
    for z in zs:
        blob += b"\x00" * 3
        offs.append(len(blob))
        blob += z
    dev = torch.device("cuda:0")
    src = torch.tensor(list(blob), dtype=torch.uint8, device=dev)
    src_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    src_len = torch.tensor([len(z) for z in zs], dtype=torch.int64, device=dev)
    caps = [len(b) + 1 for b in bufs]
    doff, acc = [], 5
    for c in caps:
        doff.append(acc)
        acc += c + 7
    dst = torch.zeros(acc, dtype=torch.uint8, device=dev)
    dst_off = torch.tensor(doff, dtype=torch.int64, device=dev)
    dst_cap = torch.tensor(caps, dtype=torch.int64, device=dev)
    dst_len = torch.zeros(len(bufs), dtype=torch.int64, device=dev)
    used = torch.zeros(len(bufs), dtype=torch.int64, device=dev)
    status = torch.zeros(len(bufs), dtype=torch.int32, device=dev)
    zg.inflate_batch_dev(src, src_off, src_len, dst, dst_off, dst_cap, dst_len, status, src_used=used)
    torch.cuda.synchronize()
    host = dst.cpu().numpy().tobytes()
    for i, b in enumerate(bufs):
        assert int(status[i]) == 0 and int(dst_len[i]) == len(b) and int(used[i]) == len(zs[i])
        assert host[doff[i]: doff[i] + len(b)] == b


def _stream_inflate(L, z, chunk, outsz, wbits):
    s = ZStream()
    assert L.inflateInit2_(C.byref(s), wbits, b"1.3.1.1-motley", C.sizeof(ZStream)) == 0
    inbuf = C.create_string_buffer(bytes(z), len(z))
    outbuf = C.create_string_buffer(outsz)
    got, pos, rc, calls = bytearray(), 0, 0, 0
    while True:
        if s.avail_in == 0 and pos < len(z):
            take = min(chunk, len(z) - pos)
            s.next_in, s.avail_in = C.addressof(inbuf) + pos, take
            pos += take
        s.next_out, s.avail_out = C.addressof(outbuf), outsz
        rc = L.inflate(C.byref(s), 0)
        calls += 1
        got += outbuf.raw[: outsz - s.avail_out]
        if rc != 0 or (pos == len(z) and s.avail_in == 0 and s.avail_out == outsz):
            break
    tin, tout = s.total_in, s.total_out
    L.inflateEnd(C.byref(s))
    return rc, bytes(got), tin, tout, calls


@pytest.mark.gpu
def test_inflate_stream_resumes_linear(zg, oracle):
    """A zpipe-style loop feeding a multi-MiB stream 4 KiB at a time: each call
    resumes at the last complete block (the window carried), so the ~1500
    calls cost linear work; output, totals and Z_STREAM_END as zlib's."""
    L = zg.load()
    L.inflateInit2_.restype = C.c_int
    L.inflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_char_p, C.c_int]
    L.inflate.restype = C.c_int
    L.inflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.inflateEnd.argtypes = [C.POINTER(ZStream)]
    data = datagen.make("mix", 6 << 20, 11)
    for level, wrap, wbits in ((6, 1, 15), (1, 2, 31), (9, 0, -15), (0, 1, 15)):
        z = oracle.compress(data, level, wrap=wrap)[1]
        rc, got, tin, tout, calls = _stream_inflate(L, z + b"tail", 4096, 65536, wbits)
        assert rc == 1 and got == data, (level, wrap, rc, len(got))
        assert tin == len(z) and tout == len(data) and calls > len(z) // 4096


@pytest.mark.gpu
def test_inflate_stream_resume_bad_trailer(zg, oracle):
    """Streaming, resumed decode: a damaged Adler-32 / CRC-32 / ISIZE trailer
    is Z_DATA_ERROR after all the data, as inflate.c:1183-1221."""
    L = zg.load()
    L.inflateInit2_.restype = C.c_int
    L.inflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_char_p, C.c_int]
    L.inflate.restype = C.c_int
    L.inflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.inflateEnd.argtypes = [C.POINTER(ZStream)]
    data = datagen.make("text", 1 << 20, 5)
    for wrap, wbits, k in ((1, 15, -1), (2, 31, -5), (2, 31, -1)):
        z = bytearray(oracle.compress(data, 6, wrap=wrap)[1])
        z[k] ^= 0x01
        rc, got, _, _, _ = _stream_inflate(L, z, 8192, 1 << 20, wbits)
        assert rc == -3 and got == data, (wrap, k, rc)
