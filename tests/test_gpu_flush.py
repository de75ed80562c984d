"""deflate() with flush calls (Z_PARTIAL_FLUSH, Z_SYNC_FLUSH, Z_FULL_FLUSH,
Z_BLOCK, refused repeats, then Z_FINISH) through libzgpu's z_stream API on the
GPU, against

  * tests/golden/flush_golden.json -- call sequences run through the compiled
    reference (deflate.c:763-1265): the status of every call, the output length
    after every call and the sha256 of the whole stream;
  * the oracle's zo_deflate_flushes (oracle/zoracle.c) on further random call
    sequences, and on the stream prefix each flush call hands out.

Bit-exact, level 0 included (tests/golden/stored_golden.json)."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import datagen
from zhelpers import ZStream, flush_events

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
VERSION = b"1.3.1.1-motley"


def _lib(zg):
    L = zg.load()
    L.deflateInit2_.restype = C.c_int
    L.deflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_char_p, C.c_int]
    L.deflate.restype = C.c_int
    L.deflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.deflateEnd.restype = C.c_int
    L.deflateEnd.argtypes = [C.POINTER(ZStream)]
    return L


def replay(L, data, calls, level, wbits, strategy, chunk=None):
    """Run a call sequence [(input_len, flush)]; with ``chunk`` every call is
    zpipe's loop (repeat while avail_out == 0 with a fresh ``chunk``-byte
    buffer).  Returns (status per call, total_out after each call, stream)."""
    data = bytes(data)
    s = ZStream()
    assert L.deflateInit2_(C.byref(s), level, 8, wbits, 8, strategy, VERSION, C.sizeof(ZStream)) == 0
    inbuf = C.create_string_buffer(data, max(len(data), 1))
    cap = chunk or (2 * len(data) + 1024 + 16 * len(calls))
    outbuf = C.create_string_buffer(cap)
    out, sts, lens, pos = bytearray(), [], [], 0
    for take, flush in calls:
        s.next_in = C.addressof(inbuf) + pos
        s.avail_in = take
        pos += take
        rounds = 0
        while True:
            s.next_out, s.avail_out = C.addressof(outbuf), cap
            rc = L.deflate(C.byref(s), flush)
            out += outbuf.raw[:cap - s.avail_out]
            rounds += 1
            assert rounds < 1_000_000
            if chunk is None or s.avail_out != 0:
                break
        sts.append(rc)
        lens.append(s.total_out)
        assert s.avail_in == 0
    assert L.deflateEnd(C.byref(s)) == 0
    return sts, lens, bytes(out)


@pytest.fixture(scope="module")
def flush_golden():
    with open(os.path.join(HERE, "golden", "flush_golden.json")) as f:
        return json.load(f)["cases"]


def _case_input(c):
    data = datagen.make(c["kind"], c["n"], c["seed"])
    assert hashlib.sha256(bytes(data)).hexdigest() == c["input_sha256"]
    return data


def test_flush_golden_streams(zg, flush_golden):
    L = _lib(zg)
    for c in flush_golden:
        data = _case_input(c)
        sts, lens, whole = replay(L, data, c["calls"], c["level"], c["wbits"], c["strategy"])
        tag = (c["kind"], c["n"], c["level"], c["strategy"], c["wbits"])
        assert sts == c["status"], tag
        # output after every call, Z_NO_FLUSH calls included
        for i, ((take, flush), got, want) in enumerate(zip(c["calls"], lens, c["out_len"])):
            assert got == want, (tag, i, take, flush)
        assert len(whole) == c["len"], tag
        assert hashlib.sha256(whole).hexdigest() == c["sha256"], tag


def _plan(rng, n):
    calls, pos = [], 0
    while pos < n:
        take = int(min(n - pos, rng.choice([0, 1, 2, 3, 5, 250, 3000, 33000, 66000, 140000])))
        calls.append((take, int(rng.choice([0, 1, 2, 2, 3, 5]))))
        pos += take
        if rng.random() < 0.2:
            calls.append((0, int(rng.choice([1, 2, 3, 5]))))
    calls.append((0, 4))
    return calls


def test_flush_random_vs_oracle(zg, oracle):
    """Random call sequences; every flush call's output is the oracle's stream
    prefix (open end: complete bytes, no trailer), the end is its stream."""
    L = _lib(zg)
    rng = np.random.default_rng(int(os.environ.get("ZGPU_FLUSH_SEED", "31")))
    kinds = ["text", "mix", "runs", "random", "records", "markup"]
    for t in range(int(os.environ.get("ZGPU_FLUSH_CASES", "24"))):
        n = int(rng.choice([0, 2, 700, 50000, 200000, 600000]))
        data = datagen.make(kinds[t % len(kinds)], n, 900 + t)
        level = 1 + t % 9
        strategy = int(rng.choice([0, 0, 1, 2, 3, 4]))
        wbits = int(rng.choice([15, -15, 31]))
        wrap = {15: 1, -15: 0, 31: 2}[wbits]
        calls = _plan(rng, n)
        sts, lens, whole = replay(L, data, calls, level, wbits, strategy)
        ev = flush_events(calls)
        rc, want = oracle.deflate_flushes(data, ev, level, wrap, strategy, finish=True)
        tag = (t, n, level, strategy, wbits)
        assert rc == 0 and whole == want, tag
        assert sts[-1] == 1, tag
        pos = 0
        for i, (take, flush) in enumerate(calls[:-1]):
            pos += take
            if flush == 0 or sts[i] != 0:
                continue
            rc, pre = oracle.deflate_flushes(data[:pos], flush_events(calls[:i + 1]), level, wrap, strategy,
                                             finish=False)
            assert rc == 0 and lens[i] == len(pre) and whole[:len(pre)] == pre, (tag, i)


@pytest.mark.parametrize("level,strategy", [(6, 0), (9, 1), (4, 3), (2, 2), (1, 0), (3, 4)])
def test_flush_many_calls(zg, oracle, level, strategy):
    """Hundreds of flush calls on a multi-MiB stream: every job after the
    first resumes at the last flush (levels 1..3 with their hash chains carried
    over), so the work stays linear; the stream is the oracle's."""
    import time
    L = _lib(zg)
    n = 3 << 20
    data = datagen.make("mix", n, 77 + level)
    rng = np.random.default_rng(level)
    calls, pos = [], 0
    while pos < n:
        take = int(min(n - pos, rng.integers(1, 12000)))
        calls.append((take, int(rng.choice([0, 1, 2, 2, 5]))))
        pos += take
    calls.append((0, 4))
    t0 = time.time()
    sts, _, whole = replay(L, data, calls, level, 15, strategy)
    took = time.time() - t0
    rc, want = oracle.deflate_flushes(data, flush_events(calls), level, 1, strategy, finish=True)
    assert rc == 0 and whole == want, (level, strategy, len(calls))
    assert sts[-1] == 1
    assert took < 60, took


def test_flush_small_output_buffers(zg, flush_golden):
    """zpipe-style loops with small output buffers: a flush call that runs
    out of output before its marker completes it on the repeat call (no second
    marker); the stream is the golden one whenever no marker ends exactly at the
    end of a buffer (zlib.h: avail_out greater than six)."""
    L = _lib(zg)
    done = 0
    for c in flush_golden:
        if c["n"] < 1000 or done >= 12:
            continue
        data = _case_input(c)
        for chunk in (997, 16384):
            _, _, whole = replay(L, data, c["calls"], c["level"], c["wbits"], c["strategy"], chunk=chunk)
            _, _, ref = replay(L, data, c["calls"], c["level"], c["wbits"], c["strategy"])
            if whole != ref:
                # a repeated marker: the stream must still decode to the input
                import zlib as pyzlib
                wb = {15: 15, -15: -15, 31: 31}[c["wbits"]]
                assert pyzlib.decompress(whole, wb) == bytes(data)
            else:
                assert hashlib.sha256(whole).hexdigest() == c["sha256"]
        done += 1
    assert done > 0


def test_stored_golden_streams(zg):
    """Level 0 over deflate() calls (deflate_stored, deflate.c:1635-1815):
    status and total output after EVERY call (level-0 output is not deferred)
    and the stream, against tests/golden/stored_golden.json."""
    L = _lib(zg)
    with open(os.path.join(HERE, "golden", "stored_golden.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        data = _case_input(c)
        sts, lens, whole = replay(L, data, c["calls"], 0, c["wbits"], 0)
        tag = (c["kind"], c["n"], c["wbits"], c["seed"])
        assert sts == c["status"], tag
        assert lens == c["out_len"], tag
        assert len(whole) == c["len"] and hashlib.sha256(whole).hexdigest() == c["sha256"], tag


def test_stored_random_vs_oracle(zg, oracle):
    L = _lib(zg)
    rng = np.random.default_rng(int(os.environ.get("ZGPU_STORED_SEED", "9")))
    for t in range(16):
        n = int(rng.choice([0, 3, 40000, 70000, 300000]))
        data = bytes(datagen.make(["text", "random", "mix"][t % 3], n, 40 + t))
        calls, pos = [], 0
        while pos < n:
            take = int(min(n - pos, rng.choice([0, 1, 1000, 32767, 32768, 65535, 65536, 100000])))
            calls.append((take, int(rng.choice([0, 0, 1, 2, 3, 5]))))
            pos += take
        calls.append((0, 4))
        wbits = int(rng.choice([15, -15, 31]))
        sts, lens, whole = replay(L, data, calls, 0, wbits, 0)
        rc, osts, olens, want = oracle.deflate_stored_calls(data, calls, {15: 1, -15: 0, 31: 2}[wbits])
        assert rc == 0 and sts == osts and lens == olens and whole == want, (t, n, wbits)


def test_flush_errors(zg):
    L = _lib(zg)
    buf = C.create_string_buffer(b"abc", 3)
    out = C.create_string_buffer(64)
    # a repeated flush with no new input is refused (deflate.c:1002-1005)
    s = ZStream()
    assert L.deflateInit2_(C.byref(s), 6, 8, 15, 8, 0, VERSION, C.sizeof(ZStream)) == 0
    s.next_in, s.avail_in = C.addressof(buf), 3
    s.next_out, s.avail_out = C.addressof(out), 64
    assert L.deflate(C.byref(s), 2) == 0
    n1 = s.total_out
    s.next_out, s.avail_out = C.addressof(out), 64
    assert L.deflate(C.byref(s), 2) == -5
    assert L.deflate(C.byref(s), 1) == -5          # lower rank
    assert L.deflate(C.byref(s), 3) == 0           # higher rank: acted on
    assert s.total_out == n1 + 5
    assert L.deflateEnd(C.byref(s)) == 0


def test_wasm_stream_api_flushes(zg, oracle):
    """The WASM front end's streaming names (src/wasm_module.c:168-215) pass
    the flush value through to deflate(): flush calls included, the stream is
    the oracle's."""
    L = zg.load()
    L.zlib_deflate_init.restype = C.c_void_p
    L.zlib_deflate_init.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
    L.zlib_deflate_process.restype = C.c_int
    L.zlib_deflate_process.argtypes = [C.c_void_p, C.c_void_p, C.c_uint, C.c_void_p, C.c_uint, C.c_int]
    L.zlib_deflate_end.argtypes = [C.c_void_p]
    L.zlib_stream_total_out.restype = C.c_ulong
    L.zlib_stream_total_out.argtypes = [C.c_void_p]
    data = bytes(datagen.make("text", 200000, 5))
    calls = [(50000, 2), (0, 1), (70000, 0), (30000, 5), (50000, 3), (0, 2), (0, 4)]
    h = L.zlib_deflate_init(6, 15, 8, 0)
    assert h
    inbuf = C.create_string_buffer(data, len(data))
    out = bytearray()
    obuf = C.create_string_buffer(1 << 20)
    pos = 0
    for take, flush in calls:
        rc = L.zlib_deflate_process(h, C.addressof(inbuf) + pos, take, obuf, len(obuf), flush)
        pos += take
        assert rc in (0, 1, -5), (take, flush, rc)
        out += obuf.raw[:L.zlib_stream_total_out(h) - len(out)]   # each call writes from the buffer start
    L.zlib_deflate_end(C.c_void_p(h))
    rc, want = oracle.deflate_flushes(data, flush_events(calls), 6, 1, 0, finish=True)
    assert rc == 0 and bytes(out) == want


def test_deflate_reset_copy_pending(zg, oracle):
    L = _lib(zg)
    L.deflateReset.argtypes = [C.POINTER(ZStream)]
    L.deflateCopy.argtypes = [C.POINTER(ZStream), C.POINTER(ZStream)]
    L.deflatePending.argtypes = [C.POINTER(ZStream), C.POINTER(C.c_uint), C.POINTER(C.c_int)]
    data = bytes(datagen.make("mix", 150000, 8))
    inbuf = C.create_string_buffer(data, len(data))
    cap = 2 * len(data) + 4096

    def run(s, start, calls):
        out, pos = bytearray(), start
        buf = C.create_string_buffer(cap)
        for take, flush in calls:
            s.next_in, s.avail_in = C.addressof(inbuf) + pos, take
            s.next_out, s.avail_out = C.addressof(buf), cap
            L.deflate(C.byref(s), flush)
            out += buf.raw[:cap - s.avail_out]
            pos += take
        return bytes(out)

    s = ZStream()
    assert L.deflateInit2_(C.byref(s), 6, 8, 15, 8, 0, VERSION, C.sizeof(ZStream)) == 0
    head = run(s, 0, [(60000, 1)])                       # Z_PARTIAL_FLUSH: a partial byte stays
    pend, bits = C.c_uint(99), C.c_int(99)
    assert L.deflatePending(C.byref(s), C.byref(pend), C.byref(bits)) == 0
    assert pend.value == 0 and 0 <= bits.value < 8
    t = ZStream()
    assert L.deflateCopy(C.byref(t), C.byref(s)) == 0
    tail_s = run(s, 60000, [(90000, 4)])
    tail_t = run(t, 60000, [(90000, 4)])
    assert tail_s == tail_t
    rc, want = oracle.deflate_flushes(data, [(60000, 1)], 6, 1, 0, finish=True)
    assert rc == 0 and head + tail_s == want
    assert L.deflateEnd(C.byref(t)) == 0
    # deflateReset: the same stream object compresses afresh
    assert L.deflateReset(C.byref(s)) == 0
    assert s.total_in == 0 and s.total_out == 0
    again = run(s, 0, [(150000, 4)])
    assert again == oracle.compress(data, 6)[1]
    assert L.deflateEnd(C.byref(s)) == 0


def test_inflate_sync_flushed_stream_progressively(zg, oracle):
    """An open, sync-flushed stream (what a connection carries): inflate() fed
    up to each flush point hands out all the data before it (zlib.h,
    Z_SYNC_FLUSH), without waiting for the end of the stream."""
    L = zg.load()
    L.inflateInit2_.restype = C.c_int
    L.inflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_char_p, C.c_int]
    L.inflate.restype = C.c_int
    L.inflate.argtypes = [C.POINTER(ZStream), C.c_int]
    L.inflateEnd.argtypes = [C.POINTER(ZStream)]
    data = bytes(datagen.make("mix", 400000, 21))
    cuts = [0, 1000, 5000, 70000, 70001, 200000, 399990, 400000]
    for level in (0, 1, 6, 9):
        events = [(c, 2) for c in cuts[1:]]
        if level:
            rc, stream = oracle.deflate_flushes(data, events, level, 1, 0, finish=False)
            # where each flush call's output ends: the stream of its prefix
            ends = [len(oracle.deflate_flushes(data[:c], events[:i + 1], level, 1, 0, finish=False)[1])
                    for i, c in enumerate(cuts[1:])]
        else:
            rc, _, ends, stream = oracle.deflate_stored_calls(
                data, [(b - a, 2) for a, b in zip(cuts, cuts[1:])], 1)
        assert rc == 0
        s = ZStream()
        assert L.inflateInit2_(C.byref(s), 15, VERSION, C.sizeof(ZStream)) == 0
        inbuf = C.create_string_buffer(stream, len(stream))
        out = C.create_string_buffer(len(data) + 64)
        s.next_out, s.avail_out = C.addressof(out), len(data) + 64
        prev = 0
        for c, e in zip(cuts[1:], ends):
            s.next_in, s.avail_in = C.addressof(inbuf) + prev, e - prev
            rc = L.inflate(C.byref(s), 2)
            assert rc == 0, (level, c, rc)
            assert s.total_out == c and out.raw[:c] == data[:c], (level, c, s.total_out)
            prev = e
        assert L.inflateEnd(C.byref(s)) == 0
