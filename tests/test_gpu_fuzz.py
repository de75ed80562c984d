"""Randomized differential sessions of the streaming deflate(): seeded random
z_stream call sequences (levels 1-9, strategies 0-3, zlib / raw / gzip
wrappers, windowBits 9..15, memLevel 1..9, every flush kind, input chunks of
0 bytes to 200 KB, output buffers down to 1 byte, preset dictionaries) replayed
on libzgpu.so and on the system zlib of the machine the test runs on, call by
call: every return code and the whole stream must be equal.

The system zlib (1.2.11 on the GPU image) is upstream zlib, whose deflate
levels 1-9 produce the reference's (1.3.1.1-motley) bytes (BASELINE.md 3.1,
the bench's byte-identical CPU baseline).  Left out, because they changed
between those versions: level 0 (deflate_stored's 1.2.12 fixes), Z_FIXED
(1.3's _tr_flush_block weighs a stored block against the fixed-code length),
deflateParams (1.2.12 moved its flush condition from high_water to
last_flush) and deflatePrime (its Z_BUF_ERROR threshold follows the symbol
buffer layout); the reference's own sessions pin those
(tests/golden/zstream_golden.json, api_golden.json)."""
import ctypes
import ctypes.util
import random

import numpy as np
import pytest

import datagen
from zhelpers import run_zsession

pytestmark = pytest.mark.gpu

KINDS = ("text", "mix", "runs", "records", "markup", "random")
FLUSHES = (0, 0, 0, 1, 2, 3, 5)           # Z_NO_FLUSH (more often), PARTIAL, SYNC, FULL, BLOCK


def _session(rng):
    level = rng.randint(1, 9)
    strategy = rng.choice((0, 0, 0, 1, 2, 3))
    wb = rng.choice((15, 15, 9, 10, 12, 13, 14))
    wrap = rng.choice(("zlib", "raw", "gzip"))
    wbits = {"zlib": wb, "raw": -wb, "gzip": wb + 16}[wrap]
    mem = rng.choice((8, 8, 1, 2, 5, 7, 9))
    ops = [["init", level, wbits, mem, strategy]]
    if wrap != "gzip" and rng.random() < 0.15:
        ops.append(["dict", datagen.make("text", rng.randint(1, 40000), rng.randint(0, 999))])
    total = rng.randint(0, 600000)
    data = b"".join(datagen.make(rng.choice(KINDS), max(1, total // 3), rng.randint(0, 10 ** 6))
                    for _ in range(3))[:total]
    pos, ncall = 0, rng.randint(1, 10)
    for i in range(ncall):
        last = i == ncall - 1
        n = len(data) - pos if last else min(len(data) - pos, rng.choice((0, 1, 2, 100, 5000, 70000, 200000)))
        op = ["deflate", data[pos:pos + n], 4 if last else rng.choice(FLUSHES)]
        if rng.random() < 0.25:                  # small output buffers, zpipe-style loop
            op.append(rng.choice((1, 7, 64, 1000, 16384)) if n + len(data) < 20000 else
                      rng.choice((1000, 16384, 65536)))
        ops.append(op)
        pos += n
    return ops


def _system_zlib():
    name = ctypes.util.find_library("z") or "libz.so.1"
    return ctypes.CDLL(name)


def _pending_session(rng):
    """deflate() calls that end with output still pending -- a flush that ran
    out of output space -- followed by a call that brings MORE input (zlib.h
    asks for the same flush again with no new input; zlib's deflate carries
    on: the flush already happened, its bytes wait in pending), then the rest
    of the session as usual."""
    level = rng.randint(1, 9)
    ops = [["init", level, rng.choice((15, -15, 31)), 8, rng.choice((0, 0, 1))]]
    data = b"".join(datagen.make(rng.choice(KINDS), 60000, rng.randint(0, 10 ** 6)) for _ in range(4))
    pos = 0
    for _ in range(rng.randint(2, 6)):
        n = rng.choice((100, 5000, 30000))
        ops.append(["deflate1", data[pos:pos + n], rng.choice((1, 2, 3, 5, 0)), rng.choice((1, 10, 200, 3000))])
        pos += n
    ops.append(["deflate", data[pos:], 4])
    return ops


@pytest.mark.parametrize("block", range(4))
def test_random_pending_flush_sessions_vs_system_zlib(zg, block):
    """Every single call's status / avail_in / avail_out and the stream.
    Seed block 1 holds session 21: a gzip stream whose first Z_BLOCK call
    gets exactly the 10 header bytes of output space (see
    test_first_call_output_space_is_the_header)."""
    libz = _system_zlib()
    L = zg.load()
    rng = random.Random(3131 + block)
    bad = []
    for k in range(30):
        ops = _pending_session(rng)
        rz, z = run_zsession(libz, ops)
        rg, g = run_zsession(L, ops)
        if rz != rg or z != g:
            bad.append((k, [o[:1] + ([len(o[1])] if o[0].startswith("deflate") else list(o[1:2])) + list(o[2:])
                            for o in ops], rz, rg, len(z), len(g)))
    assert not bad, bad[:2]


@pytest.mark.parametrize("block", range(4))
def test_random_deflate_sessions_vs_system_zlib(zg, block):
    libz = _system_zlib()
    L = zg.load()
    rng = random.Random(20261017 + block)
    bad = []
    for k in range(30):
        ops = _session(rng)
        rz, z = run_zsession(libz, ops)
        rg, g = run_zsession(L, ops)
        if rz != rg or z != g:
            bad.append((k, [o[:1] + ([len(o[1])] if o[0] in ("deflate", "dict") else list(o[1:2])) + list(o[2:])
                            for o in ops], rz, rg, len(z), len(g)))
    assert not bad, bad[:3]


def _istream(rng, libz, small_out=False, flushes=(0, 0, 2, 5)):
    """A stream from system zlib (any level and strategy, flushes inside) and
    a random inflate call sequence over it: input fed in random pieces, calls
    with Z_NO_FLUSH / Z_SYNC_FLUSH / Z_BLOCK, sometimes cut short (a truncated
    stream).  Output space per call: 1 MiB, or (small_out) 1 byte to 1 MiB."""
    level = rng.randint(0, 9)
    strategy = rng.choice((0, 0, 1, 2, 3, 4))
    wb = rng.choice((15, 15, 9, 11, 14))
    wrap = rng.choice(("zlib", "raw", "gzip"))
    wbits = {"zlib": wb, "raw": -wb, "gzip": wb + 16}[wrap]
    total = rng.randint(0, 400000)
    data = b"".join(datagen.make(rng.choice(KINDS), max(1, total // 2), rng.randint(0, 10 ** 6))
                    for _ in range(2))[:total]
    cuts = sorted(rng.randint(0, len(data)) for _ in range(rng.randint(0, 4)))
    zops, pos = [["init", level, wbits, 8, strategy]], 0
    for c in cuts + [len(data)]:
        zops.append(["deflate", data[pos:c], 4 if c == len(data) else rng.choice((0, 1, 2, 3, 5))])
        pos = c
    _, z = run_zsession(libz, zops)
    if rng.random() < 0.15:
        z = z[:rng.randint(0, len(z))]
    dec = {"zlib": rng.choice((wb, 15, 47)), "raw": -15 if rng.random() < 0.5 else -wb,
           "gzip": rng.choice((wb + 16, 31, 47))}[wrap]
    ops = [["init", dec]]
    if wrap == "gzip" and rng.random() < 0.5:
        ops.append(["header", rng.choice((0, 4, 64)), rng.choice((0, 8, 256)), rng.choice((0, 8, 256))])
    for _ in range(rng.randint(1, 25)):
        ops.append(["feed", rng.choice((1, 3, 100, 4096, 70000, 1 << 30))])
        ops.append(["inflate", rng.choice(flushes),
                    rng.choice((1, 100, 5000, 1 << 16, 1 << 20)) if small_out else 1 << 20])
    ops += [["feed", 1 << 30], ["loop", 0, 1 << 20]]
    return z, ops


@pytest.mark.parametrize("block", range(3))
def test_random_inflate_sessions_vs_system_zlib(zg, block):
    """Every call's status, avail_in, total_in, total_out (and Z_BLOCK's
    data_type), the output and the gzip header fields."""
    from zhelpers import run_iops
    libz = _system_zlib()
    L = zg.load()
    rng = random.Random(4242 + block)
    bad = []
    for k in range(30):
        z, ops = _istream(rng, libz)
        rz = run_iops(libz, z, ops)
        rg = run_iops(L, z, ops)
        if rz != rg:
            bad.append((k, len(z), ops[:3], rz[0][:6], rg[0][:6]))
    assert not bad, bad[:3]


@pytest.mark.parametrize("block", range(2))
def test_random_inflate_small_output_vs_system_zlib(zg, block):
    """Output space down to 1 byte per call: every call's status, avail_in,
    total_in, total_out (and Z_BLOCK's data_type), the output and the gzip
    header fields equal the reference's.  A call whose output space ends
    before its input stops reading where inflate.c does (inf_leave after the
    symbol it has no room for), so the input handed back and
    presented again matches call by call."""
    from zhelpers import run_iops
    libz = _system_zlib()
    L = zg.load()
    rng = random.Random(7373 + block)
    bad = []
    for k in range(30):
        z, ops = _istream(rng, libz, small_out=True)
        rz = run_iops(libz, z, ops)
        rg = run_iops(L, z, ops)
        if rz != rg:
            first = next((i for i, (a, b) in enumerate(zip(rz[0], rg[0])) if a != b), None)
            bad.append((k, len(z), first, ops[:3], rz[0][first] if first is not None else None,
                        rg[0][first] if first is not None else None))
    assert not bad, bad[:3]


@pytest.mark.parametrize("block", range(2))
def test_random_inflate_trees_vs_system_zlib(zg, block):
    """inflate(Z_TREES) among Z_NO_FLUSH / Z_BLOCK calls, output space down to
    1 byte: every call's status, avail_in, total_in, total_out and data_type
    (+ 256 at a block header's end, inflate.c LEN_ / COPY_), the output and
    the gzip header fields equal the system zlib's."""
    from zhelpers import run_iops
    libz = _system_zlib()
    L = zg.load()
    rng = random.Random(6161 + block)
    bad = []
    for k in range(30):
        z, ops = _istream(rng, libz, small_out=True, flushes=(0, 5, 6, 6))
        rz = run_iops(libz, z, ops)
        rg = run_iops(L, z, ops)
        if rz != rg:
            first = next((i for i, (a, b) in enumerate(zip(rz[0], rg[0])) if a != b), None)
            bad.append((k, len(z), first, ops[:3], rz[0][first] if first is not None else None,
                        rg[0][first] if first is not None else None))
    assert not bad, bad[:3]


@pytest.mark.parametrize("block", range(3))
def test_random_batches_vs_system_zlib(zg, block):
    """The batched hot path (zgpu_compress_batch2) on random batches: 200-1500
    buffers of 0 bytes to 300 KB from every generator kind, one random setting
    per batch (level 1-9, strategy 0-3, zlib / raw / gzip, windowBits 9-15,
    memLevel 1-9); every stream equal to system zlib's (compressobj with the
    same parameters)."""
    import zlib as pyzlib
    rng = random.Random(99 + block)
    for _ in range(4):
        level = rng.randint(1, 9)
        strategy = rng.choice((0, 0, 1, 2, 3))
        wb = rng.choice((15, 15, 9, 12, 14))
        wbits = rng.choice((wb, -wb, wb + 16))
        mem = rng.choice((8, 8, 1, 4, 9))
        count = rng.randint(200, 1500)
        bufs = [datagen.make(rng.choice(KINDS), rng.choice((0, 1, 2, 3, 100, 5000, 70000, 300000,
                                                            rng.randint(0, 300000))), rng.randint(0, 10 ** 6))
                for _ in range(count)]
        got = zg.compress_batch2(bufs, level=level, window_bits=wbits, mem_level=mem, strategy=strategy)
        bad = []
        for i, (b, (st, z)) in enumerate(zip(bufs, got)):
            c = pyzlib.compressobj(level, pyzlib.DEFLATED, wbits, mem, strategy)
            want = c.compress(b) + c.flush()
            if st != 0 or z != want:
                bad.append((i, len(b), st, len(z), len(want)))
        assert not bad, (level, strategy, wbits, mem, count, bad[:5])


def _header_sessions():
    """First calls whose output space is exactly the header (zlib 2 bytes,
    gzip 10): the compress function then runs with no output space."""
    S = []
    data = b"".join(datagen.make(k, 40000, 77) for k in ("text", "mix", "runs"))
    for level in (1, 3, 4, 6, 9):
        for strategy in (0, 2, 3):
            for wbits, hl in ((15, 2), (31, 10)):
                for n in (0, 1, 2, 5000, 100000):
                    for flush in (0, 1, 2, 3, 4, 5):
                        # the calls after the first re-present what it left (zlib.h: next_in / avail_in);
                        # after Z_FINISH only Z_FINISH follows, with no new input (zlib.h)
                        fin = flush == 4
                        S.append([["init", level, wbits, 8, strategy], ["deflate1", data[:n], flush, hl],
                                  ["deflate1", b"", flush, 7, True],
                                  ["deflate", b"" if fin else data[n:n + 3000], 4 if fin else 2, None, True],
                                  ["deflate", b"" if fin else data[n + 3000:n + 9000], 4]])
    return S


def test_first_call_output_space_is_the_header(zg):
    """deflate_slow stops at its first lazy literal and the call's flush never
    happens; one byte, or deflate_fast / _huff / _rle, cut the block without
    the flush's marker; fill_window reads at most window_size bytes (the
    100000-byte calls).  Every call's status / avail_in / avail_out and the
    stream equal system zlib's."""
    libz = _system_zlib()
    L = zg.load()
    bad = []
    for k, ops in enumerate(_header_sessions()):
        rg, g = run_zsession(L, ops)
        rz, z = run_zsession(libz, ops)
        if rz != rg or z != g:
            bad.append((k, ops[0], [len(ops[1][1]), ops[1][2]], rz, rg, len(z), len(g)))
    kinds = sorted({(b[1][1], b[1][4], b[1][2], b[2][0], b[2][1]) for b in bad})
    assert not bad, (len(bad), kinds[:20], bad[:2])


def _dict_header_sessions():
    """First calls after deflateSetDictionary whose output space is exactly the 6-byte zlib header with
    its DICTID.  deflate_slow then stops at its first lazy literal; where the input's first three bytes
    are nowhere in the dictionary its first decision finds no match and the literal comes at the second,
    as with no history.  Under Z_NO_FLUSH the stop's place does not matter (the next call goes on from it
    with the same state), so those are modelled too (round 6), unless the first read could fill a block
    before the first literal.  Those sessions (and every deflate_fast / _huff / _rle one) are compared
    with the system zlib; the others must be refused with strm->msg (returned as `refused`)."""
    rng = np.random.default_rng(606)
    data = b"".join(datagen.make(k, 40000, 78) for k in ("text", "mix", "runs"))
    S = []
    for level in (1, 3, 4, 6, 9):
        for strategy in (0, 1, 2, 3):
            for n in (0, 1, 2, 3, 300, 5000, 100000):
                for flush in (0, 2, 3, 4):
                    for dk in ("absent", "present", "long", "none"):
                        first = data[:3]
                        if dk == "none":                   # no dictionary: the 2-byte header
                            fin = flush == 4
                            S.append((False,
                                      [["init", level, 15, 8, strategy], ["deflate1", data[:n], flush, 2],
                                       ["deflate1", b"", flush, 7, True],
                                       ["deflate", b"" if fin else data[n:n + 3000], 4 if fin else 2, None, True],
                                       ["deflate", b"" if fin else data[n + 3000:n + 9000], 4]]))
                            continue
                        if dk == "present":
                            d = bytes(rng.integers(0, 256, 3000, dtype=np.uint8)) + data[:64]
                        else:
                            size = 40000 if dk == "long" else 3000
                            while True:                # random bytes without the input's first string
                                d = bytes(rng.integers(0, 256, size, dtype=np.uint8))
                                if first not in d:
                                    break
                        fin = flush == 4
                        slow = level >= 4 and strategy in (0, 1)
                        # refused: a flush call (or a first read that could fill a block before its first
                        # literal) whose input's first string is in the dictionary
                        dl = len(d[-32768:])
                        refused = slow and n >= 3 and first in d[-32768:] and (flush != 0 or
                                                                               min(n, 65536 - dl) >= 3 * 16383)
                        S.append((refused, [["init", level, 15, 8, strategy], ["dict", d],
                                            ["deflate1", data[:n], flush, 6],
                                            ["deflate1", b"", flush, 7, True],
                                            ["deflate", b"" if fin else data[n:n + 3000], 4 if fin else 2, None, True],
                                            ["deflate", b"" if fin else data[n + 3000:n + 9000], 4]]))
    return S


def _dict_header_no_flush_sessions():
    """Z_NO_FLUSH first calls after deflateSetDictionary whose output space is exactly the 6-byte header,
    where the dictionary holds the input's start or all of it (the parse may match to the input's end
    before its first literal): lazy levels, Z_FILTERED, memLevels 3 / 8 / 9, input sizes around
    MIN_LOOKAHEAD and up to the first read.  Refused where the first read could fill a block before the
    first literal (3 bytes a symbol for a whole symbol buffer)."""
    data = b"".join(datagen.make(k, 40000, 79) for k in ("text", "runs", "mix"))
    S = []
    for level in (4, 6, 9):
        for strategy in (0, 1):
            for mem in (3, 8, 9):
                for n in (3, 10, 261, 262, 263, 1000, 5000, 20000, 40000):
                    for dk in ("prefix", "whole"):
                        d = data[80000:83000] + (data[:64] if dk == "prefix" else data[:n])
                        dl = min(len(d), 32768)
                        refused = n >= 3 and min(n, 65536 - dl) >= 3 * ((1 << (mem + 6)) - 1)
                        S.append((refused, [["init", level, 15, mem, strategy], ["dict", d],
                                            ["deflate1", data[:n], 0, 6],
                                            ["deflate1", b"", 0, 7, True],
                                            ["deflate", data[n:n + 3000], 2, None, True],
                                            ["deflate", data[n + 3000:n + 9000], 4]]))
    return S


def test_first_call_dictionary_header_no_flush(zg):
    """Round 6: a Z_NO_FLUSH first call whose output space is exactly a preset dictionary's header is
    modelled even when the dictionary holds the input (its first decisions find matches): the call stops
    at its first lazy literal or at need_more, and the next call goes on from there with the same state,
    which is the model's stop at need_more.  Every call's status / avail_in / avail_out and the stream
    equal the system zlib's; the sessions whose first read could fill a block first are refused."""
    libz = _system_zlib()
    L = zg.load()
    bad, n_ref, n_cmp = [], 0, 0
    for k, (refused, ops) in enumerate(_dict_header_no_flush_sessions()):
        rg, g = run_zsession(L, ops)
        if refused:
            if rg[2][0] != -2 or rg[2][2] != 6:
                bad.append(("refusal", k, ops[0], len(ops[2][1]), rg[:3]))
            n_ref += 1
            continue
        rz, z = run_zsession(libz, ops)
        n_cmp += 1
        if rz != rg or z != g:
            bad.append((k, ops[0], len(ops[2][1]), rz, rg, len(z), len(g)))
    assert not bad, (len(bad), bad[:3])
    assert n_cmp > 0 and n_ref > 0


def test_first_call_output_space_is_the_dictionary_header(zg):
    """A first deflate() call whose output space is exactly a preset dictionary's 6-byte header (VERDICT
    r5, zlib.h refusal 4): every call's status / avail_in / avail_out and the stream equal the system
    zlib's where the input's first string is not in the dictionary (and at every level without the lazy
    parse); where it is, the call is refused (Z_STREAM_ERROR with strm->msg) before any output.  The
    sessions without a dictionary, Z_FILTERED among them, found the pause that k_parse_slow's next job
    carried behind its resume point (zgpu_api.cpp drop_pause_behind_resume)."""
    libz = _system_zlib()
    L = zg.load()
    bad, refused_ok = [], 0
    for k, (refused, ops) in enumerate(_dict_header_sessions()):
        rg, g = run_zsession(L, ops)
        if refused:
            # the refused first call: Z_STREAM_ERROR, its output space untouched
            j = 2 if ops[1][0] == "dict" else 1
            if rg[j][0] != -2 or rg[j][2] != ops[j][3]:
                bad.append(("refusal", k, ops[0], len(ops[j][1]), ops[j][2], rg[:j + 1]))
            else:
                refused_ok += 1
            continue
        rz, z = run_zsession(libz, ops)
        if rz != rg or z != g:
            bad.append((k, ops[0], [op[:1] + [len(op[1])] + op[2:4] for op in ops[1:3]], rz, rg, len(z), len(g)))
    assert not bad, (len(bad), bad[:3])
    assert refused_ok > 0
