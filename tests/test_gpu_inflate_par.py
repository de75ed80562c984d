"""The block-parallel decode of a lone stream (zgpu_api.cpp inflate_par,
zgpu_inflate.hip k_infl_scan1/2, k_infl_sym, k_infl_resolve).  A lone stream
of at least 32 KiB (compressed) takes it; the result must be uncompress2's: the bytes,
Z_OK and the input consumed for valid streams of every level, strategy and
wrapper (fixed-code and stored blocks, flushes, trailing bytes), and the
sequential path's exact answer wherever the parallel one gives up (damage,
truncation, a short output buffer).  Expected values come from the system
zlib of the machine the test runs on (uncompress2 through ctypes)."""
import ctypes
import ctypes.util
import json
import os
import subprocess
import sys
import zlib as pyzlib

import pytest

import datagen

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _stream(data, level, strategy=0, wbits=15, flushes=0, seed=0):
    c = pyzlib.compressobj(level, pyzlib.DEFLATED, wbits, 8, strategy)
    if not flushes:
        return c.compress(data) + c.flush()
    out, step = [], max(1, len(data) // (flushes + 1))
    for i in range(0, len(data), step):
        out.append(c.compress(data[i:i + step]))
        out.append(c.flush((pyzlib.Z_SYNC_FLUSH, pyzlib.Z_FULL_FLUSH, pyzlib.Z_BLOCK)[(i // step + seed) % 3]))
    out.append(c.flush())
    return b"".join(out)


def _sys_uncompress2(z, cap):
    libz = ctypes.CDLL(ctypes.util.find_library("z") or "libz.so.1")
    libz.uncompress2.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulong), ctypes.c_char_p,
                                 ctypes.POINTER(ctypes.c_ulong)]
    out = ctypes.create_string_buffer(max(cap, 1))
    dl, sl = ctypes.c_ulong(cap), ctypes.c_ulong(len(z))
    rc = libz.uncompress2(out, ctypes.byref(dl), z, ctypes.byref(sl))
    return rc, out.raw[:dl.value], sl.value


def _valid_cases(small):
    mk = datagen.make
    if small:
        sizes = [0, 1, 100, 5000, 70000, 300000]
    else:
        sizes = [(1 << 20) + 7, 3 << 20, (8 << 20) + 1]
    cases = []
    for i, n in enumerate(sizes):
        data = b"".join(mk(k, n // 3 + 1, 500 + i) for k in ("text", "mix", "runs"))[:n]
        for level, strategy in ((6, 0), (1, 0), (9, 0), (0, 0), (6, 4), (6, 2), (4, 3), (7, 1)):
            for wb in (15, 31, -15):
                cases.append((f"n{n}-L{level}-s{strategy}-w{wb}", data, _stream(data, level, strategy, wb), wb))
        cases.append((f"n{n}-flushes", data, _stream(data, 6, 0, 15, flushes=7, seed=i), 15))
    return cases


def _par_count(zg):
    f = zg.load().zgpu_debug_par_inflates
    f.restype = ctypes.c_uint64
    return f()


def _check(zg, cases):
    bad = []
    for name, data, z, wb in cases:
        wrap = 0 if wb < 0 else (2 if wb > 15 else 1)
        before = _par_count(zg)
        (st, out, used), = zg.uncompress_batch([z], [len(data) + 10], wrap)
        if st != 0 or out != data or used != len(z):
            bad.append((name, st, len(out), used, len(z)))
        # the parallel decode took it (not a stream under 64 bytes, nor a Z_FIXED one of many blocks: the
        # scan finds no fixed-code header, and after 16 of them the sequential decode is the faster one)
        if _par_count(zg) != before + 1 and len(z) >= 64 and not ("-s4-" in name and len(data) > 100000):
            bad.append((name, "not on the parallel path"))
        if wrap == 1:
            zt = z + b"trailing bytes"
            got = zg.uncompress2(zt, len(data))
            want = _sys_uncompress2(zt, len(data))
            if got != want:
                bad.append((name + "-uncompress2", got[0], len(got[1]), got[2], want[0], len(want[1]), want[2]))
    return bad


def test_lone_large_streams(zg):
    bad = _check(zg, [c for c in _valid_cases(False) if len(c[2]) >= 32 * 1024])
    assert not bad, bad[:5]


def test_lone_streams_that_fall_back(zg):
    """Damage, truncation and short output buffers: uncompress2's answer
    (status, bytes written, input used) exactly, through the sequential path
    the parallel decode hands over to."""
    data = b"".join(datagen.make(k, 1 << 20, 601) for k in ("text", "mix"))
    z = _stream(data, 6)
    cases = []
    for at in (len(z) // 3, len(z) // 2, len(z) - 3):        # a flipped byte: data error or check failure
        zz = bytearray(z)
        zz[at] ^= 0x55
        cases.append((bytes(zz), len(data)))
    cases += [(z[:len(z) // 2], len(data)), (z[:-2], len(data)), (z, len(data) - 1000), (z, 100)]
    for zz, cap in cases:
        got = zg.uncompress2(zz, cap)
        want = _sys_uncompress2(zz, cap)
        assert got == want, (len(zz), cap, got[0], len(got[1]), got[2], want[0], len(want[1]), want[2])


_CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
import zgpu
assert zgpu.load().zgpu_init() == 0
import test_gpu_inflate_par as T
print("BAD " + json.dumps(T._check(zgpu, T._valid_cases(True))))
"""


def test_small_streams_on_the_parallel_path(zg):
    """Small streams (empty, one block, a few blocks) with the parallel decode
    forced on (ZGPU_PAR_INFLATE_MIN=0), in a child process since the library
    reads the setting once."""
    env = dict(os.environ, ZGPU_PAR_INFLATE_MIN="0",
               PYTHONPATH=os.pathsep.join([os.path.join(os.path.dirname(HERE), "zlib.wasm_amd"), HERE,
                                           os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", _CHILD, HERE], env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("BAD ")][-1]
    assert json.loads(line[4:]) == [], line
