"""GPU parity of the a18 helper names (src/zlib_simd_optimized.c:27,74,210,296),
called through libzgpu's C ABI, against the oracle's zlib-correct restatements
(oracle/zoracle.c: slide_hash deflate.c:187-209, longest_match
deflate.c:1356-1497).  The reference's own versions are WASM-SIMD code that does
not build here and deviates from zlib where SURVEY a18 says (remainder entries
of slide_hash, chunkmemset's splat for odd distances), so parity is pinned by
the restatement of deflate.c, not by reference outputs."""
import ctypes as C

import numpy as np
import pytest

import datagen

pytestmark = pytest.mark.gpu

U16P = C.POINTER(C.c_uint16)


def _bind(L, prefix):
    f = getattr(L, prefix + "slide_hash" + ("_simd" if prefix == "zlib_" else ""))
    f.restype = None
    f.argtypes = [U16P, U16P, C.c_uint32, C.c_uint32, C.c_uint16 if prefix == "zlib_" else C.c_uint32]
    g = getattr(L, prefix + "compare256" + ("_simd" if prefix == "zlib_" else ""))
    g.restype = C.c_uint32
    g.argtypes = [C.c_char_p, C.c_char_p]
    h = getattr(L, prefix + "longest_match" + ("_simd" if prefix == "zlib_" else ""))
    h.restype = C.c_uint32
    h.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, U16P, C.c_uint32,
                  C.POINTER(C.c_uint32)]
    m = getattr(L, prefix + "chunkmemset" + ("_simd" if prefix == "zlib_" else ""))
    m.restype = None
    m.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.c_uint32]
    return f, g, h, m


@pytest.fixture(scope="module")
def fns(zg, oracle):
    return _bind(zg.load(), "zlib_"), _bind(oracle.L, "zo_")


def test_slide_hash(fns):
    (gs, *_), (os_, *_) = fns
    rng = np.random.default_rng(1)
    for hs, ws, wsize in [(32768, 32768, 32768), (1000, 777, 4096), (17, 0, 512), (0, 33, 32768)]:
        head = rng.integers(0, 65536, hs, dtype=np.uint16)
        prev = rng.integers(0, 65536, ws, dtype=np.uint16)
        a, b = head.copy(), prev.copy()
        gs(a.ctypes.data_as(U16P), b.ctypes.data_as(U16P), hs, ws, wsize)
        os_(head.ctypes.data_as(U16P), prev.ctypes.data_as(U16P), hs, ws, wsize)
        assert np.array_equal(a, head) and np.array_equal(b, prev), (hs, ws, wsize)


def test_compare256(fns):
    (_, gc, *_), (_, oc, *_) = fns
    rng = np.random.default_rng(2)
    for k in list(range(0, 257, 7)) + [255, 256]:
        a = rng.integers(0, 256, 256, dtype=np.uint8)
        b = a.copy()
        if k < 256:
            b[k] ^= 1 + int(rng.integers(0, 255))
        assert gc(a.tobytes(), b.tobytes()) == oc(a.tobytes(), b.tobytes()) == k


def _zlib_state(data, strstart, wmask):
    """prev[] as deflate's INSERT_STRING leaves it after inserting 1..strstart
    (window-relative positions; 0 is NIL)."""
    head = {}
    prev = np.zeros(wmask + 1, dtype=np.uint16)
    for q in range(1, strstart + 1):
        h = ((data[q] & 31) << 10) ^ (data[q + 1] << 5) ^ data[q + 2]
        prev[q & wmask] = head.get(h, 0)
        head[h] = q
    return prev


@pytest.mark.parametrize("kind", ["text", "runs", "four", "mix"])
def test_longest_match(fns, kind):
    (*_, gl, _), (*_, ol, _) = fns
    wmask = 32767
    data = np.frombuffer(datagen.make(kind, 65536, 3), dtype=np.uint8)
    window = data.tobytes()
    rng = np.random.default_rng(3)
    for strstart in sorted(int(x) for x in rng.integers(300, 65536 - 262, 6)):
        prev = _zlib_state(data, strstart, wmask)
        for prev_length, chain, lookahead in [(2, 128, 258), (3, 4096, 300), (8, 32, 1000), (2, 4, 5)]:
            ms_g, ms_o = C.c_uint32(7), C.c_uint32(7)
            rg = gl(window, strstart, prev_length, 8, chain, lookahead, prev.ctypes.data_as(U16P), wmask,
                    C.byref(ms_g))
            ro = ol(window, strstart, prev_length, 8, chain, lookahead, prev.ctypes.data_as(U16P), wmask,
                    C.byref(ms_o))
            assert (rg, ms_g.value) == (ro, ms_o.value), (kind, strstart, prev_length, chain, lookahead)


def test_chunkmemset(fns):
    (*_, gm), (*_, om) = fns
    rng = np.random.default_rng(4)
    for dist in list(range(1, 21)) + [64, 300]:
        for ln in (0, 1, 15, 16, 17, 100, 1000):
            src = rng.integers(0, 256, max(dist, 1), dtype=np.uint8).tobytes()
            a, b = C.create_string_buffer(ln + 1), C.create_string_buffer(ln + 1)
            gm(a, src, dist, ln)
            om(b, src, dist, ln)
            assert a.raw == b.raw, (dist, ln)
