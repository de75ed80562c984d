"""Python mirror of the reference's front-end over libzgpu.so.

The reference's host API is the TypeScript ``Zlib`` class (src/lib/index.ts:88-271)
sitting on the WASM exports of src/wasm_module.c.  Here the same surface sits on
the C ABI of libzgpu.so (include/zgpu.h): ``Zlib.compress`` returns the same
result record (data, originalSize, compressedSize, compressionRatio,
processingTime, plus ``gpuAccelerated`` in place of ``simdAccelerated``) and
raises ``ZlibCompressionError`` on failure; ``crc32``/``adler32`` take
``(data, init)`` — the reference's TS wrappers pass (ptr, len) to a
(crc, buf, len) export (SURVEY §0 finding 3), which is not reproduced.

Batched and device-resident entry points (``compress_batch``,
``deflate_batch_dev``, ``crc32_batch_dev``, ...) are the new extension.

torch is imported before the library is loaded so that libzgpu.so binds to the
same HIP runtime (libamdhip64.so.7) torch uses; device buffers are torch tensors.
"""
import ctypes as C
import os
import time
from dataclasses import dataclass

try:  # share torch's HIP runtime (must precede loading libzgpu.so)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libzgpu.so")

Z_OK, Z_STREAM_END, Z_STREAM_ERROR, Z_MEM_ERROR, Z_BUF_ERROR = 0, 1, -2, -4, -5
ZGPU_ENODEV = -100
WRAP_RAW, WRAP_ZLIB, WRAP_GZIP = 0, 1, 2
KIND_RANDOM, KIND_SILESIA, KIND_ENWIK, KIND_SMALLVOCAB, KIND_FOUR, KIND_RUNS = 0, 1, 2, 3, 4, 5

EXPORTED_SYMBOLS = (
    # include/zgpu.h
    "zgpu_init", "zgpu_info", "zgpu_set_inflight_bytes", "zgpu_deflate_batch_dev",
    "zgpu_deflate_batch_dev_ex", "zgpu_compress_batch_ex",
    "zgpu_crc32_batch_dev", "zgpu_adler32_batch_dev", "zgpu_compress_batch",
    "zgpu_crc32_batch", "zgpu_adler32_batch", "zgpu_checksum_error", "zgpu_generate_dev", "zgpu_stage_timing",
    "zgpu_stage_timing_read", "zgpu_inflate_batch_dev", "zgpu_uncompress_batch",
    "zgpu_deflate_batch_dev2", "zgpu_compress_batch2",
    # include/zgpu_zlib.h
    "zlibVersion", "compress", "compress2", "compressBound", "deflateInit_",
    "deflateInit2_", "deflate", "deflateEnd", "deflateBound", "deflateReset", "deflateCopy", "deflatePending", "crc32", "crc32_z",
    "crc32_combine", "crc32_combine64", "crc32_combine_gen", "crc32_combine_gen64",
    "crc32_combine_op", "adler32", "adler32_z", "adler32_combine", "adler32_combine64",
    "uncompress", "uncompress2", "inflateInit_", "inflateInit2_", "inflate", "inflateEnd",
    "inflateReset", "inflateGetHeader", "inflateSync", "inflateCopy", "deflateSetDictionary", "deflateParams", "deflateTune", "deflatePrime",
    "deflateSetHeader", "inflateSetDictionary",
    "zError", "zlibCompileFlags", "get_crc_table", "deflateUsed", "deflateGetDictionary",
    "deflateResetKeep", "inflateReset2", "inflateResetKeep", "inflatePrime", "inflateGetDictionary",
    "inflateSyncPoint", "inflateUndermine", "inflateValidate", "inflateMark", "inflateCodesUsed",
    "inflateBackInit_", "inflateBack", "inflateBackEnd",
    # include/zgpu_wasm.h
    "zlib_compress_buffer", "zlib_crc32", "zlib_adler32", "zlib_compress_bound",
    "zlib_get_version", "zlib_compress_simd", "zlib_compress_simd_full",
    "zlib_compress_simd_buffer", "zlib_crc32_simd_optimized", "zlib_crc32_simd_enhanced",
    "zlib_adler32_simd", "zlib_decompress_buffer", "zlib_decompress_optimized",
    "zlib_decompress", "zlib_compress_optimized", "zlib_compress", "zlib_deflate_init",
    "zlib_deflate_process", "zlib_deflate_end", "zlib_inflate_init", "zlib_inflate_process",
    "zlib_inflate_end", "zlib_stream_avail_in", "zlib_stream_avail_out", "zlib_stream_total_in",
    "zlib_stream_total_out", "zlib_slide_hash_simd", "zlib_compare256_simd",
    "zlib_longest_match_simd", "zlib_chunkmemset_simd",
    # include/zgpu_debug.h (test-only)
    "zgpu_debug_stages", "zgpu_debug_par_inflates", "zgpu_debug_parse_fallbacks",
)


class ZlibError(Exception):
    pass


class ZlibCompressionError(ZlibError):
    pass


def compress_bound(n):
    """compressBound (compress.c:72-75)."""
    return n + (n >> 12) + (n >> 14) + (n >> 25) + 13


_lib = None


def load(path=LIB_PATH):
    """Load libzgpu.so (raises if it was not built: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ZlibError(f"{path} missing: run __graft_entry__.build() (no CPU fallback exists)")
    L = C.CDLL(path)
    P, U64, U32, I32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    L.zgpu_init.restype = I32
    L.zgpu_info.restype = C.c_char_p
    L.zgpu_set_inflight_bytes.restype = C.c_size_t
    L.zgpu_set_inflight_bytes.argtypes = [C.c_size_t]
    L.zgpu_deflate_batch_dev.restype = I32
    L.zgpu_deflate_batch_dev.argtypes = [P, P, P, P, P, P, P, P, U32, I32, I32, P]
    L.zgpu_deflate_batch_dev_ex.restype = I32
    L.zgpu_deflate_batch_dev_ex.argtypes = [P, P, P, P, P, P, P, P, U32, I32, I32, I32, P]
    for f in ("zgpu_crc32_batch_dev", "zgpu_adler32_batch_dev"):
        getattr(L, f).restype = I32
        getattr(L, f).argtypes = [P, P, P, P, P, U32, P]
    L.zgpu_compress_batch.restype = I32
    L.zgpu_compress_batch.argtypes = [P, P, P, P, P, C.c_size_t, I32, I32]
    L.zgpu_compress_batch_ex.restype = I32
    L.zgpu_compress_batch_ex.argtypes = [P, P, P, P, P, C.c_size_t, I32, I32, I32]
    L.zgpu_compress_batch2.restype = I32
    L.zgpu_compress_batch2.argtypes = [P, P, P, P, P, C.c_size_t, I32, I32, I32, I32]
    L.zgpu_deflate_batch_dev2.restype = I32
    L.zgpu_deflate_batch_dev2.argtypes = [P, P, P, P, P, P, P, P, U32, I32, I32, I32, I32, P]
    for f in ("zgpu_crc32_batch", "zgpu_adler32_batch"):
        getattr(L, f).restype = I32
        getattr(L, f).argtypes = [P, P, P, P, C.c_size_t]
    L.zgpu_generate_dev.restype = I32
    L.zgpu_generate_dev.argtypes = [P, U64, U32, I32, U64, U64, P]
    L.zgpu_stage_timing.restype = None
    L.zgpu_stage_timing.argtypes = [I32]
    L.zgpu_stage_timing_read.restype = I32
    L.zgpu_stage_timing_read.argtypes = [P, P, I32]
    L.compress2.restype = I32
    L.compress2.argtypes = [P, C.POINTER(C.c_ulong), P, C.c_ulong, I32]
    L.compressBound.restype = C.c_ulong
    L.compressBound.argtypes = [C.c_ulong]
    for f in ("crc32_z", "adler32_z"):
        getattr(L, f).restype = C.c_ulong
        getattr(L, f).argtypes = [C.c_ulong, P, C.c_size_t]
    for f in ("crc32_combine64", "adler32_combine64"):
        getattr(L, f).restype = C.c_ulong
        getattr(L, f).argtypes = [C.c_ulong, C.c_ulong, C.c_int64]
    L.zlibVersion.restype = C.c_char_p
    L.zlib_compress_simd.restype = I32
    L.zlib_compress_simd.argtypes = [P, C.c_size_t, P, C.POINTER(C.c_size_t), I32]
    L.zgpu_inflate_batch_dev.restype = I32
    L.zgpu_inflate_batch_dev.argtypes = [P, P, P, P, P, P, P, P, P, U32, I32, P]
    L.zgpu_uncompress_batch.restype = I32
    L.zgpu_uncompress_batch.argtypes = [P, P, P, P, P, P, C.c_size_t, I32]
    L.uncompress2.restype = I32
    L.uncompress2.argtypes = [P, C.POINTER(C.c_ulong), P, C.POINTER(C.c_ulong)]
    L.uncompress.restype = I32
    L.uncompress.argtypes = [P, C.POINTER(C.c_ulong), P, C.c_ulong]
    _lib = L
    return L


def _ptr_array(bufs):
    arr = (C.c_void_p * len(bufs))()
    keep = []
    for i, b in enumerate(bufs):
        cb = C.create_string_buffer(bytes(b), max(len(b), 1))
        keep.append(cb)
        arr[i] = C.addressof(cb)
    return arr, keep


STRATEGY_DEFAULT, STRATEGY_FILTERED, STRATEGY_HUFFMAN_ONLY, STRATEGY_RLE, STRATEGY_FIXED = 0, 1, 2, 3, 4


def conservative_bound(n):
    """deflateBound's bound for non-default parameters (deflate.c:887-897):
    valid for every strategy."""
    return n + ((n + 7) >> 3) + ((n + 63) >> 6) + 5


def compress_batch(bufs, level=6, wrap=WRAP_ZLIB, caps=None, strategy=0):
    """Compress independent host buffers on the GPU; returns [(status, bytes)].
    ``strategy`` is deflateInit2_'s (0 default, 1 filtered, 2 huffman only,
    3 rle, 4 fixed)."""
    L = load()
    n = len(bufs)
    src, keep = _ptr_array(bufs)
    lens = (C.c_size_t * n)(*[len(b) for b in bufs])
    extra = 12 if wrap == WRAP_GZIP else 0        # deflateBound wraplen 18 vs 6
    if caps is None:
        if strategy == 0:
            caps = [compress_bound(len(b)) + extra for b in bufs]
        else:                                        # + deflateBound's wraplen
            caps = [conservative_bound(len(b)) + (18 if wrap == WRAP_GZIP else 6) for b in bufs]
    outs = [C.create_string_buffer(max(c, 1)) for c in caps]
    dst = (C.c_void_p * n)(*[C.addressof(o) for o in outs])
    dlen = (C.c_size_t * n)(*caps)
    st = (C.c_int * n)()
    rc = L.zgpu_compress_batch_ex(src, lens, dst, dlen, st, n, level, wrap, strategy)
    if rc:
        raise ZlibCompressionError(f"zgpu_compress_batch failed: {rc}")
    del keep
    return [(st[i], outs[i].raw[: dlen[i]]) for i in range(n)]


def compress_batch2(bufs, level=6, window_bits=15, mem_level=8, strategy=0, caps=None):
    """compress_batch with deflateInit2_'s windowBits (8..15 zlib, -15..-9 raw,
    25..31 gzip) and memLevel (1..9); returns [(status, bytes)]."""
    L = load()
    n = len(bufs)
    src, keep = _ptr_array(bufs)
    lens = (C.c_size_t * n)(*[len(b) for b in bufs])
    if caps is None:                                 # deflateBound's conservative bound + wrapper
        caps = [conservative_bound(len(b)) + 18 for b in bufs]
    outs = [C.create_string_buffer(max(c, 1)) for c in caps]
    dst = (C.c_void_p * n)(*[C.addressof(o) for o in outs])
    dlen = (C.c_size_t * n)(*caps)
    st = (C.c_int * n)()
    rc = L.zgpu_compress_batch2(src, lens, dst, dlen, st, n, level, window_bits, mem_level, strategy)
    if rc:
        raise ZlibCompressionError(f"zgpu_compress_batch2 failed: {rc}")
    del keep
    return [(st[i], outs[i].raw[: dlen[i]]) for i in range(n)]


WRAP_AUTO = 3


def uncompress_batch(bufs, caps, wrap=WRAP_ZLIB):
    """Inflate independent host streams on the GPU: [(status, bytes, consumed)]
    with uncompress2 semantics per stream (``caps[i]`` = output capacity)."""
    L = load()
    n = len(bufs)
    src, keep = _ptr_array(bufs)
    lens = (C.c_size_t * n)(*[len(b) for b in bufs])
    outs = [C.create_string_buffer(max(c, 1)) for c in caps]
    dst = (C.c_void_p * n)(*[C.addressof(o) for o in outs])
    dlen = (C.c_size_t * n)(*caps)
    used = (C.c_size_t * n)()
    st = (C.c_int * n)()
    rc = L.zgpu_uncompress_batch(src, lens, dst, dlen, used, st, n, wrap)
    if rc:
        raise ZlibError(f"zgpu_uncompress_batch failed: {rc}")
    del keep
    return [(st[i], outs[i].raw[: dlen[i]], used[i]) for i in range(n)]


def uncompress2(data, cap):
    """zlib uncompress2() through the drop-in symbol: (rc, bytes, consumed)."""
    L = load()
    data = bytes(data)
    out = C.create_string_buffer(max(cap, 1))
    dl, sl = C.c_ulong(cap), C.c_ulong(len(data))
    rc = L.uncompress2(out, C.byref(dl), data, C.byref(sl))
    return rc, out.raw[: dl.value], sl.value


def inflate_batch_dev(src, src_off, src_len, dst, dst_off, dst_cap, dst_len, status, src_used=None,
                      wrap=WRAP_ZLIB, stream=None):
    rc = load().zgpu_inflate_batch_dev(_dp(src), _dp(src_off), _dp(src_len), _dp(dst), _dp(dst_off),
                                       _dp(dst_cap), _dp(dst_len), _dp(src_used), _dp(status),
                                       src_len.numel(), wrap, _stream(stream))
    if rc:
        raise ZlibError(f"zgpu_inflate_batch_dev failed: {rc}")


def _checksum_batch(fn, bufs, inits):
    L = load()
    n = len(bufs)
    src, keep = _ptr_array(bufs)
    lens = (C.c_size_t * n)(*[len(b) for b in bufs])
    init = (C.c_uint32 * n)(*inits) if inits is not None else None
    out = (C.c_uint32 * n)()
    rc = getattr(L, fn)(src, lens, init, out, n)
    if rc:
        raise ZlibError(f"{fn} failed: {rc}")
    del keep
    return list(out)


def crc32_batch(bufs, inits=None):
    return _checksum_batch("zgpu_crc32_batch", bufs, inits)


def adler32_batch(bufs, inits=None):
    return _checksum_batch("zgpu_adler32_batch", bufs, inits)


def compress2(data, level=6, cap=None):
    """zlib compress2() through the drop-in symbol; returns (rc, bytes)."""
    L = load()
    data = bytes(data)
    cap = compress_bound(len(data)) if cap is None else cap
    out = C.create_string_buffer(max(cap, 1))
    n = C.c_ulong(cap)
    rc = L.compress2(out, C.byref(n), data, len(data), level)
    return rc, bytes(memoryview(out)[:n.value])           # (string_at's size is a C int)


def crc32(data, crc=0):
    data = bytes(data)
    return load().crc32_z(crc, data, len(data))


def adler32(data, adler=1):
    data = bytes(data)
    return load().adler32_z(adler, data, len(data))


# ---------------- device-resident (torch tensors as HBM buffers) ----------------

def _dp(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream):
    if stream is None:
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    return C.c_void_p(stream)


def deflate_batch_dev(src, src_off, src_len, dst, dst_off, dst_cap, dst_len, status,
                      level=6, wrap=WRAP_ZLIB, stream=None, strategy=0):
    rc = load().zgpu_deflate_batch_dev_ex(_dp(src), _dp(src_off), _dp(src_len), _dp(dst),
                                          _dp(dst_off), _dp(dst_cap), _dp(dst_len), _dp(status),
                                          src_len.numel(), level, wrap, strategy, _stream(stream))
    if rc:
        raise ZlibCompressionError(f"zgpu_deflate_batch_dev failed: {rc}")


def crc32_batch_dev(src, off, length, out, init=None, stream=None):
    rc = load().zgpu_crc32_batch_dev(_dp(src), _dp(off), _dp(length), _dp(init), _dp(out),
                                     length.numel(), _stream(stream))
    if rc:
        raise ZlibError(f"zgpu_crc32_batch_dev failed: {rc}")


def adler32_batch_dev(src, off, length, out, init=None, stream=None):
    rc = load().zgpu_adler32_batch_dev(_dp(src), _dp(off), _dp(length), _dp(init), _dp(out),
                                       length.numel(), _stream(stream))
    if rc:
        raise ZlibError(f"zgpu_adler32_batch_dev failed: {rc}")


def generate_dev(dst, length, count, kind, seed=1, first_index=0, stream=None):
    rc = load().zgpu_generate_dev(_dp(dst), length, count, kind, seed, first_index, _stream(stream))
    if rc:
        raise ZlibError(f"zgpu_generate_dev failed: {rc}")


STAGES = ("checksum", "links", "match", "parse_lazy", "parse_greedy", "encode")


def stage_timing(enable=True):
    load().zgpu_stage_timing(1 if enable else 0)


def stage_timing_read():
    """{stage: (total_ms, launches)} for the stages of zgpu_deflate_batch_dev."""
    ms = (C.c_double * len(STAGES))()
    n = (C.c_uint64 * len(STAGES))()
    load().zgpu_stage_timing_read(ms, n, len(STAGES))
    return {s: (ms[i], n[i]) for i, s in enumerate(STAGES)}


def debug_stages(data, level):
    """Test-only: (link u16[n], rfull u32[n], rquart u32[n]) from the GPU stages."""
    import numpy as np
    data = bytes(data)
    n = len(data)
    link = np.zeros(max(n, 1), dtype=np.uint16)
    rf = np.zeros(max(n, 1), dtype=np.uint32)
    rq = np.zeros(max(n, 1), dtype=np.uint32)
    L = load()
    L.zgpu_debug_stages.restype = C.c_int
    L.zgpu_debug_stages.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    rc = L.zgpu_debug_stages(data, n, level, link.ctypes.data, rf.ctypes.data, rq.ctypes.data)
    if rc:
        raise ZlibError(f"zgpu_debug_stages failed: {rc}")
    return link[:n], rf[:n], rq[:n]


def set_inflight_bytes(n):
    return load().zgpu_set_inflight_bytes(n)


def info():
    return load().zgpu_info().decode()


# ---------------- the reference's TS surface ----------------

@dataclass
class ZlibResult:
    """src/lib/types.ts:71-78."""
    data: bytes
    originalSize: int
    compressedSize: int
    compressionRatio: float
    processingTime: float
    gpuAccelerated: bool = True


class Zlib:
    """src/lib/index.ts ``Zlib`` — compress / crc32 / adler32 / getVersion."""

    def __init__(self):
        load()

    def compress(self, data, level=6):
        t0 = time.perf_counter()
        data = bytes(data)
        rc, out = compress2(data, level if level is not None else 6)
        if rc != Z_OK:
            raise ZlibCompressionError(f"Compression failed with code: {rc}")
        ms = (time.perf_counter() - t0) * 1e3
        return ZlibResult(out, len(data), len(out), len(data) / max(len(out), 1), ms)

    def crc32(self, data, crc=0):
        return crc32(data, crc)

    def adler32(self, data, adler=1):
        return adler32(data, adler)

    def getVersion(self):
        return load().zlibVersion().decode()
