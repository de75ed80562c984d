"""ctypes helpers for the test suite (TEST INFRASTRUCTURE).

* ``Oracle``    — oracle/liboracle.so, our C restatement of the reference path.
* ``Reference`` — oracle/_ref/libzref.so, the reference compiled from
  /root/reference.  It exists only in the build container (it never travels to
  the GPU box), so tests that need it skip when it is absent.
"""
import ctypes as C
import hashlib
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libzref.so")

Z_OK, Z_STREAM_END, Z_STREAM_ERROR, Z_MEM_ERROR, Z_BUF_ERROR = 0, 1, -2, -4, -5


def build_oracle():
    """(Re)build the oracle checker library; cheap when up to date."""
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)


def compress_bound(n):
    return n + (n >> 12) + (n >> 14) + (n >> 25) + 13


class Oracle:
    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        L = C.CDLL(path)
        L.zo_compress.restype = C.c_int
        L.zo_compress.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p,
                                  C.c_size_t, C.c_int, C.c_int]
        L.zo_pp_compress.restype = C.c_int
        L.zo_pp_compress.argtypes = L.zo_compress.argtypes
        L.zo_compress2.restype = C.c_int
        L.zo_compress2.argtypes = L.zo_compress.argtypes + [C.c_int]
        for f in ("zo_crc32", "zo_adler32"):
            getattr(L, f).restype = C.c_uint32
            getattr(L, f).argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        for f in ("zo_crc32_combine", "zo_adler32_combine"):
            getattr(L, f).restype = C.c_uint32
            getattr(L, f).argtypes = [C.c_uint32, C.c_uint32, C.c_int64]
        L.zo_uncompress3.restype = C.c_int
        L.zo_uncompress3.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p,
                                     C.POINTER(C.c_size_t), C.c_int]
        L.zo_deflate_flushes.restype = C.c_int
        L.zo_deflate_flushes.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p, C.c_size_t,
                                         C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                         C.c_int]
        L.zo_deflate_stored_calls.restype = C.c_int
        L.zo_deflate_stored_calls.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p, C.c_size_t,
                                              C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                              C.c_void_p]
        L.zo_pp_links.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.zo_pp_match.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p,
                                  C.c_void_p, C.c_void_p]
        L.zo_generate.restype = C.c_int
        L.zo_generate.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_uint64, C.c_uint64]
        self.L = L

    def generate(self, length, count, kind, seed, first_index=0):
        """The bytes zgpu_generate_dev(kind, seed, first_index) writes (host
        build of zgpu_gen.h): a list of `count` buffers of `length` bytes."""
        import numpy as np
        buf = np.zeros(length * count + 4, dtype=np.uint8)
        assert self.L.zo_generate(buf.ctypes.data, length, count, kind, seed, first_index) == 0
        return [buf[i * length:(i + 1) * length].tobytes() for i in range(count)]

    def _compress(self, fn, data, level, wrap, cap):
        data = bytes(data)
        if cap is None:
            cap = compress_bound(len(data)) + 32
        out = C.create_string_buffer(max(cap, 1))
        n = C.c_size_t(cap)
        rc = fn(out, C.byref(n), data, len(data), level, wrap)
        return rc, out.raw[: n.value]

    def compress(self, data, level=6, wrap=1, cap=None, strategy=0):
        if strategy:
            return self._compress(lambda o, n, d, ln, lv, w: self.L.zo_compress2(o, n, d, ln, lv, w, strategy),
                                  data, level, wrap, cap)
        return self._compress(self.L.zo_compress, data, level, wrap, cap)

    def deflate_stored_calls(self, data, calls, wrap=1):
        """zo_deflate_stored_calls: level 0 over [(input_len, flush)] ->
        (rc, statuses, output length after each call, stream)."""
        data = bytes(data)
        nc = len(calls)
        take = (C.c_size_t * max(nc, 1))(*[c[0] for c in calls])
        fl = (C.c_int * max(nc, 1))(*[c[1] for c in calls])
        st = (C.c_int * max(nc, 1))()
        ol = (C.c_size_t * max(nc, 1))()
        cap = compress_bound(len(data)) + 64 + 16 * nc
        out = C.create_string_buffer(cap)
        n = C.c_size_t(cap)
        rc = self.L.zo_deflate_stored_calls(out, C.byref(n), data, len(data), wrap, take, fl, nc, st, ol)
        return rc, list(st[:nc]), list(ol[:nc]), out.raw[: n.value]

    def deflate_flushes(self, data, events, level=6, wrap=1, strategy=0, finish=True):
        """zo_deflate_flushes: (rc, stream) for flush events [(pos, flush)]."""
        data = bytes(data)
        nf = len(events)
        fpos = (C.c_size_t * max(nf, 1))(*[e[0] for e in events])
        ftyp = (C.c_int * max(nf, 1))(*[e[1] for e in events])
        cap = compress_bound(len(data)) + 64 + 16 * nf
        out = C.create_string_buffer(cap)
        n = C.c_size_t(cap)
        rc = self.L.zo_deflate_flushes(out, C.byref(n), data, len(data), level, wrap, strategy, fpos, ftyp,
                                       nf, 1 if finish else 0)
        return rc, out.raw[: n.value]

    def pp_compress(self, data, level=6, wrap=1, cap=None):
        return self._compress(self.L.zo_pp_compress, data, level, wrap, cap)

    def uncompress(self, src, cap, wrap=1):
        """uncompress2 semantics for any wrapper: (status, output, consumed)."""
        src = bytes(src)
        out = C.create_string_buffer(max(cap, 1))
        dl, sl = C.c_size_t(cap), C.c_size_t(len(src))
        rc = self.L.zo_uncompress3(out, C.byref(dl), src, C.byref(sl), wrap)
        return rc, out.raw[: dl.value], sl.value

    def crc32(self, data, crc=0):
        data = bytes(data)
        return self.L.zo_crc32(crc, data, len(data))

    def adler32(self, data, adler=1):
        data = bytes(data)
        return self.L.zo_adler32(adler, data, len(data))

    def links(self, data):
        import numpy as np
        data = bytes(data)
        out = np.zeros(len(data), dtype=np.uint16)
        self.L.zo_pp_links(data, len(data), out.ctypes.data)
        return out

    def match(self, data, level, links):
        import numpy as np
        data = bytes(data)
        full = np.zeros(len(data), dtype=np.uint32)
        quarter = np.zeros(len(data), dtype=np.uint32)
        self.L.zo_pp_match(data, len(data), level, links.ctypes.data,
                           full.ctypes.data, quarter.ctypes.data)
        return full, quarter


class ZStream(C.Structure):
    """z_stream as laid out by zlib.h:90-110 on LP64."""
    _fields_ = [("next_in", C.c_void_p), ("avail_in", C.c_uint), ("total_in", C.c_ulong),
                ("next_out", C.c_void_p), ("avail_out", C.c_uint), ("total_out", C.c_ulong),
                ("msg", C.c_char_p), ("state", C.c_void_p), ("zalloc", C.c_void_p),
                ("zfree", C.c_void_p), ("opaque", C.c_void_p), ("data_type", C.c_int),
                ("adler", C.c_ulong), ("reserved", C.c_ulong)]


class Reference:
    """The compiled reference (build container only)."""

    def __init__(self, path=REF_SO):
        L = C.CDLL(path)
        L.compress2.restype = C.c_int
        L.compress2.argtypes = [C.c_void_p, C.POINTER(C.c_ulong), C.c_void_p, C.c_ulong, C.c_int]
        L.crc32.restype = C.c_ulong
        L.crc32.argtypes = [C.c_ulong, C.c_void_p, C.c_uint]
        L.adler32.restype = C.c_ulong
        L.adler32.argtypes = [C.c_ulong, C.c_void_p, C.c_uint]
        L.crc32_combine.restype = C.c_ulong
        L.crc32_combine.argtypes = [C.c_ulong, C.c_ulong, C.c_long]
        L.adler32_combine.restype = C.c_ulong
        L.adler32_combine.argtypes = [C.c_ulong, C.c_ulong, C.c_long]
        L.zlibVersion.restype = C.c_char_p
        L.deflateInit2_.restype = C.c_int
        L.deflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_char_p, C.c_int]
        L.deflate.restype = C.c_int
        L.deflate.argtypes = [C.POINTER(ZStream), C.c_int]
        L.deflateEnd.restype = C.c_int
        L.deflateEnd.argtypes = [C.POINTER(ZStream)]
        L.uncompress2.restype = C.c_int
        L.uncompress2.argtypes = [C.c_void_p, C.POINTER(C.c_ulong), C.c_void_p, C.POINTER(C.c_ulong)]
        L.inflateInit2_.restype = C.c_int
        L.inflateInit2_.argtypes = [C.POINTER(ZStream), C.c_int, C.c_char_p, C.c_int]
        L.inflate.restype = C.c_int
        L.inflate.argtypes = [C.POINTER(ZStream), C.c_int]
        L.inflateEnd.restype = C.c_int
        L.inflateEnd.argtypes = [C.POINTER(ZStream)]
        self.L = L
        self.version = L.zlibVersion()

    def uncompress(self, src, cap, wrap=1):
        """(status, output, consumed).  wrap 1 calls the reference's own
        uncompress2; the other wrappers run uncompress2's loop (uncompr.c:24-80)
        over the reference's inflateInit2_/inflate (windowBits -15, 31, 47)."""
        src = bytes(src)
        out = C.create_string_buffer(max(cap, 1))
        if wrap == 1:
            dl, sl = C.c_ulong(cap), C.c_ulong(len(src))
            rc = self.L.uncompress2(out, C.byref(dl), src, C.byref(sl))
            return rc, out.raw[: dl.value], sl.value
        inbuf = C.create_string_buffer(src, max(len(src), 1))
        strm = ZStream()
        wbits = {0: -15, 2: 31, 3: 47}[wrap]
        assert self.L.inflateInit2_(C.byref(strm), wbits, self.version, C.sizeof(ZStream)) == Z_OK
        probe = cap == 0
        buf1 = C.create_string_buffer(1)
        left = 1 if probe else cap
        strm.next_in = C.addressof(inbuf)
        strm.avail_in = len(src)
        strm.next_out = C.addressof(buf1) if probe else C.addressof(out)
        strm.avail_out = left
        left = 0
        while True:
            err = self.L.inflate(C.byref(strm), 0)
            if err != Z_OK:
                break
        consumed = len(src) - strm.avail_in
        total = strm.total_out
        if probe and total and err == -5:
            left = 1
        avail_out = strm.avail_out
        self.L.inflateEnd(C.byref(strm))
        if err == 1:
            rc = Z_OK
        elif err == 2:
            rc = -3
        elif err == -5 and left + avail_out:
            rc = -3
        else:
            rc = err
        return rc, (b"" if probe else out.raw[:total]), consumed

    def compress2(self, data, level=6, cap=None):
        data = bytes(data)
        if cap is None:
            cap = compress_bound(len(data))
        out = C.create_string_buffer(max(cap, 1))
        n = C.c_ulong(cap)
        rc = self.L.compress2(out, C.byref(n), data, len(data), level)
        return rc, out.raw[: n.value]

    def deflate(self, data, level=6, wbits=15, chunk=None, strategy=0, mem_level=8):
        """deflateInit2 + deflate; wbits -15 raw, 15 zlib, 31 gzip.  ``chunk``
        feeds the input in pieces with Z_NO_FLUSH before Z_FINISH."""
        data = bytes(data)
        strm = ZStream()
        rc = self.L.deflateInit2_(C.byref(strm), level, 8, wbits, mem_level, strategy, self.version,
                                  C.sizeof(ZStream))
        assert rc == Z_OK, rc
        cap = len(data) + (len(data) >> 3) + (len(data) >> 6) + 64
        out = C.create_string_buffer(cap)
        inbuf = C.create_string_buffer(data, max(len(data), 1))
        base_in = C.addressof(inbuf)
        strm.next_out = C.addressof(out)
        strm.avail_out = cap
        pos = 0
        step = chunk or max(len(data), 1)
        while True:
            take = min(step, len(data) - pos)
            strm.next_in = base_in + pos
            strm.avail_in = take
            pos += take
            flush = 4 if pos >= len(data) else 0
            rc = self.L.deflate(C.byref(strm), flush)
            if flush == 4:
                break
        assert rc == Z_STREAM_END, rc
        total = strm.total_out
        self.L.deflateEnd(C.byref(strm))
        return out.raw[:total]

    def init_rc(self, level, wbits, mem_level, strategy=0):
        """deflateInit2_'s return code (the stream is ended again if it opened)."""
        strm = ZStream()
        rc = self.L.deflateInit2_(C.byref(strm), level, 8, wbits, mem_level, strategy, self.version,
                                  C.sizeof(ZStream))
        if rc == Z_OK:
            self.L.deflateEnd(C.byref(strm))
        return rc

    def bound(self, level, wbits, mem_level, strategy, n):
        """deflateBound(n) of a freshly initialised stream."""
        strm = ZStream()
        assert self.L.deflateInit2_(C.byref(strm), level, 8, wbits, mem_level, strategy, self.version,
                                    C.sizeof(ZStream)) == Z_OK
        self.L.deflateBound.restype = C.c_ulong
        self.L.deflateBound.argtypes = [C.POINTER(ZStream), C.c_ulong]
        b = self.L.deflateBound(C.byref(strm), n)
        self.L.deflateEnd(C.byref(strm))
        return int(b)

    def deflate_calls(self, data, calls, level=6, wbits=15, strategy=0):
        """deflate() over a call sequence [(input_len, flush), ...] (the lengths
        sum to len(data), the last call is Z_FINISH or not); returns
        (status per call, output length after each call, whole output)."""
        data = bytes(data)
        strm = ZStream()
        rc = self.L.deflateInit2_(C.byref(strm), level, 8, wbits, 8, strategy, self.version,
                                  C.sizeof(ZStream))
        assert rc == Z_OK, rc
        cap = compress_bound(len(data)) + 64 + 16 * len(calls)
        out = C.create_string_buffer(cap)
        inbuf = C.create_string_buffer(data, max(len(data), 1))
        strm.next_out = C.addressof(out)
        strm.avail_out = cap
        pos, sts, lens = 0, [], []
        for take, flush in calls:
            strm.next_in = C.addressof(inbuf) + pos
            strm.avail_in = take
            pos += take
            sts.append(self.L.deflate(C.byref(strm), flush))
            lens.append(strm.total_out)
        total = strm.total_out
        self.L.deflateEnd(C.byref(strm))
        return sts, lens, out.raw[:total]

    def crc32(self, data, crc=0):
        data = bytes(data)
        return self.L.crc32(crc, data, len(data))

    def adler32(self, data, adler=1):
        data = bytes(data)
        return self.L.adler32(adler, data, len(data))


def flush_events(calls):
    """The flush events zlib acts on for a call sequence: a flush call with no
    new input whose RANK is not above the previous call's is refused with
    Z_BUF_ERROR (deflate.c:1002-1005).  Returns [(position, flush), ...]."""
    rank = lambda f: f * 2 - (9 if f > 4 else 0)
    ev, pos, last = [], 0, -2
    for take, flush in calls:
        pos += take
        if flush not in (0, 4) and not (take == 0 and rank(flush) <= rank(last)):
            ev.append((pos, flush))
        last = flush
    return ev


def reference_available():
    return os.path.exists(REF_SO)


class GzHeader(C.Structure):
    """gz_header as zlib.h declares it (deflateSetHeader)."""
    _fields_ = [("text", C.c_int), ("time", C.c_ulong), ("xflags", C.c_int), ("os", C.c_int),
                ("extra", C.c_void_p), ("extra_len", C.c_uint), ("extra_max", C.c_uint),
                ("name", C.c_void_p), ("name_max", C.c_uint), ("comment", C.c_void_p),
                ("comm_max", C.c_uint), ("hcrc", C.c_int), ("done", C.c_int)]


def _bind_zstream(L):
    P = C.POINTER(ZStream)
    for name, res, args in (
            ("deflateInit2_", C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int]),
            ("deflate", C.c_int, [P, C.c_int]), ("deflateEnd", C.c_int, [P]),
            ("deflateSetDictionary", C.c_int, [P, C.c_void_p, C.c_uint]),
            ("deflateParams", C.c_int, [P, C.c_int, C.c_int]),
            ("deflateTune", C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int]),
            ("deflatePrime", C.c_int, [P, C.c_int, C.c_int]),
            ("deflateSetHeader", C.c_int, [P, C.POINTER(GzHeader)]),
            ("inflateInit2_", C.c_int, [P, C.c_int, C.c_char_p, C.c_int]),
            ("inflate", C.c_int, [P, C.c_int]), ("inflateEnd", C.c_int, [P]),
            ("inflateSetDictionary", C.c_int, [P, C.c_void_p, C.c_uint]),
            ("deflateBound", C.c_ulong, [P, C.c_ulong]),
            ("inflateGetHeader", C.c_int, [P, C.POINTER(GzHeader)]),
            ("inflateSync", C.c_int, [P]), ("inflateCopy", C.c_int, [P, P]),
            # the rest of zlib.h's z_stream calls (round 4)
            ("deflateUsed", C.c_int, [P, C.POINTER(C.c_int)]),
            ("deflateGetDictionary", C.c_int, [P, C.c_void_p, C.POINTER(C.c_uint)]),
            ("deflateResetKeep", C.c_int, [P]), ("deflateReset", C.c_int, [P]),
            ("inflateReset", C.c_int, [P]), ("inflateReset2", C.c_int, [P, C.c_int]),
            ("inflateResetKeep", C.c_int, [P]), ("inflatePrime", C.c_int, [P, C.c_int, C.c_int]),
            ("inflateGetDictionary", C.c_int, [P, C.c_void_p, C.POINTER(C.c_uint)]),
            ("inflateSyncPoint", C.c_int, [P]), ("inflateUndermine", C.c_int, [P, C.c_int]),
            ("inflateValidate", C.c_int, [P, C.c_int]), ("inflateMark", C.c_long, [P]),
            ("inflateCodesUsed", C.c_ulong, [P]),
            ("inflateBackInit_", C.c_int, [P, C.c_int, C.c_void_p, C.c_char_p, C.c_int]),
            ("inflateBack", C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
            ("inflateBackEnd", C.c_int, [P])):
        try:
            f = getattr(L, name)
        except AttributeError:                   # an older system zlib (no deflateUsed, ...)
            continue
        f.restype = res
        f.argtypes = args


def run_zsession(L, ops, version=b"1.3.1.1-motley"):
    """Run a scripted z_stream deflate session on library L (the reference or
    libzgpu.so) and return (return codes / adler values per op, stream bytes).
    ops: ("init", level, windowBits, memLevel, strategy), ("dict", bytes),
    ("tune", good, lazy, nice, chain), ("params", level, strategy),
    ("prime", bits, value), ("header", dict of gz_header fields),
    ("deflate", bytes, flush[, out]), ("bound", sourceLen).  Output space is
    ample unless a deflate op gives `out`: then every call gets `out` bytes and
    the op repeats the call until the input is taken and the call ends with
    space left (or Z_STREAM_END), as zpipe.c's loop does."""
    _bind_zstream(L)
    s = ZStream()
    out, rcs, keep = bytearray(), [], []
    left = b""                                   # input the last "deflate1" call did not take
    obuf_n = 1 << 16

    def with_out(call, extra=0):
        n = obuf_n + extra
        ob = C.create_string_buffer(n)
        s.next_out, s.avail_out = C.addressof(ob), n
        rc = call()
        out.extend(ob.raw[: n - s.avail_out])
        return rc

    for op in ops:
        k = op[0]
        if k == "init":
            rcs.append(L.deflateInit2_(C.byref(s), op[1], 8, op[2], op[3], op[4], version, C.sizeof(ZStream)))
        elif k == "dict":
            b = C.create_string_buffer(op[1], len(op[1]))
            rcs.append((L.deflateSetDictionary(C.byref(s), b, len(op[1])), s.adler))
        elif k == "tune":
            rcs.append(L.deflateTune(C.byref(s), *op[1:]))
        elif k == "params":
            rcs.append(with_out(lambda: L.deflateParams(C.byref(s), op[1], op[2]), 1 << 20))
        elif k == "prime":
            rcs.append(L.deflatePrime(C.byref(s), op[1], op[2]))
        elif k == "header":
            h = GzHeader()
            f = op[1]
            h.text, h.time, h.os, h.hcrc = f.get("text", 0), f.get("time", 0), f.get("os", 3), f.get("hcrc", 0)
            for fld in ("extra", "name", "comment"):
                if fld in f:
                    buf = C.create_string_buffer(f[fld], len(f[fld]) + (0 if fld == "extra" else 1))
                    keep.append(buf)
                    setattr(h, fld, C.addressof(buf))
            if "extra" in f:
                h.extra_len = len(f["extra"])
            keep.append(h)
            rcs.append(L.deflateSetHeader(C.byref(s), C.byref(h)))
        elif k == "deflate":
            data, flush = op[1], op[2]
            if len(op) > 4 and op[4]:
                data = left + data
            ib = C.create_string_buffer(data, len(data))
            keep.append(ib)
            s.next_in, s.avail_in = C.addressof(ib), len(data)
            seq = []
            if len(op) > 3 and op[3]:            # small output buffers: one call per `out` bytes
                ob = C.create_string_buffer(op[3])
                for _ in range(200000):
                    s.next_out, s.avail_out = C.addressof(ob), op[3]
                    rc = L.deflate(C.byref(s), flush)
                    out.extend(ob.raw[: op[3] - s.avail_out])
                    seq.append(rc)
                    if rc < 0 or rc == 1 or (s.avail_in == 0 and s.avail_out != 0):
                        break
                rcs.append(seq)
                continue
            for _ in range(1000):
                rc = with_out(lambda: L.deflate(C.byref(s), flush), len(data) + len(data) // 2)
                seq.append(rc)
                if rc < 0 or rc == 1 or (s.avail_in == 0 and s.avail_out != 0):
                    break
            rcs.append(seq)
        elif k == "deflate1":                    # ONE call with `out` bytes of space (a flush may stay pending)
            data, flush, n = op[1], op[2], op[3]
            if len(op) > 4 and op[4]:            # "cont": the input the last call left comes first (zlib.h)
                data = left + data
            ib = C.create_string_buffer(data, len(data))
            keep.append(ib)
            s.next_in, s.avail_in = C.addressof(ib), len(data)
            ob = C.create_string_buffer(max(n, 1))
            s.next_out, s.avail_out = C.addressof(ob), n
            rc = L.deflate(C.byref(s), flush)
            out.extend(ob.raw[: n - s.avail_out])
            rcs.append([rc, s.avail_in, s.avail_out])
            left = data[len(data) - s.avail_in:] if s.avail_in else b""
        elif k == "bound":
            rcs.append(int(L.deflateBound(C.byref(s), op[1])))
        elif k == "pending":                     # deflatePending: rc, bytes, bits
            pn, pb = C.c_uint(0), C.c_int(0)
            rcs.append([L.deflatePending(C.byref(s), C.byref(pn), C.byref(pb)), pn.value, pb.value])
        elif k == "used":                        # deflateUsed
            b = C.c_int(-99)
            rcs.append([L.deflateUsed(C.byref(s), C.byref(b)), b.value])
        elif k == "getdict":                     # deflateGetDictionary: rc, length, sha256
            n = C.c_uint(0)
            rc = L.deflateGetDictionary(C.byref(s), None, C.byref(n))
            buf = C.create_string_buffer(max(n.value, 1))
            n2 = C.c_uint(0)
            rc2 = L.deflateGetDictionary(C.byref(s), buf, C.byref(n2))
            rcs.append([rc, rc2, n2.value, hashlib.sha256(buf.raw[:n2.value]).hexdigest()[:16]])
        elif k == "resetkeep":
            rcs.append(L.deflateResetKeep(C.byref(s)))
        elif k == "reset":
            rcs.append(L.deflateReset(C.byref(s)))
        else:
            raise ValueError(k)
    L.deflateEnd(C.byref(s))
    return rcs, bytes(out)


def run_isession(L, z, wbits=15, dictionary=None, chunk=1 << 30, version=b"1.3.1.1-motley"):
    """Inflate z on library L through the z_stream API, answering Z_NEED_DICT
    with `dictionary` (or setting it up front for raw streams, wbits < 0);
    returns (return codes, output)."""
    _bind_zstream(L)
    s = ZStream()
    rcs = [L.inflateInit2_(C.byref(s), wbits, version, C.sizeof(ZStream))]
    if dictionary is not None and wbits < 0:
        rcs.append(L.inflateSetDictionary(C.byref(s), dictionary, len(dictionary)))
    ib = C.create_string_buffer(bytes(z), len(z))
    ob = C.create_string_buffer(1 << 20)
    out, pos = bytearray(), 0
    for _ in range(100000):
        if s.avail_in == 0 and pos < len(z):
            take = min(chunk, len(z) - pos)
            s.next_in, s.avail_in = C.addressof(ib) + pos, take
            pos += take
        s.next_out, s.avail_out = C.addressof(ob), 1 << 20
        rc = L.inflate(C.byref(s), 0)
        out.extend(ob.raw[: (1 << 20) - s.avail_out])
        if rc == 2:                                      # Z_NEED_DICT
            rcs.append(("need", s.adler, s.total_in))
            d = dictionary if dictionary is not None else b""
            r = L.inflateSetDictionary(C.byref(s), d, len(d))
            rcs.append(r)
            if r != 0:
                break
            continue
        if rc != 0 or (pos == len(z) and s.avail_in == 0 and s.avail_out != 0):
            rcs.append(rc)
            break
    L.inflateEnd(C.byref(s))
    return rcs, bytes(out)


def _gen_bytes(spec):
    import datagen
    return datagen.make(*spec)


def run_iops(L, z, ops, version=b"1.3.1.1-motley"):
    """A scripted z_stream inflate session over the compressed bytes z on
    library L (the reference or libzgpu.so); returns (per-op results, the
    output of each stream, the gz_header fields).  ops:
      ("init", windowBits)            inflateInit2_
      ("header", extra_max, name_max, comm_max)   inflateGetHeader
      ("feed", n)                     n more bytes of z become available input
      ("skip", n)                     the next n bytes of z are dropped (a damaged stretch)
      ("inflate", flush, out)         one call with `out` bytes of output space
      ("loop", flush, out)            calls until Z_STREAM_END, an error, or a call that
                                      makes no progress
      ("sync",)                       inflateSync
      ("copy",)                       inflateCopy of the active stream; ("use", k) drives stream k
      ("dict", hex | [kind, n, seed])  inflateSetDictionary (given, or datagen bytes)
    Each call records (rc, avail_in, total_in, total_out[, data_type when the
    flush is Z_BLOCK and rc is Z_OK]), inflateSync (rc, avail_in, total_in)."""
    _bind_zstream(L)
    zb = C.create_string_buffer(bytes(z), max(len(z), 1))
    base = C.addressof(zb)
    streams = [ZStream()]
    outs = [bytearray()]
    cur = [0]
    act = 0
    end = 0                              # end of the input made available so far
    res, keep = [], []
    hdr = None

    def call(flush, n):
        nonlocal end
        s = streams[act]
        ob = C.create_string_buffer(max(n, 1))
        s.next_out, s.avail_out = C.addressof(ob), n
        rc = L.inflate(C.byref(s), flush)
        outs[act].extend(ob.raw[: n - s.avail_out])
        got = n - s.avail_out
        r = [rc, s.avail_in, s.total_in, s.total_out]
        if flush in (5, 6) and rc == 0:          # Z_BLOCK, Z_TREES
            r.append(s.data_type)
        return r, got

    for op in ops:
        k = op[0]
        s = streams[act]
        if k == "init":
            res.append(L.inflateInit2_(C.byref(s), op[1], version, C.sizeof(ZStream)))
            s.next_in, s.avail_in = base, 0
        elif k == "header":
            hdr = GzHeader()
            bufs = [C.create_string_buffer(b"\xee" * max(m, 1), max(m, 1)) for m in op[1:4]]
            keep.extend(bufs)
            hdr.extra, hdr.extra_max = C.addressof(bufs[0]), op[1]
            hdr.name, hdr.name_max = C.addressof(bufs[1]), op[2]
            hdr.comment, hdr.comm_max = C.addressof(bufs[2]), op[3]
            hdr.done = 7
            hdr._bufs = bufs
            res.append(L.inflateGetHeader(C.byref(s), C.byref(hdr)))
        elif k in ("feed", "skip"):
            at = (s.next_in or base) - base
            if k == "skip":
                at = min(len(z), at + op[1])
                end = max(end, at)
            else:
                end = min(len(z), max(end, at) + op[1])
            s.next_in, s.avail_in = base + at, end - at
        elif k == "inflate":
            r, _ = call(op[1], op[2])
            res.append(r)
        elif k == "loop":
            seq = []
            for _ in range(100000):
                r, got = call(op[1], op[2])
                seq.append(r)
                if r[0] != 0 or (got == 0 and streams[act].avail_in == 0):
                    break
            res.append(seq)
        elif k == "sync":
            rc = L.inflateSync(C.byref(s))
            res.append([rc, s.avail_in, s.total_in])
        elif k == "copy":
            d = ZStream()
            res.append(L.inflateCopy(C.byref(d), C.byref(s)))
            streams.append(d)
            outs.append(bytearray())
        elif k == "use":
            act = op[1]
        elif k == "dict":
            d = bytes.fromhex(op[1]) if isinstance(op[1], str) else _gen_bytes(op[1])
            res.append(L.inflateSetDictionary(C.byref(s), d, len(d)))
        # the rest of zlib.h's inflate calls (round 4)
        elif k == "getdict":                     # inflateGetDictionary: rc, length, sha256
            n = C.c_uint(0)
            rc = L.inflateGetDictionary(C.byref(s), None, C.byref(n))
            buf = C.create_string_buffer(max(n.value, 1))
            n2 = C.c_uint(0)
            rc2 = L.inflateGetDictionary(C.byref(s), buf, C.byref(n2))
            res.append([rc, rc2, n2.value, hashlib.sha256(buf.raw[:n2.value]).hexdigest()[:16]])
        elif k == "mark":
            res.append(int(L.inflateMark(C.byref(s))))
        elif k == "codes":
            res.append(int(L.inflateCodesUsed(C.byref(s))))
        elif k == "syncpoint":
            res.append(L.inflateSyncPoint(C.byref(s)))
        elif k == "validate":
            res.append(L.inflateValidate(C.byref(s), op[1]))
        elif k == "undermine":
            res.append(L.inflateUndermine(C.byref(s), op[1]))
        elif k == "reset":
            res.append([L.inflateReset(C.byref(s)), s.total_in, s.total_out, s.adler])
            outs[act] = bytearray()
        elif k == "reset2":
            res.append([L.inflateReset2(C.byref(s), op[1]), s.adler])
            outs[act] = bytearray()
        elif k == "resetkeep":
            res.append([L.inflateResetKeep(C.byref(s)), s.adler])
            outs[act] = bytearray()
        elif k == "prime":
            res.append(L.inflatePrime(C.byref(s), op[1], op[2]))
        elif k == "adler":
            res.append(int(s.adler))
        else:
            raise ValueError(k)
    for s in streams:
        L.inflateEnd(C.byref(s))
    fields = None
    if hdr is not None:
        raw = lambda p, m: None if not p else C.string_at(p, m).hex()
        fields = {"text": hdr.text, "time": hdr.time, "xflags": hdr.xflags, "os": hdr.os,
                  "extra_len": hdr.extra_len, "extra": raw(hdr.extra, hdr.extra_max),
                  "name": raw(hdr.name, hdr.name_max), "comment": raw(hdr.comment, hdr.comm_max),
                  "hcrc": hdr.hcrc, "done": hdr.done}
    return res, [bytes(o) for o in outs], fields


def run_dsession(L, data, plan, level=6, wbits=15, mem=8, strategy=0, version=b"1.3.1.1-motley",
                 max_calls=20000):
    """deflate() over `data` on library L the way a caller with a fixed-size
    output buffer drives it, recording what every call does.

    plan: [(new_input, flush, avail_out, loop), ...].  Each entry offers
    `new_input` more bytes (unconsumed input stays offered: next_in / avail_in
    continue where the library left them) and calls deflate(flush) with
    `avail_out` bytes of output space; with loop set it calls again (no new
    input) while the call used up all of avail_out, as zpipe.c does.
    Returns (records, stream): one (return code, avail_in after, bytes
    written) per call."""
    _bind_zstream(L)
    s = ZStream()
    rc = L.deflateInit2_(C.byref(s), level, 8, wbits, mem, strategy, version, C.sizeof(ZStream))
    assert rc == 0, rc
    ib = C.create_string_buffer(bytes(data), max(len(data), 1))
    base = C.addressof(ib)
    out, recs, offered = bytearray(), [], 0
    ob = C.create_string_buffer(max([1 << 20] + [p[2] for p in plan]))
    for new, flush, avail, loop in plan:
        offered = min(len(data), offered + new)
        while True:
            s.next_in = base + s.total_in
            s.avail_in = offered - s.total_in
            s.next_out, s.avail_out = C.addressof(ob), avail
            r = L.deflate(C.byref(s), flush)
            got = avail - s.avail_out
            out.extend(ob.raw[:got])
            recs.append((r, s.avail_in, got))
            if len(recs) >= max_calls or not loop or r not in (0, -5) or s.avail_out != 0 or r == 1:
                break
        if len(recs) >= max_calls:
            break
    L.deflateEnd(C.byref(s))
    return recs, bytes(out)


IN_FUNC = C.CFUNCTYPE(C.c_uint, C.c_void_p, C.POINTER(C.c_void_p))
OUT_FUNC = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint)


def run_back(L, z, wbits=15, in_chunk=1 << 30, first=0, out_fail_at=None, version=b"1.3.1.1-motley"):
    """inflateBackInit_ / inflateBack / inflateBackEnd over the raw stream z on
    library L: in() hands out `in_chunk` bytes per call (after `first` bytes
    given up front in next_in), out() collects (and fails on call number
    `out_fail_at`).  Returns (init rc, back rc, output, unused input length,
    next_in is NULL, end rc, out() calls)."""
    _bind_zstream(L)
    s = ZStream()
    win = C.create_string_buffer(1 << wbits)
    rc0 = L.inflateBackInit_(C.byref(s), wbits, win, version, C.sizeof(ZStream))
    zb = C.create_string_buffer(bytes(z), max(len(z), 1))
    base = C.addressof(zb)
    pos = [first]
    out = bytearray()
    ncall = [0]

    def fin(_desc, pbuf):
        n = min(in_chunk, len(z) - pos[0])
        pbuf[0] = base + pos[0]
        pos[0] += n
        return n

    def fout(_desc, buf, n):
        ncall[0] += 1
        if out_fail_at is not None and ncall[0] == out_fail_at:
            return 1
        out.extend(C.string_at(buf, n))
        return 0

    fi, fo = IN_FUNC(fin), OUT_FUNC(fout)
    s.next_in = base if first else None
    s.avail_in = first
    rc = L.inflateBack(C.byref(s), C.cast(fi, C.c_void_p), None, C.cast(fo, C.c_void_p), None)
    unused = s.avail_in if s.next_in else -1
    null_in = not s.next_in
    rc2 = L.inflateBackEnd(C.byref(s))
    return rc0, rc, bytes(out), unused, null_in, rc2, ncall[0]
