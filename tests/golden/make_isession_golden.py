"""Golden z_stream inflate sessions (inflate(Z_BLOCK), inflateGetHeader,
inflateSync, inflateCopy) from the compiled reference (oracle/_ref/libzref.so,
built from /root/reference by oracle/Makefile).  Each session's compressed
input is built by build_z() from a spec with Python's zlib (system zlib) and
a hand-made gzip header where one is needed -- no stream made by the reference
is stored.  The fixture keeps the spec, the ops, and what the reference did:
per-op results, each stream's output (length, sha256) and the gz_header fields.
Run from tests/golden: python3 make_isession_golden.py"""
import hashlib
import json
import os
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import datagen  # noqa: E402
from zhelpers import Reference, run_iops  # noqa: E402

Z_NO_FLUSH, Z_SYNC_FLUSH, Z_FULL_FLUSH, Z_FINISH, Z_BLOCK, Z_TREES = 0, 2, 3, 4, 5, 6


def build_z(spec):
    """spec: data (kind, n, seed), level, strategy, fmt ("zlib", "gzip", "raw"),
    cuts [[position, flush]] (flush points), gz (header fields for a hand-made
    gzip header: text, time, xfl, os, extra, name, comment (hex), hcrc)."""
    data = datagen.make(*spec["data"])
    fmt = spec.get("fmt", "zlib")
    wb = {"zlib": 15, "raw": -15, "gzip": -15}[fmt]
    if "zdict" in spec:
        c = zlib.compressobj(spec.get("level", 6), zlib.DEFLATED, wb, 8, spec.get("strategy", 0),
                             zdict=datagen.make(*spec["zdict"]))
    else:
        c = zlib.compressobj(spec.get("level", 6), zlib.DEFLATED, wb, 8, spec.get("strategy", 0))
    body, pos = b"", 0
    for at, fl in spec.get("cuts", []):
        body += c.compress(data[pos:at]) + c.flush(fl)
        pos = at
    body += c.compress(data[pos:]) + c.flush(Z_FINISH)
    if fmt != "gzip":
        if "cinfo" in spec:                  # a header that claims a smaller window than the stream uses
            cmf = (spec["cinfo"] << 4) | 8
            flg = body[1] & 0xe0
            flg |= 31 - ((cmf * 256 + flg) % 31)
            body = bytes([cmf, flg]) + body[2:]
        return body
    g = spec.get("gz", {})
    flg = (1 if g.get("text") else 0) | (2 if g.get("hcrc") else 0) | (4 if "extra" in g else 0) | \
          (8 if "name" in g else 0) | (16 if "comment" in g else 0)
    h = bytes([0x1f, 0x8b, 8, flg]) + struct.pack("<I", g.get("time", 0)) + bytes([g.get("xfl", 0), g.get("os", 3)])
    if "extra" in g:
        x = bytes.fromhex(g["extra"])
        h += struct.pack("<H", len(x)) + x
    for k in ("name", "comment"):
        if k in g:
            h += bytes.fromhex(g[k]) + b"\0"
    if g.get("hcrc"):
        h += struct.pack("<H", zlib.crc32(h) & 0xffff)
    return h + body + struct.pack("<II", zlib.crc32(data), len(data) & 0xffffffff)


def feed_loop(z_len, chunk, flush, out=1 << 20):
    ops = []
    for _ in range((z_len + chunk - 1) // chunk + 1):
        ops += [["feed", chunk], ["loop", flush, out]]
    return ops


def sessions():
    S = []
    mix = ["mix", 200000, 41]
    text = ["text", 120000, 42]
    # inflate(Z_BLOCK): stop at every block boundary, after the header first
    for fmt, wb in (("zlib", 15), ("gzip", 31), ("raw", -15), ("gzip", 47), ("zlib", 47)):
        for level, st in ((6, 0), (1, 0), (9, 0), (0, 0), (6, 4), (6, 2)):
            spec = {"data": mix, "level": level, "strategy": st, "fmt": fmt,
                    "cuts": [[30000, Z_SYNC_FLUSH], [90000, Z_FULL_FLUSH], [91000, Z_SYNC_FLUSH]]}
            S.append({"name": f"block-{fmt}-w{wb}-L{level}-s{st}", "spec": spec,
                      "ops": [["init", wb], ["feed", 1 << 30], ["loop", Z_BLOCK, 1 << 20]]})
    for chunk in (1, 7, 1000, 65536):
        spec = {"data": text, "level": 6, "fmt": "zlib", "cuts": [[50000, Z_SYNC_FLUSH]]}
        S.append({"name": f"block-chunks-{chunk}", "spec": spec,
                  "ops": [["init", 15]] + feed_loop(80000 if chunk > 1 else 3000, chunk, Z_BLOCK)})
    S.append({"name": "block-then-finish", "spec": {"data": mix, "fmt": "zlib", "cuts": [[60000, Z_FULL_FLUSH]]},
              "ops": [["init", 15], ["feed", 1 << 30], ["inflate", Z_BLOCK, 1 << 20], ["inflate", Z_BLOCK, 1 << 20],
                      ["inflate", Z_FINISH, 1 << 20]]})
    # inflateGetHeader: fields as the header arrives, truncation at the max sizes
    gzs = [
        {"text": 1, "time": 0x5f5e0ff1, "xfl": 2, "os": 11, "name": b"file.txt".hex(), "comment": b"a comment".hex()},
        {"time": 7, "extra": (b"AB\x04\x00wxyz" + bytes(range(40))).hex(), "hcrc": 1},
        {"name": (b"n" * 300).hex(), "comment": b"".hex(), "hcrc": 1, "os": 255},
        {},
    ]
    for i, gz in enumerate(gzs):
        for maxes in ((64, 64, 64), (4, 3, 2), (1000, 1000, 1000)):
            for chunk in (1 << 30, 5):
                spec = {"data": text, "fmt": "gzip", "gz": gz}
                ops = [["init", 31], ["header"] + list(maxes)]
                ops += [["feed", 1 << 30], ["loop", Z_NO_FLUSH, 1 << 20]] if chunk > 1000 else \
                    feed_loop(400, chunk, Z_NO_FLUSH) + [["feed", 1 << 30], ["loop", Z_NO_FLUSH, 1 << 20]]
                S.append({"name": f"gethdr-{i}-{'-'.join(map(str, maxes))}-c{min(chunk, 9999)}", "spec": spec,
                          "ops": ops})
    S.append({"name": "gethdr-zlib-auto", "spec": {"data": text, "fmt": "zlib"},
              "ops": [["init", 47], ["header", 8, 8, 8], ["feed", 1 << 30], ["loop", Z_NO_FLUSH, 1 << 20]]})
    S.append({"name": "gethdr-zlib-only", "spec": {"data": text, "fmt": "zlib"},
              "ops": [["init", 15], ["header", 8, 8, 8], ["feed", 1 << 30], ["loop", Z_NO_FLUSH, 1 << 20]]})
    S.append({"name": "gethdr-block", "spec": {"data": text, "fmt": "gzip", "gz": gzs[0],
                                               "cuts": [[40000, Z_SYNC_FLUSH]]},
              "ops": [["init", 31], ["header", 64, 64, 64], ["feed", 1 << 30], ["loop", Z_BLOCK, 1 << 20]]})
    # inflateSync: skip a damaged stretch to the next full flush point
    for fmt, wb in (("zlib", 15), ("gzip", 31), ("raw", -15)):
        cuts = [[40000, Z_FULL_FLUSH], [100000, Z_FULL_FLUSH], [150000, Z_FULL_FLUSH]]
        spec = {"data": mix, "fmt": fmt, "cuts": cuts}
        for skip in (10, 5000, 40000):
            S.append({"name": f"sync-{fmt}-skip{skip}", "spec": spec, "ops": [
                ["init", wb], ["feed", 2], ["inflate", Z_NO_FLUSH, 1 << 20], ["skip", skip], ["feed", 1 << 30],
                ["sync"], ["loop", Z_NO_FLUSH, 1 << 20], ["inflate", Z_FINISH, 1 << 20]]})
        S.append({"name": f"sync-{fmt}-first", "spec": spec, "ops": [
            ["init", wb], ["skip", 3000], ["feed", 1 << 30], ["sync"], ["loop", Z_NO_FLUSH, 1 << 20]]})
        S.append({"name": f"sync-{fmt}-split", "spec": spec, "ops": [
            ["init", wb], ["feed", 2], ["inflate", Z_NO_FLUSH, 1 << 20], ["skip", 20000],
            ["feed", 3], ["sync"], ["feed", 9000], ["sync"], ["feed", 1 << 30], ["sync"],
            ["loop", Z_NO_FLUSH, 1 << 20]]})
    S.append({"name": "sync-none", "spec": {"data": text, "fmt": "zlib"}, "ops": [
        ["init", 15], ["feed", 2], ["inflate", Z_NO_FLUSH, 1 << 20], ["sync"], ["skip", 100], ["feed", 1 << 30],
        ["sync"]]})
    # inflateSync after a call whose input ended inside a flush marker's LEN /
    # NLEN: the reference searches the whole bytes in its bit buffer first
    # (inflate.c:1388-1398), so the marker it was reading is found (round 5)
    for fmt, wb in (("zlib", 15), ("gzip", 31), ("raw", -15)):
        spec = {"data": mix, "fmt": fmt, "cuts": [[40000, Z_FULL_FLUSH], [100000, Z_SYNC_FLUSH]]}
        z = build_z(spec)
        m = z.find(b"\x00\x00\xff\xff", 100)
        for k in (1, 2, 3, 4):
            S.append({"name": f"sync-held-{fmt}-{k}", "spec": spec, "ops": [
                ["init", wb], ["feed", m + k], ["inflate", Z_NO_FLUSH, 1 << 20], ["sync"], ["feed", 3], ["sync"],
                ["feed", 1 << 30], ["sync"], ["loop", Z_NO_FLUSH, 1 << 20]]})
    # output space smaller than the stream's output, all the input at once: each
    # call stops reading where inflate.c stops for room (round 5)
    for fmt, wb in (("zlib", 15), ("gzip", 31), ("raw", -15)):
        for data, out in ((["text", 6000, 61], 1), (["mix", 60000, 62], 997), (mix, 65536)):
            spec = {"data": data, "fmt": fmt, "cuts": [[len(datagen.make(*data)) // 2, Z_SYNC_FLUSH]]}
            S.append({"name": f"smallout-{fmt}-{out}", "spec": spec,
                      "ops": [["init", wb], ["feed", 1 << 30], ["loop", Z_NO_FLUSH, out]]})
            S.append({"name": f"smallout-block-{fmt}-{out}", "spec": spec,
                      "ops": [["init", wb], ["feed", 1 << 30], ["loop", Z_BLOCK, out]]})
        S.append({"name": f"smallout-pieces-{fmt}", "spec": {"data": mix, "fmt": fmt, "cuts": [[70000, Z_SYNC_FLUSH]]},
                  "ops": [["init", wb]] + feed_loop(30000, 7000, Z_NO_FLUSH, 3001) + [["feed", 1 << 30],
                                                                                  ["loop", Z_NO_FLUSH, 1 << 20]]})
    # inflate(Z_TREES): Z_BLOCK's stops and one after each block header, before
    # its first code (mode LEN_ / COPY_, data_type + 256; round 5)
    for fmt, wb in (("zlib", 15), ("gzip", 31), ("raw", -15)):
        for level, st in ((6, 0), (0, 0), (6, 4), (1, 2)):
            spec = {"data": mix, "level": level, "strategy": st, "fmt": fmt,
                    "cuts": [[30000, Z_SYNC_FLUSH], [90000, Z_FULL_FLUSH], [91000, Z_SYNC_FLUSH]]}
            S.append({"name": f"trees-{fmt}-L{level}-s{st}", "spec": spec,
                      "ops": [["init", wb], ["feed", 1 << 30], ["loop", Z_TREES, 1 << 20]]})
        spec = {"data": text, "level": 6, "fmt": fmt, "cuts": [[50000, Z_SYNC_FLUSH]]}
        S.append({"name": f"trees-chunks-{fmt}", "spec": spec,
                  "ops": [["init", wb]] + feed_loop(40000, 997, Z_TREES, 4001) + [["feed", 1 << 30],
                                                                                ["loop", Z_TREES, 1 << 20]]})
        S.append({"name": f"trees-mixed-{fmt}", "spec": spec, "ops": [
            ["init", wb], ["feed", 30000], ["inflate", Z_NO_FLUSH, 5000], ["inflate", Z_TREES, 1 << 20],
            ["inflate", Z_TREES, 1 << 20], ["inflate", Z_BLOCK, 100], ["inflate", Z_TREES, 1 << 20],
            ["feed", 1 << 30], ["loop", Z_TREES, 1 << 20]]})
    # inflateCopy: two streams from one state
    for at in (2, 30000, 1 << 30):
        S.append({"name": f"copy-at-{at}", "spec": {"data": mix, "fmt": "zlib", "cuts": [[70000, Z_SYNC_FLUSH]]},
                  "ops": [["init", 15], ["feed", at], ["loop", Z_NO_FLUSH, 1 << 20], ["copy"], ["use", 1],
                          ["feed", 1 << 30], ["loop", Z_NO_FLUSH, 1 << 20], ["use", 0], ["feed", 1 << 30],
                          ["loop", Z_NO_FLUSH, 1 << 20]]})
    S.append({"name": "copy-after-block", "spec": {"data": mix, "fmt": "gzip", "cuts": [[70000, Z_SYNC_FLUSH]]},
              "ops": [["init", 31], ["feed", 1 << 30], ["inflate", Z_BLOCK, 1 << 20], ["inflate", Z_BLOCK, 1 << 20],
                      ["copy"], ["use", 1], ["loop", Z_NO_FLUSH, 1 << 20], ["use", 0], ["loop", Z_BLOCK, 1 << 20]]})
    # inflateSetDictionary keeps 1 << windowBits of inflateInit2_ (not of the
    # header's CINFO): a stream whose header claims a 512-byte window but which
    # reaches 30 KiB into the dictionary decodes
    for cinfo in (1, 7):
        for wb in (15, 0):
            S.append({"name": f"dict-window-cinfo{cinfo}-w{wb}", "spec": {
                "data": ["text", 60000, 51], "zdict": ["text", 32768, 52], "fmt": "zlib", "cinfo": cinfo},
                "ops": [["init", wb], ["feed", 1 << 30], ["loop", Z_NO_FLUSH, 1 << 20], ["dict", ["text", 32768, 52]],
                        ["loop", Z_NO_FLUSH, 1 << 20]]})
    return S


def run(L, sess):
    z = build_z(sess["spec"])
    res, outs, hdr = run_iops(L, z, sess["ops"])
    return {"res": res, "outs": [[len(o), hashlib.sha256(o).hexdigest()] for o in outs], "hdr": hdr}


def main():
    ref = Reference()
    out = {"reference": ref.version.decode(), "sessions": []}
    for sess in sessions():
        r = run(ref.L, sess)
        out["sessions"].append(dict(sess, **r))
    path = os.path.join(HERE, "isession_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(out['sessions'])} sessions")


if __name__ == "__main__":
    main()
