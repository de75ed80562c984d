"""Regenerate tests/golden/zstream_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so, `make -C oracle ref`):

    python tests/golden/make_zstream_golden.py

Scripted z_stream sessions over the reference's deflateSetDictionary,
deflateTune, deflateParams, deflatePrime and deflateSetHeader (deflate.c),
run by tests/zhelpers.run_zsession: each fixture records the session (ops with
data given as tests/datagen.py specs), the reference's return code of every op
and the stream's length and sha256.  Only sessions whose changes fall where
libzgpu.so's model is exact (zgpu_zlib.h) are included; tests/test_gpu_zstream.py
replays them on the GPU library.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import datagen  # noqa: E402
from zhelpers import Reference, run_zsession  # noqa: E402


def spec_bytes(x):
    if x[0] == "gen":
        d = datagen.make(x[1], x[2], x[3])
        return d[x[4]: x[5]] if len(x) > 4 else d
    return bytes.fromhex(x[1])


def materialize(ops):
    out = []
    for op in ops:
        if op[0] in ("dict",):
            out.append((op[0], spec_bytes(op[1])))
        elif op[0] == "deflate":
            out.append(("deflate", spec_bytes(op[1]), op[2]))
        elif op[0] == "header":
            f = dict(op[1])
            for k in ("extra", "name", "comment"):
                if k in f:
                    f[k] = bytes.fromhex(f[k])
            out.append(("header", f))
        else:
            out.append(tuple(op))
    return out


def sessions():
    S = []
    text = ["gen", "text", 150000, 21]
    mix = ["gen", "mix", 200000, 22]
    d_small = ["gen", "text", 300, 31]
    d_mid = ["gen", "text", 9000, 32]
    d_win = ["gen", "mix", 32768, 33]
    d_big = ["gen", "text", 50000, 34]
    # deflateSetDictionary before the first deflate(): zlib and raw wrappers,
    # fast and slow levels, strategies, dictionary sizes up to beyond the window
    for level in (1, 3, 4, 6, 9):
        for wb in (15, -15, 11):
            for d in (d_small, d_mid, d_win):
                S.append({"name": f"dict-L{level}-w{wb}-{d[2]}", "ops": [
                    ["init", level, wb, 8, 0], ["dict", d], ["deflate", text, 4]]})
    for strategy in (1, 2, 3, 4):
        S.append({"name": f"dict-L6-s{strategy}", "ops": [
            ["init", 6, 15, 8, strategy], ["dict", d_mid], ["deflate", mix, 4]]})
    S.append({"name": "dict-big-raw", "ops": [["init", 6, -15, 8, 0], ["dict", d_big], ["deflate", text, 4]]})
    S.append({"name": "dict-two", "ops": [["init", 6, 15, 8, 0], ["dict", d_small], ["dict", d_mid],
                                          ["deflate", text, 4]]})
    S.append({"name": "dict-flushes", "ops": [["init", 6, 15, 8, 0], ["dict", d_mid],
                                              ["deflate", ["gen", "text", 150000, 21, 0, 70000], 2],
                                              ["deflate", ["gen", "text", 150000, 21, 70000, 150000], 4]]})
    S.append({"name": "dict-L2-flushes", "ops": [["init", 2, 15, 8, 0], ["dict", d_mid],
                                                 ["deflate", ["gen", "mix", 200000, 22, 0, 90000], 1],
                                                 ["deflate", ["gen", "mix", 200000, 22, 90000, 200000], 4]]})
    S.append({"name": "dict-gzip-refused", "ops": [["init", 6, 31, 8, 0], ["dict", d_mid], ["deflate", text, 4]]})
    S.append({"name": "dict-after-deflate-refused", "ops": [["init", 6, 15, 8, 0],
                                                            ["deflate", ["gen", "text", 1000, 3], 0],
                                                            ["dict", d_mid], ["deflate", text, 4]]})
    # deflateTune before data and after a flush
    for level, t in ((6, (4, 4, 8, 4)), (6, (8, 16, 258, 0)), (6, (1, 300, 258, 100)), (9, (32, 258, 258, 8192)),
                     (4, (2, 10, 20, 5)), (2, (2, 6, 12, 16)), (1, (8, 3, 300, 2)), (6, (0, 0, 0, 1)),
                     (5, (300, 8, 40, 64))):
        S.append({"name": f"tune-L{level}-{'-'.join(map(str, t))}", "ops": [
            ["init", level, 15, 8, 0], ["tune"] + list(t), ["deflate", mix, 4]]})
    S.append({"name": "tune-after-flush", "ops": [
        ["init", 6, 15, 8, 0], ["deflate", ["gen", "mix", 200000, 22, 0, 100000], 2],
        ["tune", 4, 6, 32, 16], ["deflate", ["gen", "mix", 200000, 22, 100000, 200000], 4]]})
    # deflateParams: before data, after a flush, strategy switches with their own Z_BLOCK
    for a, b in ((6, 1), (1, 9), (6, 0), (0, 6), (9, 4)):
        S.append({"name": f"params-start-{a}-{b}", "ops": [
            ["init", a, 15, 8, 0], ["params", b, 0], ["deflate", text, 4]]})
    S.append({"name": "params-after-flush-6-9", "ops": [
        ["init", 6, 15, 8, 0], ["deflate", ["gen", "mix", 200000, 22, 0, 100000], 3],
        ["params", 9, 0], ["deflate", ["gen", "mix", 200000, 22, 100000, 200000], 4]]})
    S.append({"name": "params-after-flush-2-1", "ops": [
        ["init", 2, 15, 8, 0], ["deflate", ["gen", "text", 150000, 21, 0, 60000], 2],
        ["params", 1, 0], ["deflate", ["gen", "text", 150000, 21, 60000, 150000], 4]]})
    S.append({"name": "params-strategy-block", "ops": [
        ["init", 6, 15, 8, 0], ["deflate", ["gen", "mix", 200000, 22, 0, 120000], 0],
        ["params", 6, 1], ["deflate", ["gen", "mix", 200000, 22, 120000, 200000], 4]]})
    S.append({"name": "params-fixed-block", "ops": [
        ["init", 4, -15, 8, 0], ["deflate", ["gen", "text", 150000, 21, 0, 50000], 0],
        ["params", 5, 4], ["deflate", ["gen", "text", 150000, 21, 50000, 150000], 4]]})
    # deflatePrime
    for wb in (-15, 15):
        for bits, val in ((1, 1), (3, 5), (8, 0xa5), (11, 0x5a5), (16, 0xbeef), (0, 0)):
            S.append({"name": f"prime-w{wb}-{bits}", "ops": [
                ["init", 6, wb, 8, 0], ["prime", bits, val], ["deflate", text, 4]]})
    S.append({"name": "prime-twice-L1", "ops": [["init", 1, -15, 8, 0], ["prime", 5, 19], ["prime", 7, 100],
                                                ["deflate", mix, 4]]})
    S.append({"name": "prime-L0", "ops": [["init", 0, -15, 8, 0], ["prime", 6, 33], ["deflate", text, 4]]})
    S.append({"name": "prime-after-partial", "ops": [
        ["init", 6, -15, 8, 0], ["deflate", ["gen", "text", 150000, 21, 0, 40000], 1],
        ["prime", 5, 9], ["deflate", ["gen", "text", 150000, 21, 40000, 150000], 4]]})
    S.append({"name": "prime-bad", "ops": [["init", 6, -15, 8, 0], ["prime", 17, 1], ["prime", -1, 1],
                                           ["deflate", text, 4]]})
    # deflateSetHeader
    hdrs = [{"text": 1, "time": 1234567890, "os": 3},
            {"time": 7, "os": 11, "name": b"file.txt".hex(), "comment": b"a comment".hex()},
            {"text": 0, "time": 99, "os": 255, "extra": bytes(range(40)).hex(), "hcrc": 1},
            {"text": 1, "time": 0xffffffff, "os": 0, "extra": b"AB\x03\x00xyz".hex(), "name": b"n".hex(),
             "comment": b"".hex(), "hcrc": 1}]
    for i, h in enumerate(hdrs):
        for level in (1, 6, 9):
            S.append({"name": f"header-{i}-L{level}", "ops": [
                ["init", level, 31, 8, 0], ["header", h], ["deflate", text, 4]]})
    S.append({"name": "header-on-zlib-refused", "ops": [["init", 6, 15, 8, 0], ["header", hdrs[0]],
                                                        ["deflate", text, 4]]})
    # deflateTune's max_lazy is deflate_fast's max_insert_length: long matches
    # inserted position by position at levels 1..3
    runs = ["gen", "runs", 120000, 41]
    for level in (1, 2, 3):
        for lazy in (40, 100, 258):
            for data in (text, runs):
                S.append({"name": f"tune-fast-insert-L{level}-{lazy}-{data[1]}", "ops": [
                    ["init", level, 15, 8, 0], ["tune", 4, lazy, 258, 64], ["deflate", data, 4]]})
    S += sessions_r3()
    return S


def sessions_r3():
    """Round 3: z_stream controls with input pending and deflateBound after the
    state changes (deflate.c:760-905)."""
    S = []
    text = ["gen", "text", 150000, 21]
    mix = ["gen", "mix", 200000, 22]

    def part(d, a, b):
        return d[:4] + [a, b]
    # a level change within the function while the last Z_NO_FLUSH call's
    # input waits in the window: the decisions from where the parse stands
    # read the new row
    for a, b in ((6, 9), (9, 4), (4, 6), (5, 8), (7, 6), (6, 5), (1, 3), (3, 1), (2, 1)):
        for cut in (100, 5000, 77777):
            d = mix if a >= 4 else text
            S.append({"name": f"params-pending-{a}-{b}-{cut}", "ops": [
                ["init", a, 15, 8, 0], ["deflate", part(d, 0, cut), 0], ["params", b, 0],
                ["deflate", part(d, cut, d[2]), 4]]})
    for level, t in ((6, (4, 4, 16, 16)), (6, (32, 128, 258, 1024)), (9, (8, 16, 128, 128)),
                     (4, (2, 6, 40, 8)), (1, (4, 20, 32, 32)), (2, (2, 4, 8, 4)), (8, (8, 8, 8, 0))):
        S.append({"name": f"tune-pending-L{level}-{'-'.join(map(str, t))}", "ops": [
            ["init", level, 15, 8, 0], ["deflate", part(mix, 0, 64000), 0], ["tune"] + list(t),
            ["deflate", part(mix, 64000, 200000), 4]]})
    # several changes, flushes in between, raw and gzip wrappers
    for wb, lv in ((15, 6), (-15, 4), (31, 9), (15, 2)):
        S.append({"name": f"params-many-w{wb}-L{lv}", "ops": [
            ["init", lv, wb, 8, 0], ["deflate", part(mix, 0, 30000), 0],
            ["params", 9 if lv >= 4 else 1, 0], ["deflate", part(mix, 30000, 61000), 0],
            ["tune", 8, 16, 64, 32], ["deflate", part(mix, 61000, 90000), 2],
            ["params", 5 if lv >= 4 else 3, 0], ["deflate", part(mix, 90000, 120000), 0],
            ["params", 6 if lv >= 4 else 2, 0], ["deflate", part(mix, 120000, 200000), 4]]})
    # a change while the last call stopped on a full output buffer (the parse
    # stands at the end of the last block it handed out)
    for lv, nb in ((6, 9), (9, 5), (2, 3), (1, 2)):
        for out in (2000, 20000):
            S.append({"name": f"params-paused-{lv}-{nb}-{out}", "ops": [
                ["init", lv, 15, 8, 0], ["deflate", part(mix, 0, 150000), 0, out], ["params", nb, 0],
                ["deflate", part(mix, 150000, 200000), 4, out]]})
        S.append({"name": f"tune-paused-{lv}", "ops": [
            ["init", lv, 15, 8, 0], ["deflate", part(mix, 0, 150000), 0, 3000], ["tune", 4, 8, 16, 8],
            ["deflate", part(mix, 150000, 200000), 4, 3000]]})
    # deflateBound after the state changes (deflate.c:842-905: the DICTID once
    # strstart != 0, the gzip header's fields)
    S.append({"name": "bound-states-zlib", "ops": [
        ["init", 6, 15, 8, 0], ["bound", 100000], ["deflate", part(text, 0, 100), 0], ["bound", 100000],
        ["deflate", part(text, 100, 5000), 0], ["bound", 100000], ["deflate", part(text, 5000, 9000), 2],
        ["bound", 100000], ["deflate", part(text, 9000, 12000), 3], ["bound", 100000],
        ["deflate", part(text, 12000, 150000), 4], ["bound", 100000]]})
    S.append({"name": "bound-dict", "ops": [
        ["init", 6, 15, 8, 0], ["bound", 5000], ["dict", ["gen", "text", 300, 31]], ["bound", 5000],
        ["deflate", text, 4]]})
    S.append({"name": "bound-dict-raw-w12", "ops": [
        ["init", 9, -12, 8, 0], ["dict", ["gen", "text", 9000, 32]], ["bound", 5000], ["deflate", text, 4]]})
    hdr = {"text": 1, "time": 7, "os": 11, "name": b"file.txt".hex(), "comment": b"a comment".hex(),
           "extra": bytes(range(40)).hex(), "hcrc": 1}
    S.append({"name": "bound-gzip-header", "ops": [
        ["init", 6, 31, 8, 0], ["bound", 77777], ["header", hdr], ["bound", 77777], ["deflate", text, 4],
        ["bound", 77777]]})
    S.append({"name": "bound-gzip-header-w10", "ops": [
        ["init", 3, 26, 5, 0], ["header", hdr], ["bound", 77777], ["deflate", text, 4]]})
    for lv, st in ((0, 0), (1, 2), (4, 3)):
        S.append({"name": f"bound-L{lv}-s{st}", "ops": [
            ["init", lv, 15, 8, st], ["deflate", part(text, 0, 200), 0], ["bound", 1000],
            ["deflate", part(text, 200, 300), 0], ["bound", 1000], ["deflate", part(text, 300, 150000), 4]]})
    # deflateParams switching the level's function after data (deflate.c:777-803):
    # the Z_BLOCK flush, then the new function over the same window -- deflate_fast
    # inserts selectively, deflate_slow everything, deflate_stored nothing until
    # fill_window hashes its s->insert strings; gzsetparams' pattern
    # (gzwrite.c:587: a Z_BLOCK flush of the pending input, then deflateParams)
    chains = [(6, 1), (1, 6), (6, 0), (0, 6), (1, 0), (0, 1), (3, 9), (9, 2), (2, 4)]
    for a, b in chains:
        for wb in (15, -15):
            S.append({"name": f"switch-{a}-{b}-w{wb}", "ops": [
                ["init", a, wb, 8, 0], ["deflate", part(mix, 0, 70000), 0], ["params", b, 0],
                ["deflate", part(mix, 70000, 200000), 4]]})
    for seq in ((1, 0, 1), (6, 0, 6), (1, 6, 1), (6, 1, 6), (9, 2, 0, 7), (0, 3, 0, 5), (2, 0, 8, 1)):
        ops = [["init", seq[0], 15, 8, 0]]
        step = 200000 // len(seq)
        for i, lv in enumerate(seq):
            if i:
                ops.append(["params", lv, 0])
            ops.append(["deflate", part(mix, i * step, (i + 1) * step if i + 1 < len(seq) else 200000),
                        4 if i + 1 == len(seq) else 0])
        S.append({"name": "switch-seq-" + "-".join(map(str, seq)), "ops": ops})
    for a, b in ((6, 1), (1, 6), (0, 6), (6, 0), (2, 0)):
        S.append({"name": f"gzsetparams-{a}-{b}", "ops": [
            ["init", a, 31, 8, 0], ["deflate", part(text, 0, 40000), 0], ["deflate", part(text, 40000, 41000), 5],
            ["params", b, 0], ["deflate", part(text, 41000, 150000), 4]]})
        S.append({"name": f"switch-small-out-{a}-{b}", "ops": [
            ["init", a, 15, 8, 0], ["deflate", part(mix, 0, 90000), 0, 3000], ["params", b, 0],
            ["deflate", part(mix, 90000, 200000), 4, 3000]]})
    for a, b, wb, ml in ((6, 1, 10, 5), (1, 6, 12, 9), (0, 2, 9, 1), (3, 0, 11, 7)):
        S.append({"name": f"switch-{a}-{b}-w{wb}-m{ml}", "ops": [
            ["init", a, wb, ml, 0], ["deflate", part(mix, 0, 50000), 0], ["params", b, 0],
            ["deflate", part(mix, 50000, 130000), 2], ["params", a, 0], ["deflate", part(mix, 130000, 200000), 4]]})
    # small stretches between switches (the window mixes functions)
    S.append({"name": "switch-short-stretches", "ops": [
        ["init", 1, 15, 8, 0], ["deflate", part(text, 0, 20000), 0], ["params", 0, 0],
        ["deflate", part(text, 20000, 20100), 0], ["params", 6, 0], ["deflate", part(text, 20100, 21000), 0],
        ["params", 2, 0], ["deflate", part(text, 21000, 21500), 0], ["params", 7, 0],
        ["deflate", part(text, 21500, 150000), 4]]})
    # deflateSetDictionary on a raw stream after a flush (lookahead 0), at level 0
    # (deflate_stored keeps no lookahead: any time, unsent window bytes dropped),
    # and a zlib stream's dictionary at level 0 (deflate.c:550-613)
    d_small = ["gen", "text", 300, 31]
    d_mid = ["gen", "text", 9000, 32]
    d_big = ["gen", "text", 50000, 34]
    for lv in (1, 2, 6, 9):
        for d in (d_small, d_mid, d_big):
            S.append({"name": f"dict-raw-after-flush-L{lv}-{d[2]}", "ops": [
                ["init", lv, -15, 8, 0], ["deflate", part(text, 0, 60000), 2], ["dict", d],
                ["deflate", part(text, 60000, 150000), 4]]})
    S.append({"name": "dict-raw-after-noflush-refused", "ops": [
        ["init", 6, -15, 8, 0], ["deflate", part(text, 0, 60000), 0], ["dict", d_mid],
        ["deflate", part(text, 60000, 150000), 4]]})
    S.append({"name": "dict-raw-twice-flushes", "ops": [
        ["init", 4, -15, 8, 0], ["dict", d_mid], ["deflate", part(mix, 0, 50000), 3], ["dict", d_small],
        ["deflate", part(mix, 50000, 120000), 5], ["dict", d_big], ["deflate", part(mix, 120000, 200000), 4]]})
    for wb in (15, -15, -10):
        for d in (d_small, d_big):
            S.append({"name": f"dict-L0-w{wb}-{d[2]}", "ops": [
                ["init", 0, wb, 8, 0], ["dict", d], ["deflate", text, 4]]})
    S.append({"name": "dict-L0-raw-midstream", "ops": [
        ["init", 0, -15, 8, 0], ["deflate", part(text, 0, 70000), 0, 5000], ["dict", d_mid],
        ["deflate", part(text, 70000, 150000), 4, 5000]]})
    S.append({"name": "dict-L0-then-L6", "ops": [
        ["init", 0, -15, 8, 0], ["deflate", part(text, 0, 30000), 2], ["dict", d_mid], ["params", 6, 0],
        ["deflate", part(text, 30000, 150000), 4]]})
    S.append({"name": "dict-L1-then-L0-dict-L1", "ops": [
        ["init", 1, -15, 8, 0], ["deflate", part(text, 0, 30000), 0], ["params", 0, 0], ["dict", d_small],
        ["deflate", part(text, 30000, 40000), 5], ["params", 1, 0], ["deflate", part(text, 40000, 150000), 4]]})
    # strategy changes within deflate_slow / deflate_fast
    for a, sa, sb in ((6, 0, 1), (6, 1, 4), (4, 4, 0), (2, 0, 1), (1, 4, 0)):
        S.append({"name": f"strategy-{a}-{sa}-{sb}", "ops": [
            ["init", a, 15, 8, sa], ["deflate", part(mix, 0, 80000), 0], ["params", a, sb],
            ["deflate", part(mix, 80000, 200000), 4]]})
    # deflatePrime with input pending (deflate.c:731-757): the bits go into
    # bi_buf at once, after the blocks flushed so far and ahead of the block
    # in progress
    for lv, wb, st in ((6, -15, 0), (6, 15, 0), (1, -15, 0), (3, 31, 0), (9, -15, 1), (5, -15, 2), (4, -15, 3),
                       (2, -15, 2)):
        d = mix if lv >= 4 else text
        S.append({"name": f"prime-pending-L{lv}-w{wb}-s{st}", "ops": [
            ["init", lv, wb, 8, st], ["deflate", part(d, 0, 70000), 0], ["prime", 5, 19],
            ["deflate", part(d, 70000, d[2]), 4]]})
    S.append({"name": "prime-pending-twice", "ops": [
        ["init", 6, -15, 8, 0], ["deflate", part(mix, 0, 50000), 0], ["prime", 3, 5], ["prime", 16, 0xBEEF],
        ["deflate", part(mix, 50000, 120000), 0], ["prime", 7, 77], ["deflate", part(mix, 120000, 200000), 4]]})
    S.append({"name": "prime-pending-then-sync", "ops": [
        ["init", 6, -15, 8, 0], ["deflate", part(mix, 0, 90000), 0], ["prime", 6, 44],
        ["deflate", part(mix, 90000, 150000), 2], ["deflate", part(mix, 150000, 200000), 4]]})
    S.append({"name": "prime-pending-zero-bits", "ops": [
        ["init", 6, -15, 8, 0], ["deflate", part(mix, 0, 60000), 0], ["prime", 0, 1],
        ["deflate", part(mix, 60000, 200000), 4]]})
    S.append({"name": "prime-pending-small-calls", "ops": [
        ["init", 6, -15, 8, 0], ["deflate", part(mix, 0, 80000), 0, 3000], ["prime", 9, 300],
        ["deflate", part(mix, 80000, 200000), 4, 3000]]})
    S.append({"name": "prime-pending-L1-short", "ops": [
        ["init", 1, -15, 8, 0], ["deflate", part(text, 0, 500), 0], ["prime", 4, 3],
        ["deflate", part(text, 500, 150000), 4]]})
    return S


def main():
    ref = Reference()
    out = {"reference": ref.version.decode(), "sessions": []}
    for sess in sessions():
        rcs, z = run_zsession(ref.L, materialize(sess["ops"]))
        out["sessions"].append({"name": sess["name"], "ops": sess["ops"], "rcs": rcs, "len": len(z),
                                "sha256": hashlib.sha256(z).hexdigest()})
    path = os.path.join(HERE, "zstream_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(out['sessions'])} sessions")


if __name__ == "__main__":
    main()
