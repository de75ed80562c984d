"""Golden sessions of the zlib.h calls added in round 4, from the compiled
reference (oracle/_ref/libzref.so, built from /root/reference by
oracle/Makefile): deflateUsed, deflateGetDictionary, deflateResetKeep,
inflateReset2, inflateResetKeep, inflatePrime, inflateGetDictionary,
inflateSyncPoint, inflateUndermine, inflateValidate, inflateMark,
inflateCodesUsed and inflateBackInit_ / inflateBack / inflateBackEnd.

Every compressed input is rebuilt from its spec with Python's zlib (system
zlib; build_z in make_isession_golden.py) -- no stream made by the reference
is stored, only the ops and what the reference returned (codes, counters,
lengths and sha256 prefixes of outputs and windows).  The same runners
(tests/zhelpers.py run_iops / run_zsession / run_back) replay them against
libzgpu.so on the GPU (tests/test_gpu_zstream.py).
Run from tests/golden: python3 make_api_golden.py"""
import hashlib
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import datagen  # noqa: E402
from make_isession_golden import build_z  # noqa: E402
from zhelpers import Reference, run_back, run_iops, run_zsession  # noqa: E402

Z_NO_FLUSH, Z_PARTIAL_FLUSH, Z_SYNC_FLUSH, Z_FULL_FLUSH, Z_FINISH, Z_BLOCK = 0, 1, 2, 3, 4, 5
BIG = 1 << 30


def build(spec):
    """build_z, plus: "concat" (several specs back to back), "xor_tail" (flip
    the last byte: a wrong check value), "zdict_tail" (a raw stream
    compressed against the tail of other data), "shift" (the stream from bit k on,
    repacked into bytes, for inflatePrime with its first k bits), "chop" (drop
    the last n bytes), "garbage" (bytes appended after the stream)."""
    if "concat" in spec:
        z = b"".join(build(s) for s in spec["concat"])
    elif "zdict_tail" in spec:                   # a raw stream against the tail of other data
        kind, n, seed, tail = spec["zdict_tail"]
        c = zlib.compressobj(spec.get("level", 6), zlib.DEFLATED, -15, 8, 0,
                             zdict=datagen.make(kind, n, seed)[-tail:])
        z = c.compress(datagen.make(*spec["data"])) + c.flush()
    elif "cwbits" in spec:                       # a raw stream made with a small window
        c = zlib.compressobj(spec.get("level", 6), zlib.DEFLATED, -spec["cwbits"], 8, 0)
        z = c.compress(datagen.make(*spec["data"])) + c.flush()
    else:
        z = build_z(spec)
    if spec.get("xor_tail"):
        z = z[:-1] + bytes([z[-1] ^ 0x5a])
    if spec.get("shift"):
        k = spec["shift"]
        z = (int.from_bytes(z, "little") >> k).to_bytes(len(z), "little")
    if spec.get("chop"):
        z = z[:-spec["chop"]]
    if spec.get("garbage"):
        z = z + bytes(range(spec["garbage"]))
    return z


def prime_value(spec):
    """The first `shift` bits of the unshifted stream (inflatePrime's value)."""
    s = dict(spec)
    k = s.pop("shift")
    z = build(s)
    return int.from_bytes(z[:4], "little") & ((1 << k) - 1)


def sync_point(spec):
    """Bytes of the stream up to a Z_SYNC_FLUSH marker's LEN/NLEN (00 00 ff ff):
    the stored block's header byte is in, its length is not."""
    z = build(spec)
    return z.find(b"\x00\x00\xff\xff", 3)


def watch(k):
    return [["mark"], ["codes"], ["syncpoint"], ["getdict"]][:k]


def inflate_sessions():
    S = []
    text = ["text", 150000, 61]
    mix = ["mix", 200000, 62]
    # the window, inflateMark, inflateCodesUsed and inflateSyncPoint as the
    # input arrives in pieces (ample output space)
    for fmt, wb in (("zlib", 15), ("gzip", 31), ("raw", -15)):
        for data, level in ((text, 6), (mix, 9), (mix, 1)):
            spec = {"data": data, "level": level, "fmt": fmt, "cuts": [[70000, Z_SYNC_FLUSH]]}
            ops = [["init", wb]] + watch(4)
            for _ in range(12):
                ops += [["feed", 3001], ["inflate", Z_NO_FLUSH, 1 << 20]] + watch(4)
            ops += [["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20]] + watch(4)
            S.append({"name": f"watch-{fmt}-{data[0]}-L{level}", "spec": spec, "ops": ops})
    # single bytes across a dynamic block header: CODES table sizes, back counts
    spec = {"data": ["text", 20000, 63], "level": 6, "fmt": "raw"}
    ops = [["init", -15]]
    for _ in range(400):
        ops += [["feed", 1], ["inflate", Z_NO_FLUSH, 1 << 20], ["mark"], ["codes"]]
    S.append({"name": "watch-bytes-raw", "spec": spec, "ops": ops})
    # the window after a one-call Z_FINISH (never made), small output pieces
    for flush in (Z_FINISH, Z_NO_FLUSH):
        S.append({"name": f"getdict-one-call-{flush}", "spec": {"data": text, "fmt": "zlib"},
                  "ops": [["init", 15], ["feed", BIG], ["inflate", flush, 1 << 20], ["getdict"], ["codes"]]})
    S.append({"name": "getdict-after-setdict", "spec": {"data": ["text", 60000, 64], "zdict": ["text", 40000, 65],
                                                         "fmt": "raw"},
              "ops": [["init", -15], ["dict", ["text", 40000, 65]], ["getdict"], ["feed", BIG],
                      ["loop", Z_NO_FLUSH, 1 << 20], ["getdict"]]})
    S.append({"name": "getdict-small-window", "spec": {"data": ["text", 30000, 66], "fmt": "raw"},
              "ops": [["init", -9], ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20], ["getdict"]]})
    # inflateSyncPoint right before a sync marker's LEN/NLEN
    for fmt, wb in (("raw", -15), ("zlib", 15)):
        for level in (6, 1):
            spec = {"data": text, "level": level, "fmt": fmt, "cuts": [[50000, Z_SYNC_FLUSH]]}
            at = sync_point(spec)
            for d in (0, -1, 1, 2):
                S.append({"name": f"syncpoint-{fmt}-L{level}-{d}", "spec": spec,
                          "ops": [["init", wb], ["feed", at + d], ["inflate", Z_NO_FLUSH, 1 << 20], ["syncpoint"],
                                  ["mark"], ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20], ["syncpoint"]]})
    # inflateValidate(0): a wrong check value goes unnoticed, adler keeps its start
    for fmt, wb in (("zlib", 15), ("gzip", 31), ("zlib", 47), ("gzip", 47)):
        for bad in (0, 1):
            for chk in (0, 1):
                spec = {"data": ["mix", 50000, 67], "fmt": fmt, "xor_tail": bad}
                S.append({"name": f"validate-{fmt}-w{wb}-bad{bad}-chk{chk}", "spec": spec,
                          "ops": [["init", wb], ["validate", chk], ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20],
                                  ["adler"]]})
    S.append({"name": "validate-pieces", "spec": {"data": ["mix", 80000, 68], "fmt": "zlib", "xor_tail": 1},
              "ops": [["init", 15], ["validate", 0]] + [["feed", 9000], ["inflate", Z_NO_FLUSH, 1 << 20]] * 12 +
                     [["adler"]]})
    # inflateReset2 turns the check back on after inflateValidate(0) (inflate.c:157,
    # wrap = (windowBits >> 4) + 5); inflateReset keeps it off
    for fmt, wb in (("zlib", 15), ("gzip", 31)):
        for op in (["reset2", wb], ["reset"]):
            S.append({"name": f"validate0-{op[0]}-{fmt}-bad", "spec": {"data": ["mix", 30000, 79], "fmt": fmt,
                                                                       "xor_tail": 1},
                      "ops": [["init", wb], ["validate", 0], op, ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20],
                              ["adler"]]})
    # inflateReset2 / inflateReset / inflateResetKeep between concatenated streams
    two = {"concat": [{"data": ["text", 40000, 69], "fmt": "zlib"}, {"data": ["mix", 30000, 70], "fmt": "raw"}]}
    S.append({"name": "reset2-zlib-then-raw", "spec": two,
              "ops": [["init", 15], ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20], ["reset2", -15],
                      ["loop", Z_NO_FLUSH, 1 << 20], ["getdict"], ["reset2", 99], ["reset2", -16], ["reset2", 7]]})
    keep = {"concat": [{"data": ["text", 50000, 71], "fmt": "raw"},
                       {"data": ["text", 30000, 72], "fmt": "raw", "zdict_tail": ["text", 50000, 71, 32768]}]}
    for op in ("resetkeep", "reset2"):
        S.append({"name": f"{op}-raw-window", "spec": keep,
                  "ops": [["init", -15], ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20], ["getdict"],
                          [op] + ([-15] if op == "reset2" else []), ["getdict"], ["loop", Z_NO_FLUSH, 1 << 20],
                          ["getdict"]]})
    S.append({"name": "reset-zlib-twice", "spec": {"concat": [{"data": ["mix", 20000, 73], "fmt": "zlib"},
                                                              {"data": ["mix", 20000, 74], "fmt": "zlib"}]},
              "ops": [["init", 15], ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20], ["reset"], ["getdict"],
                      ["loop", Z_NO_FLUSH, 1 << 20]]})
    # inflatePrime: a raw stream from bit k on, its first k bits primed (zran.c)
    for k in (1, 3, 7, 8, 13):
        spec = {"data": ["mix", 40000, 75], "level": 6, "fmt": "raw", "shift": k}
        v = prime_value(spec)
        parts = [["prime", k - k // 2, v & ((1 << (k - k // 2)) - 1)], ["prime", k // 2, v >> (k - k // 2)]] \
            if k > 1 else [["prime", k, v]]
        S.append({"name": f"prime-{k}", "spec": spec,
                  "ops": [["init", -15]] + parts + [["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20]]})
    spec = {"data": ["text", 30000, 76], "zdict": ["text", 20000, 77], "fmt": "raw", "shift": 5}
    S.append({"name": "prime-dict", "spec": spec,
              "ops": [["init", -15], ["prime", 5, prime_value(spec)], ["dict", ["text", 20000, 77]], ["feed", BIG],
                      ["loop", Z_NO_FLUSH, 1 << 20]]})
    S.append({"name": "prime-clear-and-limits", "spec": {"data": ["text", 5000, 78], "fmt": "raw"},
              "ops": [["init", -15], ["prime", -1, 0], ["prime", 0, 5], ["prime", 17, 0], ["prime", 16, 0],
                      ["prime", 16, 0], ["prime", 1, 0], ["prime", -1, 0], ["feed", BIG],
                      ["loop", Z_NO_FLUSH, 1 << 20]]})
    S.append({"name": "undermine", "spec": {"data": ["text", 5000, 79], "fmt": "zlib"},
              "ops": [["init", 15], ["undermine", 1], ["undermine", 0], ["feed", BIG], ["loop", Z_NO_FLUSH, 1 << 20]]})
    return S


def deflate_sessions():
    """deflate ops carry a data slice [kind, n, seed, start, end] (datagen),
    made into bytes when the session runs (run_deflate)"""
    S = []
    t = ["text", 100000, 81]
    m = ["mix", 100000, 82]
    sl = lambda d, a, b: d + [a, b]
    for level in (0, 1, 6, 9):
        for wb in (15, -15, 31):
            ops = [["init", level, wb, 8, 0], ["used"], ["getdict"]]
            for i, fl in enumerate((Z_NO_FLUSH, Z_SYNC_FLUSH, Z_PARTIAL_FLUSH, Z_BLOCK, Z_NO_FLUSH, Z_SYNC_FLUSH)):
                ops += [["deflate", sl(m, i * 9000, (i + 1) * 9000), fl], ["used"], ["getdict"]]
            ops += [["deflate", sl(t, 0, 40000), Z_NO_FLUSH], ["used"], ["getdict"],
                    ["deflate", sl(t, 40000, 100000), Z_FINISH], ["used"], ["getdict"]]
            S.append({"name": f"used-getdict-L{level}-w{wb}", "ops": ops})
        S.append({"name": f"used-one-shot-L{level}", "ops": [["init", level, 15, 8, 0],
                                                             ["deflate", sl(m, 0, 100000), Z_FINISH],
                                                             ["used"], ["getdict"]]})
        S.append({"name": f"used-small-out-L{level}", "ops": [["init", level, 15, 8, 0],
                                                              ["deflate", sl(t, 0, 60000), Z_NO_FLUSH, 4000], ["used"],
                                                              ["getdict"], ["deflate", sl(t, 60000, 100000), Z_FINISH, 4000],
                                                              ["used"]]})
    for strategy in (1, 2, 3, 4):
        S.append({"name": f"used-strategy-{strategy}", "ops": [["init", 6, 15, 8, strategy],
                                                               ["deflate", sl(m, 0, 50000), Z_SYNC_FLUSH], ["used"],
                                                               ["deflate", sl(m, 50000, 100000), Z_FINISH], ["used"]]})
    for wb in (-15, 15, -10):
        S.append({"name": f"getdict-setdict-w{wb}", "ops": [["init", 6, wb, 8, 0], ["dict", sl(t, 0, 50000)], ["getdict"],
                                                            ["deflate", sl(m, 0, 20000), Z_NO_FLUSH], ["getdict"],
                                                            ["deflate", sl(m, 0, 0), Z_FINISH], ["getdict"]]})
        S.append({"name": f"getdict-setdict-L0-w{wb}", "ops": [["init", 0, wb, 8, 0], ["dict", sl(t, 0, 500)], ["getdict"],
                                                               ["deflate", sl(m, 0, 20000), Z_SYNC_FLUSH], ["getdict"]]})
    # deflateParams between deflate_slow and Z_HUFFMAN_ONLY / Z_RLE after data
    # (deflate.c:760-803; the gzsetparams pattern, gzwrite.c:587)
    for strat in (2, 3):
        for level, wb in ((6, 15), (9, -15), (5, 31), (6, -9)):
            S.append({"name": f"params-hr{strat}-L{level}-w{wb}", "ops": [
                ["init", level, wb, 8, 0], ["deflate", sl(m, 0, 30000), Z_NO_FLUSH], ["params", level, strat],
                ["deflate", sl(m, 30000, 50000), Z_NO_FLUSH], ["params", level, 0],
                ["deflate", sl(m, 50000, 100000), Z_FINISH], ["used"]]})
    S.append({"name": "params-hr-toggles-L9", "ops": [
        ["init", 9, -15, 8, 0], ["deflate", sl(t, 0, 20000), Z_SYNC_FLUSH], ["params", 9, 3],
        ["deflate", sl(t, 20000, 26000), Z_NO_FLUSH], ["params", 9, 0], ["deflate", sl(t, 26000, 60000), Z_NO_FLUSH],
        ["params", 9, 2], ["deflate", sl(t, 60000, 61000), Z_NO_FLUSH], ["params", 9, 0],
        ["deflate", sl(t, 61000, 100000), Z_FINISH]]})
    S.append({"name": "params-hr-gzsetparams", "ops": [
        ["init", 6, 31, 8, 0], ["deflate", sl(m, 0, 40000), Z_NO_FLUSH], ["params", 6, 2],
        ["deflate", sl(m, 40000, 41000), Z_NO_FLUSH], ["params", 5, 0], ["deflate", sl(m, 41000, 100000), Z_FINISH]]})
    S.append({"name": "params-hr-huff-rle-slow", "ops": [
        ["init", 7, 15, 8, 0], ["deflate", sl(t, 0, 35000), Z_NO_FLUSH], ["params", 7, 2],
        ["deflate", sl(t, 35000, 45000), Z_NO_FLUSH], ["params", 7, 3], ["deflate", sl(t, 45000, 52000), Z_NO_FLUSH],
        ["params", 8, 0], ["deflate", sl(t, 52000, 100000), Z_FINISH]]})
    S.append({"name": "params-hr-small-out", "ops": [
        ["init", 6, 15, 8, 0], ["deflate", sl(m, 0, 30000), Z_NO_FLUSH, 3000], ["params", 6, 2],
        ["deflate", sl(m, 30000, 60000), Z_NO_FLUSH, 3000], ["params", 6, 0],
        ["deflate", sl(m, 60000, 100000), Z_FINISH, 3000]]})
    S.append({"name": "params-hr-immediate", "ops": [
        ["init", 6, 15, 8, 0], ["deflate", sl(t, 0, 30000), Z_NO_FLUSH], ["params", 6, 2], ["params", 6, 0],
        ["deflate", sl(t, 30000, 100000), Z_FINISH]]})
    # the same from deflate_fast levels (round 5): the chains resume from the
    # snapshot at the Z_BLOCK flush, the stretch left out of what is inserted
    for strat in (2, 3):
        for level, wb in ((1, 15), (2, -15), (3, 31), (1, -9), (3, 12)):
            S.append({"name": f"params-hrf{strat}-L{level}-w{wb}", "ops": [
                ["init", level, wb, 8, 0], ["deflate", sl(m, 0, 30000), Z_NO_FLUSH], ["params", level, strat],
                ["deflate", sl(m, 30000, 50000), Z_NO_FLUSH], ["params", level, 0],
                ["deflate", sl(m, 50000, 100000), Z_FINISH], ["used"]]})
    S.append({"name": "params-hrf-toggles-L2", "ops": [
        ["init", 2, -15, 8, 0], ["deflate", sl(t, 0, 20000), Z_SYNC_FLUSH], ["params", 2, 3],
        ["deflate", sl(t, 20000, 26000), Z_NO_FLUSH], ["params", 1, 0], ["deflate", sl(t, 26000, 60000), Z_NO_FLUSH],
        ["params", 3, 2], ["deflate", sl(t, 60000, 61000), Z_NO_FLUSH], ["params", 3, 0],
        ["deflate", sl(t, 61000, 100000), Z_FINISH]]})
    S.append({"name": "params-hrf-gzsetparams", "ops": [
        ["init", 1, 31, 8, 0], ["deflate", sl(m, 0, 40000), Z_NO_FLUSH], ["params", 1, 2],
        ["deflate", sl(m, 40000, 41000), Z_NO_FLUSH], ["params", 1, 0], ["deflate", sl(m, 41000, 100000), Z_FINISH]]})
    S.append({"name": "params-hrf-long-stretch", "ops": [
        ["init", 3, 15, 8, 0], ["deflate", sl(t, 0, 20000), Z_NO_FLUSH], ["params", 3, 3],
        ["deflate", sl(t, 20000, 70000), Z_NO_FLUSH], ["params", 3, 0], ["deflate", sl(t, 70000, 100000), Z_FINISH]]})
    S.append({"name": "params-hrf-small-out", "ops": [
        ["init", 1, 15, 8, 0], ["deflate", sl(m, 0, 30000), Z_NO_FLUSH, 3000], ["params", 1, 2],
        ["deflate", sl(m, 30000, 60000), Z_NO_FLUSH, 3000], ["params", 2, 0],
        ["deflate", sl(m, 60000, 100000), Z_FINISH, 3000]]})
    S.append({"name": "params-hrf-mem5", "ops": [
        ["init", 2, 15, 5, 0], ["deflate", sl(t, 0, 30000), Z_NO_FLUSH], ["params", 2, 2],
        ["deflate", sl(t, 30000, 45000), Z_NO_FLUSH], ["params", 2, 0], ["deflate", sl(t, 45000, 100000), Z_FINISH]]})
    S.append({"name": "resetkeep-fresh", "ops": [["init", 6, 15, 8, 0], ["resetkeep"],
                                                 ["deflate", sl(m, 0, 100000), Z_FINISH], ["used"], ["reset"],
                                                 ["resetkeep"], ["deflate", sl(t, 0, 100000), Z_FINISH]]})
    S += resetkeep_sessions()
    S += prime_paused_sessions()
    return S


def prime_paused_sessions():
    """deflatePrime after a deflate() call that stopped on a full output buffer
    inside its input (round 6, deflate.c:731-757): the bits go after the block
    the call flushed last.  The next call offers more input, the same input
    again (the part the last call left), or a flush; primes in a row; every
    compress function and wrapper.  The reference keeps that call's output
    pending with pending_out moved on, and deflatePrime's put_byte writes a
    completed byte at pending_buf[pending] -- inside the output still to go --
    so only bits that complete no byte (deflatePending's bits + the primed
    ones < 8, read from the reference here) give a whole stream; the rest are
    refused (tests/test_gpu_zstream.py::test_prime_after_pause_refusal)."""
    S = []
    t = ["text", 300000, 84]
    m = ["mix", 300000, 85]
    sl = lambda d, a, b: d + [a, b]
    ref = Reference()
    for lv, st, wb, d, out in ((6, 0, 15, t, 1500), (9, 0, -15, m, 3000), (4, 1, 31, t, 700), (2, 0, 15, m, 2000),
                               (1, 0, -15, t, 5000), (6, 3, 15, m, 1500), (6, 2, -15, t, 4000), (7, 4, 15, m, 30000),
                               (5, 0, -12, t, 1000), (3, 0, 13, m, 2500), (8, 0, 15, t, 900), (6, 1, -15, m, 6000)):
        base = [["init", lv, wb, 8, st], ["deflate1", sl(d, 0, 150000), Z_NO_FLUSH, out], ["pending"]]
        rcs, _ = run_deflate_raw(ref.L, base)
        k = 7 - rcs[-1][2]                         # bits that complete no byte
        if k < 1:
            continue
        tag = f"L{lv}-s{st}-w{wb}"
        S.append({"name": f"pp-more-{tag}", "ops": base + [
            ["prime", k, 0x55], ["pending"], ["deflate", sl(d, 150000, 300000), Z_FINISH, 4000, True]]})
        S.append({"name": f"pp-flush-{tag}", "ops": base + [
            ["prime", k, 1], ["deflate1", sl(d, 0, 0), Z_SYNC_FLUSH, 1 << 20, True],
            ["deflate", sl(d, 150000, 300000), Z_FINISH]]})
        S.append({"name": f"pp-finish-{tag}", "ops": base + [
            ["prime", k, 0x2a], ["deflate1", sl(d, 0, 0), Z_FINISH, 1 << 20, True]]})
        if k >= 2:
            S.append({"name": f"pp-same-{tag}", "ops": base + [
                ["prime", k - 1, 0x5a5], ["deflate1", sl(d, 0, 0), Z_NO_FLUSH, out, True], ["prime", 1, 1],
                ["pending"], ["deflate1", sl(d, 0, 0), Z_NO_FLUSH, 1 << 20, True],
                ["deflate", sl(d, 150000, 300000), Z_FINISH]]})
            S.append({"name": f"pp-twice-{tag}", "ops": base + [
                ["prime", 1, 1], ["prime", k - 1, 0x7f], ["pending"],
                ["deflate", sl(d, 150000, 200000), Z_SYNC_FLUSH, 0, True], ["deflate", sl(d, 200000, 300000), Z_FINISH]]})
    return S


def run_deflate_raw(L, ops):
    return run_zsession(L, [[o[0], _slice(o[1])] + o[2:] if o[0] in ("deflate", "dict", "deflate1") else o
                            for o in ops])


def resetkeep_sessions():
    """deflateResetKeep carrying the window of a deflate_slow stream into the next
    one (round 6, deflate.c:635-671): after Z_FINISH and after flushes that took
    all their input, zlib / raw / gzip, window sizes 9-15, old streams long
    enough to have slid, preset dictionaries, repeated keeps, small output
    space, parameter changes before the new input"""
    S = []
    t = ["text", 100000, 81]
    m = ["mix", 100000, 82]
    sl = lambda d, a, b: d + [a, b]
    K = [["getdict"], ["resetkeep"], ["getdict"]]
    S.append({"name": "rk-finish-L6", "ops": [["init", 6, 15, 8, 0], ["deflate", sl(t, 0, 30000), Z_FINISH]] + K +
              [["deflate", sl(t, 30000, 100000), Z_FINISH], ["used"]]})
    S.append({"name": "rk-raw-L9", "ops": [["init", 9, -15, 8, 0], ["deflate", sl(m, 0, 80000), Z_FINISH]] + K +
              [["deflate", sl(m, 80000, 100000), Z_FINISH]]})
    S.append({"name": "rk-gzip-L5", "ops": [["init", 5, 31, 8, 0], ["deflate", sl(t, 0, 50000), Z_FINISH]] + K +
              [["deflate", sl(t, 50000, 100000), Z_FINISH]]})
    S.append({"name": "rk-slid-L6", "ops": [["init", 6, 15, 8, 0], ["deflate", sl(m, 0, 100000), Z_NO_FLUSH],
                                            ["deflate", sl(t, 0, 60000), Z_FINISH]] + K +
              [["deflate", sl(t, 60000, 100000), Z_FINISH]]})
    S.append({"name": "rk-slid-L8-raw", "ops": [["init", 8, -15, 8, 0], ["deflate", sl(t, 0, 100000), Z_NO_FLUSH],
                                                ["deflate", sl(m, 0, 23456), Z_FINISH]] + K +
              [["deflate", sl(m, 23456, 90000), Z_FINISH]]})
    for wb, lv, d in ((9, 6, t), (-12, 4, m), (10, 9, m), (-9, 7, t), (13, 5, t), (27, 6, m)):
        S.append({"name": f"rk-w{wb}-L{lv}", "ops": [["init", lv, wb, 8, 0], ["deflate", sl(d, 0, 40000), Z_FINISH]] +
                  K + [["deflate", sl(d, 40000, 70000), Z_FINISH]]})
    for fl in (Z_SYNC_FLUSH, Z_PARTIAL_FLUSH, Z_BLOCK):
        S.append({"name": f"rk-after-flush{fl}", "ops": [["init", 6, 15, 8, 0], ["deflate", sl(t, 0, 40000), fl]] + K +
                  [["deflate", sl(t, 40000, 80000), Z_FINISH]]})
    S.append({"name": "rk-after-full-flush", "ops": [["init", 6, 15, 8, 0], ["deflate", sl(t, 0, 40000), Z_NO_FLUSH],
                                                     ["deflate", sl(t, 40000, 50000), Z_FULL_FLUSH]] + K +
              [["deflate", sl(t, 50000, 90000), Z_FINISH]]})
    S.append({"name": "rk-full-flush-then-finish", "ops": [["init", 6, 15, 8, 0],
                                                           ["deflate", sl(t, 0, 30000), Z_FULL_FLUSH],
                                                           ["deflate", sl(t, 30000, 60000), Z_FINISH]] + K +
              [["deflate", sl(t, 60000, 100000), Z_FINISH]]})
    S.append({"name": "rk-twice-L7", "ops": [["init", 7, 15, 8, 0], ["deflate", sl(m, 0, 20000), Z_FINISH]] + K +
              [["deflate", sl(m, 20000, 40000), Z_FINISH]] + K + [["deflate", sl(m, 40000, 70000), Z_FINISH]]})
    S.append({"name": "rk-small-out", "ops": [["init", 6, 15, 8, 0], ["deflate", sl(t, 0, 30000), Z_FINISH, 700]] +
              K + [["deflate", sl(t, 30000, 100000), Z_FINISH, 1000]]})
    S.append({"name": "rk-old-dict", "ops": [["init", 6, 15, 8, 0], ["dict", sl(t, 90000, 99000)],
                                             ["deflate", sl(t, 0, 30000), Z_FINISH]] + K +
              [["deflate", sl(t, 30000, 60000), Z_FINISH]]})
    S.append({"name": "rk-dict-only", "ops": [["init", 6, 15, 8, 0], ["dict", sl(t, 0, 5000)]] + K +
              [["deflate", sl(t, 5000, 40000), Z_FINISH]]})
    for lv, st in ((9, 1), (4, 4), (6, 2), (6, 3), (5, 0)):
        S.append({"name": f"rk-then-params-{lv}-{st}", "ops": [["init", 6, 15, 8, 0],
                                                               ["deflate", sl(t, 0, 30000), Z_FINISH]] + K +
                  [["params", lv, st], ["deflate", sl(t, 30000, 100000), Z_FINISH]]})
    for n in (1, 2, 3, 4):
        S.append({"name": f"rk-tiny-{n}", "ops": [["init", 6, 15, 8, 0], ["deflate", sl(t, 0, n), Z_FINISH]] + K +
                  [["deflate", sl(t, n, 5000), Z_FINISH]]})
    for ml, st in ((1, 0), (9, 1), (5, 4)):
        S.append({"name": f"rk-m{ml}-s{st}", "ops": [["init", 6, 15, ml, st], ["deflate", sl(m, 0, 50000), Z_FINISH]] +
                  K + [["deflate", sl(m, 50000, 100000), Z_FINISH]]})
    S.append({"name": "rk-new-chunks", "ops": [["init", 6, 15, 8, 0], ["deflate", sl(t, 0, 30000), Z_FINISH]] + K +
              [["deflate", sl(t, 30000, 30100), Z_NO_FLUSH], ["deflate", sl(t, 30100, 45000), Z_SYNC_FLUSH],
               ["deflate", sl(t, 45000, 100000), Z_FINISH]]})
    return S


def back_cases():
    C = []
    for kind, level in (("text", 6), ("mix", 9), ("runs", 1), ("mix", 0)):
        for wbits in (15, 9):
            for chunk, first in ((BIG, 0), (4096, 0), (777, 100)):
                # a w9 window gets a stream made with a w9 window: with distances
                # beyond the window the reference's inflate_fast loop copies stale
                # window bytes before it reports the error, not a
                # behaviour to pin
                spec = {"data": [kind, 90000, 91], "level": level, "fmt": "raw"}
                if wbits < 15:
                    spec["cwbits"] = wbits
                C.append({"name": f"back-{kind}-L{level}-w{wbits}-c{chunk}-f{first}",
                          "spec": spec, "wbits": wbits, "in_chunk": chunk, "first": first})
    small = {"data": ["text", 1500, 92], "level": 6, "fmt": "raw"}
    C.append({"name": "back-bytes", "spec": small, "wbits": 15, "in_chunk": 1, "first": 0})
    C.append({"name": "back-truncated", "spec": dict(small, chop=5), "wbits": 15, "in_chunk": 64, "first": 0})
    C.append({"name": "back-garbage-after", "spec": dict(small, garbage=40), "wbits": 15, "in_chunk": BIG, "first": 0})
    C.append({"name": "back-out-fails", "spec": {"data": ["mix", 90000, 93], "fmt": "raw", "cwbits": 10}, "wbits": 10,
              "in_chunk": BIG, "first": 0, "out_fail_at": 3})
    C.append({"name": "back-corrupt", "spec": {"data": ["text", 9000, 94], "fmt": "zlib"}, "wbits": 15,
              "in_chunk": BIG, "first": 0})
    return C


def run_inflate(L, sess):
    z = build(sess["spec"])
    res, outs, _ = run_iops(L, z, sess["ops"])
    return {"res": json.loads(json.dumps(res)), "outs": [[len(o), hashlib.sha256(o).hexdigest()] for o in outs]}


def _slice(spec):
    kind, n, seed, a, b = spec
    return datagen.make(kind, n, seed)[a:b]


def run_deflate(L, sess):
    ops = [[o[0], _slice(o[1])] + o[2:] if o[0] in ("deflate", "dict", "deflate1") else o for o in sess["ops"]]
    rcs, out = run_zsession(L, ops)
    return {"res": json.loads(json.dumps(rcs)), "out": [len(out), hashlib.sha256(out).hexdigest()]}


def run_backcase(L, case):
    z = build(case["spec"])
    rc0, rc, out, unused, null_in, rc2, calls = run_back(L, z, case["wbits"], case["in_chunk"], case["first"],
                                                         case.get("out_fail_at"))
    if case.get("out_fail_at"):
        # where out() fails, the reference's bit buffer has pulled input bytes
        # ahead of the failing symbol (infback.c PULLBYTE / inflate_fast's
        # 2-byte loads); the decode here has read the whole input: the unused
        # count is not pinned
        unused = None
    return {"res": json.loads(json.dumps([rc0, rc, unused, null_in, rc2])),
            "out": [len(out), hashlib.sha256(out).hexdigest()]}


def main():
    ref = Reference()
    out = {"reference": ref.version.decode(), "inflate": [], "deflate": [], "back": []}
    for sess in inflate_sessions():
        out["inflate"].append(dict(sess, **run_inflate(ref.L, sess)))
    for sess in deflate_sessions():
        out["deflate"].append(dict(sess, **run_deflate(ref.L, sess)))
    for case in back_cases():
        out["back"].append(dict(case, **run_backcase(ref.L, case)))
    path = os.path.join(HERE, "api_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"), sort_keys=True)
    print(f"wrote {path}: {len(out['inflate'])} inflate, {len(out['deflate'])} deflate, {len(out['back'])} back")


if __name__ == "__main__":
    main()
