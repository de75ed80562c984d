"""GPU parity of the z_stream controls (deflateSetDictionary, deflateTune,
deflateParams, deflatePrime, deflateSetHeader, inflateSetDictionary): scripted
sessions replayed on libzgpu.so against the compiled reference's return codes
and streams, frozen in tests/golden/zstream_golden.json by
tests/golden/make_zstream_golden.py."""
import hashlib
import json
import os
import sys

import pytest

import datagen
from zhelpers import run_isession, run_zsession

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_zstream_golden import materialize  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zs_golden():
    with open(os.path.join(HERE, "golden", "zstream_golden.json")) as f:
        return json.load(f)


def _rc_equal(op, got, want):
    if op[0] == "dict":                     # (rc, strm->adler); the adler only where the call succeeded
        return got[0] == want[0] and (want[0] != 0 or got[1] == want[1])
    return got == want


def test_zstream_sessions_vs_reference(zg, zs_golden):
    L = zg.load()
    bad = []
    for sess in zs_golden["sessions"]:
        rcs, z = run_zsession(L, materialize(sess["ops"]))
        ok = len(rcs) == len(sess["rcs"]) and all(
            _rc_equal(op, tuple(g) if isinstance(g, tuple) else g, tuple(w) if op[0] == "dict" else w)
            for op, g, w in zip(sess["ops"], rcs, sess["rcs"]))
        if not ok or len(z) != sess["len"] or hashlib.sha256(z).hexdigest() != sess["sha256"]:
            bad.append((sess["name"], rcs, sess["rcs"], len(z), sess["len"]))
    if bad:
        print("BAD SESSIONS:", [b[0] for b in bad])
    assert not bad, ([b[0] for b in bad], bad[:3])


def test_inflate_with_dictionary(zg):
    """A zlib stream with FDICT: Z_NEED_DICT with the header consumed and
    strm->adler = DICTID, a wrong dictionary is Z_DATA_ERROR, the right one
    decodes; a raw stream takes its dictionary before the first input.
    total_in stays 0 at Z_NEED_DICT: the reference returns from DICT after
    RESTORE() without counting the call's input (isession_golden.json)."""
    L = zg.load()
    data = datagen.make("text", 200000, 40)
    dic = datagen.make("text", 20000, 41)
    for level, wb in ((6, 15), (1, 15), (9, 12)):
        _, z = run_zsession(L, [("init", level, wb, 8, 0), ("dict", dic), ("deflate", data, 4)])
        for chunk in (1 << 30, 4096):
            rcs, out = run_isession(L, z, wb, dic, chunk)
            assert out == data and rcs[-1] == 1, (level, wb, chunk, rcs[:4])
            assert rcs[1][0] == "need" and rcs[1][2] == 0
        rcs, out = run_isession(L, z, wb, dic[:-1] + b"?")
        assert rcs[-1] == -3 and out == b""
    _, z = run_zsession(L, [("init", 6, -15, 8, 0), ("dict", dic), ("deflate", data, 4)])
    rcs, out = run_isession(L, z, -15, dic, 3000)
    assert out == data and rcs[-1] == 1


def test_inflate_api_sessions_golden(zg):
    """inflate(Z_BLOCK), inflateGetHeader, inflateSync and inflateCopy
    (inflate.c:1267-1269, :1330, :1375, :1439) replayed on libzgpu.so against
    the compiled reference's results (tests/golden/isession_golden.json): every
    call's return code, avail_in, total_in, total_out and (Z_BLOCK) data_type,
    each stream's output, the gz_header fields."""
    import json
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    from make_isession_golden import run
    g = json.load(open(os.path.join(here, "golden", "isession_golden.json")))
    L = zg.load()
    bad = []
    for sess in g["sessions"]:
        r = run(L, sess)
        if r["res"] != sess["res"] or r["outs"] != sess["outs"] or r["hdr"] != sess["hdr"]:
            bad.append(sess["name"])
    print("BAD SESSIONS:", bad)
    assert not bad


def test_round4_zlib_h_calls_golden(zg):
    """The zlib.h calls added in round 4 replayed on libzgpu.so against the
    compiled reference's results (tests/golden/api_golden.json,
    make_api_golden.py): deflateUsed, deflateGetDictionary, deflateResetKeep
    (deflate.c:616-728), inflateReset2, inflateResetKeep, inflatePrime,
    inflateGetDictionary, inflateSyncPoint, inflateUndermine, inflateValidate,
    inflateMark, inflateCodesUsed (inflate.c:105-1527) with every call's return
    code and counters around them, and inflateBack over in() / out() callbacks
    (infback.c): return code, output, unused input."""
    import json
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    from make_api_golden import run_backcase, run_deflate, run_inflate
    g = json.load(open(os.path.join(here, "golden", "api_golden.json")))
    L = zg.load()
    bad = []
    for sess in g["inflate"]:
        r = run_inflate(L, sess)
        if r["res"] != sess["res"] or r["outs"] != sess["outs"]:
            bad.append(sess["name"])
    for sess in g["deflate"]:
        r = run_deflate(L, sess)
        if r["res"] != sess["res"] or r["out"] != sess["out"]:
            bad.append(sess["name"])
    for case in g["back"]:
        r = run_backcase(L, case)
        if r["res"] != case["res"] or r["out"] != case["out"]:
            bad.append(case["name"])
    print("BAD SESSIONS:", bad)
    assert not bad


def test_resetkeep_refusals(zg):
    """deflateResetKeep carries a deflate_slow stream's window into the next
    stream (the api_golden rk-* sessions); the carried states it does not model
    return Z_STREAM_ERROR with strm->msg and leave the stream as it was: a
    deflate_fast or deflate_stored stream, input still in the lookahead, a
    stream whose function changed after data, and after a carried window a
    preset dictionary or a switch to level 0 or to a deflate_fast level, whose
    longest_match would start from the prev_length deflate_slow left
    (zgpu_api.cpp deflateResetKeep, deflateParams)."""
    L = zg.load()
    d = datagen.make("text", 60000, 41)
    fin = lambda a, b: ["deflate", d[a:b], 4]
    cases = [
        ([["init", 1, 15, 8, 0], fin(0, 20000), ["resetkeep"]], -2),                   # deflate_fast
        ([["init", 0, -15, 8, 0], fin(0, 20000), ["resetkeep"]], -2),                  # deflate_stored
        ([["init", 6, 15, 8, 0], ["deflate", d[:100], 0], ["resetkeep"]], -2),         # lookahead
        ([["init", 6, 15, 8, 0], ["deflate", d[:20000], 0], ["params", 2, 0],
          ["deflate", d[20000:30000], 0], ["params", 6, 0], ["deflate", d[30000:31000], 2],
          ["resetkeep"]], -2),                                                           # mixed functions
        ([["init", 6, -15, 8, 0], fin(0, 20000), ["resetkeep"], ["dict", d[:3000]]], -2),
        ([["init", 6, -15, 8, 0], fin(0, 20000), ["resetkeep"], ["params", 0, 0]], -2),
        ([["init", 6, 15, 8, 0], fin(0, 20000), ["resetkeep"], ["params", 2, 0]], -2),  # deflate_fast next
    ]
    for ops, want in cases:
        rcs, _ = run_zsession(L, ops + [["deflate", d[40000:], 4]])
        got = rcs[len(ops) - 1]
        got = got[0] if isinstance(got, (tuple, list)) else got
        assert got == want, (ops[-1], rcs)
        assert rcs[-1][-1] == 1 or rcs[-1][-1] == -5, rcs         # the stream goes on (or has ended)


def test_prime_after_pause_refusal(zg):
    """deflatePrime after a call that stopped on a full output buffer inside its
    input is modelled where the bits complete no byte (api_golden pp-*
    sessions); bits that would complete one are refused: the reference's
    put_byte writes that byte at pending_buf[pending], inside the output still
    pending, and its stream ends with a stale buffer byte (zgpu_api.cpp
    deflatePrime).  The stream goes on as if the call had not been made."""
    import zlib as pyzlib
    L = zg.load()
    d = datagen.make("text", 200000, 42)
    base = [["init", 6, -15, 8, 0], ["deflate1", d[:150000], 0, 1500], ["pending"]]
    rcs, _ = run_zsession(L, base)
    assert rcs[1][2] == 0 and rcs[1][1] > 0, rcs         # stopped on a full output buffer inside its input
    held = rcs[-1][2]
    rcs, z = run_zsession(L, base + [["prime", 8 - held, 3], ["deflate", d[150000:], 4, 4000, True]])
    assert rcs[3] == -2, rcs
    assert rcs[-1][-1] == 1, rcs
    assert pyzlib.decompressobj(-15).decompress(z) == d


def test_params_huff_rle_refusals(zg):
    """deflateParams between deflate_slow or deflate_fast and Z_HUFFMAN_ONLY /
    Z_RLE after data is modelled (test_round4_zlib_h_calls_golden's params-hr-*
    and params-hrf-* sessions); the switches it does not model return
    Z_STREAM_ERROR with strm->msg set and leave the stream usable: a stretch
    left for the other function than it began from, memLevel 9 from
    deflate_slow, and a stretch whose first call offered a single byte
    (zgpu_api.cpp deflateParams)."""
    import zlib as pyzlib
    L = zg.load()
    d = datagen.make("text", 60000, 31)
    cases = [
        ([["init", 2, 15, 8, 0], ["deflate", d[:20000], 0], ["params", 2, 2],
          ["deflate", d[20000:30000], 0], ["params", 6, 0]], -2),                       # fast -> huff -> slow
        ([["init", 6, 15, 9, 0], ["deflate", d[:20000], 0], ["params", 6, 3]], -2),   # memLevel 9
        ([["init", 6, 15, 8, 0], ["deflate", d[:20000], 0], ["params", 6, 2],
          ["deflate", d[20000:30000], 0], ["params", 2, 0]], -2),                       # huff -> fast
        ([["init", 6, 15, 8, 0], ["deflate", d[:20000], 0], ["params", 6, 2],
          ["deflate", d[20000:20001], 0], ["deflate", d[20001:30000], 0], ["params", 6, 0]], -2),   # 1-byte call
    ]
    for ops, want in cases:
        full = ops + [["deflate", d[len(d) - 10000:], 4]]
        rcs, z = run_zsession(L, full)
        assert rcs[len(ops) - 1] == want, (ops[-1], rcs)
        assert rcs[-1][-1] == 1, rcs                                    # the stream still finishes
        got = pyzlib.decompressobj().decompress(z)
        fed = b"".join(op[1] for op in full if op[0] == "deflate")
        assert got == fed
