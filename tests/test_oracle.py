"""CPU tests: pin the oracle (our C restatement) to the reference.

* against the committed golden fixtures (generated from the compiled reference
  by tests/golden/make_golden.py) — always;
* against the compiled reference itself — in the build container only, where
  oracle/_ref/libzref.so exists;
* the position-parallel formulation (the GPU's spec) against both.
"""
import hashlib
import os

import numpy as np
import pytest

import datagen
from zhelpers import Reference, reference_available


def _cases(golden, maxn=None):
    for c in golden["cases"]:
        if maxn is None or c["n"] <= maxn:
            yield c


def test_golden_inputs_regenerate(golden):
    for c in _cases(golden):
        data = datagen.make(c["kind"], c["n"], c["seed"])
        assert hashlib.sha256(data).hexdigest() == c["sha256"], (c["kind"], c["n"])


@pytest.mark.parametrize("pp", [False, True], ids=["sequential", "position-parallel"])
def test_oracle_matches_golden_all_levels(oracle, golden, pp):
    fn = oracle.pp_compress if pp else oracle.compress
    for c in _cases(golden, maxn=1 << 20):
        data = datagen.make(c["kind"], c["n"], c["seed"])
        levels = range(10) if c["n"] <= 70000 else (1, 4, 6, 9)
        for lvl in levels:
            rc, z = fn(data, lvl)
            want = c["levels"][str(lvl)]
            assert rc == 0
            assert len(z) == want["len"], (c["kind"], c["n"], lvl)
            assert hashlib.sha256(z).hexdigest() == want["sha256"], (c["kind"], c["n"], lvl)
            if "hex" in want:
                assert z.hex() == want["hex"]


def test_oracle_wrappers_golden(oracle, golden):
    for c in _cases(golden, maxn=70000):
        data = datagen.make(c["kind"], c["n"], c["seed"])
        _, raw = oracle.compress(data, 6, wrap=0)
        _, gz = oracle.compress(data, 6, wrap=2)
        assert hashlib.sha256(raw).hexdigest() == c["raw6"]["sha256"]
        assert hashlib.sha256(gz).hexdigest() == c["gzip6"]["sha256"]


def test_oracle_checksums_golden(oracle, golden):
    for c in _cases(golden):
        data = datagen.make(c["kind"], c["n"], c["seed"])
        assert oracle.crc32(data) == c["crc32"]
        assert oracle.adler32(data) == c["adler32"]
    for hexs, k in golden["known"].items():
        s = bytes.fromhex(hexs)
        assert oracle.crc32(s) == k["crc32"]
        assert oracle.adler32(s) == k["adler32"]
        for lvl in (1, 6, 9):
            assert oracle.compress(s, lvl)[1].hex() == k[f"z{lvl}"]
    # public known answers
    assert oracle.crc32(b"123456789") == 0xCBF43926
    assert oracle.adler32(b"123456789") == 0x091E01DE
    assert oracle.crc32(b"Hello, World!") == 0xEC4AC3D0


def test_oracle_combine(oracle):
    a, b = datagen.text(5000, 1), datagen.random_bytes(7777, 2)
    L = oracle.L
    assert L.zo_crc32_combine(oracle.crc32(a), oracle.crc32(b), len(b)) == oracle.crc32(a + b)
    assert L.zo_adler32_combine(oracle.adler32(a), oracle.adler32(b), len(b)) == oracle.adler32(a + b)


def test_oracle_short_output(oracle):
    """compress2 with a short destination: Z_BUF_ERROR and a prefix (compress.c:44-58)."""
    data = datagen.text(20000, 5)
    _, full = oracle.compress(data, 6)
    for cap in (0, 1, 2, 7, len(full) // 2, len(full) - 1):
        rc, z = oracle.compress(data, 6, cap=cap)
        assert rc == -5 and z == full[:cap]
    rc, z = oracle.compress(data, 6, cap=len(full))
    assert rc == 0 and z == full


@pytest.mark.skipif(not reference_available(), reason="compiled reference only in build container")
def test_oracle_vs_reference_random_sweep(oracle):
    ref = Reference()
    rng = np.random.default_rng(2024)
    for t in range(60):
        kind = ["text", "runs", "four", "random", "mix", "markup", "records"][t % 7]
        n = int(rng.choice([int(rng.integers(0, 600)), int(rng.integers(600, 40000)),
                            int(rng.integers(40000, 200000))]))
        data = datagen.make(kind, n, int(rng.integers(0, 1 << 30)))
        for lvl in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9):
            rc, want = ref.compress2(data, lvl)
            assert oracle.compress(data, lvl)[1] == want, (kind, n, lvl)
            assert oracle.pp_compress(data, lvl)[1] == want, (kind, n, lvl)


@pytest.mark.skipif(not reference_available(), reason="compiled reference only in build container")
def test_oracle_vs_reference_short_output():
    from zhelpers import Oracle
    ref, o = Reference(), Oracle()
    data = datagen.mix(50000, 9)
    for lvl in (1, 6, 9):
        _, full = ref.compress2(data, lvl)
        for cap in (0, 1, 5, len(full) // 3, len(full) - 1):
            rc, z = ref.compress2(data, lvl, cap=cap)
            rc2, z2 = o.compress(data, lvl, cap=cap)
            assert (rc, z) == (rc2, z2)


@pytest.mark.skipif(not reference_available(), reason="compiled reference only in build container")
def test_reference_chunked_input_equals_one_shot():
    """Feeding deflate() with Z_NO_FLUSH chunks gives the one-shot stream, which
    is what lets the drop-in deflate() gather input until Z_FINISH."""
    ref = Reference()
    data = datagen.mix(200000, 4)
    for lvl in (1, 6, 9):
        one = ref.deflate(data, lvl, 15)
        for chunk in (1000, 4096, 65536):
            assert ref.deflate(data, lvl, 15, chunk=chunk) == one


@pytest.mark.skipif(not reference_available(), reason="compiled reference only in the build container")
@pytest.mark.parametrize("strategy", [1, 2, 3, 4], ids=["filtered", "huffman_only", "rle", "fixed"])
def test_oracle_strategies_vs_reference(oracle, strategy):
    """deflateInit2_(strategy) of the compiled reference (deflate.c:1190-1193,
    1964, 2051-2152, trees.c:1035) against the oracle, all levels and wrappers,
    including sizes around the window slides of each parser."""
    ref = Reference()
    rng = np.random.default_rng(300 + strategy)
    sizes = [0, 1, 2, 3, 4, 258, 259, 262, 16383, 16384, 65273, 65274, 65275, 65278, 65536,
             65537, 98304, 200000]
    for t, n in enumerate(sizes):
        kind = ["runs", "text", "mix", "random", "records", "four"][t % 6]
        data = datagen.make(kind, n, int(rng.integers(0, 1 << 30)))
        for level in (0, 1, 4, 6, 9):
            for wbits, wrap in ((15, 1), (-15, 0), (31, 2)):
                want = ref.deflate(data, level, wbits=wbits, strategy=strategy)
                rc, got = oracle.compress(data, level, wrap=wrap, strategy=strategy)
                assert rc == 0 and got == want, (kind, n, level, wrap, strategy)


def test_oracle_strategies_golden(oracle, golden):
    """Oracle vs the committed strategy fixtures (compiled-reference outputs)."""
    for c in _cases(golden, maxn=70000):
        data = datagen.make(c["kind"], c["n"], c["seed"])
        for key, want in c["strategies"].items():
            strategy, level = (int(x) for x in key.split("/"))
            rc, z = oracle.compress(data, level, wrap=1, strategy=strategy)
            assert rc == 0 and len(z) == want["len"] and hashlib.sha256(z).hexdigest() == want["sha256"], \
                (c["kind"], c["n"], key)


# ----------------------------- inflate -----------------------------

@pytest.fixture(scope="module")
def inflate_golden():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "inflate_golden.json")) as f:
        return json.load(f)


def _oracle_compress(oracle):
    return lambda d, level, wrap, strategy: oracle.compress(d, level, wrap=wrap, strategy=strategy)[1]


def test_oracle_inflate_golden(oracle, inflate_golden):
    """uncompress2 status / output / consumed of the reference on 2427 streams:
    valid ones at every level, wrapper and strategy, truncated, bit-flipped,
    with garbage tails, short outputs, the destLen == 0 probe, and crafted
    headers / block headers / code sets."""
    import inflate_cases as ic
    comp = _oracle_compress(oracle)
    bases = {}
    for c in inflate_golden["cases"]:
        if "hex" in c:
            src = bytes.fromhex(c["hex"])
        else:
            key = (c["kind"], c["n"], c["seed"], c["level"], c["wrap"], c["strategy"])
            if key not in bases:
                bases[key] = ic.base_stream(c, comp)[1]
                assert ic.sha(bases[key]) == c["base_sha256"], key   # the oracle compressor too
            src = ic.mutate(bases[key], c["mut"])
        rc, out, used = oracle.uncompress(src, c["cap"], c["dwrap"])
        e = c["expect"]
        assert (rc, len(out), ic.sha(out), used) == (e["status"], e["len"], e["sha256"], e["consumed"]), c


@pytest.mark.skipif(not reference_available(), reason="compiled reference only in build container")
def test_oracle_inflate_vs_reference_fuzz(oracle):
    import inflate_cases as ic
    ref = Reference()
    rng = np.random.default_rng(77)
    for c in ic.crafted(seed=31, count=1500):
        src = bytes.fromhex(c["hex"])
        assert oracle.uncompress(src, c["cap"], c["dwrap"]) == ref.uncompress(src, c["cap"], c["dwrap"]), c
    for t in range(60):
        data = datagen.make(["text", "mix", "runs", "random"][t % 4], int(rng.integers(0, 50000)), t)
        wrap = t % 3
        z = oracle.compress(data, int(rng.integers(0, 10)), wrap=wrap)[1]
        for _ in range(10):
            zz = bytearray(z)
            i = int(rng.integers(0, len(zz) * 8))
            zz[i >> 3] ^= 1 << (i & 7)
            cut = int(rng.integers(0, len(zz) + 1))
            for src in (bytes(zz), z[:cut]):
                cap = int(rng.integers(0, len(data) + 2))
                assert oracle.uncompress(src, cap, wrap) == ref.uncompress(src, cap, wrap), (t, i, cut)


def _flush_plan(rng, n):
    """A random deflate() call sequence over n bytes: chunk sizes from tiny to
    window-sized, flush types Z_NO_FLUSH / PARTIAL / SYNC / FULL / BLOCK,
    repeated flushes with no input, then Z_FINISH."""
    calls, pos = [], 0
    while pos < n:
        take = int(min(n - pos, rng.choice([0, 1, 2, 3, 17, 300, 4000, 40000, 70000])))
        flush = int(rng.choice([0, 0, 1, 2, 2, 3, 5]))
        calls.append((take, flush))
        pos += take
        if rng.random() < 0.15:
            calls.append((0, int(rng.choice([1, 2, 3, 5]))))
    calls.append((0, 4))
    return calls


@pytest.mark.skipif(not reference_available(), reason="compiled reference only in the build container")
def test_oracle_flushes_vs_reference(oracle):
    """deflate() call sequences with Z_PARTIAL/SYNC/FULL_FLUSH and Z_BLOCK on
    the compiled reference (deflate.c:954-1263, flush handling :1211-1233, the
    parsers' flush tails :1905-1915,2030-2042) against zo_deflate_flushes: the
    whole stream, and after every flush call the bytes written so far."""
    from zhelpers import flush_events
    ref = Reference()
    rng = np.random.default_rng(int(os.environ.get("ZO_FLUSH_SEED", 11)))
    for t in range(int(os.environ.get("ZO_FLUSH_CASES", 40))):
        kind = ["text", "mix", "runs", "random", "four"][t % 5]
        n = int(rng.choice([0, 5, 1000, 70000, 150000]))
        data = datagen.make(kind, n, 300 + t)
        level = int(rng.choice([1, 2, 3, 4, 6, 9]))
        strategy = int(rng.choice([0, 0, 0, 1, 2, 3, 4]))
        wbits = int(rng.choice([15, -15, 31]))
        wrap = {15: 1, -15: 0, 31: 2}[wbits]
        calls = _flush_plan(rng, n)
        sts, lens, whole = ref.deflate_calls(data, calls, level, wbits, strategy)
        ev = flush_events(calls)
        rc, got = oracle.deflate_flushes(data, ev, level, wrap, strategy)
        assert rc == 0 and got == whole, (t, kind, n, level, strategy, wbits)
        pos = 0
        for i, (take, flush) in enumerate(calls[:-1]):
            pos += take
            if flush in (0, 4) or sts[i] != 0:
                continue
            pre = flush_events(calls[:i + 1])
            rc, part = oracle.deflate_flushes(data[:pos], pre, level, wrap, strategy, finish=False)
            assert rc == 0 and part == whole[:lens[i]], (t, i, pos, flush)


def test_oracle_flush_golden(oracle):
    """zo_deflate_flushes against the reference's deflate() call sequences
    frozen in tests/golden/flush_golden.json (whole stream and the output
    after every flush call)."""
    import json
    import os as _os
    from zhelpers import flush_events
    with open(_os.path.join(_os.path.dirname(__file__), "golden", "flush_golden.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        data = datagen.make(c["kind"], c["n"], c["seed"])
        assert hashlib.sha256(data).hexdigest() == c["input_sha256"]
        calls = [tuple(x) for x in c["calls"]]
        wrap = {15: 1, -15: 0, 31: 2}[c["wbits"]]
        rc, got = oracle.deflate_flushes(data, flush_events(calls), c["level"], wrap, c["strategy"])
        assert rc == 0 and len(got) == c["len"] and hashlib.sha256(got).hexdigest() == c["sha256"], c["seed"]
        pos = 0
        for i, (take, flush) in enumerate(calls[:-1]):
            pos += take
            if flush in (0, 4) or c["status"][i] != 0:
                continue
            rc, part = oracle.deflate_flushes(data[:pos], flush_events(calls[:i + 1]), c["level"], wrap,
                                              c["strategy"], finish=False)
            assert rc == 0 and part == got[:c["out_len"][i]], (c["seed"], i)


def test_oracle_stored_calls_golden(oracle):
    """zo_deflate_stored_calls (level 0 over deflate() calls) against the
    reference's call sequences frozen in tests/golden/stored_golden.json:
    status and output length after every call, and the stream."""
    import json
    import os as _os
    with open(_os.path.join(_os.path.dirname(__file__), "golden", "stored_golden.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        data = datagen.make(c["kind"], c["n"], c["seed"])
        assert hashlib.sha256(data).hexdigest() == c["input_sha256"]
        calls = [tuple(x) for x in c["calls"]]
        wrap = {15: 1, -15: 0, 31: 2}[c["wbits"]]
        rc, sts, lens, got = oracle.deflate_stored_calls(data, calls, wrap)
        assert rc == 0 and sts == c["status"] and lens == c["out_len"], c["seed"]
        assert len(got) == c["len"] and hashlib.sha256(got).hexdigest() == c["sha256"], c["seed"]


@pytest.mark.skipif(not reference_available(), reason="compiled reference not built (build container only)")
def test_oracle_stored_calls_vs_reference(oracle):
    """Random level-0 call sequences through the compiled reference."""
    import os as _os
    from zhelpers import Reference
    ref = Reference()
    rng = np.random.default_rng(int(_os.environ.get("ZO_STORED_SEED", "3")))
    for t in range(int(_os.environ.get("ZO_STORED_CASES", "60"))):
        n = int(rng.choice([0, 1, 5, 1000, 40000, 70000, 200000]))
        data = datagen.make(["text", "mix", "runs", "random"][t % 4], n, 100 + t)
        calls, pos = [], 0
        while pos < n:
            take = int(min(n - pos, rng.choice([0, 1, 17, 4000, 32767, 32768, 65535, 65536, 140000])))
            calls.append((take, int(rng.choice([0, 0, 0, 1, 2, 3, 5]))))
            pos += take
            if rng.random() < 0.15:
                calls.append((0, int(rng.choice([0, 1, 2, 3, 5]))))
        calls.append((0, 4))
        wb = int(rng.choice([15, -15, 31]))
        sts, lens, whole = ref.deflate_calls(data, calls, 0, wb, 0)
        rc, osts, olens, got = oracle.deflate_stored_calls(data, calls, {15: 1, -15: 0, 31: 2}[wb])
        assert rc == 0 and osts == sts and olens == lens and got == whole, (t, n, wb)


def test_oracle_vs_bench_golden(oracle):
    """The benchmark's own inputs (host build of the device generator) and the
    oracle's streams for them, against the compiled reference's fixtures:
    C4 L6 Silesia-style buffers at bench.py's seed/indices, C3 L1, and C5's
    three 16 MiB kinds at L9, plus the all-literal
    16383*k block-count case."""
    import hashlib
    import json
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    g = json.load(open(os.path.join(here, "golden", "bench_golden.json")))
    for c in g["cases"]:
        data = oracle.generate(c["n"], 1, c["kind"], c["seed"], c["index"])[0]
        assert hashlib.sha256(data).hexdigest() == c["input_sha256"], c["name"]
        assert oracle.adler32(data) == c["adler32"] and oracle.crc32(data) == c["crc32"]
        rc, z = oracle.compress(data, c["level"])
        assert rc == 0 and len(z) == c["len"] and hashlib.sha256(z).hexdigest() == c["sha256"], \
            (c["name"], c["kind"], c["index"])
    import sys
    sys.path.insert(0, os.path.join(here, "golden"))
    from make_bench_golden import literal_input
    for e in g["literal_blocks"]:
        data = literal_input(e["n"])
        assert hashlib.sha256(data).hexdigest() == e["input_sha256"]
        for level, want in e["levels"].items():
            rc, z = oracle.compress(data, int(level))
            assert rc == 0 and hashlib.sha256(z).hexdigest() == want["sha256"], (e["k"], level)
