"""Regenerate tests/golden/bench_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so is built there from
/root/reference by `make -C oracle ref`):

    make -C oracle ref liboracle.so && python tests/golden/make_bench_golden.py

Pins the benchmark's own workloads: buffers of the device generator
(zlib.wasm_amd/csrc/zgpu_gen.h, rebuilt on the host by oracle/zgen.c) at the
seeds and global indices bench.py uses, compressed by the reference's
compress2() at the config's level: C4's Silesia-style mix at L6, C3's
enwik-style text at L1, and C5's three 16 MiB kinds (small-vocabulary text,
4-letter alphabet, byte runs) at L9 with the Adler-32 trailer (SURVEY
Appendix A.6).  Each case records the input's sha256 (so the host and device
generators are pinned too), the stream's length and sha256, and the input's
Adler-32 / CRC-32.  Plus the exact block-count case: an all-literal input of
16383*k bytes (a prefix of a de Bruijn sequence B(64, 3): no 3-byte string
repeats, so every symbol is a literal and blocks are cut at exactly 16383
symbols, deflate.h:371).
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from zhelpers import Oracle, Reference  # noqa: E402

SILESIA, ENWIK, VOCAB, FOUR, RUNS = 1, 2, 3, 4, 5
MiB = 1 << 20
# (name, kind, length, seed, global index, level)
CASES = [("C4", SILESIA, MiB, 2025, i, 6) for i in (0, 1, 2, 3, 4095, 32767, 262143)]
CASES += [("C4-L1", SILESIA, MiB, 2025, 5, 1), ("C4-L9", SILESIA, MiB, 2025, 6, 9)]
CASES += [("C3", ENWIK, MiB, 2025, i, 1) for i in (0, 1, 65535)]
CASES += [("C5", kind, 16 * MiB, 2025, 0, 9) for kind in (VOCAB, FOUR, RUNS)]
CASES += [("C5-1MiB", kind, MiB, 2025, 1, 9) for kind in (VOCAB, FOUR, RUNS)]


def de_bruijn(k, n):
    """de Bruijn sequence B(k, n) (the standard Lyndon-word construction)."""
    a = [0] * k * n
    seq = []

    def db(t, p):
        if t > n:
            if n % p == 0:
                seq.extend(a[1:p + 1])
        else:
            a[t] = a[t - p]
            db(t + 1, p)
            for j in range(a[t - p] + 1, k):
                a[t] = j
                db(t + 1, t)
    db(1, 1)
    return seq


def literal_input(n):
    s = de_bruijn(64, 3)
    s = s + s[:2]
    assert n <= len(s)
    return bytes(0x30 + x for x in s[:n])


def main():
    ref, o = Reference(), Oracle()
    out = {"reference": ref.version.decode(), "cases": [], "literal_blocks": []}
    for name, kind, n, seed, gidx, level in CASES:
        data = o.generate(n, 1, kind, seed, gidx)[0]
        rc, z = ref.compress2(data, level)
        assert rc == 0
        out["cases"].append({"name": name, "kind": kind, "n": n, "seed": seed, "index": gidx,
                             "level": level, "input_sha256": hashlib.sha256(data).hexdigest(),
                             "adler32": ref.adler32(data), "crc32": ref.crc32(data),
                             "len": len(z), "sha256": hashlib.sha256(z).hexdigest()})
        print(name, kind, n, gidx, level, "ratio %.3f" % (n / len(z)), flush=True)
    for k in (1, 2, 3, 16):
        data = literal_input(16383 * k)
        ent = {"k": k, "n": len(data), "input_sha256": hashlib.sha256(data).hexdigest(), "levels": {}}
        for level in (1, 6, 9):
            rc, z = ref.compress2(data, level)
            assert rc == 0
            ent["levels"][str(level)] = {"len": len(z), "sha256": hashlib.sha256(z).hexdigest()}
        out["literal_blocks"].append(ent)
    path = os.path.join(HERE, "bench_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(out['cases'])} cases")


if __name__ == "__main__":
    main()
