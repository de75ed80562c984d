"""Regenerate tests/golden/golden.json from the COMPILED REFERENCE.

Run in the build container only (the reference library oracle/_ref/libzref.so
is built there from /root/reference by `make -C oracle ref` and never leaves
it):

    make -C oracle ref && python tests/golden/make_golden.py

The fixture holds, per case, the input's sha256 (inputs are regenerated from
tests/datagen.py with the recorded kind/size/seed), the reference's
compress2() output length + sha256 for levels 0..9, the full output bytes for
small cases, raw-deflate (windowBits -15) and gzip (31) outputs for level 6,
deflateInit2_ strategy outputs (1..4 at levels 1/4/6/9), and crc32/adler32
values, plus a few public known answers.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import datagen  # noqa: E402
from zhelpers import Reference  # noqa: E402

# (kind, n, seed): the edge sizes of SURVEY Appendix A.6 over several data
# kinds, plus a few larger mixes.
CASES = []
for n in (0, 1, 2, 3, 4, 5, 15, 16, 17, 258, 262, 1000, 16383, 16384, 32506, 32768, 65536, 65537):
    for kind in ("random", "text", "runs", "four"):
        CASES.append((kind, n, 3 + n % 11))
for n in (100000, 300000):
    for kind in ("mix", "text", "records", "markup"):
        CASES.append((kind, n, 7))
CASES.append(("mix", 1 << 20, 11))
CASES.append(("four", 1 << 20, 12))
CASES.append(("runs", 1 << 20, 13))

FULL_BYTES_MAX = 4096


STRATEGY_MAX_N = 1 << 20


def main():
    ref = Reference()
    out = {"reference": ref.version.decode(), "cases": [], "known": {}}
    for kind, n, seed in CASES:
        data = datagen.make(kind, n, seed)
        assert len(data) == n
        case = {"kind": kind, "n": n, "seed": seed,
                "sha256": hashlib.sha256(data).hexdigest(),
                "crc32": ref.crc32(data), "adler32": ref.adler32(data), "levels": {}}
        for level in range(10):
            rc, z = ref.compress2(data, level)
            assert rc == 0
            ent = {"len": len(z), "sha256": hashlib.sha256(z).hexdigest()}
            if len(z) <= FULL_BYTES_MAX:
                ent["hex"] = z.hex()
            case["levels"][str(level)] = ent
        for name, wbits in (("raw6", -15), ("gzip6", 31)):
            z = ref.deflate(data, 6, wbits)
            case[name] = {"len": len(z), "sha256": hashlib.sha256(z).hexdigest()}
        # deflateInit2_ strategies 1..4 (Z_FILTERED, Z_HUFFMAN_ONLY, Z_RLE,
        # Z_FIXED), zlib wrapper, levels 1/4/6/9
        if n <= STRATEGY_MAX_N:
            case["strategies"] = {}
            for strategy in (1, 2, 3, 4):
                for level in (1, 4, 6, 9):
                    z = ref.deflate(data, level, 15, strategy=strategy)
                    case["strategies"][f"{strategy}/{level}"] = {
                        "len": len(z), "sha256": hashlib.sha256(z).hexdigest()}
        out["cases"].append(case)
    for s in (b"", b"123456789", b"Hello, World!", b"a"):
        out["known"][s.hex()] = {"crc32": ref.crc32(s), "adler32": ref.adler32(s),
                                 "z1": ref.compress2(s, 1)[1].hex(),
                                 "z6": ref.compress2(s, 6)[1].hex(),
                                 "z9": ref.compress2(s, 9)[1].hex()}
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(out['cases'])} cases")


if __name__ == "__main__":
    main()
