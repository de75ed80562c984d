"""Regenerate tests/golden/params_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so, `make -C oracle ref`):

    python tests/golden/make_params_golden.py

deflateInit2_'s windowBits and memLevel (deflate.c:379-524): hash_bits =
memLevel + 7 and hash_shift change the hash chains, lit_bufsize = 1 << (memLevel
+ 6) the block cut, w_size / MAX_DIST the match window and the slide schedule,
windowBits the zlib header; windowBits 8 is coded as 9.  For each (level,
windowBits, memLevel, strategy) on a few inputs the fixture records the
stream's length and sha256 (and the hex for short ones), plus deflateInit2_'s
return code for out-of-range parameters and deflateBound for each setting.
System zlib (Python's zlib, 1.2.11 here) is compared too and the settings where
it differs from the reference are listed (`system_zlib_differs`): 1.2.11's
deflate_stored predates fixes the reference has, so only the reference pins.
"""
import hashlib
import json
import os
import sys
import zlib as pyzlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import datagen  # noqa: E402
from zhelpers import Reference  # noqa: E402

INPUTS = [("text", 120000, 5), ("mix", 200000, 6), ("four", 70000, 7), ("runs", 90000, 8),
          ("random", 20000, 9), ("text", 3000, 10)]
SETTINGS = []
for wb in (8, 9, 10, 12, 14, 15):
    for ml in (1, 2, 4, 7, 8, 9):
        for level in (0, 1, 3, 4, 6, 9):
            SETTINGS.append((level, wb, ml, 0))
for wb in (-9, -12, -15, 25, 28, 31):
    for ml in (1, 5, 9):
        for level in (1, 6, 9):
            SETTINGS.append((level, wb, ml, 0))
for strategy in (1, 2, 3, 4):
    for wb, ml in ((9, 1), (11, 3), (13, 9), (15, 6)):
        for level in (1, 6):
            SETTINGS.append((level, wb, ml, strategy))
BAD = [(6, 7, 8), (6, -8, 8), (6, 24, 8), (6, 16, 8), (6, 32, 8), (6, -16, 8), (6, 15, 0), (6, 15, 10),
       (6, 8, 8), (6, 9, 1), (6, 31, 9)]


def main():
    ref = Reference()
    datas = [datagen.make(k, n, s) for k, n, s in INPUTS]
    out = {"reference": ref.version.decode(), "inputs": [list(x) for x in INPUTS], "cases": [], "init_rc": [],
           "bound": [], "system_zlib": pyzlib.ZLIB_RUNTIME_VERSION, "system_zlib_differs": []}
    for level, wb, ml, strategy in SETTINGS:
        ent = {"level": level, "window_bits": wb, "mem_level": ml, "strategy": strategy, "streams": []}
        for d in datas:
            z = ref.deflate(d, level, wb, strategy=strategy, mem_level=ml)
            c = pyzlib.compressobj(level, pyzlib.DEFLATED, wb, ml, strategy)
            if c.compress(d) + c.flush() != z:
                out["system_zlib_differs"].append([level, wb, ml, strategy])
            e = {"len": len(z), "sha256": hashlib.sha256(z).hexdigest()}
            if len(z) <= 256:
                e["hex"] = z.hex()
            ent["streams"].append(e)
        out["cases"].append(ent)
    for level, wb, ml in BAD:
        out["init_rc"].append({"level": level, "window_bits": wb, "mem_level": ml,
                               "rc": ref.init_rc(level, wb, ml)})
    for level, wb, ml, strategy in SETTINGS[:: 7]:
        for n in (0, 1000, 100000, 1 << 20):
            out["bound"].append({"level": level, "window_bits": wb, "mem_level": ml, "strategy": strategy,
                                 "n": n, "bound": ref.bound(level, wb, ml, strategy, n)})
    path = os.path.join(HERE, "params_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(out['cases'])} settings x {len(datas)} inputs")


if __name__ == "__main__":
    main()
