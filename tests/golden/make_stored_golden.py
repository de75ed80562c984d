"""Regenerate tests/golden/stored_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so, `make -C oracle ref`):

    python tests/golden/make_stored_golden.py

Level-0 deflate() call sequences (Z_NO_FLUSH chunks around min_block = 32768
and MAX_STORED = 65535, flush calls, refused repeats, Z_FINISH, repeated
Z_FINISH) over datagen inputs, every call given an output buffer large enough
for it: the reference's status per call, total output after every call, and
the length and sha256 of the stream.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import datagen  # noqa: E402
from zhelpers import Reference  # noqa: E402


def plan(rng, n):
    calls, pos = [], 0
    while pos < n:
        take = int(min(n - pos, rng.choice([0, 1, 3, 300, 20000, 32767, 32768, 40000, 65535, 65536, 140000])))
        calls.append((take, int(rng.choice([0, 0, 0, 1, 2, 3, 5]))))
        pos += take
        if rng.random() < 0.15:
            calls.append((0, int(rng.choice([0, 1, 2, 3, 5]))))
    calls.append((0, 4))
    if rng.random() < 0.3:
        calls.append((0, 4))
    return calls


def main():
    ref = Reference()
    rng = np.random.default_rng(77)
    cases = []
    for t in range(64):
        kind = ["text", "mix", "runs", "random"][t % 4]
        n = int(rng.choice([0, 1, 5, 1000, 40000, 70000, 200000, 600000]))
        seed = 700 + t
        wbits = int(rng.choice([15, -15, 31]))
        data = datagen.make(kind, n, seed)
        calls = plan(rng, n)
        sts, lens, whole = ref.deflate_calls(data, calls, 0, wbits, 0)
        cases.append({"kind": kind, "n": n, "seed": seed, "level": 0, "strategy": 0, "wbits": wbits,
                      "calls": calls, "status": sts, "out_len": lens, "len": len(whole),
                      "sha256": hashlib.sha256(whole).hexdigest(),
                      "input_sha256": hashlib.sha256(data).hexdigest()})
    with open(os.path.join(HERE, "stored_golden.json"), "w") as f:
        json.dump({"reference": ref.version.decode(), "cases": cases}, f, indent=0)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
