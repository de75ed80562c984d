"""Regenerate tests/golden/flush_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so, `make -C oracle ref`):

    python tests/golden/make_flush_golden.py

Each case is a deflate() call sequence (input lengths and flush values:
Z_NO_FLUSH, Z_PARTIAL_FLUSH, Z_SYNC_FLUSH, Z_FULL_FLUSH, Z_BLOCK, repeated
flushes with no input, then Z_FINISH) over a datagen input, with the
reference's status and total output length after every call and the length
and sha256 of the whole stream.  The inputs are regenerated from
tests/datagen.py with the recorded kind/size/seed.
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
        take = int(min(n - pos, rng.choice([0, 1, 2, 3, 17, 300, 4000, 40000, 70000, 200000])))
        flush = int(rng.choice([0, 0, 1, 2, 2, 3, 5]))
        calls.append((take, flush))
        pos += take
        if rng.random() < 0.15:
            calls.append((0, int(rng.choice([1, 2, 3, 5]))))
    calls.append((0, 4))
    return calls


def main():
    ref = Reference()
    rng = np.random.default_rng(2024)
    cases = []
    for t in range(96):
        kind = ["text", "mix", "runs", "random", "four", "records", "markup"][t % 7]
        n = int(rng.choice([0, 1, 5, 1000, 70000, 300000, 1 << 20]))
        seed = 500 + t
        level = [1, 2, 3, 4, 5, 6, 7, 8, 9][t % 9]
        strategy = int(rng.choice([0, 0, 0, 1, 2, 3, 4]))
        wbits = int(rng.choice([15, 15, -15, 31]))
        data = datagen.make(kind, n, seed)
        calls = plan(rng, n)
        sts, lens, whole = ref.deflate_calls(data, calls, level, wbits, strategy)
        cases.append({"kind": kind, "n": n, "seed": seed, "level": level, "strategy": strategy,
                      "wbits": wbits, "calls": calls, "status": sts, "out_len": lens,
                      "len": len(whole), "sha256": hashlib.sha256(whole).hexdigest(),
                      "input_sha256": hashlib.sha256(data).hexdigest()})
    with open(os.path.join(HERE, "flush_golden.json"), "w") as f:
        json.dump({"reference": ref.version.decode(), "cases": cases}, f, indent=0)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
