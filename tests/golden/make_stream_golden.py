"""Regenerate tests/golden/stream_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so, `make -C oracle ref`):

    python tests/golden/make_stream_golden.py

deflate() sessions with small output buffers and Z_NO_FLUSH input in pieces,
run by tests/zhelpers.run_dsession: zpipe.c-style loops (offer a chunk, call
again while avail_out is used up, Z_FINISH at the end) and free sequences
(each call its own input, flush and output space).  Each fixture records the
reference's return code, avail_in and output length of every call and the
stream's length and sha256; the inputs are tests/datagen.py specs.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import datagen  # noqa: E402
from zhelpers import Reference, run_dsession  # noqa: E402


def zpipe_plan(rng, n, chunk, out, flushes=False):
    plan, pos = [], 0
    while pos < n:
        take = min(chunk, n - pos)
        f = int(rng.choice([0, 0, 0, 1, 2, 3, 5])) if flushes else 0
        plan.append((take, f, out, True))
        pos += take
    plan.append((0, 4, out, True))
    return plan


def free_plan(rng, n):
    plan, pos = [], 0
    while pos < n:
        take = int(min(n - pos, rng.choice([0, 1, 17, 300, 4000, 20000, 70000])))
        f = int(rng.choice([0, 0, 0, 0, 1, 2, 3, 5]))
        out = int(rng.choice([1, 7, 100, 1000, 5000, 40000, 1 << 19] if n <= 70000 else [1000, 5000, 40000, 1 << 19]))
        plan.append((take, f, out, bool(rng.random() < 0.5)))
        pos += take
    plan.append((0, 4, int(rng.choice([1000, 3000, 1 << 19])), True))
    return plan


def main():
    ref = Reference()
    rng = np.random.default_rng(77)
    cases = []
    kinds = ["text", "mix", "runs", "random", "four", "records", "markup"]
    for t in range(140):
        kind = kinds[t % 7]
        n = int(rng.choice([0, 5, 3000, 70000, 200000, 600000]))
        seed = 900 + t
        level = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9][t % 10]
        strategy = int(rng.choice([0, 0, 0, 0, 1, 2, 3, 4]))
        wbits = int(rng.choice([15, 15, -15, 31, 12, -9]))
        mem = int(rng.choice([8, 8, 8, 1, 5, 9]))
        data = datagen.make(kind, n, seed)
        mode = t % 4
        if mode == 0:
            plan = zpipe_plan(rng, n, int(rng.choice([1024, 16384, 65536])),
                              int(rng.choice([16384, 1024, 64] if n <= 70000 else [16384, 1024])))
        elif mode == 1:
            plan = zpipe_plan(rng, n, int(rng.choice([3000, 16384])),
                              int(rng.choice([7, 100, 5000] if n <= 70000 else [700, 5000])), True)
        else:
            plan = free_plan(rng, n)
        recs, whole = run_dsession(ref.L, data, plan, level, wbits, mem, strategy)
        if len(recs) >= 6000 or not recs or recs[-1][0] != 1:
            continue
        cases.append({"kind": kind, "n": n, "seed": seed, "level": level, "strategy": strategy, "wbits": wbits,
                      "mem": mem, "plan": plan, "recs": recs, "len": len(whole),
                      "sha256": hashlib.sha256(whole).hexdigest()})
    # level 0 with output buffers smaller than a stored block (round 5: deflate_stored
    # then cuts blocks by avail_out and goes through the pending buffer,
    # deflate.c:1635-1815); their own rng, so the sessions above stay as they were
    rng0 = np.random.default_rng(1977)
    for t in range(30):
        kind = kinds[t % 7]
        out = [1, 7, 100, 700, 5000, 40000][t % 6]
        n = int(rng0.choice([300, 3000, 5000])) if out <= 7 else int(rng0.choice([3000, 70000, 200000]))
        wbits = int(rng0.choice([15, -15, 31, 9]))
        data = datagen.make(kind, n, 2000 + t)
        if t % 3 == 0:
            plan = [(n, 0, out, True), (0, 4, out, True)]
        elif t % 3 == 1:
            plan = zpipe_plan(rng0, n, int(rng0.choice([1000, 3000, 70000])), out, t % 2 == 1)
        else:
            plan = free_plan(rng0, n)
            plan = [(take, f, min(o, out) if out > 7 else out, loop) for take, f, o, loop in plan]
        recs, whole = run_dsession(ref.L, data, plan, 0, wbits, 8, 0)
        if len(recs) >= 6000 or not recs or recs[-1][0] != 1:
            continue
        cases.append({"kind": kind, "n": n, "seed": 2000 + t, "level": 0, "strategy": 0, "wbits": wbits,
                      "mem": 8, "plan": plan, "recs": recs, "len": len(whole),
                      "sha256": hashlib.sha256(whole).hexdigest()})
    with open(os.path.join(HERE, "stream_golden.json"), "w") as f:
        json.dump({"reference": ref.version.decode(), "cases": cases}, f, separators=(",", ":"))
    print(len(cases), "cases", sum(len(c["recs"]) for c in cases), "calls")


if __name__ == "__main__":
    main()
