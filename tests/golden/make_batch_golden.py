"""Regenerate tests/golden/batch_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so, `make -C oracle ref`):

    python tests/golden/make_batch_golden.py

Bench-scale parity: one whole sub-batch of the benchmark's
shape goes through zgpu_deflate_batch_dev in tests/test_gpu.py
(test_bench_scale_subbatch_golden) -- 4096 x 1 MiB Silesia-style buffers at
level 6 (one 4 GiB in-flight sub-batch, bench.py's seed and global indices
0..4095: the lane-built trees, the pipelined two-slot path) and 4096 x 1 MiB
enwik-style buffers at level 1.  A strided sample of the global indices is
compressed here by the reference's compress2(); each case records the index,
the input's sha256 (pinning the device generator), the stream's length and
sha256.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from zhelpers import Oracle, Reference  # noqa: E402

SILESIA, ENWIK = 1, 2
MiB = 1 << 20
BATCHES = [
    # (name, kind, seed, level, buffers in the launch, sampled indices)
    ("C4-L6-subbatch", SILESIA, 2025, 6, 4096, [64 * k + (37 * k) % 64 for k in range(64)]),
    ("C3-L1-subbatch", ENWIK, 2025, 1, 4096, [128 * k + (53 * k) % 128 for k in range(32)]),
]


def main():
    ref, o = Reference(), Oracle()
    out = {"reference": ref.version.decode(), "batches": []}
    for name, kind, seed, level, count, idx in BATCHES:
        cases = []
        for i in idx:
            data = o.generate(MiB, 1, kind, seed, i)[0]
            rc, z = ref.compress2(data, level)
            assert rc == 0
            cases.append({"index": i, "input_sha256": hashlib.sha256(data).hexdigest(),
                          "len": len(z), "sha256": hashlib.sha256(z).hexdigest()})
        out["batches"].append({"name": name, "kind": kind, "seed": seed, "level": level, "n": MiB,
                               "buffers": count, "cases": cases})
        print(name, len(cases), "cases", flush=True)
    path = os.path.join(HERE, "batch_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
