"""Per-stream parity at bench scale, from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so is built there from
/root/reference by `make -C oracle ref`):

    make -C oracle ref liboracle.so && python tests/golden/make_bench_shard_golden.py [ranks]

bench.py's default deflate leg compresses, on rank r, the 32768 Silesia-style
1 MiB buffers of global indices [32768 r, 32768 (r + 1)) (device generator,
seed 2025) at level 6 with the zlib wrapper.  This script rebuilds each of
those inputs on the host (oracle/zgen.c, the same generator), compresses it
with the reference's compress2() (compress.c:22-59) and records:

* rank 0, every stream: its length and the CRC-32 of its bytes
  (bench_shard_golden_r0.npz: two uint32 arrays of 32768, loaded with
  allow_pickle=False);
* ranks 0..7: the per-rank digest bench.py prints in `per_rank` (the sum of
  the stream lengths and the XOR of the stream CRC-32s), in
  bench_shard_golden.json.

bench.py then checks every stream of rank 0 (device-computed CRC-32 and
length) and the other ranks' digests against these, instead of a 64-buffer
sample.  Only data goes into the repo: lengths and check values.
"""
import json
import multiprocessing as mp
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

SILESIA = 1
MiB = 1 << 20
PER_RANK = 32768
SEED = 2025
LEVEL = 6

_o = _r = None


def _init():
    global _o, _r
    from zhelpers import Oracle, Reference
    _o, _r = Oracle(), Reference()


def _one(g):
    data = _o.generate(MiB, 1, SILESIA, SEED, g)[0]
    rc, z = _r.compress2(data, LEVEL)
    assert rc == 0, (g, rc)
    return len(z), zlib.crc32(z) & 0xffffffff


def main():
    ranks = [int(x) for x in sys.argv[1:]] or [0]
    jpath = os.path.join(HERE, "bench_shard_golden.json")
    doc = json.load(open(jpath)) if os.path.exists(jpath) else {
        "what": "bench.py default deflate leg: per-rank digests (sum of stream lengths, XOR of stream CRC-32s) "
                "of the reference's compress2() streams; rank 0 per stream in bench_shard_golden_r0.npz",
        "kind": "silesia", "buffer_bytes": MiB, "buffers_per_rank": PER_RANK, "seed": SEED, "level": LEVEL,
        "ranks": {}}
    from zhelpers import Reference
    doc["reference"] = Reference().version.decode()
    workers = int(os.environ.get("JOBS", os.cpu_count() or 4))
    with mp.Pool(workers, initializer=_init) as pool:
        for r in ranks:
            idx = range(r * PER_RANK, (r + 1) * PER_RANK)
            res = pool.map(_one, idx, chunksize=64)
            lens = np.array([x[0] for x in res], dtype=np.uint32)
            crcs = np.array([x[1] for x in res], dtype=np.uint32)
            doc["ranks"][str(r)] = {"out_bytes": int(lens.sum(dtype=np.uint64)),
                                    "stream_crc_xor": "%08x" % int(np.bitwise_xor.reduce(crcs))}
            if r == 0:
                np.savez_compressed(os.path.join(HERE, "bench_shard_golden_r0.npz"), lens=lens, crcs=crcs)
            print("rank", r, doc["ranks"][str(r)], flush=True)
            with open(jpath, "w") as f:
                json.dump(doc, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
