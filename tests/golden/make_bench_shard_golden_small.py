"""Per-rank digests of bench.py's --cpu-dry-run at a small size, from the
COMPILED REFERENCE (build container only: `make -C oracle ref liboracle.so &&
python tests/golden/make_bench_shard_golden_small.py`).

bench.py --gpus 8 --cpu-dry-run --buffers 3 --buffer-bytes 20000 compresses,
on rank r, the Silesia-style buffers of global indices [3 r, 3 r + 3) (seed
2025, the device generator's host twin) at level 6.  For each of 8 ranks this
records the digest bench.py prints in `per_rank` (sum of the stream lengths,
XOR of the stream CRC-32s) of the reference's compress2() streams, in
bench_shard_golden_small.json.  Only data goes into the repo.
"""
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

SILESIA = 1
SEED = 2025
LEVEL = 6
PER_RANK = 3
NBYTES = 20000
RANKS = 8


def main():
    from zhelpers import Oracle, Reference
    o, r = Oracle(), Reference()
    ranks = {}
    for rk in range(RANKS):
        ob = dg = 0
        for g in range(rk * PER_RANK, (rk + 1) * PER_RANK):
            data = o.generate(NBYTES, 1, SILESIA, SEED, g)[0]
            rc, z = r.compress2(data, LEVEL)
            assert rc == 0, (g, rc)
            ob += len(z)
            dg ^= zlib.crc32(z) & 0xffffffff
        ranks[str(rk)] = {"out_bytes": ob, "stream_crc_xor": "%08x" % dg}
    doc = {"what": "bench.py --cpu-dry-run per-rank digests of the reference's compress2() streams",
           "kind": "silesia", "buffer_bytes": NBYTES, "buffers_per_rank": PER_RANK, "level": LEVEL,
           "seed": SEED, "reference": r.version.decode(), "ranks": ranks}
    json.dump(doc, open(os.path.join(HERE, "bench_shard_golden_small.json"), "w"), indent=1)
    print(doc)


if __name__ == "__main__":
    main()
