"""Regenerate tests/golden/inflate_golden.json from the COMPILED REFERENCE.

Build container only (oracle/_ref/libzref.so never leaves it):

    make -C oracle ref && python tests/golden/make_inflate_golden.py

Every case is a recipe (tests/inflate_cases.py): an input from datagen.py, the
reference's deflate of it at a level / wrapper / strategy (its sha256 is
recorded, so the oracle compressor that rebuilds it elsewhere is checked too),
a mutation (none, truncation, bit flip, garbage tail) and an output capacity;
or a crafted stream in hex.  The expectation is what the reference's
uncompress2 returns (for raw and gzip: uncompress2's loop over the
reference's inflateInit2_/inflate): status, output length and sha256, and
input bytes consumed.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import inflate_cases as ic  # noqa: E402
from zhelpers import Reference  # noqa: E402


def main():
    ref = Reference()

    def compress(data, level, wrap, strategy):
        return ref.deflate(data, level, ic.WBITS[wrap], strategy=strategy)

    cases = []
    for c in ic.make_recipes():
        data, z = ic.base_stream(c, compress)
        c = ic.resolve(c, len(z))
        c["base_sha256"] = ic.sha(z)
        src = ic.mutate(z, c["mut"])
        rc, out, used = ref.uncompress(src, c["cap"], c["dwrap"])
        c["expect"] = {"status": rc, "len": len(out), "sha256": ic.sha(out), "consumed": used}
        cases.append(c)
    for c in ic.crafted():
        rc, out, used = ref.uncompress(bytes.fromhex(c["hex"]), c["cap"], c["dwrap"])
        c["expect"] = {"status": rc, "len": len(out), "sha256": ic.sha(out), "consumed": used}
        cases.append(c)
    doc = {"reference": ref.version.decode(), "cases": cases}
    with open(os.path.join(HERE, "inflate_golden.json"), "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    st = {}
    for c in cases:
        st[c["expect"]["status"]] = st.get(c["expect"]["status"], 0) + 1
    print(len(cases), "cases; statuses", st)


if __name__ == "__main__":
    main()
