"""Phase clock of the first block's tree build in k_enc_plan<true> (a ZGPU_PLAN_CLOCK build):
    python3 tools/plan_clock.py ab/libzgpu_planclk.so
Compresses a 64 KiB buffer (text, then the C1 mix) at L6 a few times and prints the
s_memtime deltas (raw ticks; calibrate against the kernel's duration) between the stamps:
0 start, 1 histogram, 2 freqs staged, 3 literal/length tree, 4 distance tree,
5 RLE counts of the bit-length tree (lane 0), 6 bit-length tree, 7 type decision,
8 plan stored; inside the literal/length tree: 10 leaves in the heap, 11 heapified,
12 merges done, 13 depths (pointer jumping), 14 lengths and overflow fix-up."""
import ctypes as C
import sys

sys.path.insert(0, "zlib.wasm_amd")
sys.path.insert(0, "tests")
import torch  # noqa: E402,F401
import zgpu  # noqa: E402
import datagen  # noqa: E402

lib = sys.argv[1]
L = zgpu.load(lib)
clk = (C.c_ulonglong * 32)()
names = {0: "start", 1: "histogram", 2: "freqs", 3: "ltree", 4: "dtree", 5: "rle", 6: "bltree", 7: "type",
         8: "stored", 10: "leaves", 11: "heapify", 12: "merges", 13: "depths", 14: "lengths"}
for kind in ("text", "mix"):
    data = bytes(datagen.make(kind, 64 * 1024, 7))
    for rep in range(3):
        rc, z = zgpu.compress2(data, level=6)
        assert rc == 0
        L.zgpu_plan_clock_read(clk)
        t = list(clk)
        seq = [0, 1, 2, 10, 11, 12, 13, 14, 3, 4, 5, 6, 7, 8]
        parts = []
        for a, b in zip(seq, seq[1:]):
            parts.append(f"{names[b]} {t[b] - t[a]}")
        print(f"{kind} rep {rep}: total {t[8] - t[0]} ticks | " + ", ".join(parts), flush=True)
