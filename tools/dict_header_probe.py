"""Probe the first-call-is-the-header sessions that differ from the system zlib (tests/test_gpu_fuzz.py):
prints each op's results on both libraries and the first differing stream byte, for a session with a
dictionary and the same session without one."""
import sys

sys.path.insert(0, "zlib.wasm_amd")
sys.path.insert(0, "tests")
import torch  # noqa: E402,F401
import zgpu  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402
from zhelpers import run_zsession  # noqa: E402

libz = F._system_zlib()
L = zgpu.load()
S = F._dict_header_sessions()
for k in (828, 834, 1170):
    refused, ops = S[k]
    for variant in ("dict", "nodict"):
        o = ops if variant == "dict" else [ops[0]] + [[op[0], op[1], op[2], 2] + op[4:] if op[0] == "deflate1" and op[3] == 6 else op for op in ops[2:]]
        rz, z = run_zsession(libz, o)
        rg, g = run_zsession(L, o)
        diff = next((i for i in range(min(len(z), len(g))) if z[i] != g[i]), None)
        print(k, variant, ops[0], "n", len(ops[2][1]), "flush", ops[2][2], "same" if (rz == rg and z == g) else "DIFF")
        print("   sys", rz[-4:], len(z))
        print("   gpu", rg[-4:], len(g), "first diff byte", diff)
