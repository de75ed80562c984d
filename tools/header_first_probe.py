"""Run the first-call-is-the-header sessions of tests/test_gpu_fuzz.py (with and without a dictionary) on
libzgpu.so and the system zlib and list every session whose calls differ, with the ops' results."""
import sys

sys.path.insert(0, "zlib.wasm_amd")
sys.path.insert(0, "tests")
import torch  # noqa: E402,F401
import zgpu  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402
from zhelpers import run_zsession  # noqa: E402

libz = F._system_zlib()
L = zgpu.load()
for k, (refused, ops) in enumerate(F._dict_header_sessions()):
    if refused:
        continue
    rz, z = run_zsession(libz, ops)
    rg, g = run_zsession(L, ops)
    if rz != rg or z != g:
        short = lambda r: [x if not (isinstance(x, list) and len(x) > 6) else x[:3] + ["...%d" % len(x)] for x in r]
        print(k, ops[0], [op[:1] + [len(op[1])] + op[2:4] for op in ops[1:3]], "sys", short(rz), len(z),
              "gpu", short(rg), len(g), flush=True)
print("done")
