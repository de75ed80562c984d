"""Trace one first-call-is-the-header session (index into tests/test_gpu_fuzz.py's _dict_header_sessions)
on libzgpu.so with the engine's stream trace (ZGPU_STREAM_TRACE, on stderr), beside the system zlib's
per-call results.  (Round 6 used it with a length guard that was then removed: profiles/r06u_*.)
    ZGPU_STREAM_TRACE=1 python3 tools/header_first_trace.py 995"""
import sys

sys.path.insert(0, "zlib.wasm_amd")
sys.path.insert(0, "tests")
import torch  # noqa: E402,F401
import zgpu  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402
from zhelpers import run_zsession  # noqa: E402

k = int(sys.argv[1])
refused, ops = F._dict_header_sessions()[k]
ops = ops[:4] + [[ops[4][0], ops[4][1], ops[4][2], None, True]]     # stop after the third op
print("ops", ops[0], [op[:1] + [len(op[1])] + op[2:4] for op in ops[1:]], flush=True)
rz, z = run_zsession(F._system_zlib(), ops)
print("sys", rz, len(z), flush=True)
rg, g = run_zsession(zgpu.load(), ops)
short = [x if not (isinstance(x, list) and len(x) > 6) else x[:4] + ["...%d" % len(x)] for x in rg]
print("gpu", short, len(g), flush=True)
