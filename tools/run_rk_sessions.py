"""Run the api_golden rk-* (deflateResetKeep) and pp-* (deflatePrime after a pause) sessions on libzgpu.so (GPU box): return codes and
streams to gpurun_out/dbg/rk.json, compared here against the compiled reference
(tools/cmp_rk_sessions.py; the goldens stay in tests/golden/)."""
import json, os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, "zlib.wasm_amd")
import zgpu
from zhelpers import run_zsession
from make_api_golden import _slice
L = zgpu.load()
g = json.load(open("tests/golden/api_golden.json"))
out = {}
for s in g["deflate"]:
    if not s["name"].startswith(("rk-", "pp-")):
        continue
    ops = [[o[0], _slice(o[1])] + o[2:] if o[0] in ("deflate", "dict", "deflate1") else o for o in s["ops"]]
    rcs, z = run_zsession(L, ops)
    out[s["name"]] = {"rcs": json.loads(json.dumps(rcs)), "z": z.hex()}
os.makedirs("gpurun_out/dbg", exist_ok=True)
json.dump(out, open("gpurun_out/dbg/rk.json", "w"))
print("done", len(out))
