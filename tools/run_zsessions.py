"""Run every golden z_stream session in order on libzgpu.so (GPU box); our streams + return codes go to gpurun_out/dbg/all.json.
Compare locally with tools/cmp_zsessions.py (the goldens stay in tests/golden/)."""
import json, os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, "zlib.wasm_amd")
import zgpu
from zhelpers import run_zsession
from make_zstream_golden import materialize
L = zgpu.load()
g = json.load(open("tests/golden/zstream_golden.json"))
out = {}
for s in g["sessions"]:
    rcs, z = run_zsession(L, materialize(s["ops"]))
    out[s["name"]] = {"rcs": rcs, "z": z.hex()}
os.makedirs("gpurun_out/dbg", exist_ok=True)
json.dump(out, open("gpurun_out/dbg/all.json", "w"))
print("done", len(out))
