"""Replay tests/golden/isession_golden.json on libzgpu.so (GPU box); writes our
results to gpurun_out/dbg/isess.json for a local diff (tools/cmp_isessions.py)."""
import json, os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, "zlib.wasm_amd")
import zgpu
from make_isession_golden import run
L = zgpu.load()
g = json.load(open("tests/golden/isession_golden.json"))
out = {s["name"]: run(L, s) for s in g["sessions"]}
os.makedirs("gpurun_out/dbg", exist_ok=True)
json.dump(out, open("gpurun_out/dbg/isess.json", "w"))
print("done", len(out))
