"""Compare gpurun_out/dbg/all.json (from tools/run_zsessions.py on the GPU box) with tests/golden/zstream_golden.json."""
import hashlib, json

out = json.load(open("gpurun_out/dbg/all.json"))
bad = []
for s in json.load(open("tests/golden/zstream_golden.json"))["sessions"]:
    o = out[s["name"]]
    z = bytes.fromhex(o["z"])
    same = len(z) == s["len"] and hashlib.sha256(z).hexdigest() == s["sha256"]
    if not same or o["rcs"] != s["rcs"]:
        bad.append((s["name"], same, o["rcs"], s["rcs"]))
print(len(out), "sessions,", len(bad), "mismatched")
for b in bad:
    print(*b)
