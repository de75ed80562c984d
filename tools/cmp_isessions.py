"""Diff gpurun_out/dbg/isess.json (tools/run_isessions.py) with the golden inflate sessions."""
import json
ours = json.load(open("gpurun_out/dbg/isess.json"))
bad = 0
for s in json.load(open("tests/golden/isession_golden.json"))["sessions"]:
    o = ours[s["name"]]
    for k in ("res", "outs", "hdr"):
        if o[k] != s[k]:
            bad += 1
            print(s["name"], k, "\n  ref:", json.dumps(s[k])[:400], "\n  gpu:", json.dumps(o[k])[:400])
            break
print(len(ours), "sessions,", bad, "mismatched")
