"""Debug aid (tools only): the compiled reference's output of the
deflateParams fast <-> huff/rle sessions of tests/golden/api_golden.json,
saved next to this script for tools/dbg/hrf_diff.py on the GPU box."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
T = os.path.join(os.path.dirname(os.path.dirname(HERE)), "tests")
sys.path.insert(0, T)
sys.path.insert(0, os.path.join(T, "golden"))
from make_api_golden import _slice, deflate_sessions  # noqa: E402
from zhelpers import Reference, run_zsession  # noqa: E402

ref = Reference()
out = {}
for sess in deflate_sessions():
    if not sess["name"].startswith("params-hrf"):
        continue
    ops = [[o[0], _slice(o[1])] + o[2:] if o[0] in ("deflate", "dict") else o for o in sess["ops"]]
    rcs, z = run_zsession(ref.L, ops)
    out[sess["name"]] = {"rcs": json.loads(json.dumps(rcs)), "z": z.hex()}
json.dump(out, open(os.path.join(HERE, "hrf_ref.json"), "w"))
print(len(out), "sessions")
