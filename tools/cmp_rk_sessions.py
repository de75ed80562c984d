"""Compare gpurun_out/dbg/rk.json (tools/run_rk_sessions.py) with the compiled reference, session by
session: return codes and the first differing output byte (build container only)."""
import json, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden")
from zhelpers import Reference, run_zsession
from make_api_golden import _slice
ref = Reference()
g = json.load(open("tests/golden/api_golden.json"))
mine = json.load(open("gpurun_out/dbg/rk.json"))
for s in g["deflate"]:
    if s["name"] not in mine:
        continue
    ops = [[o[0], _slice(o[1])] + o[2:] if o[0] in ("deflate", "dict", "deflate1") else o for o in s["ops"]]
    rcs, z = run_zsession(ref.L, ops)
    k = next(i for i, o in enumerate(ops) if o[0] in ("resetkeep", "prime"))
    _, z0 = run_zsession(ref.L, ops[:k])
    m = mine[s["name"]]
    zm = bytes.fromhex(m["z"])
    rc_ok = json.loads(json.dumps(rcs)) == m["rcs"]
    diff = next((i for i in range(min(len(z), len(zm))) if z[i] != zm[i]), None)
    if diff is None and len(z) != len(zm):
        diff = min(len(z), len(zm))
    print(f"{s['name']:28s} rcs {'ok' if rc_ok else 'DIFF'} len ref {len(z)} mine {len(zm)} old {len(z0)} "
          f"first diff {diff}" + ("" if rc_ok else f"\n   ref {json.loads(json.dumps(rcs))}\n  mine {m['rcs']}"))
