"""Debug aid (tools only, GPU box): the deflateParams fast <-> huff/rle
sessions on libzgpu.so against the reference's bytes (hrf_ref.json): per
session, the calls' results and the first byte where the streams differ,
and the data the engine's stream inflates to."""
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
R = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "tests", "golden"))
sys.path.insert(0, os.path.join(R, "zlib.wasm_amd"))
import zgpu  # noqa: E402
from make_api_golden import _slice, deflate_sessions  # noqa: E402
from zhelpers import run_zsession  # noqa: E402

L = zgpu.load()
ref = json.load(open(os.path.join(HERE, "hrf_ref.json")))
ours = {}
for sess in deflate_sessions():
    name = sess["name"]
    if name not in ref:
        continue
    ops = [[o[0], _slice(o[1])] + o[2:] if o[0] in ("deflate", "dict") else o for o in sess["ops"]]
    rcs, z = run_zsession(L, ops)
    rz = bytes.fromhex(ref[name]["z"])
    ours[name] = z.hex()
    rcs = json.loads(json.dumps(rcs))
    k = next((i for i in range(min(len(z), len(rz))) if z[i] != rz[i]), None)
    wb = ops[0][2]
    data = b"".join(o[1] for o in ops if o[0] == "deflate")
    try:
        d = zlib.decompressobj(wb if wb > 0 else wb).decompress(z)
        ok = d == data
    except zlib.error as e:
        ok = str(e)
    print(name, "OK" if (z == rz and rcs == ref[name]["rcs"]) else "BAD", "len", len(z), len(rz), "first diff", k,
          "inflates", ok)
    if rcs != ref[name]["rcs"]:
        print("   rcs ours", rcs)
        print("   rcs ref ", ref[name]["rcs"])
    if k is not None:
        print("   ours", z[max(0, k - 8):k + 24].hex())
        print("   ref ", rz[max(0, k - 8):k + 24].hex())
os.makedirs(os.path.join(R, "gpurun_out", "dbg"), exist_ok=True)
json.dump(ours, open(os.path.join(R, "gpurun_out", "dbg", "hrf_ours.json"), "w"))
