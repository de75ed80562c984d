"""Debug aid (tools only, GPU box): streaming inflate sessions on libzgpu.so
against the system zlib (the small-output randomized sessions of
tests/test_gpu_fuzz.py) and against the reference's records
(tests/golden/isession_golden.json): for each session that differs, the
first differing call with the calls around it."""
import json
import os
import random
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "tests", "golden"))
sys.path.insert(0, os.path.join(R, "zlib.wasm_amd"))
import zgpu  # noqa: E402
import test_gpu_fuzz as T  # noqa: E402
from make_isession_golden import build_z  # noqa: E402
from zhelpers import run_iops  # noqa: E402

L = zgpu.load()
libz = T._system_zlib()


def calls(ops):
    """(op, input fed so far) for each op that records a result"""
    out, fed = [], 0
    for o in ops:
        if o[0] == "feed":
            fed += o[1]
            continue
        if o[0] == "skip":
            continue
        out.append((o, fed))
    return out


def show(tag, ops, rz, rg, zlen):
    first = next((i for i, (a, b) in enumerate(zip(rz[0], rg[0])) if a != b), None)
    if first is None and rz == rg:
        return 0
    cs = calls(ops)
    print(f"{tag}: len {zlen} first {first} nres {len(rz[0])}/{len(rg[0])} outs {[len(o) for o in rz[1]]} "
          f"{[len(o) for o in rg[1]]}")
    if first is None:
        return 1
    for i in range(max(0, first - 3), min(len(rz[0]), first + 2)):
        o, fed = cs[i] if i < len(cs) else (None, None)
        a, b = rz[0][i], rg[0][i] if i < len(rg[0]) else None
        if isinstance(a, list) and a and isinstance(a[0], list):       # a loop: the first differing call in it
            j = next((k for k, (x, y) in enumerate(zip(a, b or [])) if x != y), min(len(a), len(b or [])))
            a, b = a[max(0, j - 2):j + 2], (b or [])[max(0, j - 2):j + 2]
            o = (o, "loop call", j)
        print(f"   {i} {o} fed {fed}\n      ref  {a}\n      ours {b}")
    return 1


nbad = 0
for block in (0, 1):
    rng = random.Random(7373 + block)
    for k in range(30):
        z, ops = T._istream(rng, libz, small_out=True)
        rz = run_iops(libz, z, ops)
        rg = run_iops(L, z, ops)
        if nbad < 12:
            nbad += show(f"fuzz{block}.{k}", ops, rz, rg, len(z))
print("fuzz sessions differing (first 12 shown):", nbad)
nt = 0
for block in (0, 1):
    rng = random.Random(6161 + block)
    for k in range(30):
        z, ops = T._istream(rng, libz, small_out=True, flushes=(0, 5, 6, 6))
        rz = run_iops(libz, z, ops)
        rg = run_iops(L, z, ops)
        if nt < 8:
            nt += show(f"trees{block}.{k}", ops, rz, rg, len(z))
print("Z_TREES fuzz sessions differing (first 8 shown):", nt)
g = json.load(open(os.path.join(R, "tests", "golden", "isession_golden.json")))["sessions"]
nb = 0
for sess in g:
    z = build_z(sess["spec"])
    res, outs, hdr = run_iops(L, z, sess["ops"])
    if res != sess["res"]:
        if nb < 8:
            show(sess["name"], sess["ops"], [sess["res"], [b""]], [res, outs], len(z))
        nb += 1
print("isession sessions differing:", nb)
