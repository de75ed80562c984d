"""Replay tests/golden/api_golden.json on libzgpu.so and print, per session
that differs, the first op whose result differs (expected vs got).
Usage: python tools/run_api_sessions.py [name-substring]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib.wasm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import zgpu  # noqa: E402
from make_api_golden import run_backcase, run_deflate, run_inflate  # noqa: E402


def first_diff(ops, want, got):
    for i, (w, g) in enumerate(zip(want, got)):
        if w != g:
            op = ops[i] if ops and i < len(ops) else None
            return i, op, w, g
    return len(want), None, want[len(got):], got[len(want):]


def main():
    sub = sys.argv[1] if len(sys.argv) > 1 else ""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "api_golden.json")))
    L = zgpu.load()
    nbad = 0
    for sess in g["inflate"]:
        if sub not in sess["name"]:
            continue
        r = run_inflate(L, sess)
        if r["res"] != sess["res"] or r["outs"] != sess["outs"]:
            nbad += 1
            ops = [o for o in sess["ops"] if o[0] not in ("feed", "skip", "use")]
            i, op, w, gg = first_diff(ops, sess["res"], r["res"])
            print(f"{sess['name']}: op {i} {op}: want {str(w)[:300]} got {str(gg)[:300]}; outs "
                  f"{'same' if r['outs'] == sess['outs'] else (sess['outs'], r['outs'])}", flush=True)
    for sess in g["deflate"]:
        if sub not in sess["name"]:
            continue
        r = run_deflate(L, sess)
        if r["res"] != sess["res"] or r["out"] != sess["out"]:
            nbad += 1
            i, op, w, gg = first_diff([[o[0]] + o[2:] if o[0] in ("deflate", "dict") else o for o in sess["ops"]],
                                      sess["res"], r["res"])
            print(f"{sess['name']}: op {i} {op}: want {str(w)[:300]} got {str(gg)[:300]}; out "
                  f"{'same' if r['out'] == sess['out'] else (sess['out'], r['out'])}", flush=True)
    for case in g["back"]:
        if sub not in case["name"]:
            continue
        r = run_backcase(L, case)
        if r["res"] != case["res"] or r["out"] != case["out"]:
            nbad += 1
            print(f"{case['name']}: want {case['res']} {case['out'][0]} got {r['res']} {r['out'][0]}", flush=True)
    print("sessions that differ:", nbad)


if __name__ == "__main__":
    main()
