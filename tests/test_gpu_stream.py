"""deflate() driven through small output buffers and Z_NO_FLUSH input in
pieces, on the GPU, against tests/golden/stream_golden.json: sessions run
through the compiled reference (tests/golden/make_stream_golden.py,
tests/zhelpers.run_dsession) -- zpipe.c-style loops and free call sequences
at levels 0..9, every strategy, zlib/raw/gzip wrappers, windowBits and
memLevel settings.  Every call's return code, the input it left unconsumed
(avail_in) and the bytes it wrote must be the reference's (deflate.c:763-1265:
need_more after a block when avail_out runs out, FLUSH_BLOCK), and so must the
stream."""
import hashlib
import json
import os

import pytest

import datagen
from zhelpers import run_dsession

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def stream_golden():
    with open(os.path.join(HERE, "golden", "stream_golden.json")) as f:
        return json.load(f)["cases"]


def test_stream_sessions_vs_reference(zg, stream_golden):
    L = zg.load()
    bad = []
    for c in stream_golden:
        data = datagen.make(c["kind"], c["n"], c["seed"])
        plan = [tuple(p) for p in c["plan"]]
        recs, whole = run_dsession(L, data, plan, c["level"], c["wbits"], c["mem"], c["strategy"])
        recs = [list(r) for r in recs]
        tag = (c["kind"], c["n"], c["level"], c["strategy"], c["wbits"], c["mem"])
        if recs != c["recs"] or hashlib.sha256(whole).hexdigest() != c["sha256"]:
            k = next((i for i, (a, b) in enumerate(zip(recs, c["recs"])) if a != b), min(len(recs), len(c["recs"])))
            bad.append((tag, k, recs[k:k + 2], c["recs"][k:k + 2], len(recs), len(c["recs"])))
    assert not bad, bad[:4]


_REPLAY = r"""
import hashlib, json, os, sys
sys.path.insert(0, sys.argv[1])
import datagen, zgpu
from zhelpers import run_dsession
L = zgpu.load()
bad = []
for c in json.load(open(os.path.join(sys.argv[1], "golden", "stream_golden.json")))["cases"]:
    data = datagen.make(c["kind"], c["n"], c["seed"])
    recs, whole = run_dsession(L, data, [tuple(p) for p in c["plan"]], c["level"], c["wbits"], c["mem"],
                               c["strategy"])
    if [list(r) for r in recs] != c["recs"] or hashlib.sha256(whole).hexdigest() != c["sha256"]:
        bad.append((c["kind"], c["n"], c["level"], c["strategy"], c["wbits"], c["mem"]))
print("BAD", json.dumps(bad))
"""


def test_stream_sessions_on_segmented_parse(zg):
    """The same sessions with every streaming job whose events are Z_NO_FLUSH
    stops parsed by k_pbig1..5 + k_pbig6s (ZGPU_SEG_STREAM_MIN=0; by default
    only jobs of >= 1 MiB are), in a child process since the library reads
    the setting once."""
    import subprocess
    import sys
    env = dict(os.environ, ZGPU_SEG_STREAM_MIN="0",
               PYTHONPATH=os.pathsep.join([os.path.join(os.path.dirname(HERE), "zlib.wasm_amd"),
                                           os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", _REPLAY, HERE], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("BAD ")][-1]
    assert json.loads(line[4:]) == [], line


@pytest.mark.parametrize("level", [1, 6])
def test_one_large_call_then_finish_vs_system_zlib(zg, level):
    """The session the round-4 r04c run crashed in (glibc heap corruption,
    then a SIGSEGV inside deflate()): 16 MiB of Silesia-style mix offered to
    ONE deflate(Z_NO_FLUSH) call with room for all of it, then Z_FINISH
    (tools/stream_stages.py 16).  Every device-reported length and record count
    is now checked against the host buffer it sizes before any copy
    (zgpu_api.cpp compress_host_locked); the stream must equal the system
    zlib's for the same two calls."""
    import zlib
    data = datagen.make("mix", 16 << 20, 5)
    cap = len(data) + (len(data) >> 8) + (1 << 16)
    recs, whole = run_dsession(zg.load(), data, [(len(data), 0, cap, True), (0, 4, cap, True)], level)
    c = zlib.compressobj(level)
    want = c.compress(data) + c.flush()
    assert recs[-1][0] == 1, recs
    assert hashlib.sha256(whole).hexdigest() == hashlib.sha256(want).hexdigest()
