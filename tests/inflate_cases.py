"""Inflate parity cases shared by tests/golden/make_inflate_golden.py and the
tests: a case is a RECIPE for a deflate stream (an input from datagen.py,
compressed at a level/wrapper/strategy, then mutated) or a crafted stream in
hex, plus an output capacity and the wrapper the decoder expects."""
import hashlib
import random
import struct
import zlib as _pz

import datagen

WBITS = {0: -15, 1: 15, 2: 31}


def base_stream(case, compress):
    """compress(data, level, wrap, strategy) -> bytes"""
    data = datagen.make(case["kind"], case["n"], case["seed"])
    return data, compress(data, case["level"], case["wrap"], case["strategy"])


def mutate(z, mut):
    kind = mut[0]
    if kind == "none":
        return z
    if kind == "trunc":
        return z[: mut[1]]
    if kind == "flip":
        zz = bytearray(z)
        zz[mut[1] >> 3] ^= 1 << (mut[1] & 7)
        return bytes(zz)
    if kind == "garbage":              # valid prefix + seeded random tail
        rng = random.Random(mut[2])
        return z[: mut[1]] + bytes(rng.randrange(256) for _ in range(mut[3]))
    raise ValueError(kind)


def stream_of(case, compress):
    if "hex" in case:
        return bytes.fromhex(case["hex"])
    data, z = base_stream(case, compress)
    return mutate(z, case["mut"])


def make_recipes(seed=5):
    """Seeded list of recipe cases (without expectations)."""
    rng = random.Random(seed)
    out = []
    kinds = ["text", "runs", "random", "mix", "four", "records", "markup"]
    sizes = [0, 1, 3, 258, 300, 3000, 16384, 40000, 70000, 200000]
    for t in range(140):
        kind = kinds[t % len(kinds)]
        n = sizes[t % len(sizes)] if t < 70 else rng.choice(sizes)
        base = {"kind": kind, "n": n, "seed": 100 + t,
                "level": rng.choice([0, 1, 2, 4, 6, 9]),
                "strategy": rng.choice([0, 0, 0, 1, 2, 3, 4]),
                "wrap": rng.choice([0, 1, 1, 2])}
        dwrap = base["wrap"] if base["wrap"] != 2 or t % 3 else 3
        def add(mut, cap):
            c = dict(base)
            c.update(mut=mut, cap=cap, dwrap=dwrap)
            out.append(c)
        add(["none"], n)
        add(["none"], n + 17)
        add(["none"], 0)
        if n:
            add(["none"], rng.randrange(n))
        # lengths of the base stream are not known here: mutations index
        # through a fraction resolved by the generator
        for k in range(2):
            add(["trunc_frac", rng.random()], n + 5)
        for k in range(4):
            add(["flip_frac", rng.random()], n + 64)
        add(["garbage_frac", rng.random(), rng.randrange(1 << 30), rng.randrange(1, 48)], n + 64)
    return out


def resolve(case, zlen):
    """Turn *_frac mutations into absolute ones for a base stream of zlen bytes."""
    m = case["mut"]
    if m[0] == "trunc_frac":
        case["mut"] = ["trunc", int(m[1] * (zlen + 1))]
    elif m[0] == "flip_frac":
        case["mut"] = ["flip", min(int(m[1] * zlen * 8), max(zlen * 8 - 1, 0))]
    elif m[0] == "garbage_frac":
        case["mut"] = ["garbage", int(m[1] * (zlen + 1)), m[2], m[3]]
    return case


def crafted(seed=9, count=900):
    """Random/crafted streams exercising headers, block headers and code sets."""
    rng = random.Random(seed)

    def rb(k):
        return bytes(rng.randrange(256) for _ in range(k))
    out = []
    for t in range(count):
        k = rng.choice([1, 2, 3, 5, 10, 40, 200])
        mode = t % 6
        if mode == 0:
            src, wrap = rb(k), 0
        elif mode == 1:
            src, wrap = b"\x78\x9c" + rb(k), 1
        elif mode == 2:
            first = (rng.randrange(256) & ~7) | 4 | rng.randrange(2)
            src, wrap = bytes([first]) + rb(k), 0
        elif mode == 3:
            src, wrap = rb(2) + rb(k), rng.choice([1, 3])
        elif mode == 4:
            flg = rng.randrange(32) if rng.random() < 0.9 else rng.randrange(256)
            h = b"\x1f\x8b\x08" + bytes([flg]) + rb(4) + bytes([0, 3])
            if flg & 4:
                x = rb(rng.randrange(5))
                h += struct.pack("<H", len(x)) + x
            if flg & 8:
                h += b"name\x00"
            if flg & 16:
                h += b"comment\x00"
            if flg & 2:
                c = _pz.crc32(h) & 0xFFFF
                if rng.random() < 0.3:
                    c ^= 1
                h += struct.pack("<H", c)
            data = b"hello" * k
            co = _pz.compressobj(6, 8, -15)
            body = co.compress(data) + co.flush()
            tr = struct.pack("<II", _pz.crc32(data) ^ (1 if rng.random() < 0.2 else 0),
                             len(data) + (1 if rng.random() < 0.1 else 0))
            src = h + body + tr
            if rng.random() < 0.3:
                src = src[: rng.randrange(len(src) + 1)]
            wrap = rng.choice([2, 3, 1])
        else:
            cmf = (rng.randrange(16) << 4) | 8
            flg = rng.choice([0, 0x20])
            v = (cmf << 8) | flg
            flg |= 31 - v % 31 if v % 31 else 0
            src, wrap = bytes([cmf, flg]) + rb(k), 1
        out.append({"hex": src.hex(), "dwrap": wrap, "cap": rng.choice([0, 1, 10, 1000, 100000])})
    return out


def sha(b):
    return hashlib.sha256(b).hexdigest()
