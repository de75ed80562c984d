"""Deterministic host-side test inputs (numpy only; no GPU).

The benchmark's own inputs are produced on the device (zgpu_generate_dev);
these are the host-side shapes the parity tests and golden fixtures use:
random bytes, English-like word text, byte runs, 4-letter alphabet, XML-ish
markup, little-endian binary records, and a 64 KiB-segment mix of all of them
(the "Silesia-style" shape of SURVEY §8d).
"""
import numpy as np

WORDS = ("the of and to in a is that for it as was with be by on not he this are or his "
         "from at which but have an they you were her she there one all we their been has "
         "would when who will more if no out so said what up its about into than them can "
         "only other new some could time these two may then do first any my now such like "
         "compression window stream buffer data history council government river north").split()


def random_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def text(n, seed, vocab=None):
    rng = np.random.default_rng(seed)
    words = WORDS if vocab is None else WORDS[:vocab]
    k = max(16, n // 3)
    idx = np.minimum((rng.random(k) * rng.random(k) * len(words)).astype(np.int64), len(words) - 1)
    seps = rng.choice([" ", " ", " ", " ", " ", ", ", ". ", ".\n"], size=k)
    out = "".join(w + s for w, s in zip((words[i] for i in idx), seps)).encode()
    while len(out) < n:
        out += out
    return out[:n]


def runs(n, seed):
    rng = np.random.default_rng(seed)
    vals = rng.integers(0, 256, n // 4 + 2, dtype=np.uint8)
    lens = np.where(rng.random(len(vals)) < 0.15, rng.integers(64, 512, len(vals)),
                    rng.integers(1, 48, len(vals)))
    return np.repeat(vals, lens)[:n].tobytes().ljust(n, b"\0")


def fourletter(n, seed):
    rng = np.random.default_rng(seed)
    return np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, n)].tobytes()


def markup(n, seed):
    rng = np.random.default_rng(seed)
    parts, total, rid = [], 0, int(rng.integers(0, 1 << 20))
    while total < n:
        a, b, c = (WORDS[int(i)] for i in rng.integers(0, len(WORDS), 3))
        s = (f'<row id="{rid}"><name>{a} {b}</name><city>{c}</city>'
             f'<value>{int(rng.integers(0, 100000))}</value></row>\n')
        parts.append(s)
        total += len(s)
        rid += 1
    return "".join(parts).encode()[:n]


def records(n, seed):
    rng = np.random.default_rng(seed)
    k = n // 12 + 1
    rec = np.zeros((k, 12), dtype=np.uint8)
    ids = (int(rng.integers(0, 1 << 31)) + np.arange(k)).astype(np.uint32)
    vals = (int(rng.integers(0, 1 << 24)) + np.cumsum(rng.integers(-16, 17, k))).astype(np.uint32)
    rec[:, 0:4] = ids.view(np.uint8).reshape(k, 4)
    rec[:, 4:8] = vals.view(np.uint8).reshape(k, 4)
    rec[:, 8] = rng.integers(0, 8, k)
    rec[:, 10] = np.where(rng.random(k) < 0.25, rng.integers(0, 256, k), 0)
    return rec.tobytes()[:n]


KINDS = {"random": random_bytes, "text": text, "runs": runs, "four": fourletter,
         "markup": markup, "records": records}


def mix(n, seed, seg=65536):
    """64 KiB segments: 40 % text, 20 % markup, 20 % records, 10 % random, 10 % runs."""
    rng = np.random.default_rng(seed)
    table = ["text"] * 4 + ["markup"] * 2 + ["records"] * 2 + ["random", "runs"]
    out = bytearray()
    i = 0
    while len(out) < n:
        kind = table[int(rng.integers(0, 10))]
        out += KINDS[kind](min(seg, n - len(out)), seed * 1000 + i)
        i += 1
    return bytes(out[:n])


KINDS["mix"] = mix


def make(kind, n, seed):
    return KINDS[kind](n, seed)
