"""Debug aid (tools only): a deflate stream decoded into its symbols --
(output position, length or 0 for a literal, distance) and block starts --
to find the first parse decision where two streams of the same data differ.
Usage: symtrace.py hrf_ref.json hrf_ours.json name"""
import json
import sys

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class Bits:
    def __init__(self, b, pos=0):
        self.b, self.p = b, pos * 8

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.b[self.p >> 3] >> (self.p & 7)) & 1) << i
            self.p += 1
        return v


def huff(lens):
    code, codes = 0, {}
    for L in range(1, 16):
        for s, l in enumerate(lens):
            if l == L:
                codes[(L, code)] = s
                code += 1
        code <<= 1
    return codes


def dec(br, codes):
    c, L = 0, 0
    while True:
        c = (c << 1) | br.get(1)
        L += 1
        if (L, c) in codes:
            return codes[(L, c)]


def trace(z, start):
    br, out, syms = Bits(z, start), 0, []
    while True:
        last, typ = br.get(1), br.get(2)
        syms.append(("blk", out, typ, br.p))
        if typ == 0:
            br.p = (br.p + 7) & ~7
            n = br.get(16)
            br.get(16)
            br.p += 8 * n
            out += n
        else:
            if typ == 1:
                lc = huff([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8)
                dc = huff([5] * 30)
            else:
                hl, hd, hc = br.get(5) + 257, br.get(5) + 1, br.get(4) + 4
                order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
                cl = [0] * 19
                for i in range(hc):
                    cl[order[i]] = br.get(3)
                cc, lens = huff(cl), []
                while len(lens) < hl + hd:
                    s = dec(br, cc)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + br.get(2))
                    elif s == 17:
                        lens += [0] * (3 + br.get(3))
                    else:
                        lens += [0] * (11 + br.get(7))
                lc, dc = huff(lens[:hl]), huff(lens[hl:])
            while True:
                s = dec(br, lc)
                if s < 256:
                    syms.append((out, 0, s))
                    out += 1
                elif s == 256:
                    break
                else:
                    n = LBASE[s - 257] + br.get(LEXT[s - 257])
                    d = dec(br, dc)
                    dist = DBASE[d] + br.get(DEXT[d])
                    syms.append((out, n, dist))
                    out += n
        if last:
            return syms


if __name__ == "__main__":
    ref, ours, name = json.load(open(sys.argv[1])), json.load(open(sys.argv[2])), sys.argv[3]
    a, b = bytes.fromhex(ref[name]["z"]), bytes.fromhex(ours[name])
    st = 2 if (a[0] & 0x0f) == 8 and ((a[0] << 8) | a[1]) % 31 == 0 else (10 if a[:2] == b"\x1f\x8b" else 0)
    sa, sb = trace(a, st), trace(b, st)
    k = next((i for i, (x, y) in enumerate(zip(sa, sb)) if x != y), None)
    print(name, "symbols", len(sa), len(sb), "first difference at", k)
    if k is not None:
        blocks = [s for s in sa[:k] if s[0] == "blk"]
        print("  block starts before it (ref):", blocks[-3:])
        for i in range(max(0, k - 4), k + 4):
            print("  ", i, "ref", sa[i] if i < len(sa) else None, " ours", sb[i] if i < len(sb) else None)
