"""debug tool: decode a zlib/raw deflate stream into LZ77 tokens (pos, len, dist) and block
boundaries -- to find the first decision where two streams of the same input differ."""
import sys


class Bits:
    def __init__(self, b):
        self.b, self.p = b, 0

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.b[self.p >> 3] >> (self.p & 7)) & 1) << i
            self.p += 1
        return v


def huff(lengths):
    codes, code, bl = {}, 0, [0] * 16
    for l in lengths:
        if l:
            bl[l] += 1
    nxt, code = [0] * 16, 0
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    for s, l in enumerate(lengths):
        if l:
            codes[(l, nxt[l])] = s
            nxt[l] += 1
    return codes


def sym(bits, codes):
    code, l = 0, 0
    while True:
        code = (code << 1) | bits.get(1)
        l += 1
        if (l, code) in codes:
            return codes[(l, code)]


LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LE = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DB = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
      6145, 8193, 12289, 16385, 24577]
DE = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


def tokens(z, zlib_hdr=True):
    bits = Bits(z)
    if zlib_hdr:
        bits.p = 16
    pos, toks = 0, []
    while True:
        final, typ = bits.get(1), bits.get(2)
        toks.append(("block", pos, typ, final))
        if typ == 0:
            bits.p = (bits.p + 7) & ~7
            n = bits.get(16)
            bits.get(16)
            bits.p += 8 * n
            pos += n
        else:
            if typ == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 30
            else:
                hl, hd, hc = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
                order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
                cl = [0] * 19
                for i in range(hc):
                    cl[order[i]] = bits.get(3)
                cc = huff(cl)
                L = []
                while len(L) < hl + hd:
                    s = sym(bits, cc)
                    if s < 16:
                        L.append(s)
                    elif s == 16:
                        L += [L[-1]] * (3 + bits.get(2))
                    elif s == 17:
                        L += [0] * (3 + bits.get(3))
                    else:
                        L += [0] * (11 + bits.get(7))
                ll, dl = L[:hl], L[hl:]
            lc, dc = huff(ll), huff(dl)
            while True:
                s = sym(bits, lc)
                if s < 256:
                    toks.append(("lit", pos, s))
                    pos += 1
                elif s == 256:
                    break
                else:
                    s -= 257
                    ln = LB[s] + bits.get(LE[s])
                    d = sym(bits, dc)
                    dist = DB[d] + bits.get(DE[d])
                    toks.append(("match", pos, ln, dist))
                    pos += ln
        if final:
            break
    return toks


def first_diff(a, b):
    ta, tb = tokens(a), tokens(b)
    for i, (x, y) in enumerate(zip(ta, tb)):
        if x != y:
            return i, ta[max(0, i - 4):i + 4], tb[max(0, i - 4):i + 4]
    return None
