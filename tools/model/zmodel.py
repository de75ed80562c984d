"""debug model (tools only): deflate_slow / deflate_fast of zlib 1.3.1 as a token
stream over one input with a function switch at a flush point, with switchable
quirks, to compare against the compiled reference's token streams."""
MIN_MATCH, MAX_MATCH, MIN_LOOKAHEAD = 3, 258, 262
CFG = {0: (0, 0, 0, 0), 1: (4, 4, 8, 4), 2: (4, 5, 16, 8), 3: (4, 6, 32, 32), 4: (4, 4, 16, 16), 5: (8, 16, 32, 32),
       6: (8, 16, 128, 128), 7: (8, 32, 128, 256), 8: (32, 128, 258, 1024), 9: (32, 258, 258, 4096)}
MAXD = 32768 - MIN_LOOKAHEAD


class Z:
    def __init__(self, data, level):
        self.w = data
        self.head, self.prev = {}, {}
        self.prev_length = self.match_length = MIN_MATCH - 1
        self.match_start = self.prev_match = 0
        self.match_available = 0
        self.strstart = 0
        self.insert = 0
        self.ins_h = 0
        self.toks = []
        self.set_level(level)

    def set_level(self, level):
        self.level = level
        self.good, self.lazy, self.nice, self.chain = CFG[level]

    def h(self, p):
        w = self.w
        return ((w[p] << 10) ^ (w[p + 1] << 5) ^ w[p + 2]) & 0x7fff

    def upd(self, c):
        self.ins_h = ((self.ins_h << 5) ^ c) & 0x7fff

    def ins(self, p):
        # INSERT_STRING: the rolling hash (deflate.c:141,160-163)
        self.upd(self.w[p + 2])
        h = self.ins_h
        hh = self.head.get(h, 0)
        self.prev[p] = hh
        self.head[h] = p
        return hh

    def longest(self, cur, E):
        chain = self.chain
        best = self.prev_length
        if self.prev_length >= self.good:
            chain >>= 2
        look = E - self.strstart
        nice = min(self.nice, look)
        limit = self.strstart - MAXD if self.strstart > MAXD else 0
        s = self.strstart
        while True:
            ok = self.w[cur + best] == self.w[s + best] and self.w[cur + best - 1] == self.w[s + best - 1] \
                and self.w[cur] == self.w[s] and self.w[cur + 1] == self.w[s + 1]
            if ok:
                l = 0
                while l < MAX_MATCH and s + l < len(self.w) and self.w[cur + l] == self.w[s + l]:
                    l += 1
                if l > best:
                    self.match_start = cur
                    best = l
                    if l >= nice:
                        break
            cur = self.prev.get(cur, 0)
            chain -= 1
            if not (cur > limit and chain != 0):
                break
        return best if best <= look else look

    def late_insert(self, E):
        if E - self.strstart + self.insert >= MIN_MATCH:
            s = self.strstart - self.insert
            self.ins_h = self.w[s]
            self.upd(self.w[s + 1])
            while self.insert:
                self.ins(s)
                s += 1
                self.insert -= 1
                if E - self.strstart + self.insert < MIN_MATCH:
                    break

    def fast(self, E, flush):
        self.late_insert(E)
        while True:
            look = E - self.strstart
            if look < MIN_LOOKAHEAD and not flush:
                return
            if look == 0:
                break
            hh = 0
            if look >= MIN_MATCH:
                hh = self.ins(self.strstart)
            if hh and self.strstart - hh <= MAXD:
                self.match_length = self.longest(hh, E)
            if self.match_length >= MIN_MATCH:
                self.toks.append(("match", self.strstart, self.match_length, self.strstart - self.match_start))
                look -= self.match_length
                if self.match_length <= self.lazy and look >= MIN_MATCH:
                    for k in range(1, self.match_length):
                        self.ins(self.strstart + k)
                    self.strstart += self.match_length
                else:
                    self.strstart += self.match_length
                    self.ins_h = self.w[self.strstart]
                    self.upd(self.w[self.strstart + 1])
                self.match_length = 0
            else:
                self.toks.append(("lit", self.strstart, self.w[self.strstart]))
                self.strstart += 1
        self.insert = min(self.strstart, MIN_MATCH - 1)

    def slow(self, E, flush):
        self.late_insert(E)
        while True:
            look = E - self.strstart
            if look < MIN_LOOKAHEAD and not flush:
                return
            if look == 0:
                break
            hh = 0
            if look >= MIN_MATCH:
                hh = self.ins(self.strstart)
            self.prev_length, self.prev_match = self.match_length, self.match_start
            self.match_length = MIN_MATCH - 1
            if hh and self.prev_length < self.lazy and self.strstart - hh <= MAXD:
                self.match_length = self.longest(hh, E)
                if self.match_length <= 5 and self.match_length == MIN_MATCH and \
                        self.strstart - self.match_start > 4096:
                    self.match_length = MIN_MATCH - 1
            if self.prev_length >= MIN_MATCH and self.match_length <= self.prev_length:
                mx = self.strstart + look - MIN_MATCH
                self.toks.append(("match", self.strstart - 1, self.prev_length, self.strstart - 1 - self.prev_match))
                for k in range(1, self.prev_length - 1):
                    if self.strstart + k <= mx:
                        self.ins(self.strstart + k)
                self.strstart += self.prev_length - 1
                self.prev_length = 0                      # the do-while consumes it (deflate.c:2010-2015)
                self.match_available = 0
                self.match_length = MIN_MATCH - 1
            elif self.match_available:
                self.toks.append(("lit", self.strstart - 1, self.w[self.strstart - 1]))
                self.strstart += 1
            else:
                self.match_available = 1
                self.strstart += 1
        if self.match_available:
            self.toks.append(("lit", self.strstart - 1, self.w[self.strstart - 1]))
            self.match_available = 0
        self.insert = min(self.strstart, MIN_MATCH - 1)

    def run(self, E, flush):
        (self.slow if self.level >= 4 else self.fast)(E, flush)
