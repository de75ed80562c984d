/* CPU model (tools only): speculate -> verify -> replay for the lazy parse's
 * walks.  Prefix walks of h candidates for every position, then iterate: parse
 * with exact results where known and the prefix result elsewhere, walk the
 * call sites that used an unknown value, until the parse uses none. */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
int zo_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed, uint64_t first_index);
void zo_pp_links(const uint8_t *src, size_t n, uint16_t *link);
#define MAXD 32506
typedef struct { unsigned good, lazy, nice, chain; } cfg_t;
static const cfg_t CFG[10] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32},{4,4,16,16},{8,16,32,32},
                             {8,16,128,128},{8,32,128,256},{32,128,258,1024},{32,258,258,4096}};
static cfg_t c; static uint8_t *src; static uint16_t *link; static size_t n;
/* walk p with budget B: returns result, *steps */
static uint32_t walk(size_t p, unsigned B, unsigned *steps) {
    unsigned d0 = link[p]; *steps = 0;
    if (!d0 || d0 > MAXD) return 0;
    size_t limit = p > MAXD ? p - MAXD : 0, rem = n - p;
    unsigned nice = c.nice < rem ? c.nice : rem, maxcmp = 258 < rem ? 258 : rem;
    unsigned best = 2, count = 0; size_t bpos = 0, cur = p - d0;
    for (;;) {
        count++;
        const uint8_t *m = src + cur; int stop = 0;
        if (m[0] == src[p] && m[1] == src[p + 1]) {
            unsigned len = 0; while (len < maxcmp && m[len] == src[p + len]) len++;
            if (len > best) { best = len; bpos = cur; if (len >= nice) stop = 1; }
        }
        if (stop || count >= B) break;
        unsigned d = link[cur];
        if (!d || cur - d <= limit) break;
        cur -= d;
    }
    *steps = count;
    return best >= 3 ? best << 16 | (uint32_t)(p - bpos) : 0;
}
int main(int argc, char **argv) {
    int kind = atoi(argv[1]), level = atoi(argv[2]); unsigned h = atoi(argv[3]);
    n = argc > 4 ? strtoull(argv[4], 0, 0) : (1u << 20);
    c = CFG[level];
    src = malloc(n + 300); link = malloc(2 * n);
    uint32_t *rh = malloc(4 * n), *rf = malloc(4 * n), *rq = malloc(4 * n);
    uint8_t *kf = malloc(n), *kq = malloc(n), *hexact = malloc(n);
    unsigned *need = malloc(4 * n);
    zo_generate(src, n, 1, kind, 1, 0); memset(src + n, 0, 300);
    zo_pp_links(src, n, link);
    double pre = 0, ext = 0, full_all = 0; unsigned st;
    for (size_t p = 0; p < n; p++) {
        unsigned sf; walk(p, c.chain, &sf); full_all += sf;
        unsigned Bh = h < c.chain ? h : c.chain;
        rh[p] = walk(p, Bh, &st); pre += st;
        /* exact if the walk ended before the budget (chain end / limit / nice) */
        hexact[p] = st < Bh || Bh == c.chain;
        kf[p] = kq[p] = 0;
        if (hexact[p]) { kf[p] = kq[p] = 1; rf[p] = rq[p] = rh[p]; }
        if (st < Bh && Bh >= (c.chain >> 2)) { }
        if (Bh >= (c.chain >> 2)) { /* the quart result is a prefix of this walk */
            unsigned s2; rq[p] = walk(p, c.chain >> 2, &s2); kq[p] = 1; }
    }
    int it;
    for (it = 1; it < 100; it++) {
        size_t p = 0, nn = 0; unsigned ml = 2, pl; int avail = 0;
        while (p < n) {
            size_t look = n - p; pl = ml; ml = 2;
            unsigned d0 = (look >= 3) ? link[p] : 0;
            if (d0 && d0 <= MAXD && pl < c.lazy) {
                int q = pl >= c.good; uint32_t r;
                if (q ? kq[p] : kf[p]) r = q ? rq[p] : rf[p];
                else { r = rh[p]; need[nn++] = (uint32_t)p << 1 | q; }
                unsigned rl = r >> 16;
                if (rl > pl) ml = rl; else ml = pl <= look ? pl : look;
                if (ml == 3 && (r & 0xffff) > 4096 && rl > pl) ml = 2;
            }
            if (pl >= 3 && ml <= pl) { p += pl - 1; avail = 0; ml = 2; }
            else if (avail) p++; else { avail = 1; p++; }
        }
        if (!nn) break;
        double e0 = ext;
        for (size_t i = 0; i < nn; i++) {
            size_t q = need[i] >> 1; int isq = need[i] & 1;
            if (isq) { rq[q] = walk(q, c.chain >> 2, &st); kq[q] = 1; ext += st; }
            else { rf[q] = walk(q, c.chain, &st); kf[q] = 1; ext += st;
                   rq[q] = walk(q, c.chain >> 2, &st); kq[q] = 1; }
        }
        printf("  iter %d: %zu new sites, %.2f steps/pos\n", it, nn, (ext - e0) / n);
    }
    printf("kind %d L%d h=%u: iterations %d, prefix %.2f + ext %.2f = %.2f steps/pos (%.1f%% of all-full %.2f)\n",
           kind, level, h, it, pre / n, ext / n, (pre + ext) / n, 100 * (pre + ext) / full_all, full_all / n);
    return 0;
}
