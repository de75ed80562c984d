/* CPU model (tools only, not shipped): k_parse_srt's decisions against
 * deflate_fast's.  Two parses of the same one-shot buffer at level 1..3:
 *   chain: deflate_fast as deflate.c:1824-1915 runs it (head[] / prev[] of
 *          inserted positions, longest_match over the inserted chain);
 *   srt:   k_parse_srt's formulation (zgpu_deflate.hip): candidates from the
 *          sorted runs of the 16 Ki blocks b, b-1, b-2 taken 64 at a time,
 *          an inserted-position bitmap, the head / limit / chain / nice rules
 *          applied to the lanes, lengths capped at nice and the winner
 *          extended to maxcmp.
 * Every decision (position, match length, distance) must agree.
 * Window slides are ignored (S = 0): one-shot buffers up to 64 KiB + 262
 * never slide, larger ones are checked by the GPU tests.
 * Usage: model_parse_srt kind level [n] [buffers] */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
int zo_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed, uint64_t first_index);
#define MAXD 32506
#define BS 16384
typedef struct { unsigned good, lazy, nice, chain; } cfg_t;
static const cfg_t CFG[4] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32}};
static uint32_t hash3(const uint8_t *b) { return ((b[0] & 31u) << 10) ^ ((uint32_t)b[1] << 5) ^ b[2]; }
static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}
static unsigned lcp(const uint8_t *a, const uint8_t *b, unsigned cap) {
    unsigned k = 0;
    while (k < cap && a[k] == b[k]) k++;
    return k;
}
int main(int argc, char **argv) {
    int kind = argc > 1 ? atoi(argv[1]) : 2, level = argc > 2 ? atoi(argv[2]) : 1;
    size_t n = argc > 3 ? strtoull(argv[3], 0, 0) : 60000;
    int nb = argc > 4 ? atoi(argv[4]) : 4;
    cfg_t c = CFG[level];
    uint8_t *src = calloc(n + 512, 1), *ins = calloc(n + 512, 1);
    uint32_t *head = malloc(4 * 32768), *prev = calloc(n + 512, 4);
    size_t nblk = (n + BS - 1) / BS;
    uint16_t *S = malloc(2 * nblk * BS), *off = malloc(2 * nblk * 32769);
    uint32_t *keys = malloc(4 * BS);
    uint32_t *dA = malloc(8 * (n + 1)), *dB = malloc(8 * (n + 1));
    uint64_t bad = 0, decs = 0;
    for (int bb = 0; bb < nb; bb++) {
        zo_generate(src, n, 1, kind, 2025, bb);
        memset(src + n, 0, 512);
        /* ---- chain parse (deflate_fast) */
        size_t na = 0;
        memset(head, 0, 4 * 32768);
        for (size_t p = 0; p < n;) {
            size_t look = n - p, hh = 0;
            if (look >= 3) { uint32_t h = hash3(src + p); hh = head[h]; prev[p] = hh; head[h] = (uint32_t)p; }
            unsigned ml = 0, best = 2;
            size_t ms = 0;
            if (hh > 0 && p - hh <= MAXD) {
                size_t limit = p > MAXD ? p - MAXD : 0, cur = hh;
                unsigned nice = c.nice < look ? c.nice : (unsigned)look, maxcmp = look < 258 ? (unsigned)look : 258;
                unsigned chain = c.chain;
                for (;;) {
                    unsigned len = lcp(src + cur, src + p, maxcmp);
                    if (len > best) { best = len; ms = cur; if (len >= nice) break; }
                    cur = prev[cur];
                    if (cur <= limit || --chain == 0) break;
                }
                ml = best < look ? best : (unsigned)look;
            }
            if (ml >= 3) {
                dA[na++] = (uint32_t)p; dA[na++] = ml << 16 | (uint32_t)(p - ms);
                size_t la = look - ml;
                if (ml <= c.lazy && la >= 3)
                    for (size_t j = p + 1; j < p + ml; j++) { uint32_t h = hash3(src + j); prev[j] = head[h]; head[h] = (uint32_t)j; }
                p += ml;
            } else {
                p++;
            }
        }
        /* ---- sorted runs (k_bsort) */
        for (size_t b = 0; b < nblk; b++) {
            int64_t p0 = (int64_t)b * BS, mm = (int64_t)n - 2 - p0;
            int m = mm <= 0 ? 0 : (mm < BS ? (int)mm : BS);
            for (int e = 0; e < m; e++) keys[e] = hash3(src + p0 + e) << 14 | (uint32_t)e;
            qsort(keys, m, 4, cmp_u32);
            for (int i = 0; i < m; i++) S[b * BS + i] = keys[i] & (BS - 1);
            int i = 0;
            for (uint32_t h = 0; h <= 32768; h++) {
                while (i < m && (keys[i] >> 14) < h) i++;
                off[b * 32769 + h] = (uint16_t)i;
            }
        }
        /* ---- k_parse_srt */
        size_t nbd = 0;
        memset(ins, 0, n + 512);
        for (size_t p = 0; p < n;) {
            size_t look = n - p;
            unsigned best = 2;
            size_t bq = 0;
            if (look >= 3) {
                size_t b = p / BS;
                int64_t p0 = (int64_t)b * BS;
                uint32_t rel = (uint32_t)(p - p0), h = hash3(src + p);
                /* rank of p in its block's run */
                const uint16_t *o0 = off + b * 32769;
                int i = -1;
                for (int j = o0[h]; j < o0[h + 1]; j++) if (S[b * BS + j] == rel) { i = j; break; }
                uint32_t n0 = (uint32_t)i - o0[h];
                uint32_t s1 = b >= 1 ? off[(b - 1) * 32769 + h] : 0, e1 = b >= 1 ? off[(b - 1) * 32769 + h + 1] : 0;
                uint32_t s2 = b >= 2 ? off[(b - 2) * 32769 + h] : 0, e2 = b >= 2 ? off[(b - 2) * 32769 + h + 1] : 0;
                uint32_t n01 = n0 + (e1 - s1), n012 = n01 + (e2 - s2);
                size_t limit = p > MAXD ? p - MAXD : 0;
                unsigned nice = c.nice < look ? c.nice : (unsigned)look, maxcmp = look < 258 ? (unsigned)look : 258;
                unsigned chain = c.chain;
                int head_found = 0, done = n012 == 0;
                for (uint32_t k0 = 0; !done; k0 += 64) {
                    int64_t q[64];
                    int insk[64];
                    for (int l = 0; l < 64; l++) {
                        uint32_t k = k0 + l;
                        q[l] = -1;
                        insk[l] = 0;
                        if (k >= n012) continue;
                        if (k < n0) q[l] = p0 + S[b * BS + i - 1 - k];
                        else if (k < n01) q[l] = p0 - BS + S[(b - 1) * BS + e1 - 1 - (k - n0)];
                        else q[l] = p0 - 2 * BS + S[(b - 2) * BS + e2 - 1 - (k - n01)];
                        insk[l] = ins[q[l]];
                    }
                    int hl = -1;
                    if (!head_found) {
                        for (int l = 0; l < 64; l++) if (insk[l]) { hl = l; break; }
                        if (hl < 0) { if (k0 + 64 >= n012) break; continue; }
                        if (!(q[hl] > 0 && p - q[hl] <= MAXD)) break;
                        head_found = 1;
                    }
                    int stop = 0;
                    unsigned vis = 0, nmh = 0;
                    int wl = -1; unsigned wlen = 0;
                    for (int l = 0; l < 64; l++) {
                        if (!insk[l]) continue;
                        if (l != hl && q[l] <= (int64_t)limit) { stop = 1; continue; }
                        if (vis >= chain) continue;
                        vis++;
                        unsigned len = lcp(src + q[l], src + p, 32);
                        if (len > nice) len = nice;
                        if (len >= nice && !nmh) { nmh = 1; wl = l; wlen = nice; }
                        if (!nmh && len > wlen) { wlen = len; wl = l; }
                    }
                    if (wl >= 0 && wlen > best) { best = wlen; bq = (size_t)q[wl]; }
                    chain -= vis;
                    done = nmh || chain == 0 || stop || k0 + 64 >= n012;
                }
                if (best >= nice && best >= 3) best = lcp(src + bq, src + p, maxcmp);
                ins[p] = 1;
            }
            unsigned ml = best < look ? best : (unsigned)look;
            if (ml >= 3) {
                dB[nbd++] = (uint32_t)p; dB[nbd++] = ml << 16 | (uint32_t)(p - bq);
                if (ml <= c.lazy && look - ml >= 3) for (size_t j = p + 1; j < p + ml; j++) ins[j] = 1;
                p += ml;
            } else {
                p++;
            }
        }
        decs += na / 2;
        if (na != nbd || memcmp(dA, dB, 4 * na)) {
            size_t j = 0;
            while (j < na && j < nbd && dA[j] == dB[j]) j++;
            if (bad < 3) printf("buffer %d: first difference at match %zu: chain p %u v %08x, srt p %u v %08x\n", bb, j / 2,
                                dA[j & ~1ul], dA[j | 1], dB[j & ~1ul], dB[j | 1]);
            bad++;
        }
    }
    printf("kind %d L%d n %zu: %llu matches, %llu buffers differ\n", kind, level, n, (unsigned long long)decs,
           (unsigned long long)bad);
    return bad != 0;
}
