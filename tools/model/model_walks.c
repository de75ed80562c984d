/* CPU model (tools only, not shipped): how many chain steps the lazy parse
 * really needs vs walking every position.  Links/walks/parse follow
 * oracle/zoracle.c (zo_pp_links, zo_pp_match, run_slow) on one buffer. */
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
int main(int argc, char **argv) {
    int kind = argc > 1 ? atoi(argv[1]) : 1, level = argc > 2 ? atoi(argv[2]) : 6;
    size_t n = argc > 3 ? strtoull(argv[3], 0, 0) : (1u << 20);
    int nb = argc > 4 ? atoi(argv[4]) : 4;
    cfg_t c = CFG[level];
    uint8_t *src = malloc(n + 300); uint16_t *link = malloc(2 * n);
    uint32_t *rf = malloc(4 * n), *rq = malloc(4 * n), *sf = malloc(4 * n), *sq = malloc(4 * n);
    double A_full = 0, A_quart = 0, CS = 0, CSpos = 0, EXT = 0, FS = 0, QS = 0, nonzero = 0;
    double DEC = 0;
    for (int b = 0; b < nb; b++) {
        zo_generate(src, n, 1, kind, 1, b);
        memset(src + n, 0, 300);
        zo_pp_links(src, n, link);
        unsigned bq = c.chain >> 2;
        for (size_t p = 0; p < n; p++) {
            rf[p] = rq[p] = 0; sf[p] = sq[p] = 0;
            unsigned d0 = link[p];
            if (!d0 || d0 > MAXD) continue;
            size_t limit = p > MAXD ? p - MAXD : 0, rem = n - p;
            unsigned nice = c.nice < rem ? c.nice : rem, maxcmp = 258 < rem ? 258 : rem;
            unsigned best = 2, bestq = 0, count = 0; int snapped = 0; size_t bpos = 0, bposq = 0, cur = p - d0;
            for (;;) {
                count++;
                const uint8_t *m = src + cur; int stop = 0;
                if (m[0] == src[p] && m[1] == src[p + 1]) {
                    unsigned len = 0; while (len < maxcmp && m[len] == src[p + len]) len++;
                    if (len > best) { best = len; bpos = cur; if (len >= nice) stop = 1; }
                }
                if (count == bq) { bestq = best; bposq = bpos; snapped = 1; sq[p] = count; }
                if (stop || count >= c.chain) break;
                unsigned d = link[cur];
                if (!d || cur - d <= limit) break;
                cur -= d;
            }
            if (!snapped) { bestq = best; bposq = bpos; sq[p] = count; }
            sf[p] = count;
            if (best >= 3) rf[p] = best << 16 | (uint32_t)(p - bpos);
            if (bestq >= 3) rq[p] = bestq << 16 | (uint32_t)(p - bposq);
            A_full += count; A_quart += sq[p]; nonzero++;
        }
        /* lazy parse (no window slides, no flushes) */
        size_t p = 0; unsigned ml = 2, pl; int avail = 0;
        while (p < n) {
            size_t look = n - p;
            pl = ml; ml = 2; DEC++;
            unsigned d0 = (look >= 3) ? link[p] : 0;
            if (d0 && d0 <= MAXD && pl < c.lazy) {
                int q = pl >= c.good;
                uint32_t r = q ? rq[p] : rf[p];
                CS += q ? sq[p] : sf[p]; CSpos++;
                if (q) QS++; else { FS++; EXT += sf[p] - sq[p]; }
                unsigned rl = r >> 16;
                if (rl > pl) ml = rl; else ml = pl <= look ? pl : look;
                if (ml == 3 && (r & 0xffff) > 4096 && rl > pl) ml = 2;
            }
            if (pl >= 3 && ml <= pl) { p += pl - 1; avail = 0; ml = 2; }
            else if (avail) p++;
            else { avail = 1; p++; }
        }
    }
    double N = (double)n * nb;
    printf("kind %d L%d: walks at %.1f%% of positions; steps/pos: all-full %.2f all-quart %.2f | call sites %.1f%% of pos "
           "(full %.1f%% quart %.1f%%) steps at call sites %.2f/pos; decisions %.1f%%\n",
           kind, level, 100 * nonzero / N, A_full / N, A_quart / N, 100 * CSpos / N, 100 * FS / N, 100 * QS / N, CS / N, 100*DEC/N);
    printf("  scheme quart-all + full-ext at full sites: %.2f/pos (%.1f%% of all-full)\n", (A_quart + EXT) / N,
           100 * (A_quart + EXT) / A_full);
    return 0;
}
