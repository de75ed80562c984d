/* CPU model (tools only, not shipped): quarter-chain walks at every position plus full-chain extensions on a conservative fixpoint set F (positions whose predecessor quarter result is below good_match, and the ends of candidate matches). Usage: model_walkfix kind level n buffers */
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
    int kind = atoi(argv[1]), level = atoi(argv[2]);
    size_t n = strtoull(argv[3], 0, 0); int nb = atoi(argv[4]);
    cfg_t c = CFG[level];
    uint8_t *src = malloc(n + 300); uint16_t *link = malloc(2 * n);
    uint32_t *lf = malloc(4*n), *lq = malloc(4*n), *sf = malloc(4*n), *sq = malloc(4*n);
    uint8_t *F = malloc(n), *ext = malloc(n);
    double A_full=0, A_q=0, EXTS=0, nF=0, nExt=0, iters=0;
    for (int b = 0; b < nb; b++) {
        zo_generate(src, n, 1, kind, 1, b); memset(src + n, 0, 300); zo_pp_links(src, n, link);
        unsigned bq = c.chain >> 2;
        for (size_t p = 0; p < n; p++) {
            lf[p] = lq[p] = 0; sf[p] = sq[p] = 0; ext[p] = 0;
            unsigned d0 = link[p]; if (!d0 || d0 > MAXD) continue;
            size_t limit = p > MAXD ? p - MAXD : 0, rem = n - p;
            unsigned nice = c.nice < rem ? c.nice : rem, maxcmp = 258 < rem ? 258 : rem;
            unsigned best = 2, bestq = 0, count = 0; int snapped = 0; size_t cur = p - d0;
            for (;;) {
                count++; const uint8_t *m = src + cur; int stop = 0;
                if (m[0] == src[p] && m[1] == src[p+1]) { unsigned len = 0; while (len < maxcmp && m[len] == src[p+len]) len++;
                    if (len > best) { best = len; if (len >= nice) stop = 1; } }
                if (count == bq && !stop) { bestq = best; snapped = 1; sq[p] = count; }
                if (stop || count >= c.chain) break;
                unsigned d = link[cur]; if (!d || cur - d <= limit) break; cur -= d;
            }
            if (!snapped) { bestq = best; sq[p] = count; } else ext[p] = 1;
            sf[p] = count; lf[p] = best >= 3 ? best : 0; lq[p] = bestq >= 3 ? bestq : 0;
            A_full += count; A_q += sq[p];
        }
        /* fixpoint F */
        memset(F, 0, n);
        for (size_t p = 1; p < n; p++) if (lq[p-1] < c.good) F[p] = 1;
        F[0] = 1;
        for (size_t s = 0; s < n; s++) if (lq[s] && s + lq[s] < n) F[s + lq[s]] = 1;
        int changed = 1; int it = 0;
        while (changed && it < 10) { changed = 0; it++;
            for (size_t s = 0; s < n; s++) if (F[s] && ext[s] && lf[s] && s + lf[s] < n && !F[s + lf[s]]) { F[s + lf[s]] = 1; changed = 1; } }
        iters += it;
        for (size_t p = 0; p < n; p++) if (F[p] && ext[p]) { EXTS += sf[p] - sq[p]; nExt++; }
        for (size_t p = 0; p < n; p++) nF += F[p];
    }
    double N = (double)n * nb;
    printf("kind %d L%d: all-full %.2f/pos, quarter-all %.2f/pos, ext on F %.2f/pos -> total %.2f/pos = %.1f%% of all-full; |F| %.1f%% of pos, extended %.1f%%, fixpoint iters %.1f\n",
           kind, level, A_full/N, A_q/N, EXTS/N, (A_q+EXTS)/N, 100*(A_q+EXTS)/A_full, 100*nF/N, 100*nExt/N, iters/nb);
    return 0;
}
