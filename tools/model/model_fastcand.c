/* CPU model (tools only, not shipped): levels 1-3 from precomputed candidates.
 *
 * deflate_fast (deflate.c:1824-1915) searches the chain of INSERTED positions;
 * positions strictly inside a match longer than max_insert_length are not
 * inserted (:1873-1897).  The all-positions chain (every earlier position with
 * the same hash, zo_pp_links) contains the inserted chain as a subsequence, so
 * a search can be answered from the first K all-positions candidates of p
 * (computed position-parallel, with their match lengths) as long as the
 * `chain`-th inserted one, the limit or nice is reached within them.  This
 * model runs deflate_fast exactly (one-shot input, no flushes) and counts, per
 * search, how many all-positions candidates it needs; a search needing more
 * than K falls back to walking the chain.
 * Usage: model_fastcand kind level [n] [buffers] */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
int zo_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed, uint64_t first_index);
void zo_pp_links(const uint8_t *src, size_t n, uint16_t *link);
#define MAXD 32506
typedef struct { unsigned good, lazy, nice, chain; } cfg_t;
static const cfg_t CFG[4] = {{0,0,0,0},{4,4,8,4},{4,5,16,8},{4,6,32,32}};
int main(int argc, char **argv) {
    int kind = argc > 1 ? atoi(argv[1]) : 2, level = argc > 2 ? atoi(argv[2]) : 1;
    size_t n = argc > 3 ? strtoull(argv[3], 0, 0) : (1u << 20);
    int nb = argc > 4 ? atoi(argv[4]) : 2;
    cfg_t c = CFG[level];
    uint8_t *src = malloc(n + 300), *ins = malloc(n);
    uint16_t *link = malloc(2 * n);
    enum { KS = 8 };
    const unsigned Ks[KS] = {4, 8, 12, 16, 24, 32, 48, 64};
    double over[KS] = {0}, searches = 0, decisions = 0, need_sum = 0, ins_cnt = 0, cand_len3 = 0;
    unsigned long long hist[130] = {0};
    for (int b = 0; b < nb; b++) {
        zo_generate(src, n, 1, kind, 2025, b);
        memset(src + n, 0, 300);
        memset(ins, 0, n);
        zo_pp_links(src, n, link);
        size_t p = 0;
        while (p < n) {
            size_t look = n - p;
            decisions++;
            size_t head = 0;
            unsigned need = 0;          /* all-positions candidates scanned */
            if (look >= 3) {
                /* hash_head: the most recent inserted same-hash position */
                size_t q = p;
                for (;;) {
                    unsigned d = link[q];
                    if (!d) { q = 0; break; }
                    q -= d;
                    need++;
                    if (ins[q]) break;
                    if (p - q > 32767) { q = 0; break; }
                }
                head = q;
                ins[p] = 1;
            }
            unsigned ml = 0;
            if (head != 0 && p - head <= MAXD) {
                searches++;
                size_t limit = p > MAXD ? p - MAXD : 0;
                unsigned nice = c.nice < look ? c.nice : (unsigned)look, maxcmp = look < 258 ? (unsigned)look : 258;
                unsigned best = 2, count = 0;
                size_t cur = head;
                /* need counts all-positions candidates up to the last one longest_match visits */
                for (;;) {
                    count++;
                    unsigned len = 0;
                    while (len < maxcmp && src[cur + len] == src[p + len]) len++;
                    if (len > best) { best = len; if (len >= nice) break; }
                    if (count >= c.chain) break;
                    /* next inserted candidate */
                    size_t q = cur;
                    int end = 0;
                    for (;;) {
                        unsigned d = link[q];
                        if (!d) { end = 1; break; }
                        q -= d;
                        if (q <= limit) { end = 1; break; }
                        need++;
                        if (ins[q]) break;
                    }
                    if (end) break;
                    cur = q;
                }
                ml = best >= 3 ? (best < look ? best : (unsigned)look) : 0;
                need_sum += need;
                hist[need < 129 ? need : 129]++;
                for (int k = 0; k < KS; k++) over[k] += need > Ks[k];
            }
            if (ml >= 3) {
                size_t lk = look - ml;
                if (ml <= c.lazy && lk >= 3) {
                    for (size_t j = p + 1; j < p + ml; j++) ins[j] = 1;
                }
                p += ml;
            } else {
                p++;
            }
        }
        for (size_t j = 0; j < n; j++) ins_cnt += ins[j];
        (void)cand_len3;
    }
    printf("kind %d L%d: decisions/pos %.3f, searches/pos %.3f, inserted %.1f%%, candidates needed/search %.2f;",
           kind, level, decisions / (n * (double)nb), searches / (n * (double)nb), 100.0 * ins_cnt / (n * (double)nb),
           need_sum / searches);
    for (int k = 0; k < KS; k++) printf(" >%u: %.2f%%", Ks[k], 100.0 * over[k] / searches);
    printf("\n");
    return 0;
}
