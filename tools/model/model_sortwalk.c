/* CPU model (tools only, not shipped): SIMT utilisation of k_match's walks
 * under different walk orders.  A wave runs 64 walks side by side and a round
 * lasts as long as its longest walk, so utilisation = sum(steps) / sum over
 * waves(64 * max steps).  Steps per position follow longest_match exactly
 * (oracle/zoracle.c zo_pp_links chains, quick reject irrelevant to the count,
 * stop at nice / chain / limit).  Orders:
 *   pos    positions in index order, 64 per wave
 *   cnt4k  each 4 KiB tile counting-sorted by exact step count (the k_match of
 *          rounds 1-4 sorts by an approximate count key)
 *   hash16 each 16 Ki block sorted by (hash, position): the order in which the
 *          sorted-run k_match walks (a run's candidates are contiguous)
 *   hcnt   hash16, then each 4 Ki slice of it counting-sorted by step count
 * Usage: model_sortwalk kind level [n] [buffers] */
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
static uint32_t *g_key;
static int cmp_key(const void *a, const void *b) {
    uint32_t x = g_key[*(const uint32_t *)a], y = g_key[*(const uint32_t *)b];
    if (x != y) return x < y ? -1 : 1;
    return *(const uint32_t *)a < *(const uint32_t *)b ? -1 : 1;
}
static double util(const uint32_t *steps, const uint32_t *order, size_t m, double *sum_out) {
    double s = 0, w = 0;
    for (size_t i = 0; i < m; i += 64) {
        uint32_t mx = 0;
        for (size_t j = i; j < i + 64 && j < m; j++) { s += steps[order[j]]; if (steps[order[j]] > mx) mx = steps[order[j]]; }
        w += 64.0 * mx;
    }
    *sum_out += s;
    return w;
}
int main(int argc, char **argv) {
    int kind = argc > 1 ? atoi(argv[1]) : 1, level = argc > 2 ? atoi(argv[2]) : 6;
    size_t n = argc > 3 ? strtoull(argv[3], 0, 0) : (1u << 20);
    int nb = argc > 4 ? atoi(argv[4]) : 2;
    cfg_t c = CFG[level];
    uint8_t *src = malloc(n + 300);
    uint16_t *link = malloc(2 * n);
    uint32_t *steps = malloc(4 * n), *order = malloc(4 * n), *key = malloc(4 * n);
    double S[4] = {0}, W[4] = {0};
    for (int b = 0; b < nb; b++) {
        zo_generate(src, n, 1, kind, 2025, b);
        memset(src + n, 0, 300);
        zo_pp_links(src, n, link);
        for (size_t p = 0; p < n; p++) {
            steps[p] = 0;
            unsigned d0 = link[p];
            if (!d0 || d0 > MAXD) continue;
            size_t limit = p > MAXD ? p - MAXD : 0, rem = n - p;
            unsigned nice = c.nice < rem ? c.nice : rem, maxcmp = 258 < rem ? 258 : rem;
            unsigned best = 2, count = 0;
            size_t cur = p - d0;
            for (;;) {
                count++;
                const uint8_t *m = src + cur;
                int stop = 0;
                if (m[0] == src[p] && m[1] == src[p + 1]) {
                    unsigned len = 0;
                    while (len < maxcmp && m[len] == src[p + len]) len++;
                    if (len > best) { best = len; if (len >= nice) stop = 1; }
                }
                if (stop || count >= c.chain) break;
                unsigned d = link[cur];
                if (!d || cur - d <= limit) break;
                cur -= d;
            }
            steps[p] = count;
        }
        /* pos */
        for (size_t p = 0; p < n; p++) order[p] = (uint32_t)p;
        W[0] += util(steps, order, n, &S[0]);
        /* cnt4k */
        g_key = key;
        for (size_t p = 0; p < n; p++) key[p] = 0xffffffffu - steps[p];
        for (size_t t = 0; t < n; t += 4096) qsort(order + t, (n - t) < 4096 ? n - t : 4096, 4, cmp_key);
        W[1] += util(steps, order, n, &S[1]);
        /* hash16 */
        for (size_t p = 0; p < n; p++) {
            order[p] = (uint32_t)p;
            key[p] = p + 2 < n ? ((src[p] & 31u) << 10) ^ (src[p + 1] << 5) ^ src[p + 2] : 0x8000u;
        }
        for (size_t t = 0; t < n; t += 16384) qsort(order + t, (n - t) < 16384 ? n - t : 16384, 4, cmp_key);
        W[2] += util(steps, order, n, &S[2]);
        /* hcnt: hash16 then each 4 Ki slice by step count */
        for (size_t p = 0; p < n; p++) key[p] = 0xffffffffu - steps[p];
        for (size_t t = 0; t < n; t += 4096) qsort(order + t, (n - t) < 4096 ? n - t : 4096, 4, cmp_key);
        W[3] += util(steps, order, n, &S[3]);
    }
    const char *names[4] = {"pos", "cnt4k", "hash16", "hcnt"};
    printf("kind %d level %d: steps/position %.1f;", kind, level, S[0] / ((double)n * nb));
    for (int k = 0; k < 4; k++) printf(" %s %.1f%%", names[k], 100.0 * S[k] / W[k]);
    printf("\n");
    return 0;
}
