/* CPU model (tools only, not shipped): deflate_fast (deflate.c:1824-1915) run
 * from a segment start with a warm-up.  Ground truth is the sequential greedy
 * parse, whose hash chains hold the inserted positions only (a match longer
 * than max_insert_length skips its interior).  A lane owning [s, s+S) starts
 * parsing at s-W as if every position before s-W were inserted; the model
 * reports, per lane, the first position t from which the lane's decision
 * points and insertion flags equal the truth up to s+S (the lane is exact on
 * [s, s+S) when t <= s), and whether the lane's exit matches.
 *   cc -O2 tools/model/model_fseg.c -Loracle -loracle -o /tmp/model_fseg
 *   LD_LIBRARY_PATH=oracle /tmp/model_fseg <kind> <level> <S> <W> [n] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int zo_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed, uint64_t first_index);
void zo_pp_links(const uint8_t *src, size_t n, uint16_t *link);
#define MAXD 32506
typedef struct { unsigned good, lazy, nice, chain; } cfg_t;
static const cfg_t CFG[4] = {{0, 0, 0, 0}, {4, 4, 8, 4}, {4, 5, 16, 8}, {4, 6, 32, 32}};
static cfg_t c;
static uint8_t *src;
static uint16_t *link;
static size_t n;
static unsigned long steps;

/* ins: flags; q < lo reads as inserted (the warm-up's assumption) */
static size_t prev_ins(const uint8_t *ins, size_t lo, size_t q) {
    for (;;) {
        unsigned d = link[q];
        if (!d) return 0;
        q -= d;
        steps++;
        if (q < lo || ins[q]) return q;
    }
}
static unsigned match_at(const uint8_t *ins, size_t lo, size_t p) {
    size_t cur = prev_ins(ins, lo, p);
    if (!cur || p - cur > MAXD) return 0;
    size_t limit = p > MAXD ? p - MAXD : 0, rem = n - p;
    unsigned nice = c.nice < rem ? c.nice : (unsigned)rem, maxcmp = 258 < rem ? 258 : (unsigned)rem;
    unsigned best = 2, chain = c.chain;
    for (;;) {
        unsigned len = 0;
        while (len < maxcmp && src[cur + len] == src[p + len]) len++;
        if (len > best) { best = len; if (len >= nice) break; }
        size_t nx = prev_ins(ins, lo, cur);
        if (!nx || nx <= limit || --chain == 0) break;
        cur = nx;
    }
    return best >= 3 ? best : 0;
}
/* parse [x0, x1): flags into ins[x0..x1), decision points into dp[] (1 = decision) */
static size_t parse(size_t x0, size_t x1, size_t lo, uint8_t *ins, uint8_t *dp) {
    size_t p = x0;
    for (size_t q = x0; q < x1 + 300 && q < n; q++) ins[q] = 0, dp[q] = 0;
    while (p < x1) {
        dp[p] = 1;
        if (n - p >= 3) ins[p] = 1;
        unsigned m = match_at(ins, lo, p);
        if (m) {
            if (m <= c.lazy && n - p - m >= 3)
                for (size_t q = p + 1; q < p + m; q++) ins[q] = 1;
            p += m;
        } else p++;
    }
    return p;
}

int main(int argc, char **argv) {
    int kind = atoi(argv[1]), level = atoi(argv[2]);
    size_t S = strtoull(argv[3], 0, 0), W = strtoull(argv[4], 0, 0);
    n = argc > 5 ? strtoull(argv[5], 0, 0) : (4u << 20);
    c = CFG[level];
    src = malloc(n + 300);
    link = malloc(2 * n);
    zo_generate(src, n, 1, kind, 1, 0);
    memset(src + n, 0, 300);
    zo_pp_links(src, n, link);
    uint8_t *ti = calloc(n + 300, 1), *td = calloc(n + 300, 1), *li = calloc(n + 300, 1), *ld = calloc(n + 300, 1);
    steps = 0;
    parse(0, n, 0, ti, td);
    unsigned long steps_seq = steps;
    size_t L = (n + S - 1) / S, exact = 0, worst = 0;
    unsigned long steps_lanes = 0;
    double sum_t = 0;
    for (size_t i = 1; i < L; i++) {
        size_t s = i * S, x1 = s + S < n ? s + S : n, x0 = s > W ? s - W : 0;
        steps = 0;
        size_t ex = parse(x0, x1, x0, li, ld);
        steps_lanes += steps;
        /* first t from which flags and decision points equal the truth up to x1 */
        size_t t = x1;
        while (t > x0 && li[t - 1] == ti[t - 1] && ld[t - 1] == td[t - 1]) t--;
        size_t tex = x1; while (tex < n && !td[tex]) tex++;
        int ok = t <= s && ex == (tex < n ? tex : n);
        exact += ok;
        size_t dist = t - x0;
        if (dist > worst) worst = dist;
        sum_t += dist;
    }
    printf("kind %d L%d S %zu W %zu n %zu: lanes %zu exact %zu (%.1f%%), sync after %.0f avg / %zu max bytes of the "
           "lane's start, chain steps per lane byte %.2f vs seq %.2f\n",
           kind, level, S, W, n, L - 1, exact, 100.0 * exact / (L - 1), sum_t / (L - 1), worst,
           (double)steps_lanes / ((L - 1) * (double)(S + W)), (double)steps_seq / n);
    return 0;
}
