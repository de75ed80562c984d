/* CPU model (tools only, not shipped): a segment-parallel, speculative
 * deflate_fast (deflate.c:1824-1915).  Ground truth is the sequential greedy
 * parse, whose hash chains hold the inserted positions only (a match longer
 * than max_insert_length skips its interior).  In round r every lane
 * re-parses its segment from the entry its left neighbour reported in round
 * r-1 (the first decision point at or after the segment start), reading the
 * insertion flags of earlier segments as round r-1 left them.  The rounds
 * stop when no lane's entry, last match or flags change; the parse is then
 * the sequential one.  Reports rounds, decisions re-parsed, and checks the
 * result against the sequential parse.
 *   cc -O2 tools/model/model_fast.c -Loracle -loracle -o /tmp/model_fast
 *   LD_LIBRARY_PATH=oracle /tmp/model_fast <kind> <level> <seg> [n] */
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

/* flags: the lane's own segment from `own` (this round), earlier from `old` */
typedef struct { const uint8_t *own, *old; size_t x0; } view_t;
static inline int ins_at(const view_t *v, size_t q) { return q >= v->x0 ? v->own[q] : v->old[q]; }
static unsigned long steps;

static size_t prev_ins(const view_t *v, size_t q) {      /* previous inserted same-hash position, 0 none */
    for (;;) {
        unsigned d = link[q];
        if (!d) return 0;
        q -= d;
        steps++;
        if (ins_at(v, q)) return q;
    }
}
static unsigned match_at(const view_t *v, size_t p, size_t *ms) {
    size_t cur = prev_ins(v, p);
    if (!cur || p - cur > MAXD) return 0;
    size_t limit = p > MAXD ? p - MAXD : 0, rem = n - p;
    unsigned nice = c.nice < rem ? c.nice : (unsigned)rem, maxcmp = 258 < rem ? 258 : (unsigned)rem;
    unsigned best = 2, chain = c.chain;
    for (;;) {
        unsigned len = 0;
        while (len < maxcmp && src[cur + len] == src[p + len]) len++;
        if (len > best) { best = len; *ms = cur; if (len >= nice) break; }
        size_t nx = prev_ins(v, cur);
        if (!nx || nx <= limit || --chain == 0) break;
        cur = nx;
    }
    return best >= 3 ? best : 0;
}

typedef struct { size_t exit, ls, lm; } lane_out;   /* exit: first decision point >= segment end; last match */

/* parse [entry, x1) of a lane owning [x0, x1); flags of [x0, x1) into own[] */
static lane_out parse_lane(size_t x0, size_t x1, size_t entry, size_t pls, size_t plm, uint8_t *own,
                           const uint8_t *old, unsigned long *dec) {
    view_t v = {own, old, x0};
    for (size_t q = x0; q < x1; q++) own[q] = 0;
    /* [x0, entry): interior of the left neighbour's last match (ls, lm) */
    if (plm && plm <= c.lazy && n - pls - plm >= 3)
        for (size_t q = x0; q < entry && q < x1; q++) own[q] = 1;
    size_t p = entry, ls = 0, lm = 0;
    while (p < x1) {
        (*dec)++;
        if (n - p >= 3) own[p] = 1;
        size_t ms = 0;
        unsigned m = match_at(&v, p, &ms);
        if (m) {
            if (m <= c.lazy && n - p - m >= 3)
                for (size_t q = p + 1; q < p + m && q < x1; q++) own[q] = 1;
            ls = p; lm = m;
            p += m;
        } else {
            ls = lm = 0;
            p++;
        }
    }
    lane_out o = {p, ls, lm};
    return o;
}

int main(int argc, char **argv) {
    int kind = atoi(argv[1]), level = atoi(argv[2]);
    size_t seg = strtoull(argv[3], 0, 0);
    n = argc > 4 ? strtoull(argv[4], 0, 0) : (1u << 20);
    c = CFG[level];
    src = malloc(n + 300);
    link = malloc(2 * n);
    zo_generate(src, n, 1, kind, 1, 0);
    memset(src + n, 0, 300);
    zo_pp_links(src, n, link);
    size_t L = (n + seg - 1) / seg;
    /* sequential truth: one lane */
    uint8_t *truth = calloc(n, 1), *A = calloc(n, 1), *B = calloc(n, 1);
    unsigned long dec_seq = 0;
    steps = 0;
    lane_out t = parse_lane(0, n, 0, 0, 0, truth, truth, &dec_seq);
    unsigned long steps_seq = steps;
    (void)t;
    lane_out *prev = calloc(L, sizeof(lane_out)), *cur = calloc(L, sizeof(lane_out));
    uint8_t *chg = calloc(L, 1), *chg2 = calloc(L, 1);
    unsigned long dec_total = 0, lanes_run = 0;
    steps = 0;
    int r;
    uint8_t *old = A, *nw = B;
    for (r = 1; r <= 200; r++) {
        int changed = 0;
        for (size_t i = 0; i < L; i++) {
            size_t x0 = i * seg, x1 = x0 + seg < n ? x0 + seg : n;
            size_t entry = x0, pls = 0, plm = 0;
            if (i > 0 && r > 1) { entry = prev[i - 1].exit; pls = prev[i - 1].ls; plm = prev[i - 1].lm; }
            if (entry > x1) entry = x1;
            /* skip: nothing this lane reads changed in the last round */
            int need = r <= 2;
            if (!need) {
                if (i > 0 && (prev[i - 1].exit != cur[i - 1].exit || 1)) {}
                for (size_t j = (i * seg > 32768 ? (i * seg - 32768) / seg : 0); j <= i && !need; j++)
                    if (chg[j]) need = 1;
            }
            if (need) {
                unsigned long d = 0;
                cur[i] = parse_lane(x0, x1, entry, pls, plm, nw, old, &d);
                dec_total += d;
                lanes_run++;
            } else {
                cur[i] = prev[i];
                memcpy(nw + x0, old + x0, x1 - x0);
            }
            chg2[i] = r == 1 || memcmp(nw + x0, old + x0, x1 - x0) != 0 || cur[i].exit != prev[i].exit ||
                      cur[i].lm != prev[i].lm || cur[i].ls != prev[i].ls;
            if (chg2[i]) changed = 1;
        }
        /* consistency: entries used == neighbours' exits */
        int consistent = 1;
        for (size_t i = 1; i < L && consistent; i++) {
            size_t x0 = i * seg;
            size_t used = r > 1 ? prev[i - 1].exit : x0;
            if (used != cur[i - 1].exit) consistent = 0;
        }
        memcpy(prev, cur, L * sizeof(lane_out));
        memcpy(chg, chg2, L);
        uint8_t *tmp = old; old = nw; nw = tmp;
        if (!changed && consistent) break;
    }
    int ok = memcmp(old, truth, n) == 0;
    printf("kind %d L%d seg %zu n %zu: rounds %d, lanes run %lu (%.2f x lanes), decisions %.2f x seq, "
           "chain steps %.2f x seq, exact %d\n",
           kind, level, seg, n, r, lanes_run, (double)lanes_run / L, (double)dec_total / dec_seq,
           (double)steps / steps_seq, ok);
    return 0;
}
