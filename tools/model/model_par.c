/* CPU model (tools only, not shipped): longest_match for every position as
 * independent candidate evaluations instead of a dependent chain walk
 * (SURVEY Appendix B.1).  A position's candidates are its chain in order
 * (most recent first, within MAX_DIST, at most `chain`); longest_match's
 * result is the first candidate reaching nice, else the first argmax of the
 * match lengths (the quick reject never changes it).  Reports per position:
 *   seq   candidates the sequential walk visits (stops at nice / budget / limit)
 *   par   candidates evaluated when a position's candidates go out 64 at a
 *         time and evaluation stops after the batch holding a nice match
 *   w1    4-byte words read per candidate (compare until the first mismatch,
 *         at most 4 words = 16 bytes)
 *   long  candidates that match 16+ bytes (their compare goes on, 64 bytes a
 *         round, cooperatively)
 *   lanes SIMT use if every position's candidates fill whole waves (64-lane
 *         batches per position) against a flattened list (candidates of many
 *         positions packed)
 *   cc -O2 tools/model/model_par.c -Loracle -loracle -o /tmp/model_par
 *   LD_LIBRARY_PATH=oracle /tmp/model_par <kind> <level> [n] [buffers] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int zo_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed, uint64_t first_index);
void zo_pp_links(const uint8_t *src, size_t n, uint16_t *link);
#define MAXD 32506
static const unsigned CHAIN[10] = {0, 4, 8, 32, 16, 32, 128, 256, 1024, 4096};
static const unsigned NICE[10] = {0, 8, 16, 32, 16, 32, 128, 128, 258, 258};

int main(int argc, char **argv) {
    const int kind = atoi(argv[1]), level = atoi(argv[2]);
    const size_t n = argc > 3 ? strtoull(argv[3], 0, 0) : (1u << 20);
    const int nb = argc > 4 ? atoi(argv[4]) : 4;
    const unsigned chain = CHAIN[level], nice0 = NICE[level];
    uint8_t *src = malloc(n + 300);
    uint16_t *link = malloc(2 * n);
    unsigned *cand = malloc(sizeof(unsigned) * chain);
    double npos = 0, seq = 0, par = 0, w1 = 0, lng = 0, lng_rounds = 0, batches = 0, words_chain = 0;
    for (int b = 0; b < nb; b++) {
        zo_generate(src, n, 1, kind, 1, b);
        memset(src + n, 0, 300);
        zo_pp_links(src, n, link);
        for (size_t p = 1; p + 3 <= n; p++) {
            npos++;
            const size_t limit = p > MAXD ? p - MAXD : 0;
            const unsigned rem = (unsigned)(n - p);
            const unsigned nice = nice0 < rem ? nice0 : rem, maxcmp = rem < 258 ? rem : 258;
            unsigned k = 0;
            size_t cur = p;
            while (k < chain) {
                const unsigned d = link[cur];
                if (!d || cur - d <= limit) break;
                cur -= d;
                cand[k++] = (unsigned)cur;
            }
            /* lengths; the sequential walk stops at the first nice */
            static unsigned lens[4096];
            unsigned stop = k;
            for (unsigned i = 0; i < k; i++) {
                unsigned len = 0;
                while (len < maxcmp && src[cand[i] + len] == src[p + len]) len++;
                lens[i] = len;
                if (len >= nice && stop == k) stop = i + 1;
            }
            seq += stop;
            const unsigned pb = (stop + 63) / 64;       /* batches until the one holding the nice match */
            const unsigned ev = k < pb * 64 ? k : pb * 64;
            batches += pb;
            par += ev;
            for (unsigned i = 0; i < ev; i++) {
                const unsigned len = lens[i], wr = (len + 1 + 3) / 4;
                w1 += wr < 4 ? wr : 4;
                if (len >= 16) { lng++; lng_rounds += (len + 1 - 16 + 63) / 64; }
            }
            (void)words_chain;
        }
    }
    printf("kind %d L%d: seq %.1f cand/pos, par %.1f cand/pos (%.2fx), w1 %.2f words/cand, long %.3f/pos "
           "(%.3f rounds/pos), lanes per-position batches %.1f%%\n",
           kind, level, seq / npos, par / npos, par / seq, w1 / (par > 0 ? par : 1), lng / npos, lng_rounds / npos,
           100.0 * par / (batches * 64 > 0 ? batches * 64 : 1));
    return 0;
}
