/* CPU model (tools only, not shipped): the sorted-run candidate order of
 * k_bsort / k_bwork / k_match2 (zgpu_deflate.hip) against the hash chain.
 * For every position p <= n-3 it lists the candidates k_match2 visits --
 * Sr[base(k) - k] over the three runs of p's hash in its 16 Ki block and the
 * two before -- and checks them, in order, against the prev[] chain of
 * zo_pp_links (deflate.c INSERT_STRING) down to the limit
 * max(p - MAX_DIST, 0) (the head may sit exactly at MAX_DIST).  The ring
 * offsets, slides and index arithmetic are the kernel's.
 * Usage: model_match2 kind [n] [buffers] */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
int zo_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed, uint64_t first_index);
void zo_pp_links(const uint8_t *src, size_t n, uint16_t *link);
#define MAXD 32506
#define BS 16384
static uint32_t hash3(const uint8_t *b) { return ((b[0] & 31u) << 10) ^ ((uint32_t)b[1] << 5) ^ b[2]; }
static const uint8_t *g_src;
static int cmp_hp(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}
int main(int argc, char **argv) {
    int kind = argc > 1 ? atoi(argv[1]) : 1;
    size_t n = argc > 2 ? strtoull(argv[2], 0, 0) : (1u << 20);
    int nb = argc > 3 ? atoi(argv[3]) : 2;
    uint8_t *src = calloc(n + 64, 1);
    uint16_t *link = malloc(2 * n + 2);
    size_t nblk = (n + BS - 1) / BS;
    uint16_t *S = malloc(2 * nblk * BS);
    uint16_t *off = malloc(2 * nblk * 32769);
    uint32_t *keys = malloc(4 * BS);
    uint64_t checked = 0, bad = 0, cands = 0;
    for (int bb = 0; bb < nb; bb++) {
        zo_generate(src, n, 1, kind, 2025, bb);
        g_src = src;
        zo_pp_links(src, n, link);
        /* k_bsort */
        for (size_t b = 0; b < nblk; b++) {
            int64_t p0 = (int64_t)b * BS;
            int64_t mm = (int64_t)n - 2 - p0;
            int m = mm <= 0 ? 0 : (mm < BS ? (int)mm : BS);
            for (int e = 0; e < m; e++) keys[e] = hash3(src + p0 + e) << 14 | (uint32_t)e;
            qsort(keys, m, 4, cmp_hp);
            for (int i = 0; i < m; i++) S[b * BS + i] = keys[i] & (BS - 1);
            uint16_t *o = off + b * 32769;
            int i = 0;
            for (uint32_t h = 0; h <= 32768; h++) {
                while (i < m && (keys[i] >> 14) < h) i++;
                o[h] = (uint16_t)i;
            }
        }
        /* k_bwork + k_match2's candidate order */
        for (size_t b = 0; b < nblk; b++) {
            int64_t p0 = (int64_t)b * BS;
            int64_t mm = (int64_t)n - 2 - p0;
            int m = mm <= 0 ? 0 : (mm < BS ? (int)mm : BS);
            const uint16_t *o0 = off + b * 32769, *o1 = b >= 1 ? off + (b - 1) * 32769 : 0,
                           *o2 = b >= 2 ? off + (b - 2) * 32769 : 0;
            /* the ring as k_match2 holds it while walking block b: slot s = block b-2+s */
            static uint32_t Sr[3 * BS];
            for (int s = 0; s < 3; s++) {
                int64_t bb2 = (int64_t)b - 2 + s;
                for (int j = 0; j < BS; j++)
                    Sr[s * BS + j] = bb2 >= 0 ? (uint32_t)s * BS + S[bb2 * BS + j] : 0xdeadu;
            }
            int64_t base = p0 - 2 * BS;
            for (int i = 0; i < m; i++) {
                uint32_t rel = S[b * BS + i];
                uint32_t h = hash3(src + p0 + rel);
                uint32_t n0 = i - o0[h];
                uint32_t s1 = o1 ? o1[h] : 0, e1 = o1 ? o1[h + 1] : 0, s2 = o2 ? o2[h] : 0, e2 = o2 ? o2[h + 1] : 0;
                uint32_t n1 = e1 - s1, n2 = e2 - s2, n01 = n0 + n1, n012 = n01 + n2;
                int A0 = 2 * BS + i - 1, B1 = BS + (int)e1 - 1 + (int)n0, B2 = (int)e2 - 1 + (int)n01;
                int64_t p = p0 + rel;
                int64_t labs = p > MAXD ? p - MAXD : 0;
                int lim = (int)(labs - base);
                /* the chain */
                int64_t cur = link[p] ? p - link[p] : -1;
                int head_ok = cur >= 1 && p - cur <= MAXD;
                uint32_t k = 0;
                int hv = -1;
                if (n012) {
                    int idx = 0 < n0 ? A0 : (0 < n01 ? B1 : B2);
                    hv = (int)Sr[idx];
                }
                int m2_head_ok = n012 && base + hv >= 1 && p - (base + hv) <= MAXD;
                checked++;
                if (head_ok != m2_head_ok) { if (bad < 5) printf("head p %lld b %zu i %d cur %lld hv %d base %lld n012 %u\n", (long long)p, b, i, (long long)cur, hv, (long long)base, n012); bad++; continue; }
                if (!head_ok) continue;
                for (;;) {
                    int q;
                    {
                        int idx = k < n0 ? A0 - (int)k : (k < n01 ? B1 - (int)k : B2 - (int)k);
                        if (idx < 0) idx = 0;
                        q = k < n012 ? (int)Sr[idx] : -1;
                    }
                    int chain_valid = k == 0 ? 1 : (cur > labs);
                    int m2_valid = k == 0 ? 1 : (q > lim);
                    if (chain_valid != m2_valid) { if (bad < 5) printf("valid p %lld k %u cur %lld q %d lim %d\n", (long long)p, k, (long long)cur, q, lim); bad++; break; }
                    if (!chain_valid) break;
                    if (base + q != cur) { if (bad < 5) printf("cand p %lld k %u cur %lld q %lld n0 %u n1 %u n2 %u\n", (long long)p, k, (long long)cur, (long long)(base+q), n0, n1, n2); bad++; break; }
                    cands++;
                    k++;
                    if (!link[cur]) {
                        /* chain end: k_match2 must see no further candidate above the limit */
                        int idx = k < n0 ? A0 - (int)k : (k < n01 ? B1 - (int)k : B2 - (int)k);
                        if (idx < 0) idx = 0;
                        int qn = k < n012 ? (int)Sr[idx] : -1;
                        if (qn > lim) { if (bad < 5) printf("end p %lld k %u cur %lld qn %lld\n", (long long)p, k, (long long)cur, (long long)(base+qn)); bad++; }
                        break;
                    }
                    cur -= link[cur];
                }
            }
        }
    }
    printf("kind %d: %llu positions, %llu candidates, %llu mismatches\n", kind, (unsigned long long)checked,
           (unsigned long long)cands, (unsigned long long)bad);
    return bad != 0;
}
