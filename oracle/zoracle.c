/*
 * zoracle.c — TEST INFRASTRUCTURE ONLY: the CPU checker for the GPU path.
 *
 * A plain-C restatement of the reference's compression path
 * (/root/reference = discere-os/zlib.wasm, zlib 1.3.1.1-motley).  Each function
 * names the reference code it restates.  The restatement works on absolute input
 * positions over the whole buffer instead of zlib's 64 KiB sliding window; the
 * window schedule (slides, window end) is tracked only where it changes the
 * output: the stored-block eligibility test of FLUSH_BLOCK_ONLY
 * (deflate.c:1597-1600) and the lookahead clamps near the end of input.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library; the product (libzgpu.so) never does.
 */
#include "zoracle.h"
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* constants (zutil.h:77-89, deflate.h:33-55,293-303, deflate.c:88-90)       */
/* ------------------------------------------------------------------------ */
#define WSIZE        32768u
#define WINDOW_SIZE  (2u * WSIZE)
#define MIN_MATCH    3u
#define MAX_MATCH    258u
#define MIN_LOOKAHEAD (MAX_MATCH + MIN_MATCH + 1u)     /* 262 */
#define MAX_DIST     (WSIZE - MIN_LOOKAHEAD)           /* 32506 */
#define TOO_FAR      4096u
#define LIT_BUFSIZE  16384u                            /* 1 << (memLevel 8 + 6) */
#define SYM_LIMIT    (LIT_BUFSIZE - 1u)                 /* sym_end / 3 */
#define L_CODES      286
#define D_CODES      30
#define BL_CODES     19
#define HEAP_SIZE    (2 * L_CODES + 1)
#define MAX_BITS     15
#define MAX_BL_BITS  7
#define END_BLOCK    256
#define MAX_STORED   65535u

/* configuration_table, deflate.c:112-125: good, lazy, nice, chain */
typedef struct { unsigned good, lazy, nice, chain; } zo_cfg;
static const zo_cfg CFG[10] = {
    {0, 0, 0, 0},      {4, 4, 8, 4},       {4, 5, 16, 8},     {4, 6, 32, 32},
    {4, 4, 16, 16},    {8, 16, 32, 32},    {8, 16, 128, 128}, {8, 32, 128, 256},
    {32, 128, 258, 1024}, {32, 258, 258, 4096}};

/* ------------------------------------------------------------------------ */
/* static code tables, derived from RFC 1951 §3.2.5-3.2.6 the way            */
/* tr_static_init (trees.c:303-396) derives them                             */
/* ------------------------------------------------------------------------ */
static const int xlbits[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
static const int xdbits[30] = {0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};
static const int xblbits[19] = {0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,2,3,7};
static const uint8_t bl_order[19] = {16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15};

static uint8_t  len_code[256];      /* normalized match length -> 0..28 */
static int      len_base[29];
static uint8_t  dist_code_tab[512]; /* d<256: [d]; else [256 + (d>>7)] */
static int      dist_base[30];
static uint16_t stat_lcode[288], stat_dcode[30];
static uint8_t  stat_llen[288], stat_dlen[30];
static uint32_t crc_tab[256];
static int      tables_ready;

static unsigned bitrev(unsigned code, int len) {
    unsigned r = 0;
    while (len-- > 0) { r = (r << 1) | (code & 1u); code >>= 1; }
    return r;
}

/* canonical codes from lengths (gen_codes, trees.c:203-232) */
static void canon_codes(const uint8_t *lens, uint16_t *codes, int max_code,
                        const uint16_t *count) {
    uint16_t next[MAX_BITS + 1];
    unsigned c = 0;
    for (int b = 1; b <= MAX_BITS; b++) { c = (c + count[b - 1]) << 1; next[b] = (uint16_t)c; }
    for (int n = 0; n <= max_code; n++)
        if (lens[n]) codes[n] = (uint16_t)bitrev(next[lens[n]]++, lens[n]);
}

static void init_tables(void) {
    if (tables_ready) return;
    int length = 0, code;
    for (code = 0; code < 28; code++) {
        len_base[code] = length;
        for (int k = 0; k < (1 << xlbits[code]); k++) len_code[length++] = (uint8_t)code;
    }
    len_code[255] = 28;       /* length 258 uses code 285, not 284 + 31 */
    len_base[28] = 0;
    int dist = 0;
    for (code = 0; code < 16; code++) {
        dist_base[code] = dist;
        for (int k = 0; k < (1 << xdbits[code]); k++) dist_code_tab[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < 30; code++) {
        dist_base[code] = dist << 7;
        for (int k = 0; k < (1 << (xdbits[code] - 7)); k++) dist_code_tab[256 + dist++] = (uint8_t)code;
    }
    uint16_t cnt[MAX_BITS + 1] = {0};
    for (int n = 0; n < 288; n++) {
        stat_llen[n] = (uint8_t)(n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8);
        cnt[stat_llen[n]]++;
    }
    canon_codes(stat_llen, stat_lcode, 287, cnt);
    for (int n = 0; n < 30; n++) { stat_dlen[n] = 5; stat_dcode[n] = (uint16_t)bitrev((unsigned)n, 5); }
    for (unsigned n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        crc_tab[n] = c;
    }
    tables_ready = 1;
}

static inline unsigned d_code(unsigned d) {            /* deflate.h:317-318 */
    return d < 256 ? dist_code_tab[d] : dist_code_tab[256 + (d >> 7)];
}

/* ------------------------------------------------------------------------ */
/* CRC-32 (crc32.c:694-1049) and Adler-32 (adler32.c:61-155)                 */
/* ------------------------------------------------------------------------ */
uint32_t zo_crc32(uint32_t crc, const uint8_t *buf, size_t len) {
    init_tables();
    if (buf == NULL) return 0;                         /* crc32.c:700 */
    crc = ~crc;
    while (len--) crc = (crc >> 8) ^ crc_tab[(crc ^ *buf++) & 0xffu];
    return ~crc;
}

#define POLY 0xedb88320u
static uint32_t multmodp(uint32_t a, uint32_t b) {     /* crc32.c:155-170 */
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) { p ^= b; if ((a & (m - 1)) == 0) break; }
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ POLY : b >> 1;
    }
    return p;
}
static uint32_t x2nmodp(int64_t n, unsigned k) {       /* crc32.c:176-187 */
    static uint32_t x2n[32];
    if (!x2n[0]) {
        uint32_t p = 1u << 30;                         /* x^1 */
        x2n[0] = p;
        for (int i = 1; i < 32; i++) x2n[i] = p = multmodp(p, p);
    }
    uint32_t p = 1u << 31;                             /* x^0 */
    while (n) {
        if (n & 1) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}
uint32_t zo_crc32_combine(uint32_t crc1, uint32_t crc2, int64_t len2) {
    return multmodp(x2nmodp(len2, 3), crc1) ^ crc2;   /* crc32.c:1021-1026 */
}

#define ABASE 65521u
#define ANMAX 5552u
uint32_t zo_adler32(uint32_t adler, const uint8_t *buf, size_t len) {
    uint32_t a = adler & 0xffffu, b = (adler >> 16) & 0xffffu;
    if (len == 1) {                                    /* adler32.c:71-80 */
        a += buf[0];
        if (a >= ABASE) a -= ABASE;
        b += a;
        if (b >= ABASE) b -= ABASE;
        return a | (b << 16);
    }
    if (buf == NULL) return 1;                         /* adler32.c:83-84 */
    if (len < 16) {                                    /* adler32.c:87-94 */
        while (len--) { a += *buf++; b += a; }
        if (a >= ABASE) a -= ABASE;
        b %= ABASE;
        return a | (b << 16);
    }
    while (len > 0) {                                  /* adler32.c:97-122 */
        size_t k = len < ANMAX ? len : ANMAX;
        len -= k;
        while (k--) { a += *buf++; b += a; }
        a %= ABASE;
        b %= ABASE;
    }
    return a | (b << 16);
}
uint32_t zo_adler32_combine(uint32_t adler1, uint32_t adler2, int64_t len2) {
    if (len2 < 0) return 0xffffffffu;                  /* adler32.c:133-155 */
    uint32_t rem = (uint32_t)(len2 % ABASE);
    uint32_t s1 = adler1 & 0xffffu;
    uint32_t s2 = (uint32_t)(((uint64_t)rem * s1) % ABASE);
    s1 += (adler2 & 0xffffu) + ABASE - 1;
    s2 += ((adler1 >> 16) & 0xffffu) + ((adler2 >> 16) & 0xffffu) + ABASE - rem;
    if (s1 >= ABASE) s1 -= ABASE;
    if (s1 >= ABASE) s1 -= ABASE;
    if (s2 >= (ABASE << 1)) s2 -= (ABASE << 1);
    if (s2 >= ABASE) s2 -= ABASE;
    return s1 | (s2 << 16);
}

unsigned long zo_compress_bound(unsigned long n) {    /* compress.c:72-75 */
    return n + (n >> 12) + (n >> 14) + (n >> 25) + 13;
}

/* ------------------------------------------------------------------------ */
/* bit writer: the LSB-first stream that send_bits/put_short/bi_windup       */
/* (trees.c:166-193,274-286) produce                                         */
/* ------------------------------------------------------------------------ */
typedef struct { uint8_t *buf; size_t cap, len; uint64_t acc; int nb; int oom; } bw_t;

static void bw_byte(bw_t *w, uint8_t v) {
    if (w->len == w->cap) {
        size_t nc = w->cap ? w->cap * 2 : 4096;
        uint8_t *nbuf = (uint8_t *)realloc(w->buf, nc);
        if (!nbuf) { w->oom = 1; return; }
        w->buf = nbuf; w->cap = nc;
    }
    w->buf[w->len++] = v;
}
static void bw_bits(bw_t *w, uint32_t v, int n) {
    w->acc |= (uint64_t)v << w->nb;
    w->nb += n;
    while (w->nb >= 8) { bw_byte(w, (uint8_t)w->acc); w->acc >>= 8; w->nb -= 8; }
}
static void bw_align(bw_t *w) {                        /* bi_windup */
    if (w->nb > 0) bw_byte(w, (uint8_t)w->acc);
    w->acc = 0; w->nb = 0;
}

/* ------------------------------------------------------------------------ */
/* Huffman trees (trees.c:499-706: smaller, pqdownheap, gen_bitlen,          */
/* build_tree) restated with separate freq/dad/len arrays                    */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint16_t freq[HEAP_SIZE];
    uint16_t dad[HEAP_SIZE];
    uint8_t  len[HEAP_SIZE + 1];   /* +1: scan_tree guard slot */
    uint16_t code[HEAP_SIZE];
    int      max_code;
} tree_t;

typedef struct {
    int heap[HEAP_SIZE + 1];
    int heap_len, heap_max;
    uint8_t depth[HEAP_SIZE];
    uint16_t bl_count[MAX_BITS + 1];
    int64_t opt_len, static_len;
} huff_t;

static inline int smaller(const tree_t *t, const huff_t *h, int n, int m) {
    return t->freq[n] < t->freq[m] || (t->freq[n] == t->freq[m] && h->depth[n] <= h->depth[m]);
}
static void downheap(const tree_t *t, huff_t *h, int k) {
    int v = h->heap[k], j = k << 1;
    while (j <= h->heap_len) {
        if (j < h->heap_len && smaller(t, h, h->heap[j + 1], h->heap[j])) j++;
        if (smaller(t, h, v, h->heap[j])) break;
        h->heap[k] = h->heap[j];
        k = j;
        j <<= 1;
    }
    h->heap[k] = v;
}

static void gen_lengths(tree_t *t, huff_t *h, const uint8_t *slen, const int *extra,
                        int xbase, int max_length) {
    int overflow = 0;
    for (int b = 0; b <= MAX_BITS; b++) h->bl_count[b] = 0;
    t->len[h->heap[h->heap_max]] = 0;                  /* root */
    int hh;
    for (hh = h->heap_max + 1; hh < HEAP_SIZE; hh++) {
        int n = h->heap[hh];
        int bits = t->len[t->dad[n]] + 1;
        if (bits > max_length) { bits = max_length; overflow++; }
        t->len[n] = (uint8_t)bits;
        if (n > t->max_code) continue;                 /* internal node */
        h->bl_count[bits]++;
        int xb = n >= xbase ? extra[n - xbase] : 0;
        h->opt_len += (int64_t)t->freq[n] * (bits + xb);
        if (slen) h->static_len += (int64_t)t->freq[n] * (slen[n] + xb);
    }
    if (overflow == 0) return;
    do {                                               /* trees.c:584-596 */
        int bits = max_length - 1;
        while (h->bl_count[bits] == 0) bits--;
        h->bl_count[bits]--;
        h->bl_count[bits + 1] += 2;
        h->bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    hh = HEAP_SIZE;                                    /* trees.c:603-612 */
    for (int bits = max_length; bits != 0; bits--) {
        int n = h->bl_count[bits];
        while (n != 0) {
            int m = h->heap[--hh];
            if (m > t->max_code) continue;
            if (t->len[m] != bits) {
                h->opt_len += ((int64_t)bits - t->len[m]) * t->freq[m];
                t->len[m] = (uint8_t)bits;
            }
            n--;
        }
    }
}

static void build_tree(tree_t *t, huff_t *h, int elems, const uint8_t *slen,
                       const int *extra, int xbase, int max_length) {
    int max_code = -1;
    h->heap_len = 0;
    h->heap_max = HEAP_SIZE;
    for (int n = 0; n < elems; n++) {
        if (t->freq[n] != 0) { h->heap[++h->heap_len] = max_code = n; h->depth[n] = 0; }
        else t->len[n] = 0;
    }
    while (h->heap_len < 2) {                          /* trees.c:655-661 */
        int node = h->heap[++h->heap_len] = (max_code < 2 ? ++max_code : 0);
        t->freq[node] = 1;
        h->depth[node] = 0;
        h->opt_len--;
        if (slen) h->static_len -= slen[node];
    }
    t->max_code = max_code;
    for (int n = h->heap_len / 2; n >= 1; n--) downheap(t, h, n);
    int node = elems;
    do {
        int n = h->heap[1];
        h->heap[1] = h->heap[h->heap_len--];
        downheap(t, h, 1);
        int m = h->heap[1];
        h->heap[--h->heap_max] = n;
        h->heap[--h->heap_max] = m;
        t->freq[node] = (uint16_t)(t->freq[n] + t->freq[m]);
        h->depth[node] = (uint8_t)((h->depth[n] >= h->depth[m] ? h->depth[n] : h->depth[m]) + 1);
        t->dad[n] = t->dad[m] = (uint16_t)node;
        h->heap[1] = node++;
        downheap(t, h, 1);
    } while (h->heap_len >= 2);
    h->heap[--h->heap_max] = h->heap[1];
    gen_lengths(t, h, slen, extra, xbase, max_length);
    canon_codes(t->len, t->code, max_code, h->bl_count);
}

/* code-length RLE walk shared by scan_tree / send_tree (trees.c:712-794):
 * emit(sym, extra_val, extra_bits) is called per bit-length-tree symbol. */
typedef void (*rle_sink)(void *ctx, int sym, int xval, int xbits);
static void rle_tree(const uint8_t *len, int max_code, rle_sink sink, void *ctx) {
    int prevlen = -1, curlen, nextlen = len[0], count = 0;
    int max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = n + 1 <= max_code ? len[n + 1] : 0xffff;  /* guard */
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            while (count--) sink(ctx, curlen, 0, 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) { sink(ctx, curlen, 0, 0); count--; }
            sink(ctx, 16, count - 3, 2);
        } else if (count <= 10) {
            sink(ctx, 17, count - 3, 3);
        } else {
            sink(ctx, 18, count - 11, 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}
static void count_sink(void *ctx, int sym, int xval, int xbits) {
    (void)xval; (void)xbits;
    ((tree_t *)ctx)->freq[sym]++;
}
typedef struct { bw_t *w; const tree_t *bl; } send_ctx;
static void send_sink(void *ctx, int sym, int xval, int xbits) {
    send_ctx *c = (send_ctx *)ctx;
    bw_bits(c->w, c->bl->code[sym], c->bl->len[sym]);
    if (xbits) bw_bits(c->w, (uint32_t)xval, xbits);
}

/* ------------------------------------------------------------------------ */
/* deflate state                                                             */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t *in;
    size_t n;
    zo_cfg cfg;
    int level;
    int pp;                    /* 0 = sequential restatement, 1 = position-parallel */
    /* sequential hash chains (absolute positions; 0 == NIL) */
    uint32_t *head, *prev;
    /* position-parallel data */
    uint16_t *link;
    uint32_t *rfull, *rquart;
    uint8_t  *ins;             /* inserted-set bitmap (levels 1..3, pp) */
    int strategy;              /* Z_DEFAULT_STRATEGY 0, Z_FILTERED 1, Z_HUFFMAN_ONLY 2, Z_RLE 3, Z_FIXED 4 */
    /* window schedule: S = slide offset, E = end of data read so far */
    size_t S, E;
    size_t block_start;
    /* deflate() calls with flushes (zo_deflate_flushes): the data available is
     * [0, avail); flush event fi ends at fpos[fi] with type ftype[fi];
     * insert = positions before strstart still to be hashed (deflate.c:1944) */
    size_t avail, insert;
    const size_t *fpos;
    const int *ftype;
    int nf, fi;
    int open_end;              /* the stream is not finished: no final block, no trailer */
    /* current block */
    uint32_t sym[LIT_BUFSIZE]; /* (dist << 8) | lc  (dist 0 => literal lc) */
    unsigned nsym;
    tree_t lt, dt, bt;
    huff_t hf;
    bw_t bw;
} zs_t;

static inline unsigned hash3(const uint8_t *p) {      /* UPDATE_HASH x3, deflate.c:141 */
    return (((unsigned)p[0] & 31u) << 10) ^ ((unsigned)p[1] << 5) ^ p[2];
}

/* fill_window (deflate.c:251-368), window bookkeeping only */
static size_t insert_at(zs_t *s, size_t p);
static void fill(zs_t *s, size_t p) {
    if (p - s->S >= WSIZE + MAX_DIST) s->S += WSIZE;  /* slide, :277-287 */
    if (s->E < s->avail) {                              /* read_buf, :306 */
        size_t e = s->S + WINDOW_SIZE;
        s->E = e < s->avail ? e : s->avail;
        /* hash the strings a flush left unhashed (:318-335) */
        if (s->insert && s->E - p + s->insert >= MIN_MATCH) {
            size_t str = p - s->insert;
            while (s->insert) {
                insert_at(s, str);
                str++;
                s->insert--;
                if (s->E - p + s->insert < MIN_MATCH) break;
            }
        }
    }
}

static void flush_block(zs_t *s, size_t strstart, int last);
/* end of a deflate(flush) call at p (deflate.c:2030-2042 and :1211-1233): the
 * parser has tallied its pending literal; returns 1 when the event was a
 * flush (the parse continues), 0 at the end of the stream (Z_FINISH) */
static int flush_event(zs_t *s, size_t p, size_t ins) {
    if (s->fi >= s->nf || s->fpos[s->fi] != p) return 0;
    const int t = s->ftype[s->fi++];
    s->insert = ins;
    if (s->nsym) flush_block(s, p, 0);
    bw_t *w = &s->bw;
    if (t == 1) {                                       /* Z_PARTIAL_FLUSH: _tr_align, trees.c:900 */
        bw_bits(w, 1u << 1, 3);
        bw_bits(w, 0, 7);                               /* static END_BLOCK: 7 zero bits */
    } else if (t == 2 || t == 3) {                      /* _tr_stored_block(s, 0, 0, 0) */
        bw_bits(w, 0, 3);
        bw_align(w);
        bw_byte(w, 0); bw_byte(w, 0); bw_byte(w, 0xff); bw_byte(w, 0xff);
        if (t == 3) {                                   /* Z_FULL_FLUSH: CLEAR_HASH, window reset */
            if (s->head) memset(s->head, 0, 32768 * sizeof(uint32_t));
            s->S = p;
            s->block_start = p;
            s->insert = 0;
        }
    }                                                   /* t == 5 (Z_BLOCK): nothing */
    s->avail = s->fi < s->nf ? s->fpos[s->fi] : s->n;
    return 1;
}

static void block_reset(zs_t *s) {                     /* init_block, trees.c:411-422 */
    memset(s->lt.freq, 0, sizeof s->lt.freq);
    memset(s->dt.freq, 0, sizeof s->dt.freq);
    memset(s->bt.freq, 0, sizeof s->bt.freq);
    s->lt.freq[END_BLOCK] = 1;
    s->nsym = 0;
}

/* _tr_tally_lit / _tr_tally_dist (deflate.h:354-372); returns bflush */
static int tally_lit(zs_t *s, unsigned c) {
    s->sym[s->nsym++] = c;
    s->lt.freq[c]++;
    return s->nsym == SYM_LIMIT;
}
static int tally_dist(zs_t *s, unsigned dist, unsigned lc) {
    s->sym[s->nsym++] = (dist << 8) | lc;
    s->lt.freq[len_code[lc] + 257]++;
    s->dt.freq[d_code(dist - 1)]++;
    return s->nsym == SYM_LIMIT;
}

static void emit_symbols(zs_t *s, const uint16_t *lcode, const uint8_t *llen,
                         const uint16_t *dcode, const uint8_t *dlen) {
    bw_t *w = &s->bw;                                  /* compress_block, trees.c:900-951 */
    for (unsigned i = 0; i < s->nsym; i++) {
        unsigned dist = s->sym[i] >> 8, lc = s->sym[i] & 0xffu;
        if (dist == 0) { bw_bits(w, lcode[lc], llen[lc]); continue; }
        unsigned code = len_code[lc];
        bw_bits(w, lcode[code + 257], llen[code + 257]);
        if (xlbits[code]) bw_bits(w, lc - (unsigned)len_base[code], xlbits[code]);
        dist--;
        code = d_code(dist);
        bw_bits(w, dcode[code], dlen[code]);
        if (xdbits[code]) bw_bits(w, dist - (unsigned)dist_base[code], xdbits[code]);
    }
    bw_bits(w, lcode[END_BLOCK], llen[END_BLOCK]);
}

/* FLUSH_BLOCK_ONLY (deflate.c:1597-1606) + _tr_flush_block (trees.c:997-1089) */
static void flush_block(zs_t *s, size_t strstart, int last) {
    size_t stored_len = strstart - s->block_start;
    int have_buf = s->block_start >= s->S;             /* block_start >= 0 in window terms */
    huff_t *h = &s->hf;
    h->opt_len = h->static_len = 0;
    build_tree(&s->lt, h, L_CODES, stat_llen, xlbits, 257, MAX_BITS);
    build_tree(&s->dt, h, D_CODES, stat_dlen, xdbits, 0, MAX_BITS);
    /* build_bl_tree, trees.c:800-826 */
    rle_tree(s->lt.len, s->lt.max_code, count_sink, &s->bt);
    rle_tree(s->dt.len, s->dt.max_code, count_sink, &s->bt);
    build_tree(&s->bt, h, BL_CODES, NULL, xblbits, 0, MAX_BL_BITS);
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (s->bt.len[bl_order[max_blindex]] != 0) break;
    h->opt_len += 3 * ((int64_t)max_blindex + 1) + 5 + 5 + 4;

    uint64_t opt_lenb = ((uint64_t)h->opt_len + 3 + 7) >> 3;
    uint64_t static_lenb = ((uint64_t)h->static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb || s->strategy == ZO_FIXED) opt_lenb = static_lenb;   /* trees.c:1035 */

    bw_t *w = &s->bw;
    if (stored_len + 4 <= opt_lenb && have_buf) {      /* _tr_stored_block, trees.c:860-875 */
        bw_bits(w, (0u << 1) + (unsigned)last, 3);
        bw_align(w);
        bw_byte(w, (uint8_t)stored_len);
        bw_byte(w, (uint8_t)(stored_len >> 8));
        bw_byte(w, (uint8_t)~stored_len);
        bw_byte(w, (uint8_t)(~stored_len >> 8));
        for (size_t i = 0; i < stored_len; i++) bw_byte(w, s->in[s->block_start + i]);
    } else if (static_lenb == opt_lenb) {
        bw_bits(w, (1u << 1) + (unsigned)last, 3);
        emit_symbols(s, stat_lcode, stat_llen, stat_dcode, stat_dlen);
    } else {
        bw_bits(w, (2u << 1) + (unsigned)last, 3);
        int lcodes = s->lt.max_code + 1, dcodes = s->dt.max_code + 1;
        bw_bits(w, (unsigned)(lcodes - 257), 5);      /* send_all_trees, trees.c:833-855 */
        bw_bits(w, (unsigned)(dcodes - 1), 5);
        bw_bits(w, (unsigned)(max_blindex + 1 - 4), 4);
        for (int r = 0; r <= max_blindex; r++) bw_bits(w, s->bt.len[bl_order[r]], 3);
        send_ctx sc = {w, &s->bt};
        rle_tree(s->lt.len, lcodes - 1, send_sink, &sc);
        rle_tree(s->dt.len, dcodes - 1, send_sink, &sc);
        emit_symbols(s, s->lt.code, s->lt.len, s->dt.code, s->dt.len);
    }
    block_reset(s);
    if (last) bw_align(w);
    s->block_start = strstart;
}

/* ------------------------------------------------------------------------ */
/* match finding                                                             */
/* ------------------------------------------------------------------------ */
static inline unsigned common_prefix(const uint8_t *a, const uint8_t *b, unsigned maxlen) {
    unsigned k = 0;
    while (k < maxlen && a[k] == b[k]) k++;
    return k;
}

/* longest_match (deflate.c:1356-1497), sequential hash chains.
 * Bytes past the end of input never decide the outcome (the result is
 * clamped to lookahead and nice is clamped to lookahead, :1396,:1495), so the
 * compare stops at the end of input. */
static unsigned longest_match_seq(zs_t *s, size_t p, size_t cur, unsigned prev_length,
                                  size_t *match_start) {
    unsigned chain = s->cfg.chain;
    if (prev_length >= s->cfg.good) chain >>= 2;
    size_t lookahead = s->E - p;
    unsigned nice = s->cfg.nice;
    if (nice > lookahead) nice = (unsigned)lookahead;
    size_t limit = (p - s->S) > MAX_DIST ? p - MAX_DIST : s->S;
    unsigned maxcmp = (size_t)MAX_MATCH < s->n - p ? MAX_MATCH : (unsigned)(s->n - p);
    unsigned best = prev_length;
    const uint8_t *scan = s->in + p;
    do {
        const uint8_t *m = s->in + cur;
        if (m[0] != scan[0] || m[1] != scan[1]) continue;
        unsigned len = common_prefix(scan, m, maxcmp);
        if (len > best) {
            *match_start = cur;
            best = len;
            if (len >= nice) break;
        }
    } while ((cur = s->prev[cur]) > limit && --chain != 0);
    return best <= lookahead ? best : (unsigned)lookahead;
}

/* Levels 1..3 position-parallel form: walk the all-positions links, skipping
 * positions the parse never inserted. */
static size_t next_inserted(const zs_t *s, size_t q, size_t floor_excl) {
    while (q > floor_excl && !s->ins[q]) {
        unsigned d = s->link[q];
        if (!d) return 0;
        q -= d;
    }
    return q > floor_excl ? q : 0;
}

static unsigned longest_match_ins(zs_t *s, size_t p, size_t cur, unsigned prev_length,
                                  size_t *match_start) {
    unsigned chain = s->cfg.chain;
    if (prev_length >= s->cfg.good) chain >>= 2;
    size_t lookahead = s->E - p;
    unsigned nice = s->cfg.nice;
    if (nice > lookahead) nice = (unsigned)lookahead;
    size_t limit = (p - s->S) > MAX_DIST ? p - MAX_DIST : s->S;
    unsigned maxcmp = (size_t)MAX_MATCH < s->n - p ? MAX_MATCH : (unsigned)(s->n - p);
    unsigned best = prev_length;
    const uint8_t *scan = s->in + p;
    for (;;) {
        const uint8_t *m = s->in + cur;
        if (m[0] == scan[0] && m[1] == scan[1]) {
            unsigned len = common_prefix(scan, m, maxcmp);
            if (len > best) {
                *match_start = cur;
                best = len;
                if (len >= nice) break;
            }
        }
        unsigned d = s->link[cur];
        if (!d) break;
        cur = next_inserted(s, cur - d, limit);
        if (cur == 0 || --chain == 0) break;
    }
    return best <= lookahead ? best : (unsigned)lookahead;
}

/* head of the chain at p (0 == none): INSERT_STRING's match_head */
static size_t insert_at(zs_t *s, size_t p) {
    if (s->pp) {
        s->ins[p] = 1;
        if (s->level >= 4) return s->link[p] ? p - s->link[p] : 0;
        unsigned d = s->link[p];
        if (!d) return 0;
        /* most recent inserted same-hash position; anything at or below
         * p - 32768 is out of reach of every test that follows */
        size_t lo = p > 32768 ? p - 32768 : 0;
        return next_inserted(s, p - d, lo);
    }
    unsigned h = hash3(s->in + p);
    size_t hh = s->head[h];
    s->prev[p] = (uint32_t)hh;
    s->head[h] = (uint32_t)p;
    return hh;
}

static inline int head_ok(const zs_t *s, size_t p, size_t hh) {
    /* hash_head != NIL && strstart - hash_head <= MAX_DIST (deflate.c:1853,1955);
     * NIL is window index 0, i.e. absolute S (or anything slid out). */
    return hh > s->S && p - hh <= MAX_DIST;
}

/* deflate_fast (deflate.c:1824-1915) */
static void run_fast(zs_t *s) {
    size_t p = 0, match_start = 0;
    unsigned match_length = MIN_MATCH - 1;
    for (;;) {
        if (s->E - p < MIN_LOOKAHEAD) {
            fill(s, p);
            if (s->E == p) {
                if (flush_event(s, p, p - s->S < MIN_MATCH - 1 ? p - s->S : MIN_MATCH - 1)) continue;
                break;
            }
        }
        size_t lookahead = s->E - p;
        size_t hh = 0;
        if (lookahead >= MIN_MATCH) hh = insert_at(s, p);
        if (hh && head_ok(s, p, hh))
            match_length = s->pp ? longest_match_ins(s, p, hh, MIN_MATCH - 1, &match_start)
                                 : longest_match_seq(s, p, hh, MIN_MATCH - 1, &match_start);
        int bflush;
        if (match_length >= MIN_MATCH) {
            bflush = tally_dist(s, (unsigned)(p - match_start), match_length - MIN_MATCH);
            lookahead -= match_length;
            if (match_length <= s->cfg.lazy && lookahead >= MIN_MATCH) {
                for (unsigned k = 1; k < match_length; k++) insert_at(s, p + k);
            }
            p += match_length;
            match_length = 0;
        } else {
            bflush = tally_lit(s, s->in[p]);
            p++;
        }
        if (bflush) flush_block(s, p, 0);
    }
    if (!s->open_end) flush_block(s, p, 1);
}

/* deflate_slow (deflate.c:1923-2043) */
static void run_slow(zs_t *s) {
    size_t p = 0, match_start = 0, prev_match = 0;
    unsigned match_length = MIN_MATCH - 1, prev_length;
    int match_available = 0;
    for (;;) {
        if (s->E - p < MIN_LOOKAHEAD) {
            fill(s, p);
            if (s->E == p) {
                if (s->fi < s->nf && s->fpos[s->fi] == p) {
                    if (match_available) tally_lit(s, s->in[p - 1]);   /* no flush test */
                    match_available = 0;
                    match_length = MIN_MATCH - 1;
                    flush_event(s, p, p - s->S < MIN_MATCH - 1 ? p - s->S : MIN_MATCH - 1);
                    continue;
                }
                break;
            }
        }
        size_t lookahead = s->E - p;
        size_t hh = 0;
        if (lookahead >= MIN_MATCH) hh = insert_at(s, p);
        prev_length = match_length;
        prev_match = match_start;
        match_length = MIN_MATCH - 1;
        if (hh && prev_length < s->cfg.lazy && head_ok(s, p, hh)) {
            if (s->pp) {
                uint32_t r = (prev_length >= s->cfg.good) ? s->rquart[p] : s->rfull[p];
                unsigned rl = r >> 16;
                if (rl > prev_length) { match_length = rl; match_start = p - (r & 0xffffu); }
                else match_length = prev_length <= lookahead ? prev_length : (unsigned)lookahead;
            } else {
                match_length = longest_match_seq(s, p, hh, prev_length, &match_start);
            }
            if (match_length <= 5 && (s->strategy == ZO_FILTERED ||          /* deflate.c:1964-1975 */
                                      (match_length == MIN_MATCH && p - match_start > TOO_FAR)))
                match_length = MIN_MATCH - 1;
        }
        if (prev_length >= MIN_MATCH && match_length <= prev_length) {
            size_t max_insert = p + lookahead - MIN_MATCH;
            int bflush = tally_dist(s, (unsigned)(p - 1 - prev_match), prev_length - MIN_MATCH);
            for (unsigned k = 1; k <= prev_length - 2; k++)
                if (p + k <= max_insert) insert_at(s, p + k);
            p += prev_length - 1;
            match_available = 0;
            match_length = MIN_MATCH - 1;
            if (bflush) flush_block(s, p, 0);
        } else if (match_available) {
            if (tally_lit(s, s->in[p - 1])) flush_block(s, p, 0);
            p++;
        } else {
            match_available = 1;
            p++;
        }
    }
    if (s->open_end) return;
    if (match_available) tally_lit(s, s->in[p - 1]);
    flush_block(s, p, 1);
}

/* deflate_rle (deflate.c:2051-2116): runs of the previous byte at distance 1.
 * fill_window when lookahead <= MAX_MATCH. */
static void run_rle(zs_t *s) {
    size_t p = 0;
    for (;;) {
        if (s->E - p <= MAX_MATCH) {
            fill(s, p);
            if (s->E == p) {
                if (flush_event(s, p, 0)) continue;
                break;
            }
        }
        const size_t lookahead = s->E - p;
        unsigned match_length = 0;
        if (lookahead >= MIN_MATCH && p > s->S) {       /* strstart > 0 */
            const uint8_t prev = s->in[p - 1];
            if (s->in[p] == prev && s->in[p + 1] == prev && s->in[p + 2] == prev) {
                unsigned len = 3;                          /* run length, capped at MAX_MATCH */
                while (len < MAX_MATCH && p + len < s->n && s->in[p + len] == prev) len++;
                match_length = len <= lookahead ? len : (unsigned)lookahead;
            }
        }
        int bflush;
        if (match_length >= MIN_MATCH) {
            bflush = tally_dist(s, 1, match_length - MIN_MATCH);
            p += match_length;
        } else {
            bflush = tally_lit(s, s->in[p]);
            p++;
        }
        if (bflush) flush_block(s, p, 0);
    }
    if (!s->open_end) flush_block(s, p, 1);
}

/* deflate_huff (deflate.c:2122-2152): literals only; fill_window when the
 * lookahead is 0. */
static void run_huff(zs_t *s) {
    size_t p = 0;
    for (;;) {
        if (s->E == p) {
            fill(s, p);
            if (s->E == p) {
                if (flush_event(s, p, 0)) continue;
                break;
            }
        }
        const int bflush = tally_lit(s, s->in[p]);
        p++;
        if (bflush) flush_block(s, p, 0);
    }
    if (!s->open_end) flush_block(s, p, 1);
}

/* deflate_stored (deflate.c:1635-1815) for a single deflate(Z_FINISH) call
 * with an output buffer of at least compressBound() bytes: MAX_STORED-sized
 * stored blocks straight from the input, the last one flagged final. */
static void run_stored(zs_t *s) {
    size_t left = s->n, off = 0;
    do {
        size_t len = left < MAX_STORED ? left : MAX_STORED;
        int last = len == left;
        bw_bits(&s->bw, (unsigned)last, 3);
        bw_align(&s->bw);
        bw_byte(&s->bw, (uint8_t)len);
        bw_byte(&s->bw, (uint8_t)(len >> 8));
        bw_byte(&s->bw, (uint8_t)~len);
        bw_byte(&s->bw, (uint8_t)(~len >> 8));
        for (size_t i = 0; i < len; i++) bw_byte(&s->bw, s->in[off + i]);
        off += len;
        left -= len;
        if (last) break;
    } while (1);
}

/* ------------------------------------------------------------------------ */
/* position-parallel pieces                                                  */
/* ------------------------------------------------------------------------ */
void zo_pp_links(const uint8_t *src, size_t n, uint16_t *link) {
    uint32_t *last = (uint32_t *)calloc(32768, sizeof(uint32_t));
    if (!last) return;
    for (size_t p = 0; p < n; p++) {
        link[p] = 0;
        if (p + MIN_MATCH > n) continue;
        unsigned h = hash3(src + p);
        size_t q = last[h];
        if (q != 0 && p - q <= 32767) link[p] = (uint16_t)(p - q);
        last[h] = (uint32_t)p;   /* position 0 is stored as 0 == NIL */
    }
    free(last);
}

void zo_pp_match(const uint8_t *src, size_t n, int level, const uint16_t *link,
                 uint32_t *full, uint32_t *quarter) {
    zo_cfg c = CFG[level];
    unsigned bq = c.chain >> 2;
    for (size_t p = 0; p < n; p++) {
        full[p] = quarter[p] = 0;
        unsigned d0 = link[p];
        if (!d0 || d0 > MAX_DIST) continue;
        size_t limit = p > MAX_DIST ? p - MAX_DIST : 0;
        size_t rem = n - p;
        unsigned nice = c.nice < rem ? c.nice : (unsigned)rem;
        unsigned maxcmp = MAX_MATCH < rem ? MAX_MATCH : (unsigned)rem;
        unsigned best = MIN_MATCH - 1, bestq = 0;
        size_t bpos = 0, bposq = 0;
        size_t cur = p - d0;
        unsigned count = 0;
        int snapped = 0;
        for (;;) {
            count++;
            const uint8_t *m = src + cur;
            int stop = 0;
            if (m[0] == src[p] && m[1] == src[p + 1]) {
                unsigned len = common_prefix(src + p, m, maxcmp);
                if (len > best) { best = len; bpos = cur; if (len >= nice) stop = 1; }
            }
            if (count == bq) { bestq = best; bposq = bpos; snapped = 1; }
            if (stop || count >= c.chain) break;
            unsigned d = link[cur];
            if (!d || cur - d <= limit) break;
            cur -= d;
        }
        if (!snapped) { bestq = best; bposq = bpos; }
        if (best >= MIN_MATCH) full[p] = (best << 16) | (uint32_t)(p - bpos);
        if (bestq >= MIN_MATCH) quarter[p] = (bestq << 16) | (uint32_t)(p - bposq);
    }
}

/* ------------------------------------------------------------------------ */
/* stream assembly (deflate.c:1002-1037,1236-1262; compress.c:22-59)         */
/* ------------------------------------------------------------------------ */
static int assemble(zs_t *s, uint8_t *dst, size_t *dst_len, int wrap) {
    bw_t *w = &s->bw;
    size_t body_start = 0;
    (void)body_start;
    if (w->oom) return ZO_MEM_ERROR;
    /* header and trailer are added around the body bytes */
    uint8_t hdr[10];
    size_t hlen = 0;
    if (wrap == 1) {
        unsigned header = (8u + ((15u - 8u) << 4)) << 8;
        unsigned flags = (s->strategy >= ZO_HUFFMAN_ONLY || s->level < 2) ? 0u  /* deflate.c:1009-1016 */
                         : s->level < 6 ? 1u : s->level == 6 ? 2u : 3u;
        header |= flags << 6;
        header += 31 - (header % 31);
        hdr[0] = (uint8_t)(header >> 8);
        hdr[1] = (uint8_t)header;
        hlen = 2;
    } else if (wrap == 2) {
        static const uint8_t g[10] = {31, 139, 8, 0, 0, 0, 0, 0, 0, 3};
        memcpy(hdr, g, 10);
        hdr[8] = s->level == 9 ? 2 : (s->strategy >= ZO_HUFFMAN_ONLY || s->level < 2) ? 4 : 0;  /* :1052 */
        hlen = 10;
    }
    uint8_t trl[8];
    size_t tlen = 0;
    if (s->open_end) {
    } else if (wrap == 1) {
        uint32_t a = zo_adler32(1, s->in, s->n);
        if (s->n == 0) a = 1;
        trl[0] = (uint8_t)(a >> 24); trl[1] = (uint8_t)(a >> 16);
        trl[2] = (uint8_t)(a >> 8);  trl[3] = (uint8_t)a;
        tlen = 4;
    } else if (wrap == 2) {
        uint32_t c = zo_crc32(0, s->in, s->n);
        uint32_t isz = (uint32_t)s->n;
        for (int i = 0; i < 4; i++) trl[i] = (uint8_t)(c >> (8 * i));
        for (int i = 0; i < 4; i++) trl[4 + i] = (uint8_t)(isz >> (8 * i));
        tlen = 8;
    }
    size_t total = hlen + w->len + tlen, cap = *dst_len, k = 0;
    for (size_t i = 0; i < hlen && k < cap; i++) dst[k++] = hdr[i];
    for (size_t i = 0; i < w->len && k < cap; i++) dst[k++] = w->buf[i];
    for (size_t i = 0; i < tlen && k < cap; i++) dst[k++] = trl[i];
    *dst_len = k;
    return total <= cap ? ZO_OK : ZO_BUF_ERROR;
}

static int compress_events(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                           int level, int wrap, int pp, int strategy, const size_t *fpos,
                           const int *ftype, int nf, int finish);
static int compress_common(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                           int level, int wrap, int pp, int strategy) {
    return compress_events(dst, dst_len, src, n, level, wrap, pp, strategy, NULL, NULL, 0, 1);
}
static int compress_events(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                           int level, int wrap, int pp, int strategy, const size_t *fpos,
                           const int *ftype, int nf, int finish) {
    init_tables();
    if (level == -1) level = 6;
    if (level < 0 || level > 9 || wrap < 0 || wrap > 2 || !dst_len) return ZO_STREAM_ERROR;
    if (strategy < 0 || strategy > ZO_FIXED) return ZO_STREAM_ERROR;
    if (n && !src) return ZO_STREAM_ERROR;
    if (!dst) { *dst_len = 0; return ZO_STREAM_ERROR; }
    zs_t *s = (zs_t *)calloc(1, sizeof(zs_t));
    if (!s) return ZO_MEM_ERROR;
    s->in = src;
    s->n = n;
    s->fpos = fpos;
    s->ftype = ftype;
    s->nf = nf;
    s->fi = 0;
    s->avail = nf ? fpos[0] : n;
    s->open_end = !finish;
    s->level = level;
    s->cfg = CFG[level];
    s->pp = pp;
    s->strategy = strategy;
    int rc = ZO_MEM_ERROR;
    size_t nn = n ? n : 1;
    if (pp) {
        s->link = (uint16_t *)malloc(nn * sizeof(uint16_t));
        s->ins = (uint8_t *)calloc(nn, 1);
        if (!s->link || !s->ins) goto out;
        zo_pp_links(src, n, s->link);
        if (level >= 4) {
            s->rfull = (uint32_t *)malloc(nn * sizeof(uint32_t));
            s->rquart = (uint32_t *)malloc(nn * sizeof(uint32_t));
            if (!s->rfull || !s->rquart) goto out;
            zo_pp_match(src, n, level, s->link, s->rfull, s->rquart);
        }
    } else {
        s->head = (uint32_t *)calloc(32768, sizeof(uint32_t));
        s->prev = (uint32_t *)calloc(nn, sizeof(uint32_t));
        if (!s->head || !s->prev) goto out;
    }
    block_reset(s);
    /* deflate.c:1190-1193 */
    if (level == 0) run_stored(s);
    else if (strategy == ZO_HUFFMAN_ONLY) run_huff(s);
    else if (strategy == ZO_RLE) run_rle(s);
    else if (level <= 3) run_fast(s);
    else run_slow(s);
    rc = assemble(s, dst, dst_len, wrap);
out:
    free(s->head); free(s->prev); free(s->link); free(s->ins);
    free(s->rfull); free(s->rquart); free(s->bw.buf);
    free(s);
    return rc;
}

int zo_compress(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                int level, int wrap) {
    return compress_common(dst, dst_len, src, n, level, wrap, 0, 0);
}

int zo_compress2(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                 int level, int wrap, int strategy) {
    return compress_common(dst, dst_len, src, n, level, wrap, 0, strategy);
}

int zo_pp_compress(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                   int level, int wrap) {
    return compress_common(dst, dst_len, src, n, level, wrap, 1, 0);
}

int zo_pp_compress2(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                    int level, int wrap, int strategy) {
    return compress_common(dst, dst_len, src, n, level, wrap, 1, strategy);
}

/* ------------------------------------------------------------------------ */
/* a18 helpers, zlib-correct                                                 */
/* ------------------------------------------------------------------------ */
void zo_slide_hash(uint16_t *head, uint16_t *prev, uint32_t hash_size, uint32_t window_size,
                   uint32_t wsize) {                          /* deflate.c:187-209 */
    for (uint32_t i = 0; i < hash_size; i++) head[i] = (uint16_t)(head[i] >= wsize ? head[i] - wsize : 0);
    for (uint32_t i = 0; i < window_size; i++) prev[i] = (uint16_t)(prev[i] >= wsize ? prev[i] - wsize : 0);
}

uint32_t zo_compare256(const uint8_t *a, const uint8_t *b) {
    uint32_t k = 0;
    while (k < 256 && a[k] == b[k]) k++;
    return k;
}

/* deflate.c:1356-1497 with UNALIGNED_OK undefined: quick reject on scan_end,
 * scan_end1, scan[0], scan[1]; byte 2 is not compared; bytes 3.. up to
 * MAX_MATCH in the unrolled loop's units (32 groups of 8 end exactly at 258) */
uint32_t zo_longest_match(const uint8_t *window, uint32_t strstart, uint32_t prev_length,
                          uint32_t good, uint32_t chain, uint32_t lookahead, const uint16_t *prev,
                          uint32_t wmask, uint32_t *match_start) {
    const uint32_t wsize = wmask + 1, max_dist = wsize - MIN_LOOKAHEAD;
    const uint8_t *scan = window + strstart;
    uint32_t best = prev_length;
    uint32_t nice = MAX_MATCH < lookahead ? MAX_MATCH : lookahead;
    const uint32_t limit = strstart > max_dist ? strstart - max_dist : 0;
    if (prev_length >= good) chain >>= 2;
    uint32_t cur = prev[strstart & wmask];
    if (!(cur > limit) || chain == 0) return best <= lookahead ? best : lookahead;
    do {
        const uint8_t *m = window + cur;
        if (m[best] != scan[best] || m[best - 1] != scan[best - 1] || m[0] != scan[0] || m[1] != scan[1])
            continue;
        uint32_t len = 3;
        while (len < MAX_MATCH && scan[len] == m[len]) len++;
        if (len > best) {
            *match_start = cur;
            best = len;
            if (len >= nice) break;
        }
    } while ((cur = prev[cur & wmask]) > limit && --chain != 0);
    return best <= lookahead ? best : lookahead;
}

void zo_chunkmemset(uint8_t *dest, const uint8_t *src, uint32_t dist, uint32_t len) {
    for (uint32_t i = 0; i < len; i++) dest[i] = src[i % dist];
}

/* deflate() driven by a sequence of calls (see zoracle.h) */
int zo_deflate_flushes(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n, int level,
                       int wrap, int strategy, const size_t *fpos, const int *ftype, int nf,
                       int finish) {
    if (level == -1) level = 6;
    if (level == 0 && nf) return ZO_STREAM_ERROR;      /* deflate_stored's blocks follow avail_out */
    for (int i = 0; i < nf; i++) {
        if (fpos[i] > n || (i && fpos[i] < fpos[i - 1])) return ZO_STREAM_ERROR;
        if (ftype[i] != 1 && ftype[i] != 2 && ftype[i] != 3 && ftype[i] != 5) return ZO_STREAM_ERROR;
    }
    if (!finish && (nf == 0 || fpos[nf - 1] != n)) return ZO_STREAM_ERROR;
    return compress_events(dst, dst_len, src, n, level, wrap, 0, strategy, fpos, ftype, nf, finish);
}

/* ------------------------------------------------------------------------ */
/* level 0 driven by deflate() calls (deflate.c:763-1265 over deflate_stored, */
/* :1635-1815) with an output buffer that always holds a call's output: the  */
/* first loop of deflate_stored copies stored blocks of up to MAX_STORED     */
/* bytes straight from the window and the input -- a Z_NO_FLUSH call only    */
/* while a block of at least min_block (= w_size, 32768) is available, any   */
/* other call everything; what a Z_NO_FLUSH call leaves (< 32768 bytes) waits */
/* in the window.  Then deflate()'s markers (block_done) and the trailer.     */
/* ------------------------------------------------------------------------ */
static void stored_block(bw_t *w, const uint8_t *a, size_t na, const uint8_t *b, size_t nb, int last) {
    const size_t len = na + nb;                                  /* _tr_stored_block, trees.c:863-876 */
    bw_bits(w, (unsigned)last, 3);
    bw_align(w);
    bw_byte(w, (uint8_t)len);
    bw_byte(w, (uint8_t)(len >> 8));
    bw_byte(w, (uint8_t)~len);
    bw_byte(w, (uint8_t)(~len >> 8));
    for (size_t i = 0; i < na; i++) bw_byte(w, a[i]);
    for (size_t i = 0; i < nb; i++) bw_byte(w, b[i]);
}

int zo_deflate_stored_calls(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n, int wrap,
                            const size_t *take, const int *flush, int ncalls, int *status, size_t *out_len) {
    init_tables();
    if (!dst || !dst_len || wrap < 0 || wrap > 2 || (n && !src)) return ZO_STREAM_ERROR;
    bw_t w = {0};
    /* header (deflate.c:1002-1073): level 0 -> FLEVEL 0 / XFL 4 */
    uint8_t hdr[10];
    size_t hlen = 0;
    if (wrap == 1) {
        unsigned h = (8u + ((15u - 8u) << 4)) << 8;
        h += 31 - (h % 31);
        hdr[0] = (uint8_t)(h >> 8); hdr[1] = (uint8_t)h; hlen = 2;
    } else if (wrap == 2) {
        static const uint8_t g[10] = {31, 139, 8, 0, 0, 0, 0, 0, 4, 3};
        memcpy(hdr, g, 10); hlen = 10;
    }
    size_t pos = 0, buf = 0;            /* input consumed; bytes of it still in the window */
    int last_flush = -2, finished = 0, rc = ZO_OK;
    for (int i = 0; i < ncalls; i++) {
        const int f = flush[i];
        size_t avail = take[i];
        if (pos + avail > n || f < 0 || f > 5) { rc = ZO_STREAM_ERROR; break; }
        int st = ZO_OK;
        const int old = last_flush;
        last_flush = f;
        if (finished && f != 4) st = ZO_STREAM_ERROR;              /* :976-979 */
        else if (avail == 0 && (f * 2 - (f > 4 ? 9 : 0)) <= (old * 2 - (old > 4 ? 9 : 0)) && f != 4)
            st = ZO_BUF_ERROR;                                     /* :1002-1005 */
        else if (finished && avail) st = ZO_BUF_ERROR;
        else if (!finished) {
            size_t total = buf + avail;
            int last = 0;
            const uint8_t *wb = src + pos - buf;                   /* window bytes not yet sent */
            for (;;) {                                             /* :1652-1725 */
                const size_t len = total < MAX_STORED ? total : MAX_STORED;
                if (len < 32768 && ((len == 0 && f != 4) || f == 0)) break;
                last = f == 4 && len == total;
                stored_block(&w, wb, len, NULL, 0, last);
                wb += len;
                total -= len;
                if (last) break;
            }
            pos += avail;
            buf = total;
            if (last) {                                            /* finish_done: trailer */
                finished = 1;
                st = 1;                                            /* Z_STREAM_END */
            } else if (f != 0 && f != 4 && buf == 0) {             /* block_done: :1211-1233 */
                if (f == 1) { bw_bits(&w, 1u << 1, 3); bw_bits(&w, 0, 7); }
                else if (f == 2 || f == 3) {
                    bw_bits(&w, 0, 3); bw_align(&w);
                    bw_byte(&w, 0); bw_byte(&w, 0); bw_byte(&w, 0xff); bw_byte(&w, 0xff);
                }
            }
        } else {
            st = 1;                                                /* repeated Z_FINISH */
        }
        if (status) status[i] = st;
        if (out_len) out_len[i] = hlen + w.len + (finished ? (wrap == 1 ? 4 : wrap == 2 ? 8 : 0) : 0);
    }
    if (rc == ZO_OK && w.oom) rc = ZO_MEM_ERROR;
    if (rc == ZO_OK) {
        uint8_t trl[8];
        size_t tlen = 0;
        if (finished && wrap == 1) {
            const uint32_t a = zo_adler32(1, src, pos);
            trl[0] = (uint8_t)(a >> 24); trl[1] = (uint8_t)(a >> 16); trl[2] = (uint8_t)(a >> 8); trl[3] = (uint8_t)a;
            tlen = 4;
        } else if (finished && wrap == 2) {
            const uint32_t c = zo_crc32(0, src, pos);
            for (int k = 0; k < 4; k++) trl[k] = (uint8_t)(c >> (8 * k));
            for (int k = 0; k < 4; k++) trl[4 + k] = (uint8_t)((uint32_t)pos >> (8 * k));
            tlen = 8;
        }
        size_t k = 0;
        const size_t cap = *dst_len;
        for (size_t j = 0; j < hlen && k < cap; j++) dst[k++] = hdr[j];
        for (size_t j = 0; j < w.len && k < cap; j++) dst[k++] = w.buf[j];
        for (size_t j = 0; j < tlen && k < cap; j++) dst[k++] = trl[j];
        if (hlen + w.len + tlen > cap) rc = ZO_BUF_ERROR;
        *dst_len = k;
    }
    free(w.buf);
    return rc;
}
