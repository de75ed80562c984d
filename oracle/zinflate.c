/*
 * zinflate.c — TEST INFRASTRUCTURE ONLY (never linked into the product path).
 *
 * Plain-C restatement of the reference's decompression path (discere-os/zlib.wasm
 * @ zlib 1.3.1.1-motley): inflate()'s state machine (inflate.c:622-1221), the
 * code-set rules of inflate_table (inftrees.c:100-134,297-301) and uncompress2's
 * result mapping (uncompr.c:24-85).  It is the checker for the GPU inflate.
 *
 * The machine follows inflate()'s slow path bit for bit: NEEDBITS pulls whole
 * bytes only until the bits in hand cover what the next step needs, and codes
 * are decoded canonically with the same minimal pulls as inflate's table loop
 * ("pull until here.bits <= bits" ends exactly when the true code length is in
 * hand).  inflate_fast (inffast.c) decodes the same symbols and reports the
 * same errors; on return it gives back whole unused bytes, so the bytes it has
 * consumed at any stop are the slow path's too.  The number of input bytes
 * consumed at a stop is therefore what uncompress2 reports in *sourceLen.
 *
 * Parity is pinned against the compiled reference by tests/test_oracle.py
 * (container) and by tests/golden/inflate_golden.json (everywhere).
 */
#include <string.h>
#include "zoracle.h"

enum { ZI_END = 0, ZI_DATA = 1, ZI_DICT = 2, ZI_OUTFULL = 3, ZI_INEND = 4 };

typedef struct {
    const uint8_t *in;
    size_t n, pos;          /* pos: bytes pulled (consumed) */
    uint64_t hold;
    unsigned bits;
    uint8_t *out;
    size_t cap, put;
} zi_t;

/* NEEDBITS (inflate.c:497-501): 1 when k bits are in hand, 0 when input ran out */
static int need(zi_t *s, unsigned k) {
    while (s->bits < k) {
        if (s->pos >= s->n) return 0;
        s->hold |= (uint64_t)s->in[s->pos++] << s->bits;
        s->bits += 8;
    }
    return 1;
}
static unsigned bitsv(zi_t *s, unsigned k) { return (unsigned)(s->hold & ((1ull << k) - 1)); }
static void drop(zi_t *s, unsigned k) { s->hold >>= k; s->bits -= k; }
static void initbits(zi_t *s) { s->hold = 0; s->bits = 0; }
static void bytebits(zi_t *s) { drop(s, s->bits & 7); }

/* a canonical code (RFC 1951 3.2.2) with inflate_table's acceptance rules */
typedef struct {
    uint16_t count[16];
    uint16_t sym[320];
    int max;            /* longest length, 0: no symbols */
    int incomplete;     /* only legal as a single 1-bit code (inftrees.c:132) */
} zcode_t;

enum { T_CODES, T_LENS, T_DISTS };

/* inftrees.c:100-134: 0 ok, -1 over-subscribed or incomplete where not allowed */
static int build(zcode_t *c, const uint16_t *lens, int n, int type) {
    uint16_t offs[16];
    memset(c->count, 0, sizeof c->count);
    for (int i = 0; i < n; i++) c->count[lens[i]]++;
    c->max = 0;
    for (int l = 15; l >= 1; l--)
        if (c->count[l]) { c->max = l; break; }
    c->incomplete = 0;
    if (c->max == 0) return 0;                       /* decodes as invalid, 1 bit */
    int left = 1;
    for (int l = 1; l <= 15; l++) {
        left <<= 1;
        left -= c->count[l];
        if (left < 0) return -1;
    }
    if (left > 0 && (type == T_CODES || c->max != 1)) return -1;
    c->incomplete = left > 0;
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + c->count[l];
    for (int i = 0; i < n; i++)
        if (lens[i]) c->sym[offs[lens[i]]++] = (uint16_t)i;
    return 0;
}

/* one code: 1 and *sym, 0 input ran out, -1 an invalid entry (1 bit dropped;
 * the code-length code with no symbols yields symbol 0 the same way,
 * inflate.c:940-948 never looks at op) */
static int decode(zi_t *s, const zcode_t *c, int *sym) {
    if (c->max == 0 || c->incomplete) {
        if (!need(s, 1)) return 0;
        if (c->max == 0 || (s->hold & 1)) { drop(s, 1); *sym = 0; return -1; }
        drop(s, 1);
        *sym = c->sym[0];
        return 1;
    }
    unsigned code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; len++) {
        if (!need(s, (unsigned)len)) return 0;
        code |= (unsigned)(s->hold >> (len - 1)) & 1u;
        const unsigned cnt = c->count[len];
        if (code - first < cnt) {
            drop(s, (unsigned)len);
            *sym = c->sym[index + (code - first)];
            return 1;
        }
        index += cnt;
        first = (first + cnt) << 1;
        code <<= 1;
    }
    return -1;   /* unreachable for accepted codes */
}

static const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                      3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257,
                                       385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193,
                                       12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8,
                                       9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

/* the gzip header (inflate.c:629-637,671-807); returns ZI_* or -1 to go on */
static int gzip_header(zi_t *s) {
    uint8_t hb[4];
    uint32_t check;
    hb[0] = 0x1f; hb[1] = 0x8b;
    check = zo_crc32(0, hb, 2);
    initbits(s);
    if (!need(s, 16)) return ZI_INEND;                               /* FLAGS */
    const unsigned flags = bitsv(s, 16);
    if ((flags & 0xff) != 8) return ZI_DATA;                         /* unknown compression method */
    if (flags & 0xe000) return ZI_DATA;                              /* unknown header flags set */
    const int hcrc = (flags & 0x0200) != 0;
    if (hcrc) { hb[0] = flags & 0xff; hb[1] = flags >> 8; check = zo_crc32(check, hb, 2); }
    initbits(s);
    if (!need(s, 32)) return ZI_INEND;                               /* TIME */
    if (hcrc) { for (int k = 0; k < 4; k++) hb[k] = (uint8_t)(s->hold >> (8 * k)); check = zo_crc32(check, hb, 4); }
    initbits(s);
    if (!need(s, 16)) return ZI_INEND;                               /* OS */
    if (hcrc) { hb[0] = s->hold & 0xff; hb[1] = (s->hold >> 8) & 0xff; check = zo_crc32(check, hb, 2); }
    initbits(s);
    if (flags & 0x0400) {                                            /* EXLEN, EXTRA */
        if (!need(s, 16)) return ZI_INEND;
        const unsigned xlen = bitsv(s, 16);
        if (hcrc) { hb[0] = xlen & 0xff; hb[1] = xlen >> 8; check = zo_crc32(check, hb, 2); }
        initbits(s);
        size_t copy = xlen;
        if (copy > s->n - s->pos) copy = s->n - s->pos;
        if (hcrc) check = zo_crc32(check, s->in + s->pos, copy);
        s->pos += copy;
        if (copy < xlen) return ZI_INEND;
    }
    for (unsigned f = 0x0800; f <= 0x1000; f <<= 1) {                 /* NAME, COMMENT */
        if (!(flags & f)) continue;
        if (s->pos >= s->n) return ZI_INEND;
        size_t copy = 0;
        unsigned c;
        do c = s->in[s->pos + copy++]; while (c && s->pos + copy < s->n);
        if (hcrc) check = zo_crc32(check, s->in + s->pos, copy);
        s->pos += copy;
        if (c) return ZI_INEND;
    }
    if (hcrc) {                                                      /* HCRC */
        if (!need(s, 16)) return ZI_INEND;
        if (bitsv(s, 16) != (check & 0xffff)) return ZI_DATA;        /* header crc mismatch */
        initbits(s);
    }
    return -1;
}

/* inflate.c:622-1221 run to a stop; wrap: 0 raw, 1 zlib, 2 gzip, 3 zlib or gzip */
static int run(zi_t *s, int wrap) {
    int gz = 0;
    if (wrap) {                                                      /* HEAD */
        if (!need(s, 16)) return ZI_INEND;
        if ((wrap & 2) && bitsv(s, 16) == 0x8b1f) {
            const int r = gzip_header(s);
            if (r >= 0) return r;
            gz = 1;
        } else {
            if (!(wrap & 1) || ((bitsv(s, 8) << 8) + ((s->hold >> 8) & 0xff)) % 31) return ZI_DATA;
            if (bitsv(s, 4) != 8) return ZI_DATA;                    /* unknown compression method */
            drop(s, 4);
            if (bitsv(s, 4) + 8 > 15) return ZI_DATA;                /* invalid window size */
            const int fdict = (s->hold & 0x200) != 0;
            initbits(s);
            if (fdict) {                                             /* DICTID, DICT */
                if (!need(s, 32)) return ZI_INEND;
                initbits(s);
                return ZI_DICT;
            }
        }
    }
    uint16_t lens[320];
    zcode_t lc, dc;
    for (;;) {                                                       /* TYPEDO */
        if (!need(s, 3)) return ZI_INEND;
        const int last = bitsv(s, 1);
        drop(s, 1);
        const unsigned type = bitsv(s, 2);
        drop(s, 2);
        if (type == 3) return ZI_DATA;                               /* invalid block type */
        if (type == 0) {                                             /* STORED, COPY */
            bytebits(s);
            if (!need(s, 32)) return ZI_INEND;
            if ((s->hold & 0xffff) != (((s->hold >> 16) & 0xffff) ^ 0xffff)) return ZI_DATA;
            size_t len = s->hold & 0xffff;
            initbits(s);
            while (len) {
                size_t copy = len;
                if (copy > s->n - s->pos) copy = s->n - s->pos;
                if (copy > s->cap - s->put) copy = s->cap - s->put;
                if (copy == 0) return s->put == s->cap ? ZI_OUTFULL : ZI_INEND;
                memcpy(s->out + s->put, s->in + s->pos, copy);
                s->put += copy;
                s->pos += copy;
                len -= copy;
            }
        } else {
            if (type == 1) {                                         /* fixedtables, inflate.c:255-285 */
                int i = 0;
                while (i < 144) lens[i++] = 8;
                while (i < 256) lens[i++] = 9;
                while (i < 280) lens[i++] = 7;
                while (i < 288) lens[i++] = 8;
                build(&lc, lens, 288, T_LENS);
                for (i = 0; i < 32; i++) lens[i] = 5;
                build(&dc, lens, 32, T_DISTS);
            } else {                                                 /* TABLE, LENLENS, CODELENS */
                if (!need(s, 14)) return ZI_INEND;
                const int nlen = (int)bitsv(s, 5) + 257; drop(s, 5);
                const int ndist = (int)bitsv(s, 5) + 1; drop(s, 5);
                const int ncode = (int)bitsv(s, 4) + 4; drop(s, 4);
                if (nlen > 286 || ndist > 30) return ZI_DATA;        /* too many length or distance symbols */
                int have = 0;
                while (have < ncode) {
                    if (!need(s, 3)) return ZI_INEND;
                    lens[kOrder[have++]] = (uint16_t)bitsv(s, 3);
                    drop(s, 3);
                }
                while (have < 19) lens[kOrder[have++]] = 0;
                zcode_t cc;
                if (build(&cc, lens, 19, T_CODES)) return ZI_DATA;   /* invalid code lengths set */
                have = 0;
                while (have < nlen + ndist) {
                    int sym;
                    const int r = decode(s, &cc, &sym);
                    if (r == 0) return ZI_INEND;
                    if (sym < 16) { lens[have++] = (uint16_t)sym; continue; }
                    unsigned len, copy;
                    if (sym == 16) {
                        if (!need(s, 2)) return ZI_INEND;
                        if (have == 0) return ZI_DATA;               /* invalid bit length repeat */
                        len = lens[have - 1];
                        copy = 3 + bitsv(s, 2); drop(s, 2);
                    } else if (sym == 17) {
                        if (!need(s, 3)) return ZI_INEND;
                        len = 0;
                        copy = 3 + bitsv(s, 3); drop(s, 3);
                    } else {
                        if (!need(s, 7)) return ZI_INEND;
                        len = 0;
                        copy = 11 + bitsv(s, 7); drop(s, 7);
                    }
                    if (have + (int)copy > nlen + ndist) return ZI_DATA;
                    while (copy--) lens[have++] = (uint16_t)len;
                }
                if (lens[256] == 0) return ZI_DATA;                  /* missing end-of-block */
                if (build(&lc, lens, nlen, T_LENS)) return ZI_DATA;  /* invalid literal/lengths set */
                if (build(&dc, lens + nlen, ndist, T_DISTS)) return ZI_DATA;   /* invalid distances set */
            }
            for (;;) {                                               /* LEN .. MATCH / LIT */
                int sym;
                int r = decode(s, &lc, &sym);
                if (r == 0) return ZI_INEND;
                if (r < 0) return ZI_DATA;                           /* invalid literal/length code */
                if (sym < 256) {
                    if (s->put == s->cap) return ZI_OUTFULL;
                    s->out[s->put++] = (uint8_t)sym;
                    continue;
                }
                if (sym == 256) break;
                if (sym > 285) return ZI_DATA;                       /* fixed codes 286/287 */
                sym -= 257;
                if (!need(s, kLenExtra[sym])) return ZI_INEND;
                const unsigned len = kLenBase[sym] + bitsv(s, kLenExtra[sym]);
                drop(s, kLenExtra[sym]);
                int ds;
                r = decode(s, &dc, &ds);
                if (r == 0) return ZI_INEND;
                if (r < 0 || ds > 29) return ZI_DATA;                /* invalid distance code */
                if (!need(s, kDistExtra[ds])) return ZI_INEND;
                const size_t dist = kDistBase[ds] + bitsv(s, kDistExtra[ds]);
                drop(s, kDistExtra[ds]);
                if (s->put == s->cap) return ZI_OUTFULL;             /* MATCH: room first */
                if (dist > s->put) return ZI_DATA;                   /* invalid distance too far back */
                size_t copy = len;
                if (copy > s->cap - s->put) copy = s->cap - s->put;
                for (size_t k = 0; k < copy; k++) s->out[s->put + k] = s->out[s->put + k - dist];
                s->put += copy;
                if (copy < len) return ZI_OUTFULL;
            }
        }
        if (last) break;
    }
    bytebits(s);                                                     /* CHECK, LENGTH */
    if (wrap && !gz) {
        if (!need(s, 32)) return ZI_INEND;
        const uint32_t h = (uint32_t)s->hold;
        const uint32_t want = (h >> 24) | ((h >> 8) & 0xff00) | ((h << 8) & 0xff0000) | (h << 24);
        if (want != zo_adler32(1, s->out, s->put)) return ZI_DATA;   /* incorrect data check */
        initbits(s);
    } else if (gz) {
        if (!need(s, 32)) return ZI_INEND;
        if ((uint32_t)s->hold != zo_crc32(0, s->out, s->put)) return ZI_DATA;
        initbits(s);
        if (!need(s, 32)) return ZI_INEND;
        if ((uint32_t)s->hold != (uint32_t)s->put) return ZI_DATA;   /* incorrect length check */
        initbits(s);
    }
    return ZI_END;
}

int zo_inflate_run(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, int wrap,
                   size_t *out_len, size_t *consumed) {
    zi_t s;
    memset(&s, 0, sizeof s);
    s.in = src; s.n = n; s.out = dst; s.cap = cap;
    const int r = run(&s, wrap);
    *out_len = s.put;
    *consumed = s.pos;
    return r;
}

/* uncompr.c:24-85 over any wrapper: status as uncompress2 returns it */
int zo_uncompress3(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t *src_len, int wrap) {
    uint8_t buf[1];
    size_t cap = *dst_len, put, pos;
    const int usebuf = cap == 0;
    if (usebuf) { dst = buf; cap = 1; }
    const int r = zo_inflate_run(src, *src_len, dst, cap, wrap, &put, &pos);
    *src_len = pos;
    if (!usebuf) *dst_len = put;
    if (r == ZI_END) return ZO_OK;
    if (r == ZI_DATA || r == ZI_DICT) return ZO_DATA_ERROR;
    /* inflate ends with Z_BUF_ERROR: data error unless the output is full
     * (with the 1-byte probe buffer any output counts as room left) */
    if (usebuf) return ZO_DATA_ERROR;
    return put < cap ? ZO_DATA_ERROR : ZO_BUF_ERROR;
}

int zo_uncompress2(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t *src_len) {
    return zo_uncompress3(dst, dst_len, src, src_len, 1);
}
