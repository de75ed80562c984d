// zgpu_gen.h — the seeded synthetic workloads of the benchmark configs
// (SURVEY §8(d)), as plain functions that compile both for the device
// (zgpu_gen.hip, inputs generated in HBM) and for the host (oracle/zgen.c, so
// the tests can rebuild the exact bytes the benchmark compresses and pin them
// with golden fixtures).  Every 4 KiB chunk is a pure function of
// (kind, seed, buffer index, chunk index).
//
//   kind 0  uniform random bytes                         (C2, CRC-32)
//   kind 1  "Silesia-style" mix, 64 KiB segments:         (C4, level 6)
//           40 % English-like prose, 20 % XML-ish markup, 20 % binary records
//           (12-byte LE structs, slowly varying fields), 10 % random, 10 % runs
//   kind 2  "enwik-style": 4 KiB segments, 70 % text / 30 % markup  (C3, level 1)
//   kind 3  small-vocabulary text (16 words)              (C5, level 9)
//   kind 4  4-letter alphabet "ACGT", i.i.d.              (C5's deepest chains)
//   kind 5  byte runs                                     (C5's high-ratio case)
#ifndef ZGPU_GEN_H
#define ZGPU_GEN_H

#include <stdint.h>

#ifdef __HIPCC__
#define ZG_FN __host__ __device__ inline
#define ZG_CONST __constant__
#else
#define ZG_FN static inline
#define ZG_CONST static const
#endif

#define ZG_CHUNK 4096u
#define ZG_NUM_WORDS 85

// the 85-word list of tests/datagen.py (WORDS)
ZG_CONST char zg_words[] =
    "the\0of\0and\0to\0in\0a\0is\0that\0for\0it\0as\0was\0with\0be\0by\0on\0not\0he\0"
    "this\0are\0or\0his\0from\0at\0which\0but\0have\0an\0they\0you\0were\0her\0she\0"
    "there\0one\0all\0we\0their\0been\0has\0would\0when\0who\0will\0more\0if\0no\0out\0"
    "so\0said\0what\0up\0its\0about\0into\0than\0them\0can\0only\0other\0new\0some\0"
    "could\0time\0these\0two\0may\0then\0do\0first\0any\0my\0now\0such\0like\0"
    "compression\0window\0stream\0buffer\0data\0history\0council\0government\0river\0north\0";

ZG_FN uint64_t zg_splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

typedef struct { uint64_t s; } ZgRng;
ZG_FN uint64_t zg_next(ZgRng *r) {
    r->s ^= r->s << 13;
    r->s ^= r->s >> 7;
    r->s ^= r->s << 17;
    return r->s;
}
ZG_FN uint32_t zg_below(ZgRng *r, uint32_t k) { return (uint32_t)(((zg_next(r) >> 32) * (uint64_t)k) >> 32); }

// byte sink for one chunk of `end` bytes at dst (4-byte aligned): bytes are
// gathered into little-endian words and stored a word at a time
typedef struct {
    uint8_t *dst;
    uint32_t pos, end, acc;
} ZgSink;
ZG_FN int zg_full(const ZgSink *o) { return o->pos >= o->end; }
ZG_FN void zg_put(ZgSink *o, uint32_t b) {
    if (o->pos >= o->end) return;
    o->acc |= (b & 0xffu) << (8 * (o->pos & 3));
    o->pos++;
    if ((o->pos & 3) == 0) {
        uint32_t *w = (uint32_t *)(void *)(o->dst + o->pos - 4);
        *w = o->acc;
        o->acc = 0;
    }
}
ZG_FN void zg_finish(ZgSink *o) {
    const uint32_t r = o->pos & 3;
    for (uint32_t k = 0; k < r; k++) o->dst[o->pos - r + k] = (uint8_t)(o->acc >> (8 * k));
}

ZG_CONST uint16_t zg_word_offs[ZG_NUM_WORDS] = {
    0,4,7,11,14,17,19,22,27,31,34,37,41,46,49,52,55,59,62,67,
    71,74,78,83,86,92,96,101,104,109,113,118,122,126,132,136,140,143,149,154,
    158,164,169,173,178,183,186,189,193,196,201,206,209,213,219,224,229,234,238,243,
    249,253,258,264,269,275,279,283,288,291,297,301,304,308,313,318,330,337,344,351,
    356,364,372,383,389};
ZG_FN void zg_put_word(ZgSink *o, int idx) {
    for (int k = zg_word_offs[idx]; zg_words[k]; k++) zg_put(o, (uint8_t)zg_words[k]);
}

// product of two uniforms: Zipf-like skew towards the first words (datagen.text)
ZG_FN int zg_zipf(ZgRng *r, int vocab) {
    const uint64_t x = zg_next(r);
    const uint64_t a = x & 0xffffu, b = (x >> 16) & 0xffffu;
    return (int)(((a * b) >> 16) * (uint64_t)vocab >> 16);
}

// word text, separators as datagen.text: 5/8 " ", then ", ", ". ", ".\n"
ZG_FN void zg_text(ZgSink *o, ZgRng *r, int vocab) {
    while (!zg_full(o)) {
        zg_put_word(o, zg_zipf(r, vocab));
        const uint32_t s = zg_below(r, 8);
        if (s < 5) zg_put(o, ' ');
        else if (s == 5) { zg_put(o, ','); zg_put(o, ' '); }
        else if (s == 6) { zg_put(o, '.'); zg_put(o, ' '); }
        else { zg_put(o, '.'); zg_put(o, '\n'); }
    }
}

// Silesia-style prose: sentences of 4..15 words, Zipf skew over three
// uniforms, and every ZG_REPEAT-th percent of sentences repeats one of the last
// 16 (names, phrases and boilerplate recur in real corpora).  A sentence is a
// pure function of its seed, so a repeat regenerates it from the seed.
#ifndef ZG_REPEAT
#define ZG_REPEAT 35
#endif
ZG_FN int zg_zipf3(ZgRng *r, int vocab) {
    const uint64_t x = zg_next(r);
    const uint64_t a = x & 0xffffu, b = (x >> 16) & 0xffffu, c = (x >> 32) & 0xffffu;
    return (int)(((((a * b) >> 16) * c) >> 16) * (uint64_t)vocab >> 16);
}
ZG_FN void zg_sentence(ZgSink *o, uint64_t sseed, int vocab) {
    ZgRng r;
    r.s = zg_splitmix(sseed) | 1u;
    const uint32_t n = 4 + zg_below(&r, 12);
    for (uint32_t i = 0; i < n; i++) {
        zg_put_word(o, zg_zipf3(&r, vocab));
        if (i + 1 < n) zg_put(o, ' ');
    }
    const uint32_t e = zg_below(&r, 3);
    zg_put(o, e == 2 ? ',' : '.');
    zg_put(o, e == 1 ? '\n' : ' ');
}
ZG_FN void zg_prose(ZgSink *o, ZgRng *r, int vocab) {
    uint64_t ring[16];
    uint32_t nr = 0;
    while (!zg_full(o)) {
        uint64_t sseed;
        if (nr && zg_below(r, 100) < ZG_REPEAT) {
            sseed = ring[zg_below(r, nr < 16 ? nr : 16)];
        } else {
            sseed = zg_next(r);
            ring[nr++ & 15] = sseed;
        }
        zg_sentence(o, sseed, vocab);
    }
}

ZG_FN void zg_dec(ZgSink *o, uint32_t v) {
    char buf[12];
    int k = 0;
    do { buf[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) zg_put(o, (uint8_t)buf[--k]);
}
ZG_FN void zg_str(ZgSink *o, const char *s) {
    while (*s) zg_put(o, (uint8_t)*s++);
}

// datagen.markup: one <row> per record, uniform word choice, sequential ids
ZG_FN void zg_markup(ZgSink *o, ZgRng *r) {
    uint32_t id = zg_below(r, 1u << 20);
    while (!zg_full(o)) {
        zg_str(o, "<row id=\"");
        zg_dec(o, id++);
        zg_str(o, "\"><name>");
        zg_put_word(o, (int)zg_below(r, ZG_NUM_WORDS));
        zg_put(o, ' ');
        zg_put_word(o, (int)zg_below(r, ZG_NUM_WORDS));
        zg_str(o, "</name><city>");
        zg_put_word(o, (int)zg_below(r, ZG_NUM_WORDS));
        zg_str(o, "</city><value>");
        zg_dec(o, zg_below(r, 100000));
        zg_str(o, "</value></row>\n");
    }
}

// datagen.records' layout: 12-byte LE structs {u32 id++, u32 val += [-16,16],
// u8 type 0..7, 0, u8 flag (5 %: random), 0}
ZG_FN void zg_records(ZgSink *o, ZgRng *r) {
    uint32_t id = (uint32_t)zg_next(r) & 0x7fffffffu, val = (uint32_t)zg_next(r) & 0xffffffu;
    while (!zg_full(o)) {
        for (int k = 0; k < 4; k++) zg_put(o, id >> (8 * k));
        for (int k = 0; k < 4; k++) zg_put(o, val >> (8 * k));
        const uint32_t ty = zg_below(r, 8), fl = zg_below(r, 20) == 0 ? zg_below(r, 256) : 0;
        zg_put(o, ty); zg_put(o, 0); zg_put(o, fl); zg_put(o, 0);
        id++;
        val += zg_below(r, 33) - 16;
    }
}

ZG_FN void zg_random(ZgSink *o, ZgRng *r) {
    while (!zg_full(o)) {
        const uint64_t x = zg_next(r);
        for (int k = 0; k < 8; k++) zg_put(o, (uint32_t)(x >> (8 * k)));
    }
}

// datagen.runs: random byte values, 15 % long runs (64..511), else 1..47
ZG_FN void zg_runs(ZgSink *o, ZgRng *r) {
    while (!zg_full(o)) {
        const uint32_t b = zg_below(r, 256);
        const uint32_t len = zg_below(r, 100) < 15 ? 64 + zg_below(r, 448) : 1 + zg_below(r, 47);
        for (uint32_t k = 0; k < len && !zg_full(o); k++) zg_put(o, b);
    }
}

ZG_FN void zg_four(ZgSink *o, ZgRng *r) {
    while (!zg_full(o)) {
        const uint64_t x = zg_next(r);
        for (int k = 0; k < 32; k++) zg_put(o, (uint8_t)"ACGT"[(x >> (2 * k)) & 3]);
    }
}

// Chunk c (ZG_CHUNK bytes) of buffer gidx of a batch of `len`-byte buffers.
ZG_FN void zg_chunk(uint8_t *dst, uint64_t len, int kind, uint64_t seed, uint64_t gidx, uint64_t c) {
    const uint64_t bseed = zg_splitmix(seed ^ zg_splitmix(gidx * 0x9e3779b97f4a7c15ull + (uint64_t)kind));
    const uint64_t at = c * ZG_CHUNK;
    ZgSink o;
    o.dst = dst;
    o.pos = 0;
    o.acc = 0;
    o.end = (uint32_t)((len - at) < ZG_CHUNK ? (len - at) : ZG_CHUNK);
    int sk;
    switch (kind) {
    case 0: sk = 3; break;
    case 1: {
        const uint64_t seg = at >> 16;
        const uint32_t u = (uint32_t)(zg_splitmix(bseed ^ (0x5e6e0000ull + seg)) % 10);
        sk = u < 4 ? 0 : u < 6 ? 1 : u < 8 ? 2 : u < 9 ? 3 : 4;
        break;
    }
    case 2: {
        const uint32_t u = (uint32_t)(zg_splitmix(bseed ^ (0xe1417000ull + c)) % 10);
        sk = u < 7 ? 0 : 1;
        break;
    }
    case 3: sk = 5; break;
    case 4: sk = 6; break;
    default: sk = 7; break;
    }
    ZgRng r;
    r.s = zg_splitmix(bseed + c * 0xd1b54a32d192ed03ull) | 1u;
    switch (sk) {
    case 0: if (kind == 1) zg_prose(&o, &r, ZG_NUM_WORDS); else zg_text(&o, &r, ZG_NUM_WORDS); break;
    case 1: zg_markup(&o, &r); break;
    case 2: zg_records(&o, &r); break;
    case 3: zg_random(&o, &r); break;
    case 4: zg_runs(&o, &r); break;
    case 5: zg_text(&o, &r, 16); break;
    case 6: zg_four(&o, &r); break;
    default: zg_runs(&o, &r); break;
    }
    zg_finish(&o);
}

#endif  // ZGPU_GEN_H
