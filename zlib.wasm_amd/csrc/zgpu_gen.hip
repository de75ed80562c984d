// zgpu_gen.hip — seeded synthetic workloads, generated in HBM (DESIGN.md
// §Workloads).  Inputs of the benchmark configs are far too large to stage over
// PCIe inside a timed loop, so they are produced on the device.  Every 4 KiB
// chunk is a pure function of (kind, seed, buffer index, chunk index) and is
// written by one thread, so generation is embarrassingly parallel.
//
//   kind 0  uniform random bytes                         (C2, CRC-32)
//   kind 1  "Silesia-style" mix, 64 KiB segments:         (C4, level 6)
//           40 % English-like text, 20 % XML-ish markup, 20 % binary records
//           (12-byte LE structs, slowly varying fields), 10 % random, 10 % runs
//   kind 2  "enwik-style": 4 KiB segments, 70 % text / 30 % markup  (C3, level 1)
//   kind 3  small-vocabulary text (16 words)              (C5, level 9)
#include "zgpu_internal.h"

namespace zgpu {

__constant__ char c_words[] =
    "the\0of\0and\0to\0in\0a\0is\0that\0for\0it\0as\0was\0with\0be\0by\0on\0not\0he\0"
    "this\0are\0or\0his\0from\0at\0which\0but\0have\0an\0they\0you\0were\0her\0she\0"
    "there\0one\0all\0we\0their\0been\0has\0would\0when\0who\0will\0more\0if\0no\0out\0"
    "so\0said\0what\0up\0its\0about\0into\0than\0them\0can\0only\0other\0new\0some\0"
    "could\0time\0these\0two\0may\0then\0do\0first\0any\0my\0now\0such\0like\0our\0"
    "over\0man\0me\0even\0most\0made\0after\0also\0did\0many\0before\0must\0through\0"
    "back\0years\0where\0much\0your\0way\0well\0down\0should\0because\0each\0just\0"
    "those\0people\0how\0too\0little\0state\0good\0very\0make\0world\0still\0own\0see\0"
    "men\0work\0long\0get\0here\0between\0both\0life\0being\0under\0never\0day\0same\0"
    "another\0know\0while\0last\0might\0us\0great\0old\0year\0off\0come\0since\0against\0"
    "go\0came\0right\0used\0take\0three\0compression\0window\0stream\0buffer\0data\0"
    "history\0council\0government\0river\0north\0system\0number\0city\0music\0record\0";
constexpr int kNumWords = 150;

__device__ inline uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

struct Rng {
    uint64_t s;
    __device__ inline uint64_t next() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
    __device__ inline uint32_t below(uint32_t k) { return (uint32_t)(((next() >> 32) * (uint64_t)k) >> 32); }
};

// byte sink writing a [lo, hi) window of a chunk with dword stores
struct Sink {
    uint8_t *dst;      // chunk base
    uint32_t pos, end; // current byte, chunk length
    uint32_t acc;
    __device__ inline bool full() const { return pos >= end; }
    __device__ inline void put(uint32_t b) {
        if (pos >= end) return;
        acc |= (b & 0xffu) << (8 * (pos & 3));
        pos++;
        if ((pos & 3) == 0) { *reinterpret_cast<uint32_t *>(dst + pos - 4) = acc; acc = 0; }
    }
    __device__ inline void finish() {
        const uint32_t r = pos & 3;
        for (uint32_t k = 0; k < r; k++) dst[pos - r + k] = (uint8_t)(acc >> (8 * k));
    }
};

__device__ inline const char *word_at(int idx) {
    const char *p = c_words;
    // word table is tiny; walk it (constant cache)
    for (int i = 0; i < idx; i++) { while (*p) p++; p++; }
    return p;
}

__device__ inline int zipf_index(Rng &r, int vocab) {
    const uint64_t x = r.next();
    const uint64_t a = x & 0xffffu, b = (x >> 16) & 0xffffu;   // product of two uniforms: skewed
    return (int)(((a * b) >> 16) * (uint64_t)vocab >> 16);
}

__device__ void gen_text(Sink &o, Rng &r, int vocab) {
    bool cap = true;
    while (!o.full()) {
        const char *w = word_at(zipf_index(r, vocab));
        bool first = true;
        for (; *w; w++) {
            uint32_t c = (uint8_t)*w;
            if (first && cap) c -= 32;
            first = false;
            o.put(c);
        }
        cap = false;
        const uint32_t s = r.below(100);
        if (s < 80) o.put(' ');
        else if (s < 88) { o.put(','); o.put(' '); }
        else if (s < 95) { o.put('.'); o.put(' '); cap = true; }
        else { o.put('.'); o.put('\n'); cap = true; }
    }
}

__device__ void put_dec(Sink &o, uint32_t v) {
    char buf[12];
    int k = 0;
    do { buf[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) o.put((uint8_t)buf[--k]);
}
__device__ void put_str(Sink &o, const char *s) { while (*s) o.put((uint8_t)*s++); }

__device__ void gen_markup(Sink &o, Rng &r, int vocab) {
    uint32_t id = (uint32_t)(r.next() & 0xfffff);
    while (!o.full()) {
        put_str(o, "<row id=\"");
        put_dec(o, id++);
        put_str(o, "\"><name>");
        put_str(o, word_at(zipf_index(r, vocab)));
        o.put(' ');
        put_str(o, word_at(zipf_index(r, vocab)));
        put_str(o, "</name><city>");
        put_str(o, word_at(zipf_index(r, vocab)));
        put_str(o, "</city><value>");
        put_dec(o, r.below(100000));
        put_str(o, "</value></row>\n");
    }
}

__device__ void gen_records(Sink &o, Rng &r) {
    uint32_t id = (uint32_t)r.next(), val = (uint32_t)r.next() & 0xffffff;
    while (!o.full()) {
        for (int k = 0; k < 4; k++) o.put(id >> (8 * k));
        for (int k = 0; k < 4; k++) o.put(val >> (8 * k));
        const uint32_t ty = r.below(8), fl = r.below(4) == 0 ? r.below(256) : 0;
        o.put(ty); o.put(0); o.put(fl); o.put(0);
        id++;
        val += r.below(33) - 16;
    }
}

__device__ void gen_random(Sink &o, Rng &r) {
    while (!o.full()) {
        uint64_t x = r.next();
        for (int k = 0; k < 8; k++) o.put((uint32_t)(x >> (8 * k)));
    }
}

__device__ void gen_runs(Sink &o, Rng &r) {
    while (!o.full()) {
        const uint32_t b = r.below(4) == 0 ? 0u : r.below(256);
        const uint32_t len = r.below(8) == 0 ? 64 + r.below(448) : 1 + r.below(48);
        for (uint32_t k = 0; k < len && !o.full(); k++) o.put(b);
    }
}

constexpr uint32_t kChunk = 4096;

__global__ void k_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed,
                           uint64_t first_index) {
    const uint64_t chunks_per = (len + kChunk - 1) / kChunk;
    const uint64_t total = chunks_per * count;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = t / chunks_per, c = t % chunks_per;
        const uint64_t gidx = first_index + b;
        const uint64_t bseed = splitmix(seed ^ splitmix(gidx * 0x9e3779b97f4a7c15ull + (uint64_t)kind));
        Rng r;
        r.s = splitmix(bseed + c * 0xd1b54a32d192ed03ull) | 1u;
        Sink o;
        o.dst = dst + b * len + c * kChunk;
        o.pos = 0;
        o.end = (uint32_t)((len - c * kChunk) < kChunk ? (len - c * kChunk) : kChunk);
        o.acc = 0;
        int sk;
        switch (kind) {
        case 0: sk = 3; break;
        case 1: {
            const uint32_t seg = (uint32_t)((c * kChunk) >> 16);
            const uint32_t u = (uint32_t)(splitmix(bseed ^ (0x5e6e0000ull + seg)) % 10);
            sk = u < 4 ? 0 : u < 6 ? 1 : u < 8 ? 2 : u < 9 ? 3 : 4;
            break;
        }
        case 2: {
            const uint32_t u = (uint32_t)(splitmix(bseed ^ (0xe1417000ull + c)) % 10);
            sk = u < 7 ? 0 : 1;
            break;
        }
        default: sk = 5; break;
        }
        switch (sk) {
        case 0: gen_text(o, r, kNumWords); break;
        case 1: gen_markup(o, r, kNumWords); break;
        case 2: gen_records(o, r); break;
        case 3: gen_random(o, r); break;
        case 4: gen_runs(o, r); break;
        default: gen_text(o, r, 16); break;
        }
        o.finish();
    }
}

int launch_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed,
                    uint64_t first_index, hipStream_t st) {
    if (count == 0 || len == 0) return 0;
    if ((len & 3) || (reinterpret_cast<uintptr_t>(dst) & 3)) return (int)hipErrorInvalidValue;
    const uint64_t total = ((len + kChunk - 1) / kChunk) * count;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 65535) blocks = 65535;
    hipLaunchKernelGGL(k_generate, dim3((uint32_t)blocks), dim3(256), 0, st, dst, len, count, kind,
                       seed, first_index);
    return (int)hipGetLastError();
}

}  // namespace zgpu
