// zgpu_inflate.hip — batched inflate for gfx950: output, status and bytes
// consumed identical to the reference's uncompress2 (uncompr.c:24-85) over
// inflate() (inflate.c:622-1221) on every stream, valid or not.
//
// Per sub-batch of independent streams:
//   k_inflate_decode  wave/stream  the inflate state machine: headers, block
//                                  headers, code tables (built in LDS by all 64
//                                  lanes), symbol decode.  Decoder state is
//                                  wave-uniform (every lane computes the same,
//                                  LDS reads are broadcasts made scalar with
//                                  readfirstlane), so staging the input, building
//                                  tables and flushing output use the whole wave
//                                  without divergence.  Literals and stored bytes
//                                  go to the output; each match becomes a record
//                                  (pos, len, dist) in HBM.
//   k_inflate_copy    wave/stream  resolves the matches in order through a 40 KiB
//                                  LDS window (32 KiB history + a 4 KiB output
//                                  chunk + one match of overhang), one lane per
//                                  byte of a match.
//   checksums                      k_adler32 / k_crc32 over the output (trailer)
//   k_inflate_finish  thread/stream  trailer checks and uncompress2's status map.
#include "zgpu_internal.h"

namespace zgpu {

constexpr int kIRing = 2048;          // staged input bytes
constexpr int kOBuf = 1024;           // staged literal bytes
constexpr int kMBuf = 64;             // staged match records
constexpr int kLRoot = 10, kDRoot = 8, kCRoot = 7;
constexpr uint32_t kSymBad = 0x1ff;   // table entry symbol of an invalid code (1 bit)
constexpr uint32_t kLong = 0x8000;    // table entry flag: code longer than the root
constexpr uint32_t kBadEntry = kSymBad | (1u << 9);

struct Canon {                        // canonical decode of codes longer than the root
    uint16_t count[16], first[16], offs[16];
    uint16_t sorted[288];
};

struct InfLDS {
    union { uint8_t b[kIRing + 16]; uint32_t w[(kIRing + 16) / 4]; } ring;
    uint8_t obuf[kOBuf];
    uint64_t mbuf[kMBuf];
    uint16_t lt[1 << kLRoot], dt[1 << kDRoot], ct[1 << kCRoot];
    Canon lcan, dcan;
    uint16_t lens[320];
    uint32_t cu[48];                  // codes_used's count / next code / codes left per length
};

__device__ __constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                                 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__device__ __constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                               3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__device__ __constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                                 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
                                                 4097, 6145, 8193, 12289, 16385, 24577};
__device__ __constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7,
                                               8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__device__ __constant__ uint8_t c_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __attribute__((always_inline)) inline uint32_t uni(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __attribute__((always_inline)) inline uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

enum { kCodes = 0, kLens = 1, kDists = 2 };

// inflate_table's acceptance rules (inftrees.c:100-134,297-301) and a decode
// table: root entries sym | len << 9 for codes up to `root` bits, kLong at the
// root prefix of longer codes (canonical decode from `can`), kBadEntry where no
// code lands (an empty or a single-1-bit code).  Wave-uniform; returns false on
// an over-subscribed or forbidden incomplete set.
template <int kRoot>
__device__ bool build_code(const uint16_t *lens, int n, int type, uint16_t *T, Canon *can, int lane) {
    uint32_t cnt[16];
#pragma unroll
    for (int l = 0; l < 16; l++) cnt[l] = 0;
    for (int c = 0; c < n; c += 64) {
        const int s = c + lane;
        const uint32_t l = s < n ? lens[s] : 0u;
#pragma unroll
        for (int lv = 1; lv <= 15; lv++) cnt[lv] += (uint32_t)__builtin_popcountll(__ballot(l == (uint32_t)lv));
    }
    int max = 0;
#pragma unroll
    for (int lv = 1; lv <= 15; lv++)
        if (cnt[lv]) max = lv;
    for (int e = lane; e < (1 << kRoot); e += 64) T[e] = (uint16_t)kBadEntry;
    if (max == 0) { __syncthreads(); return true; }
    int left = 1;
#pragma unroll
    for (int lv = 1; lv <= 15; lv++) {
        left = 2 * left - (int)cnt[lv];
        if (left < 0) return false;                  // over-subscribed (uniform)
    }
    if (left > 0 && (type == kCodes || max != 1)) return false;
    uint32_t first[16], offs[16];
    {
        uint32_t code = 0, off = 0;
        first[0] = 0; offs[0] = 0;
#pragma unroll
        for (int lv = 1; lv <= 15; lv++) {
            code = (code + cnt[lv - 1]) << 1;
            first[lv] = code;
            offs[lv] = off;
            off += cnt[lv];
        }
    }
    const bool longs = max > kRoot;
    if (longs && lane < 16) {
        uint32_t f = 0, o = 0, k = 0;
#pragma unroll
        for (int lv = 0; lv < 16; lv++)
            if (lane == lv) { f = first[lv]; o = offs[lv]; k = cnt[lv]; }
        can->first[lane] = (uint16_t)f;
        can->offs[lane] = (uint16_t)o;
        can->count[lane] = (uint16_t)k;
    }
    __syncthreads();
    uint32_t rc[16];
#pragma unroll
    for (int l = 0; l < 16; l++) rc[l] = 0;
    for (int c = 0; c < n; c += 64) {
        const int s = c + lane;
        const uint32_t l = s < n ? lens[s] : 0u;
        uint32_t code = 0, off = 0;
#pragma unroll
        for (int lv = 1; lv <= 15; lv++) {
            const uint64_t m = __ballot(l == (uint32_t)lv);
            if (l == (uint32_t)lv) {
                const uint32_t rank = rc[lv] + lanes_below(m);
                code = first[lv] + rank;
                off = offs[lv] + rank;
            }
            rc[lv] += (uint32_t)__builtin_popcountll(m);
        }
        if (l) {
            const uint32_t rev = __brev(code) >> (32 - l);
            if (longs) can->sorted[off] = (uint16_t)s;
            if (l <= (uint32_t)kRoot) {
                for (uint32_t e = rev; e < (1u << kRoot); e += 1u << l) T[e] = (uint16_t)(s | (l << 9));
            } else {
                T[rev & ((1u << kRoot) - 1)] = (uint16_t)kLong;
            }
        }
    }
    __syncthreads();
    return true;
}

// one code from `hold` (>= 15 bits in hand or zero padded); returns the symbol
// (kSymBad for an invalid code) and its length
template <int kRoot>
__device__ __attribute__((always_inline)) inline uint32_t dec_code(const uint16_t *T, const Canon *can,
                                                                   uint64_t hold, uint32_t &len) {
    const uint32_t e = uni(T[(uint32_t)hold & ((1u << kRoot) - 1)]);
    if (!(e & kLong)) { len = (e >> 9) & 15u; return e & 0x1ffu; }
    const uint32_t c = __brev((uint32_t)hold);
    for (uint32_t l = kRoot + 1; l <= 15; l++) {
        const uint32_t code = c >> (32 - l);
        const uint32_t f = uni(can->first[l]), k = uni(can->count[l]);
        if (code - f < k) { len = l; return uni(can->sorted[uni(can->offs[l]) + code - f]); }
    }
    len = 1;
    return kSymBad;
}

struct Rd {                           // wave-uniform bit reader over the LDS input ring
    uint64_t hold;
    uint32_t bits, ipos, rbase;
};

__device__ __attribute__((always_inline)) inline void ring_stage(InfLDS &S, Rd &r, const uint8_t *in,
                                                                 uint32_t n, uint32_t base, int lane) {
    __syncthreads();
    for (uint32_t i = (uint32_t)lane; i < (uint32_t)(kIRing + 16) / 4; i += 64) {
        uint32_t w = 0;
        const uint32_t x = base + 4 * i;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (x + k < n) w |= (uint32_t)in[x + k] << (8 * k);
        S.ring.w[i] = w;
    }
    r.rbase = base;
    __syncthreads();
}

// NEEDBITS-style: at least 32 bits in `hold` (zeros beyond the input)
__device__ __attribute__((always_inline)) inline void refill(InfLDS &S, Rd &r, const uint8_t *in, uint32_t n,
                                                             int lane) {
    if (r.bits >= 32) return;
    uint32_t o = r.ipos - r.rbase;
    if (r.ipos < r.rbase || o + 8 > (uint32_t)kIRing) {
        ring_stage(S, r, in, n, r.ipos & ~3u, lane);
        o = r.ipos - r.rbase;
    }
    const uint32_t w0 = uni(S.ring.w[o >> 2]), w1 = uni(S.ring.w[(o >> 2) + 1]);
    const uint32_t v = __builtin_amdgcn_alignbyte(w1, w0, o & 3u);
    r.hold |= (uint64_t)v << r.bits;
    r.bits += 32;
    r.ipos += 4;
}

__device__ __attribute__((always_inline)) inline uint64_t bitpos(const Rd &r) {
    return (uint64_t)r.ipos * 8 - r.bits;
}
__device__ __attribute__((always_inline)) inline void dropb(Rd &r, uint32_t k) { r.hold >>= k; r.bits -= k; }
__device__ __attribute__((always_inline)) inline void seek(Rd &r, uint32_t byte) { r.hold = 0; r.bits = 0; r.ipos = byte; }

// inflateCodesUsed (inflate.c:1521-1527): the code-table entries inftrees.c's
// inflate_table uses for a code of n lengths at root bits (inflate.c's lenbits 9
// / distbits 6): 1 << root for the root table (root clamped to [min, max]
// length) plus, for every run of codes longer than root that shares its top root
// bits, a sub-table of 1 << curr entries, curr grown while the codes still to
// place overfill it (inftrees.c:214-300).  2 for a code with no lengths.
// Uniform across the wave; run only for streams that ask (InflateJob::zcodes).
// Lane 0 walks the lengths with its per-length tables in LDS (cu): dynamically
// indexed register arrays would put k_inflate_decode's frame in scratch and
// raise its register count for a call that only inflateCodesUsed needs.
__device__ __attribute__((noinline)) uint32_t codes_used(const uint16_t *lens, int n, int root, uint32_t *cu,
                                                         int lane) {
    __syncthreads();
    uint32_t used = 0;
    if (lane == 0) {
        uint32_t *cnt = cu, *next = cu + 16, *rem = cu + 32;
        for (int L = 0; L < 16; L++) cnt[L] = 0;
        for (int i = 0; i < n; i++) cnt[lens[i] & 15u]++;
        cnt[0] = 0;
        int max = 15;
        while (max >= 1 && cnt[max] == 0) max--;
        if (max == 0) {
            used = 2;
        } else {
            int min = 1;
            while (min < max && cnt[min] == 0) min++;
            if (root > max) root = max;
            if (root < min) root = min;
            used = 1u << root;
            uint32_t code = 0;
            next[0] = rem[0] = 0;
            for (int L = 1; L < 16; L++) {
                code = (code + (L > 1 ? cnt[L - 1] : 0u)) << 1;
                next[L] = code;
                rem[L] = cnt[L];
            }
            uint32_t low = 0xffffffffu;
            for (int L = root + 1; L <= max; L++) {
                for (int i = 0; i < n; i++) {
                    if (lens[i] != (uint16_t)L) continue;
                    const uint32_t key = next[L] >> (L - root);
                    if (key != low) {
                        int curr = L - root, left = 1 << curr;
                        while (curr + root < max) {
                            left -= (int)rem[curr + root];
                            if (left <= 0) break;
                            curr++;
                            left <<= 1;
                        }
                        used += 1u << curr;
                        low = key;
                    }
                    next[L]++;
                    rem[L]--;
                }
            }
        }
        cu[47] = used;
    }
    __syncthreads();
    return cu[47];
}

// kIdx: the streaming inflate()'s consumption index (InflateJob::eidx / bidx)
// kW: waves per SIMD the register budget is cut for (0: the compiler's
// choice, 125 VGPRs = 4 waves; 5: 96 VGPRs and a 64-byte spill).  Batches of
// 2048 streams or more take kW = 5: the C4 inflate leg 12.27 -> 12.57 GB/s
// (profiles/r05y2_ab_inflate_five_waves.log); 6 or more waves do not fit.
// ZGPU_INFL_W5=0 keeps 4 waves everywhere, =2 takes 5 for every batch (tests).
template <bool kIdx, int kW = 0>
__global__ __launch_bounds__(64, kW ? kW : 1) void k_inflate_decode(InflateJob job) {
    __shared__ InfLDS S;
    const int lane = threadIdx.x;
    const uint32_t bi = blockIdx.x, g = job.first + bi;
    const uint32_t n = (uint32_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    const uint64_t cap0 = job.dst_cap[g];
    const bool counting = job.count_only != 0;
    const bool probe = cap0 == 0 && !counting;
    const uint32_t cap = counting ? 0xffffffffu : probe ? 1u : (uint32_t)cap0;
    uint8_t *out = counting ? nullptr : job.dst + job.dst_off[g];
    uint64_t *mrec = counting ? nullptr : job.mrec + job.mrec_off[bi];
    const uint64_t inbits = (uint64_t)n * 8;
    const int wrap = job.wrap;

    Rd r;
    r.hold = 0; r.bits = 0; r.ipos = 0; r.rbase = 0;
    const uint64_t rb = job.res_bit ? job.res_bit[g] : 0;       // resume: the block header's bit
    ring_stage(S, r, in, n, (uint32_t)(rb >> 3) & ~3u, lane);

    uint32_t put = job.res_hist ? job.res_hist[g] : 0, ob = put, nm = 0, pbyte = 0;
    uint32_t stop = kIEnd;
    uint64_t used = 0, used_bad = 0;
    uint32_t chk_kind = 0, chk_want = 0, isize = 0;
    bool gz = false;
    uint64_t blk_bit = 0;                            // the last block boundary reached
    uint32_t blk_put = 0;
    uint32_t zlast = 0;                              // BFINAL of the current block (data_type)
    bool ztype = (job.stop_mode & 4u) != 0;          // waiting at a block header in mode TYPE
    bool zstored = false;                            // stopped in mode STORED with no bits held (inflateSyncPoint)
    // inflateMark's value where the input ran out (inflate.c:1510-1519): back << 16, plus a stored
    // block's bytes left (COPY); back = -1 outside a length/distance symbol
    int64_t zmark = -65536;
    uint32_t zcodes = 0xffffffffu;                   // inflateCodesUsed of the last dynamic block (none: ~0)
    // a gzip header cut short: the bits inflate.c holds there (-1: from the reader).  Its
    // fields come in NEEDBITS groups (magic 16, CM+FLG 16, MTIME 32, XFL+OS 16, XLEN 16, HCRC
    // 16 bits) with extra / name / comment bytes taken as they come (inflate.c:629-807)
    int64_t zhold = -1;
    if (job.res_bit) {
        seek(r, (uint32_t)(rb >> 3));
        refill(S, r, in, n, lane);
        dropb(r, (uint32_t)(rb & 7));
        blk_bit = rb;
        blk_put = put;
    }

    auto ceil_used = [&]() -> uint64_t { return (bitpos(r) + 7) >> 3; };
    uint32_t ne = 0, nbk = 0;                        // index entries / block boundaries recorded (kIdx)
    auto index_hdr = [&]() {                         // a block header's end: bit | 1 << 62 | BFINAL << 63
        if (kIdx) {
            if (lane == 0 && nbk < job.bcap) {
                job.bidx[2 * (uint64_t)nbk] = bitpos(r) | 1ull << 62 | (uint64_t)zlast << 63;
                job.bidx[2 * (uint64_t)nbk + 1] = put;
            }
            nbk++;
        }
    };
    auto index_sym = [&](uint32_t out_end, bool stored, uint64_t v) {
        if (kIdx) {
            if (lane == 0 && ne < job.ecap) {
                job.eidx[2 * (uint64_t)ne] = (uint64_t)out_end | (uint64_t)stored << 32 | (uint64_t)zlast << 33;
                job.eidx[2 * (uint64_t)ne + 1] = v;
            }
            ne++;
        }
    };
    auto flush_obuf = [&](uint32_t upto) {          // output bytes [ob, upto), upto <= ob + kOBuf
        __syncthreads();
        if (!probe && !counting)
            for (uint32_t i = (uint32_t)lane; i < upto - ob; i += 64) out[ob + i] = S.obuf[i];
        __syncthreads();
    };
    auto flush_mbuf = [&](uint32_t k) {             // the last k staged records
        __syncthreads();
        if (!counting && (uint32_t)lane < k) mrec[nm - k + (uint32_t)lane] = S.mbuf[lane];
        __syncthreads();
    };

    // ---------------- HEAD (inflate.c:622-669) / gzip header (:629-807) ----------------
    if (wrap && !job.res_bit) {
        refill(S, r, in, n, lane);
        if (bitpos(r) + 16 > inbits) { stop = kIInEnd; used = n; goto done; }
        const uint32_t h16 = (uint32_t)r.hold & 0xffffu;
        if ((wrap & 2) && h16 == 0x8b1fu) {
            gz = true;
            // header fields straight from global memory (a few bytes)
            if (n < 4) { zhold = 8ll * (n - 2); stop = kIInEnd; used = n; goto done; }
            const uint32_t flags = in[2] | ((uint32_t)in[3] << 8);
            if ((flags & 0xffu) != 8u || (flags & 0xe000u)) { stop = kIData; used = 4; goto done; }
            uint32_t p = 10;
            if (n < p) { zhold = 8ll * (n < 8 ? n - 4 : n - 8); stop = kIInEnd; used = n; goto done; }
            if (flags & 0x0400u) {                                   // FEXTRA
                if (n < p + 2) { zhold = 8ll * (n - p); stop = kIInEnd; used = n; goto done; }
                const uint32_t xlen = in[p] | ((uint32_t)in[p + 1] << 8);
                p += 2;
                if (n - p < xlen) { zhold = 0; stop = kIInEnd; used = n; goto done; }
                p += xlen;
            }
            for (uint32_t f = 0x0800u; f <= 0x1000u; f <<= 1) {      // FNAME, FCOMMENT
                if (!(flags & f)) continue;
                uint32_t z = 0xffffffffu;
                for (uint32_t q = p; q < n && z == 0xffffffffu; q += 64) {
                    const uint32_t x = q + (uint32_t)lane;
                    const uint64_t m = __ballot(x < n && in[x] == 0);
                    if (m) z = q + (uint32_t)__builtin_ctzll(m);
                }
                if (z == 0xffffffffu) { zhold = 0; stop = kIInEnd; used = n; goto done; }
                p = z + 1;
            }
            if (flags & 0x0200u) {                                   // FHCRC
                if (n < p + 2) { zhold = 8ll * (n - p); stop = kIInEnd; used = n; goto done; }
                uint32_t c = 0xffffffffu;
                for (uint32_t q = 0; q < p; q++) c = job.crc_byte[(c ^ in[q]) & 0xffu] ^ (c >> 8);
                c = ~c;
                const uint32_t want = in[p] | ((uint32_t)in[p + 1] << 8);
                p += 2;
                if (want != (c & 0xffffu)) { stop = kIData; used = p; goto done; }
            }
            seek(r, p);
        } else {
            const uint32_t wlen = ((h16 >> 4) & 15u) + 8u;
            if (!(wrap & 1) || ((((h16 & 0xffu) << 8) + (h16 >> 8)) % 31u) || (h16 & 15u) != 8u ||
                wlen > 15u || (job.wbits && wlen > (uint32_t)job.wbits)) {
                stop = kIData; used = 2; goto done;
            }
            dropb(r, 16);
            if (h16 & 0x2000u) {                                     // FDICT: DICTID, Z_NEED_DICT
                if (n < 6) { stop = kIInEnd; used = n; } else { stop = kIDict; used = 6; }
                goto done;
            }
        }
    }

    if (wrap && !job.res_bit) ztype = true;                     // after the header: TYPE (raw starts in TYPEDO)
    if (wrap && !job.res_bit && (job.stop_mode & 1u)) {        // Z_BLOCK: before the first block
        blk_bit = bitpos(r);
        blk_put = put;
        stop = kIBlock;
        used = blk_bit >> 3;
        goto done;
    }

    // ---------------- blocks (inflate.c:827-1181) ----------------
    for (;;) {
        refill(S, r, in, n, lane);
        if (bitpos(r) + 3 > inbits) { stop = kIInEnd; used = n; goto done; }
        const uint32_t last = (uint32_t)r.hold & 1u, type = ((uint32_t)r.hold >> 1) & 3u;
        dropb(r, 3);
        zlast = last;
        ztype = false;
        if (type == 3) { stop = kIData; used = ceil_used(); goto done; }
        if (type == 0) {                                             // STORED, COPY
            dropb(r, r.bits & 7u);
            refill(S, r, in, n, lane);
            if (bitpos(r) + 32 > inbits) { zstored = bitpos(r) == inbits; stop = kIInEnd; used = n; goto done; }
            const uint32_t len = (uint32_t)r.hold & 0xffffu, nlen = ((uint32_t)r.hold >> 16) & 0xffffu;
            if (len != (nlen ^ 0xffffu)) { stop = kIData; used = (bitpos(r) >> 3) + 4; goto done; }
            dropb(r, 32);
            index_hdr();
            if ((job.stop_mode & 8u) && bitpos(r) > job.trees_after) {   // Z_TREES: mode COPY_, before the bytes
                blk_bit = bitpos(r);
                blk_put = put;
                stop = kITrees;
                used = blk_bit >> 3;
                goto done;
            }
            const uint32_t bp = (uint32_t)(bitpos(r) >> 3);
            flush_obuf(put);
            uint32_t cnt = len;
            if (cnt > n - bp) cnt = n - bp;
            if (cnt > cap - put) cnt = cap - put;
            if (cnt) index_sym(put + cnt, true, bp);
            if (probe) { if (cnt) pbyte = in[bp]; }
            else if (!counting) for (uint32_t i = (uint32_t)lane; i < cnt; i += 64) out[put + i] = in[bp + i];
            put += cnt;
            ob = put;
            seek(r, bp + cnt);
            if (cnt < len) {
                zmark = -65536 + (int64_t)(len - cnt);      // COPY: length bytes still to copy
                if (put == cap) { stop = kIFull; used = bp + cnt; } else { stop = kIInEnd; used = n; }
                goto done;
            }
        } else {
            if (type == 1) {                                         // fixedtables (inflate.c:255-285)
                for (int i = lane; i < 288; i += 64)
                    S.lens[i] = (uint16_t)(i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8);
                __syncthreads();
                build_code<kLRoot>(S.lens, 288, kLens, S.lt, &S.lcan, lane);
                for (int i = lane; i < 32; i += 64) S.lens[i] = 5;
                __syncthreads();
                build_code<kDRoot>(S.lens, 32, kDists, S.dt, &S.dcan, lane);
            } else {                                                 // TABLE, LENLENS, CODELENS
                refill(S, r, in, n, lane);
                if (bitpos(r) + 14 > inbits) { stop = kIInEnd; used = n; goto done; }
                const uint32_t nlen = ((uint32_t)r.hold & 31u) + 257;
                const uint32_t ndist = (((uint32_t)r.hold >> 5) & 31u) + 1;
                const uint32_t ncode = (((uint32_t)r.hold >> 10) & 15u) + 4;
                dropb(r, 14);
                if (nlen > 286 || ndist > 30) { stop = kIData; used = ceil_used(); goto done; }
                uint32_t cl = 0;                                     // lane i: length of code-length code i
                {
                    uint32_t have = 0;
                    while (have < ncode) {
                        refill(S, r, in, n, lane);
                        if (bitpos(r) + 3 > inbits) { stop = kIInEnd; used = n; goto done; }
                        const uint32_t v = (uint32_t)r.hold & 7u;
                        if ((uint32_t)lane == c_order[have]) cl = v;
                        dropb(r, 3);
                        have++;
                    }
                }
                if (lane < 19) S.lens[lane] = (uint16_t)cl;
                __syncthreads();
                if (!build_code<kCRoot>(S.lens, 19, kCodes, S.ct, nullptr, lane)) {
                    stop = kIData; used = ceil_used(); goto done;
                }
                // mode CODELENS: state->next holds the code-length code's table (inflateCodesUsed)
                const uint32_t zcl = job.zcodes ? codes_used(S.lens, 19, 7, S.cu, lane) : 0u;
                uint32_t have = 0;
                const uint32_t total = nlen + ndist;
                while (have < total) {
                    refill(S, r, in, n, lane);
                    const uint32_t e = uni(S.ct[(uint32_t)r.hold & 127u]);
                    const uint32_t L = (e >> 9) & 15u, sym = e & 0x1ffu;
                    // a repeat code and its extra bits are read together (inflate.c
                    // CODELENS: NEEDBITS(here.bits + 2/3/7)), so a short input keeps both
                    const uint32_t xb = sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u;
                    if (bitpos(r) + L + xb > inbits) { zcodes = zcl; stop = kIInEnd; used = n; goto done; }
                    dropb(r, L);
                    if (sym == kSymBad || sym < 16) {                // empty code-length code: 0 per bit
                        if (lane == 0) S.lens[have] = (uint16_t)(sym == kSymBad ? 0 : sym);
                        have++;
                        continue;
                    }
                    uint32_t len, rep;
                    if (sym == 16) {
                        if (bitpos(r) + 2 > inbits) { stop = kIInEnd; used = n; goto done; }
                        if (have == 0) { stop = kIData; used = (bitpos(r) + 2 + 7) >> 3; goto done; }
                        __syncthreads();
                        len = uni(S.lens[have - 1]);
                        rep = 3 + ((uint32_t)r.hold & 3u);
                        dropb(r, 2);
                    } else if (sym == 17) {
                        if (bitpos(r) + 3 > inbits) { stop = kIInEnd; used = n; goto done; }
                        len = 0;
                        rep = 3 + ((uint32_t)r.hold & 7u);
                        dropb(r, 3);
                    } else {
                        if (bitpos(r) + 7 > inbits) { stop = kIInEnd; used = n; goto done; }
                        len = 0;
                        rep = 11 + ((uint32_t)r.hold & 127u);
                        dropb(r, 7);
                    }
                    if (have + rep > total) { stop = kIData; used = ceil_used(); goto done; }
                    for (uint32_t k = (uint32_t)lane; k < rep; k += 64) S.lens[have + k] = (uint16_t)len;
                    have += rep;
                }
                __syncthreads();
                if (uni(S.lens[256]) == 0) { stop = kIData; used = ceil_used(); goto done; }
                if (!build_code<kLRoot>(S.lens, (int)nlen, kLens, S.lt, &S.lcan, lane)) {
                    stop = kIData; used = ceil_used(); goto done;
                }
                if (!build_code<kDRoot>(S.lens + nlen, (int)ndist, kDists, S.dt, &S.dcan, lane)) {
                    stop = kIData; used = ceil_used(); goto done;
                }
                if (job.zcodes)
                    zcodes = codes_used(S.lens, (int)nlen, 9, S.cu, lane) + codes_used(S.lens + nlen, (int)ndist, 6, S.cu, lane);
            }
            index_hdr();
            if ((job.stop_mode & 8u) && bitpos(r) > job.trees_after) {   // Z_TREES: mode LEN_, before the first code
                blk_bit = bitpos(r);
                blk_put = put;
                stop = kITrees;
                used = ceil_used();
                goto done;
            }
            // ---------------- LEN .. MATCH / LIT ----------------
            for (;;) {
                refill(S, r, in, n, lane);
                uint32_t L;
                const uint32_t sym = dec_code<kLRoot>(S.lt, &S.lcan, r.hold, L);
                if (bitpos(r) + L > inbits) { zmark = 0; stop = kIInEnd; used = n; goto done; }   // LEN: back 0
                dropb(r, L);
                if (sym < 256) {
                    index_sym(put + 1, false, bitpos(r));
                    if (put == cap) { stop = kIFull; used = ceil_used(); goto done; }
                    if (probe) pbyte = sym;
                    else if (lane == 0) S.obuf[put - ob] = (uint8_t)sym;
                    put++;
                    if (put - ob == (uint32_t)kOBuf) { flush_obuf(put); ob = put; }
                    continue;
                }
                if (sym == 256) break;
                if (sym > 285) { stop = kIData; used = ceil_used(); goto done; }   // kSymBad, 286, 287
                const uint32_t ls = sym - 257, xl = c_lext[ls];
                if (bitpos(r) + xl > inbits) { zmark = (int64_t)L << 16; stop = kIInEnd; used = n; goto done; }
                const uint32_t len = c_lbase[ls] + ((uint32_t)r.hold & ((1u << xl) - 1u));
                dropb(r, xl);
                refill(S, r, in, n, lane);
                uint32_t DL;
                const uint32_t ds = dec_code<kDRoot>(S.dt, &S.dcan, r.hold, DL);
                if (bitpos(r) + DL > inbits) { zmark = (int64_t)(L + xl) << 16; stop = kIInEnd; used = n; goto done; }
                dropb(r, DL);
                if (ds > 29) { stop = kIData; used = ceil_used(); goto done; }
                const uint32_t xd = c_dext[ds];
                if (bitpos(r) + xd > inbits) { zmark = (int64_t)(L + xl + DL) << 16; stop = kIInEnd; used = n; goto done; }
                const uint32_t dist = c_dbase[ds] + ((uint32_t)r.hold & ((1u << xd) - 1u));
                dropb(r, xd);
                index_sym(put + len, false, bitpos(r));
                if (put == cap) { stop = kIFull; used = ceil_used(); goto done; }    // MATCH: room first
                // too far back (inflateBack: beyond its window, infback.c:494-499)
                if (dist > put || (job.dmax && dist > job.dmax)) { stop = kIData; used = ceil_used(); goto done; }
                const uint32_t copy = len < cap - put ? len : cap - put;
                if (lane == 0) S.mbuf[nm & (kMBuf - 1)] = (uint64_t)put | ((uint64_t)copy << 32) | ((uint64_t)dist << 41);
                nm++;
                if ((nm & (kMBuf - 1)) == 0) flush_mbuf(kMBuf);
                put += copy;
                while (put - ob >= (uint32_t)kOBuf) { flush_obuf(ob + kOBuf); ob += kOBuf; }
                if (copy < len) { stop = kIFull; used = ceil_used(); goto done; }
            }
        }
        ztype = true;                                // END_BLOCK: mode TYPE
        if (job.stop_mode & 2u) {                    // Z_BLOCK: stop at it (after the last block too)
            blk_bit = bitpos(r);
            blk_put = put;
            stop = kIBlock;
            used = (blk_bit + 7) >> 3;
            goto done;
        }
        if (kIdx) {                                  // the index: every block's end, the last one flagged
            if (lane == 0 && nbk < job.bcap) {
                job.bidx[2 * (uint64_t)nbk] = bitpos(r) | (uint64_t)last << 63;
                job.bidx[2 * (uint64_t)nbk + 1] = put;
            }
            nbk++;
        }
        if (last) break;
        blk_bit = bitpos(r);                         // a block boundary: resumable here
        blk_put = put;
    }
    ztype = false;                                   // TYPEDO -> CHECK

    // ---------------- CHECK, LENGTH (inflate.c:1183-1221) ----------------
    dropb(r, r.bits & 7u);
    if (wrap && !gz) {
        refill(S, r, in, n, lane);
        if (bitpos(r) + 32 > inbits) { stop = kIInEnd; used = n; goto done; }
        const uint32_t h = (uint32_t)r.hold;
        chk_want = (h >> 24) | ((h >> 8) & 0xff00u) | ((h << 8) & 0xff0000u) | (h << 24);
        dropb(r, 32);
        chk_kind = 1;
        used = used_bad = bitpos(r) >> 3;
    } else if (gz) {
        refill(S, r, in, n, lane);
        if (bitpos(r) + 32 > inbits) { stop = kIInEnd; used = n; goto done; }
        chk_want = (uint32_t)r.hold;
        dropb(r, 32);
        chk_kind = 2;
        used_bad = bitpos(r) >> 3;
        refill(S, r, in, n, lane);
        if (bitpos(r) + 32 > inbits) {
            isize = 3;
            used = n;
        } else {
            isize = (uint32_t)r.hold == put ? 1 : 2;
            dropb(r, 32);
            used = bitpos(r) >> 3;
        }
    } else {
        used = bitpos(r) >> 3;
    }
    stop = kIEnd;

done:
    flush_obuf(put);
    if (nm & (kMBuf - 1)) flush_mbuf(nm & (kMBuf - 1));
    if (lane == 0) {
        InflateRec rc;
        rc.put = put;
        rc.used = used;
        rc.used_bad = used_bad;
        rc.stop = stop;
        rc.nmatch = nm;
        rc.chk_kind = chk_kind;
        rc.chk_want = chk_want;
        rc.isize = isize;
        rc.pbyte = pbyte;
        job.rec[bi] = rc;
        job.dst_len[g] = probe ? 0 : put;            // the checksum kernels read this
        if (kIdx) {
            job.icnt[0] = ne;
            job.icnt[1] = nbk;
        }
        if (job.blk_out) {
            job.blk_out[2 * (uint64_t)g] = blk_bit;
            job.blk_out[2 * (uint64_t)g + 1] = blk_put;
        }
        if (job.zstate_out) {
            const uint64_t bp = bitpos(r);
            const uint64_t held = zhold >= 0 ? (uint64_t)zhold : (bp <= inbits ? inbits - bp : 0);
            job.zstate_out[2 * (uint64_t)g] = held | (uint64_t)zlast << 32 |
                                              (uint64_t)(ztype ? 1 : 0) << 33 | (uint64_t)(zstored ? 1 : 0) << 34;
            job.zstate_out[2 * (uint64_t)g + 1] = (uint64_t)(uint32_t)(int32_t)zmark | (uint64_t)zcodes << 32;
        }
    }
}

// ------------------------------------------------------------------------
// k_inflate_copy — matches in stream order through an LDS window.
// ------------------------------------------------------------------------
constexpr uint32_t kWin = 40960;       // >= 32768 + kChunk + 258
constexpr uint32_t kChunk = 4096;
constexpr uint32_t kLaneCopy = 32;     // matches this short are copied one lane each (k_inflate_copy)

__device__ __attribute__((always_inline)) inline uint32_t wslot(uint32_t p) { return p % kWin; }

__global__ __launch_bounds__(64) void k_inflate_copy(InflateJob job) {
    __shared__ uint8_t W[kWin];
    const int lane = threadIdx.x;
    const uint32_t bi = blockIdx.x, g = job.first + bi;
    const InflateRec rc = job.rec[bi];
    if (job.dst_cap[g] == 0 || rc.nmatch == 0) return;
    const uint32_t put = (uint32_t)rc.put, nm = rc.nmatch;
    uint8_t *out = job.dst + job.dst_off[g];
    const uint64_t *M = job.mrec + job.mrec_off[bi];
    uint32_t loaded = 0, mi = 0, mbase = 0;
    uint64_t mreg = (uint32_t)lane < nm ? M[lane] : 0;
    // the first chunk that holds a match; earlier output is final already
    const uint32_t p0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mreg);
    uint32_t c0 = p0 >= 32768u + kChunk ? ((p0 - 32768u) / kChunk) * kChunk : 0u;
    loaded = c0 >= 32768u ? c0 - 32768u : 0u;
    for (; c0 < put && mi < nm; c0 += kChunk) {
        const uint32_t c1 = c0 + kChunk < put ? c0 + kChunk : put;
        const uint32_t want = c1 + 258 < put ? c1 + 258 : put;
        for (uint32_t p = loaded + (uint32_t)lane; p < want; p += 64) W[wslot(p)] = out[p];
        loaded = want;
        __syncthreads();
        while (mi < nm) {
            if (mi - mbase >= 64) {
                mbase = mi;
                mreg = mbase + (uint32_t)lane < nm ? M[mbase + lane] : 0;
            }
            const int k = (int)(mi - mbase);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mreg, k);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mreg >> 32), k);
            const uint32_t pos = lo;
            if (pos >= c1) break;
            const uint32_t len = hi & 511u, dist = hi >> 9;
            // round 5: a run of short matches, one lane each (lane = record mbase + lane).
            // Lane k leads; a later lane joins while its source ends before the lead's
            // position (all final bytes: literals or earlier matches), so no lane reads
            // what another writes, and a lane copies its own bytes in order (a source
            // overlapping its own destination included)
            if (len <= kLaneCopy) {
                const uint32_t ml = (uint32_t)mreg, mh = (uint32_t)(mreg >> 32);
                const uint32_t lp = ml, ll = mh & 511u, ld = mh >> 9;
                const bool in_run = lane >= k && mbase + (uint32_t)lane < nm && lp < c1 && ll <= kLaneCopy &&
                                    (lane == k || lp - ld + ll <= pos);
                const uint64_t stop_m = __ballot(!in_run && lane >= k);
                const int end = stop_m ? (int)__builtin_ctzll(stop_m) : 64;     // lanes [k, end)
                if (lane >= k && lane < end) {
                    const uint32_t s0 = lp - ld;
                    for (uint32_t j = 0; j < ll; j++) W[wslot(lp + j)] = W[wslot(s0 + j)];
                }
                mi = mbase + (uint32_t)end;
                continue;
            }
            const uint32_t s0 = pos - dist;
            if (dist >= len) {
                for (uint32_t j = (uint32_t)lane; j < len; j += 64) W[wslot(pos + j)] = W[wslot(s0 + j)];
            } else {
                for (uint32_t j = (uint32_t)lane; j < len; j += 64) W[wslot(pos + j)] = W[wslot(s0 + j % dist)];
            }
            mi++;
        }
        __syncthreads();
        // [c0, want): final below c1; the overhang holds literals, the tails of
        // matches that started in this chunk and (harmless) unresolved bytes
        // that a later chunk rewrites
        for (uint32_t p = c0 + (uint32_t)lane; p < want; p += 64) out[p] = W[wslot(p)];
        __syncthreads();
    }
    // output after the last chunk holding a match is literal-only and final
}

// ------------------------------------------------------------------------
// k_inflate_finish — trailer checks and uncompress2's result (uncompr.c:62-84)
// ------------------------------------------------------------------------
__global__ void k_inflate_finish(InflateJob job) {
    const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
    if (bi >= job.count) return;
    const uint32_t g = job.first + bi;
    const InflateRec rc = job.rec[bi];
    const uint64_t cap0 = job.dst_cap[g];
    const bool probe = cap0 == 0;
    uint32_t stop = rc.stop;
    uint64_t used = rc.used;
    if (stop == kIEnd && rc.chk_kind) {
        uint32_t got;
        if (probe) {                               // at most one byte was produced
            if (rc.chk_kind == 1) {
                got = rc.put ? ((1u + rc.pbyte) | ((1u + rc.pbyte) << 16)) : 1u;
            } else {
                got = rc.put ? ~(job.crc_byte[(0xffffffffu ^ rc.pbyte) & 0xffu] ^ 0x00ffffffu) : 0u;
            }
        } else {
            got = rc.chk_kind == 1 ? job.adler[bi] : job.crc[bi];
        }
        if (got != rc.chk_want) { stop = kIData; used = rc.used_bad; }
        else if (rc.chk_kind == 2 && rc.isize == 2) stop = kIData;
        else if (rc.chk_kind == 2 && rc.isize == 3) stop = kIInEnd;
    }
    int32_t status;
    if (stop == kIEnd) status = 0;                                    // Z_OK
    else if (stop == kIData || stop == kIDict) status = -3;          // Z_DATA_ERROR
    else status = (probe || rc.put < cap0) ? -3 : -5;                // Z_BUF_ERROR only when full
    job.status[g] = status;
    if (job.stop_out) job.stop_out[g] = stop;
    job.dst_len[g] = probe ? 0 : rc.put;
    if (job.src_used) job.src_used[g] = used;
}

// ------------------------------------------------------------------------
// Block-parallel decode of a lone large stream (zgpu_api.cpp inflate_par).
// deflate's blocks are found without decoding what precedes them: every bit
// offset is tried as a block header, the candidates that pass are decoded
// count-only (k_inflate_decode, InflateJob::count_only) for their end, and the
// host follows the chain of ends from the first block.  Then every block of
// the chain is decoded at its output offset (literals in place, matches as
// records), k_infl_sym resolves each block's matches with the bytes before
// the block as references (an output position), and k_infl_resolve replaces
// the references block by block in stream order.
// ------------------------------------------------------------------------
// 64 bits of the stream from bit b (zero past n)
__device__ inline uint64_t bits_at(const uint8_t *in, uint64_t n, uint64_t b) {
    const uint64_t B = b >> 3;
    uint64_t lo = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) lo |= (uint64_t)(B + k < n ? in[B + k] : 0) << (8 * k);
    const uint32_t sh = (uint32_t)(b & 7);
    const uint64_t nx = B + 8 < n ? in[B + 8] : 0;
    return sh ? (lo >> sh) | (nx << (64 - sh)) : lo;
}

// k_infl_scan1: bit offsets [b0, b1) that could hold a stored block header
// (LEN == ~NLEN at the next byte, the block inside the input) or a dynamic one
// (HLIT <= 29, HDIST <= 29, a complete code-length code: inftrees.c's CODES
// rule).  Candidates are appended to list (at most cap; *cnt counts all).
__global__ __launch_bounds__(256) void k_infl_scan1(const uint8_t *in, uint64_t n, uint64_t b0, uint64_t b1,
                                                   uint64_t *list, uint32_t cap, uint32_t *cnt) {
    const uint64_t b = b0 + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= b1) return;
    const uint64_t w = bits_at(in, n, b);
    const uint32_t type = (uint32_t)(w >> 1) & 3u;
    bool ok = false;
    if (type == 0) {
        const uint64_t p = (b + 3 + 7) >> 3;
        if (p + 4 <= n) {
            const uint32_t len = in[p] | ((uint32_t)in[p + 1] << 8), nlen = in[p + 2] | ((uint32_t)in[p + 3] << 8);
            ok = len == (nlen ^ 0xffffu) && p + 4 + len <= n;
        }
    } else if (type == 2) {
        const uint32_t hlit = (uint32_t)(w >> 3) & 31u, hdist = (uint32_t)(w >> 8) & 31u;
        const uint32_t ncode = ((uint32_t)(w >> 13) & 15u) + 4;
        if (hlit <= 29 && hdist <= 29) {
            const uint64_t v = bits_at(in, n, b + 17);               // 3 bits per code-length code length
            uint32_t kraft = 0;
            for (uint32_t i = 0; i < ncode; i++) {
                const uint32_t l = (uint32_t)(v >> (3 * i)) & 7u;
                if (l) kraft += 128u >> l;
            }
            ok = kraft == 128u;
        }
    }
    if (ok) {
        const uint32_t k = atomicAdd(cnt, 1u);
        if (k < cap) list[k] = b;
    }
}

// k_infl_scan2: one thread per scan1 candidate; a dynamic header's code
// lengths are decoded with its code-length code and both codes checked as
// inflate_table would (over-subscribed: never; incomplete: only a single
// 1-bit code; END_BLOCK present; no repeat before the first length and no
// run past HLIT + HDIST).  Survivors go to out (the stored ones pass).
struct BitRd {
    const uint8_t *in;
    uint64_t n, pos;          // next bit
    __device__ inline uint32_t get(uint32_t k) {     // k <= 32
        const uint64_t v = bits_at(in, n, pos);
        pos += k;
        return k == 32 ? (uint32_t)v : (uint32_t)v & ((1u << k) - 1u);
    }
};
__global__ __launch_bounds__(256) void k_infl_scan2(const uint8_t *in, uint64_t n, const uint64_t *list,
                                                   uint32_t count, uint64_t *out, uint32_t cap, uint32_t *cnt) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= count) return;
    const uint64_t b = list[t];
    BitRd r{in, n, b};
    const uint32_t hdr = r.get(3);
    bool ok = true;
    if (((hdr >> 1) & 3u) == 2u) {
        const uint32_t nlen = r.get(5) + 257, ndist = r.get(5) + 1, ncode = r.get(4) + 4;
        uint64_t cl = 0;                                            // 3 bits per symbol 0..18
        for (uint32_t i = 0; i < ncode; i++) cl |= (uint64_t)r.get(3) << (3 * c_order[i]);
        uint32_t ccnt[8];
#pragma unroll
        for (int l = 0; l < 8; l++) ccnt[l] = 0;
        for (uint32_t s2 = 0; s2 < 19; s2++) {
            const uint32_t l = (uint32_t)(cl >> (3 * s2)) & 7u;
#pragma unroll
            for (int q = 1; q < 8; q++) ccnt[q] += l == (uint32_t)q;
        }
        const uint32_t total = nlen + ndist;
        uint32_t have = 0, prev = 0;
        uint32_t lk = 0, dk = 0, lmax = 0, dmax = 0, l256 = 0;      // Kraft sums in 2^-15 units
        auto put_len = [&](uint32_t l, uint32_t rep) {
            // lengths l for symbols have .. have + rep - 1
            const uint32_t la = have < nlen ? (have + rep < nlen ? rep : nlen - have) : 0;
            if (l) {
                lk += la << (15 - l);
                dk += (rep - la) << (15 - l);
                if (la) lmax = lmax > l ? lmax : l;
                if (rep > la) dmax = dmax > l ? dmax : l;
                if (have <= 256 && 256 < have + rep) l256 = l;
            }
            have += rep;
        };
        while (ok && have < total) {
            // canonical decode, one bit at a time (codes are sent MSB first)
            uint32_t code = 0, first = 0, sym = 0xffu;
#pragma unroll
            for (int l = 1; l < 8; l++) {
                if (sym == 0xffu) {
                    code |= r.get(1);
                    const uint32_t c = ccnt[l];
                    if (code - first < c) {
                        uint32_t k = code - first;                  // the k-th symbol of length l
                        for (uint32_t s2 = 0; s2 < 19; s2++)
                            if (((uint32_t)(cl >> (3 * s2)) & 7u) == (uint32_t)l) {
                                if (k == 0) { sym = s2; break; }
                                k--;
                            }
                    } else {
                        first = (first + c) << 1;
                        code <<= 1;
                    }
                }
            }
            if (sym == 0xffu) { ok = false; break; }
            if (sym < 16) { put_len(sym, 1); prev = sym; continue; }
            uint32_t rep, l = 0;
            if (sym == 16) { if (have == 0) { ok = false; break; } l = prev; rep = 3 + r.get(2); }
            else if (sym == 17) rep = 3 + r.get(3);
            else rep = 11 + r.get(7);
            if (have + rep > total) { ok = false; break; }
            put_len(l, rep);
            prev = l;
        }
        if (ok) ok = l256 != 0 && lk <= 32768u && dk <= 32768u && (lk == 32768u || lmax == 1) &&
                     (dk == 32768u || dmax <= 1) && r.pos <= 8 * n;
    }
    if (ok) {
        const uint32_t k = atomicAdd(cnt, 1u);
        if (k < cap) out[k] = b;
    }
}

// k_infl_sym: one workgroup per block of the chain.  The block's output is
// [o0, o1); its literals are in place (out) or, decoded in a candidate's slot,
// at lit + (p - o0) (ParBlk::lit != ~0); its matches (records pos | len << 32 |
// dist << 41, pos relative to o0 - base_hist) are resolved in order through a
// 40 Ki-entry LDS ring of 32-bit symbols: a byte b is 0x80000000 | b, a byte
// before o0 is its output position.  sym[o0, o1) receives the block's
// symbols; a literal-only block from a slot is copied to out instead.  A match
// reaching before the stream's first byte sets *err (inflate.c: "invalid
// distance too far back"; the slot decode could not see it).
struct ParBlk { uint64_t o0, o1, base, moff, lit; uint32_t nm, pad; };
constexpr uint32_t kSWin = 40960;
__global__ __launch_bounds__(64) void k_infl_sym(uint8_t *out, const uint8_t *slots, uint32_t *sym,
                                                 const ParBlk *blks, const uint64_t *mrec_slots,
                                                 const uint64_t *mrec_inplace, uint32_t *err) {
    __shared__ uint32_t W[kSWin];
    const int lane = threadIdx.x;
    const ParBlk B = blks[blockIdx.x];
    const uint32_t o0 = (uint32_t)B.o0, o1 = (uint32_t)B.o1, base = (uint32_t)B.base, nm = B.nm;
    const bool inplace = B.lit == ~0ull;
    const uint8_t *lit = inplace ? out + o0 : slots + B.lit;       // the block's byte p at lit[p - o0]
    if (nm == 0) {
        if (!inplace)
            for (uint32_t p = o0 + (uint32_t)lane; p < o1; p += 64) out[p] = lit[p - o0];
        return;
    }
    const uint64_t *M = (inplace ? mrec_inplace : mrec_slots) + B.moff;
    auto slot = [](uint32_t p) { return p % kSWin; };
    uint32_t loaded = o0, done = o0, mi = 0, mbase = 0, bad = 0;
    uint64_t mreg = (uint32_t)lane < nm ? M[lane] : 0;
    for (uint32_t c0 = o0; c0 < o1 && mi < nm; c0 += kChunk) {
        const uint32_t c1 = c0 + kChunk < o1 ? c0 + kChunk : o1;
        const uint32_t want = c1 + 258 < o1 ? c1 + 258 : o1;
        for (uint32_t p = loaded + (uint32_t)lane; p < want; p += 64) W[slot(p)] = 0x80000000u | lit[p - o0];
        loaded = want;
        __syncthreads();
        while (mi < nm) {
            if (mi - mbase >= 64) {
                mbase = mi;
                mreg = mbase + (uint32_t)lane < nm ? M[mbase + lane] : 0;
            }
            const int k = (int)(mi - mbase);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mreg, k);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mreg >> 32), k);
            const uint32_t pos = base + lo;
            if (pos >= c1) break;
            const uint32_t len = hi & 511u, dist = hi >> 9;
            bad |= dist > pos;
            const uint32_t s0 = pos - dist;
            // every source is before pos (j % dist when the match overlaps itself)
            for (uint32_t j = (uint32_t)lane; j < len; j += 64) {
                const uint32_t s2 = dist >= len ? s0 + j : s0 + j % dist;
                W[slot(pos + j)] = s2 < o0 ? s2 : W[slot(s2)];
            }
            mi++;
        }
        __syncthreads();
        for (uint32_t p = c0 + (uint32_t)lane; p < c1; p += 64) sym[p] = W[slot(p)];
        done = c1;
        __syncthreads();
    }
    // the last chunk's overhang (tails of its matches), then literals only
    for (uint32_t p = done + (uint32_t)lane; p < loaded; p += 64) sym[p] = W[slot(p)];
    for (uint32_t p = loaded + (uint32_t)lane; p < o1; p += 64) sym[p] = 0x80000000u | lit[p - o0];
    if (bad && lane == 0) atomicOr(err, 1u);
}

// k_infl_resolve: one block's symbols into bytes; its references point before
// the block, whose bytes the launches before this one made final.
__global__ __launch_bounds__(256) void k_infl_resolve(uint8_t *out, const uint32_t *sym, uint64_t o0, uint64_t o1) {
    const uint64_t p = o0 + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= o1) return;
    const uint32_t v = sym[p];
    out[p] = (v & 0x80000000u) ? (uint8_t)v : out[v];
}

int launch_infl_scan1(const uint8_t *in, uint64_t n, uint64_t b0, uint64_t b1, uint64_t *list, uint32_t cap,
                      uint32_t *cnt, hipStream_t st) {
    if (b1 <= b0) return 0;
    hipLaunchKernelGGL(k_infl_scan1, dim3((unsigned)((b1 - b0 + 255) / 256)), dim3(256), 0, st, in, n, b0, b1, list,
                       cap, cnt);
    return (int)hipGetLastError();
}
int launch_infl_scan2(const uint8_t *in, uint64_t n, const uint64_t *list, uint32_t count, uint64_t *out,
                      uint32_t cap, uint32_t *cnt, hipStream_t st) {
    if (count == 0) return 0;
    hipLaunchKernelGGL(k_infl_scan2, dim3((count + 255) / 256), dim3(256), 0, st, in, n, list, count, out, cap, cnt);
    return (int)hipGetLastError();
}
int launch_infl_sym(uint8_t *out, const uint8_t *slots, uint32_t *sym, const void *blks, uint32_t nblk,
                    const uint64_t *mrec_slots, const uint64_t *mrec_inplace, uint32_t *err, hipStream_t st) {
    if (nblk == 0) return 0;
    hipLaunchKernelGGL(k_infl_sym, dim3(nblk), dim3(64), 0, st, out, slots, sym, (const ParBlk *)blks, mrec_slots,
                       mrec_inplace, err);
    return (int)hipGetLastError();
}
int launch_infl_resolve(uint8_t *out, const uint32_t *sym, uint64_t o0, uint64_t o1, hipStream_t st) {
    if (o1 <= o0) return 0;
    hipLaunchKernelGGL(k_infl_resolve, dim3((unsigned)((o1 - o0 + 255) / 256)), dim3(256), 0, st, out, sym, o0, o1);
    return (int)hipGetLastError();
}

static int infl_w5() {
    static const int v = [] { const char *e = getenv("ZGPU_INFL_W5"); return e ? atoi(e) : 1; }();
    return v;
}

int launch_inflate_stage(int stage, const InflateJob &job, hipStream_t st) {
    if (job.count == 0) return 0;
    switch (stage) {
    case 0:
        if (job.eidx) hipLaunchKernelGGL(k_inflate_decode<true>, dim3(job.count), dim3(64), 0, st, job);
        else if (infl_w5() == 2 || (infl_w5() == 1 && job.count >= 2048))
            hipLaunchKernelGGL((k_inflate_decode<false, 5>), dim3(job.count), dim3(64), 0, st, job);
        else hipLaunchKernelGGL(k_inflate_decode<false>, dim3(job.count), dim3(64), 0, st, job);
        break;
    case 1: hipLaunchKernelGGL(k_inflate_copy, dim3(job.count), dim3(64), 0, st, job); break;
    case 2: hipLaunchKernelGGL(k_inflate_finish, dim3((job.count + 255) / 256), dim3(256), 0, st, job); break;
    default: return -1;
    }
    return (int)hipGetLastError();
}

}  // namespace zgpu
