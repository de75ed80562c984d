// zgpu_deflate.hip — batched deflate for gfx950, bit-identical to the
// reference deflate.c/trees.c (zlib 1.3.1.1-motley) at the same level.
//
// Pipeline per sub-batch of independent buffers:
//   k_links      1024 thr/buf  hash-chain links: link[p] = distance to the most
//                              recent earlier position with the same 3-byte
//                              hash (UPDATE_HASH/INSERT_STRING, deflate.c:141,160),
//                              from 8 Ki-position chunks radix-sorted by hash in LDS
//   k_count      256 thr/buf   levels 4..9: per position, the number of same-hash
//                              candidates in its window (capped at the chain
//                              budget): the order in which k_match walks a tile
//   k_match      1024 thr/buf  levels 4..9: longest_match (deflate.c:1356-1497) at
//                              EVERY position for the full and the quartered chain
//                              budget, 32 KiB window + links staged in LDS, walks
//                              of similar expected length run side by side
//   k_parse_slow wave/buffer   deflate_slow's lazy parse (deflate.c:1923-2043) over
//                              the per-position results -> symbols + block cuts
//   k_parse_fast wave/buffer   deflate_fast (deflate.c:1824-1915), levels 1..3,
//                              whose insertions depend on the parse
//   k_encode     256 thr/buf   per block: histogram, zlib's Huffman construction
//                              (trees.c:499-706), block-type choice
//                              (trees.c:997-1089), parallel bit packing through an
//                              LDS staging window; zlib/gzip framing + trailer
#include "zgpu_internal.h"
#include <cstdlib>
#include <cstdio>

namespace zgpu {

__constant__ CodeTables c_ct;

// nblocks value a segmented parse leaves for buffers it hands to k_parse_slow
constexpr uint32_t kParseFallback = 0xffffffffu;

// ------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------
__device__ inline uint32_t hash3(uint32_t b0, uint32_t b1, uint32_t b2) {
    return ((b0 & 31u) << 10) ^ (b1 << 5) ^ b2;        // UPDATE_HASH x3, hash_shift 5
}
// UPDATE_HASH x3 for any memLevel: ((b0 << 2s) ^ (b1 << s) ^ b2) & mask; with
// 3s >= hash_bits the rolling hash depends on these three bytes only
__device__ inline uint32_t hashp(uint32_t b0, uint32_t b1, uint32_t b2, const WinP &w) {
    return ((b0 << (2 * w.shift)) ^ (b1 << w.shift) ^ b2) & w.mask;
}
__device__ inline WinP job_win(const DeflateJob &job) { return win_params(job.wbits, job.hbits); }

// unaligned 4-byte read from an LDS byte array (two aligned dwords + alignbyte)
__device__ inline uint32_t lds32u(const uint8_t *base, int off) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(base + (off & ~3));
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(off & 3));
}


// Stage bytes src[start .. start+count) of a buffer of length n into LDS
// (dst[0..count)), zero outside [0, n).  count % 16 == 0, dst 16-B aligned.
// Every lane issues all of its loads before any LDS store, so a tile costs
// about one memory latency instead of one per element.
template <int kThreads, int kMaxChunksPerThread>
__device__ inline void stage_bytes(uint8_t *dst, const uint8_t *src, int64_t start, int count,
                                   int64_t n, int tid) {
    const int nchunks = count >> 4;
    uint4 v[kMaxChunksPerThread];
#pragma unroll
    for (int k = 0; k < kMaxChunksPerThread; k++) {
        const int c = tid + k * kThreads;
        v[k] = make_uint4(0, 0, 0, 0);
        if (c >= nchunks) continue;
        const int64_t x = start + 16ll * c;
        if (x >= 0 && x + 16 <= n) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(src + x);
            const uint32_t sh = (uint32_t)(a & 3u);
            const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
            if (sh == 0) {
                v[k].x = q[0]; v[k].y = q[1]; v[k].z = q[2]; v[k].w = q[3];
            } else {
                const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
                v[k].x = __builtin_amdgcn_alignbyte(d1, d0, sh);
                v[k].y = __builtin_amdgcn_alignbyte(d2, d1, sh);
                v[k].z = __builtin_amdgcn_alignbyte(d3, d2, sh);
                v[k].w = __builtin_amdgcn_alignbyte(d4, d3, sh);
            }
        } else if (x + 16 > 0 && x < n) {
            uint32_t w[4] = {0, 0, 0, 0};
            for (int j = 0; j < 16; j++) {
                const int64_t o = x + j;
                if (o >= 0 && o < n) w[j >> 2] |= (uint32_t)src[o] << (8 * (j & 3));
            }
            v[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxChunksPerThread; k++) {
        const int c = tid + k * kThreads;
        if (c < nchunks) reinterpret_cast<uint4 *>(dst)[c] = v[k];
    }
}

// Stage u32 words src[start .. start+count) (start % 4 == 0, count % 4 == 0)
// into LDS, zero at or beyond `limit`.
template <int kThreads, int kMaxChunksPerThread>
__device__ inline void stage_words(uint32_t *dst, const uint32_t *src, int64_t start, int count,
                                   int64_t limit, int tid) {
    const int nchunks = count >> 2;
    uint4 v[kMaxChunksPerThread];
#pragma unroll
    for (int k = 0; k < kMaxChunksPerThread; k++) {
        const int c = tid + k * kThreads;
        const int64_t x = start + 4ll * c;
        v[k] = make_uint4(0, 0, 0, 0);
        if (c < nchunks && x < limit) {
            if (x + 4 <= limit) v[k] = *reinterpret_cast<const uint4 *>(src + x);
            else {
                v[k].x = src[x];
                if (x + 1 < limit) v[k].y = src[x + 1];
                if (x + 2 < limit) v[k].z = src[x + 2];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxChunksPerThread; k++) {
        const int c = tid + k * kThreads;
        if (c < nchunks) reinterpret_cast<uint4 *>(dst)[c] = v[k];
    }
}

// ------------------------------------------------------------------------
// k_links — link[p] = p - q for the most recent q < p (q != 0, q <= n-3) with
// the same hash, 0 when there is none, the distance exceeds 32767 or p > n-3:
// the chain prev[] would hold.  One 1024-thread workgroup per buffer.
// Positions are taken kLC at a time.  Each chunk's keys (hash << 13 | index)
// are radix-sorted in LDS (two stable 8-bit passes over the 15-bit hash; the
// index in the low bits keeps equal hashes in position order), so the previous
// position with p's hash is the previous key in sorted order, or, for the
// first of its hash in the chunk, head[hash]: INSERT_STRING's head[]
// (deflate.c:160-163) as it stands at the chunk boundary.  head[] holds the
// low 16 bits of positions and is swept every 32 Ki positions like slide_hash
// (deflate.c:187-209), so no live entry is ever 64 Ki positions old.
// ------------------------------------------------------------------------
constexpr int kLC = 8192;
constexpr int kLThreads = 1024;
// the sort key of a position k_links does not insert (SkipSpec): past every
// real hash (hash_bits <= 15 there), so those keys sort last and touch no head
constexpr uint32_t kSkipHash = 1u << 15;
constexpr int kLWaves = kLThreads / 64;
constexpr int kLPer = kLC / kLThreads;

// One stable counting-sort pass of src[0..m) into dst by the 8-bit digit at
// `shift` (dst may be src: every key is in registers before the first
// barrier).  Wave w owns elements w*512 + j*64 + lane; equal digits within a
// wave step are ranked with ballots, counts are scanned digit-major across
// waves, so the scatter keeps element order within a digit.  (Round 5: equal
// digits found through a per-wave table of 256 lane masks, each lane ORing its
// bit into its digit's entry and reading it back, took a quarter of the vector
// instructions and ran slower: 45.7 against 43.4 ms per 4 GiB.)
__device__ __attribute__((always_inline)) inline void links_radix_pass(const uint32_t *src, uint32_t *dst, int m,
                                                                       int shift, uint16_t (*wcnt)[256],
                                                                       int *wsum, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int k = tid; k < kLWaves * 256; k += kLThreads) (&wcnt[0][0])[k] = 0;
    __syncthreads();
    uint32_t key[kLPer], rank[kLPer];
#pragma unroll
    for (int j = 0; j < kLPer; j++) {
        const int e = wave * (64 * kLPer) + j * 64 + lane;
        const bool valid = e < m;
        key[j] = valid ? src[e] : 0u;
        const uint32_t d = (key[j] >> shift) & 0xffu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bb : ~bb;
        }
        rank[j] = 0;
        if (valid) {
            const uint32_t base = wcnt[wave][d];
            rank[j] = base + (uint32_t)__popcll(peers & below);
            if ((peers & below) == 0) wcnt[wave][d] = (uint16_t)(base + __popcll(peers));
        }
    }
    __syncthreads();
    // exclusive scan over (digit, wave), digit-major: thread t owns 4 entries
    int v[4], tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int idx = tid * 4 + k;
        v[k] = wcnt[idx & (kLWaves - 1)][idx >> 4];
        tot += v[k];
    }
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wave; w++) wbase += wsum[w];
    int run = wbase + incl - tot;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int idx = tid * 4 + k;
        wcnt[idx & (kLWaves - 1)][idx >> 4] = (uint16_t)run;
        run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kLPer; j++) {
        const int e = wave * (64 * kLPer) + j * 64 + lane;
        if (e < m) dst[wcnt[wave][(key[j] >> shift) & 0xffu] + rank[j]] = key[j];
    }
    __syncthreads();
}

// kH head entries (1 << hash_bits, <= 32768 in the default layout; 65536 for
// memLevel 9 with kC = 2048-position chunks so head[] fits in LDS)
// kSegs: one workgroup per segment [s0, s1) of job.seg (few large buffers,
// see k_match): a link reaches back at most 32767 positions, so the segment
// starts its chains empty at the chunk t0 <= s0 - 32768 and writes the links
// of [s0, s1) only.
// kGH (job.links_gh: every buffer >= kLinksGhMin bytes, no segments, no
// uploaded chains): head[] holds 32-bit positions in the buffer's key[] region
// (k_count overwrites it next on the same stream) instead of LDS, so it needs
// no sweep and the workgroup takes 56 KiB of LDS instead of 120: two fit a CU
// and one's barriers overlap the other's work.  LDS otherwise: head 64 KiB,
// keys 32 KiB (sorted in place), links 16 KiB (holding the chunk's bytes until
// the keys are made), counts 8 KiB.
template <int kC, int kH, bool kSegs, bool kGH>
__device__ __attribute__((always_inline)) inline void links_body(const DeflateJob &job) {
    static_assert(kC <= kLC && (kC & (kC - 1)) == 0 && kC >= 32, "chunk");
    static_assert(!kGH || (!kSegs && kH == 32768), "global head: the default layout, whole buffers");
    __shared__ uint16_t head[kGH ? 1 : kH];
    __shared__ uint32_t ka[kC];
    __shared__ __attribute__((aligned(16))) uint16_t lk[kC];      // links by chunk index
    uint8_t *const stage = reinterpret_cast<uint8_t *>(lk);       // first the chunk's kC + 16 bytes
    __shared__ uint16_t wcnt[kLWaves][256];
    __shared__ int wsum[kLWaves];
    const int tid = threadIdx.x;
    const uint32_t bi = kSegs ? job.seg[2 * blockIdx.x] : blockIdx.x;
    const uint32_t g = job.first + bi;
    const int64_t n = (int64_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    uint16_t *out = job.link + job.ws_off[bi];
    const WinP wp = job_win(job);
    const int64_t s0 = kSegs ? (int64_t)job.seg[2 * blockIdx.x + 1] : 0;
    const int64_t s1 = kSegs && s0 + (int64_t)job.seg_len < n ? s0 + (int64_t)job.seg_len : n;
    const int64_t t0 = kSegs && s0 > 32768 ? (s0 - 32768) / kC * kC : 0;

    uint32_t *const ghead = kGH ? reinterpret_cast<uint32_t *>(job.key + job.ws_off[bi]) : nullptr;
    // "position t0 - 32768": older than any chain from t0 on reaches
    if constexpr (kGH)
        for (int i = tid; i < kH; i += kLThreads) ghead[i] = (uint32_t)-32768;
    else
        for (int i = tid; i < kH; i += kLThreads) head[i] = (uint16_t)((t0 - 32768) & 0xffff);
    const int64_t lk_n = !kSegs && !kGH && job.lk_head ? (int64_t)job.lk_n : 0;
    for (int64_t c0 = t0; c0 < s1; c0 += kC) {
        __syncthreads();
        if (c0 + kC <= lk_n) continue;                       // links as uploaded (deflate_fast's chains)
        if (kGH) {
        } else if (c0 <= lk_n && job.lk_head) {              // the chains at lk_n: head[] of the uploaded state
            // (entries may lie inside this chunk, below lk_n: no sweep here, the
            // age test is this one)
            const int hn = (int)wp.mask + 1;                 // hash_size entries were uploaded
            for (int i = tid; i < kH; i += kLThreads) {
                const int64_t q = i < hn ? (int64_t)job.lk_head[i] : 0;
                head[i] = (uint16_t)(q != 0 && c0 - q < 32768 ? q & 0xffff : (c0 - 32768) & 0xffff);
            }
            __syncthreads();
        } else if ((c0 & 32767) == 0 && c0 > 0) {            // slide sweep (slide_hash analogue)
            const uint32_t now = (uint32_t)c0;
            for (int i = tid; i < kH; i += kLThreads) {
                const uint32_t age = (now - head[i]) & 0xffffu;
                if (age == 0 || age >= 32768u) head[i] = (uint16_t)((now - 32768u) & 0xffffu);
            }
        }
        stage_bytes<kLThreads, (kC + 16) / 16 / kLThreads + 1>(stage, in, c0, kC + 16, n, tid);
        __syncthreads();
        const int cnt = (int)((n - c0) < kC ? (n - c0) : kC);            // positions in the chunk
        const int m = (int)((n - 2 - c0) < kC ? ((n - 2 - c0) > 0 ? n - 2 - c0 : 0) : kC);   // p <= n-3
        // positions below lk_n keep their uploaded links and are not inserted
        // again: only the chunk's positions from e0 on are keyed and sorted
        const int e0 = lk_n > c0 ? (int)(lk_n - c0) : 0;
        const int ms = m > e0 ? m - e0 : 0;
        for (int e = e0 + tid; e < m; e += kLThreads) {
            uint32_t h = hashp(stage[e], stage[e + 1], stage[e + 2], wp);
            if (job.sk.n) {                                  // huff/rle stretches (SkipSpec)
                const uint32_t p = (uint32_t)c0 + (uint32_t)e;
                for (uint32_t k = 0; k < job.sk.n; k++)
                    if (p >= job.sk.a[k] && p < job.sk.b[k]) h = kSkipHash;
            }
            ka[e - e0] = h << 13 | (uint32_t)e;
        }
        // (the passes' first barrier also ends the reads of stage[] above)
        links_radix_pass(ka, ka, ms, 13, wcnt, wsum, tid);
        links_radix_pass(ka, ka, ms, 21, wcnt, wsum, tid);
        // sorted: ka[i] = hash << 13 | e, hashes ascending, e ascending within a hash
        for (int i = tid; i < ms; i += kLThreads) {
            const uint32_t key = ka[i];
            const uint32_t h = key >> 13, e = key & (kLC - 1);
            const uint32_t p = (uint32_t)c0 + e;
            uint32_t d;
            if (h == kSkipHash) d = 0;                                       // not inserted (SkipSpec)
            else if (i > 0 && (ka[i - 1] >> 13) == h) d = e - (ka[i - 1] & (kLC - 1));
            else if (kGH) d = p - ghead[h];
            else d = (p - head[h]) & 0xffffu;
            lk[e] = (uint16_t)((d != 0 && d <= 32767u && d != p) ? d : 0u);   // position 0 is NIL
        }
        __syncthreads();
        for (int i = tid; i < ms; i += kLThreads) {
            const uint32_t key = ka[i];
            if ((key >> 13) != kSkipHash && (i == ms - 1 || (ka[i + 1] >> 13) != (key >> 13))) {
                if (kGH) ghead[key >> 13] = (uint32_t)c0 + (key & (kLC - 1));
                else head[key >> 13] = (uint16_t)(((uint32_t)c0 + (key & (kLC - 1))) & 0xffffu);
            }
        }
        if (kSegs) {
            const int w0 = s0 > c0 ? (int)(s0 - c0) : 0, w1 = (int)(s1 - c0 < cnt ? s1 - c0 : cnt);
            for (int e = tid + w0; e < w1; e += kLThreads) out[c0 + e] = e < m ? lk[e] : (uint16_t)0;
        } else {
            for (int e = tid + e0; e < cnt; e += kLThreads) out[c0 + e] = e < m ? lk[e] : (uint16_t)0;
        }
    }
}

template <int kC, int kH, bool kSegs = false>
__global__ __launch_bounds__(kLThreads) void k_links(DeflateJob job) {
    links_body<kC, kH, kSegs, false>(job);
}

// two workgroups per CU: at most 64 VGPRs (8 waves per SIMD)
__global__ __launch_bounds__(kLThreads, 8) void k_links_gh(DeflateJob job) {
    links_body<kLC, 32768, false, true>(job);
}

// ------------------------------------------------------------------------
// k_links_seg1 — k_links for one segment [s0, s1) of a sub-batch of few
// large buffers (job.seg; hash_bits <= 15, no uploaded chains, segments of at
// most kLS1Max positions), without walking the 32 Ki window before s0 chunk
// by chunk.  A link needs from before s0 only head[] as it stands there (the
// most recent inserted q < s0 per hash, deflate.c:160-163), and that is an
// order-free maximum: one pass of LDS atomicMax over the window's positions
// (32 per thread, their bytes loaded at once).  The segment then takes kLS1C
// positions at a time as k_links does, head[] holding 32-bit positions + 1
// (0: none, so no sweep).  A lone 64 KiB compress2 walked 5 chunks of 8 Ki
// per segment in a row before this (107 us).
// ------------------------------------------------------------------------
constexpr int kLS1C = 2048;
constexpr int64_t kLS1Max = 16384;
__global__ __launch_bounds__(kLThreads) void k_links_seg1(DeflateJob job) {
    __shared__ uint32_t head[32768];
    __shared__ uint32_t ka[kLS1C];
    __shared__ __attribute__((aligned(16))) uint16_t lk[kLS1C + 16];   // first the chunk's bytes
    uint8_t *const stage = reinterpret_cast<uint8_t *>(lk);
    __shared__ uint16_t wcnt[kLWaves][256];
    __shared__ int wsum[kLWaves];
    const int tid = threadIdx.x;
    const uint32_t bi = job.seg[2 * blockIdx.x];
    const uint32_t g = job.first + bi;
    const int64_t n = (int64_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    uint16_t *out = job.link + job.ws_off[bi];
    const WinP wp = job_win(job);
    const int64_t s0 = (int64_t)job.seg[2 * blockIdx.x + 1];
    const int64_t s1 = s0 + (int64_t)job.seg_len < n ? s0 + (int64_t)job.seg_len : n;
    auto skipped = [&](int64_t p) {                      // huff/rle stretches (SkipSpec): not inserted
        for (uint32_t k = 0; k < job.sk.n; k++)
            if ((uint64_t)p >= job.sk.a[k] && (uint64_t)p < job.sk.b[k]) return true;
        return false;
    };
    for (int i = tid; i < 32768; i += kLThreads) head[i] = 0;
    __syncthreads();
    {   // the window [max(1, s0 - 32767), s0): q is a candidate of some p >= s0 (position 0 is NIL)
        const int64_t w0 = s0 - 32767 > 1 ? s0 - 32767 : 1, w1 = s0 < n - 2 ? s0 : n - 2;
        const int64_t q0 = w0 + 32ll * tid;
        if (q0 < w1) {
            uint32_t wb[9];                              // bytes q0 .. q0 + 35
            const uintptr_t a = reinterpret_cast<uintptr_t>(in + q0);
            const uint32_t sh = (uint32_t)(a & 3u);
            const uint32_t *qw = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
            const int64_t lim = n - q0;                  // bytes of the buffer from q0 on
            uint32_t d[10];
#pragma unroll
            for (int j = 0; j < 10; j++)                 // whole words inside the buffer's allocation
                d[j] = 4ll * j - (int64_t)sh < lim ? qw[j] : 0u;
#pragma unroll
            for (int j = 0; j < 9; j++) wb[j] = sh ? __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh) : d[j];
#pragma unroll
            for (int j = 0; j < 32; j++) {
                const int64_t q = q0 + j;
                if (q >= w1) break;
                const uint32_t b0 = (wb[j >> 2] >> (8 * (j & 3))) & 0xffu;
                const uint32_t b1 = (wb[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xffu;
                const uint32_t b2 = (wb[(j + 2) >> 2] >> (8 * ((j + 2) & 3))) & 0xffu;
                if (job.sk.n && skipped(q)) continue;
                atomicMax(&head[hashp(b0, b1, b2, wp)], (uint32_t)q + 1u);
            }
        }
    }
    for (int64_t c0 = s0; c0 < s1; c0 += kLS1C) {
        __syncthreads();
        stage_bytes<kLThreads, 1>(stage, in, c0, ((kLS1C + 16) / 16) * 16, n, tid);
        __syncthreads();
        const int cnt = (int)((s1 - c0) < kLS1C ? (s1 - c0) : kLS1C);
        const int m = (int)((n - 2 - c0) < cnt ? ((n - 2 - c0) > 0 ? n - 2 - c0 : 0) : cnt);   // p <= n-3
        for (int e = tid; e < m; e += kLThreads) {
            uint32_t h = hashp(stage[e], stage[e + 1], stage[e + 2], wp);
            if (job.sk.n && skipped(c0 + e)) h = kSkipHash;
            ka[e] = h << 11 | (uint32_t)e;
        }
        links_radix_pass(ka, ka, m, 11, wcnt, wsum, tid);
        links_radix_pass(ka, ka, m, 19, wcnt, wsum, tid);
        for (int i = tid; i < m; i += kLThreads) {
            const uint32_t key = ka[i];
            const uint32_t h = key >> 11, e = key & (kLS1C - 1);
            const int64_t p = c0 + e;
            int64_t dd;
            if (h == kSkipHash) dd = 0;
            else if (i > 0 && (ka[i - 1] >> 11) == h) dd = e - (ka[i - 1] & (kLS1C - 1));
            else dd = head[h] ? p - ((int64_t)head[h] - 1) : 0;
            lk[e] = (uint16_t)(dd > 0 && dd <= 32767 && dd != p ? dd : 0);     // position 0 is NIL
        }
        __syncthreads();
        for (int i = tid; i < m; i += kLThreads) {
            const uint32_t key = ka[i];
            if ((key >> 11) != kSkipHash && (i == m - 1 || (ka[i + 1] >> 11) != (key >> 11)))
                head[key >> 11] = (uint32_t)(c0 + (key & (kLS1C - 1))) + 1u;
        }
        for (int e = tid; e < cnt; e += kLThreads) out[c0 + e] = e < m ? lk[e] : (uint16_t)0;
    }
}

// ------------------------------------------------------------------------
// k_count — the order in which k_match walks a tile's positions.  For every
// position p: the number of earlier positions q in (p - MAX_DIST, p) with the
// same hash, i.e. the candidates a chain walk from p can visit, capped at the
// level's chain budget (walks stop there) and compressed to a byte.  The
// sliding-window counts live in LDS, two u16 counters per word, updated with
// atomics: the position leaving the window is subtracted, p is added and the
// value before the add is p's count.  Within one 64-position step the atomics
// are unordered, so a count may be off by the step's own same-hash positions:
// the key is a scheduling hint that orders walks by expected length (similar
// lengths share a wave) and decides no result.
// ------------------------------------------------------------------------
constexpr int kCntStage = 4096;
// 1024 threads (16 waves) per buffer: the LDS atomics' latency is hidden by
// more waves (k_count 14.3 -> 9.5 ms per 4 GiB L6 sub-batch); the wider
// unordered step perturbs the hint slightly (k_match +1.7 ms), net -2.7 ms
// (profiles/r03n_ab_links_count.log).  Prefetching the next stage into
// registers gained nothing here or in k_links.
constexpr int kCntThreads = 1024;

__device__ __attribute__((always_inline)) inline uint32_t walk_key(uint32_t c, uint32_t chain) {
    if (c > chain) c = chain;
    if (c < 128) return c;
    const uint32_t k = 128 + ((c - 128) >> 5);
    return k < 255 ? k : 255;
}

// 16 waves per buffer; thread t takes positions t, t + 1024, ... of each staged
// 4 KiB, without barriers between them (their order only perturbs the hint).
// kSegs: one workgroup per segment [s0, s1) of job.seg, counting from the
// stage at or before s0 - MAX_DIST (the window of s0) and writing [s0, s1).
template <bool kSegs = false>
__global__ __launch_bounds__(kCntThreads) void k_count(DeflateJob job) {
    __shared__ uint32_t cnt[16384];
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kCntStage + 16];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[kCntStage + 16];
    const int tid = threadIdx.x;
    const uint32_t bi = kSegs ? job.seg[2 * blockIdx.x] : blockIdx.x;
    const uint32_t g = job.first + bi;
    const int64_t n = (int64_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    uint8_t *key = job.key + job.ws_off[bi];
    const uint32_t chain = job.cfg.chain;
    const int64_t s0 = kSegs ? (int64_t)job.seg[2 * blockIdx.x + 1] : 0;
    const int64_t s1 = kSegs && s0 + (int64_t)job.seg_len < n ? s0 + (int64_t)job.seg_len : n;
    const int64_t c0 = kSegs && s0 > kMaxDist ? (s0 - kMaxDist) / kCntStage * kCntStage : 0;
    for (int i = tid; i < 16384; i += kCntThreads) cnt[i] = 0;
    int64_t tstart = c0;
    if (kSegs && s0 > 0) {
        // the window of s0, [s0 - MAX_DIST, s0), counted in one pass (32 positions per thread, their
        // bytes loaded at once) instead of stage after stage from c0 (a lone 64 KiB compress2: 9 stages
        // per 4 KiB segment); the stages then run from s0, as the window slides over counted positions
        static_assert(kMaxDist <= 32 * kCntThreads, "one pass");
        __syncthreads();
        const int64_t w0 = s0 - kMaxDist > 1 ? s0 - kMaxDist : 1;    // s0's first stage subtracts s0 - MAX_DIST
        const int64_t q0 = w0 + 32ll * tid;
        if (q0 < s0) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(in + q0);
            const uint32_t sh = (uint32_t)(a & 3u);
            const uint32_t *qw = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
            const int64_t lim = n - q0;
            uint32_t d[10], wb[9];
#pragma unroll
            for (int j = 0; j < 10; j++) d[j] = 4ll * j - (int64_t)sh < lim ? qw[j] : 0u;
#pragma unroll
            for (int j = 0; j < 9; j++) wb[j] = sh ? __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh) : d[j];
#pragma unroll
            for (int j = 0; j < 32; j++) {
                const int64_t q = q0 + j;
                if (q >= s0 || q + 3 > n) break;
                const uint32_t h = hash3((wb[j >> 2] >> (8 * (j & 3))) & 0xffu,
                                         (wb[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xffu,
                                         (wb[(j + 2) >> 2] >> (8 * ((j + 2) & 3))) & 0xffu);
                atomicAdd(&cnt[h >> 1], 1u << ((h & 1u) * 16));
            }
        }
        tstart = s0;
    }
    for (int64_t t0 = tstart; t0 < s1; t0 += kCntStage) {
        __syncthreads();
        stage_bytes<kCntThreads, (kCntStage + 16) / 16 / kCntThreads + 1>(s_in, in, t0, kCntStage + 16, n, tid);
        stage_bytes<kCntThreads, (kCntStage + 16) / 16 / kCntThreads + 1>(s_out, in, t0 - kMaxDist,
                                                                         kCntStage + 16, n, tid);
        __syncthreads();
        const int64_t tend = (t0 + kCntStage < n) ? t0 + kCntStage : n;
        for (int64_t p = t0 + tid; p < tend; p += kCntThreads) {
            const int j = (int)(p - t0);
            const int64_t q = p - kMaxDist;                   // leaves p's window
            if (q >= 1 && q >= c0 && q + 3 <= n) {              // (counted: q >= c0, or in s0's window)
                const uint32_t h = hash3(s_out[j], s_out[j + 1], s_out[j + 2]);
                atomicSub(&cnt[h >> 1], 1u << ((h & 1u) * 16));
            }
            uint32_t k = 0;
            if (p >= 1 && p + 3 <= n) {
                const uint32_t h = hash3(s_in[j], s_in[j + 1], s_in[j + 2]);
                const uint32_t old = atomicAdd(&cnt[h >> 1], 1u << ((h & 1u) * 16));
                k = walk_key((old >> ((h & 1u) * 16)) & 0xffffu, chain);
            }
            if (!kSegs || (p >= s0 && p < s1)) key[p] = (uint8_t)k;
        }
    }
}

// ------------------------------------------------------------------------
// k_match — levels 4..9.  One 1024-thread workgroup per buffer walks tiles of
// kMT positions.  LDS holds input bytes [ts-32768, ts+kMT+272) and links
// [ts-32768, ts+kMT); between tiles both slide down by kMT.  Every position's
// walk follows longest_match exactly (quick reject, first strictly longer
// match wins, stop at nice, chain budget, limit = max(p-MAX_DIST, 0)), records
// the result after chain/4 candidates too, and stores (len<<16 | dist).
// ------------------------------------------------------------------------
constexpr int kMW = 32768, kMT = 4096, kMPad = 272;
static_assert(kMT == (int)kMatchTile, "segment starts (host) must be k_match tile boundaries");
constexpr int kME = kMW + kMT + kMPad;                     // 37136 words = 148.5 KiB
constexpr int kMatchThreads = 1024;

// LDS word for window position q:  link(q) | byte[q] << 16 | byte[q+1] << 24.
// One ds_read_b32 yields both the chain link and the first two bytes of a
// candidate; the quick-reject pair at best-1 is the high half of word best-1.
__device__ inline uint32_t get4(const uint32_t *E, int i) {      // bytes i..i+3
    return (E[i] >> 16) | (E[i + 2] & 0xffff0000u);
}

// "no predecessor" (link 0) is stored as 0xffff in LDS: m - 0xffff is always
// <= the walk's limit, so the chain-end test folds into the limit test.
__device__ inline uint32_t nil_link(uint32_t l) { return l ? l : 0xffffu; }

// Tile prefetch: what thread t writes into the LDS window for a tile, loaded
// from HBM into registers one tile ahead (while the previous tile's walks
// run): bytes ts+4t .. ts+4t+4 (words 4t..4t+3), for t < kMPad/4 the pad
// words kMT+4t.., the links of positions ts+4t.., and the walk keys of
// positions ts+t+1024u (u = 0..3).
static_assert(kMT / 4 == kMatchThreads && kMPad % 4 == 0 && kMPad / 4 <= kMatchThreads && kMW % 4 == 0,
              "tile prefetch: 4 words per thread");
struct TilePre {
    uint32_t b[4];        // packed word bytes (byte[q] | byte[q+1] << 8) for words 4t+u
    uint32_t pb[4];       // same for pad words kMT + 4t + u (t < kMPad / 4)
    uint32_t lk[4];       // links (raw, 0 = none)
    uint32_t key[4];
};

__device__ __attribute__((always_inline)) inline uint32_t ldb(const uint8_t *in, int64_t q, int64_t n) {
    return (q >= 0 && q < n) ? (uint32_t)in[q] : 0u;
}

__device__ __attribute__((always_inline)) inline void tile_prefetch(TilePre &P, int64_t ts, int64_t n,
                                                                    const uint8_t *in, const uint16_t *L,
                                                                    const uint8_t *K, int tid) {
    const int64_t q0 = ts + 4 * tid;
    uint32_t x[5];
#pragma unroll
    for (int u = 0; u < 5; u++) x[u] = ldb(in, q0 + u, n);
#pragma unroll
    for (int u = 0; u < 4; u++) P.b[u] = x[u] | x[u + 1] << 8;
    if (tid < kMPad / 4) {
        const int64_t q1 = ts + kMT + 4 * tid;
#pragma unroll
        for (int u = 0; u < 5; u++) x[u] = ldb(in, q1 + u, n);
#pragma unroll
        for (int u = 0; u < 4; u++) P.pb[u] = x[u] | x[u + 1] << 8;
    }
    if (q0 + 4 <= n) {
        const uint2 v = *reinterpret_cast<const uint2 *>(L + q0);   // 8-B aligned: ws_off % 64 == 0
        P.lk[0] = v.x & 0xffffu; P.lk[1] = v.x >> 16; P.lk[2] = v.y & 0xffffu; P.lk[3] = v.y >> 16;
    } else {
#pragma unroll
        for (int u = 0; u < 4; u++) P.lk[u] = q0 + u < n ? (uint32_t)L[q0 + u] : 0u;
    }
    if (K) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t q = ts + tid + u * kMatchThreads;
            P.key[u] = q < n ? (uint32_t)K[q] : 0u;
        }
    }
}

// Tile load from the prefetched registers: slide the window down by kMT words
// (later tiles), then write words kMW.. of the new tile and its pad.
// kIdx: the low half of a word is the LDS word index of the predecessor (0:
// none, or older than the window -- index 0 is always beyond a walk's limit),
// so a chain step needs no subtraction; sliding lowers every index by kMT,
// saturating at 0 (one packed 16-bit subtract per word).
// Otherwise the low half is the distance to it (0xffff: none, nil_link).
__device__ __attribute__((always_inline)) inline uint32_t slide_idx(uint32_t w) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const us2 v = __builtin_bit_cast(us2, w);
    const us2 d = {(unsigned short)kMT, (unsigned short)0};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(v, d));
}
template <bool kIdx = false>
__device__ __attribute__((always_inline)) inline void tile_store(uint32_t *E, const TilePre &P, int64_t ts,
                                                                 int tid) {
    if (ts == 0) {
        for (int i = tid; i < kMW; i += kMatchThreads) E[i] = 0;
    } else {
        // kMW/4 uint4 chunks, thread t moves chunks t (mod kMatchThreads) in
        // increasing order: no chunk is overwritten before it is read
        uint4 *dE = reinterpret_cast<uint4 *>(E);
        for (int c = tid; c < kMW / 4; c += kMatchThreads) {
            uint4 v = dE[c + kMT / 4];
            if (kIdx) v = make_uint4(slide_idx(v.x), slide_idx(v.y), slide_idx(v.z), slide_idx(v.w));
            dE[c] = v;
        }
        __syncthreads();
    }
    const int w0 = kMW + 4 * tid;
    uint4 v;
    if (kIdx) {
        // masked to the low half: a position no chain reaches may carry any
        // link (a deflate_fast window's uninserted positions keep stale prev[]
        // entries), which must not spill into its bytes
        v.x = P.b[0] << 16 | (P.lk[0] ? ((uint32_t)(w0 + 0) - P.lk[0]) & 0xffffu : 0u);
        v.y = P.b[1] << 16 | (P.lk[1] ? ((uint32_t)(w0 + 1) - P.lk[1]) & 0xffffu : 0u);
        v.z = P.b[2] << 16 | (P.lk[2] ? ((uint32_t)(w0 + 2) - P.lk[2]) & 0xffffu : 0u);
        v.w = P.b[3] << 16 | (P.lk[3] ? ((uint32_t)(w0 + 3) - P.lk[3]) & 0xffffu : 0u);
    } else {
        v.x = P.b[0] << 16 | nil_link(P.lk[0]);
        v.y = P.b[1] << 16 | nil_link(P.lk[1]);
        v.z = P.b[2] << 16 | nil_link(P.lk[2]);
        v.w = P.b[3] << 16 | nil_link(P.lk[3]);
    }
    *reinterpret_cast<uint4 *>(E + w0) = v;
    if (tid < kMPad / 4)
        *reinterpret_cast<uint4 *>(E + kMW + kMT + 4 * tid) =
            make_uint4(P.pb[0] << 16, P.pb[1] << 16, P.pb[2] << 16, P.pb[3] << 16);
}

// The compare: the first 16 scan bytes are held in registers (loaded once per
// walk); a hit reads the candidate word by word (most compares end in the
// first 4-8 bytes) and longer matches continue 16 bytes (both sides) per LDS
// round trip.
struct Scan16 { uint32_t s0, s1, s2, s3; };


// ------------------------------------------------------------------------
// The deferred-compare walk.  A lane whose candidate passes the quick reject
// would compare at once while the other 63 lanes of its wave wait (3.4 % of
// the steps compare, yet 86 % of a wave's steps would run the compare code).
// The compare is therefore taken out of the step:
//   1. the first kD0 candidates of every walk are compared by the whole wave
//      together (all lanes start their walks at the same time), so the walk
//      goes on with the best the chain's head gives -- that is where most
//      improvements happen;
//   2. the step tests the quick reject against that (stale) best and, on a
//      pass, pushes the candidate into a kDQ-deep per-lane queue; a stale best
//      is never larger than the true one, so the queue holds every candidate
//      the exact walk would compare (and some it would reject);
//   3. when some lane's queue is (nearly) full, at the chain/4 budget snapshot
//      and at the end, the wave empties the queues together, oldest first,
//      applying longest_match's rule (a strictly longer match wins, stop at
//      nice) with the true running best: the result equals longest_match's
//      (deflate.c:1417-1497) for every position.  A lane that reaches nice in
//      a flush drops its later entries and steps.
// The measured alternatives (queue depths 3..8, 1..4 steps per exit test, a
// one-integer quick reject, two walks per lane, flushes inside the step loop,
// ...) are recorded in DESIGN.md 4.3; only the fastest ships.
// ------------------------------------------------------------------------
constexpr int kD0 = 2;      // leading candidates compared by the whole wave
constexpr int kDQ = 6;      // deferred-compare queue depth (even: flushes take entries in pairs)
constexpr int kDU = 3;      // chain steps per exit test
__device__ inline uint32_t ufl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// bytes i..i+3 from the packed words: one byte permute (v_perm_b32) of the
// high halves of E[i] and E[i+2]
__device__ __attribute__((always_inline)) inline uint32_t get4p(const uint32_t *E, int i) {
    return __builtin_amdgcn_perm(E[i + 2], E[i], 0x07060302u);
}

// lowest set bit of x, or 0xffffffff for x == 0 (v_ffbl_b32's own result)
__device__ __attribute__((always_inline)) inline uint32_t ffbl(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// index of the first differing byte of two 16-byte strings given as four
// xor words, 16 if none.  ffbl(x_j) | 32 j is 32 j + ctz(x_j), or stays
// 0xffffffff when x_j == 0, so one min over the four needs no branch.
__device__ __attribute__((always_inline)) inline int diff16(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    const uint32_t b = min(min(ffbl(x0), ffbl(x1) | 32u), min(ffbl(x2) | 64u, ffbl(x3) | 96u));
    return (int)(min(b, 128u) >> 3);
}

// LCP of the scan at s and the candidate at m, capped at maxcmp: 16 bytes per
// LDS round trip (all reads of a round issued before any test).
__device__ __attribute__((always_inline)) inline int lcp16(const uint32_t *E, int m, int s, const Scan16 &S,
                                                           int maxcmp) {
    int k = diff16(get4p(E, m) ^ S.s0, get4p(E, m + 4) ^ S.s1, get4p(E, m + 8) ^ S.s2, get4p(E, m + 12) ^ S.s3);
    if (k >= 16) {
        while (k < maxcmp) {
            const int r = diff16(get4p(E, m + k) ^ get4p(E, s + k), get4p(E, m + k + 4) ^ get4p(E, s + k + 4),
                                 get4p(E, m + k + 8) ^ get4p(E, s + k + 8), get4p(E, m + k + 12) ^ get4p(E, s + k + 12));
            k += r;
            if (r < 16) break;
        }
    }
    return k < maxcmp ? k : maxcmp;
}
// lcp16 of two candidates m1, m0 against the same scan: the first 16 bytes of
// both in one round trip
__device__ __attribute__((always_inline)) inline void lcp16x2(const uint32_t *E, int m1, int m0, int s,
                                                              const Scan16 &S, int maxcmp, int &l1, int &l0) {
    const uint32_t a0 = get4p(E, m1) ^ S.s0, a1 = get4p(E, m1 + 4) ^ S.s1, a2 = get4p(E, m1 + 8) ^ S.s2,
                   a3 = get4p(E, m1 + 12) ^ S.s3;
    const uint32_t b0 = get4p(E, m0) ^ S.s0, b1 = get4p(E, m0 + 4) ^ S.s1, b2 = get4p(E, m0 + 8) ^ S.s2,
                   b3 = get4p(E, m0 + 12) ^ S.s3;
    int k1 = diff16(a0, a1, a2, a3), k0 = diff16(b0, b1, b2, b3);
    auto more = [&](int m, int k) {
        while (k < maxcmp) {
            const int r = diff16(get4p(E, m + k) ^ get4p(E, s + k), get4p(E, m + k + 4) ^ get4p(E, s + k + 4),
                                 get4p(E, m + k + 8) ^ get4p(E, s + k + 8), get4p(E, m + k + 12) ^ get4p(E, s + k + 12));
            k += r;
            if (r < 16) break;
        }
        return k;
    };
    if (k1 >= 16) k1 = more(m1, k1);
    if (k0 >= 16) k0 = more(m0, k0);
    l1 = k1 < maxcmp ? k1 : maxcmp;
    l0 = k0 < maxcmp ? k0 : maxcmp;
}
__device__ inline uint32_t match_rec(int best, int s4, int bpos4) {
    return best >= kMinMatch ? (((uint32_t)best << 16) | (uint32_t)((s4 - bpos4) >> 2)) : 0u;
}


#ifdef ZGPU_MATCH_STATS
// statistics build only (tools/match_stats.py): per-lane counters in registers,
// added to g_mstat once per thread at the end of k_match
__device__ unsigned long long g_mstat[8];
// MSTAT: every lane adds v; MSTATW: the wave adds v once (its first active lane)
#define MSTAT(i, v) atomicAdd(&g_mstat[i], (unsigned long long)(v))
#define MSTATW(i, v) do { if ((int)__lane_id() == __builtin_ctzll(__ballot(1))) atomicAdd(&g_mstat[i], (unsigned long long)(v)); } while (0)
extern "C" int zgpu_match_stats_read(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mstat), sizeof(g_mstat)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_mstat), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// The walk state between flushes: candidate m (byte address m4 = 4 m) has its
// two words em (link index, bytes m, m+1) and eb (bytes m+best-1, m+best)
// loaded; the queue holds byte addresses, newest in q[0].
struct DWQ {
    int m4, limit4, be4, occ;
    int q[kDQ];
    uint32_t em, eb, scan01, scanE;
};
// Steps every lane of the wave until the uniform budget count `end` is
// reached, some lane's queue is nearly full or no lane has a candidate left.
// kDU steps per exit test: the loop's ballots and budget compare are scalar
// work every wave of the CU shares one scalar unit for.  A lane whose walk has
// ended keeps stepping harmlessly (links only go back, so it stays past its
// limit and queues nothing); the queue test fires kDU - 1 entries early so
// that kDU steps cannot overflow it, and single steps are taken when fewer
// than kDU are left of the budget, so the stops are those of one step per
// test.  `count` is wave-uniform (all lanes start their walks together).
__device__ __attribute__((always_inline)) inline void dwq_steps(DWQ &w, const char *Eb, uint32_t &count,
                                                                uint32_t end) {
    auto step = [&]() {
        const int m4n = (int)((w.em << 2) & 0x3fffcu);
        const uint32_t emn = *reinterpret_cast<const uint32_t *>(Eb + m4n);
        const uint32_t ebn = *reinterpret_cast<const uint32_t *>(Eb + m4n + w.be4);
        const bool pass = (w.m4 > w.limit4) & ((w.em >> 16) == w.scan01) & ((w.eb >> 16) == w.scanE);
#pragma unroll
        for (int j = kDQ - 1; j > 0; j--) w.q[j] = pass ? w.q[j - 1] : w.q[j];
        w.q[0] = pass ? w.m4 : w.q[0];
        w.occ += pass ? 1 : 0;
        w.m4 = m4n;
        w.em = emn;
        w.eb = ebn;
    };
    for (;;) {
        if (end - count >= (uint32_t)kDU) {
#pragma unroll
            for (int u = 0; u < kDU; u++) step();
            count += kDU;
        } else {
            step();
            count += 1;
        }
        const uint64_t walkers = __ballot(w.m4 > w.limit4), full = __ballot(w.occ >= kDQ - (kDU - 1));
        if (count >= end || walkers == 0 || full != 0) break;
    }
}

// One position's longest_match with deferred compares.  Every lane of the
// wave that took a position calls this together (the flushes are wave-wide
// decisions taken with ballots).
// Out receives the results: out.full(rec, exact) -- the walk's result with the
// budget cfg.chain, exact = the walk ended before the budget (chain end, the
// limit or nice), so a longer budget gives the same result -- and, with
// want_q, out.quart(rec) after chain/4 candidates.
// k_match's records: rfull[p] = the full-budget result; where the quartered
// budget's result differs (16.6 % of positions at level 6 on the Silesia-style
// mix, 1.2 % at level 9) bit kQDiff is set and rquart[p] holds it, and rquart
// is not written elsewhere (round 6, VERDICT r5 #2: the parse reads one record
// per decision, the walks write ~4 B per position instead of 8).
constexpr uint32_t kQDiff = 1u << 31;
struct MOutRQ {
    uint32_t *rf, *rq;
    int64_t p;
    mutable uint32_t q = 0;
    mutable bool hq = false;
    __device__ __attribute__((always_inline)) inline void full(uint32_t r, bool) const {
        const bool d = hq && q != r;
        if (d) rq[p] = q;
        rf[p] = d ? r | kQDiff : r;
    }
    __device__ __attribute__((always_inline)) inline void quart(uint32_t r) const {
        q = r;
        hq = true;
    }
    __device__ __attribute__((always_inline)) inline void steps(uint32_t) const {}
};
template <typename Out>
__device__ __attribute__((always_inline)) inline void dwq_walk(const uint32_t *E, int64_t p, int64_t B, int64_t n,
                                                               const LevelCfg &cfg, const Out &out,
                                                               int want_q, int64_t max_dist) {
    const int s = (int)(p - B);
    const uint32_t e0 = E[s];
    const uint32_t d0 = (e0 & 0xffffu) ? (uint32_t)s - (e0 & 0xffffu) : 0xffffu;
    if (d0 > (uint32_t)max_dist) {                 // deflate.c:1955: strstart - hash_head <= MAX_DIST
        if (want_q) out.quart(0u);
        out.full(0u, true);
        return;
    }
    const int64_t labs = p > max_dist ? p - max_dist : 0;
    const int limit4 = (int)(labs - B) * 4;
    const int64_t rem = n - p;
    const int nice = rem < cfg.nice ? (int)rem : cfg.nice;
    const int maxcmp = rem < kMaxMatch ? (int)rem : kMaxMatch;
    const uint32_t chain = (uint32_t)cfg.chain;
    const uint32_t qc = want_q ? chain >> 2 : chain;
    const int s4 = s * 4;
    const Scan16 S{get4(E, s), get4(E, s + 4), get4(E, s + 8), get4(E, s + 12)};
    int best = kMinMatch - 1, bpos4 = 0;
    int m4 = (int)(e0 & 0xffffu) * 4;
    uint32_t count = 0;
    bool walking = true;
    bool need_q = want_q != 0;
#pragma unroll
    for (int k = 0; k < kD0; k++) {                 // the chain's head, compared by the whole wave
        if (walking) {
            const int m = m4 >> 2;
            const uint32_t em = E[m];
            const int len = lcp16(E, m, s, S, maxcmp);
            if (len > best) { best = len; bpos4 = m4; }
            count++;
            const int m4n = (int)((em & 0xffffu) << 2);
            if (best >= nice || m4n <= limit4 || count >= chain) walking = false;
            if (need_q && count == qc && walking) {
                out.quart(match_rec(best, s4, bpos4));
                need_q = false;
            }
            m4 = m4n;
        }
    }
    if (!walking) {
        const uint32_t r = match_rec(best, s4, bpos4);
        if (need_q) out.quart(r);
        out.steps(count);
        out.full(r, best >= nice || m4 <= limit4);
        return;
    }
    const char *Eb = reinterpret_cast<const char *>(E);
#ifdef ZGPU_MATCH_STATS
    MSTATW(4, 1);                                      // wave walk groups past the head compares
    MSTAT(6, 1);                                       // lane walks past the head compares
#endif
    DWQ w;
    w.m4 = m4;
    w.limit4 = limit4;
    w.be4 = (best - 1) * 4;
    w.occ = 0;
#pragma unroll
    for (int j = 0; j < kDQ; j++) w.q[j] = 0;
    w.scan01 = e0 >> 16;
    w.scanE = E[s + best - 1] >> 16;
    w.em = *reinterpret_cast<const uint32_t *>(Eb + m4);
    w.eb = *reinterpret_cast<const uint32_t *>(Eb + m4 + w.be4);
    count = ufl(count);
    for (;;) {
        const uint32_t end = count < qc ? qc : chain;
        const int best0 = best;
        dwq_steps(w, Eb, count, end);
        walking = w.m4 > limit4 && count < chain;
#ifdef ZGPU_MATCH_STATS
        MSTATW(0, 1);                                  // wave flushes
        MSTAT(2, (uint64_t)w.occ);                     // entries compared in flushes
        MSTAT(3, 1);                                   // lane-flushes (lanes taking part)
#endif
        // every entry, oldest first: entry j (< occ) is the (occ - j)-th oldest
        // two entries per round (slots j, j - 1): the first 16 bytes of both
        // candidates are read in one LDS round trip.  A flush used to take one
        // round per slot, 3.6 rounds per flush with 7 of 64 lanes comparing on
        // average (tools/match_stats.py): 326 -> 320 ms per 4 GiB L6 launch.
        static_assert(kDQ % 2 == 0, "entries are taken in pairs");
#pragma unroll
        for (int j = kDQ - 1; j >= 1; j -= 2) {
            const bool c1 = j < w.occ, c0 = j - 1 < w.occ;    // c1 implies c0
            if (__ballot(c0) != 0) {
                int l1, l0;
                lcp16x2(E, c1 ? w.q[j] >> 2 : 0, c0 ? w.q[j - 1] >> 2 : 0, s, S, maxcmp, l1, l0);
#ifdef ZGPU_MATCH_STATS
                MSTATW(1, 1);                                 // wave rounds of the flushes
                MSTAT(5, (c1 && l1 >= 16 ? 1 : 0) + (c0 && l0 >= 16 ? 1 : 0));   // compares past 16 bytes
#endif
                if (c1 && l1 > best) {
                    best = l1;
                    bpos4 = w.q[j];
                    if (l1 >= nice) { walking = false; w.occ = 0; }
                }
                if (c0 && j - 1 < w.occ && l0 > best) {
                    best = l0;
                    bpos4 = w.q[j - 1];
                    if (l0 >= nice) { walking = false; w.occ = 0; }
                }
            }
        }
        w.occ = 0;
        const bool fin = !walking;
        if (need_q && (count >= qc || fin)) {          // deflate.c:1390-1392 (chain >>= 2)
            out.quart(match_rec(best, s4, bpos4));
            need_q = false;
        }
        if (fin) break;
        if (best != best0) {                           // the quick reject now tests the new best
            w.be4 = (best - 1) * 4;
            w.scanE = E[s + best - 1] >> 16;
            w.eb = *reinterpret_cast<const uint32_t *>(Eb + w.m4 + w.be4);
        }
    }
    out.steps(count);
    out.full(match_rec(best, s4, bpos4), best >= nice || w.m4 <= limit4);
}


// The deflate(flush) calls of a flush job (DeflateJob::fl_pos/fl_type): the
// parse runs as if the input ended at the next flush position (deflate() has
// not seen more), and when it stands there with the window drained the call's
// flush is acted on (deflate.c:2030-2042, :1211-1233).  Positions are read
// uniformly (every lane the same value).
struct FlushEv {
    const uint64_t *pos;
    const uint32_t *type;
    const uint64_t *aux;
    uint32_t n, i;
    // a flush call's input ends at p
    __device__ inline bool at(int64_t p) const {
        return i < n && kind() != 0 && kind() != kEvPause && kind() != kEvPrime && (int64_t)ufl64(pos[i]) == p;
    }
    // a deflatePrime call right after the stop just passed (kEvPrime)
    __device__ inline bool prime() const { return i < n && kind() == kEvPrime; }
    __device__ inline uint32_t prime_arg() const { return (uint32_t)ufl64(aux[i]); }
    // the end of a Z_NO_FLUSH call's input, reached: all of it read (E == lim)
    __device__ inline bool stop_at(int64_t e, int64_t lim) const { return i < n && kind() == 0 && e == lim; }
    // the block just flushed ends where a call stopped on a full output buffer
    __device__ inline bool pause_at(int64_t x) const {
        return i < n && kind() == kEvPause && (int64_t)ufl64(aux[i]) == x;
    }
    __device__ inline uint32_t kind() const { return (uint32_t)__builtin_amdgcn_readfirstlane((int)type[i]); }
    __device__ inline int64_t limit(int64_t end) const { return i < n ? (int64_t)ufl64(pos[i]) : end; }
    __device__ static inline uint64_t ufl64(uint64_t v) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
        return ((uint64_t)hi << 32) | lo;
    }
};
__device__ inline FlushEv flush_ev(const DeflateJob &job) { return FlushEv{job.fl_pos, job.fl_type, job.fl_aux, job.nfl, 0}; }

// first flush position > p: the end of the input deflate() has seen when the
// parse decides at p (longest_match's nice / lookahead clamp), else n.  The
// ends of Z_NO_FLUSH calls do not count: the parse decides no position within
// MIN_LOOKAHEAD of one before the next call's input is there (DeflateJob::mlim).
__device__ inline int64_t flush_limit(const DeflateJob &job, int64_t p, int64_t n) {
    uint32_t lo = 0, hi = job.nmlim;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((int64_t)job.mlim[mid] > p) hi = mid;
        else lo = mid + 1;
    }
    return lo < job.nmlim ? (int64_t)job.mlim[lo] : n;
}

// configuration rows in force at decision point p: the number of changes at
// or before p (DeflateJob::cfg_pos), 0 for none
__device__ inline uint32_t cfg_count(const DeflateJob &job, int64_t p) {
    uint32_t k = 0;
    while (k < job.ncfg && (int64_t)job.cfg_pos[k] <= p) k++;
    return k;
}
__device__ inline LevelCfg cfg_row(const DeflateJob &job, uint32_t k) { return k ? job.cfg_tab[k - 1] : job.cfg; }

template <bool kEv = false, bool kSegs = false>
__global__ __launch_bounds__(kMatchThreads) void k_match(DeflateJob job, int want_q) {
    constexpr int kSortBuckets = 64;
    __shared__ __attribute__((aligned(16))) uint32_t E[kME];
    __shared__ int next_i;
    __shared__ uint16_t s_perm[kMT];
    __shared__ int s_hist[kSortBuckets], s_base[kSortBuckets];
    const int tid = threadIdx.x;
    // one workgroup per buffer, or -- a sub-batch of few large buffers -- per
    // segment [s0, s1) of a buffer (job.seg: buffer, start): a position's walk
    // needs only the 32 KiB before it, so a segment first stages the kMW/kMT
    // tiles before s0 without walking them
    const uint32_t bi = kSegs ? job.seg[2 * blockIdx.x] : blockIdx.x;
    const uint32_t g = job.first + bi;
    const int64_t n = (int64_t)job.src_len[g];
    const int64_t s0 = kSegs ? (int64_t)job.seg[2 * blockIdx.x + 1] : 0;
    const int64_t s1 = kSegs && s0 + (int64_t)job.seg_len < n ? s0 + (int64_t)job.seg_len : n;
    const int64_t t0 = kSegs && s0 > kMW ? s0 - kMW : 0;
    const uint8_t *in = job.src + job.src_off[g];
    const uint16_t *L = job.link + job.ws_off[bi];
    uint32_t *rf = job.rfull + job.ws_off[bi];
    uint32_t *rq = job.rquart + job.ws_off[bi];
    const uint8_t *K = job.key + job.ws_off[bi];
    const LevelCfg cfg = job.cfg;
    const int64_t max_dist = job_win(job).max_dist;

    // A segment that starts inside its buffer loads its first window in one go
    // (round 6): the kMW positions before s0, its first tile and the pad, the
    // link of each turned into its predecessor's word index directly (0 when
    // that lies before the window, below every walk's limit).  It used to stage
    // the kMW/kMT tiles before s0 one after another (a lone 64 KiB compress2:
    // eight dependent tile loads per segment).
    const bool one_shot = kSegs && s0 > 0;
    const int64_t tstart = one_shot ? s0 : t0;
    if (one_shot) {
        const int64_t wb = s0 - kMW;                 // position of word 0 (s0 is a multiple of kMT)
        constexpr int kQuads = (kME + 4 * kMatchThreads - 1) / (4 * kMatchThreads);
        constexpr int kBatch = 5;
        static_assert(kQuads <= 2 * kBatch, "two batches of quad loads");
#pragma unroll
        for (int b0 = 0; b0 < kQuads; b0 += kBatch) {
            uint32_t x[kBatch][5], lk[kBatch][4];
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                const int w = 4 * (tid + (b0 + u) * kMatchThreads);
                const int64_t q = wb + w;
#pragma unroll
                for (int v = 0; v < 5; v++) x[u][v] = ldb(in, q + v, n);
                if (w < kMW + kMT && q >= 0 && q + 4 <= n) {
                    const uint2 t = *reinterpret_cast<const uint2 *>(L + q);   // 8-B aligned: ws_off % 64 == 0
                    lk[u][0] = t.x & 0xffffu; lk[u][1] = t.x >> 16; lk[u][2] = t.y & 0xffffu; lk[u][3] = t.y >> 16;
                } else {
#pragma unroll
                    for (int v = 0; v < 4; v++)
                        lk[u][v] = w < kMW + kMT && q + v >= 0 && q + v < n ? (uint32_t)L[q + v] : 0u;
                }
            }
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                const int w = 4 * (tid + (b0 + u) * kMatchThreads);
                if (b0 + u >= kQuads || w >= kME) continue;
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    const uint32_t l = lk[u][v];
                    const uint32_t wi = (uint32_t)(w + v);
                    E[w + v] = (x[u][v] | x[u][v + 1] << 8) << 16 | (l && wi >= l ? (wi - l) & 0xffffu : 0u);
                }
            }
        }
    }
    TilePre P;
    tile_prefetch(P, tstart, n, in, L, K, tid);
    for (int64_t ts = tstart; ts < s1; ts += kMT) {
        const int64_t B = ts - kMW;
        const int tile_n = kSegs && ts < s0 ? 0 : (int)((n - ts) < kMT ? (n - ts) : kMT);   // 0: staging only
        if (!(one_shot && ts == tstart)) tile_store<true>(E, P, ts, tid);
        if (tid == 0) next_i = 0;
        if (tid < kSortBuckets) s_hist[tid] = 0;
        __syncthreads();
        // counting sort of the tile's positions by key (64 buckets), longest
        // first: the 64 walks a wave runs side by side then have similar
        // lengths (SIMT utilisation 63 % -> 90 % at L6, 20 % -> 93 % at L9).
        // Thread t takes positions t + 1024u, so within a bucket the ranks come
        // out nearly in position order and a wave's lanes get nearby positions
        // (nearby candidates, fewer LDS bank conflicts).
        int bk[4], rk[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = tid + u * kMatchThreads;
            bk[u] = kSortBuckets - 1 - (i < tile_n ? (int)(P.key[u] >> 2) : 0);
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            rk[u] = tid + u * kMatchThreads < tile_n ? atomicAdd(&s_hist[bk[u]], 1) : 0;
        __syncthreads();
        if (tid < 64) {                              // exclusive scan of the bucket sizes
            const int v = s_hist[tid];
            int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if (tid >= o) incl += t;
            }
            s_base[tid] = incl - v;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (tid + u * kMatchThreads < tile_n)
                s_perm[s_base[bk[u]] + rk[u]] = (uint16_t)(tid + u * kMatchThreads);
        __syncthreads();
        if (ts + kMT < s1) tile_prefetch(P, ts + kMT, n, in, L, K, tid);   // lands during the walks
        // a streaming job whose configuration changes inside this tile walks it
        // once per row, each pass taking the positions of its row: the budget
        // count of a wave's walks stays uniform
        const uint32_t k0 = kEv && tile_n ? cfg_count(job, ts) : 0;
        const uint32_t k1 = kEv && tile_n ? cfg_count(job, ts + tile_n - 1) : 0;
        for (uint32_t k = k0; k <= k1; k++) {
            const LevelCfg c = kEv ? cfg_row(job, k) : cfg;
            const int64_t lo = k ? (int64_t)job.cfg_pos[k - 1] : -1;
            const int64_t hi = kEv && k < job.ncfg ? (int64_t)job.cfg_pos[k] : INT64_MAX;
            if (k > k0) {
                __syncthreads();
                if (tid == 0) next_i = 0;
                __syncthreads();
            }
            for (;;) {
                const int i = atomicAdd(&next_i, 1);
                if (i >= tile_n) break;
                const int64_t p = ts + (int)s_perm[i];
                if (kEv && (p < lo || p >= hi)) continue;
                // a flush job's search at p sees the input up to the next flush
                // position only (nice and the compare length are clamped to it)
                const int64_t nl = kEv ? flush_limit(job, p, n) : n;
                dwq_walk(E, p, B, nl, c, MOutRQ{rf, rq, p}, want_q, max_dist);
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------
// block bookkeeping shared by both parses (lane 0 only)
// ------------------------------------------------------------------------
// a uniform value as a VGPR operand (the compiler then treats it as divergent):
// k_parse_fast forms its addresses on the vector side, off the scalar unit
__device__ inline uint32_t vg(uint32_t x) {        // identity DPP move (quad_perm 0,1,2,3)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xE4, 0xF, 0xF, false);
}

template <typename P>
struct ParseOutT {
    uint32_t *sym;
    BlockRec *blk;
    uint32_t nsym, blk_nsym, blk_sym_start, nblk;
    P block_start, S, E;
    P wsize, max_dist;      // w_size, MAX_DIST (deflate.c:440-444)
    uint32_t sym_limit;           // lit_bufsize - 1 (deflate.c:455, deflate.h:371)
    bool lead;               // the lane that stores (the state itself is wave-uniform)
    bool vaddr = false;      // symbol stores through a VGPR index (vg)
    uint64_t *srec = nullptr;     // a streaming job's records (DeflateJob::srec)

    __device__ inline void rec(P strstart, bool res) {      // srec[4 nblk + 2, + 3]
        if (lead && srec) {
            srec[4ull * nblk + 2] = ((uint64_t)S << 32) | (uint64_t)strstart;
            srec[4ull * nblk + 3] = (uint64_t)E | (res ? 1ull << 63 : 0ull);
        }
    }

    __device__ inline void win(const WinP &w) { wsize = w.wsize; max_dist = w.max_dist; sym_limit = w.sym_limit; }
    __device__ inline bool tally(uint32_t v) {          // _tr_tally_*: returns bflush
        if (vaddr) sym[vg(nsym)] = v;
        else if (lead) sym[nsym] = v;
        nsym++;
        return ++blk_nsym == sym_limit;
    }
    __device__ inline void flush(P strstart, bool last) {   // FLUSH_BLOCK_ONLY
        BlockRec r;
        r.sym_start = blk_sym_start;
        r.nsym = blk_nsym;
        r.in_start = (uint64_t)block_start;
        r.in_end = (uint64_t)strstart;
        r.flags = (last ? 1u : 0u) | (block_start >= S ? 2u : 0u);
        r.pad = 0;
        if (lead) blk[nblk] = r;
        rec(strstart, true);
        nblk++;
        block_start = strstart;
        blk_sym_start = nsym;
        blk_nsym = 0;
    }
    // the bits a deflate(flush) call appends after its blocks (kBlkMarker)
    // (a prime's marker stands inside the block in progress: no resume point)
    __device__ inline void marker(P strstart, uint32_t kind, uint32_t arg = 0) {
        BlockRec r;
        r.sym_start = blk_sym_start;
        r.nsym = 0;
        r.in_start = r.in_end = (uint64_t)strstart;
        r.flags = kBlkMarker | (kind << 4);
        r.pad = arg;
        if (lead) blk[nblk] = r;
        rec(strstart, kind != kMarkPrime);
        nblk++;
    }
    // fill_window (deflate.c:251-368), bookkeeping only; n = the end of the
    // input deflate() has been given so far
    __device__ inline void fill(P p, P n) {
        if (p - S >= wsize + max_dist) S += wsize;
        if (E < n) { P e = S + 2 * wsize; E = e < n ? e : n; }
    }
};
using ParseOut = ParseOutT<int64_t>;


// ------------------------------------------------------------------------
// k_parse_slow — deflate_slow over precomputed per-position results.
// One wave per buffer, executed wave-uniformly: every lane runs the same
// state machine on scalar (SGPR) state, values read from LDS are made uniform
// with readfirstlane, and only lane 0 stores.  Runs of positions with no usable
// match (the literal branch of deflate.c:2007-2019 repeated) are detected 64
// at a time with a ballot and emitted in bulk.
// ------------------------------------------------------------------------
constexpr int kPT = 4096;


struct ParseU {                     // wave-uniform parse output state
    uint32_t *sym;
    BlockRec *blk;
    uint32_t nsym, blk_nsym, blk_sym_start, nblk;
    uint32_t block_start, S, E;
    uint32_t wsize, max_dist, sym_limit;     // w_size, MAX_DIST, lit_bufsize - 1
    uint64_t *srec;                          // a streaming job's records (DeflateJob::srec)
    __device__ inline void rec(uint32_t strstart, bool res, int lane) {
        if (lane == 0 && srec) {
            srec[4ull * nblk + 2] = ((uint64_t)S << 32) | strstart;
            srec[4ull * nblk + 3] = (uint64_t)E | (res ? 1ull << 63 : 0ull);
        }
    }
    // FLUSH_BLOCK_ONLY; res: the lazy state after it is the simple one
    // (nothing pending, or a pending literal whose own match is < MIN_MATCH)
    __device__ inline void flush(uint32_t strstart, bool last, int lane, bool res = true) {
        rec(strstart, res, lane);
        if (lane == 0) {
            BlockRec r;
            r.sym_start = blk_sym_start;
            r.nsym = blk_nsym;
            r.in_start = block_start;
            r.in_end = strstart;
            r.flags = (last ? 1u : 0u) | (block_start >= S ? 2u : 0u);
            r.pad = 0;
            blk[nblk] = r;
        }
        nblk++;
        block_start = strstart;
        blk_sym_start = nsym;
        blk_nsym = 0;
    }
    __device__ inline bool tally1(uint32_t v, int lane) {                   // _tr_tally_*
        if (lane == 0) sym[nsym] = v;
        nsym++;
        return ++blk_nsym == sym_limit;
    }
    __device__ inline void marker(uint32_t strstart, uint32_t kind, int lane, uint32_t arg = 0) {   // see ParseOut::marker
        if (lane == 0) {
            BlockRec r;
            r.sym_start = blk_sym_start;
            r.nsym = 0;
            r.in_start = r.in_end = strstart;
            r.flags = kBlkMarker | (kind << 4);
            r.pad = arg;
            blk[nblk] = r;
        }
        rec(strstart, kind != kMarkPrime, lane);
        nblk++;
    }
    __device__ inline void fill(uint32_t p, uint32_t n) {                   // fill_window bookkeeping
        if (p - S >= wsize + max_dist) S += wsize;
        if (E < n) { uint32_t e = S + 2 * wsize; E = e < n ? e : n; }
    }
};

// longest_match (deflate.c:1356-1497) from best_len 0, over the buffer and its
// links in global memory, wave-uniform: deflate_slow's searches right after a
// function switch that left match_length 0 (DeflateJob::zm0).  With best_len 0
// the quick reject compares match[-1] with scan[-1] (scan_end1) until a
// candidate is taken; from then on it is the usual walk.  Returns the length
// (0: nothing taken) clamped to the lookahead, *ms the match start; *searched
// false when there is no valid chain head (deflate.c:1955).
__device__ uint32_t walk_best0(const uint8_t *in, const uint16_t *lk, uint32_t p, uint32_t n, uint32_t lookahead,
                               uint32_t S, uint32_t max_dist, const LevelCfg &cfg, uint32_t *ms, bool *searched,
                               int lane) {
    const uint32_t d0 = lk[p];
    *searched = d0 != 0 && d0 <= max_dist;
    if (!*searched) return kMinMatch - 1;
    uint32_t chain = cfg.good == 0 ? cfg.chain >> 2 : cfg.chain;   // prev_length (0) >= good_match
    const uint32_t nice = lookahead < cfg.nice ? lookahead : cfg.nice;
    const uint32_t limit = p - S > max_dist ? p - max_dist : S;
    const uint32_t maxcmp = n - p < (uint32_t)kMaxMatch ? n - p : (uint32_t)kMaxMatch;
    int best = 0;
    uint32_t cur = p - d0, start = 0;
    for (;;) {
        // quick reject: match[best], match[best-1] and the first two bytes
        const bool pass = in[cur + best] == in[p + best] && in[cur + best - 1] == in[p + best - 1] &&
                          in[cur] == in[p] && in[cur + 1] == in[p + 1];
        if (pass) {
            uint32_t len = maxcmp;
            for (uint32_t k0 = 0; k0 < maxcmp; k0 += 64) {
                const uint32_t k = k0 + (uint32_t)lane;
                const uint64_t m = __ballot(k < maxcmp && in[cur + k] != in[p + k]);
                if (m) { len = k0 + (uint32_t)__builtin_ctzll(m); break; }
            }
            if ((int)len > best) {
                start = cur;
                best = (int)len;
                if (len >= nice) break;
            }
        }
        // (unsigned: a link may reach back before the buffer, which is past the limit)
        const uint32_t d = lk[cur];
        if (d == 0 || d >= cur - limit || --chain == 0) break;
        cur -= d;
    }
    *ms = start;
    return (uint32_t)best <= lookahead ? (uint32_t)best : lookahead;
}

// kT: the staged tile.  The fallback launch after k_parse_seg (only_flagged)
// takes kT = 256 (2.3 KiB of LDS instead of 36): in the pipeline its
// workgroups, nearly all of which return at once, then fit beside k_match's
// 153.6 KiB instead of waiting for CUs it has freed (14-18 ms per sub-batch on
// the caller's stream, profiles/r05v2_kernel_stats_C4_32768x1MiB_L6.csv).
template <int kT>
__global__ __launch_bounds__(64) void k_parse_slow(DeflateJob job, int only_flagged) {
    __shared__ __attribute__((aligned(16))) uint32_t s_rf[kT];
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kT + 16];   // in[t0-16 .. t0+kT)
    const int lane = threadIdx.x;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const uint32_t n = (uint32_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    const uint32_t *rf = job.rfull + job.ws_off[bi];
    const uint32_t *rq = job.rquart + job.ws_off[bi];
    const LevelCfg cfg = job.cfg;
    bool use_q = cfg.good < cfg.lazy;
    const bool filtered = job.strategy == 1;
    uint32_t lazy = cfg.lazy, good = cfg.good;
    uint32_t ci = 0;                              // configuration changes acted on
    if (only_flagged && job.nblocks[bi] != kParseFallback) return;

    ParseU po;
    po.sym = job.sym + job.ws_off[bi];
    po.blk = job.blocks + job.blk_off[bi];
    po.nsym = po.blk_nsym = po.blk_sym_start = po.nblk = 0;
    {
        const WinP wp = job_win(job);
        po.wsize = (uint32_t)wp.wsize; po.max_dist = (uint32_t)wp.max_dist; po.sym_limit = wp.sym_limit;
    }
    // a resumed flush job starts at its last flush: window read up to there
    // (E), nothing pending, a new block (deflate.c state after :2030-2042); one
    // resumed at a block cut has read up to e0 and nothing pending either
    // (ParseU::flush's res)
    // match_length before the first decision: 2, or what a function switch left (zm0)
    uint32_t p = job.start, match_start = 0, match_length = job.srec ? (uint32_t)job.zm0 : kMinMatch - 1;
    uint32_t zprev = job.srec ? (uint32_t)job.zp0 : kMinMatch - 1;   // deflate_state's prev_length
    const uint16_t *lk = job.link + job.ws_off[bi];
    po.block_start = p; po.S = 0; po.E = job.e0 > p ? job.e0 : p;
    po.srec = job.srec;
    bool avail = false, done = false;
    FlushEv fe = flush_ev(job);
    while (fe.prime()) {                       // deflatePrime at the resume point (a pause behind it): bits first
        if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
        po.marker(p, kMarkPrime, lane, fe.prime_arg());
        fe.i++;
    }
    uint32_t lim = (uint32_t)fe.limit(n);      // input deflate() has been given

    uint32_t t0 = p & ~15u;
    while (!done) {
        stage_words<64, kT / 4 / 64>(s_rf, rf, t0, kT, n, lane);

        stage_bytes<64, (kT + 16) / 16 / 64 + 1>(s_in, in, (int64_t)t0 - 16, kT + 16, n, lane);
        __syncthreads();
        const bool tile_to_end = (uint64_t)t0 + kT >= n;
        for (;;) {
            if (!tile_to_end && p + 64 > t0 + kT) break;         // reload, keep 64 lookahead
            if (p > po.E) { done = true; break; }                 // guard: never parse past the input read
            if (po.E - p < (uint32_t)kMinLookahead) {
                po.fill(p, lim);
                // a Z_NO_FLUSH call's input is used up: need_more (deflate.c:1941-1944);
                // the next call's fill_window goes on from here
                while (fe.stop_at(po.E, lim) && po.E - p < (uint32_t)kMinLookahead) {
                    if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                    fe.i++;
                    while (fe.prime()) {                          // deflatePrime: its bits go out here
                        if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                        po.marker(p, kMarkPrime, lane, fe.prime_arg());
                        fe.i++;
                    }
                    if (fe.i == fe.n && job.open_end) { done = true; break; }
                    lim = (uint32_t)fe.limit(n);
                    po.fill(p, lim);
                }
                if (done) break;
                if (po.E == p) {
                    if (fe.at(p)) {
                        // a deflate(flush) call ends here (deflate.c:2030-2042): the
                        // pending literal is tallied without a flush test, the
                        // block is flushed if it holds symbols, then the marker
                        if (avail) po.tally1(ufl(s_in[p - 1 - t0 + 16]), lane);
                        avail = false;
                        match_length = kMinMatch - 1;
                        if (po.blk_nsym) po.flush(p, false, lane);
                        if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                        po.marker(p, fe.kind(), lane);
                        if (lane == 0 && job.flush_out) job.flush_out[2] = po.S;
                        fe.i++;
                        lim = (uint32_t)fe.limit(n);
                        continue;
                    }
                    done = true;
                    break;
                }
            }
            const uint32_t lookahead = po.E - p;
            // ---- bulk literals: no pending match, far from the window end ----
            // (not while match_length is 0: each of those decisions searches
            // from best_len 0 and may end the state, see walk_best0)
            if (match_length < kMinMatch && match_length != 0 && p + 64 + kMinLookahead <= po.E) {
                const uint32_t r = s_rf[p - t0 + lane] & ~kQDiff;
                const uint32_t rl = r >> 16;
                const bool hit = rl >= kMinMatch &&
                                 !(rl <= 5u && (filtered || (rl == kMinMatch && (r & 0xffffu) > (uint32_t)kTooFar)));
                const uint64_t mask = __ballot(hit);
                const uint32_t k = mask ? (uint32_t)__builtin_ctzll(mask) : 64u;
                if (k > 0) {
                    uint32_t a = avail ? p - 1 : p;
                    const uint32_t b = p + k - 1;
                    while (a < b) {
                        const uint32_t room = po.sym_limit - po.blk_nsym;
                        const uint32_t take = (b - a) < room ? (b - a) : room;
                        if ((uint32_t)lane < take) po.sym[po.nsym + lane] = s_in[a + lane - t0 + 16];
                        po.nsym += take;
                        po.blk_nsym += take;
                        a += take;
                        if (po.blk_nsym == po.sym_limit) {
                            po.flush(a, false, lane);
                            if (fe.pause_at(a)) {
                                if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                                fe.i++;
                                while (fe.prime()) {          // deflatePrime while the call stood here
                                    if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                                    po.marker(a, kMarkPrime, lane, fe.prime_arg());
                                    fe.i++;
                                }
                                lim = (uint32_t)fe.limit(n);
                            }
                        }
                    }
                    avail = true;
                    p += k;
                    zprev = kMinMatch - 1;
                    continue;
                }
            }
            // ---- one deflate_slow step (deflate.c:1946-2027) ----
            while (ci < job.ncfg && p >= (uint32_t)job.cfg_pos[ci]) {   // deflateParams / deflateTune
                lazy = job.cfg_tab[ci].lazy;
                good = job.cfg_tab[ci].good;
                use_q = good < lazy;
                ci++;
            }
            const uint32_t prev_length = match_length, prev_match = match_start;
            zprev = prev_length;
            match_length = kMinMatch - 1;
            if (lookahead >= kMinMatch && prev_length < lazy) {
                if (prev_length == 0) {                    // after a function switch (DeflateJob::zm0)
                    uint32_t ms = 0;
                    bool searched = false;
                    const uint32_t ml = walk_best0(in, lk, p, n, lookahead, po.S, po.max_dist, LevelCfg{good, lazy,
                                                   ci ? job.cfg_tab[ci - 1].nice : cfg.nice,
                                                   ci ? job.cfg_tab[ci - 1].chain : cfg.chain}, &ms, &searched, lane);
                    if (searched) {
                        match_length = ml;
                        match_start = ms;
                        if (match_length <= 5u && (filtered || (match_length == kMinMatch && p - match_start > (uint32_t)kTooFar)))
                            match_length = kMinMatch - 1;
                    }
                } else {
                    const uint32_t w = ufl(s_rf[p - t0]);
                    const uint32_t r = (use_q && prev_length >= good && (w & kQDiff)) ? ufl(rq[p]) : w & ~kQDiff;
                    const uint32_t rl = r >> 16;
                    if (rl > prev_length) {
                        match_length = rl;
                        match_start = p - (r & 0xffffu);
                        if (match_length <= 5u && (filtered || (match_length == kMinMatch && p - match_start > (uint32_t)kTooFar)))
                            match_length = kMinMatch - 1;              // deflate.c:1964-1975
                    }
                }
            }
            if (prev_length >= kMinMatch && match_length <= prev_length) {
                const uint32_t dist = p - 1 - prev_match;
                const bool bflush = po.tally1((dist << 8) | (prev_length - kMinMatch), lane);
                p += prev_length - 1;
                avail = false;
                zprev = 0;                                 // the insert loop counts prev_length down to 0
                match_length = kMinMatch - 1;
                if (bflush) {
                    po.flush(p, false, lane);
                    if (fe.pause_at(p)) {
                        if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                        fe.i++;
                        while (fe.prime()) {                  // deflatePrime while the call stood here
                            if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                            po.marker(p, kMarkPrime, lane, fe.prime_arg());
                            fe.i++;
                        }
                        lim = (uint32_t)fe.limit(n);
                    }
                }
            } else if (avail) {
                const uint32_t lit = ufl(s_in[p - 1 - t0 + 16]);
                // a new job starting at p would find the same state only when
                // nothing longer than MIN_MATCH - 1 was pending here
                if (po.tally1(lit, lane)) {
                    // (a match_length of 0 is no state a new job starts in)
                    po.flush(p, false, lane, prev_length < kMinMatch && match_length != 0);
                    if (fe.pause_at(p)) {
                        if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                        fe.i++;
                        while (fe.prime()) {                  // deflatePrime while the call stood here
                            if (lane == 0 && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                            po.marker(p, kMarkPrime, lane, fe.prime_arg());
                            fe.i++;
                        }
                        lim = (uint32_t)fe.limit(n);
                    }
                }
                p++;
            } else {
                avail = true;
                p++;
            }
        }
        if (done) {
            if (!job.open_end) {
                if (avail) po.tally1(ufl(s_in[p - 1 - t0 + 16]), lane);
                po.flush(p, true, lane);
            }
            if (lane == 0) job.nblocks[bi] = po.nblk;
            if (lane == 0 && job.flush_out) job.flush_out[4] = (uint64_t)zprev | (uint64_t)match_length << 16;
        }
        t0 = p & ~15u;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------
// k_parse_seg — deflate_slow parsed by 256 lanes per buffer (levels 4..9).
//
// The lazy parse is a deterministic state machine over decision points whose
// state is (match_length, match_start, match_available).  Whenever
// match_length < MIN_MATCH the state is "simple" and fully described by
// match_available.  The buffer is cut into <= kParseLanes segments of >= 512 B,
// one lane each (several independent load chains per buffer hide latency).
//  pass 1  lane i parses its segment from the simple state (.., avail=0) and
//          records (2 bits per position, lane-private words in global memory)
//          the simple states it stands in;
//  pass 2  lane i runs on into segment i+1 until it stands at a position in the
//          same simple state lane i+1 recorded there: from that point the two
//          parses coincide, so the true parse is lane 0 on [0,y0), lane 1 on
//          [y0,y1), ...  (measured: they meet within ~20 positions on average,
//          ~500 at most on byte runs);
//          Pass 1 also stages its symbols at stage[x0 + k] (16-byte stores);
//  replay  lane i counts the pass-1 symbols of steps before y(i-1) (replaying
//          its first ~20 positions) and replays its run-on [pass-1 end, y(i)),
//          staging those symbols in its own (now dead) state words, so every
//          position is parsed about once;
//  compact a block prefix sum of the counts gives each lane its first symbol
//          index; the symbols are copied into sym[], a wave scan of their
//          lengths gives their start positions, and every 16383rd symbol
//          records its end (the block cut of _tr_tally, deflate.h:371);
//  blocks  block records from the cuts; the fill_window slides before a flush
//          at decision point d are #{k : T_k <= d} (the k-th slide happens at
//          the first decision point >= T_k), which is the block_start >= 0 test
//          of the stored-block choice (deflate.c:1597-1600).
// A buffer whose lanes fail to meet within the next segment, or whose run-on
// has more symbols than the lane has state words, is flagged
// (nblocks = ~0) for k_parse_slow.
// ------------------------------------------------------------------------
// buffers k_parse_seg handed to k_parse_slow: [0] a lane did not meet its
// neighbour within the next segment, [1] a run-on outgrew the lane's state words
__device__ unsigned long long g_parse_fb[2];
int parse_fallback_counts(uint64_t *out) {
    unsigned long long v[2] = {0, 0};
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_parse_fb), sizeof v) != hipSuccess) return -1;
    out[0] = v[0];
    out[1] = v[1];
    return 0;
}

constexpr int kSegMin = 512;
constexpr int kParseLanes = 256;                  // segments (lanes) per buffer
static_assert(kParseLanes == (int)kParseLanesHost, "host lane groups");
constexpr uint32_t kEnd = 0xffffffffu;

struct WCache {
    uint32_t base;
    uint32_t x, y, z, w;       // four separate registers: no indexable array
};
__device__ __attribute__((always_inline)) inline uint32_t sel4(uint32_t x, uint32_t y, uint32_t z,
                                                               uint32_t w, uint32_t k) {
    const uint32_t lo = (k & 1u) ? y : x, hi = (k & 1u) ? w : z;
    return (k & 2u) ? hi : lo;
}
__device__ __attribute__((always_inline)) inline uint32_t wget(const uint32_t *a, uint32_t p, WCache &c) {
    const uint32_t b = p & ~3u;
    if (b != c.base) {
        const uint4 v = *reinterpret_cast<const uint4 *>(a + b);
        c.x = v.x; c.y = v.y; c.z = v.z; c.w = v.w;
        c.base = b;
    }
    return sel4(c.x, c.y, c.z, c.w, p & 3u);
}
struct BCache {
    uintptr_t base;
    uint32_t x, y, z, w;
};
__device__ __attribute__((always_inline)) inline uint32_t bget(const uint8_t *in, uint32_t x, BCache &c) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(in + x);
    const uintptr_t b = a & ~(uintptr_t)15;
    if (b != c.base) {
        const uint4 v = *reinterpret_cast<const uint4 *>(b);
        c.x = v.x; c.y = v.y; c.z = v.z; c.w = v.w;
        c.base = b;
    }
    const uint32_t o = (uint32_t)(a - b);
    return (sel4(c.x, c.y, c.z, c.w, o >> 2) >> (8 * (o & 3u))) & 0xffu;
}

// 64-byte lines for the lone-buffer parse (k_pbig1..3): there a wave holds
// every segment of a buffer and each line a lane leaves is a dependent load of
// its serial parse; a 64 B line is four positions' worth of a 16 B one
struct WCache16 {
    uint32_t base;
    uint4 a, b, c, d;
};
__device__ __attribute__((always_inline)) inline uint32_t sel16(const uint4 &a, const uint4 &b, const uint4 &c,
                                                                const uint4 &d, uint32_t k) {
    const uint32_t j = k & 3u;
    return sel4(sel4(a.x, a.y, a.z, a.w, j), sel4(b.x, b.y, b.z, b.w, j), sel4(c.x, c.y, c.z, c.w, j),
                sel4(d.x, d.y, d.z, d.w, j), k >> 2);
}
__device__ __attribute__((always_inline)) inline uint32_t wget(const uint32_t *a, uint32_t p, WCache16 &c) {
    const uint32_t b = p & ~15u;
    if (b != c.base) {
        const uint4 *q = reinterpret_cast<const uint4 *>(a + b);
        c.a = q[0]; c.b = q[1]; c.c = q[2]; c.d = q[3];
        c.base = b;
    }
    return sel16(c.a, c.b, c.c, c.d, p & 15u);
}
struct BCache64 {
    uintptr_t base;
    uint4 a, b, c, d;
};
__device__ __attribute__((always_inline)) inline uint32_t bget(const uint8_t *in, uint32_t x, BCache64 &c) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(in + x);
    const uintptr_t b = a & ~(uintptr_t)63;
    if (b != c.base) {
        const uint4 *q = reinterpret_cast<const uint4 *>(b);
        c.a = q[0]; c.b = q[1]; c.c = q[2]; c.d = q[3];
        c.base = b;
    }
    const uint32_t o = (uint32_t)(a - b);
    return (sel16(c.a, c.b, c.c, c.d, o >> 2) >> (8 * (o & 3u))) & 0xffu;
}

// reads straight from an LDS copy of [base, ...) (k_pbig1s): no line cache
struct WDirect { uint32_t base; };
__device__ __attribute__((always_inline)) inline uint32_t wget(const uint32_t *a, uint32_t p, WDirect &c) {
    return a[p - c.base];
}
struct BDirect { uint32_t base; };
__device__ __attribute__((always_inline)) inline uint32_t bget(const uint8_t *in, uint32_t x, BDirect &c) {
    return in[x - c.base];
}
__device__ inline void cache_reset(WCache &c) { c.base = 0xffffffffu; }
__device__ inline void cache_reset(WCache16 &c) { c.base = 0xffffffffu; }
__device__ inline void cache_reset(BCache &c) { c.base = ~(uintptr_t)0; }
__device__ inline void cache_reset(BCache64 &c) { c.base = ~(uintptr_t)0; }
__device__ inline void cache_reset(WDirect &) {}
__device__ inline void cache_reset(BDirect &) {}

template <typename WC, typename BC>
struct SlowLaneT {
    uint32_t p, ml, ms, avail;
    WC cf;
    BC cb;
};
using SlowLane = SlowLaneT<WCache, BCache>;          // k_parse_seg: many lanes in flight hide the loads
using SlowLaneW = SlowLaneT<WCache16, BCache64>;     // k_pbig*
using SlowLaneD = SlowLaneT<WDirect, BDirect>;       // k_pbig1s

// one deflate_slow decision (deflate.c:1946-2027) on precomputed results.
// Returns 0 (no symbol), 1 (literal at spos), 2 (match starting at spos, len).
template <typename Lane>
__device__ __attribute__((always_inline)) inline int slow_step(Lane &L, uint32_t n, const uint32_t *rf, const uint32_t *rq,
                                const uint8_t *in, const LevelCfg &cfg, bool use_q, bool filtered,
                                uint32_t &sym, uint32_t &spos, uint32_t &slen) {
    const uint32_t p = L.p;
    const uint32_t prev_length = L.ml, prev_match = L.ms;
    uint32_t ml = kMinMatch - 1;
    if (n - p >= (uint32_t)kMinMatch && prev_length < cfg.lazy) {
        const uint32_t w = wget(rf, p, L.cf);
        // the quartered budget's result where it differs from the full one (kQDiff)
        const uint32_t r = (use_q && prev_length >= cfg.good && (w & kQDiff)) ? rq[p] : w & ~kQDiff;
        const uint32_t rl = r >> 16;
        if (rl > prev_length) {
            ml = rl;
            L.ms = p - (r & 0xffffu);
            if (ml <= 5u && (filtered || (ml == (uint32_t)kMinMatch && p - L.ms > (uint32_t)kTooFar)))
                ml = kMinMatch - 1;                        // deflate.c:1964-1975
        }
    }
    if (prev_length >= (uint32_t)kMinMatch && ml <= prev_length) {
        sym = ((p - 1 - prev_match) << 8) | (prev_length - kMinMatch);
        spos = p - 1;
        slen = prev_length;
        L.p = p + prev_length - 1;
        L.avail = 0;
        L.ml = kMinMatch - 1;
        return 2;
    }
    L.ml = ml;
    if (L.avail) {
        sym = bget(in, p - 1, L.cb);
        spos = p - 1;
        slen = 1;
        L.p = p + 1;
        return 1;
    }
    L.avail = 1;
    L.p = p + 1;
    return 0;
}

// p at which the k-th window slide (k >= 1) becomes due: fill_window is called
// when lookahead < MIN_LOOKAHEAD and slides when strstart >= WSIZE+MAX_DIST
// (deflate.c:277); with all input present the window end is min(n, S + 64K).
__device__ inline int64_t slide_threshold(uint32_t k, uint32_t n, int64_t refill, const WinP &w) {
    // fill_window runs at a decision point p with lookahead E - p <= refill
    // (261 for deflate_slow/fast, 258 for deflate_rle, 0 for deflate_huff) and
    // slides when p - S >= WSIZE + MAX_DIST (deflate.c:277); all input is
    // present, so the window end is E = min(n, S + 2 WSIZE).
    const int64_t S = w.wsize * (k - 1);
    const int64_t E = (int64_t)n > S + 2 * w.wsize ? S + 2 * w.wsize : (int64_t)n;
    const int64_t a = E - refill, b = S + w.wsize + w.max_dist;
    return a > b ? a : b;
}

template <typename Lane>
__device__ __attribute__((always_inline)) inline void lane_init(Lane &L, uint32_t p, uint32_t avail) {
    L.p = p; L.ml = kMinMatch - 1; L.ms = 0; L.avail = avail;
    cache_reset(L.cf);
    cache_reset(L.cb);
}

// Four symbols buffered in registers and stored as one 16-byte word: a lane's
// staging writes are sequential, so whole 16 B go to memory at a time.
struct SymBuf {
    uint32_t v0, v1, v2, v3;
    uint32_t k;                 // symbols pushed
    __device__ __attribute__((always_inline)) inline void push(uint32_t *dst, uint32_t v) {
        const uint32_t j = k & 3u;
        if (j == 0) v0 = v; else if (j == 1) v1 = v; else if (j == 2) v2 = v; else v3 = v;
        k++;
        if ((k & 3u) == 0) *reinterpret_cast<uint4 *>(dst + k - 4) = make_uint4(v0, v1, v2, v3);
    }
    __device__ __attribute__((always_inline)) inline void flush(uint32_t *dst) {
        const uint32_t j = k & 3u, b = k & ~3u;
        if (j > 0) dst[b] = v0;
        if (j > 1) dst[b + 1] = v1;
        if (j > 2) dst[b + 2] = v2;
    }
};

// The block records of a segmented lazy parse (k_parse_seg, k_lzp): the cuts
// left blk[b].in_end (strstart at the flush) and blk[b].pad (its decision
// point) for b < ncut; block ncut is the last.  A block is stored-eligible
// while its start has not slid out of the window: the slides before its flush
// come from the closed-form schedule (slide_threshold).  Every cut field is
// read before any record is written; all kT threads of the block call this.
template <int kT>
__device__ __attribute__((always_inline)) inline void seg_block_records(BlockRec *blk, uint32_t n, uint32_t total,
                                                                        uint32_t ncut, const WinP &wp, int lane) {
    const uint32_t symlim = wp.sym_limit;
    uint32_t nthr = 0;
    while (slide_threshold(nthr + 1, n, kMinLookahead - 1, wp) <= (int64_t)n) nthr++;
    constexpr int kRecs = kT >= 1024 ? 2 : 8;
    BlockRec r[kRecs];
    for (uint32_t b0 = 0; b0 <= ncut; b0 += kT * kRecs) {
#pragma unroll
        for (int u = 0; u < kRecs; u++) {
            const uint32_t b = b0 + (uint32_t)u * kT + (uint32_t)lane;
            if (b > ncut) continue;
            const bool last = b == ncut;
            const uint64_t in_end = last ? n : blk[b].in_end;
            const uint64_t pd = last ? n : blk[b].pad;
            const uint64_t in_start = b == 0 ? 0 : blk[b - 1].in_end;
            uint32_t slides = 0;
            while (slides < nthr && slide_threshold(slides + 1, n, kMinLookahead - 1, wp) <= (int64_t)pd) slides++;
            r[u].sym_start = b * symlim;
            r[u].nsym = last ? total - b * symlim : symlim;
            r[u].in_start = in_start;
            r[u].in_end = in_end;
            r[u].flags = (last ? 1u : 0u) | (in_start >= (uint64_t)wp.wsize * slides ? 2u : 0u);
            r[u].pad = 0;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kRecs; u++) {
            const uint32_t b = b0 + (uint32_t)u * kT + (uint32_t)lane;
            if (b <= ncut) blk[b] = r[u];
        }
        __threadfence_block();
        __syncthreads();
    }
}

__global__ __launch_bounds__(kParseLanes) void k_parse_seg(DeflateJob job) {
    const WinP wp = job_win(job);
    const uint32_t symlim = wp.sym_limit;
    __shared__ uint32_t s_y[kParseLanes], s_sig[kParseLanes];
    __shared__ uint32_t s_wsum[kParseLanes / 64];
    __shared__ int s_fail;
    __shared__ uint32_t s_first_end, s_final;
    const int lane = threadIdx.x;
    const int wl = lane & 63, wv = lane >> 6;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const uint32_t n = (uint32_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    const uint32_t *rf = job.rfull + job.ws_off[bi];
    const uint32_t *rq = job.rquart + job.ws_off[bi];
    uint32_t *sym = job.sym + job.ws_off[bi];
    uint32_t *stg = job.stage + job.ws_off[bi];
    uint32_t *sst = job.pstate + (job.ws_off[bi] >> 4);      // 2 bits per position
    BlockRec *blk = job.blocks + job.blk_off[bi];
    const LevelCfg cfg = job.cfg;
    const bool use_q = cfg.good < cfg.lazy;
    const bool filtered = job.strategy == 1;

    uint32_t nseg = (n + kSegMin - 1) / kSegMin;
    nseg = nseg < 1 ? 1 : nseg > (uint32_t)kParseLanes ? (uint32_t)kParseLanes : nseg;
    const uint32_t seg = (((n + nseg - 1) / nseg) + 15u) & ~15u;      // lanes never share a state word
    auto xb = [&](uint32_t i) -> uint32_t { uint64_t v = (uint64_t)i * seg; return v < n ? (uint32_t)v : n; };
    const bool active = (uint32_t)lane < nseg;
    if (lane == 0) { s_fail = 0; s_first_end = kParseLanes; s_final = 0; }

    // ---- pass 1: speculative parse of the own segment [x0, seg_end) from the
    // simple state.  Its symbols are staged at stg[x0 + k] (a symbol starts
    // inside the segment, so k < seg); the simple states it stands in go to
    // sst[] one 16-position word at a time (words it jumps over are zeroed).
    SlowLane L;
    uint32_t sym_v, spos, slen;
    const uint32_t x0 = xb(lane);
    lane_init(L, x0, 0);
    const uint32_t seg_end = (uint32_t)lane + 1 >= nseg ? n : xb(lane + 1);
    SymBuf sb{0, 0, 0, 0, 0};
    if (active && x0 < seg_end) {
        uint32_t widx = x0 >> 4, wcur = 0;
        while (L.p < seg_end) {
            const uint32_t wi = L.p >> 4;
            if (wi != widx) {
                sst[widx] = wcur;
                for (uint32_t z = widx + 1; z < wi; z++) sst[z] = 0;
                widx = wi;
                wcur = 0;
            }
            if (L.ml < (uint32_t)kMinMatch) wcur |= 1u << (2 * (L.p & 15u) + L.avail);
            if (slow_step(L, n, rf, rq, in, cfg, use_q, filtered, sym_v, spos, slen)) sb.push(stg + x0, sym_v);
        }
        sst[widx] = wcur;
        for (uint32_t z = widx + 1; z <= (seg_end - 1) >> 4; z++) sst[z] = 0;
        sb.flush(stg + x0);
    }
    const uint32_t k1 = sb.k;
    const uint32_t e_p = L.p, e_ml = L.ml, e_ms = L.ms, e_av = L.avail;   // where pass 1 stopped
    __threadfence_block();
    __syncthreads();

    // ---- pass 2: run on until the parse meets lane+1's recorded state
    uint32_t y = kEnd, sig = 0;
    if (active && (uint32_t)lane + 1 < nseg) {
        const uint32_t next_start = xb(lane + 1);
        const uint32_t stop = (uint32_t)lane + 2 >= nseg ? n : xb(lane + 2);
        uint32_t ridx = 0xffffffffu, rw = 0;
        for (;;) {
            if (L.p >= n) { y = kEnd; break; }
            if (L.p >= stop) { atomicOr(&s_fail, 1); break; }
            if (L.p >= next_start && L.ml < (uint32_t)kMinMatch) {
                if ((L.p >> 4) != ridx) { ridx = L.p >> 4; rw = sst[ridx]; }
                if ((rw >> (2 * (L.p & 15u) + L.avail)) & 1u) { y = L.p; sig = L.avail; break; }
            }
            slow_step(L, n, rf, rq, in, cfg, use_q, filtered, sym_v, spos, slen);
        }
    }
    if (active && y == kEnd) atomicMin(&s_first_end, (uint32_t)lane);
    s_y[lane] = y;
    s_sig[lane] = sig;
    __threadfence_block();
    __syncthreads();
    if (s_fail) {
        if (lane == 0) {
            job.nblocks[bi] = kParseFallback;
            atomicAdd(&g_parse_fb[0], 1ull);
        }
        return;
    }
    // the true parse is lane i's on [y(i-1), y(i)) (lane 0 from 0; y = kEnd: to
    // n); lanes after the first one that reached n have nothing to do
    const bool mine = active && (uint32_t)lane <= s_first_end;
    const uint32_t start = lane > 0 ? s_y[lane - 1] : 0u;
    const uint32_t start_av = lane > 0 ? s_sig[lane - 1] : 0u;
    const uint32_t yend = s_y[lane];
    const uint32_t end = yend == kEnd ? n : yend;

    // ---- prefix: pass 1's symbols from steps before y(i-1) are not lane i's
    // (the parse meets the true one there); count them by replaying pass 1
    uint32_t kstart = 0;
    if (mine && lane > 0) {
        lane_init(L, x0, 0);
        while (L.p < start)
            if (slow_step(L, n, rf, rq, in, cfg, use_q, filtered, sym_v, spos, slen)) kstart++;
    }
    // ---- run-on: replay pass 2 from where pass 1 stopped and stage its
    // symbols in the lane's own (now dead) state words; the last lane's final
    // pending literal goes there too (tallied without a flush test)
    uint32_t rcnt = 0;
    uint32_t *ron = sst + (x0 >> 4);
    const uint32_t rcap = (seg_end - x0 + 15u) >> 4;
    if (mine) {
        L.p = e_p; L.ml = e_ml; L.ms = e_ms; L.avail = e_av;
        L.cf.base = 0xffffffffu;
        L.cb.base = ~(uintptr_t)0;
        while (L.p < end) {
            if (slow_step(L, n, rf, rq, in, cfg, use_q, filtered, sym_v, spos, slen)) {
                if (rcnt < rcap) ron[rcnt] = sym_v;
                rcnt++;
            }
        }
        if (yend == kEnd && L.avail) {
            if (rcnt < rcap) ron[rcnt] = bget(in, n - 1, L.cb);
            rcnt++;
            s_final = 1;
        }
        if (rcnt > rcap) atomicOr(&s_fail, 1);
    }
    const uint32_t c1 = mine ? k1 - kstart : 0u;        // staged pass-1 symbols that are lane i's
    const uint32_t cnt = c1 + rcnt;
    // exclusive block prefix sum of cnt
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (wl >= o) incl += t;
    }
    if (wl == 63) s_wsum[wv] = incl;
    __threadfence_block();
    __syncthreads();
    if (s_fail) {
        if (lane == 0) {
            job.nblocks[bi] = kParseFallback;
            atomicAdd(&g_parse_fb[1], 1ull);
        }
        return;
    }
    uint32_t woff = 0, total = 0;
    for (int k = 0; k < kParseLanes / 64; k++) {
        const uint32_t t = s_wsum[k];
        if (k < wv) woff += t;
        total += t;
    }
    const uint32_t base = woff + incl - cnt;
    const uint32_t ncut = total / symlim - ((s_final && total % symlim == 0) ? 1u : 0u);
    // the symbols of lane i tile the input from y(i-1) - sig(i-1) (its first
    // symbol may be the literal pending at y(i-1))
    const uint32_t pos0 = start - start_av;

    // ---- compaction: every wave copies its own lanes' symbols, 64 at a time,
    // into sym[]; a wave scan of the symbol lengths gives each symbol's start,
    // and every 16383rd symbol records its block cut in blk[b].in_end / .pad
    for (int j = 0; j < 64; j++) {
        const uint32_t jc = __shfl(cnt, j, 64), jb = __shfl(base, j, 64);
        if (jc == 0) continue;
        const uint32_t jc1 = __shfl(c1, j, 64), jx = __shfl(x0, j, 64), jk = __shfl(kstart, j, 64);
        uint32_t run = __shfl(pos0, j, 64);
        const uint32_t *s1 = stg + jx + jk, *s2 = sst + (jx >> 4);
        for (uint32_t c = 0; c < jc; c += 64) {
            const uint32_t idx = c + (uint32_t)wl;
            const bool have = idx < jc;
            const uint32_t v = have ? (idx < jc1 ? s1[idx] : s2[idx - jc1]) : 0u;
            const uint32_t len = have ? (v < 256u ? 1u : (v & 0xffu) + (uint32_t)kMinMatch) : 0u;
            uint32_t li = len;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(li, o, 64);
                if (wl >= o) li += t;
            }
            const uint32_t sp = run + li - len;
            run += __shfl(li, 63, 64);
            if (have) {
                const uint32_t gi = jb + idx;
                sym[gi] = v;
                if ((gi + 1) % symlim == 0 && (gi + 1) / symlim <= ncut) {
                    const uint32_t b = (gi + 1) / symlim - 1;
                    blk[b].in_end = (uint64_t)(sp + len);
                    blk[b].pad = sp + 1;                        // decision point of the flush
                }
            }
        }
    }
    __threadfence_block();
    __syncthreads();

    seg_block_records<kParseLanes>(blk, n, total, ncut, wp, lane);
    if (lane == 0) job.nblocks[bi] = ncut + 1;
}

#ifdef ZGPU_LZP
// ------------------------------------------------------------------------
// k_lzp — levels 4..7 of a batch job: longest_match where deflate_slow asks
// for it, and deflate_slow itself, in one kernel (round 6; an A/B build only:
// make -C zlib.wasm_amd lzp -> libzgpu_lzp.so, ZGPU_LZP=1.  Exact, but 2.7x
// slower than k_match + k_parse_seg on the bench's sub-batch: DESIGN.md 4.15).
//
// k_match walks every position's chain with the full budget, but the lazy
// parse calls longest_match at about a quarter of the positions
// (deflate.c:1955-1976) and takes the quartered budget where prev_length >=
// good_match (:1390-1392).  tools/model/model_walks.c counts 76 chain steps
// per position for the Silesia-style mix at level 6 against 11 at the parse's
// call sites.  The sites depend on the results, so this kernel speculates and
// verifies, tile by tile, with the window in LDS:
//
//   1. every position of a tile is walked with the quartered budget (its
//      result Q(p)); a walk that ends before the budget (chain end, limit,
//      nice) is exact for the full budget too (kZX);
//   2. one wave parses the tile (deflate_slow's rules, slow_step) from the
//      state the previous tile left, taking Q(p) as a guess where the full
//      result F(p) is needed and unknown, and lists the guessed sites on the
//      parse's path;
//   3. the listed sites are walked with the full budget (F), and 2 repeats
//      until the path uses no guess.  Then the tile's symbols and block cuts
//      are written as k_parse_seg writes them.
// The result is deflate_slow's parse exactly: the final path uses the exact
// result at every decision, and a walk's result is a pure function of the
// position and its budget.
//
// Step s of a workgroup (one buffer) stages tile s and runs two things side
// by side: the walker waves take the quarter walks of tile s, and the parser
// wave (wave 15) runs the rounds of tile s-1, whose full walks the walkers
// take first whenever some are posted (the parser takes them too while it
// waits).  The window therefore covers tile s-1's history and both tiles:
// words [0, kZH) before tile s-1, tile s-1, tile s and the compare pad.
//
// The parse of a tile (2048 positions) is k_parse_seg's segmented parse on
// one wave: lane i parses positions [a + 32 i, a + 32 i + 32) from the simple
// state (lane 0 from the carried state), records the simple states it stands
// in (2 bits per position), then runs on until it stands in a state a later
// lane recorded; the stitched path follows those meets from lane 0.
// ------------------------------------------------------------------------
constexpr int kZT = 2048;                       // positions per tile
constexpr int kZH = 32512;                      // window words before the parse tile (>= MAX_DIST, 16-aligned)
constexpr int kZE = kZH + 2 * kZT + kMPad;      // 36880 words = 144.1 KiB
constexpr int kZThreads = 1024;
constexpr int kZParser = kZThreads / 64 - 1;    // the parser wave
constexpr int kZSeg = kZT / 64;                 // parse positions per lane
constexpr int kZReq = 512;                      // full-walk request ring (tile offsets)
constexpr uint32_t kZF = 1u << 30;              // ZQ word: the full-budget result
constexpr uint32_t kZX = 1u << 31;              // quarter walk ended before its budget: full = quarter
constexpr uint32_t kZEnd = 0xffffffffu;
static_assert(kZSeg == 32, "two 16-position state words per lane");
static_assert(kZT / 2 == kZThreads, "tile staging: 2 words per thread");
static_assert(kMPad / 4 <= kZThreads && kZH % 16 == 0, "pad staging");

#ifdef ZGPU_LZP_STATS
// statistics build only (tools/lzp_stats.py): [0] tiles parsed, [1] rounds,
// [2] full walks requested, [3] quarter walks, [4] quarter steps, [5] full
// walks, [6] full steps, [7] requests dropped (ring full), [8..15] rounds
// per tile histogram (1..7, 8+); parser clock (s_memtime) in [16] passes 1-2,
// [17] stitch + replay, [18] waiting for its full walks, [19] symbols, [20]
// whole tile; [21] clock of a step (wave 0), [22] walker waves' idle polls,
// [23] speculative full walks
__device__ unsigned long long g_zstat[32];
#define ZSTAT(i, v) atomicAdd(&g_zstat[i], (unsigned long long)(v))
#define ZCLK() __builtin_amdgcn_s_memtime()
extern "C" int zgpu_lzp_stats_read(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zstat), sizeof(g_zstat)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_zstat), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define ZCLK() 0ull
#endif

// what thread t stages for a tile: words 2t, 2t+1 (bytes, links), the walk
// keys of positions ts + t and ts + t + 1024, and for t < kMPad/4 four pad words
struct ZPre {
    uint32_t b[2], pb[4], lk[2], key[2];
};
__device__ __attribute__((always_inline)) inline void zpre_load(ZPre &P, int64_t ts, int64_t n, const uint8_t *in,
                                                                const uint16_t *L, const uint8_t *K, int tid) {
    const int64_t q0 = ts + 2 * tid;
    const uint32_t x0 = ldb(in, q0, n), x1 = ldb(in, q0 + 1, n), x2 = ldb(in, q0 + 2, n);
    P.b[0] = x0 | x1 << 8;
    P.b[1] = x1 | x2 << 8;
    if (tid < kMPad / 4) {
        const int64_t q1 = ts + kZT + 4 * tid;
        uint32_t x[5];
#pragma unroll
        for (int u = 0; u < 5; u++) x[u] = ldb(in, q1 + u, n);
#pragma unroll
        for (int u = 0; u < 4; u++) P.pb[u] = x[u] | x[u + 1] << 8;
    }
    if (q0 + 2 <= n) {
        const uint32_t v = *reinterpret_cast<const uint32_t *>(L + q0);   // 4-B aligned: ws_off % 64 == 0
        P.lk[0] = v & 0xffffu;
        P.lk[1] = v >> 16;
    } else {
        P.lk[0] = q0 < n ? (uint32_t)L[q0] : 0u;
        P.lk[1] = 0u;
    }
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const int64_t q = ts + tid + u * kZThreads;
        P.key[u] = q < n ? (uint32_t)K[q] : 0u;
    }
}
// the new tile goes to words [kZH + kZT, kZH + 2 kZT) and its pad after it;
// the low half of a word is the LDS word index of the position's predecessor
// (0: none), as in k_match (tile_store<true>)
__device__ __attribute__((always_inline)) inline void zpre_store(uint32_t *E, const ZPre &P, int tid) {
    const int w0 = kZH + kZT + 2 * tid;
    uint2 v;
    v.x = P.b[0] << 16 | (P.lk[0] ? ((uint32_t)w0 - P.lk[0]) & 0xffffu : 0u);
    v.y = P.b[1] << 16 | (P.lk[1] ? ((uint32_t)(w0 + 1) - P.lk[1]) & 0xffffu : 0u);
    *reinterpret_cast<uint2 *>(E + w0) = v;
    if (tid < kMPad / 4)
        *reinterpret_cast<uint4 *>(E + kZH + 2 * kZT + 4 * tid) =
            make_uint4(P.pb[0] << 16, P.pb[1] << 16, P.pb[2] << 16, P.pb[3] << 16);
}
// window slide by kZT words: thread t moves the 2-word chunks t + 1024 k in
// increasing k; the chunk it reads (c + kZT/2 = c + 1024) is the one it writes
// next, so no chunk is overwritten before it is read.  Predecessor indexes
// drop by kZT, saturating at 0 (older than the window: beyond every limit).
__device__ __attribute__((always_inline)) inline void zslide(uint32_t *E, int tid) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const us2 d = {(unsigned short)kZT, (unsigned short)0};
    auto sl = [&](uint32_t w) {
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(us2, w), d));
    };
    uint2 *dE = reinterpret_cast<uint2 *>(E);
    constexpr int kChunks = (kZH + kZT) / 2;
    static_assert(kZT / 2 == kZThreads, "self-contained slide chains");
    for (int c = tid; c < kChunks; c += kZThreads) {
        const uint2 v = dE[c + kZT / 2];
        dE[c] = make_uint2(sl(v.x), sl(v.y));
    }
}

// walk outputs: the quarter walk's result (global, with the exact flag), a
// full walk's result (LDS, over the parse tile's quarter word)
// (statistics build: `c` receives the walk's step count)
struct ZOutQ {
    uint32_t *dst;
    mutable uint32_t c = 0;
    __device__ __attribute__((always_inline)) inline void full(uint32_t r, bool exact) const {
        *dst = r | (exact ? kZX : 0u);
    }
    __device__ __attribute__((always_inline)) inline void quart(uint32_t) const {}
    __device__ __attribute__((always_inline)) inline void steps(uint32_t k) const { c = k; }
};
struct ZOutF {
    uint32_t *dst;
    mutable uint32_t c = 0;
    __device__ __attribute__((always_inline)) inline void full(uint32_t r, bool) const { *dst = r | kZF; }
    __device__ __attribute__((always_inline)) inline void quart(uint32_t) const {}
    __device__ __attribute__((always_inline)) inline void steps(uint32_t k) const { c = k; }
};

struct ZLane {
    uint32_t p, ml, ms, av;
};
// one deflate_slow decision (deflate.c:1946-2027), as slow_step, on the parse
// tile's results: ZQ[p - a] holds Q(p) (bit kZX: = F(p)) or, once walked,
// F(p) (bit kZF; Q(p) is then still in the global rq[p]).  A decision that
// needs F(p) while only the inexact Q(p) is known takes Q(p) and sets guess.
// Returns 0 (no symbol), 1 (literal at spos), 2 (match at spos, slen); kSym:
// also the symbol (only the emission needs it: no byte read in the passes).
// The step is one LDS read and selects: the parse wave's loops are a chain of
// dependent steps, so its latency, not its issue count, is what costs.
template <bool kSym>
__device__ __attribute__((always_inline)) inline uint32_t zstep(ZLane &L, uint32_t n, const uint32_t *ZQ, uint32_t a,
                                                                const uint32_t *rqg, const uint32_t *E, int64_t B,
                                                                const LevelCfg &cfg, bool use_q, bool filtered,
                                                                bool &guess, uint32_t &sym, uint32_t &spos,
                                                                uint32_t &slen) {
    const uint32_t p = L.p, pl = L.ml, pm = L.ms;
    const bool srch = (n - p >= (uint32_t)kMinMatch) & (pl < cfg.lazy);
    const bool wantq = use_q & (pl >= cfg.good);
    uint32_t w = ZQ[p - a];
    if (srch & wantq & ((w & kZF) != 0u)) w = rqg[p];        // the quarter result, under a full one (rare)
    guess = srch & !wantq & ((w & (kZF | kZX)) == 0u);
    const uint32_t rl = srch ? (w >> 16) & 0x1ffu : 0u;
    const bool better = rl > pl;
    uint32_t ml = better ? rl : (uint32_t)kMinMatch - 1;
    const uint32_t ms = better ? p - (w & 0xffffu) : pm;
    const bool drop = (ml <= 5u) & (filtered | ((ml == (uint32_t)kMinMatch) & (p - ms > (uint32_t)kTooFar)));
    ml = drop ? (uint32_t)kMinMatch - 1 : ml;                  // deflate.c:1964-1975
    const bool emit = (pl >= (uint32_t)kMinMatch) & (ml <= pl);
    if (kSym) {
        sym = emit ? ((p - 1 - pm) << 8) | (pl - kMinMatch) : (E[(int64_t)p - 1 - B] >> 16) & 0xffu;
        spos = p - 1;
        slen = emit ? pl : 1u;
    }
    const uint32_t code = emit ? 2u : L.av;
    L.p = emit ? p + pl - 1 : p + 1;
    L.ms = ms;
    L.ml = emit ? (uint32_t)kMinMatch - 1 : ml;
    L.av = emit ? 0u : 1u;
    return code;
}

__device__ __attribute__((always_inline)) inline uint32_t lds_ld(const uint32_t *a) {
    return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ __launch_bounds__(kZThreads) void k_lzp(DeflateJob job) {
    constexpr int kSortBuckets = 64;
    __shared__ __attribute__((aligned(16))) uint32_t E[kZE];
    __shared__ __attribute__((aligned(16))) uint32_t ZQ[kZT];
    __shared__ uint16_t perm[kZT];
    __shared__ uint32_t rec[kZT / 16];
    __shared__ uint16_t req[kZReq];
    __shared__ uint32_t zst[64];
    __shared__ int s_hist[kSortBuckets], s_base[kSortBuckets];
    __shared__ uint32_t sdone[kZT / 32];          // speculative full walks done (results in job.rfull)
    __shared__ uint32_t c_qnext, c_rhead, c_rtail, c_rdone, c_pdone, c_post, c_total, c_final, c_snext;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const uint32_t n = (uint32_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    const uint16_t *Lk = job.link + job.ws_off[bi];
    const uint8_t *K = job.key + job.ws_off[bi];
    uint32_t *rqg = job.rquart + job.ws_off[bi];
    uint32_t *sym = job.sym + job.ws_off[bi];
    BlockRec *blk = job.blocks + job.blk_off[bi];
    const LevelCfg cfg = job.cfg;
    LevelCfg cfgq = cfg;
    cfgq.chain = cfg.chain >> 2 ? cfg.chain >> 2 : 1u;
    const WinP wp = job_win(job);
    const int64_t max_dist = wp.max_dist;
    const uint32_t symlim = wp.sym_limit;
    const bool use_q = cfg.good < cfg.lazy;
    const bool filtered = job.strategy == 1;
    // the sort key of a quarter walk: k_count's candidate count, capped at the budget
    const uint32_t kcap = walk_key(cfgq.chain, cfg.chain);
    const uint32_t S = (n + kZT - 1) / kZT;

    // the parser wave's carried state (uniform): where the parse stands at the
    // start of the next tile, the symbols written so far
    uint32_t cp = 0, cml = kMinMatch - 1, cms = 0, cav = 0, symbase = 0, sfinal = 0;

    ZPre P;
    zpre_load(P, 0, n, in, Lk, K, tid);
    const bool prio = job.lzp_flags & 1;
    const bool spec = (job.lzp_flags & 2) && job.rfull;
    uint32_t *rfs = job.rfull ? job.rfull + job.ws_off[bi] : nullptr;
#ifdef ZGPU_LZP_STATS
    unsigned long long st_qw = 0, st_qs = 0, st_fw = 0, st_fs = 0, st_idle = 0, st_sw = 0;
#endif
    for (uint32_t s = 0; s <= S; s++) {
        const uint64_t t_step = ZCLK();
        const int64_t ts = (int64_t)s * kZT;                 // tile s (quarter walks)
        const int64_t B = ts - kZT - kZH;                    // word w <-> position B + w
        const int tile_n = s < S ? (int)((int64_t)n - ts < kZT ? (int64_t)n - ts : kZT) : 0;
        const uint32_t a = s ? (s - 1) * kZT : 0u;          // tile s-1 (parse) [a, b)
        const uint32_t b = s ? (a + kZT < n ? a + kZT : n) : 0u;
        // ---- staging
        if (s == 0) {
            for (int i = tid; i < kZH + kZT; i += kZThreads) E[i] = 0;
        } else {
            zslide(E, tid);
            __syncthreads();
        }
        if (tile_n) zpre_store(E, P, tid);
        if (s) {                                            // tile s-1's quarter results
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t i = (uint32_t)tid + (uint32_t)u * kZThreads;
                ZQ[i] = a + i < n ? rqg[a + i] : 0u;
            }
        }
        if (tid < kSortBuckets) s_hist[tid] = 0;
        if (tid < kZT / 32) sdone[tid] = 0;
        if (tid == 0) {
            c_qnext = 0;
            c_rhead = c_rtail = c_rdone = 0;
            c_pdone = s ? 0u : 1u;
            c_snext = 0;
        }
        __syncthreads();
        int bk[2], rk[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int i = tid + u * kZThreads;
            const uint32_t k = P.key[u] < kcap ? P.key[u] : kcap;
            bk[u] = kSortBuckets - 1 - (i < tile_n ? (int)(k >> 2) : 0);
            if (bk[u] < 0) bk[u] = 0;
            rk[u] = i < tile_n ? atomicAdd(&s_hist[bk[u]], 1) : 0;
        }
        __syncthreads();
        if (tid < 64) {
            const int v = s_hist[tid];
            int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if (tid >= o) incl += t;
            }
            s_base[tid] = incl - v;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; u++)
            if (tid + u * kZThreads < tile_n) perm[s_base[bk[u]] + rk[u]] = (uint16_t)(tid + u * kZThreads);
        __syncthreads();
        if (s + 1 < S) zpre_load(P, ts + kZT, n, in, Lk, K, tid);     // lands during the walks

        // ---- full walks posted by the parser (tile s-1 offsets), wave-wide
        // claims of up to 64; returns false when none were pending
        auto ext_walks = [&](int pr) -> bool {
            const uint32_t h = ufl(lds_ld(&c_rhead)), t = ufl(lds_ld(&c_rtail));
            if (h >= t) return false;
            const uint32_t take = t - h < 64u ? t - h : 64u;
            uint32_t got = 0;
            if (lane == 0) got = atomicCAS(&c_rhead, h, h + take) == h;
            if (!ufl(got)) return true;                      // lost the claim: look again
            if (prio) __builtin_amdgcn_s_setprio(2);
            if ((uint32_t)lane < take) {
                const uint32_t off = req[(h + (uint32_t)lane) % kZReq];
                const ZOutF o{ZQ + off};
                dwq_walk(E, (int64_t)a + off, B, n, cfg, o, 0, max_dist);
#ifdef ZGPU_LZP_STATS
                st_fw++;
                st_fs += o.c;
#endif
            }
            if (prio) {
                if (pr == 3) __builtin_amdgcn_s_setprio(3);
                else __builtin_amdgcn_s_setprio(0);
            }
            __threadfence_block();
            if (lane == 0) atomicAdd(&c_rdone, take);
            return true;
        };

        // ---- the parser wave: rounds over tile s-1, then its symbols
        if (wave == kZParser && s) {
            if (prio) __builtin_amdgcn_s_setprio(3);
            uint64_t t0 = ZCLK(), t_p12 = 0, t_rep = 0, t_wait = 0;
            const uint32_t x0 = a + (uint32_t)kZSeg * (uint32_t)lane;
            const uint32_t x1 = x0 + kZSeg < b ? x0 + kZSeg : b;
            const bool act = x0 < b;
            const bool tail_tile = b == n;
            bool gs;
            uint32_t sv, sp, sl;
            auto init = [&](ZLane &L) {
                if (lane == 0) L = ZLane{cp, cml, cms, cav};
                else L = ZLane{x0, kMinMatch - 1, 0, 0};
            };
            auto step = [&](ZLane &L) {
                return zstep<false>(L, n, ZQ, a, rqg, E, B, cfg, use_q, filtered, gs, sv, sp, sl);
            };
            auto step_sym = [&](ZLane &L) {
                return zstep<true>(L, n, ZQ, a, rqg, E, B, cfg, use_q, filtered, gs, sv, sp, sl);
            };
            uint32_t rounds = 0, last = 0, st_p = 0, en = 0, cnt = 0;
            uint32_t merged = 0;                  // this lane's 32 positions: speculative results taken
            (void)rounds;
            bool on = false;
            for (;;) {
                rounds++;
                uint64_t t1 = ZCLK();
                if (spec) {                       // take the speculative full walks done so far
                    uint32_t m = lds_ld(&sdone[lane]) & ~merged;
                    merged |= m;
                    while (m) {
                        const uint32_t j = (uint32_t)__builtin_ctz(m);
                        m &= m - 1;
                        const uint32_t o = (uint32_t)kZSeg * (uint32_t)lane + j;
                        if (!(ZQ[o] & kZF)) ZQ[o] = rfs[a + o] | kZF;
                    }
                    __threadfence_block();
                }
                // pass 1: the own segment, recording the simple states
                ZLane L;
                init(L);
                if (act) {
                    uint32_t r0 = 0, r1 = 0;
                    while (L.p < x1) {
                        const uint32_t o = L.p - x0;
                        const uint32_t bit = L.ml < (uint32_t)kMinMatch ? 1u << (2 * (o & 15u) + L.av) : 0u;
                        r0 |= o < 16 ? bit : 0u;
                        r1 |= o < 16 ? 0u : bit;
                        step(L);
                    }
                    rec[(x0 - a) >> 4] = r0;
                    rec[((x0 - a) >> 4) + 1] = r1;
                }
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                // pass 2: run on until a later lane's recorded state
                uint32_t y = kZEnd, tgt = 0, sig = 0;
                if (act) {
                    while (L.p < b) {
                        if (L.p >= x1 && L.ml < (uint32_t)kMinMatch) {
                            const uint32_t o = L.p - a;
                            if ((rec[o >> 4] >> (2 * (o & 15u) + L.av)) & 1u) {
                                y = L.p;
                                sig = L.av;
                                tgt = o / kZSeg;
                                break;
                            }
                        }
                        step(L);
                    }
                }
                {
                    const uint64_t t2 = ZCLK();
                    t_p12 += t2 - t1;
                    t1 = t2;
                }
                // stitch: lane 0, then each meet's lane, until a lane reaches b
                uint32_t cur = 0;
                uint64_t mask = 0;
                for (;;) {
                    mask |= 1ull << cur;
                    const uint32_t yv = (uint32_t)__builtin_amdgcn_readlane((int)y, (int)cur);
                    if (yv == kZEnd) break;
                    const uint32_t j = (uint32_t)__builtin_amdgcn_readlane((int)tgt, (int)cur);
                    const uint32_t sg = (uint32_t)__builtin_amdgcn_readlane((int)sig, (int)cur);
                    if (lane == 0) zst[j] = (yv - a) | sg << 16;
                    cur = j;
                }
                last = cur;
                if (lane == 0) c_post = 0;
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                on = (mask >> lane) & 1ull;
                st_p = lane == 0 ? cp : a + (zst[lane] & 0xffffu);
                en = (uint32_t)lane == last ? b : y;
                // replay the path: count the symbols, list the guessed sites
                const uint32_t tail0 = ufl(lds_ld(&c_rtail));
                cnt = 0;
                uint32_t ng = 0;
                if (on) {
                    init(L);
                    while (L.p < en) {
                        const uint32_t p0 = L.p;
                        const uint32_t k = step(L);
                        if (p0 >= st_p) {
                            cnt += k != 0;
                            if (gs) {
                                ng++;
                                const uint32_t i = atomicAdd(&c_post, 1u);
                                if (i < (uint32_t)kZReq) req[(tail0 + i) % kZReq] = (uint16_t)(p0 - a);
                            }
                        }
                    }
                }
                uint32_t tot = ng;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) tot += __shfl_xor(tot, o, 64);
                tot = ufl(tot);
                {
                    const uint64_t t2 = ZCLK();
                    t_rep += t2 - t1;
                    t1 = t2;
                }
                if (tot == 0) break;
                const uint32_t posted = tot < (uint32_t)kZReq ? tot : (uint32_t)kZReq;
#ifdef ZGPU_LZP_STATS
                if (lane == 0) {
                    ZSTAT(2, posted);
                    ZSTAT(7, tot - posted);
                }
#endif
                __threadfence_block();
                if (lane == 0) __hip_atomic_store(&c_rtail, tail0 + posted, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                // take full walks until this round's are done
                for (;;) {
                    if (ext_walks(3)) continue;
                    if (ufl(lds_ld(&c_rdone)) >= tail0 + posted) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                __threadfence_block();
                t_wait += ZCLK() - t1;
            }
            const uint64_t t_emit = ZCLK();
#ifdef ZGPU_LZP_STATS
            if (lane == 0) {
                ZSTAT(0, 1);
                ZSTAT(1, rounds);
                ZSTAT(8 + (rounds > 8 ? 7 : rounds - 1), 1);
            }
#endif
            // the symbols: lane i's on the path from st_p to en, in path order
            uint32_t incl = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o, 64);
                if (lane >= o) incl += t;
            }
            uint32_t gi = symbase + incl - cnt;
            ZLane L;
            init(L);
            if (on) {
                while (L.p < en) {
                    const uint32_t p0 = L.p;
                    const uint32_t k = step_sym(L);
                    if (p0 >= st_p && k) {
                        sym[gi] = sv;
                        if ((gi + 1) % symlim == 0) {                 // the flush at this symbol (deflate.h:371)
                            const uint32_t bx = (gi + 1) / symlim - 1;
                            blk[bx].in_end = (uint64_t)(sp + sl);
                            blk[bx].pad = sp + 1;                     // its decision point
                        }
                        gi++;
                    }
                }
            }
            uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            const uint32_t np = (uint32_t)__builtin_amdgcn_readlane((int)L.p, (int)last);
            const uint32_t nml = (uint32_t)__builtin_amdgcn_readlane((int)L.ml, (int)last);
            const uint32_t nms = (uint32_t)__builtin_amdgcn_readlane((int)L.ms, (int)last);
            const uint32_t nav = (uint32_t)__builtin_amdgcn_readlane((int)L.av, (int)last);
            if (tail_tile && nav) {                 // the pending literal at the end, tallied without a flush test
                if ((uint32_t)lane == last) sym[gi] = (E[(int64_t)n - 1 - B] >> 16) & 0xffu;
                total++;
                sfinal = 1;
            }
            cp = np; cml = nml; cms = nms; cav = nav;
            symbase += total;
            __threadfence_block();
            if (lane == 0) __hip_atomic_store(&c_pdone, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (prio) __builtin_amdgcn_s_setprio(0);
#ifdef ZGPU_LZP_STATS
            if (lane == 0) {
                const uint64_t t3 = ZCLK();
                ZSTAT(16, t_p12);
                ZSTAT(17, t_rep);
                ZSTAT(18, t_wait);
                ZSTAT(19, t3 - t_emit);
                ZSTAT(20, t3 - t0);
            }
#else
            (void)t0; (void)t_p12; (void)t_rep; (void)t_wait; (void)t_emit;
#endif
        }

        // ---- walkers (and the parser once its tile is done)
        for (;;) {
            if (ext_walks(0)) continue;
            if (ufl(lds_ld(&c_qnext)) < (uint32_t)tile_n) {
                uint32_t i0 = 0;
                if (lane == 0) i0 = atomicAdd(&c_qnext, 64u);
                i0 = ufl(i0);
                const uint32_t i = i0 + (uint32_t)lane;
                if (i < (uint32_t)tile_n) {
                    const int64_t p = ts + perm[i];
                    const ZOutQ o{rqg + p};
                    dwq_walk(E, p, B, n, cfgq, o, 0, max_dist);
#ifdef ZGPU_LZP_STATS
                    st_qw++;
                    st_qs += o.c;
#endif
                }
                continue;
            }
            if (ufl(lds_ld(&c_pdone))) break;
            // idle while the parser works: full walks of the parse tile's inexact
            // positions (results in rfs, taken by the parser at its next round)
            if (spec && s && ufl(lds_ld(&c_snext)) < b - a) {
                uint32_t o0 = 0;
                if (lane == 0) o0 = atomicAdd(&c_snext, 64u);
                const uint32_t o = ufl(o0) + (uint32_t)lane;
                if (o < b - a && !(ZQ[o] & (kZF | kZX))) {
                    const ZOutQ so{rfs + a + o};
                    dwq_walk(E, (int64_t)a + o, B, n, cfg, so, 0, max_dist);
                    __threadfence_block();
                    atomicOr(&sdone[o >> 5], 1u << (o & 31u));
#ifdef ZGPU_LZP_STATS
                    st_sw++;
#endif
                }
                continue;
            }
#ifdef ZGPU_LZP_STATS
            st_idle++;
#endif
            __builtin_amdgcn_s_sleep(2);
        }
        __threadfence_block();
        __syncthreads();
#ifdef ZGPU_LZP_STATS
        if (tid == 0) ZSTAT(21, ZCLK() - t_step);
#else
        (void)t_step;
#endif
    }
#ifdef ZGPU_LZP_STATS
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        st_qw += __shfl_xor(st_qw, o, 64);
        st_qs += __shfl_xor(st_qs, o, 64);
        st_fw += __shfl_xor(st_fw, o, 64);
        st_fs += __shfl_xor(st_fs, o, 64);
        st_sw += __shfl_xor(st_sw, o, 64);
    }
    if (lane == 0) {
        ZSTAT(3, st_qw);
        ZSTAT(4, st_qs);
        ZSTAT(5, st_fw);
        ZSTAT(6, st_fs);
        ZSTAT(22, st_idle);
        ZSTAT(23, st_sw);
    }
#endif
    if (wave == kZParser && lane == 0) {
        c_total = symbase;
        c_final = sfinal;
    }
    __syncthreads();
    const uint32_t total = c_total;
    const uint32_t ncut = total / symlim - ((c_final && total % symlim == 0) ? 1u : 0u);
    seg_block_records<kZThreads>(blk, n, total, ncut, wp, tid);
    if (tid == 0) job.nblocks[bi] = ncut + 1;
}

#endif  // ZGPU_LZP
int lzp_built() {
#ifdef ZGPU_LZP
    return 1;
#else
    return 0;
#endif
}

// ------------------------------------------------------------------------
// k_pbig1..6 — k_parse_seg's speculative segmented lazy parse for a sub-batch
// of few large buffers (a lone compress2, say), with a buffer's segments
// spread over many workgroups instead of one.  The steps are k_parse_seg's;
// each block-wide barrier of k_parse_seg becomes a kernel boundary, and what
// its lanes kept in registers or LDS across a barrier lives in PLane records:
//   k_pbig1  pass 1 of every segment (symbols staged, simple states recorded)
//   k_pbig2  pass 2: run on into the next segment until the two parses meet
//   k_pbig3  replays: the prefix before y(i-1), the run-on up to y(i)
//   k_pbig4  per buffer: exclusive scan of the lanes' symbol counts
//   k_pbig5  compaction into sym[] and the block cuts
//   k_pbig6  block records (slides before each flush by binary search)
// A buffer whose lanes do not meet within the next segment goes to
// k_parse_slow (nblocks = kParseFallback), as with k_parse_seg.
// DeflateJob::pgrp maps a workgroup to (buffer, first lane); a buffer has
// ceil(n / pseg) lanes, the global index of its lane 0 is plbase[buffer].
// ------------------------------------------------------------------------
struct PCtx {
    uint32_t bi, lane, nl, n, seg, gl;
    uint32_t st;             // where lane 0 starts: 0, or a streaming job's resume point (job.start)
    bool active;
    const uint8_t *in;
    const uint32_t *rf, *rq;
    uint32_t *sym, *stg, *sst;
    BlockRec *blk;
    __device__ inline uint32_t xb(uint32_t i) const {
        const uint64_t v = (uint64_t)st + (uint64_t)i * seg;
        return v < n ? (uint32_t)v : n;
    }
    __device__ inline uint32_t seg_end() const { return lane + 1 >= nl ? n : xb(lane + 1); }
};
__device__ inline uint32_t pbig_lanes(uint32_t n, uint32_t seg) {
    const uint32_t k = (n + seg - 1) / seg;
    return k ? k : 1u;
}
__device__ inline PCtx pbig_ctx(const DeflateJob &job, uint32_t grp = blockIdx.x, uint32_t tl = threadIdx.x) {
    PCtx c;
    c.bi = job.pgrp[2 * grp];
    c.lane = job.pgrp[2 * grp + 1] + tl;
    const uint32_t g = job.first + c.bi;
    c.n = (uint32_t)job.src_len[g];
    c.seg = job.pseg;
    c.st = job.start;
    c.nl = pbig_lanes(c.n - c.st, c.seg);
    c.active = c.lane < c.nl;
    c.gl = job.plbase[c.bi] + c.lane;
    c.in = job.src + job.src_off[g];
    c.rf = job.rfull + job.ws_off[c.bi];
    c.rq = job.rquart + job.ws_off[c.bi];
    c.sym = job.sym + job.ws_off[c.bi];
    c.stg = job.stage + job.ws_off[c.bi];
    c.sst = job.pstate + (job.ws_off[c.bi] >> 4);
    c.blk = job.blocks + job.blk_off[c.bi];
    return c;
}

__global__ __launch_bounds__(kParseLanes) void k_pbig1(DeflateJob job) {
    const PCtx c = pbig_ctx(job);
    if (c.lane == 0) job.pbuf[c.bi] = PBuf{0u, kEnd, 0u, 0u};
    if (!c.active) return;
    const LevelCfg cfg = job.cfg;
    const bool use_q = cfg.good < cfg.lazy, filtered = job.strategy == 1;
    SlowLaneW L;
    uint32_t sym_v, spos, slen;
    const uint32_t x0 = c.xb(c.lane), seg_end = c.seg_end();
    lane_init(L, x0, 0);
    SymBuf sb{0, 0, 0, 0, 0};
    if (x0 < seg_end) {                               // as k_parse_seg's pass 1
        uint32_t widx = x0 >> 4, wcur = 0;
        while (L.p < seg_end) {
            const uint32_t wi = L.p >> 4;
            if (wi != widx) {
                c.sst[widx] = wcur;
                for (uint32_t z = widx + 1; z < wi; z++) c.sst[z] = 0;
                widx = wi;
                wcur = 0;
            }
            if (L.ml < (uint32_t)kMinMatch) wcur |= 1u << (2 * (L.p & 15u) + L.avail);
            if (slow_step(L, c.n, c.rf, c.rq, c.in, cfg, use_q, filtered, sym_v, spos, slen)) sb.push(c.stg + x0, sym_v);
        }
        c.sst[widx] = wcur;
        for (uint32_t z = widx + 1; z <= (seg_end - 1) >> 4; z++) c.sst[z] = 0;
        sb.flush(c.stg + x0);
    }
    PLane &r = job.plane[c.gl];
    r.e_p = L.p; r.e_ml = L.ml; r.e_ms = L.ms; r.e_av = L.avail;
    r.k1 = sb.k;
}

// k_pbig1s — k_pbig1 for 256-byte segments (preach > 1), one wave of 64 lanes per workgroup, with the
// lanes' records and bytes in LDS.  Pass 1 reads only its own segment's rfull words and bytes, so the
// wave's 64 segments (16 KiB of positions) are copied in once, coalesced, and every step reads LDS.  In
// k_pbig1 the lanes' record lines come from L2 and nearly every step of the wave waits for some lane's
// line (a lane crosses a 64-byte line every few steps, and 64 lanes share the wait).
constexpr int kP1sLanes = 64, kP1sSpan = kP1sLanes * (int)kSmallSeg;
__global__ __launch_bounds__(kP1sLanes) void k_pbig1s(DeflateJob job) {
    __shared__ uint32_t s_rf[kP1sSpan];
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kP1sSpan + 16];
    const uint32_t grp = blockIdx.x / (kParseLanes / kP1sLanes), q = blockIdx.x % (kParseLanes / kP1sLanes);
    const PCtx c = pbig_ctx(job, grp, q * kP1sLanes + threadIdx.x);
    const uint32_t l0 = c.lane - threadIdx.x;          // the wave's first lane
    if (l0 >= c.nl) return;                            // uniform: no lane of this wave exists
    if (c.lane == 0) job.pbuf[c.bi] = PBuf{0u, kEnd, 0u, 0u};
    const uint32_t X0 = c.xb(l0);
    const uint32_t X1 = l0 + kP1sLanes >= c.nl ? c.n : c.xb(l0 + kP1sLanes);   // X1 - X0 <= kP1sSpan
    {   // coalesced 16-byte loads, 16 per thread in flight per batch (X0 is a multiple of 256)
        const int tid = threadIdx.x;
        const uint32_t nw = ((X1 - X0) + 3u) & ~3u;
#pragma unroll 1
        for (uint32_t b = 0; b < nw; b += 4096)
            stage_words<kP1sLanes, 16>(s_rf + b, c.rf, (int64_t)X0 + b, (int)(nw - b < 4096 ? nw - b : 4096),
                                       (int64_t)X1, tid);
        stage_bytes<kP1sLanes, (kP1sSpan + 16) / 16 / kP1sLanes + 1>(s_in, c.in, X0, (int)(((X1 - X0) + 15u) & ~15u),
                                                                   (int64_t)c.n, tid);
    }
    __syncthreads();
    if (!c.active) return;
    const LevelCfg cfg = job.cfg;
    const bool use_q = cfg.good < cfg.lazy, filtered = job.strategy == 1;
    SlowLaneD L;
    L.cf.base = X0;
    L.cb.base = X0;
    uint32_t sym_v, spos, slen;
    const uint32_t x0 = c.xb(c.lane), seg_end = c.seg_end();
    lane_init(L, x0, 0);
    SymBuf sb{0, 0, 0, 0, 0};
    if (x0 < seg_end) {                               // as k_pbig1
        uint32_t widx = x0 >> 4, wcur = 0;
        while (L.p < seg_end) {
            const uint32_t wi = L.p >> 4;
            if (wi != widx) {
                c.sst[widx] = wcur;
                for (uint32_t z = widx + 1; z < wi; z++) c.sst[z] = 0;
                widx = wi;
                wcur = 0;
            }
            if (L.ml < (uint32_t)kMinMatch) wcur |= 1u << (2 * (L.p & 15u) + L.avail);
            if (slow_step(L, c.n, s_rf, c.rq, s_in, cfg, use_q, filtered, sym_v, spos, slen)) sb.push(c.stg + x0, sym_v);
        }
        c.sst[widx] = wcur;
        for (uint32_t z = widx + 1; z <= (seg_end - 1) >> 4; z++) c.sst[z] = 0;
        sb.flush(c.stg + x0);
    }
    PLane &r = job.plane[c.gl];
    r.e_p = L.p; r.e_ml = L.ml; r.e_ms = L.ms; r.e_av = L.avail;
    r.k1 = sb.k;
}

__global__ __launch_bounds__(kParseLanes) void k_pbig2(DeflateJob job) {
    const PCtx c = pbig_ctx(job);
    if (!c.active) return;
    const LevelCfg cfg = job.cfg;
    const bool use_q = cfg.good < cfg.lazy, filtered = job.strategy == 1;
    PLane &r = job.plane[c.gl];
    SlowLaneW L;
    lane_init(L, r.e_p, r.e_av);
    L.ml = r.e_ml; L.ms = r.e_ms;
    uint32_t sym_v, spos, slen;
    uint32_t y = kEnd, sig = 0;
    bool fail = false;
    if (c.lane + 1 < c.nl) {                          // as k_parse_seg's pass 2
        const uint32_t next_start = c.xb(c.lane + 1);
        const uint32_t reach = job.preach > 1 ? job.preach : 1u;
        const uint32_t stop = c.lane + 1 + reach >= c.nl ? c.n : c.xb(c.lane + 1 + reach);
        uint32_t ridx = 0xffffffffu, rw = 0;
        for (;;) {
            if (L.p >= c.n) { y = kEnd; break; }
            if (L.p >= stop) { fail = true; break; }
            if (L.p >= next_start && L.ml < (uint32_t)kMinMatch) {
                if ((L.p >> 4) != ridx) { ridx = L.p >> 4; rw = c.sst[ridx]; }
                if ((rw >> (2 * (L.p & 15u) + L.avail)) & 1u) { y = L.p; sig = L.avail; break; }
            }
            slow_step(L, c.n, c.rf, c.rq, c.in, cfg, use_q, filtered, sym_v, spos, slen);
        }
    }
    r.y = y;
    r.sig = sig;
    if (fail) atomicOr(&job.pbuf[c.bi].fail, 1u);
    if (y == kEnd) atomicMin(&job.pbuf[c.bi].first_end, c.lane);
}

// The lanes whose symbols make the stream: lane 0, then the lane whose segment
// holds lane 0's meet y(0), then the one holding that lane's meet, ... (the
// chain of meets); each takes its pass-1 symbols from the previous meet on and
// its run-on up to its own.  With preach 1 every meet lies in the next segment,
// so the chain is every lane up to the first whose run-on reached the end.
__global__ __launch_bounds__(kParseLanes) void k_pbig3(DeflateJob job) {
    __shared__ uint32_t s_st[kParseLanes], s_p0[kParseLanes];
    __shared__ uint64_t s_on[kParseLanes / 64];
    const PCtx c = pbig_ctx(job);
    if (job.pbuf[c.bi].fail) return;                  // uniform: a workgroup's lanes share a buffer
    const bool chain = job.preach > 1;                // the buffer is this workgroup's (nl <= kParseLanes)
    const int tid = threadIdx.x;
    if (chain) {
        if (tid < 64) {
            // wave 0: the lanes' next chain lane, 64 at a time in registers, followed with readlane
            const uint32_t gl0 = job.plbase[c.bi];
            uint32_t e = 0, prev_y = c.st, prev_sig = 0;
            bool done = false;
            for (uint32_t w = 0; w < (uint32_t)kParseLanes; w += 64) {
                uint64_t on = 0;
                if (!done && w < c.nl) {
                    const uint32_t li = w + (uint32_t)tid;
                    uint32_t y = kEnd, sg = 0;
                    if (li < c.nl) { y = job.plane[gl0 + li].y; sg = job.plane[gl0 + li].sig; }
                    const uint32_t nx = y == kEnd ? kEnd : (y - c.st) / c.seg;
                    while (e < w + 64) {                  // wave-uniform
                        const uint32_t k = e - w;
                        on |= 1ull << k;
                        if (tid == 0) { s_st[e] = prev_y; s_p0[e] = prev_y - prev_sig; }
                        const uint32_t ye = (uint32_t)__builtin_amdgcn_readlane((int)y, (int)k);
                        if (ye == kEnd) { done = true; break; }
                        prev_sig = (uint32_t)__builtin_amdgcn_readlane((int)sg, (int)k);
                        prev_y = ye;
                        e = (uint32_t)__builtin_amdgcn_readlane((int)nx, (int)k);
                    }
                }
                if (tid == 0) s_on[w >> 6] = on;
            }
        }
        __syncthreads();
    }
    if (!c.active) return;
    const LevelCfg cfg = job.cfg;
    const bool use_q = cfg.good < cfg.lazy, filtered = job.strategy == 1;
    PLane &r = job.plane[c.gl];
    bool mine;
    uint32_t start, p0;
    if (chain) {
        mine = (s_on[c.lane >> 6] >> (c.lane & 63u)) & 1u;
        start = s_st[c.lane];
        p0 = s_p0[c.lane];
    } else {
        mine = c.lane <= job.pbuf[c.bi].first_end;
        start = c.lane > 0 ? job.plane[c.gl - 1].y : 0u;
        p0 = c.lane > 0 ? job.plane[c.gl - 1].y - job.plane[c.gl - 1].sig : c.st;
    }
    const uint32_t x0 = c.xb(c.lane), seg_end = c.seg_end();
    const uint32_t yend = r.y, end = yend == kEnd ? c.n : yend;
    SlowLaneW L;
    const uint32_t *rfp = c.rf;
    const uint8_t *inp = c.in;
    uint32_t sym_v, spos, slen;
    uint32_t kstart = 0;
    if (mine && c.lane > 0) {                         // pass-1 symbols before the previous meet are not this lane's
        lane_init(L, x0, 0);
        while (L.p < start)
            if (slow_step(L, c.n, rfp, c.rq, inp, cfg, use_q, filtered, sym_v, spos, slen)) kstart++;
    }
    uint32_t rcnt = 0;
    // the run-on, staged in the lane's dead state words (or its pron slot)
    uint32_t *ron = chain ? job.pron + (size_t)c.gl * kRonCap : c.sst + (x0 >> 4);
    const uint32_t rcap = chain ? kRonCap : (seg_end - x0 + 15u) >> 4;
    if (mine) {
        lane_init(L, r.e_p, r.e_av);
        L.ml = r.e_ml; L.ms = r.e_ms;
        while (L.p < end) {
            if (slow_step(L, c.n, rfp, c.rq, inp, cfg, use_q, filtered, sym_v, spos, slen)) {
                if (rcnt < rcap) ron[rcnt] = sym_v;
                rcnt++;
            }
        }
        if (yend == kEnd && L.avail) {                // the final pending literal
            if (rcnt < rcap) ron[rcnt] = bget(inp, c.n - 1, L.cb);
            rcnt++;
            job.pbuf[c.bi].fin = 1u;
        }
        if (rcnt > rcap) atomicOr(&job.pbuf[c.bi].fail, 1u);
    }
    r.kstart = kstart;
    r.rcnt = rcnt;
    r.cnt = mine ? r.k1 - kstart + rcnt : 0u;
    r.p0 = p0;
}

constexpr int kPScanThreads = 1024;
__global__ __launch_bounds__(kPScanThreads) void k_pbig4(DeflateJob job) {
    __shared__ uint32_t s_wsum[kPScanThreads / 64];
    const int tid = threadIdx.x, wl = tid & 63, wv = tid >> 6;
    const uint32_t bi = blockIdx.x;
    const uint32_t n = (uint32_t)job.src_len[job.first + bi];
    const uint32_t nl = pbig_lanes(n - job.start, job.pseg);
    PLane *pl = job.plane + job.plbase[bi];
    if (job.pbuf[bi].fail) {
        if (tid == 0) job.nblocks[bi] = kParseFallback;
        return;
    }
    uint32_t run = 0;
    for (uint32_t c0 = 0; c0 < nl; c0 += kPScanThreads) {
        const uint32_t i = c0 + (uint32_t)tid;
        const uint32_t v = i < nl ? pl[i].cnt : 0u;
        uint32_t incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (wl >= o) incl += t;
        }
        if (wl == 63) s_wsum[wv] = incl;
        __syncthreads();
        uint32_t woff = 0, tot = 0;
        for (int k = 0; k < kPScanThreads / 64; k++) {
            const uint32_t t = s_wsum[k];
            if (k < wv) woff += t;
            tot += t;
        }
        if (i < nl) pl[i].base = run + woff + incl - v;
        run += tot;
        __syncthreads();
    }
    if (tid == 0) job.pbuf[bi].total = run;
}

// one workgroup per lane group as k_pbig1..3, with kP5Threads threads: the
// group's lanes are copied by all its waves in turn (lane t by wave t mod
// waves), where k_parse_seg's compaction has each wave copy its own 64 lanes.
// A lone buffer's 64..256 lanes are then not one wave's serial chain.
constexpr int kP5Threads = 1024;
__global__ __launch_bounds__(kP5Threads) void k_pbig5(DeflateJob job) {
    const PCtx c = pbig_ctx(job);                     // per-buffer fields only (lane is threadIdx-based)
    const PBuf pb = job.pbuf[c.bi];
    if (pb.fail) return;                              // uniform: a workgroup's lanes share a buffer
    const int wl = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t symlim = job_win(job).sym_limit;
    const uint32_t total = pb.total;
    const uint32_t ncut = total / symlim - ((pb.fin && total % symlim == 0) ? 1u : 0u);
    const bool filtered = job.strategy == 1;
    const uint32_t lane0 = job.pgrp[2 * blockIdx.x + 1], gl0 = job.plbase[c.bi];
    for (uint32_t tl = (uint32_t)wv; tl < (uint32_t)kParseLanes; tl += kP5Threads / 64) {
        const uint32_t jl = lane0 + tl;
        if (jl >= c.nl) break;                        // wave-uniform
        const PLane &r = job.plane[gl0 + jl];
        const uint32_t jc = r.cnt;
        if (jc == 0) continue;
        const uint32_t jb = r.base, jc1 = jc - r.rcnt, jx = c.xb(jl), jk = r.kstart;
        uint32_t run = r.p0;                          // the lane's symbols tile the input from here
        const uint32_t *s1 = c.stg + jx + jk;
        const uint32_t *s2 = job.preach > 1 ? job.pron + (size_t)(gl0 + jl) * kRonCap : c.sst + (jx >> 4);
        for (uint32_t k = 0; k < jc; k += 64) {
            const uint32_t idx = k + (uint32_t)wl;
            const bool have = idx < jc;
            const uint32_t v = have ? (idx < jc1 ? s1[idx] : s2[idx - jc1]) : 0u;
            const uint32_t len = have ? (v < 256u ? 1u : (v & 0xffu) + (uint32_t)kMinMatch) : 0u;
            uint32_t li = len;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(li, o, 64);
                if (wl >= o) li += t;
            }
            const uint32_t sp = run + li - len;
            run += __shfl(li, 63, 64);
            if (have) {
                const uint32_t gi = jb + idx;
                c.sym[gi] = v;
                if ((gi + 1) % symlim == 0 && (gi + 1) / symlim <= ncut) {
                    const uint32_t b = (gi + 1) / symlim - 1;
                    c.blk[b].in_end = (uint64_t)(sp + len);
                    c.blk[b].pad = sp + 1;                // decision point of the flush
                    // a streaming job's resume flag (k_pbig6s): a block cut by a
                    // literal leaves the simple state only when the search at the
                    // literal found nothing usable (k_parse_slow's flush res).
                    // rfull is the longest of the searches the parse may read
                    // there (rquart walks a prefix of the same chain).
                    if (job.srec) {
                        bool usable = false;
                        if (v < 256u) {
                            const uint32_t r = c.rf[sp] & ~kQDiff, rl = r >> 16;
                            usable = rl >= (uint32_t)kMinMatch &&
                                     !(rl <= 5u && (filtered || (rl == (uint32_t)kMinMatch && (r & 0xffffu) > (uint32_t)kTooFar)));
                        }
                        c.blk[b].flags = usable ? 1u : 0u;
                    }
                }
            }
        }
    }
}

// #{k >= 1 : slide_threshold(k) <= p}: the thresholds grow with k
__device__ inline uint32_t slides_upto(int64_t p, uint32_t n, int64_t refill, const WinP &w) {
    uint32_t lo = 0, hi = (uint32_t)(n / w.wsize) + 2;     // slide_threshold(hi + 1) > n >= p
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (slide_threshold(mid, n, refill, w) <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// one thread per block record; grid (blocks / 256, buffers)
__global__ __launch_bounds__(256) void k_pbig6(DeflateJob job) {
    const uint32_t bi = blockIdx.y;
    const PBuf pb = job.pbuf[bi];
    if (pb.fail) return;
    const WinP wp = job_win(job);
    const uint32_t symlim = wp.sym_limit;
    const uint32_t n = (uint32_t)job.src_len[job.first + bi];
    const uint32_t total = pb.total;
    const uint32_t ncut = total / symlim - ((pb.fin && total % symlim == 0) ? 1u : 0u);
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b == 0) job.nblocks[bi] = ncut + 1;
    if (b > ncut) return;
    BlockRec *blk = job.blocks + job.blk_off[bi];
    const bool last = b == ncut;
    // a record's in_end is rewritten with its own value, so the neighbour's
    // read of it (in_start) is safe in any order
    const uint64_t in_end = last ? n : blk[b].in_end;
    const uint64_t pd = last ? n : blk[b].pad;
    const uint64_t in_start = b == 0 ? 0 : blk[b - 1].in_end;
    const uint32_t slides = slides_upto((int64_t)pd, n, kMinLookahead - 1, wp);
    BlockRec r;
    r.sym_start = b * symlim;
    r.nsym = last ? total - b * symlim : symlim;
    r.in_start = in_start;
    r.in_end = in_end;
    r.flags = (last ? 1u : 0u) | (in_start >= (uint64_t)wp.wsize * slides ? 2u : 0u);
    r.pad = 0;
    blk[b] = r;
}

// ------------------------------------------------------------------------
// k_pbig6s — the block records of a streaming job parsed by k_pbig1..5, one
// workgroup.  The job's events are Z_NO_FLUSH stops only, so its symbols and
// block cuts are those of a parse of the whole input from job.start; what
// the stops change is fill_window's bookkeeping (the window offset S and the
// input read E recorded per block, k_parse_slow's ParseU::fill), which
// blocks come before each stop (ev_blk) and, for an open job, where it ends.
// That bookkeeping changes only at decision points p with E - p < 262
// (deflate.c:1941-1944 / :251-368): a slide once p - S >= w_size + MAX_DIST,
// a read up to min(S + 2 w_size, the call's input end), a stop when that end
// is reached.  Lane 0 replays the changes in order as thresholds "at the first
// decision point >= x" (a timeline: from x on the state is (S, E)); each block
// then looks its flush decision point up.  Where a slide and a threshold
// closer than 257 bytes (any 257 consecutive positions hold a decision point:
// a match skips at most 256) meet with no decision point known between them,
// the order is undetermined here and the job goes to k_parse_slow.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pbig6s(DeflateJob job) {
    __shared__ uint32_t s_ntl, s_bad, s_nb;
    const int tid = threadIdx.x;
    const PBuf pb = job.pbuf[0];
    if (pb.fail) return;                              // k_pbig4 flagged it already
    const WinP wp = job_win(job);
    const uint32_t symlim = wp.sym_limit, W = (uint32_t)wp.wsize, MD = (uint32_t)wp.max_dist;
    const uint32_t n = (uint32_t)job.src_len[job.first];
    const uint32_t total = pb.total;
    const uint32_t ncut = total / symlim - ((pb.fin && total % symlim == 0) ? 1u : 0u);
    const uint32_t st = job.start, nev = job.nfl;
    BlockRec *blk = job.blocks + job.blk_off[0];
    uint4 *tl = reinterpret_cast<uint4 *>(job.tl);
    uint32_t *ez = job.tl + 4ull * job.ntl;           // per stop: the point it triggers at
    // a decision point known in [a, b): the start or a block's flush point
    auto has_dp = [&](uint32_t a, uint32_t b) -> bool {
        if (st >= a && st < b) return true;
        uint32_t lo = 0, hi = ncut;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (blk[mid].pad < a) lo = mid + 1;
            else hi = mid;
        }
        return lo < ncut && blk[lo].pad < b;
    };
    if (tid == 0) {
        uint32_t S = 0, E = job.e0 > st ? job.e0 : st, i = 0;
        uint32_t lim = nev ? (uint32_t)job.fl_pos[0] : n;
        uint32_t k = 0, bad = 0;
        tl[k++] = make_uint4(0u, S, E, 0u);
        for (;;) {
            if (k + 2 > job.ntl) { bad = 1; break; }
            const uint32_t Z = E > (uint32_t)kMinLookahead - 1 ? E - ((uint32_t)kMinLookahead - 1) : 0u;
            const uint32_t Ts = S + W + MD;
            if (E == lim && i == nev) {               // all input read (closed): slides to the end
                const uint32_t x = Z > Ts ? Z : Ts;
                if (x > n) break;
                S += W;
                tl[k++] = make_uint4(x, S, E, 0u);
                continue;
            }
            // a read (E < lim) or a stop (E == lim) at the first decision point
            // p >= Z, where the slide test runs first: p >= Ts?
            bool slide;
            if (Z >= Ts) slide = true;
            else if (Ts - Z >= 257u || has_dp(Z, Ts)) slide = false;
            else { bad = 1; break; }
            if (slide) S += W;
            if (E < lim) {
                const uint32_t e = S + 2 * W;
                E = e < lim ? e : lim;
                tl[k++] = make_uint4(Z, S, E, 0u);
                continue;
            }
            ez[i++] = Z;                              // the stop: need_more, then the next call's read
            if (i == nev && job.open_end) {
                tl[k++] = make_uint4(Z, S, E, 0u);
                break;
            }
            lim = i < nev ? (uint32_t)job.fl_pos[i] : n;
            const uint32_t e = S + 2 * W;
            E = e < lim ? e : lim;
            tl[k++] = make_uint4(Z, S, E, 0u);
        }
        s_ntl = k;
        s_bad = bad;
    }
    __syncthreads();
    if (s_bad) {
        if (tid == 0) job.nblocks[0] = kParseFallback;
        return;
    }
    const uint32_t ntl = s_ntl;
    // blocks before each stop: those flushed at a decision point below its trigger
    for (uint32_t i = tid; i < nev; i += 256) {
        uint32_t lo = 0, hi = ncut;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (blk[mid].pad < ez[i]) lo = mid + 1;
            else hi = mid;
        }
        if (job.ev_blk) job.ev_blk[i] = lo;
        if (i + 1 == nev && job.open_end) s_nb = lo;
    }
    if (tid == 0 && !(nev && job.open_end)) s_nb = ncut + 1;
    __syncthreads();
    const uint32_t nb = s_nb;
    for (uint32_t b = tid; b < nb; b += 256) {
        const bool last = !job.open_end && b == ncut;
        const uint32_t in_end = last ? n : (uint32_t)blk[b].in_end;
        const uint32_t pd = last ? n : blk[b].pad;
        const bool res = last || blk[b].flags == 0u;
        const uint32_t in_start = b == 0 ? st : (uint32_t)blk[b - 1].in_end;
        uint32_t lo = 0, hi = ntl - 1;                // the last timeline entry at or before pd
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (tl[mid].x <= pd) lo = mid;
            else hi = mid - 1;
        }
        const uint4 t = tl[lo];
        job.srec[4ull * b + 2] = ((uint64_t)t.y << 32) | in_end;
        job.srec[4ull * b + 3] = (uint64_t)t.z | (res ? 1ull << 63 : 0ull);
        BlockRec r;
        r.sym_start = b * symlim;
        r.nsym = last ? total - b * symlim : symlim;
        r.in_start = in_start;
        r.in_end = in_end;
        r.flags = (last ? 1u : 0u) | (in_start >= t.y ? 2u : 0u);
        r.pad = 0;
        blk[b] = r;
    }
    if (tid == 0) {
        job.nblocks[0] = nb;
        if (job.flush_out) job.flush_out[4] = (uint64_t)(kMinMatch - 1) | (uint64_t)(kMinMatch - 1) << 16;
    }
}

// ------------------------------------------------------------------------
// Block records of a parse whose every symbol is flush-tested (deflate_huff,
// deflate_rle): block b ends after symbol 16383(b+1)-1; its flush happens at
// the decision point of that symbol (its start), so the slides before it are
// #{k : T_k <= start} with the parser's refill threshold; the last block is
// flushed at n.  cut_end/cut_pd: per cut, the end and decision point.
// ------------------------------------------------------------------------
__device__ void cut_blocks(BlockRec *blk, uint32_t n, uint32_t total, const uint32_t *cut_end,
                           const uint32_t *cut_pd, int64_t refill, int tid, int nthreads, const WinP &wp) {
    const uint32_t symlim = wp.sym_limit;
    const uint32_t ncut = total / symlim;
    uint32_t nthr = 0;
    while (slide_threshold(nthr + 1, n, refill, wp) <= (int64_t)n) nthr++;
    for (uint32_t b = tid; b <= ncut; b += nthreads) {
        const bool last = b == ncut;
        const uint64_t in_end = last ? n : cut_end[b];
        const uint64_t pd = last ? n : cut_pd[b];
        const uint64_t in_start = b == 0 ? 0 : cut_end[b - 1];
        uint32_t slides = 0;
        while (slides < nthr && slide_threshold(slides + 1, n, refill, wp) <= (int64_t)pd) slides++;
        BlockRec r;
        r.sym_start = b * symlim;
        r.nsym = last ? total - b * symlim : symlim;
        r.in_start = in_start;
        r.in_end = in_end;
        r.flags = (last ? 1u : 0u) | (in_start >= (uint64_t)wp.wsize * slides ? 2u : 0u);
        r.pad = 0;
        blk[b] = r;
    }
}

// k_parse_huff — Z_HUFFMAN_ONLY (deflate_huff, deflate.c:2122-2152): every byte
// is a literal; the window refills when the lookahead is 0.
constexpr int kHuffThreads = 256;
__global__ __launch_bounds__(kHuffThreads) void k_parse_huff(DeflateJob job) {
    const int tid = threadIdx.x;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const uint32_t n = (uint32_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    uint32_t *sym = job.sym + job.ws_off[bi];
    BlockRec *blk = job.blocks + job.blk_off[bi];
    const WinP wp = job_win(job);
    const uint32_t symlim = wp.sym_limit;
    for (uint32_t i = tid; i < n; i += kHuffThreads) sym[i] = in[i];
    // cut ends / decision points live in the rfull workspace (unused here)
    uint32_t *cut_end = job.rfull + job.ws_off[bi];
    uint32_t *cut_pd = cut_end + (n / symlim + 1);
    const uint32_t ncut = n / symlim;
    for (uint32_t b = tid; b < ncut; b += kHuffThreads) {
        cut_end[b] = (b + 1) * symlim;
        cut_pd[b] = (b + 1) * symlim - 1;
    }
    __threadfence_block();
    __syncthreads();
    cut_blocks(blk, n, n, cut_end, cut_pd, 0, tid, kHuffThreads, wp);
    if (tid == 0) job.nblocks[bi] = ncut + 1;
}

// k_parse_rle — Z_RLE (deflate_rle, deflate.c:2051-2116): a run of the previous
// byte of length >= 3 (capped at 258 and at the lookahead) becomes a match at
// distance 1; the window refills when the lookahead is <= 258.  One lane per
// buffer walks the input; symbols and cut points go to the workspace.
__global__ __launch_bounds__(64) void k_parse_rle(DeflateJob job) {
    const int lane = threadIdx.x;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const uint32_t n = (uint32_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    uint32_t *sym = job.sym + job.ws_off[bi];
    BlockRec *blk = job.blocks + job.blk_off[bi];
    const WinP wp = job_win(job);
    const uint32_t symlim = wp.sym_limit;
    uint32_t *cut_end = job.rfull + job.ws_off[bi];
    uint32_t *cut_pd = cut_end + (n / symlim + 1);
    __shared__ uint32_t s_total;
    if (lane == 0) {
        BCache cb;
        cb.base = ~(uintptr_t)0;
        uint32_t p = 0, cnt = 0;
        while (p < n) {
            uint32_t len = 0;
            if (n - p >= (uint32_t)kMinMatch && p > 0) {
                const uint32_t prev = bget(in, p - 1, cb);
                if (bget(in, p, cb) == prev && bget(in, p + 1, cb) == prev && bget(in, p + 2, cb) == prev) {
                    len = 3;
                    const uint32_t cap = n - p < (uint32_t)kMaxMatch ? n - p : (uint32_t)kMaxMatch;
                    while (len < cap && bget(in, p + len, cb) == prev) len++;
                }
            }
            uint32_t v, sl;
            if (len >= (uint32_t)kMinMatch) { v = (1u << 8) | (len - kMinMatch); sl = len; }
            else { v = bget(in, p, cb); sl = 1; }
            sym[cnt] = v;
            if ((cnt + 1) % symlim == 0) {
                cut_end[cnt / symlim] = p + sl;
                cut_pd[cnt / symlim] = p;
            }
            cnt++;
            p += sl;
        }
        s_total = cnt;
    }
    __threadfence_block();
    __syncthreads();
    const uint32_t total = s_total;
    cut_blocks(blk, n, total, cut_end, cut_pd, kMaxMatch, lane, 64, wp);
    if (lane == 0) job.nblocks[bi] = total / symlim + 1;
}

// ------------------------------------------------------------------------
// k_parse_ev — Z_HUFFMAN_ONLY / Z_RLE parse of a flush job (deflate_huff,
// deflate.c:2122-2152; deflate_rle, :2051-2116), one lane, sequential: the
// window schedule decides where its blocks end once flush calls cut the input
// (fill_window at lookahead 0 resp. <= MAX_MATCH), and flush jobs are the
// streaming API's, one buffer at a time.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_parse_ev(DeflateJob job) {
    if (threadIdx.x != 0) return;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const int64_t n = (int64_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    const bool rle = job.strategy == 3;
    ParseOut po;
    po.sym = job.sym + job.ws_off[bi];
    po.blk = job.blocks + job.blk_off[bi];
    po.nsym = po.blk_nsym = po.blk_sym_start = po.nblk = 0;
    po.win(job_win(job));
    po.lead = true;
    int64_t p = job.start;                      // a resumed job: see k_parse_slow
    po.block_start = p; po.S = 0; po.E = (int64_t)job.e0 > p ? (int64_t)job.e0 : p;
    po.srec = job.srec;
    FlushEv fe = flush_ev(job);
    while (fe.prime()) {                       // deflatePrime at the resume point (a pause behind it): bits first
        if (job.ev_blk) job.ev_blk[fe.i] = po.nblk;
        po.marker(p, kMarkPrime, fe.prime_arg());
        fe.i++;
    }
    int64_t lim = fe.limit(n);
    bool done = false;
    for (;;) {
        if (p > po.E) break;                                      // guard: never parse past the input read
        if (rle ? po.E - p <= kMaxMatch : po.E == p) {
            po.fill(p, lim);
            // a Z_NO_FLUSH call's input is used up: need_more (deflate.c:2065-2068, :2129-2134)
            while (fe.stop_at(po.E, lim) && (rle ? po.E - p <= kMaxMatch : po.E == p)) {
                if (job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                fe.i++;
                while (fe.prime()) {                              // deflatePrime: its bits go out here
                    if (job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                    po.marker(p, kMarkPrime, fe.prime_arg());
                    fe.i++;
                }
                if (fe.i == fe.n && job.open_end) { done = true; break; }
                lim = fe.limit(n);
                po.fill(p, lim);
            }
            if (done) break;
            if (po.E == p) {
                if (fe.at(p)) {
                    if (po.blk_nsym) po.flush(p, false);
                    if (job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                    po.marker(p, fe.kind());
                    if (job.flush_out) job.flush_out[2] = (uint64_t)po.S;
                    fe.i++;
                    lim = fe.limit(n);
                    continue;
                }
                break;
            }
        }
        const int64_t lookahead = po.E - p;
        uint32_t len = 0;
        if (rle && lookahead >= kMinMatch && p > po.S) {      // strstart > 0
            const uint8_t c = in[p - 1];
            if (in[p] == c && in[p + 1] == c && in[p + 2] == c) {
                len = kMinMatch;
                while (len < (uint32_t)kMaxMatch && p + len < n && in[p + len] == c) len++;
                if (len > lookahead) len = (uint32_t)lookahead;
            }
        }
        bool bflush;
        if (len >= (uint32_t)kMinMatch) {
            bflush = po.tally((1u << 8) | (len - kMinMatch));
            p += len;
        } else {
            bflush = po.tally(in[p]);
            p++;
        }
        if (bflush) {
            po.flush(p, false);
            if (fe.pause_at(p)) {
                if (job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                fe.i++;
                while (fe.prime()) {                                  // deflatePrime while the call stood here
                    if (job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                    po.marker(p, kMarkPrime, fe.prime_arg());
                    fe.i++;
                }
                lim = fe.limit(n);
            }
        }
    }
    if (!job.open_end) po.flush(p, true);
    job.nblocks[bi] = po.nblk;
}

// ------------------------------------------------------------------------
// k_parse_fast — levels 1..3 (deflate_fast).  Insertion inside a match depends
// on its length (deflate.c:1873-1897), so hash chains are maintained exactly
// as zlib does it, sequentially: head[] (absolute positions, per buffer, in
// global memory) and prev[] as 16-bit distances.  One wave per buffer runs the
// parse wave-uniformly (every lane holds the same state; lane 0 stores), so the
// chain walk (longest_match with prev_length == MIN_MATCH-1) compares a
// candidate 64 bytes per memory round trip, one byte per lane, with the next
// link loaded in the same round trip.
// ------------------------------------------------------------------------
// kEv: a flush job (events, a resumed start, late hashing); batch jobs run
// the <false> instance, whose loop carries none of that.
// kOne (the only instance built; kOne false is the round-2 walk): one
// memory round trip per chain candidate.  The link and the candidate's 64
// bytes are loaded together (the round-2 walk made the link uniform before it
// requested the bytes: two round trips), the bytes through a clamped index
// instead of a bounds branch, and the scan side of the compare is taken from
// the register window once per position instead of once per candidate.
// P: the position type.  A batch whose buffers are all under 2^31 bytes
// (DeflateJob::pos31) runs on int32_t: the parse is one wave-uniform program
// whose state lives in SGPRs, and 64-bit positions doubled its scalar
// arithmetic (add/addc pairs, 64-bit compares) -- at 28 waves per CU sharing
// one scalar unit, scalar issue is what bounds it.
//
// kLds (batch jobs of few buffers, hash_bits <= 15): one wave per CU, with
// head[], prev[] and the window's bytes in the CU's 160 KiB of LDS instead of
// HBM, so a chain step waits for LDS rather than an L2 / HBM round trip.
//   s_head: hash_size 16-bit entries, a position's low 16 bits; the age
//           p - entry (mod 64 Ki) is exact for entries under 64 Ki positions
//           old, and a sweep every 16 Ki positions turns every entry older than
//           32 Ki into one that reads as older (an age >= 32768 is no candidate:
//           MAX_DIST < 32768)
//   s_prev: prev[] as a 32 Ki ring (a chain only steps between positions within
//           MAX_DIST of p)
//   s_ring: in[q] at q mod 32 Ki for q in [p - MAX_DIST, p + 262): the
//           candidates (> p - MAX_DIST, their byte before, up to 258 after) and
//           the scan side (p .. p + 257) of every compare.  Filled byte-exact
//           to p + 262 from a prefetched 128-byte register window.
constexpr uint32_t kFastRing = 32768;
template <bool kEv, bool kOne, typename P, bool kLds = false>
__global__ __launch_bounds__(64) void k_parse_fast(DeflateJob job, uint32_t *heads) {
    static_assert(!kLds || (!kEv && kOne), "the LDS variant serves batch jobs");
    __shared__ uint16_t s_head[kLds ? 32768 : 1];
    __shared__ uint16_t s_prev[kLds ? kFastRing : 1];
    __shared__ uint8_t s_ring[kLds ? kFastRing : 1];
    constexpr uint32_t kRM = kFastRing - 1;
    const int lane = threadIdx.x;
    const bool lead = lane == 0;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const P n = (P)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    uint16_t *prev = job.link + job.ws_off[bi];
    const WinP wp = job_win(job);
    const uint32_t hsize = wp.mask + 1;                  // hash_size = 1 << hash_bits
    uint32_t *head = heads + (size_t)bi * hsize;
    LevelCfg cfg = job.cfg;
    uint32_t ci = 0;                                     // configuration changes acted on
    // a resumed flush job (start > 0) finds head[] and prev[] as the last job
    // left them, rebased to its buffer (zgpu_api.cpp deflate_part)
    if (kLds) {
        for (int i = lane; i < (int)hsize; i += 64) s_head[i] = 0x8000;   // "32 Ki before position 0"
    } else if (!kEv || job.start == 0 || (job.dict && !job.keep_head)) {
        for (int i = lane; i < (int)hsize; i += 64) head[i] = 0;
    }
    __threadfence_block();
    __syncthreads();

    ParseOutT<P> po;
    const P max_dist = (P)wp.max_dist;
    po.sym = job.sym + job.ws_off[bi];
    po.blk = job.blocks + job.blk_off[bi];
    po.nsym = po.blk_nsym = po.blk_sym_start = po.nblk = 0;
    po.win(job_win(job));
    const P start = kEv ? (P)job.start : 0;
    po.block_start = start; po.S = 0; po.E = kEv && (P)job.e0 > start ? (P)job.e0 : start;
    po.lead = kOne || lead;                              // kOne: all lanes store the symbols
    po.vaddr = kOne;
    if (kEv) po.srec = job.srec;

    // input window in registers: lane j holds in[wb + j] (w0) and in[wb + 64 + j]
    // (w1); it is moved forward 64 bytes at a time, so hashing and the scan side
    // of a compare need no memory round trip
    P wb = -128;
    uint32_t w0 = 0, w1 = 0;
    // in[x], 0 past the end: a clamped load and a select (kOne), no exec-mask branch
    auto ld = [&](P x) -> uint32_t {
        if (!kOne) return x < n ? (uint32_t)in[x] : 0u;
        const uint32_t v = in[(uint32_t)(x < n ? x : n - 1)];
        return x < n ? v : 0u;
    };
    // kOne: lane j also holds hv = the hash of position wb + j (its bytes are
    // all in the window), made when the window moves, so INSERT_STRING's hash
    // is one readlane instead of three byte reads and the hash arithmetic on
    // the scalar unit
    uint32_t hv = 0;
    auto wsee = [&](P x) {                        // make [x, x + 66) resident
        if (x >= wb && x + 66 <= wb + 128) return;
        const P nb = x & ~(P)63;
        if (nb == wb + 64) { w0 = w1; w1 = ld(nb + 64 + lane); }
        else { w0 = ld(nb + lane); w1 = ld(nb + 64 + lane); }
        wb = nb;
        if (kOne) {
            const int l1 = (lane + 1) & 63, l2 = (lane + 2) & 63;
            const uint32_t a1 = (uint32_t)__shfl((int)w0, l1, 64), c1 = (uint32_t)__shfl((int)w1, l1, 64);
            const uint32_t a2 = (uint32_t)__shfl((int)w0, l2, 64), c2 = (uint32_t)__shfl((int)w1, l2, 64);
            hv = hashp(w0, lane < 63 ? a1 : c1, lane < 62 ? a2 : c2, wp);
        }
    };
    auto wbyte = [&](P x) -> uint32_t {           // uniform x in the window
        const int o = (int)(x - wb);
        return (uint32_t)__builtin_amdgcn_readlane((int)(o < 64 ? w0 : w1), o & 63);
    };
    auto whash = [&](P q) -> uint32_t {
        if (kOne) {
            const int o = (int)(q - wb);
            if (o < 64) return (uint32_t)__builtin_amdgcn_readlane((int)hv, o);
        }
        return hashp(wbyte(q), wbyte(q + 1), wbyte(q + 2), wp);
    };
    auto insert = [&](P q) -> P {           // INSERT_STRING
        const uint32_t h = whash(q);
        if (kLds) {
            const uint32_t age = ufl(((uint32_t)q - (uint32_t)s_head[h]) & 0xffffu);   // one address: uniform
            const P hh = (age != 0 && age < 32768u) ? q - (P)age : 0;
            s_prev[(uint32_t)q & kRM] = hh != 0 ? (uint16_t)age : (uint16_t)0;
            s_head[h] = (uint16_t)q;
            return hh;
        }
        const P hh = ufl(head[kOne ? vg(h) : h]);
        const P d = q - hh;
        // kOne: every lane stores the same (uniform) value, which keeps the
        // scalar exec-mask save/restore of a lane-0 store off the parse's path
        if (kOne || lead) {
            if (kOne) {                                  // addresses in VGPRs (vg)
                prev[vg((uint32_t)q)] = (hh != 0 && d <= 32767) ? (uint16_t)d : 0;
                head[vg(h)] = (uint32_t)q;
            } else {
                prev[q] = (hh != 0 && d <= 32767) ? (uint16_t)d : 0;
                head[h] = (uint32_t)q;
            }
        }
        return hh;
    };
    // common prefix of in[a..] and in[p..], capped at maxcmp (a < p); the scan
    // side of the first 64 bytes comes from the register window
    auto common = [&](P a, P pp, int maxcmp) -> int {
        const int o = (int)(pp - wb) + lane;            // < 128 + 63
        const uint32_t x0 = (uint32_t)__shfl((int)w0, o & 63, 64), x1 = (uint32_t)__shfl((int)w1, o & 63, 64);
        const uint32_t sb = o < 64 ? x0 : x1;           // wsee(pp): pp - wb <= 62
        {
            const bool diff = lane < maxcmp && ld(a + lane) != sb;
            const uint64_t m = __ballot(diff);
            if (m) return __builtin_ctzll(m);
        }
        for (int k0 = 64; k0 < maxcmp; k0 += 64) {
            const int k = k0 + lane;
            const bool diff = k < maxcmp && ld(a + k) != ld(pp + k);
            const uint64_t m = __ballot(diff);
            if (m) return k0 + __builtin_ctzll(m);
        }
        return maxcmp;
    };
    auto common_from = [&](P a, P pp, int maxcmp, int k0) -> int {   // bytes k0.. from memory
        for (; k0 < maxcmp; k0 += 64) {
            const int kk = k0 + lane;
            const int kc = kk < maxcmp ? kk : maxcmp - 1;
            const uint32_t x = kLds ? (uint32_t)s_ring[(uint32_t)(a + kc) & kRM] : (uint32_t)in[(uint32_t)(a + kc)];
            const uint32_t y = kLds ? (uint32_t)s_ring[(uint32_t)(pp + kc) & kRM] : (uint32_t)in[(uint32_t)(pp + kc)];
            const uint64_t m = __ballot((kk < maxcmp) & (x != y));
            if (m) return k0 + __builtin_ctzll(m);
        }
        return maxcmp;
    };

    if (kEv && job.dict)                                  // a preset dictionary's strings, or a window
        for (P q = (P)job.pre_from; q < (P)job.pre_ins; q++) {   // parsed by a function that inserts all
            bool skip = false;                           // but a deflate_huff / deflate_rle stretch (SkipSpec)
            for (uint32_t k = 0; k < job.sk.n; k++)
                if ((uint32_t)q >= job.sk.a[k] && (uint32_t)q < job.sk.b[k]) skip = true;
            if (skip) continue;
            wsee(q);
            insert(q);
        }
    // kLds: the byte ring's fill point rf, and the 64-aligned register window
    // [fb, fb + 128) it is filled from (f1 is loaded 64 bytes before it is needed)
    P rf = 0, fb = 0, sweep_at = 16384;
    uint32_t f0 = 0, f1 = 0;
    if (kLds && n > 0) { f0 = ld(lane); f1 = ld(64 + lane); }
    auto ring_fill = [&](P target) {
        while (rf < target) {
            if (rf >= fb + 64) { f0 = f1; fb += 64; f1 = ld(fb + 64 + lane); }
            const P e = target < fb + 64 ? target : fb + 64;
            const P q = fb + lane;
            if (q >= rf && q < e) s_ring[(uint32_t)q & kRM] = (uint8_t)f0;
            rf = e;
        }
    };
    auto rbyte = [&](P x) -> uint32_t { return kLds ? (uint32_t)s_ring[(uint32_t)x & kRM] : (uint32_t)in[(uint32_t)x]; };
    P p = start, match_start = 0;
    // deflate_state's prev_length, which deflate_fast never writes: every search
    // starts from it (2, or what deflate_slow left behind a function switch,
    // DeflateJob::zp0); match_length as the job finds it (zm0)
    const int best0 = kEv ? job.zp0 : kMinMatch - 1;
    uint32_t match_length = kEv ? (uint32_t)job.zm0 : kMinMatch - 1;
    FlushEv fe = flush_ev(job);
    while (kEv && fe.prime()) {         // deflatePrime at the resume point (a pause behind it): bits first
        if (lead && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
        po.marker(p, kMarkPrime, fe.prime_arg());
        fe.i++;
    }
    P lim = kEv ? (P)fe.limit(n) : n;   // input deflate() has been given
    // s->insert: strings a flush left unhashed (a resumed job starts right
    // after a flush at its window offset + start; none at a block cut)
    P pend = (kEv && job.cut) ? 0 : p < kMinMatch - 1 ? p : kMinMatch - 1;
    // right after a deflate_huff / deflate_rle stretch (a SkipSpec range ending
    // at the start): their flush leaves s->insert = 0 (deflate.c:2108, 2144)
    if (kEv)
        for (uint32_t k = 0; k < job.sk.n; k++)
            if ((P)job.sk.b[k] == p) pend = 0;
    // a streaming job keeps head[] as it stands at its last cut (the block or
    // marker record snap[hsize]): a later job resumes there
    auto snapshot = [&]() {
        if (!kEv || !job.snap) return;
        __threadfence_block();
        for (uint32_t i = (uint32_t)lane; i < hsize; i += 64) job.snap[i] = head[i];
        if (lead) job.snap[hsize] = po.nblk - 1;
    };
    auto fill = [&]() {
        const bool reads = kEv && po.E < lim;
        po.fill(p, lim);
        // fill_window hashes the strings the last flush left unhashed once
        // new input is read (deflate.c:318-335)
        if (reads && pend && po.E - p + pend >= kMinMatch) {
            P str = p - pend;
            while (pend) {
                wsee(str);
                insert(str);
                str++;
                pend--;
                if (po.E - p + pend < kMinMatch) break;
            }
        }
    };
    for (;;) {
        if (p > po.E) break;                                      // guard: never parse past the input read
        if (po.E - p < kMinLookahead) {
            fill();
            // a Z_NO_FLUSH call's input is used up: need_more (deflate.c:1841-1844)
            bool done = false;
            while (kEv && fe.stop_at(po.E, lim) && po.E - p < kMinLookahead) {
                if (lead && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                fe.i++;
                while (fe.prime()) {                              // deflatePrime: its bits go out here
                    if (lead && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                    po.marker(p, kMarkPrime, fe.prime_arg());
                    fe.i++;
                }
                if (fe.i == fe.n && job.open_end) { done = true; break; }
                lim = (P)fe.limit(n);
                fill();
            }
            if (done) break;
            if (po.E == p) {
                if (kEv && fe.at(p)) {
                    // a deflate(flush) call ends here (deflate.c:1903-1914, :1211-1233)
                    pend = p - po.S < kMinMatch - 1 ? p - po.S : kMinMatch - 1;
                    if (po.blk_nsym) po.flush(p, false);
                    if (lead && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                    po.marker(p, fe.kind());
                    snapshot();
                    if (lead && job.flush_out) job.flush_out[2] = (uint64_t)po.S;
                    fe.i++;
                    lim = (P)fe.limit(n);
                    continue;
                }
                break;
            }
        }
        wsee(p);
        if (kLds) {
            if (p >= sweep_at) {                          // s_head: entries 32 Ki old read as older
                for (uint32_t i = (uint32_t)lane; i < hsize; i += 64) {
                    const uint32_t age = ((uint32_t)p - (uint32_t)s_head[i]) & 0xffffu;
                    if (age == 0 || age >= 32768u) s_head[i] = (uint16_t)((uint32_t)p - 32768u);
                }
                sweep_at = p + 16384;
            }
            ring_fill(n - p > 262 ? p + 262 : n);         // slot of p - 32506 is the next to go
        }
        if (kEv)                                         // deflateParams / deflateTune
            while (ci < job.ncfg && p >= (P)job.cfg_pos[ci]) cfg = job.cfg_tab[ci++];
        P lookahead = po.E - p;
        P hh = 0;
        if (lookahead >= kMinMatch) hh = insert(p);
        if (hh > po.S && p - hh <= max_dist) {
            // longest_match (deflate.c:1356-1497), prev_length == 2: the first
            // candidate with the longest prefix wins, stop at nice, chain, limit
            // prev_length stays MIN_MATCH-1 under deflate_fast: the budget is
            // quartered only for a deflateTune good_length <= 2 (deflate.c:1390)
            uint32_t chain = (uint32_t)best0 >= cfg.good ? cfg.chain >> 2 : cfg.chain;
            const int nice = lookahead < (P)cfg.nice ? (int)lookahead : (int)cfg.nice;
            const P limit = (p - po.S) > max_dist ? p - max_dist : po.S;
            const P rem = n - p;
            const int maxcmp = rem < kMaxMatch ? (int)rem : kMaxMatch;
            int best = best0;
            P cur = hh;
            uint32_t sb = 0;
            const int lc = lane < maxcmp ? lane : maxcmp - 1;
            if (kOne) {                                  // scan bytes p + lane, from the register window
                const int o = (int)(p - wb) + lane;
                const uint32_t x0 = (uint32_t)__shfl((int)w0, o & 63, 64), x1 = (uint32_t)__shfl((int)w1, o & 63, 64);
                sb = o < 64 ? x0 : x1;
            }
            for (;;) {
                uint32_t d;
                int k;
                if (kOne) {
                    // link and candidate bytes in one round trip; cur + lc < n
                    // since cur < p and maxcmp <= n - p.  Only the first kC0
                    // candidate bytes are loaded (most compares end there): a
                    // 16-byte span crosses a cache line far less often than 64
                    // (DeflateJob::fcmp: 64, the round-3 compare)
                    const int c0 = (kLds || job.fcmp) ? 64 : 16;
                    const uint32_t dv = kLds ? (uint32_t)s_prev[(uint32_t)cur & kRM] : (uint32_t)prev[vg((uint32_t)cur)];
                    uint32_t cbyte = 0;
                    if (lane < c0) cbyte = rbyte(cur + lc);
                    __builtin_amdgcn_sched_barrier(0);       // both loads issued before either is used
                    const int mc = maxcmp < c0 ? maxcmp : c0;
                    const uint64_t m = __ballot(lane < mc && cbyte != sb);
                    k = m ? (int)__builtin_ctzll(m) : (maxcmp <= c0 ? maxcmp : common_from(cur, p, maxcmp, c0));
                    d = ufl(dv);
                } else {
                    d = ufl(prev[cur]);
                    k = common(cur, p, maxcmp);
                }
                // from best_len 0 the quick reject also compares the bytes
                // before the strings (scan_end1 = scan[-1]) and the first two
                if (k > best && (best != 0 || (k >= 2 && rbyte(cur - 1) == rbyte(p - 1)))) {
                    match_start = cur;
                    best = k;
                    if (k >= nice) break;
                }
                if (d == 0) break;
                cur -= d;
                if (cur <= limit || --chain == 0) break;
            }
            match_length = (P)best <= lookahead ? (uint32_t)best : (uint32_t)lookahead;
        }
        bool bflush;
        if (match_length >= kMinMatch) {
            bflush = po.tally(((uint32_t)(p - match_start) << 8) | (match_length - kMinMatch));
            lookahead -= match_length;
            if (match_length <= cfg.lazy && lookahead >= kMinMatch && match_length <= 48) {
                // positions p+1 .. p+len-1 (at most 5 unless deflateTune), one
                // lane each: the head loads go out together; a position whose
                // hash a lower lane also inserts takes that lane's position (zlib
                // inserts in order)
                const uint32_t cntk = match_length - 1;
                const bool mine = (uint32_t)lane < cntk;
                const P q = p + 1 + lane;
                uint32_t h = 0xffffffffu;
                const int ob = (int)(p + 1 - wb);            // window offset of p + 1
                if (kOne && ob + (int)cntk <= 64) {
                    // lane k < cntk: the hash of p + 1 + k, from the window's hashes
                    const uint32_t hx = (uint32_t)__shfl((int)hv, (ob + lane) & 63, 64);
                    h = mine ? hx : 0xffffffffu;
                } else {
                    for (uint32_t k = 0; k < cntk; k++) {
                        const uint32_t hk = whash(p + 1 + k);
                        if ((uint32_t)lane == k) h = hk;
                    }
                }
                P hh0 = 0;
                if (kLds) {
                    const uint32_t age = mine ? ((uint32_t)q - (uint32_t)s_head[h]) & 0xffffu : 0u;
                    hh0 = (age != 0 && age < 32768u) ? q - (P)age : 0;
                } else {
                    hh0 = mine ? (P)head[h] : 0;
                }
                P hq = hh0;
                bool last = mine;
                for (uint32_t k = 0; k < cntk; k++) {
                    const uint32_t hk = kOne ? (uint32_t)__builtin_amdgcn_readlane((int)h, (int)k)
                                             : (uint32_t)__shfl((int)h, (int)k, 64);
                    if (mine && hk == h) {
                        if (k < (uint32_t)lane) hq = p + 1 + k;        // a lower lane's position
                        if (k > (uint32_t)lane) last = false;          // a higher lane writes head
                    }
                }
                if (mine) {
                    const P dd = q - hq;
                    const uint16_t lk = (hq != 0 && dd <= 32767) ? (uint16_t)dd : 0;
                    if (kLds) {
                        s_prev[(uint32_t)q & kRM] = lk;
                        if (last) s_head[h] = (uint16_t)q;
                    } else {
                        prev[q] = lk;
                        if (last) head[h] = (uint32_t)q;
                    }
                }
            } else if (match_length <= cfg.lazy && lookahead >= kMinMatch) {
                // deflateTune's longer max_insert_length: one insert at a time
                for (uint32_t k = 1; k < match_length; k++) {
                    wsee(p + k);
                    insert(p + k);
                }
            }
            p += match_length;
            match_length = 0;
        } else {
            bflush = po.tally(wbyte(p));
            p++;
        }
        if (bflush) {
            po.flush(p, false);
            snapshot();
            if (kEv && fe.pause_at(p)) {
                if (lead && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                fe.i++;
                while (fe.prime()) {                                  // deflatePrime while the call stood here
                    if (lead && job.ev_blk) job.ev_blk[fe.i] = po.nblk;
                    po.marker(p, kMarkPrime, fe.prime_arg());
                    fe.i++;
                }
                lim = (P)fe.limit(n);
            }
        }
    }
    if (!kEv || !job.open_end) po.flush(p, true);
    if (lead) job.nblocks[bi] = po.nblk;
    if (kEv && lead && job.flush_out) job.flush_out[4] = (uint64_t)best0 | (uint64_t)match_length << 16;
}

// ------------------------------------------------------------------------
// k_encode — one 256-thread workgroup per buffer.
// ------------------------------------------------------------------------
constexpr int kEncThreads = 256;
constexpr int kStgWords = 2048;                 // 8 KiB output staging window
constexpr int kEncGroup = kEncThreads / 64;     // blocks whose trees are built at once (one per wave)
constexpr int kStgBits = kStgWords * 32;
// k_enc_emit's staging window (4 KiB): small enough that a k_enc_emit
// workgroup (5.0 KiB of LDS) fits beside k_match's 153.6 KiB on a CU, so the
// pipeline runs both at once: 10426 -> 10606 MB/s on the C4 shard
// (profiles/r03q_ab_coresident_encode.log)
constexpr int kEmitStgWords = 1024;
constexpr int kEmitStgBits = kEmitStgWords * 32;
constexpr int kWNodeSlots = (kHeapSize + 63) / 64;   // w_build: tree nodes per lane (9)
constexpr unsigned kEncWaveBuildMax = 1024;          // w_build below this many buffers per launch

struct TreeLDSLane {                     // what the one-lane build (t_build) uses
    // leaves: freq/code; all nodes: dad/len (internal-node freqs live in heap keys)
    uint16_t lfreq[kLCodes], lcode[kLCodes], ldad[kHeapSize];
    uint8_t llen[kHeapSize + 1];
    uint16_t dfreq[kDCodes], dcode[kDCodes], ddad[2 * kDCodes + 1];
    uint8_t dlen[2 * kDCodes + 2];
    uint16_t bfreq[kBLCodes], bcode[kBLCodes], bdad[2 * kBLCodes + 1];
    uint8_t blen[2 * kBLCodes + 2];
    uint32_t heap[kHeapSize + 1];        // packed keys, see hkey()
    uint16_t bl_count[kMaxBits + 1];
};
struct TreeLDS : TreeLDSLane {
    uint32_t pj[kWNodeSlots * 64];       // w_build: pointer-jumping exchange (dad | depth << 16)
};

struct TreeRef {
    uint16_t *freq, *dad, *code;
    uint8_t *len;
    int max_code;
};

// Heap entries carry their own sort key: freq (16 bits) | depth (6) | node (10).
// zlib's smaller(n, m) (trees.c:499-501: freq, then depth, ties "<=") is then
// hkey(n) >> 10 <= hkey(m) >> 10, and a heap level costs one LDS round trip.
__device__ inline uint32_t hkey(uint32_t freq, uint32_t depth, uint32_t node) {
    return (freq << 16) | (depth << 10) | node;
}
// (a >> 10) <= (b >> 10)  <=>  a < ((b >> 10) + 1) << 10  <=>  a <= (b | 1023): one OR, no shifts
__device__ inline bool hle(uint32_t a, uint32_t b) { return a <= (b | 1023u); }

__device__ void t_downheap(uint32_t *heap, int heap_len, int k) {        // pqdownheap
    const uint32_t v = heap[k];
    int j = k << 1;
    while (j <= heap_len) {
        uint32_t hj = heap[j];
        if (j < heap_len) {
            const uint32_t hj1 = heap[j + 1];
            if (hle(hj1, hj)) { j++; hj = hj1; }
        }
        if (hle(v, hj)) break;
        heap[k] = hj;
        k = j;
        j <<= 1;
    }
    heap[k] = v;
}

__device__ void t_gen_codes(TreeRef &t, const uint16_t *bl_count) {       // gen_codes
    uint32_t next[kMaxBits + 1];
    uint32_t c = 0;
#pragma unroll
    for (int b = 1; b <= kMaxBits; b++) { c = (c + bl_count[b - 1]) << 1; next[b] = c; }
    for (int n = 0; n <= t.max_code; n++) {
        const int len = t.len[n];
        if (!len) continue;
        uint32_t code = 0;
#pragma unroll
        for (int b = 1; b <= kMaxBits; b++)            // register-resident next[] (no scratch)
            if (b == len) code = next[b]++;
        t.code[n] = (uint16_t)(__brev(code) >> (32 - len));
    }
}

// build_tree + gen_bitlen (trees.c:540-706); slen == nullptr for the bl tree.
// Single lane; opt_len/static_len accumulate in registers.
__device__ void t_build(TreeRef &t, TreeLDSLane &h, int elems, const uint8_t *slen, const uint8_t *extra,
                        int xbase, int max_length, int64_t &opt_len, int64_t &static_len) {
    uint32_t *heap = h.heap;
    int max_code = -1, heap_len = 0, heap_max = kHeapSize;
    for (int n = 0; n < elems; n++) {
        const uint32_t f = t.freq[n];
        if (f != 0) { heap[++heap_len] = hkey(f, 0, (uint32_t)n); max_code = n; }
        else t.len[n] = 0;
    }
    while (heap_len < 2) {
        const int node = max_code < 2 ? ++max_code : 0;
        heap[++heap_len] = hkey(1, 0, (uint32_t)node);
        t.freq[node] = 1;
        opt_len--;
        if (slen) static_len -= slen[node];
    }
    t.max_code = max_code;
    for (int n = heap_len / 2; n >= 1; n--) t_downheap(heap, heap_len, n);
    uint32_t node = (uint32_t)elems;
    do {
        const uint32_t kn = heap[1];
        heap[1] = heap[heap_len--];
        t_downheap(heap, heap_len, 1);
        const uint32_t km = heap[1];
        heap[--heap_max] = kn;
        heap[--heap_max] = km;
        const uint32_t f = (kn >> 16) + (km >> 16);
        const uint32_t dn = (kn >> 10) & 63u, dm = (km >> 10) & 63u;
        t.dad[kn & 1023u] = t.dad[km & 1023u] = (uint16_t)node;
        heap[1] = hkey(f, (dn >= dm ? dn : dm) + 1, node);
        node++;
        t_downheap(heap, heap_len, 1);
    } while (heap_len >= 2);
    heap[--heap_max] = heap[1];

    // gen_bitlen
    int overflow = 0;
    for (int b = 0; b <= kMaxBits; b++) h.bl_count[b] = 0;
    t.len[heap[heap_max] & 1023u] = 0;
    for (int hh = heap_max + 1; hh < kHeapSize; hh++) {
        const uint32_t key = heap[hh];
        const int n = (int)(key & 1023u);
        int bits = t.len[t.dad[n]] + 1;
        if (bits > max_length) { bits = max_length; overflow++; }
        t.len[n] = (uint8_t)bits;
        if (n > max_code) continue;
        h.bl_count[bits]++;
        const int xb = n >= xbase ? extra[n - xbase] : 0;
        const int64_t f = (int64_t)(key >> 16);
        opt_len += f * (bits + xb);
        if (slen) static_len += f * (slen[n] + xb);
    }
    if (overflow != 0) {
        do {
            int bits = max_length - 1;
            while (h.bl_count[bits] == 0) bits--;
            h.bl_count[bits]--;
            h.bl_count[bits + 1] += 2;
            h.bl_count[max_length]--;
            overflow -= 2;
        } while (overflow > 0);
        int hh = kHeapSize;
        for (int bits = max_length; bits != 0; bits--) {
            int n = h.bl_count[bits];
            while (n != 0) {
                const int m = (int)(heap[--hh] & 1023u);
                if (m > max_code) continue;
                if (t.len[m] != bits) {
                    opt_len += ((int64_t)bits - t.len[m]) * t.freq[m];
                    t.len[m] = (uint8_t)bits;
                }
                n--;
            }
        }
    }
    t_gen_codes(t, h.bl_count);
}

// ---- w_build: build_tree + gen_bitlen + gen_codes (trees.c:540-706, 589-625) by a whole wave ----
// The heap lives in five VGPRs across the wave's lanes: heap[j] is lane j & 63 of register j >> 6
// (heap_len <= 286 < 320). A heap access is a readlane/writelane with a wave-uniform index instead of
// a dependent LDS round trip of one lane, and the sequence of heap operations -- hence every tie
// pqdownheap breaks -- is trees.c's. The node depths of gen_bitlen come from pointer jumping over the
// dad links, bl_count and the codes of gen_codes from per-length ballots.
struct RHeap { uint32_t r[5]; };

__device__ __attribute__((always_inline)) inline uint32_t rl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __attribute__((always_inline)) inline uint32_t wl(uint32_t v, uint32_t l, uint32_t old) {
    return (threadIdx.x & 63u) == l ? v : old;      // v_cmp + v_cndmask (no writelane builtin here)
}
template <int D>   // j on heap level D (2^D <= j < 2^(D+1))
__device__ __attribute__((always_inline)) inline uint32_t rget(const RHeap &H, uint32_t j) {
    if constexpr (D <= 5) return rl(H.r[0], j);
    else if constexpr (D == 6) return rl(H.r[1], j & 63u);
    else if constexpr (D == 7) return (j & 64u) ? rl(H.r[3], j & 63u) : rl(H.r[2], j & 63u);
    else return rl(H.r[4], j & 63u);
}
template <int D>
__device__ __attribute__((always_inline)) inline void rset(RHeap &H, uint32_t j, uint32_t v) {
    if constexpr (D <= 5) H.r[0] = wl(v, j, H.r[0]);
    else if constexpr (D == 6) H.r[1] = wl(v, j & 63u, H.r[1]);
    else if constexpr (D == 7) {
        if (j & 64u) H.r[3] = wl(v, j & 63u, H.r[3]);
        else H.r[2] = wl(v, j & 63u, H.r[2]);
    } else H.r[4] = wl(v, j & 63u, H.r[4]);
}
__device__ __attribute__((always_inline)) inline uint32_t rget_any(const RHeap &H, uint32_t j) {
    switch (j >> 6) {
    case 0: return rl(H.r[0], j);
    case 1: return rl(H.r[1], j & 63u);
    case 2: return rl(H.r[2], j & 63u);
    case 3: return rl(H.r[3], j & 63u);
    default: return rl(H.r[4], j & 63u);
    }
}
// Slots past heap_len hold kHInf, a key above every real one (freqs < 2^16
// with depth and node below), so a sift needs no bounds tests: an absent
// child is never the smaller one (zlib takes j + 1 only when it exists and is
// <= heap[j]) and v <= kHInf ends the sift where zlib finds no child.
constexpr uint32_t kHInf = 0xffffffffu;
// children j, j + 1 (j even, same register) on heap level L
template <int L>
__device__ __attribute__((always_inline)) inline void rget2(const RHeap &H, uint32_t j, uint32_t &a, uint32_t &b) {
    const uint32_t l = j & 63u;
    if constexpr (L <= 5) { a = rl(H.r[0], l); b = rl(H.r[0], l + 1); }
    else if constexpr (L == 6) { a = rl(H.r[1], l); b = rl(H.r[1], l + 1); }
    else if constexpr (L == 7) {                     // per-register reads (a select of registers would index H)
        const uint32_t a2 = rl(H.r[2], l), b2 = rl(H.r[2], l + 1), a3 = rl(H.r[3], l), b3 = rl(H.r[3], l + 1);
        a = (j & 64u) ? a3 : a2;
        b = (j & 64u) ? b3 : b2;
    } else {                                         // slots 320.. are past any heap_len (<= 286)
        a = j < 320u ? rl(H.r[4], l) : kHInf;
        b = j < 320u ? rl(H.r[4], l + 1) : kHInf;
    }
}
__device__ __attribute__((always_inline)) inline void rset_any(RHeap &H, uint32_t j, uint32_t v) {
    const bool me = (threadIdx.x & 63u) == (j & 63u);
#pragma unroll
    for (int r = 0; r < 5; r++) H.r[r] = (me && (j >> 6) == (uint32_t)r) ? v : H.r[r];
}
// pqdownheap (trees.c:509-527) of key v entering at node k of level D.  `live` (~0 or 0) says whether v
// is still moving down, and a level writes its node only while live.  Reads come from S, the heap as it
// was when the sift began: a sift writes only nodes above the ones it reads, so the reads never wait on
// the writes.  Every ZGPU_SIFT_EXIT levels a wave-uniform test ends a sift that has placed v: 1 (a test
// per level) took the runs block's merges 708k -> 641k clock ticks against the branchy sift it replaced;
// 2, 3 and 9 levels between tests were slower than that, the levels walked past the placement costing
// more than the tests (profiles/r06y_plan_clock_onewave_sift_exit_variants.log, r06z_*).
#ifndef ZGPU_SIFT_EXIT
#define ZGPU_SIFT_EXIT 1
#endif
template <int D>
__device__ __attribute__((always_inline)) inline void rset_if(RHeap &H, uint32_t k, uint32_t v, uint32_t live) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t t = (k & 63u) | (~live & 64u);          // 64: no lane
    if constexpr (D <= 5) H.r[0] = lane == t ? v : H.r[0];
    else if constexpr (D == 6) H.r[1] = lane == t ? v : H.r[1];
    else if constexpr (D == 7) {
        const uint32_t hi = (k & 64u) ? t : 64u, lo = (k & 64u) ? 64u : t;
        H.r[2] = lane == lo ? v : H.r[2];
        H.r[3] = lane == hi ? v : H.r[3];
    } else H.r[4] = lane == t ? v : H.r[4];
}
template <int D>
__device__ __attribute__((always_inline)) inline void r_sift(RHeap &H, const RHeap &S, uint32_t k, uint32_t v,
                                                             uint32_t live) {
    if constexpr (D < 8) {
        const uint32_t j = k << 1;
        uint32_t a, b;
        rget2<D + 1>(S, j, a, b);
        const bool right = hle(b, a);                   // trees.c:515: heap[j+1] <= heap[j]
        uint32_t j1 = j + 1;                            // opaque: jn stays one s_cselect, not VALU ops
        asm volatile("" : "+s"(j1));
        const uint32_t hj = right ? b : a, jn = right ? j1 : j;
        const uint32_t go = hle(v, hj) ? 0u : live;      // trees.c:518: v moves below k
        rset_if<D>(H, k, go ? hj : v, live);
        if constexpr ((D + 1) % ZGPU_SIFT_EXIT == 0) {
            if (go == 0) return;
        }
        r_sift<D + 1>(H, S, jn, v, go);
    } else {
        rset_if<8>(H, k, v, live);
    }
}
template <int D>
__device__ __attribute__((always_inline)) inline void r_sift0(RHeap &H, uint32_t k, uint32_t v) {
    const RHeap S = H;
    r_sift<D>(H, S, k, v, ~0u);
}
// heap[j] for any j < 320 without a branch: one readlane per register and scalar selects
__device__ __attribute__((always_inline)) inline uint32_t rget_sel(const RHeap &H, uint32_t j) {
    const uint32_t l = j & 63u, r = j >> 6;
    const uint32_t v0 = rl(H.r[0], l), v1 = rl(H.r[1], l), v2 = rl(H.r[2], l), v3 = rl(H.r[3], l),
                   v4 = rl(H.r[4], l);
    const uint32_t x = r == 0 ? v0 : v1, y = r == 2 ? v2 : v3;
    return r >= 4 ? v4 : (r >= 2 ? y : x);
}
__device__ inline void r_down_any(RHeap &H, int heap_len, uint32_t k) {   // build_tree's heapify
    const uint32_t v = rget_any(H, k);
    switch (31 - __builtin_clz(k)) {
    case 0: r_sift0<0>(H, k, v); break;
    case 1: r_sift0<1>(H, k, v); break;
    case 2: r_sift0<2>(H, k, v); break;
    case 3: r_sift0<3>(H, k, v); break;
    case 4: r_sift0<4>(H, k, v); break;
    case 5: r_sift0<5>(H, k, v); break;
    case 6: r_sift0<6>(H, k, v); break;
    default: r_sift0<7>(H, k, v); break;                 // k <= heap_len / 2 < 256
    }
}

// ZGPU_PLAN_CLOCK (a timing build, tools/plan_clock.py): s_memtime stamps of
// the first block's tree build in k_enc_plan<true>, written by lane 0 with
// vector stores; zgpu_plan_clock_read copies them out
#ifdef ZGPU_PLAN_CLOCK
__device__ unsigned long long g_pclk[32];
#define PCLK(i) do { if (pclk && (threadIdx.x & 63u) == 0) pclk[i] = (unsigned long long)__builtin_amdgcn_s_memtime(); } while (0)
extern "C" int zgpu_plan_clock_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pclk), sizeof(g_pclk)) == hipSuccess ? 0 : -1;
}
#else
#define PCLK(i) do { (void)pclk; } while (0)
#endif
// Called by all 64 lanes of a wave with wave-uniform arguments; opt_len/static_len stay uniform.
__device__ __attribute__((always_inline)) inline void w_build(TreeRef &t, TreeLDS &h, int elems, const uint8_t *slen, const uint8_t *extra,
                        int xbase, int max_length, int64_t &opt_len, int64_t &static_len,
                        unsigned long long *pclk = nullptr) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t *hs = h.heap;
    int max_code = -1, heap_len = 0;
    for (int c = 0; c < elems; c += 64) {              // the leaves, in symbol order
        const int n = c + (int)lane;
        const uint32_t f = n < elems ? t.freq[n] : 0u;
        const uint64_t m = __ballot(f != 0);
        if (f != 0) hs[heap_len + 1 + __popcll(m & below)] = hkey(f, 0, (uint32_t)n);
        else if (n < elems) t.len[n] = 0;
        if (m) max_code = c + 63 - __clzll(m);
        heap_len += __popcll(m);
    }
    while (heap_len < 2) {                             // trees.c:560-569
        const int node = max_code < 2 ? ++max_code : 0;
        heap_len++;
        if (lane == 0) { hs[heap_len] = hkey(1, 0, (uint32_t)node); t.freq[node] = 1; }
        opt_len--;
        if (slen) static_len -= slen[node];
    }
    t.max_code = max_code;
    __builtin_amdgcn_wave_barrier();
    PCLK(10);
    RHeap H;
#pragma unroll
    for (int r = 0; r < 5; r++) {
        const int j = r * 64 + (int)lane;
        H.r[r] = (j >= 1 && j <= heap_len) ? hs[j] : kHInf;
    }
    for (int k = heap_len / 2; k >= 1; k--) r_down_any(H, heap_len, (uint32_t)k);
    PCLK(11);
    int heap_max = kHeapSize;
    uint32_t node = (uint32_t)elems;
    uint32_t gidx[5];                                  // the heap slot each lane holds per register
#pragma unroll
    for (int r = 0; r < 5; r++) gidx[r] = (uint32_t)(r * 64) + lane;
    do {                                               // trees.c:583-604
        const uint32_t kn = rl(H.r[0], 1);
        const uint32_t last = rget_sel(H, (uint32_t)heap_len);
#pragma unroll
        for (int r = 0; r < 5; r++) H.r[r] = gidx[r] == (uint32_t)heap_len ? kHInf : H.r[r];
        heap_len--;
        r_sift0<0>(H, 1, last);
        const uint32_t km = rl(H.r[0], 1);
        heap_max -= 2;
        if (lane == 0) {
            hs[heap_max + 1] = kn;
            hs[heap_max] = km;
            t.dad[kn & 1023u] = (uint16_t)node;
            t.dad[km & 1023u] = (uint16_t)node;
        }
        const uint32_t f = (kn >> 16) + (km >> 16);
        const uint32_t dn = (kn >> 10) & 63u, dm = (km >> 10) & 63u;
        r_sift0<0>(H, 1, hkey(f, (dn >= dm ? dn : dm) + 1, node));
        node++;
    } while (heap_len >= 2);
    heap_max--;
    const uint32_t rootn = rl(H.r[0], 1) & 1023u;
    if (lane == 0) hs[heap_max] = rl(H.r[0], 1);
    __builtin_amdgcn_wave_barrier();
    PCLK(12);

    // gen_bitlen (trees.c:406-485): depth of every node by pointer jumping; len = min(depth, max_length),
    // overflow = nodes deeper than max_length (a clamped parent pushes its children past it too)
    uint32_t key[kWNodeSlots], pd[kWNodeSlots];        // heap key; dad | depth << 16
#pragma unroll
    for (int i = 0; i < kWNodeSlots; i++) {
        const int hh = heap_max + (int)lane + 64 * i;
        const bool valid = hh < kHeapSize;
        key[i] = valid ? hs[hh] : hkey(0, 0, rootn);
        const uint32_t n = key[i] & 1023u;
        pd[i] = n == rootn ? rootn : (t.dad[n] | (1u << 16));
        if (valid) h.pj[n] = pd[i];
    }
    for (int r = 0; r < 9; r++) {                      // 2^9 > the deepest tree (285)
        bool open = false;
#pragma unroll
        for (int i = 0; i < kWNodeSlots; i++) open |= (pd[i] & 0xffffu) != rootn;
        if (!__any(open)) break;
        // in place: the wave's reads of a round are all issued before its writes, and LDS keeps one
        // wave's instructions in order
        __builtin_amdgcn_wave_barrier();
        uint32_t w[kWNodeSlots];
#pragma unroll
        for (int i = 0; i < kWNodeSlots; i++) w[i] = h.pj[pd[i] & 0xffffu];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kWNodeSlots; i++) {
            pd[i] = (w[i] & 0xffffu) | (((pd[i] >> 16) + (w[i] >> 16)) << 16);
            if (heap_max + (int)lane + 64 * i < kHeapSize) h.pj[key[i] & 1023u] = pd[i];
        }
    }
    PCLK(13);
    int overflow = 0;
    int64_t ol = 0, sl = 0;
    uint32_t bc[kMaxBits + 1];
#pragma unroll
    for (int b = 0; b <= kMaxBits; b++) bc[b] = 0;
#pragma unroll
    for (int i = 0; i < kWNodeSlots; i++) {
        const bool valid = heap_max + (int)lane + 64 * i < kHeapSize;
        const int dep = (int)(pd[i] >> 16), n = (int)(key[i] & 1023u);
        const int bits = dep > max_length ? max_length : dep;
        const bool leaf = valid && n <= max_code;
        if (valid) {
            overflow += dep > max_length;
            t.len[n] = (uint8_t)bits;
        }
        if (leaf) {
            const int xb = n >= xbase ? extra[n - xbase] : 0;
            ol += (int64_t)(key[i] >> 16) * (bits + xb);
            if (slen) sl += (int64_t)(key[i] >> 16) * (slen[n] + xb);
        }
#pragma unroll
        for (int b = 1; b <= kMaxBits; b++) bc[b] += (uint32_t)__popcll(__ballot(leaf && bits == b));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        overflow += __shfl_xor(overflow, o, 64);
        ol += __shfl_xor(ol, o, 64);
        sl += __shfl_xor(sl, o, 64);
    }
    opt_len += ol;
    static_len += sl;
    if (overflow != 0) {                               // trees.c:446-484, one lane
        int64_t dl = 0;
        if (lane == 0) {
            for (int b = 0; b <= kMaxBits; b++) h.bl_count[b] = (uint16_t)bc[b];
            do {
                int bits = max_length - 1;
                while (h.bl_count[bits] == 0) bits--;
                h.bl_count[bits]--;
                h.bl_count[bits + 1] += 2;
                h.bl_count[max_length]--;
                overflow -= 2;
            } while (overflow > 0);
            int hh = kHeapSize;
            for (int bits = max_length; bits != 0; bits--) {
                int n = h.bl_count[bits];
                while (n != 0) {
                    const int m = (int)(hs[--hh] & 1023u);
                    if (m > max_code) continue;
                    if (t.len[m] != bits) {
                        dl += ((int64_t)bits - t.len[m]) * t.freq[m];
                        t.len[m] = (uint8_t)bits;
                    }
                    n--;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        opt_len += __shfl(dl, 0, 64);
#pragma unroll
        for (int b = 0; b <= kMaxBits; b++) bc[b] = h.bl_count[b];
    }
    PCLK(14);
    // gen_codes (trees.c:589-625): a length's codes go to its symbols in symbol order
    uint32_t next[kMaxBits + 1];
    uint32_t c = 0;
#pragma unroll
    for (int b = 1; b <= kMaxBits; b++) { c = (c + bc[b - 1]) << 1; next[b] = c; }
    __builtin_amdgcn_wave_barrier();
    for (int c0 = 0; c0 <= max_code; c0 += 64) {
        const int n = c0 + (int)lane;
        const int len = n <= max_code ? t.len[n] : 0;
        uint32_t code = 0;
#pragma unroll
        for (int b = 1; b <= kMaxBits; b++) {
            const uint64_t m = __ballot(len == b);
            if (len == b) code = next[b] + (uint32_t)__popcll(m & below);
            next[b] += (uint32_t)__popcll(m);
        }
        if (len) t.code[n] = (uint16_t)(__brev(code) >> (32 - len));
    }
    __builtin_amdgcn_wave_barrier();
}

// code-length RLE walk of scan_tree/send_tree (trees.c:712-794)
template <typename Sink>
__device__ void t_rle(const uint8_t *len, int max_code, Sink sink) {
    int prevlen = -1, curlen, nextlen = len[0], count = 0;
    int max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = n + 1 <= max_code ? len[n + 1] : 0xffff;
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            while (count--) sink(curlen, 0, 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) { sink(curlen, 0, 0); count--; }
            sink(16, count - 3, 2);
        } else if (count <= 10) {
            sink(17, count - 3, 3);
        } else {
            sink(18, count - 11, 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

// scan_tree's counts (trees.c:712-757) by a whole wave.  zlib cuts each maximal run of equal code lengths
// into pieces on its own: a run starts in the state max_count 7 / min_count 4 (138 / 3 for zeros) whatever
// precedes it, and its pieces' codes depend only on the run's value v and length L.  Nonzero: L < 4 -> L
// codes v; L <= 7 -> v + REP_3_6; longer: v + REP_3_6 for the first 7, REP_3_6 per 6 after, and a rest r
// of 3..5 -> REP_3_6, 1..2 -> r codes v.  Zero: REPZ_11_138 per 138, and a rest of 11..137 -> REPZ_11_138,
// 3..10 -> REPZ_3_10, 1..2 -> r zeros.  Each run's first lane adds them into bc[19] (LDS).
__device__ __attribute__((always_inline)) inline void w_rle_count(const uint8_t *len, int max_code, uint32_t *bc) {
    const uint32_t lane = threadIdx.x & 63u;
    const int nch = (max_code + 64) >> 6;                       // chunks of 64 entries: 0 .. max_code
    uint64_t m[5] = {0, 0, 0, 0, 0};                            // run starts per chunk (max_code < 320)
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const int n = c * 64 + (int)lane;
        const bool st = c < nch && n <= max_code && (n == 0 || len[n] != len[n - 1]);
        m[c] = __ballot(st);
    }
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const int n = c * 64 + (int)lane;
        if (!((m[c] >> lane) & 1u)) continue;
        // the next run start after n: later in this chunk, else the first in a later chunk, else max_code + 1
        const uint64_t above = lane == 63 ? 0ull : m[c] & (~0ull << (lane + 1));
        int nx = max_code + 1;
        if (above) nx = c * 64 + (int)__ffsll((long long)above) - 1;
        else {
#pragma unroll
            for (int d = c + 1; d < 5; d++)
                if (nx == max_code + 1 && m[d]) nx = d * 64 + (int)__ffsll((long long)m[d]) - 1;
        }
        const uint32_t L = (uint32_t)(nx - n), v = len[n];
        if (v != 0) {
            if (L < 4) atomicAdd(&bc[v], L);
            else {
                atomicAdd(&bc[v], 1u);
                uint32_t rep = 1, lit = 0;
                if (L > 7) {
                    const uint32_t R = L - 7, r = R % 6;
                    rep += R / 6;
                    if (r >= 3) rep++;
                    else lit = r;
                }
                atomicAdd(&bc[16], rep);
                if (lit) atomicAdd(&bc[v], lit);
            }
        } else {
            const uint32_t r = L % 138;
            uint32_t z11 = L / 138;
            if (r >= 11) z11++;
            else if (r >= 3) atomicAdd(&bc[17], 1u);
            else if (r) atomicAdd(&bc[0], r);
            if (z11) atomicAdd(&bc[18], z11);
        }
    }
}

// Output bit stream, staged in LDS: stg[] holds output bits
// [sbase, sbase + kStgBits); everything below sbase is in global memory.
struct Stage {
    uint32_t *stg;
    uint8_t *out;          // buffer's output
    uint64_t cap;          // bytes writable
    int64_t sbase;         // bit offset of stg[0] (multiple of 32)
};

__device__ inline void stg_or(uint32_t *stg, int64_t rel, uint64_t v) {  // v < 2^49
    const int w = (int)(rel >> 5), sh = (int)(rel & 31);
    const uint32_t lo = (uint32_t)(v << sh);
    const uint32_t mid = sh ? (uint32_t)(v >> (32 - sh)) : (uint32_t)(v >> 32);
    const uint32_t hi = sh > 16 ? (uint32_t)(v >> (64 - sh)) : 0u;
    if (lo) atomicOr(&stg[w], lo);
    if (mid) atomicOr(&stg[w + 1], mid);
    if (hi) atomicOr(&stg[w + 2], hi);
}

// write completed words below bit `upto` to global, keep the partial word
__device__ __attribute__((always_inline)) inline void stg_flush(Stage &st, int64_t upto, bool final_flush) {
    const int tid = threadIdx.x;
    const int64_t rel = upto - st.sbase;
    const int full = (int)(rel >> 5);
    const int nwords = final_flush ? (int)((rel + 31) >> 5) : full;
    const uint64_t byte0 = (uint64_t)st.sbase >> 3;
    const uint64_t endbyte = final_flush ? (uint64_t)((upto + 7) >> 3) : byte0 + 4ull * (uint64_t)full;
    for (int w = tid; w < nwords; w += kEncThreads) {
        const uint32_t v = st.stg[w];
        const uint64_t b = byte0 + 4ull * w;
        uint8_t *o = st.out + b;
        if (((reinterpret_cast<uintptr_t>(o) & 3) == 0) && b + 4 <= endbyte && b + 4 <= st.cap) {
            *reinterpret_cast<uint32_t *>(o) = v;
        } else {
            for (int k = 0; k < 4; k++)
                if (b + k < endbyte && b + k < st.cap) o[k] = (uint8_t)(v >> (8 * k));
        }
    }
    __syncthreads();
    if (!final_flush) {
        const uint32_t keep = st.stg[full];
        __syncthreads();
        for (int w = tid; w < kStgWords; w += kEncThreads) st.stg[w] = 0;
        __syncthreads();
        if (tid == 0) st.stg[0] = keep;
        st.sbase += 32ll * full;
        __syncthreads();
    }
}

// build_bl_tree's tail and _tr_flush_block's choice (trees.c:887-905, 997-1074): the block's type, header
// fields and length in bits (from its 3-bit header through END_BLOCK; for a stored block the input length
// is what counts).  One lane, after the three trees.
template <typename TL>
__device__ inline void plan_decide(const DeflateJob &job, const BlockRec &br, const TL &T, int64_t opt_len,
                                   int64_t static_len, int lmax_code, int dmax_code, int &type, int &lmax,
                                   int &dmax, int &blmax, uint64_t &bits) {
    int max_blindex;
    for (max_blindex = kBLCodes - 1; max_blindex >= 3; max_blindex--)
        if (T.blen[c_ct.bl_order[max_blindex]] != 0) break;
    opt_len += 3 * ((int64_t)max_blindex + 1) + 5 + 5 + 4;
    uint64_t opt_lenb = ((uint64_t)opt_len + 3 + 7) >> 3;
    const uint64_t static_lenb = ((uint64_t)static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb || job.strategy == 4) opt_lenb = static_lenb;   // trees.c:1035
    const uint64_t stored_len = br.in_end - br.in_start;
    if (stored_len + 4 <= opt_lenb && (br.flags & kBlkStored)) type = 0;       // trees.c:1027-1074
    else if (static_lenb == opt_lenb) type = 1;
    else type = 2;
    lmax = lmax_code;
    dmax = dmax_code;
    blmax = max_blindex;
    bits = type == 2 ? (uint64_t)opt_len + 3 : (uint64_t)static_len + 3;
}

// One block's histogram (_tr_tally's freq updates, deflate.h:354-372), trees
// (build_tree / gen_bitlen / gen_codes, trees.c:499-706; the whole wave with
// w_build or lane 0 with t_build) and type (_tr_flush_block, trees.c:997-1074)
// into T.  Lane 0 returns the header fields and the block's length in bits
// from its 3-bit header through END_BLOCK (static or dynamic; for a stored
// block the input length is what counts).
template <bool kWaveTrees, typename TL>
__device__ __attribute__((always_inline)) inline void block_plan(const DeflateJob &job, const BlockRec br,
                                                                 const uint32_t *sym, TL &T, uint32_t *hl,
                                                                 uint32_t *hd, int lane, int &type, int &lmax,
                                                                 int &dmax, int &blmax, uint64_t &bits,
                                                                 unsigned long long *pclk = nullptr) {
    PCLK(0);
    for (int i = lane; i < kLCodes; i += 64) hl[i] = 0;
    if (lane < kDCodes) hd[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    // eight symbols per lane in flight: the wave's loads go out together
    // instead of one dependent round trip per 64 symbols (a lone block's
    // histogram is one wave's latency chain)
    constexpr uint32_t kHU = 8;
    for (uint32_t i0 = 0; i0 < br.nsym; i0 += 64 * kHU) {
        uint32_t v[kHU];
#pragma unroll
        for (uint32_t u = 0; u < kHU; u++) {
            const uint32_t i = i0 + 64 * u + (uint32_t)lane;
            v[u] = i < br.nsym ? sym[br.sym_start + i] : 0xffffffffu;
        }
        // every table lookup of the batch is issued before the first atomic: one
        // load latency per batch, not one per symbol (a lone block's histogram)
        uint32_t li[kHU], di[kHU];
#pragma unroll
        for (uint32_t u = 0; u < kHU; u++) {
            const uint32_t dist = v[u] >> 8, lc = v[u] & 0xffu, d = dist - 1u;
            const bool m = v[u] != 0xffffffffu && dist != 0;
            li[u] = m ? c_ct.len_code[lc] + 257u : lc;
            di[u] = m ? (d < 256 ? c_ct.dist_code[d] : c_ct.dist_code[256 + ((d >> 7) & 255u)]) : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kHU; u++) {
            if (v[u] == 0xffffffffu) continue;
            atomicAdd(&hl[li[u]], 1u);
            if (v[u] >> 8) atomicAdd(&hd[di[u]], 1u);
        }
    }
    __builtin_amdgcn_wave_barrier();
    PCLK(1);
    for (int i = lane; i < kLCodes; i += 64) T.lfreq[i] = i == kEndBlock ? 1 : (uint16_t)hl[i];
    if (lane < kDCodes) T.dfreq[lane] = (uint16_t)hd[lane];
    if (lane < kBLCodes) T.bfreq[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    int64_t opt_len = 0, static_len = 0;
    TreeRef lt{T.lfreq, T.ldad, T.lcode, T.llen, 0};
    TreeRef dt{T.dfreq, T.ddad, T.dcode, T.dlen, 0};
    TreeRef bt{T.bfreq, T.bdad, T.bcode, T.blen, 0};
    auto cnt = [&](int s, int, int) { T.bfreq[s]++; };
    if constexpr (kWaveTrees) {
        PCLK(2);
        w_build(lt, T, kLCodes, c_ct.stat_llen, c_ct.xlbits, 257, kMaxBits, opt_len, static_len, pclk);
        PCLK(3);
        w_build(dt, T, kDCodes, c_ct.stat_dlen, c_ct.xdbits, 0, kMaxBits, opt_len, static_len);
        PCLK(4);
        // the histogram words are dead: they take scan_tree's counts (w_rle_count, all lanes)
        if (lane < kBLCodes) hl[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        w_rle_count(T.llen, lt.max_code, hl);
        w_rle_count(T.dlen, dt.max_code, hl);
        __builtin_amdgcn_wave_barrier();
        if (lane < kBLCodes) T.bfreq[lane] = (uint16_t)hl[lane];
        __builtin_amdgcn_wave_barrier();
        PCLK(5);
        w_build(bt, T, kBLCodes, nullptr, c_ct.xblbits, 0, kMaxBLBits, opt_len, static_len);
        PCLK(6);
    } else if (lane == 0) {
        t_build(lt, T, kLCodes, c_ct.stat_llen, c_ct.xlbits, 257, kMaxBits, opt_len, static_len);
        t_build(dt, T, kDCodes, c_ct.stat_dlen, c_ct.xdbits, 0, kMaxBits, opt_len, static_len);
        t_rle(T.llen, lt.max_code, cnt);
        t_rle(T.dlen, dt.max_code, cnt);
        t_build(bt, T, kBLCodes, nullptr, c_ct.xblbits, 0, kMaxBLBits, opt_len, static_len);
    }
    if (lane == 0) plan_decide(job, br, T, opt_len, static_len, lt.max_code, dt.max_code, type, lmax, dmax, blmax, bits);
    PCLK(7);
}

template <bool kWaveTrees>
__global__ __launch_bounds__(kEncThreads) void k_encode(DeflateJob job) {
    __shared__ uint32_t stg[kStgWords];
    __shared__ TreeLDS TT[kEncGroup];
    __shared__ uint32_t HL[kEncGroup][kLCodes], HD[kEncGroup][kDCodes];
    __shared__ uint32_t wsum[kEncThreads / 64];
    __shared__ int64_t s_obit;
    __shared__ struct { int type, lmax, dmax, blmax; } s_hdr[kEncGroup];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const int64_t n = (int64_t)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    const uint32_t *sym = job.sym + job.ws_off[bi];
    const BlockRec *blk = job.blocks + job.blk_off[bi];
    const int level = job.level;

    Stage st;
    st.stg = stg;
    st.out = job.dst + job.dst_off[g];
    st.cap = job.dst_cap[g];
    st.sbase = 0;
    for (int w = tid; w < kStgWords; w += kEncThreads) stg[w] = 0;
    __syncthreads();

    // single-lane bit writer into the staging window
    auto put = [&](uint64_t v, int nb) {      // caller ensures room
        stg_or(stg, s_obit - st.sbase, v);
        s_obit += nb;
    };
    // bi_used at the record's last bi_windup (trees.c: ((bi_valid - 1) & 7) + 1,
    // deflateUsed), 0 when the record has none (tid 0)
    int wu = 0, wu_last = 0;
    auto windup_mark = [&]() { wu = wu_last = (int)((s_obit - 1) & 7) + 1; };
    // a streaming job's record k (tid 0): the output bit after it, the
    // partial byte there (still in the staging window) and wu << 8
    auto stream_rec = [&](uint32_t k) {
        if (!job.srec) return;
        const int64_t r = s_obit - st.sbase;
        job.srec[4ull * k] = (uint64_t)s_obit;
        job.srec[4ull * k + 1] = ((stg[r >> 5] >> (((r >> 3) & 3) * 8)) & ((1u << (r & 7)) - 1u)) | (uint64_t)wu << 8;
        wu = 0;
    };

    if (tid == 0) {
        s_obit = job.bit0;                      // a resumed flush job: the partial byte's bits
        stg[0] = job.byte0;
        if (job.wrap == 1) {                    // zlib header (deflate.c:1004-1037)
            uint32_t header = (8u + ((uint32_t)(job.wbits - 8) << 4)) << 8;
            uint32_t flags = (job.strategy >= 2 || level < 2) ? 0u : level < 6 ? 1u : level == 6 ? 2u : 3u;
            header |= flags << 6;
            header += 31 - (header % 31);
            put(header >> 8, 8);
            put(header & 0xffu, 8);
        } else if (job.wrap == 2) {             // gzip header (deflate.c:1060-1073)
            const uint32_t xfl = level == 9 ? 2u : (job.strategy >= 2 || level < 2) ? 4u : 0u;   // deflate.c:1052
            put(31, 8); put(139, 8); put(8, 8); put(0, 8);
            put(0, 32);
            put(xfl, 8); put(3, 8);             // OS_CODE (zutil.h:184)
        }
    }
    __syncthreads();

    if (level == 0 && !job.plan) {
        // deflate_stored (deflate.c:1635-1815) with a compressBound()-sized
        // output: MAX_STORED-byte stored blocks, last one final.
        int64_t done = 0;
        do {
            const int64_t left = n - done;
            const int64_t len = left < 65535 ? left : 65535;
            const bool last = len == left;
            if (s_obit - st.sbase + 128 > kStgBits) stg_flush(st, s_obit, false);
            if (tid == 0) {
                put(last ? 1u : 0u, 3);
                s_obit = (s_obit + 7) & ~7ll;
                put((uint32_t)len & 0xffffu, 16);
                put((~(uint32_t)len) & 0xffffu, 16);
            }
            __syncthreads();
            int64_t copied = 0;
            while (copied < len) {
                const int64_t room = (st.sbase + kStgBits - 64 - s_obit) >> 3;
                const int64_t take = (len - copied) < room ? (len - copied) : room;
                const int64_t ob = s_obit - st.sbase;
                for (int64_t k = tid; k < take; k += kEncThreads)
                    stg_or(stg, ob + 8 * k, in[done + copied + k]);
                __syncthreads();
                if (tid == 0) s_obit += 8 * take;
                __syncthreads();
                copied += take;
                stg_flush(st, s_obit, false);
            }
            done += len;
            if (last) break;
        } while (true);
        wu_last = 8;                                    // the final block's bi_windup, byte aligned already
    } else {
        const uint32_t nblk = job.nblocks[bi];
        for (uint32_t g0 = 0; g0 < nblk; g0 += kEncGroup) {
            // ---- trees of kEncGroup blocks at once: wave w owns block g0 + w ----
            {
                const uint32_t kb = g0 + (uint32_t)wave;
                if (kb < nblk && level != 0 && !(blk[kb].flags & kBlkMarker)) {
                    int type, lmax, dmax, blmax;
                    uint64_t bits;
                    block_plan<kWaveTrees>(job, blk[kb], sym, TT[wave], HL[wave], HD[wave], lane, type, lmax, dmax,
                                           blmax, bits);
                    if (lane == 0) {
                        s_hdr[wave].type = type;
                        s_hdr[wave].lmax = lmax;
                        s_hdr[wave].dmax = dmax;
                        s_hdr[wave].blmax = blmax;
                    }
                }
            }
            __syncthreads();
          for (int w = 0; w < kEncGroup && g0 + (uint32_t)w < nblk; w++) {
            const uint32_t k = g0 + (uint32_t)w;
            const BlockRec br = blk[k];
            const bool last = br.flags & kBlkLast;
            TreeLDS &T = TT[w];
            if (br.flags & kBlkMarker) {
                // what the deflate(flush) call appends (deflate.c:1211-1233)
                if (s_obit - st.sbase + 128 > kStgBits) stg_flush(st, s_obit, false);
                if (tid == 0) {
                    const uint32_t kind = blk_marker_kind(br.flags);
                    if (job.flush_out) job.flush_out[0] = (uint64_t)s_obit;
                    if (kind == 1) {                    // _tr_align (trees.c:900-904)
                        put(1u << 1, 3);                // STATIC_TREES, not last
                        put(0, 7);                      // END_BLOCK in the static tree
                    } else if (kind == 2 || kind == 3) {   // _tr_stored_block(s, 0, 0, 0)
                        put(0, 3);
                        windup_mark();
                        s_obit = (s_obit + 7) & ~7ll;
                        put(0, 16);
                        put(0xffffu, 16);
                    } else if (kind == kMarkPrime) {       // deflatePrime's bits (deflate.c:731-757)
                        const uint32_t nb = br.pad >> 16;
                        if (nb) put(br.pad & ((1u << nb) - 1u), (int)nb);
                    }
                    stream_rec(k);
                }
                __syncthreads();
                continue;
            }
            // room for the largest block header (dynamic trees: < 5000 bits)
            if (s_obit - st.sbase + 6144 > kStgBits) stg_flush(st, s_obit, false);
            if (tid == 0) {
                const int type = level == 0 ? 0 : s_hdr[w].type;   // a level-0 plan: stored
                const uint64_t stored_len = br.in_end - br.in_start;
                put((uint32_t)(type << 1) + (last ? 1u : 0u), 3);
                if (type == 0) {
                    windup_mark();
                    s_obit = (s_obit + 7) & ~7ll;
                    put((uint32_t)stored_len & 0xffffu, 16);
                    put((~(uint32_t)stored_len) & 0xffffu, 16);
                } else if (type == 2) {
                    const int lcodes = s_hdr[w].lmax + 1, dcodes = s_hdr[w].dmax + 1;
                    const int max_blindex = s_hdr[w].blmax;
                    put((uint32_t)(lcodes - 257), 5);
                    put((uint32_t)(dcodes - 1), 5);
                    put((uint32_t)(max_blindex + 1 - 4), 4);
                    for (int r = 0; r <= max_blindex; r++) put(T.blen[c_ct.bl_order[r]], 3);
                    auto snd = [&](int s, int xv, int xb) {
                        put(T.bcode[s], T.blen[s]);
                        if (xb) put((uint32_t)xv, xb);
                    };
                    t_rle(T.llen, lcodes - 1, snd);
                    t_rle(T.dlen, dcodes - 1, snd);
                }
            }
            __syncthreads();
            const int type = level == 0 ? 0 : s_hdr[w].type;
            if (type == 0) {
                // stored: raw bytes (byte aligned)
                const int64_t len = (int64_t)(br.in_end - br.in_start);
                int64_t copied = 0;
                while (copied < len) {
                    stg_flush(st, s_obit, false);
                    const int64_t room = (st.sbase + kStgBits - 64 - s_obit) >> 3;
                    const int64_t take = (len - copied) < room ? (len - copied) : room;
                    const int64_t ob = s_obit - st.sbase;
                    for (int64_t i = tid; i < take; i += kEncThreads)
                        stg_or(stg, ob + 8 * i, in[br.in_start + copied + i]);
                    __syncthreads();
                    if (tid == 0) s_obit += 8 * take;
                    __syncthreads();
                    copied += take;
                }
            } else {
                const uint16_t *lcode = type == 1 ? c_ct.stat_lcode : T.lcode;
                const uint8_t *llen = type == 1 ? c_ct.stat_llen : T.llen;
                uint32_t nxt = (uint32_t)tid < br.nsym ? sym[br.sym_start + tid] : 0u;   // loaded a batch ahead
                for (uint32_t base = 0; base < br.nsym + 1; base += kEncThreads) {
                    // +1: the END_BLOCK code rides in the last batch
                    const uint32_t i = base + tid;
                    const uint32_t cur = nxt;
                    if (i + kEncThreads < br.nsym) nxt = sym[br.sym_start + i + kEncThreads];
                    uint64_t v = 0;
                    int nb = 0;
                    if (i < br.nsym) {
                        const uint32_t s = cur;
                        const uint32_t dist = s >> 8, lc = s & 0xffu;
                        if (dist == 0) {
                            v = lcode[lc]; nb = llen[lc];
                        } else {
                            const uint32_t code = c_ct.len_code[lc];
                            v = lcode[code + 257]; nb = llen[code + 257];
                            const int xl = c_ct.xlbits[code];
                            if (xl) { v |= (uint64_t)(lc - c_ct.len_base[code]) << nb; nb += xl; }
                            const uint32_t d = dist - 1;
                            const uint32_t dc = d < 256 ? c_ct.dist_code[d] : c_ct.dist_code[256 + (d >> 7)];
                            const uint32_t dcv = type == 1 ? c_ct.stat_dcode[dc] : T.dcode[dc];
                            const int dl = type == 1 ? 5 : T.dlen[dc];
                            v |= (uint64_t)dcv << nb; nb += dl;
                            const int xd = c_ct.xdbits[dc];
                            if (xd) { v |= (uint64_t)(d - c_ct.dist_base[dc]) << nb; nb += xd; }
                        }
                    } else if (i == br.nsym) {
                        v = lcode[kEndBlock]; nb = llen[kEndBlock];
                    }
                    // block-wide exclusive scan of nb
                    int incl = nb;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        int t = __shfl_up(incl, o, 64);
                        if (lane >= o) incl += t;
                    }
                    if (lane == 63) wsum[wave] = (uint32_t)incl;
                    __syncthreads();
                    int wpre = 0, total = 0;
                    for (int w = 0; w < kEncThreads / 64; w++) {
                        if (w < wave) wpre += (int)wsum[w];
                        total += (int)wsum[w];
                    }
                    const int excl = wpre + incl - nb;
                    if (s_obit - st.sbase + total + 64 > kStgBits) stg_flush(st, s_obit, false);
                    if (nb) stg_or(stg, s_obit - st.sbase + excl, v);
                    __syncthreads();
                    if (tid == 0) s_obit += total;
                    __syncthreads();
                }
            }
            if (last && tid == 0) {                  // bi_windup
                windup_mark();
                s_obit = (s_obit + 7) & ~7ll;
            }
            __syncthreads();
            if (job.srec) {                      // a streaming job: where this block ends
                if (tid == 0) stream_rec(k);
                __syncthreads();
            }
          }
        }
    }
    // trailer
    __syncthreads();
    if (s_obit - st.sbase + 96 > kStgBits) stg_flush(st, s_obit, false);
    if (tid == 0 && job.wind) job.wind[bi] = (uint8_t)wu_last;
    if (tid == 0) {
        const uint32_t ck = job.check[bi];
        if (job.wrap == 1) {                    // Adler-32, big-endian (deflate.c:1253-1256)
            put(ck >> 24, 8); put((ck >> 16) & 0xffu, 8); put((ck >> 8) & 0xffu, 8); put(ck & 0xffu, 8);
        } else if (job.wrap == 2) {             // CRC-32 + ISIZE, little-endian
            put(ck, 32);
            put((uint32_t)n, 32);
        }
    }
    __syncthreads();
    if (tid == 0 && job.flush_out) {
        const int64_t r = s_obit - st.sbase;
        job.flush_out[1] = (uint64_t)s_obit;
        job.flush_out[3] = (stg[r >> 5] >> (((r >> 3) & 3) * 8)) & 0xffu;
    }
    stg_flush(st, s_obit, true);
    if (tid == 0) {
        const uint64_t total = (uint64_t)(s_obit >> 3);
        job.dst_len[g] = total <= st.cap ? total : st.cap;
        job.status[g] = total <= st.cap ? 0 : -5;
    }
}

// ------------------------------------------------------------------------
// k_enc_plan / k_enc_scan / k_enc_emit — k_encode for a sub-batch of few large
// buffers, with a buffer's blocks spread over many workgroups instead of one:
//   k_enc_plan  one wave per block: block_plan (trees, type, length in bits),
//               the code tables into EncPlan records
//   k_enc_scan  one workgroup per buffer: every block's first output bit (a
//               stored block aligns after its 3-bit header, the last block
//               winds up to a byte), the output length, and zeroes the words
//               two blocks share
//   k_enc_emit  one workgroup per block: the block's bits at its offset,
//               written through an LDS window as k_encode does; the words a
//               block shares with its neighbours (its first and last) are
//               or-ed in atomically, every other word is the block's alone
// Block 0 also writes the zlib/gzip header, the last block the trailer.
// ------------------------------------------------------------------------
// a buffer's block records fit its region of the block / plan arrays (n /
// sym_limit + 2 records, zgpu_api.cpp): the plan of block nblocks is the end mark
__device__ inline bool enc_blocks_ok(const DeflateJob &job, uint32_t bi, uint32_t nblk) {
    const uint64_t n = job.src_len[job.first + bi];
    return nblk >= 1 && (uint64_t)nblk + 1 <= n / job_win(job).sym_limit + 2;
}

template <bool kWaveTrees>
__global__ __launch_bounds__(kEncThreads) void k_enc_plan(DeflateJob job) {
    __shared__ TreeLDS TT[kEncGroup];
    __shared__ uint32_t HL[kEncGroup][kLCodes], HD[kEncGroup][kDCodes];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t bi = blockIdx.y;
    const uint32_t kb = blockIdx.x * kEncGroup + (uint32_t)wave;
    const uint32_t nblk = job.nblocks[bi];
    if (kb >= nblk || !enc_blocks_ok(job, bi, nblk)) return;   // per wave: no workgroup barrier below
    const BlockRec br = job.blocks[job.blk_off[bi] + kb];
    TreeLDS &T = TT[wave];
    int type = 0, lmax = 0, dmax = 0, blmax = 0;
    uint64_t bits = 0;
#ifdef ZGPU_PLAN_CLOCK
    unsigned long long *pclk = kb == 0 && bi == 0 ? g_pclk : nullptr;
#else
    unsigned long long *pclk = nullptr;
#endif
    block_plan<kWaveTrees>(job, br, job.sym + job.ws_off[bi], T, HL[wave], HD[wave], lane, type, lmax, dmax, blmax,
                           bits, pclk);
    EncPlan &P = job.eplan[job.blk_off[bi] + kb];
    __builtin_amdgcn_wave_barrier();                  // lane 0's tables (t_build) before the copy
    type = __shfl(type, 0, 64);
    if (lane == 0) {
        P.type = (uint8_t)type;
        P.lmax = (uint16_t)lmax;
        P.dmax = (uint16_t)dmax;
        P.blmax = (uint16_t)blmax;
        P.bits = bits;
    }
    if (type == 2) {
        for (int i = lane; i < kLCodes; i += 64) { P.lcode[i] = T.lcode[i]; P.llen[i] = T.llen[i]; }
        if (lane < kDCodes) { P.dcode[lane] = T.dcode[lane]; P.dlen[lane] = T.dlen[lane]; }
        if (lane < kBLCodes) { P.bcode[lane] = T.bcode[lane]; P.blen[lane] = T.blen[lane]; }
    }
    PCLK(8);
}

// k_enc_plan2 — the wave trees for sub-batches of few blocks (a lone compress2), two waves per block:
// the pair splits the block's histogram; wave 0 builds the literal/length tree while wave 1 builds the
// distance tree (its heap scratch in the pair's second TreeLDS); each counts the code-length runs of its
// own tree for the bit-length tree (scan_tree, trees.c:712-757; the counts are sums, so their order does
// not matter); wave 0 then builds the bit-length tree and decides.  Against k_enc_plan<true> (one wave
// per block) the distance tree and half the histogram leave the critical path.
constexpr int kPlan2Pairs = kEncThreads / 128;
__global__ __launch_bounds__(kEncThreads) void k_enc_plan2(DeflateJob job) {
    static_assert(kEncGroup == 2 * kPlan2Pairs, "a TreeLDS per wave");
    __shared__ TreeLDS TT[kEncGroup];
    __shared__ uint32_t HL[kPlan2Pairs][kLCodes], HD[kPlan2Pairs][kDCodes], BC[kPlan2Pairs][kBLCodes];
    __shared__ int64_t s_len[kPlan2Pairs][2];
    __shared__ int s_dmax[kPlan2Pairs];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, pair = wave >> 1, wp = wave & 1;
    const uint32_t bi = blockIdx.y;
    const uint32_t kb = blockIdx.x * kPlan2Pairs + (uint32_t)pair;
    const uint32_t nblk = job.nblocks[bi];
    const bool active = kb < nblk && enc_blocks_ok(job, bi, nblk);   // every wave reaches every barrier
    BlockRec br{};
    if (active) br = job.blocks[job.blk_off[bi] + kb];
    const uint32_t *sym = job.sym + job.ws_off[bi];
    TreeLDS &T = TT[2 * pair];
    uint32_t *hl = HL[pair], *hd = HD[pair];
    for (int i = (wp << 6) | lane; i < kLCodes; i += 128) hl[i] = 0;
    if (wp == 0 && lane < kDCodes) hd[lane] = 0;
    if (wp == 1 && lane < kBLCodes) BC[pair][lane] = 0;
    __syncthreads();
    if (active) {                                      // the histogram, batches of 512 symbols alternating
        constexpr uint32_t kHU = 8;
        for (uint32_t i0 = (uint32_t)wp * 64 * kHU; i0 < br.nsym; i0 += 2 * 64 * kHU) {
            uint32_t v[kHU], li[kHU], di[kHU];
#pragma unroll
            for (uint32_t u = 0; u < kHU; u++) {
                const uint32_t i = i0 + 64 * u + (uint32_t)lane;
                v[u] = i < br.nsym ? sym[br.sym_start + i] : 0xffffffffu;
            }
#pragma unroll
            for (uint32_t u = 0; u < kHU; u++) {
                const uint32_t dist = v[u] >> 8, lc = v[u] & 0xffu, d = dist - 1u;
                const bool m = v[u] != 0xffffffffu && dist != 0;
                li[u] = m ? c_ct.len_code[lc] + 257u : lc;
                di[u] = m ? (d < 256 ? c_ct.dist_code[d] : c_ct.dist_code[256 + ((d >> 7) & 255u)]) : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < kHU; u++) {
                if (v[u] == 0xffffffffu) continue;
                atomicAdd(&hl[li[u]], 1u);
                if (v[u] >> 8) atomicAdd(&hd[di[u]], 1u);
            }
        }
    }
    __syncthreads();
    if (active) {
        for (int i = (wp << 6) | lane; i < kLCodes; i += 128) T.lfreq[i] = i == kEndBlock ? 1 : (uint16_t)hl[i];
        if (wp == 0 && lane < kDCodes) T.dfreq[lane] = (uint16_t)hd[lane];
    }
    __syncthreads();
    int64_t opt_len = 0, static_len = 0;
    TreeRef lt{T.lfreq, T.ldad, T.lcode, T.llen, 0};
    TreeRef dt{T.dfreq, T.ddad, T.dcode, T.dlen, 0};
    TreeRef bt{T.bfreq, T.bdad, T.bcode, T.blen, 0};
    if (active) {
        if (wp == 0) w_build(lt, T, kLCodes, c_ct.stat_llen, c_ct.xlbits, 257, kMaxBits, opt_len, static_len);
        else w_build(dt, TT[2 * pair + 1], kDCodes, c_ct.stat_dlen, c_ct.xdbits, 0, kMaxBits, opt_len, static_len);
        __builtin_amdgcn_wave_barrier();
        if (wp == 0) {
            w_rle_count(T.llen, lt.max_code, BC[pair]);
        } else {
            w_rle_count(T.dlen, dt.max_code, BC[pair]);
            if (lane == 0) {
                s_len[pair][0] = opt_len;
                s_len[pair][1] = static_len;
                s_dmax[pair] = dt.max_code;
            }
        }
    }
    __syncthreads();
    if (!active || wp != 0) return;
    if (lane < kBLCodes) T.bfreq[lane] = (uint16_t)BC[pair][lane];
    opt_len += s_len[pair][0];
    static_len += s_len[pair][1];
    __builtin_amdgcn_wave_barrier();
    w_build(bt, T, kBLCodes, nullptr, c_ct.xblbits, 0, kMaxBLBits, opt_len, static_len);
    int type = 0, lmax = 0, dmax = 0, blmax = 0;
    uint64_t bits = 0;
    if (lane == 0) plan_decide(job, br, T, opt_len, static_len, lt.max_code, s_dmax[pair], type, lmax, dmax, blmax, bits);
    EncPlan &P = job.eplan[job.blk_off[bi] + kb];
    __builtin_amdgcn_wave_barrier();                  // lane 0's tables (t_build) before the copy
    type = __shfl(type, 0, 64);
    if (lane == 0) {
        P.type = (uint8_t)type;
        P.lmax = (uint16_t)lmax;
        P.dmax = (uint16_t)dmax;
        P.blmax = (uint16_t)blmax;
        P.bits = bits;
    }
    if (type == 2) {
        for (int i = lane; i < kLCodes; i += 64) { P.lcode[i] = T.lcode[i]; P.llen[i] = T.llen[i]; }
        if (lane < kDCodes) { P.dcode[lane] = T.dcode[lane]; P.dlen[lane] = T.dlen[lane]; }
        if (lane < kBLCodes) { P.bcode[lane] = T.bcode[lane]; P.blen[lane] = T.blen[lane]; }
    }
}

// k_enc_plan for batches (one-lane tree builds): one wave per block and the
// smallest tree storage (no w_build exchange; the symbol histograms share the
// heap's words, dead before the build starts), 5.6 KiB of LDS, so that plan
// workgroups fit beside k_match's 153.6 KiB on a CU while the pipeline runs
// both: 10606 -> 10807 MB/s on the C4 shard with the smaller k_enc_emit
// (profiles/r03q_ab_coresident_encode.log)
__global__ __launch_bounds__(64) void k_enc_plan1(DeflateJob job) {
    __shared__ TreeLDSLane T;
    const int lane = threadIdx.x;
    const uint32_t bi = blockIdx.y;
    const uint32_t kb = blockIdx.x;
    const uint32_t nblk = job.nblocks[bi];
    if (kb >= nblk || !enc_blocks_ok(job, bi, nblk)) return;
    const BlockRec br = job.blocks[job.blk_off[bi] + kb];
    static_assert(sizeof(T.heap) >= sizeof(uint32_t) * (kLCodes + kDCodes), "histograms in the heap's words");
    uint32_t *hl = T.heap, *hd = T.heap + kLCodes;
    int type = 0, lmax = 0, dmax = 0, blmax = 0;
    uint64_t bits = 0;
    block_plan<false>(job, br, job.sym + job.ws_off[bi], T, hl, hd, lane, type, lmax, dmax, blmax, bits);
    EncPlan &P = job.eplan[job.blk_off[bi] + kb];
    __builtin_amdgcn_wave_barrier();                  // lane 0's tables (t_build) before the copy
    type = __shfl(type, 0, 64);
    if (lane == 0) {
        P.type = (uint8_t)type;
        P.lmax = (uint16_t)lmax;
        P.dmax = (uint16_t)dmax;
        P.blmax = (uint16_t)blmax;
        P.bits = bits;
    }
    if (type == 2) {
        for (int i = lane; i < kLCodes; i += 64) { P.lcode[i] = T.lcode[i]; P.llen[i] = T.llen[i]; }
        if (lane < kDCodes) { P.dcode[lane] = T.dcode[lane]; P.dlen[lane] = T.dlen[lane]; }
        if (lane < kBLCodes) { P.bcode[lane] = T.bcode[lane]; P.blen[lane] = T.blen[lane]; }
    }
}

// 256 threads (3 KiB of LDS): a k_enc_scan workgroup fits beside k_match on a CU, as k_enc_plan1 and
// k_enc_emit do (no measurable change on the C4 shard: profiles/r03r_ab_scan256.log); the offsets
// are a serial walk over the blocks either way
constexpr int kEScanThreads = 256;
__device__ inline uint64_t wrap_head_bits(int wrap) { return wrap == 1 ? 16 : wrap == 2 ? 80 : 0; }
__device__ inline uint64_t wrap_tail_bits(int wrap) { return wrap == 1 ? 32 : wrap == 2 ? 64 : 0; }

// zero the bytes of output word w (4-byte aligned, of the word array that
// starts a3 bytes before the buffer's output) that lie in [lo, hi) bytes
__device__ inline void zero_word_bytes(uint8_t *out, uint32_t a3, int64_t w, int64_t lo, int64_t hi) {
    for (int j = 0; j < 4; j++) {
        const int64_t b = 4 * w + j - (int64_t)a3;
        if (b >= lo && b < hi) out[b] = 0;
    }
}

__global__ __launch_bounds__(kEScanThreads) void k_enc_scan(DeflateJob job) {
    __shared__ uint64_t s_v[kEScanThreads];
    __shared__ uint32_t s_ty[kEScanThreads];
    __shared__ uint64_t s_off;
    const int tid = threadIdx.x;
    const uint32_t bi = blockIdx.x, g = job.first + bi;
    const uint32_t nblk = job.nblocks[bi];
    const BlockRec *blk = job.blocks + job.blk_off[bi];
    EncPlan *pl = job.eplan + job.blk_off[bi];
    uint8_t *out = job.dst + job.dst_off[g];
    const int64_t cap = (int64_t)job.dst_cap[g];
    const uint32_t a3 = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 3u);
    const uint64_t tb = wrap_tail_bits(job.wrap);
    if (job.srec && nblk == 0) {                           // a streaming job that stops before its first block
        if (tid == 0) {
            if (cap > 0) out[0] = (uint8_t)job.byte0;      // the partial byte it resumed at, as k_encode leaves it
            job.dst_len[g] = 0;
            job.status[g] = 0;
            if (job.flush_out) { job.flush_out[1] = job.bit0; job.flush_out[3] = job.byte0; }
        }
        return;
    }
    if (!enc_blocks_ok(job, bi, nblk)) {                   // never expected: report, write nothing
        if (tid == 0) { job.dst_len[g] = 0; job.status[g] = -2; }
        return;
    }
    if (tid == 0) s_off = wrap_head_bits(job.wrap) + job.bit0;   // a resumed streaming job: after the partial byte
    __syncthreads();
    for (uint32_t c0 = 0; c0 < nblk; c0 += kEScanThreads) {
        const uint32_t m = nblk - c0 < (uint32_t)kEScanThreads ? nblk - c0 : (uint32_t)kEScanThreads;
        if ((uint32_t)tid < m) {
            const uint32_t k = c0 + tid;
            const BlockRec br = blk[k];
            const uint32_t ty = pl[k].type;
            s_ty[tid] = ty | (br.flags & kBlkLast ? 4u : 0u);
            s_v[tid] = ty == 0 ? br.in_end - br.in_start : pl[k].bits;
        }
        __syncthreads();
        if (tid == 0) {                                    // the offsets, in order
            uint64_t off = s_off;
            for (uint32_t i = 0; i < m; i++) {
                const uint64_t st = off, v = s_v[i];
                const uint32_t ty = s_ty[i];
                // bi_used at the block's last bi_windup (deflateUsed): after a
                // stored block's header, at the end of the last block
                uint32_t wu = (ty & 3u) == 0 ? (uint32_t)((off + 3 - 1) & 7) + 1 : 0u;
                off = (ty & 3u) == 0 ? ((off + 3 + 7) & ~7ull) + 32 + 8 * v : off + v;
                if (ty & 4u) wu = (uint32_t)((off - 1) & 7) + 1;
                if ((ty & 4u) && job.wind) job.wind[bi] = (uint8_t)wu;
                if (ty & 4u) off = (off + 7) & ~7ull;      // bi_windup
                if (job.srec) pl[c0 + i].pad0 = (uint8_t)wu;   // k_enc_rec
                s_v[i] = st;
            }
            s_off = off;
        }
        __syncthreads();
        const uint64_t after = s_off;
        const bool fin = c0 + m == nblk;
        if ((uint32_t)tid < m) {
            const uint32_t k = c0 + tid;
            const uint64_t st = s_v[tid];
            pl[k].start = st;
            // the block's range of output bits: block 0 from the stream
            // header on, the last one through the trailer
            const int64_t rs = k == 0 ? 0 : (int64_t)st;
            const int64_t re = (uint32_t)tid + 1 < m ? (int64_t)s_v[tid + 1] : (int64_t)after + (fin ? (int64_t)tb : 0);
            if (re > rs) {
                const int64_t lo = rs >> 3, hi = (re + 7) >> 3 < cap ? (re + 7) >> 3 : cap;
                const int64_t w0 = (rs + 8 * a3) >> 5, w1 = (re - 1 + 8 * a3) >> 5;
                zero_word_bytes(out, a3, w0, lo, hi);
                if (w1 != w0) zero_word_bytes(out, a3, w1, lo, hi);
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        const uint64_t total = s_off + tb;
        pl[nblk].start = total;                            // the last block's range end
        const uint64_t bytes = total >> 3;
        job.dst_len[g] = bytes <= (uint64_t)cap ? bytes : (uint64_t)cap;
        job.status[g] = bytes <= (uint64_t)cap ? 0 : -5;
    }
}

__global__ __launch_bounds__(kEncThreads) void k_enc_emit(DeflateJob job) {
    __shared__ uint32_t stg[kEmitStgWords];
    __shared__ uint16_t s_lcode[kLCodes], s_dcode[kDCodes], s_bcode[kBLCodes];
    __shared__ uint8_t s_llen[kLCodes], s_dlen[kDCodes], s_blen[kBLCodes];
    __shared__ uint32_t wsum2[2][kEncThreads / 64];
    __shared__ int64_t s_obit, s_sbase;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t bi = blockIdx.y, k = blockIdx.x;
    const uint32_t nblk = job.nblocks[bi];
    if (k >= nblk || !enc_blocks_ok(job, bi, nblk)) return;   // uniform per workgroup
    const uint32_t g = job.first + bi;
    const uint8_t *in = job.src + job.src_off[g];
    const uint32_t *sym = job.sym + job.ws_off[bi];
    const EncPlan *pl = job.eplan + job.blk_off[bi];
    const BlockRec br = job.blocks[job.blk_off[bi] + k];
    const bool last = br.flags & kBlkLast;
    const int type = pl[k].type;
    uint8_t *out = job.dst + job.dst_off[g];
    const int64_t cap = (int64_t)job.dst_cap[g];
    const uint32_t a3 = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 3u);
    uint32_t *ow = reinterpret_cast<uint32_t *>(out - a3);
    const int64_t sh = 8 * (int64_t)a3;                   // stream bit x is bit x + sh of ow[]
    const int64_t rs = k == 0 ? 0 : (int64_t)pl[k].start, re = (int64_t)pl[k + 1].start;
    const int64_t wfirst = (rs + sh) >> 5, wlast = (re - 1 + sh) >> 5;
    for (int w = tid; w < kEmitStgWords; w += kEncThreads) stg[w] = 0;
    if (type == 2) {
        const EncPlan &P = pl[k];
        for (int i = tid; i < kLCodes; i += kEncThreads) { s_lcode[i] = P.lcode[i]; s_llen[i] = P.llen[i]; }
        if (tid < kDCodes) { s_dcode[tid] = P.dcode[tid]; s_dlen[tid] = P.dlen[tid]; }
        if (tid < kBLCodes) { s_bcode[tid] = P.bcode[tid]; s_blen[tid] = P.blen[tid]; }
    } else if (type == 1) {                                // static trees (trees.c:292)
        for (int i = tid; i < kLCodes; i += kEncThreads) { s_lcode[i] = c_ct.stat_lcode[i]; s_llen[i] = c_ct.stat_llen[i]; }
        if (tid < kDCodes) { s_dcode[tid] = c_ct.stat_dcode[tid]; s_dlen[tid] = 5; }
    }
    if (tid == 0) {
        s_sbase = ((rs + sh) >> 5) << 5;
        s_obit = (k == 0 ? 0 : (int64_t)pl[k].start) + sh;
    }
    __syncthreads();

    int64_t sbase = s_sbase;
    auto put = [&](uint64_t v, int nb) {                  // lane 0 only; caller ensures room
        stg_or(stg, s_obit - sbase, v);
        s_obit += nb;
    };
    // completed words below aligned bit `upto` to global (all of them: fin)
    auto eflush = [&](int64_t upto, bool fin) {
        __syncthreads();                                   // the staged bits of every thread
        const int64_t rel = upto - sbase;
        const int full = (int)(rel >> 5);
        const int nwords = fin ? (int)((rel + 31) >> 5) : full;
        for (int w = tid; w < nwords; w += kEncThreads) {
            const int64_t gw = (sbase >> 5) + w;
            const int64_t b0 = 4 * gw - (int64_t)a3;
            uint32_t mask = 0xffffffffu;
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (b0 + j < 0 || b0 + j >= cap) mask &= ~(0xffu << (8 * j));
            const uint32_t v = stg[w] & mask;
            if (gw == wfirst || gw == wlast) {             // shared with a neighbour: zeroed by k_enc_scan
                if (v) atomicOr(&ow[gw], v);
            } else if (mask == 0xffffffffu) {
                ow[gw] = v;
            } else {                                       // cut by the capacity: this block's bytes only
                uint8_t *ob = reinterpret_cast<uint8_t *>(ow + gw);
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if ((mask >> (8 * j)) & 0xffu) ob[j] = (uint8_t)(v >> (8 * j));
            }
        }
        __syncthreads();
        if (!fin) {
            const uint32_t keep = stg[full];
            __syncthreads();
            for (int w = tid; w < kEmitStgWords; w += kEncThreads) stg[w] = 0;
            __syncthreads();
            if (tid == 0) stg[0] = keep;
            sbase += 32ll * full;
            __syncthreads();
        }
    };
    if (tid == 0) {
        // lane 0's header bits go through a register bit writer: whole words are stored to the staging
        // words (zeroed above, no other writer yet), where put()'s LDS read-modify-write of s_obit and
        // atomic ORs per call were dependent round trips (a full literal tree's header is ~300 calls)
        uint64_t acc = 0;
        int nacc = (int)((s_obit - sbase) & 31);
        int wi = (int)((s_obit - sbase) >> 5);
        auto put = [&](uint64_t v, int nb) {              // v < 2^32, nb <= 32
            acc |= v << nacc;
            nacc += nb;
            if (nacc >= 32) {
                stg[wi++] = (uint32_t)acc;
                acc >>= 32;
                nacc -= 32;
            }
        };
        auto align8 = [&] {
            nacc = (nacc + 7) & ~7;
            if (nacc >= 32) {
                stg[wi++] = (uint32_t)acc;
                acc >>= 32;
                nacc -= 32;
            }
        };
        if (k == 0 && job.bit0) put(job.byte0, (int)job.bit0);   // a resumed streaming job's partial byte
        if (k == 0 && job.wrap == 1) {                     // zlib header (deflate.c:1004-1037)
            uint32_t header = (8u + ((uint32_t)(job.wbits - 8) << 4)) << 8;
            const int level = job.level;
            uint32_t flags = (job.strategy >= 2 || level < 2) ? 0u : level < 6 ? 1u : level == 6 ? 2u : 3u;
            header |= flags << 6;
            header += 31 - (header % 31);
            put(header >> 8, 8);
            put(header & 0xffu, 8);
        } else if (k == 0 && job.wrap == 2) {              // gzip header (deflate.c:1060-1073)
            const int level = job.level;
            const uint32_t xfl = level == 9 ? 2u : (job.strategy >= 2 || level < 2) ? 4u : 0u;
            put(31, 8); put(139, 8); put(8, 8); put(0, 8);
            put(0, 32);
            put(xfl, 8); put(3, 8);
        }
        const uint64_t stored_len = br.in_end - br.in_start;
        put((uint32_t)(type << 1) + (last ? 1u : 0u), 3);
        if (type == 0) {
            align8();
            put((uint32_t)stored_len & 0xffffu, 16);
            put((~(uint32_t)stored_len) & 0xffffu, 16);
        } else if (type == 2) {                            // send_all_trees (trees.c:800-824)
            const int lcodes = pl[k].lmax + 1, dcodes = pl[k].dmax + 1, max_blindex = pl[k].blmax;
            put((uint32_t)(lcodes - 257), 5);
            put((uint32_t)(dcodes - 1), 5);
            put((uint32_t)(max_blindex + 1 - 4), 4);
            for (int r = 0; r <= max_blindex; r++) put(s_blen[c_ct.bl_order[r]], 3);
            auto snd = [&](int sy, int xv, int xb) {
                put(s_bcode[sy], s_blen[sy]);
                if (xb) put((uint32_t)xv, xb);
            };
            t_rle(s_llen, lcodes - 1, snd);
            t_rle(s_dlen, dcodes - 1, snd);
        }
        if (nacc > 0) stg[wi] = (uint32_t)acc;
        s_obit = sbase + 32ll * wi + nacc;
    }
    __syncthreads();
    if (type == 0) {                                       // stored: the raw bytes
        const int64_t len = (int64_t)(br.in_end - br.in_start);
        int64_t copied = 0;
        while (copied < len) {
            eflush(s_obit, false);
            const int64_t room = (sbase + kEmitStgBits - 64 - s_obit) >> 3;
            const int64_t take = (len - copied) < room ? (len - copied) : room;
            const int64_t ob = s_obit - sbase;
            for (int64_t i = tid; i < take; i += kEncThreads) stg_or(stg, ob + 8 * i, in[br.in_start + copied + i]);
            __syncthreads();
            if (tid == 0) s_obit += 8 * take;
            __syncthreads();
            copied += take;
        }
    } else {
        // a symbol's code (compress_block, trees.c:1105-1135) from LDS and arithmetic, no dependent loads of
        // c_ct.  _length_code (trees.c:1113-1125): lc < 8 is its own code, 255 is code 28; else with b =
        // floor(log2 lc), code 4(b-1) + bits b-1..b-2 of lc, and the b-2 bits below are the extra bits.
        // d_code (trees.c:80-85): for d >= 4, with b = floor(log2 d), code 2b + bit b-1 of d, base (2 | that
        // bit) << (b-1), so d - base = d mod 2^(b-1)
        auto code = [&](uint32_t sy, uint64_t &v, int &nb) {
            const uint32_t dist = sy >> 8, lc = sy & 0xffu;
            if (dist == 0) {
                v = s_lcode[lc]; nb = s_llen[lc];
                return;
            }
            const uint32_t bl = 31u - (uint32_t)__clz((int)(lc | 1u));
            const uint32_t lcd = lc < 8 ? lc : lc == 255 ? 28u : 4 * (bl - 1) + ((lc >> (bl - 2)) & 3u);
            const uint32_t xl = lc < 8 || lc == 255 ? 0u : bl - 2;
            v = s_lcode[lcd + 257]; nb = s_llen[lcd + 257];
            v |= (uint64_t)(lc & ((1u << xl) - 1u)) << nb; nb += (int)xl;
            const uint32_t d = dist - 1;
            const uint32_t b = 31u - (uint32_t)__clz((int)(d | 1u));
            const uint32_t dc = d < 4 ? d : 2 * b + ((d >> (b - 1)) & 1u);
            const uint32_t xd = d < 4 ? 0u : b - 1;
            v |= (uint64_t)s_dcode[dc] << nb; nb += s_dlen[dc];
            v |= (uint64_t)(d & ((1u << xd) - 1u)) << nb; nb += (int)xd;
        };
        // two symbols per thread (2t, 2t + 1 of a batch of 512: at most 48 bits each, so a batch fits the
        // staging window after a flush) and one barrier per batch: every thread keeps the bit position,
        // the wave sums alternate between two slots, and a flush starts with its own barrier.  The next
        // batch's symbols are loaded while this one is scanned and placed.
        constexpr uint32_t kBatch = 2 * kEncThreads;
        static_assert(kBatch * 48 + 64 <= (uint32_t)kEmitStgBits - 32, "a batch fits the window after a flush");
        const uint32_t i0 = 2u * (uint32_t)tid;
        uint32_t n0 = i0 < br.nsym ? sym[br.sym_start + i0] : 0u;
        uint32_t n1 = i0 + 1 < br.nsym ? sym[br.sym_start + i0 + 1] : 0u;
        int64_t ob = s_obit;
        int par = 0;
        for (uint32_t base = 0; base < br.nsym + 1; base += kBatch) {   // +1: END_BLOCK
            const uint32_t i = base + i0;
            const uint32_t c0 = n0, c1 = n1;
            if (i + kBatch < br.nsym) n0 = sym[br.sym_start + i + kBatch];
            if (i + kBatch + 1 < br.nsym) n1 = sym[br.sym_start + i + kBatch + 1];
            uint64_t v0 = 0, v1 = 0;
            int nb0 = 0, nb1 = 0;
            if (i < br.nsym) code(c0, v0, nb0);
            else if (i == br.nsym) { v0 = s_lcode[kEndBlock]; nb0 = s_llen[kEndBlock]; }
            if (i + 1 < br.nsym) code(c1, v1, nb1);
            else if (i + 1 == br.nsym) { v1 = s_lcode[kEndBlock]; nb1 = s_llen[kEndBlock]; }
            const int nb = nb0 + nb1;
            int incl = nb;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if (lane >= o) incl += t;
            }
            if (lane == 63) wsum2[par][wave] = (uint32_t)incl;
            __syncthreads();
            int wpre = 0, total = 0;
            for (int w = 0; w < kEncThreads / 64; w++) {
                if (w < wave) wpre += (int)wsum2[par][w];
                total += (int)wsum2[par][w];
            }
            const int excl = wpre + incl - nb;
            if (ob - sbase + total + 64 > kEmitStgBits) eflush(ob, false);
            if (nb0) stg_or(stg, ob - sbase + excl, v0);
            if (nb1) stg_or(stg, ob - sbase + excl + nb0, v1);
            ob += total;
            par ^= 1;
        }
        __syncthreads();                                   // every symbol placed before the trailer / flush
        if (tid == 0) s_obit = ob;
        __syncthreads();
    }
    if (last) {
        if (s_obit - sbase + 160 > kEmitStgBits) eflush(s_obit, false);
        if (tid == 0) {
            s_obit = (s_obit + 7) & ~7ll;                  // bi_windup
            const uint32_t ck = job.check[bi];
            if (job.wrap == 1) {                           // Adler-32, big-endian (deflate.c:1253-1256)
                put(ck >> 24, 8); put((ck >> 16) & 0xffu, 8); put((ck >> 8) & 0xffu, 8); put(ck & 0xffu, 8);
            } else if (job.wrap == 2) {                    // CRC-32 + ISIZE, little-endian
                put(ck, 32);
                put((uint32_t)job.src_len[g], 32);
            }
        }
        __syncthreads();
    }
    // the bits written must be the bits k_enc_scan placed (block_plan's
    // opt_len / static_len): a difference would overlap or gap the
    // neighbouring blocks, so it is reported as an error, never as bytes
    if (tid == 0 && s_obit != re + sh) job.status[g] = -2;
    eflush(s_obit, true);
}

// a streaming job's records from the block encoder (k_encode's stream_rec):
// srec[4k] the output bit after block k, srec[4k + 1] the partial byte there
// and bi_used << 8; flush_out[1] / [3] the end bit and its partial byte.  One
// thread per block, after k_enc_emit has written every byte.
__global__ __launch_bounds__(256) void k_enc_rec(DeflateJob job) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    const uint32_t nblk = job.nblocks[0];
    if (k >= nblk || !enc_blocks_ok(job, 0, nblk)) return;
    const uint32_t g = job.first;
    const EncPlan *pl = job.eplan + job.blk_off[0];
    const uint8_t *out = job.dst + job.dst_off[g];
    const uint64_t cap = job.dst_cap[g];
    const uint64_t e = pl[k + 1].start;
    const uint32_t part = (e & 7) && (e >> 3) < cap ? out[e >> 3] & ((1u << (e & 7)) - 1u) : 0u;
    job.srec[4ull * k] = e;
    job.srec[4ull * k + 1] = part | (uint64_t)pl[k].pad0 << 8;
    if (k + 1 == nblk && job.flush_out) {
        job.flush_out[1] = e;
        job.flush_out[3] = part;
    }
}

// ------------------------------------------------------------------------
// host-side launch
// ------------------------------------------------------------------------
int launch_tables_upload(const CodeTables *ct, const CrcTables *) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(c_ct), ct, sizeof(CodeTables));
}

// ------------------------------------------------------------------------
// The sorted runs (round 5): k_bsort, k_bwork<true> for k_parse_srt (levels
// 2..3 of few buffers, hash_bits <= 15).  (Round 5 also walked levels 4..9
// from them, k_match2: 2x slower than k_match, removed in round 6.)
//
// longest_match's candidates for position p are the earlier positions with
// p's hash, most recent first, while they lie within MAX_DIST (deflate.c
// :1356-1497 over the prev[] chain).  k_match walks that
// chain link by link: every step is a dependent LDS round trip, and the walk is
// bound by their latency.  Here the chain is not followed but
// read: each block of kSortBlock positions is sorted by (hash, position)
// (k_bsort), so a position's candidates are the entries just before its own in
// its block, then its hash's run in the block before, then in the one before
// that -- three contiguous runs whose bounds are known up front (k_bwork).
// Every candidate's address is then a function of its rank alone, so a lane's
// next candidates can be loaded before the current one is tested.
// ------------------------------------------------------------------------
constexpr int kBSThreads = 1024;
constexpr int kBSWaves = kBSThreads / 64;
constexpr int kBSPer = kSortBlock / kBSThreads;     // keys per thread (16)
constexpr int kBSlice = 4096;                       // k_bwork's count-sorted slices
static_assert(kSortBlock == 16384, "positions are 14-bit block-relative in the sort keys");

// the sub-batch buffer a flat block belongs to: the last bi with bblk[bi] <= g
__device__ inline uint32_t block_buffer(const uint32_t *bblk, uint32_t count, uint32_t g) {
    uint32_t lo = 0, hi = count - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (bblk[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// One stable counting-sort pass (8-bit digit at `shift`) of src[0..m) into dst:
// wave w owns elements w*1024 + j*64 + lane; equal digits within a wave step
// are ranked with ballots, counts scanned digit-major across the 16 waves.
__device__ __attribute__((always_inline)) inline void bs_radix_pass(const uint32_t *src, uint32_t *dst, int m,
                                                                    int shift, uint16_t (*wcnt)[256], int *wsum,
                                                                    int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int k = tid; k < kBSWaves * 256; k += kBSThreads) (&wcnt[0][0])[k] = 0;
    __syncthreads();
    uint32_t key[kBSPer], rank[kBSPer];
#pragma unroll
    for (int j = 0; j < kBSPer; j++) {
        const int e = wave * (64 * kBSPer) + j * 64 + lane;
        const bool valid = e < m;
        key[j] = valid ? src[e] : 0u;
        const uint32_t d = (key[j] >> shift) & 0xffu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bb : ~bb;
        }
        rank[j] = 0;
        if (valid) {
            const uint32_t base = wcnt[wave][d];
            rank[j] = base + (uint32_t)__popcll(peers & below);
            if ((peers & below) == 0) wcnt[wave][d] = (uint16_t)(base + __popcll(peers));
        }
    }
    __syncthreads();
    int v[4], tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int idx = tid * 4 + k;
        v[k] = wcnt[idx & (kBSWaves - 1)][idx >> 4];
        tot += v[k];
    }
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wave; w++) wbase += wsum[w];
    int run = wbase + incl - tot;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int idx = tid * 4 + k;
        wcnt[idx & (kBSWaves - 1)][idx >> 4] = (uint16_t)run;
        run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kBSPer; j++) {
        const int e = wave * (64 * kBSPer) + j * 64 + lane;
        if (e < m) dst[wcnt[wave][(key[j] >> shift) & 0xffu] + rank[j]] = key[j];
    }
    __syncthreads();
}

// k_bsort — one workgroup per block: its inserted positions (p <= n-3,
// INSERT_STRING needs MIN_MATCH bytes of lookahead) sorted by (hash, position)
// into srt, and the block's hash table off[0 .. hash_size] into boff.
__global__ __launch_bounds__(kBSThreads) void k_bsort(DeflateJob job) {
    __shared__ uint32_t ka[kSortBlock], kb[kSortBlock];
    __shared__ __attribute__((aligned(16))) uint8_t by[kSortBlock + 16];
    __shared__ uint16_t wcnt[kBSWaves][256];
    __shared__ int wsum[kBSWaves];
    const int tid = threadIdx.x;
    const uint32_t g = blockIdx.x;
    const uint32_t bi = block_buffer(job.bblk, job.count, g);
    const int64_t p0 = (int64_t)(g - job.bblk[bi]) * kSortBlock;
    const int64_t n = (int64_t)job.src_len[job.first + bi];
    const uint8_t *in = job.src + job.src_off[job.first + bi];
    const WinP wp = job_win(job);
    const int hsize = (int)wp.mask + 1;
    stage_bytes<kBSThreads, (kSortBlock + 16) / 16 / kBSThreads + 1>(by, in, p0, kSortBlock + 16, n, tid);
    __syncthreads();
    const int m = (int)(n - 2 - p0 <= 0 ? 0 : (n - 2 - p0 < kSortBlock ? n - 2 - p0 : kSortBlock));
    for (int e = tid; e < m; e += kBSThreads) ka[e] = hashp(by[e], by[e + 1], by[e + 2], wp) << 14 | (uint32_t)e;
    bs_radix_pass(ka, kb, m, 14, wcnt, wsum, tid);
    bs_radix_pass(kb, ka, m, 22, wcnt, wsum, tid);
    uint16_t *S = job.srt + job.ws_off[bi] + p0;
    for (int i = tid; i < m; i += kBSThreads) S[i] = (uint16_t)(ka[i] & (kSortBlock - 1));
    // off[h] = entries with a hash below h: a run's start is marked at its
    // hash, then a suffix minimum fills the hashes without entries
    uint16_t *off = reinterpret_cast<uint16_t *>(kb);
    for (int h = tid; h < hsize; h += kBSThreads) off[h] = 0xffffu;
    __syncthreads();
    for (int i = tid; i < m; i += kBSThreads) {
        const uint32_t h = ka[i] >> 14;
        if (i == 0 || (ka[i - 1] >> 14) != h) off[h] = (uint16_t)i;
    }
    __syncthreads();
    const int per = (hsize + kBSThreads - 1) / kBSThreads;      // hashes per thread (32 at hash_bits 15)
    const int h0 = tid * per, h1 = min(h0 + per, hsize);
    uint32_t smin = 0xffffu;
    for (int h = h0; h < h1; h++) smin = min(smin, (uint32_t)off[h]);
    // suffix minimum of the threads' minima: over the wave, then over the waves
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t suf = smin;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_down((int)suf, o, 64);
        if (lane + o < 64) suf = min(suf, t);
    }
    if (lane == 0) wsum[wave] = (int)suf;
    __syncthreads();
    uint32_t carry = (uint32_t)m;                                // past the last run: every entry is below
    for (int w = wave + 1; w < kBSWaves; w++) carry = min(carry, (uint32_t)wsum[w]);
    {
        const uint32_t nxt = (uint32_t)__shfl_down((int)suf, 1, 64);   // minimum of the later lanes of this wave
        if (lane < 63) carry = min(carry, nxt);
    }
    uint16_t *go = job.boff + (size_t)g * kSortOffStride;
    for (int h = h1 - 1; h >= h0; h--) {
        carry = min(carry, (uint32_t)off[h]);
        go[h] = (uint16_t)carry;
    }
    if (tid == 0) go[hsize] = (uint16_t)m;
}

// k_bwork — one workgroup per block: a work item per sorted entry i of the
// block (position rel, hash h): its own run's candidates (the n0 entries
// before i), and h's runs in the two blocks before (end e1 / e2, length
// n1 / n2).  Each 4096-entry slice is counting-sorted by the candidate count
// (capped at the chain budget; k_count's key), longest first, so the 64
// walks of a wave have similar lengths (tools/model/model_sortwalk.c: 98.6 %
// SIMT utilisation at L6 against 78 % in plain sorted order).
// kPos (levels 1..3, k_parse_srt): the items are stored by position
// instead (work[rel] for the block's position rel; no count sort), for the
// sequential parse to read in position order.
template <bool kPos>
__global__ __launch_bounds__(kBSThreads) void k_bwork(DeflateJob job) {
    __shared__ uint16_t S[kSortBlock];
    __shared__ uint16_t off[kSortOffStride];
    __shared__ __attribute__((aligned(16))) uint8_t by[kSortBlock + 16];
    __shared__ int s_hist[kSortBlock / kBSlice][64], s_base[kSortBlock / kBSlice][64];
    const int tid = threadIdx.x;
    const uint32_t g = blockIdx.x;
    const uint32_t bi = block_buffer(job.bblk, job.count, g);
    const uint32_t b = g - job.bblk[bi];
    const int64_t p0 = (int64_t)b * kSortBlock;
    const int64_t n = (int64_t)job.src_len[job.first + bi];
    const uint8_t *in = job.src + job.src_off[job.first + bi];
    const WinP wp = job_win(job);
    const int hsize = (int)wp.mask + 1;
    const int m = (int)(n - 2 - p0 <= 0 ? 0 : (n - 2 - p0 < kSortBlock ? n - 2 - p0 : kSortBlock));
    const uint16_t *gS = job.srt + job.ws_off[bi] + p0;
    const uint16_t *gO = job.boff + (size_t)g * kSortOffStride;
    for (int i = tid; i < m; i += kBSThreads) S[i] = gS[i];
    for (int h = tid; h <= hsize; h += kBSThreads) off[h] = gO[h];
    stage_bytes<kBSThreads, (kSortBlock + 16) / 16 / kBSThreads + 1>(by, in, p0, kSortBlock + 16, n, tid);
    if (tid < (kSortBlock / kBSlice) * 64) (&s_hist[0][0])[tid] = 0;
    __syncthreads();
    const uint16_t *o1 = b >= 1 ? job.boff + (size_t)(g - 1) * kSortOffStride : nullptr;
    const uint16_t *o2 = b >= 2 ? job.boff + (size_t)(g - 2) * kSortOffStride : nullptr;
    const uint32_t chain = job.cfg.chain;
    uint4 it[kBSPer];
    int bk[kBSPer], rk[kBSPer];
#pragma unroll
    for (int u = 0; u < kBSPer; u++) {
        const int i = tid + u * kBSThreads;
        rk[u] = 0;
        bk[u] = 0;
        it[u] = make_uint4(0, 0, 0, 0);
        if (i >= m) continue;
        const uint32_t rel = S[i];
        const uint32_t h = hashp(by[rel], by[rel + 1], by[rel + 2], wp);
        const uint32_t n0 = (uint32_t)i - off[h];
        const uint32_t s1 = o1 ? o1[h] : 0u, e1 = o1 ? o1[h + 1] : 0u;
        const uint32_t s2 = o2 ? o2[h] : 0u, e2 = o2 ? o2[h + 1] : 0u;
        it[u] = make_uint4((uint32_t)i | rel << 16, n0 | (e1 - s1) << 16, e1 | e2 << 16, e2 - s2);
        if (kPos) {
            job.work[job.ws_off[bi] + p0 + rel] = it[u];
            continue;
        }
        const uint32_t c = n0 + (e1 - s1) + (e2 - s2);
        bk[u] = 63 - (int)(walk_key(c, chain) >> 2);
    }
    if (kPos) return;
#pragma unroll
    for (int u = 0; u < kBSPer; u++)
        if (tid + u * kBSThreads < m) rk[u] = atomicAdd(&s_hist[u / (kBSlice / kBSThreads)][bk[u]], 1);
    __syncthreads();
    if (tid < (kSortBlock / kBSlice) * 64) {                  // exclusive scan per slice
        const int sl = tid >> 6, l = tid & 63;
        const int v = s_hist[sl][l];
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (l >= o) incl += t;
        }
        s_base[sl][l] = incl - v;
    }
    __syncthreads();
    uint4 *W = job.work + job.ws_off[bi] + p0;
#pragma unroll
    for (int u = 0; u < kBSPer; u++) {
        const int sl = u / (kBSlice / kBSThreads);
        if (tid + u * kBSThreads < m) W[sl * kBSlice + s_base[sl][bk[u]] + rk[u]] = it[u];
    }
}

// The rings of k_parse_srt (levels 2..3 from the sorted runs): the sorted
// entries and bytes of three blocks.  (k_match2, the sorted-run walk of levels
// 4..9, measured 2x slower than k_match and left the library in round 6;
// DESIGN 4.14.)
constexpr int kM2Pad = 304;                       // bytes past block b: compares read <= 258 + 16 + 3 past a position
constexpr int kM2Ring = 3 * kSortBlock;

// 4 bytes at any offset of the byte ring
__device__ __attribute__((always_inline)) inline uint32_t b4(const uint8_t *B, int q) {
#ifdef ZGPU_LDS_UNALIGNED
    uint32_t x;
    asm volatile("ds_read_b32 %0, %1" : "=v"(x) : "v"((uint32_t)(uintptr_t)(B + q)));
    return x;
#else
    return lds32u(B, q);
#endif
}
// 16 bytes at any offset: 5 aligned dwords, 4 byte-aligns
__device__ __attribute__((always_inline)) inline void b16(const uint8_t *B, int q, uint32_t &x0, uint32_t &x1,
                                                          uint32_t &x2, uint32_t &x3) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(B + (q & ~3));
    const uint32_t sh = (uint32_t)(q & 3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    x0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
    x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    x2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
    x3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
}
// ------------------------------------------------------------------------
// k_parse_srt — deflate_fast (levels 1..3, deflate.c:1824-1915) of a batch
// job from the sorted runs (k_bsort, k_bwork<true>).  One wave per buffer,
// the CU's LDS holding the sorted entries and bytes of the blocks b-2..b of
// the parse position and a bitmap of the positions deflate_fast
// has inserted (blocks b-2..b+1).
//
// deflate_fast searches the chain of INSERTED positions: a position strictly
// inside a match longer than max_insert_length is not inserted (:1873-1897).
// That chain is the sorted run of p's hash, most recent first, without the
// positions whose bit is clear (exact).  So a decision
// reads up to 64 candidates at once -- lane k takes the k-th same-hash
// position before p -- tests their bits, takes the first `chain` inserted ones
// above the limit (the head at exactly MAX_DIST included, deflate.c:1853) and
// compares them side by side; the first reaching nice, else the first
// longest, is longest_match's result (:1417-1497).  No link is chased and no
// head[] / prev[] is kept: the run info of the next 64 positions is loaded
// ahead, and every other access is to LDS.
// ------------------------------------------------------------------------
constexpr int kPSBits = 4 * kSortBlock / 32;        // bitmap words: blocks b-2 .. b+1

// kG (batches of many buffers): the sorted entries and the bytes are read
// from global memory (L2) instead of LDS rings, so that a wave needs only its
// 8 KiB bitmap and 20 parses share a CU instead of one.
template <typename P, bool kG = false>
__global__ __launch_bounds__(64) void k_parse_srt(DeflateJob job) {
    __shared__ __attribute__((aligned(16))) uint16_t Sr[kG ? 8 : kM2Ring];
    __shared__ __attribute__((aligned(16))) uint8_t Bw[kG ? 16 : kM2Ring + kM2Pad];
    __shared__ uint32_t Bi[kPSBits];
    const int lane = threadIdx.x;
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t bi = blockIdx.x;
    const uint32_t g = job.first + bi;
    const P n = (P)job.src_len[g];
    const uint8_t *in = job.src + job.src_off[g];
    const uint16_t *gS = job.srt + job.ws_off[bi];
    const uint4 *gW = job.work + job.ws_off[bi];
    const WinP wp = job_win(job);
    const LevelCfg cfg = job.cfg;
    ParseOutT<P> po;
    po.sym = job.sym + job.ws_off[bi];
    po.blk = job.blocks + job.blk_off[bi];
    po.nsym = po.blk_nsym = po.blk_sym_start = po.nblk = 0;
    po.win(wp);
    po.block_start = 0; po.S = 0; po.E = 0;
    po.lead = true;
    po.vaddr = true;
    const P max_dist = (P)wp.max_dist;
    auto mcount = [&](P b) -> int {
        const P r = n - 2 - b * kSortBlock;
        return r <= 0 ? 0 : (r < kSortBlock ? (int)r : kSortBlock);
    };
    auto ld16 = [&](P x) -> uint4 {                     // 16 input bytes from x, zero outside [0, n)
        if (x >= 0 && x + 16 <= n) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(in + x);
            const uint32_t sh = (uint32_t)(a & 3u);
            const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
            if (sh == 0) return make_uint4(q[0], q[1], q[2], q[3]);
            const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
            return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                              __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
        }
        uint32_t w[4] = {0, 0, 0, 0};
        for (int j = 0; j < 16; j++)
            if (x + j >= 0 && x + j < n) w[j >> 2] |= (uint32_t)in[x + j] << (8 * (j & 3));
        return make_uint4(w[0], w[1], w[2], w[3]);
    };
    P blk = 0;                                          // the block in ring slot 2
    P gbase = -2 * (P)kSortBlock;                       // absolute position of ring offset 0 (kG)
    // ring accessors: LDS, or (kG) the same offsets mapped to global memory
    auto sr = [&](int idx) -> uint32_t {                // ring entry idx (slot idx >> 14)
        if (!kG) return Sr[idx];
        const P b = blk - 2 + (idx >> 14);
        return (uint32_t)(idx & ~(kSortBlock - 1)) + (uint32_t)gS[b * kSortBlock + (idx & (kSortBlock - 1))];
    };
    auto bw = [&](int x) -> uint32_t {                  // ring byte x
        if (!kG) return Bw[x];
        const P a = gbase + x;
        return a < n ? (uint32_t)in[a] : 0u;
    };
    auto b16r = [&](int x, uint32_t &a0, uint32_t &a1, uint32_t &a2, uint32_t &a3) {
        if (!kG) { b16(Bw, x, a0, a1, a2, a3); return; }
        const uint4 v = ld16(gbase + x);
        a0 = v.x; a1 = v.y; a2 = v.z; a3 = v.w;
    };
    auto cand = [&](uint32_t k, int A0, int B1, int B2, uint32_t n0, uint32_t n01, uint32_t n012) -> int {
        const int idx = k < n0 ? A0 - (int)k : (k < n01 ? B1 - (int)k : B2 - (int)k);
        int q = -1;
        if (k < n012) q = (int)sr(idx);                 // only real entries are read (kG: global memory)
        return q;
    };
    // block b into ring slot 2 (entries as ring offsets), its bytes + pad, and
    // its bitmap slot b+1 (slot 3) cleared; slide first unless b == 0
    auto load_block = [&](P b) {
        gbase = (b - 2) * (P)kSortBlock;
        if (kG) {                                       // only the bitmap lives in LDS
            if (b > 0)
                for (int c = lane; c < 3 * kSortBlock / 32; c += 64) Bi[c] = Bi[c + kSortBlock / 32];
            else
                for (int c = lane; c < kPSBits; c += 64) Bi[c] = 0;
            for (int c = lane; c < kSortBlock / 32; c += 64) Bi[3 * kSortBlock / 32 + c] = 0;
            __syncthreads();
            return;
        }
        if (b > 0) {
            uint4 *dS = reinterpret_cast<uint4 *>(Sr);
            typedef unsigned short us2 __attribute__((ext_vector_type(2)));
            auto sub = [](uint32_t x) {
                const us2 d = {(unsigned short)kSortBlock, (unsigned short)kSortBlock};
                return __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, x) - d);
            };
            for (int c = lane; c < 2 * kSortBlock / 8; c += 64) {
                const uint4 v = dS[c + kSortBlock / 8];
                dS[c] = make_uint4(sub(v.x), sub(v.y), sub(v.z), sub(v.w));
            }
            uint4 *dB = reinterpret_cast<uint4 *>(Bw);
            for (int c = lane; c < 2 * kSortBlock / 16; c += 64) dB[c] = dB[c + kSortBlock / 16];
            for (int c = lane; c < 3 * kSortBlock / 32; c += 64) Bi[c] = Bi[c + kSortBlock / 32];
        } else {
            for (int c = lane; c < kPSBits; c += 64) Bi[c] = 0;
        }
        for (int c = lane; c < kSortBlock / 32; c += 64) Bi[3 * kSortBlock / 32 + c] = 0;
        const int m = mcount(b);
        const uint16_t *src = gS + b * kSortBlock;
        for (int e = 8 * lane; e < kSortBlock; e += 512) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (e + 8 <= m) v = *reinterpret_cast<const uint4 *>(src + e);
            else if (e < m) {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int j = 0; j < 8 && e + j < m; j++) w[j >> 1] |= (uint32_t)src[e + j] << (16 * (j & 1));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            const uint32_t o = 2u * kSortBlock * 0x10001u;
            *reinterpret_cast<uint4 *>(Sr + 2 * kSortBlock + e) = make_uint4(v.x + o, v.y + o, v.z + o, v.w + o);
        }
        const P p0 = b * kSortBlock;
        for (int c = lane; c < (kSortBlock + kM2Pad) / 16; c += 64)
            *reinterpret_cast<uint4 *>(Bw + 2 * kSortBlock + 16 * c) = ld16(p0 + 16 * c);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    };
    // run info of positions [rb, rb + 64) in lanes (cur), the next 64 (nxt)
    P rb = 0;
    uint4 cur = make_uint4(0, 0, 0, 0), nxt = cur;
    auto ri_load = [&](P x) -> uint4 { return x + lane < n ? gW[x + lane] : make_uint4(0, 0, 0, 0); };
    if (n > 0) {
        load_block(0);
        cur = ri_load(0);
        nxt = ri_load(64);
    }
    const P nblk = (n + kSortBlock - 1) / kSortBlock;
    P p = 0;
    uint32_t match_length = kMinMatch - 1;
    const P lim = n;
    while (p < n) {
        if (po.E - p < kMinLookahead) {
            po.fill(p, lim);
        }
        while (p >= (blk + 1) * kSortBlock && blk + 1 < nblk) load_block(++blk);
        if (p >= rb + 64) {
            if (p < rb + 128) { cur = nxt; rb += 64; }
            else { rb = p & ~(P)63; cur = ri_load(rb); }
            nxt = ri_load(rb + 64);
        }
        const P base = blk * kSortBlock - 2 * kSortBlock;   // absolute position of ring offset 0
        const P lookahead = po.E - p;
        const int vp = (int)(p - base);
        uint32_t best = kMinMatch - 1, bq = 0;
        bool searched = false;                          // longest_match ran (a head within MAX_DIST)
        if (lookahead >= kMinMatch) {
            // INSERT_STRING(p): its bit goes in after the search (p is no candidate of itself)
            const int o = (int)(p - rb);
            const uint32_t ix = (uint32_t)__builtin_amdgcn_readlane((int)cur.x, o);
            const uint32_t iy = (uint32_t)__builtin_amdgcn_readlane((int)cur.y, o);
            const uint32_t iz = (uint32_t)__builtin_amdgcn_readlane((int)cur.z, o);
            const uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)cur.w, o);
            const int i = (int)(ix & 0xffffu);
            const uint32_t n0 = iy & 0xffffu, n01 = n0 + (iy >> 16), n012 = n01 + n2;
            const int A0 = 2 * kSortBlock + i - 1, B1 = kSortBlock + (int)(iz & 0xffffu) - 1 + (int)n0,
                      B2 = (int)(iz >> 16) - 1 + (int)n01;
            const P limit = (p - po.S) > max_dist ? p - max_dist : po.S;
            const int lim = (int)(limit - base);
            const int nice = lookahead < (P)cfg.nice ? (int)lookahead : (int)cfg.nice;
            const P rem = n - p;
            const int maxcmp = rem < kMaxMatch ? (int)rem : kMaxMatch;
            uint32_t chain = cfg.chain;                   // prev_length == 2 < good: no quartering
            bool head = false, done = n012 == 0;
            for (uint32_t k0 = 0; !done; k0 += 64) {
                const uint32_t k = k0 + (uint32_t)lane;
                const int q = cand(k, A0, B1, B2, n0, n01, n012);
                const bool valid = k < n012;
                const bool ins = valid && ((Bi[(uint32_t)q >> 5] >> ((uint32_t)q & 31u)) & 1u);
                const uint64_t insm = __ballot(ins);
                uint64_t elig;
                int hl = -1;
                if (!head) {
                    if (insm == 0) {                      // no inserted candidate in these 64
                        if (k0 + 64 >= n012) break;
                        continue;
                    }
                    // the head (hash_head): within the window and MAX_DIST, else no search
                    hl = __builtin_ctzll(insm);
                    const int hq = __builtin_amdgcn_readlane(q, hl);
                    const P hqa = base + hq;
                    if (!(hqa > po.S && p - hqa <= max_dist)) break;
                    head = true;
                    searched = true;
                }
                // after the head, the chain visits inserted candidates while they
                // lie above the limit (positions only go down from lane to lane),
                // `chain` of them at most
                elig = __ballot(ins && (lane == hl || q > lim));
                const uint64_t stopm = __ballot(ins && lane != hl && q <= lim);
                const uint64_t vis = elig;
                const uint32_t pre = (uint32_t)__popcll(vis & below);
                const bool mine = ((vis >> lane) & 1ull) && pre < chain;
                const uint32_t nv = (uint32_t)min((uint64_t)chain, (uint64_t)__popcll(vis));
                int len = 0;
                if (mine) {
                    uint32_t a0, a1, a2, a3, c0, c1, c2, c3;
                    b16r(q, a0, a1, a2, a3);
                    b16r(vp, c0, c1, c2, c3);
                    len = diff16(a0 ^ c0, a1 ^ c1, a2 ^ c2, a3 ^ c3);
                    while (len >= 16 && len < nice) {
                        b16r(q + len, a0, a1, a2, a3);
                        b16r(vp + len, c0, c1, c2, c3);
                        const int r = diff16(a0 ^ c0, a1 ^ c1, a2 ^ c2, a3 ^ c3);
                        len += r;
                        if (r < 16) break;
                    }
                    len = len < nice ? len : nice;
                }
                // the first to reach nice, else the first longest (strictly longer wins)
                const uint64_t nm = __ballot(mine && len >= nice);
                int wl = -1, wlen = 0;
                if (nm) {
                    wl = __builtin_ctzll(nm);
                    wlen = nice;
                } else {
                    uint32_t key = mine ? ((uint32_t)len << 8) | (uint32_t)(63 - lane) : 0u;
#pragma unroll
                    for (int sh = 1; sh < 64; sh <<= 1) key = max(key, (uint32_t)__shfl_xor((int)key, sh, 64));
                    key = ufl(key);
                    if ((key >> 8) > best) { wl = 63 - (int)(key & 0xffu); wlen = (int)(key >> 8); }
                }
                if (wl >= 0 && (uint32_t)wlen > best) {
                    best = (uint32_t)wlen;
                    bq = (uint32_t)__builtin_amdgcn_readlane(q, wl);
                }
                chain -= nv;
                done = nm != 0 || chain == 0 || stopm != 0 || k0 + 64 >= n012;
            }
            if (best >= (uint32_t)nice && best >= kMinMatch) {
                // the winner's true length, past nice up to maxcmp (64 bytes a round)
                int L = (int)best;
                while (L < maxcmp) {
                    const int kk = L + lane;
                    const int kc = kk < maxcmp ? kk : maxcmp - 1;
                    const uint64_t mm = __ballot((kk < maxcmp) & (bw((int)bq + kc) != bw(vp + kc)));
                    if (mm) { L += __builtin_ctzll(mm); break; }
                    L += 64;
                    if (L > maxcmp) L = maxcmp;
                }
                best = (uint32_t)(L < maxcmp ? L : maxcmp);
            }
            if (lane == 0) atomicOr(&Bi[(uint32_t)vp >> 5], 1u << ((uint32_t)vp & 31u));
        }
        // s->match_length: the search's result, else what the last decision left
        if (searched) match_length = best <= (uint32_t)lookahead ? best : (uint32_t)lookahead;
        bool bflush;
        if (searched && match_length >= kMinMatch) {
            bflush = po.tally(((uint32_t)(vp - (int)bq) << 8) | (match_length - kMinMatch));
            const P la = lookahead - (P)match_length;
            if (match_length <= cfg.lazy && la >= kMinMatch) {
                // the strings inside a short match are inserted (deflate.c:1873-1884)
                const uint32_t v = (uint32_t)vp + (uint32_t)lane + 1u;
                if ((uint32_t)lane < match_length - 1u) atomicOr(&Bi[v >> 5], 1u << (v & 31u));
            }
            p += match_length;
            match_length = 0;
        } else {
            bflush = po.tally(bw(vp));
            p++;
        }
        if (bflush) po.flush(p, false);
    }
    po.flush(p, true);
    if (lane == 0) job.nblocks[bi] = po.nblk;
}

static bool fb_bigtile() {
    static const bool v = [] { const char *e = getenv("ZGPU_FB_BIGTILE"); return e && e[0] == '1'; }();
    return v;
}

int launch_deflate_stage(int stage, const DeflateJob &job, uint32_t *heads, hipStream_t st) {
    const dim3 grid(job.count);
    switch (stage) {
    case 0:
        if (job.seg && !job.lk_head) {                          // few large buffers: per segment
            const dim3 sgrid(job.nseg);
            static const bool ls1 = [] { const char *e = getenv("ZGPU_LINKS_SEG1"); return !e || e[0] != '0'; }();
            if (job.hbits > 15) hipLaunchKernelGGL((k_links<2048, 65536, true>), sgrid, dim3(kLThreads), 0, st, job);
            else if (ls1 && (int64_t)job.seg_len <= kLS1Max)
                hipLaunchKernelGGL(k_links_seg1, sgrid, dim3(kLThreads), 0, st, job);
            else hipLaunchKernelGGL((k_links<kLC, 32768, true>), sgrid, dim3(kLThreads), 0, st, job);
            hipLaunchKernelGGL(k_count<true>, sgrid, dim3(kCntThreads), 0, st, job);
            break;
        }
        if (job.hbits > 15) hipLaunchKernelGGL((k_links<2048, 65536>), grid, dim3(kLThreads), 0, st, job);
        else if (job.links_gh && !job.lk_head) hipLaunchKernelGGL(k_links_gh, grid, dim3(kLThreads), 0, st, job);
        else hipLaunchKernelGGL((k_links<kLC, 32768>), grid, dim3(kLThreads), 0, st, job);
        hipLaunchKernelGGL(k_count<false>, grid, dim3(kCntThreads), 0, st, job);
        break;
    case 1: {
        const int wq = (int)(job.cfg.good < job.cfg.lazy) | job.cfg_q;   // the parse reads rquart (prev_length >= good)
        const dim3 mgrid(job.seg ? job.nseg : job.count);   // per segment or per buffer
        const bool ev = job.nfl || job.ncfg;                // a streaming job (zgpu_api.cpp deflate())
        if (ev && job.seg)
            hipLaunchKernelGGL((k_match<true, true>), mgrid, dim3(kMatchThreads), 0, st, job, wq);
        else if (ev)
            hipLaunchKernelGGL((k_match<true, false>), mgrid, dim3(kMatchThreads), 0, st, job, wq);
        else if (job.seg)                                       // few large buffers: per segment
            hipLaunchKernelGGL((k_match<false, true>), mgrid, dim3(kMatchThreads), 0, st, job, wq);
        else
            hipLaunchKernelGGL((k_match<false, false>), mgrid, dim3(kMatchThreads), 0, st, job, wq);
        break;
    }
    case 2: hipLaunchKernelGGL(k_parse_slow<kPT>, grid, dim3(64), 0, st, job, 0); break;
    case 5: hipLaunchKernelGGL(k_parse_seg, grid, dim3(kParseLanes), 0, st, job); break;
    case 6:                                     // ZGPU_FB_BIGTILE=1 (A/B): the 36 KiB tile here too
        // few buffers (no pipeline; a flagged buffer may be 16 MiB or more, where
        // 256-position tiles would reload 20x as often): the 36 KiB tile
        if (fb_bigtile() || job.count < 512) hipLaunchKernelGGL(k_parse_slow<kPT>, grid, dim3(64), 0, st, job, 1);
        else hipLaunchKernelGGL(k_parse_slow<256>, grid, dim3(64), 0, st, job, 1);
        break;
    case 3: {
        const bool ev = job.nfl || job.start || job.srec;
        // few buffers (a lone compress2 at L1-3): head / prev / window in LDS, one wave per CU
        static const uint32_t lds_max = [] {
            const char *e = std::getenv("ZGPU_FAST_LDS_MAX");     // A/B: 0 turns the variant off
            return e ? (uint32_t)std::atoi(e) : 256u;
        }();
        if (ev) hipLaunchKernelGGL((k_parse_fast<true, true, int64_t>), grid, dim3(64), 0, st, job, heads);
        else if (job.count <= lds_max && job.hbits <= 15 && job.pos31)
            hipLaunchKernelGGL((k_parse_fast<false, true, int32_t, true>), grid, dim3(64), 0, st, job, heads);
        else if (job.count <= lds_max && job.hbits <= 15)
            hipLaunchKernelGGL((k_parse_fast<false, true, int64_t, true>), grid, dim3(64), 0, st, job, heads);
        else if (job.pos31) hipLaunchKernelGGL((k_parse_fast<false, true, int32_t>), grid, dim3(64), 0, st, job, heads);
        else hipLaunchKernelGGL((k_parse_fast<false, true, int64_t>), grid, dim3(64), 0, st, job, heads);
        break;
    }
    case 4: {
        // Tree build: the whole wave (w_build) for launches of few buffers, where one block's build is the
        // kernel's latency; one lane (t_build) for large batches, where the other resident waves hide it
        // and t_build's fewer registers and instructions win. ZGPU_ENCODE_VARIANT=1 / 2 forces lane / wave.
        static const int ev = [] { const char *e = getenv("ZGPU_ENCODE_VARIANT"); return e ? atoi(e) : 0; }();
        const bool lane_build = ev == 1 || (ev != 2 && grid.x >= kEncWaveBuildMax);
        if (lane_build) hipLaunchKernelGGL(k_encode<false>, grid, dim3(kEncThreads), 0, st, job);
        else hipLaunchKernelGGL(k_encode<true>, grid, dim3(kEncThreads), 0, st, job);
        break;
    }
    case 11: {
        const dim3 pg(job.npgrp), bg((job.maxblk + 255) / 256, job.count);
        // 256-byte segments: pass 1 from LDS copies (k_pbig1s stages exactly this segment size)
        const bool staged = job.preach == kSmallReach && job.pseg == kSmallSeg;
        const dim3 sgq(job.npgrp * (kParseLanes / kP1sLanes));
        if (staged) hipLaunchKernelGGL(k_pbig1s, sgq, dim3(kP1sLanes), 0, st, job);
        else hipLaunchKernelGGL(k_pbig1, pg, dim3(kParseLanes), 0, st, job);
        hipLaunchKernelGGL(k_pbig2, pg, dim3(kParseLanes), 0, st, job);
        hipLaunchKernelGGL(k_pbig3, pg, dim3(kParseLanes), 0, st, job);
        hipLaunchKernelGGL(k_pbig4, grid, dim3(kPScanThreads), 0, st, job);
        hipLaunchKernelGGL(k_pbig5, pg, dim3(kP5Threads), 0, st, job);
        hipLaunchKernelGGL(k_pbig6, bg, dim3(256), 0, st, job);
        break;
    }
    case 13: {                                              // a streaming job: k_pbig1..5, k_pbig6s
        const dim3 pg(job.npgrp);
        hipLaunchKernelGGL(k_pbig1, pg, dim3(kParseLanes), 0, st, job);
        hipLaunchKernelGGL(k_pbig2, pg, dim3(kParseLanes), 0, st, job);
        hipLaunchKernelGGL(k_pbig3, pg, dim3(kParseLanes), 0, st, job);
        hipLaunchKernelGGL(k_pbig4, grid, dim3(kPScanThreads), 0, st, job);
        hipLaunchKernelGGL(k_pbig5, pg, dim3(kP5Threads), 0, st, job);
        hipLaunchKernelGGL(k_pbig6s, dim3(1), dim3(256), 0, st, job);
        break;
    }
    case 12: {
        // trees on the whole wave while few blocks are in flight (latency), on
        // one lane when many are (the other waves hide it), as for k_encode
        const dim3 plg((job.maxblk + kEncGroup - 1) / kEncGroup, job.count), eg(job.maxblk, job.count);
        static const bool plan_lane = std::getenv("ZGPU_PLAN_LANE") != nullptr;   // A/B: one-lane trees always
        static const bool plan_one = std::getenv("ZGPU_PLAN_ONEWAVE") != nullptr;  // A/B: one wave per block
        const dim3 plg2((job.maxblk + kPlan2Pairs - 1) / kPlan2Pairs, job.count);
        if ((uint64_t)job.maxblk * job.count < 16384 && !plan_lane && !plan_one)
            hipLaunchKernelGGL(k_enc_plan2, plg2, dim3(kEncThreads), 0, st, job);
        else if ((uint64_t)job.maxblk * job.count < 16384 && !plan_lane)
            hipLaunchKernelGGL(k_enc_plan<true>, plg, dim3(kEncThreads), 0, st, job);
        else
            hipLaunchKernelGGL(k_enc_plan1, dim3(job.maxblk, job.count), dim3(64), 0, st, job);
        hipLaunchKernelGGL(k_enc_scan, grid, dim3(kEScanThreads), 0, st, job);
        hipLaunchKernelGGL(k_enc_emit, eg, dim3(kEncThreads), 0, st, job);
        if (job.srec) hipLaunchKernelGGL(k_enc_rec, dim3((job.maxblk + 255) / 256), dim3(256), 0, st, job);
        break;
    }
    case 14:                                                // the sorted-run match: sort, work items
        if (job.nsblk) {
            hipLaunchKernelGGL(k_bsort, dim3(job.nsblk), dim3(kBSThreads), 0, st, job);
            hipLaunchKernelGGL(k_bwork<true>, dim3(job.nsblk), dim3(kBSThreads), 0, st, job);
        }
        break;
    case 16:                                                // levels 1..3 from the sorted runs
        {
            // few buffers: rings in LDS (one parse per CU); many: the rings'
            // data from L2 and 20 parses per CU (ZGPU_SRT_LDS_MAX: the limit)
            static const uint32_t lds_max = [] {
                const char *e = std::getenv("ZGPU_SRT_LDS_MAX");
                return e ? (uint32_t)std::atoi(e) : 512u;
            }();
            const bool gl = job.count > lds_max;
            if (job.pos31 && gl) hipLaunchKernelGGL((k_parse_srt<int32_t, true>), grid, dim3(64), 0, st, job);
            else if (job.pos31) hipLaunchKernelGGL(k_parse_srt<int32_t>, grid, dim3(64), 0, st, job);
            else if (gl) hipLaunchKernelGGL((k_parse_srt<int64_t, true>), grid, dim3(64), 0, st, job);
            else hipLaunchKernelGGL(k_parse_srt<int64_t>, grid, dim3(64), 0, st, job);
        }
        break;
#ifdef ZGPU_LZP
    case 17: hipLaunchKernelGGL(k_lzp, grid, dim3(kZThreads), 0, st, job); break;   // match + lazy parse (k_lzp)
#endif
    case 7: hipLaunchKernelGGL(k_parse_huff, grid, dim3(kHuffThreads), 0, st, job); break;
    case 8: hipLaunchKernelGGL(k_parse_rle, grid, dim3(64), 0, st, job); break;
    case 9: hipLaunchKernelGGL(k_count<false>, grid, dim3(kCntThreads), 0, st, job); break;
    case 10: hipLaunchKernelGGL(k_parse_ev, grid, dim3(64), 0, st, job); break;
    default: return -1;
    }
    return (int)hipGetLastError();
}

}  // namespace zgpu
