// zgpu_checksum.hip — batched CRC-32 and Adler-32 for gfx950.
//
// G lanes per buffer (64, or 16 for batches of many buffers).  The buffer is
// viewed as left-padded with zeros to a multiple of 16*G bytes ("rows"); lane i
// owns the 16-byte chunk at 16*i of every row.  Zero padding in front leaves a zero-init CRC and the
// Adler sums unchanged, so no lane ever handles a ragged tail.
//
// CRC-32 (crc32.c:694-1010): the init value is folded in by XOR-ing ~init into
// the first four data bytes (for len >= 4 the register state after a message
// M from init s equals the zero-init state of M ^ s), so the whole buffer is a
// single linear (zero-init) CRC R and crc32(init, M) = ~R.  A chunk's CRC is
// 32 lookups in conflict-free 16-entry nibble tables in LDS; rows are combined
// per lane by Horner (advance by one row of zero bytes, 8 lookups), lanes by a
// log2(G)-level shuffle tree (advance by 16<<l bytes) — crc32_combine
// (crc32.c:1021) with the
// x^(8n) multipliers pre-tabulated.
//
// k_crc32s (the default; k_crc32 above is kept for A/B as ZGPU_CRC_NIBBLE=1)
// replaces the nibble lookups by slice-by-4 byte tables, replicated per lane
// group: 1 LDS lookup per byte instead of 2.5 (4.0 -> 4.35 TB/s on C2, where a
// plain 16-byte streaming read of the same 4 GiB reaches 6.0 TB/s).
//
// Adler-32 (adler32.c:61-125): per chunk the byte sum and the position-weighted
// sum via v_dot4_u32_u8; weights are distances to the (virtual) end of the
// buffer, so A = a0 + Σx and B = b0 + L*a0 + Σ (L-j+1) x_j with one modulo at the
// end.  Tiny buffers (len < 16, len == 1 paths of adler32.c; len < 4 for CRC)
// take the reference's scalar path in lane 0.
#include "zgpu_internal.h"
#include <cstdlib>

namespace zgpu {

constexpr int kCkBlock = 256;                 // 4 waves per workgroup
constexpr uint32_t kAdlerBase = 65521u;

__device__ inline void load_chunk16(const uint8_t *buf, int64_t x, uint64_t L, uint32_t w[4]) {
    // bytes buf[x .. x+16), zero where x+j < 0; never reads outside [buf, buf+L)
    if (x >= 0) {
        const uint8_t *p = buf + x;
        uintptr_t a = reinterpret_cast<uintptr_t>(p);
        uint32_t sh = (uint32_t)(a & 3u);
        const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
        if (sh == 0) {
            if ((a & 15u) == 0) {
                uint4 v = *reinterpret_cast<const uint4 *>(p);
                w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            } else {
                w[0] = q[0]; w[1] = q[1]; w[2] = q[2]; w[3] = q[3];
            }
        } else {
            uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
            w[0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
            w[1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
            w[2] = __builtin_amdgcn_alignbyte(d3, d2, sh);
            w[3] = __builtin_amdgcn_alignbyte(d4, d3, sh);
        }
        (void)L;
        return;
    }
    w[0] = w[1] = w[2] = w[3] = 0;
    if (x + 16 <= 0) return;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        int64_t o = x + j;
        if (o >= 0) w[j >> 2] |= (uint32_t)buf[o] << (8 * (j & 3));
    }
}

// Nibble-table lookups with byte addresses pre-masked: lo/hi hold 4*nibble for
// the low/high nibble of each byte, so every lookup address is one byte extract.
__device__ inline uint32_t nib_at(const uint32_t *t, uint32_t addr4) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(t) + addr4);
}

// acc ^ XOR of the 8 nibble lookups of word x in tables t[0..7] (16 entries each)
__device__ inline uint32_t crc_word(uint32_t x, const uint32_t *t, uint32_t acc = 0) {
    uint32_t lo = (x << 2) & 0x3c3c3c3cu, hi = (x >> 2) & 0x3c3c3c3cu;
    asm volatile("" : "+v"(lo), "+v"(hi));   // keep the masks: 1 extract per address
    uint32_t a = nib_at(t + 0 * 16, lo & 0xffu), b = nib_at(t + 1 * 16, hi & 0xffu);
    uint32_t c = nib_at(t + 2 * 16, (lo >> 8) & 0xffu), d = nib_at(t + 3 * 16, (hi >> 8) & 0xffu);
    uint32_t e = nib_at(t + 4 * 16, (lo >> 16) & 0xffu), f = nib_at(t + 5 * 16, (hi >> 16) & 0xffu);
    uint32_t g = nib_at(t + 6 * 16, lo >> 24), h = nib_at(t + 7 * 16, hi >> 24);
    return ((acc ^ a) ^ (b ^ c)) ^ ((d ^ e) ^ (f ^ g)) ^ h;
}

__device__ inline uint32_t crc_shift(uint32_t x, const uint32_t (*t)[16]) {
    return crc_word(x, &t[0][0]);
}

// G lanes per buffer (16 or 64): a row is 16*G bytes; 64/G buffers per wave.
// G = 16 halves the lane-combine tree (4 levels, shared by 4 buffers) and is
// used for batches of many small buffers; G = 64 for few large ones.
template <int G>
__global__ __launch_bounds__(kCkBlock) void k_crc32(const uint8_t *__restrict__ src,
                                                    const uint64_t *__restrict__ off,
                                                    const uint64_t *__restrict__ len,
                                                    const uint32_t *__restrict__ init,
                                                    uint32_t *__restrict__ out, uint32_t count,
                                                    const CrcTables *__restrict__ tab) {
    constexpr int kLog = G == 64 ? 6 : 4;
    constexpr uint64_t kRow = 16u * G;
    constexpr uint32_t kPerWave = 64 / G;
    __shared__ uint32_t s_nib[32][16];
    __shared__ uint32_t s_sh[7][8][16];
    __shared__ uint32_t s_byte[256];
    for (int i = threadIdx.x; i < 32 * 16; i += kCkBlock) (&s_nib[0][0])[i] = (&tab->nib[0][0])[i];
    for (int i = threadIdx.x; i < 7 * 8 * 16; i += kCkBlock) (&s_sh[0][0][0])[i] = (&tab->shift[0][0][0])[i];
    for (int i = threadIdx.x; i < 256; i += kCkBlock) s_byte[i] = tab->byte[i];
    __syncthreads();

    const int lane = threadIdx.x & (G - 1);
    const uint32_t grp = (threadIdx.x >> 6) * kPerWave + ((threadIdx.x & 63) >> kLog);
    const uint32_t stride = gridDim.x * (kCkBlock / 64) * kPerWave;
    for (uint32_t b = blockIdx.x * (kCkBlock / 64) * kPerWave + grp; b < count; b += stride) {
        const uint64_t L = len[b];
        const uint8_t *buf = src + off[b];
        const uint32_t c0 = init ? init[b] : 0u;
        if (L < 4) {                                   // crc32.c byte loop (tiny input)
            if (lane == 0) {
                uint32_t c = ~c0;
                for (uint64_t i = 0; i < L; i++) c = (c >> 8) ^ s_byte[(c ^ buf[i]) & 0xffu];
                out[b] = ~c;
            }
            continue;
        }
        const uint64_t V = (L + kRow - 1) & ~(kRow - 1);
        const int64_t pad = (int64_t)(V - L);
        const uint32_t xv = ~c0;
        uint32_t acc = 0;
        for (uint64_t row = 0; row < V; row += kRow) {
            const int64_t x = (int64_t)row + 16 * lane - pad;
            uint32_t w[4];
            load_chunk16(buf, x, L, w);
            if (x < 4 && x + 16 > 0) {                 // fold ~init into data bytes 0..3
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    int64_t o = x + j;
                    if (o >= 0 && o < 4) w[j >> 2] ^= ((xv >> (8 * o)) & 0xffu) << (8 * (j & 3));
                }
            }
            uint32_t c = crc_word(w[0], s_nib[0], crc_shift(acc, s_sh[kLog]));
            c = crc_word(w[1], s_nib[8], c);
            c = crc_word(w[2], s_nib[16], c);
            acc = crc_word(w[3], s_nib[24], c);
        }
#pragma unroll
        for (int l = 0; l < kLog; l++) {
            uint32_t other = __shfl_down(acc, 1 << l, G);
            acc = crc_word(acc, &s_sh[l][0][0], other);
        }
        if (lane == 0) out[b] = ~acc;
    }
}

// ------------------------------------------------------------------------
// k_crc32s — the same CRC with 64-byte chunks and slice-by-4 byte tables
// (crc32.c's braid-free word loop: 4 lookups per 4 bytes, crc32.c:725-745
// style), for 1 lookup per byte instead of the nibble kernel's 2.5.  G lanes
// per buffer; lane i owns the 64-byte chunk at 64*i of every row of 64*G bytes
// and runs slice-by-4 through it, rows are joined by advancing the lane's CRC
// over the (G-1)*64-byte gap, lanes by the shuffle tree (64 << l bytes).
// Random byte indexes would hit the 32 LDS banks ~3.5-way; every table is
// therefore stored 16 times, entry e of copy c at word e*16 + c, and lane l
// reads copy l % 16: bank c or c + 16, so at most 2-way (lanes l and l + 16),
// in 64 KiB, which leaves room for two 1024-thread blocks per CU (32 copies,
// conflict-free but one block per CU, measured 2 % slower).
// ------------------------------------------------------------------------
constexpr int kCsBlock = 1024;
#ifndef ZGPU_CRC_COPY_LOG
#define ZGPU_CRC_COPY_LOG 4                   // A/B builds: 5 = 32 copies (tools/jobs/r06j.sh)
#endif
constexpr int kCsCopyLog = ZGPU_CRC_COPY_LOG; // 16 copies per table: 64 KiB, two blocks per CU

__device__ __attribute__((always_inline)) inline uint32_t s4_at(const uint8_t *T, uint32_t t, uint32_t e,
                                                                uint32_t loff) {
    return *reinterpret_cast<const uint32_t *>(T + (t << (kCsCopyLog + 10)) + (e << (kCsCopyLog + 2)) + loff);
}

__device__ __attribute__((always_inline)) inline uint32_t s4_step(uint32_t c, uint32_t w, const uint8_t *T,
                                                                  uint32_t loff) {
    c ^= w;
    return (s4_at(T, 3, c & 0xffu, loff) ^ s4_at(T, 2, (c >> 8) & 0xffu, loff)) ^
           (s4_at(T, 1, (c >> 16) & 0xffu, loff) ^ s4_at(T, 0, c >> 24, loff));
}

template <int G>
__global__ __launch_bounds__(kCsBlock) void k_crc32s(const uint8_t *__restrict__ src,
                                                     const uint64_t *__restrict__ off,
                                                     const uint64_t *__restrict__ len,
                                                     const uint32_t *__restrict__ init,
                                                     uint32_t *__restrict__ out, uint32_t count,
                                                     const CrcTables *__restrict__ tab) {
    constexpr int kLog = G == 64 ? 6 : 4;
    constexpr uint64_t kRow = 64u * G;
    constexpr uint32_t kPerWave = 64 / G;
    constexpr int kGap = G == 64 ? 7 : 6;              // sh64 index of the (G-1)*64-byte gap
    __shared__ __attribute__((aligned(16))) uint32_t s_t[4 * 256 << kCsCopyLog];
    __shared__ uint32_t s_sh[kCrcSh64Tabs][8][16];
    __shared__ uint32_t s_byte[256];
    for (int i = threadIdx.x; i < (4 * 256 << kCsCopyLog); i += kCsBlock) s_t[i] = (&tab->s4[0][0])[i >> kCsCopyLog];
    for (int i = threadIdx.x; i < kCrcSh64Tabs * 8 * 16; i += kCsBlock) (&s_sh[0][0][0])[i] = (&tab->sh64[0][0][0])[i];
    for (int i = threadIdx.x; i < 256; i += kCsBlock) s_byte[i] = tab->byte[i];
    __syncthreads();
    const uint8_t *T = reinterpret_cast<const uint8_t *>(s_t);
    const uint32_t loff = (threadIdx.x & ((1u << kCsCopyLog) - 1u)) << 2;

    const int lane = threadIdx.x & (G - 1);
    const uint32_t grp = (threadIdx.x >> 6) * kPerWave + ((threadIdx.x & 63) >> kLog);
    const uint32_t stride = gridDim.x * (kCsBlock / 64) * kPerWave;
    // the next buffer's offset, length and init are loaded one buffer ahead
    uint32_t b = blockIdx.x * (kCsBlock / 64) * kPerWave + grp;
    uint64_t nL = 0, nO = 0;
    uint32_t nI = 0;
    if (b < count) { nL = len[b]; nO = off[b]; nI = init ? init[b] : 0u; }
    for (; b < count; b += stride) {
        const uint64_t L = nL;
        const uint8_t *buf = src + nO;
        const uint32_t c0 = nI;
        if (b + stride < count) { nL = len[b + stride]; nO = off[b + stride]; nI = init ? init[b + stride] : 0u; }
        if (L < 4) {                                   // crc32.c byte loop (tiny input)
            if (lane == 0) {
                uint32_t c = ~c0;
                for (uint64_t i = 0; i < L; i++) c = (c >> 8) ^ s_byte[(c ^ buf[i]) & 0xffu];
                out[b] = ~c;
            }
            continue;
        }
        const uint64_t V = (L + kRow - 1) & ~(kRow - 1);
        const int64_t pad = (int64_t)(V - L);
        const uint32_t xv = ~c0;
        uint32_t acc = 0;
        auto chunk = [&](int64_t x, uint32_t (&w)[16]) {
            if (x < 4 && x + 64 > 0) {                 // fold ~init into data bytes 0..3
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const int64_t o = x + j;
                    if (o >= 0 && o < 4) w[j >> 2] ^= ((xv >> (8 * o)) & 0xffu) << (8 * (j & 3));
                }
            }
            acc = crc_word(acc, &s_sh[kGap][0][0]);
#pragma unroll
            for (int k = 0; k < 16; k++) acc = s4_step(acc, w[k], T, loff);
        };
        // rows in pairs: both rows' 128 bytes per lane are loaded before the
        // lookups start (one workgroup of 16 waves per CU needs the extra
        // bytes in flight to keep HBM busy)
        uint64_t row = 0;
        for (; row + 2 * kRow <= V; row += 2 * kRow) {
            const int64_t x = (int64_t)row + 64 * lane - pad;
            uint32_t wa[16], wb[16];
#pragma unroll
            for (int q = 0; q < 4; q++) load_chunk16(buf, x + 16 * q, L, wa + 4 * q);
#pragma unroll
            for (int q = 0; q < 4; q++) load_chunk16(buf, x + (int64_t)kRow + 16 * q, L, wb + 4 * q);
            chunk(x, wa);
            chunk(x + (int64_t)kRow, wb);
        }
        if (row < V) {
            const int64_t x = (int64_t)row + 64 * lane - pad;
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; q++) load_chunk16(buf, x + 16 * q, L, w + 4 * q);
            chunk(x, w);
        }
#pragma unroll
        for (int l = 0; l < kLog; l++) {
            const uint32_t other = __shfl_down(acc, 1 << l, G);
            acc = crc_word(acc, &s_sh[l][0][0], other);
        }
        if (lane == 0) out[b] = ~acc;
    }
}

__device__ inline uint32_t dot4(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot4(a, b, c, false);
}

__global__ __launch_bounds__(kCkBlock) void k_adler32(const uint8_t *__restrict__ src,
                                                      const uint64_t *__restrict__ off,
                                                      const uint64_t *__restrict__ len,
                                                      const uint32_t *__restrict__ init,
                                                      uint32_t *__restrict__ out, uint32_t count) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    for (uint32_t b = blockIdx.x * (kCkBlock / 64) + wave; b < count; b += gridDim.x * (kCkBlock / 64)) {
        const uint64_t L = len[b];
        const uint8_t *buf = src + off[b];
        const uint32_t a0 = init ? init[b] : 1u;
        if (L < 16) {                                  // adler32.c:71-94 verbatim semantics
            if (lane == 0) {
                uint32_t a = a0 & 0xffffu, s2 = (a0 >> 16) & 0xffffu;
                if (L == 1) {
                    a += buf[0];
                    if (a >= kAdlerBase) a -= kAdlerBase;
                    s2 += a;
                    if (s2 >= kAdlerBase) s2 -= kAdlerBase;
                } else {
                    for (uint64_t i = 0; i < L; i++) { a += buf[i]; s2 += a; }
                    if (a >= kAdlerBase) a -= kAdlerBase;
                    s2 %= kAdlerBase;
                }
                out[b] = a | (s2 << 16);
            }
            continue;
        }
        const uint64_t V = (L + 1023) & ~(uint64_t)1023;
        const int64_t pad = (int64_t)(V - L);
        uint64_t s1 = 0, s2 = 0;
        for (uint64_t row = 0; row < V; row += 1024) {
            const int64_t x = (int64_t)row + 16 * lane - pad;
            uint32_t w[4];
            load_chunk16(buf, x, L, w);
            uint32_t sx = dot4(w[0], 0x01010101u, 0);
            sx = dot4(w[1], 0x01010101u, sx);
            sx = dot4(w[2], 0x01010101u, sx);
            sx = dot4(w[3], 0x01010101u, sx);
            uint32_t sj = dot4(w[0], 0x03020100u, 0);
            sj = dot4(w[1], 0x07060504u, sj);
            sj = dot4(w[2], 0x0b0a0908u, sj);
            sj = dot4(w[3], 0x0f0e0d0cu, sj);
            // weight of chunk byte j = V - (row + 16*lane) - j
            const uint64_t wt = (V - row - 16u * (uint64_t)lane) % kAdlerBase;
            s1 += sx;
            s2 += wt * sx + kAdlerBase - sj;
        }
#pragma unroll
        for (int l = 32; l >= 1; l >>= 1) {
            s1 += __shfl_down(s1, l, 64);
            s2 += __shfl_down(s2, l, 64);
        }
        if (lane == 0) {
            const uint64_t A0 = a0 & 0xffffu, B0 = (a0 >> 16) & 0xffffu;
            uint64_t A = (A0 + s1) % kAdlerBase;
            uint64_t B = (B0 + (L % kAdlerBase) * A0 + s2 % kAdlerBase) % kAdlerBase;
            out[b] = (uint32_t)A | ((uint32_t)B << 16);
        }
    }
}

// ------------------------------------------------------------------------
// Few large buffers: one wave per buffer leaves the GPU idle (256 x 16 MiB is
// 256 waves), so each buffer is cut into `parts` row ranges, one wave each
// (k_*_part), and a per-buffer finish joins them (k_*_fin).
//
// Adler-32: the weights of k_adler32 are distances to the buffer's (virtual)
// end, so the partial sums of row ranges simply add (atomics into two u64 per
// buffer).  CRC-32: each part is a zero-init linear CRC over its rows; the
// finish joins them by Horner, crc(A||B) = x^(8|B|) * crc(A) ^ crc(B)
// (crc32_combine, crc32.c:1021-1026, multmodp/x2nmodp :155-187).
// ------------------------------------------------------------------------
__device__ inline void adler_rows(const uint8_t *buf, uint64_t L, uint64_t V, int64_t pad, uint64_t r0,
                                  uint64_t r1, int lane, uint64_t &s1, uint64_t &s2) {
    uint64_t row = r0;
    for (; row + 4 <= r1; row += 4) {                 // 4 rows (64 B per lane) in flight
        uint32_t w[4][4];
#pragma unroll
        for (int q = 0; q < 4; q++) load_chunk16(buf, (int64_t)((row + q) << 10) + 16 * lane - pad, L, w[q]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t sx = dot4(w[q][0], 0x01010101u, 0);
            sx = dot4(w[q][1], 0x01010101u, sx);
            sx = dot4(w[q][2], 0x01010101u, sx);
            sx = dot4(w[q][3], 0x01010101u, sx);
            uint32_t sj = dot4(w[q][0], 0x03020100u, 0);
            sj = dot4(w[q][1], 0x07060504u, sj);
            sj = dot4(w[q][2], 0x0b0a0908u, sj);
            sj = dot4(w[q][3], 0x0f0e0d0cu, sj);
            const uint64_t wt = (V - ((row + q) << 10) - 16u * (uint64_t)lane) % kAdlerBase;
            s1 += sx;
            s2 += wt * sx + kAdlerBase - sj;
        }
    }
    for (; row < r1; row++) {
        uint32_t w[4];
        load_chunk16(buf, (int64_t)(row << 10) + 16 * lane - pad, L, w);
        uint32_t sx = dot4(w[0], 0x01010101u, 0);
        sx = dot4(w[1], 0x01010101u, sx);
        sx = dot4(w[2], 0x01010101u, sx);
        sx = dot4(w[3], 0x01010101u, sx);
        uint32_t sj = dot4(w[0], 0x03020100u, 0);
        sj = dot4(w[1], 0x07060504u, sj);
        sj = dot4(w[2], 0x0b0a0908u, sj);
        sj = dot4(w[3], 0x0f0e0d0cu, sj);
        const uint64_t wt = (V - (row << 10) - 16u * (uint64_t)lane) % kAdlerBase;
        s1 += sx;
        s2 += wt * sx + kAdlerBase - sj;
    }
}

__global__ __launch_bounds__(kCkBlock) void k_adler32_part(const uint8_t *__restrict__ src,
                                                           const uint64_t *__restrict__ off,
                                                           const uint64_t *__restrict__ len,
                                                           unsigned long long *__restrict__ acc,
                                                           uint32_t count, uint32_t parts) {
    const int lane = threadIdx.x & 63;
    const uint64_t item = (uint64_t)blockIdx.x * (kCkBlock / 64) + (threadIdx.x >> 6);
    if (item >= (uint64_t)count * parts) return;
    const uint32_t b = (uint32_t)(item / parts), p = (uint32_t)(item % parts);
    const uint64_t L = len[b];
    if (L < 16) return;
    const uint64_t V = (L + 1023) & ~(uint64_t)1023, rows = V >> 10, per = (rows + parts - 1) / parts;
    const uint64_t r0 = (uint64_t)p * per, r1 = r0 + per < rows ? r0 + per : rows;
    if (r0 >= r1) return;
    uint64_t s1 = 0, s2 = 0;
    adler_rows(src + off[b], L, V, (int64_t)(V - L), r0, r1, lane, s1, s2);
#pragma unroll
    for (int l = 32; l >= 1; l >>= 1) {
        s1 += __shfl_down(s1, l, 64);
        s2 += __shfl_down(s2, l, 64);
    }
    if (lane == 0) {
        atomicAdd(&acc[2 * b], (unsigned long long)s1);
        atomicAdd(&acc[2 * b + 1], (unsigned long long)s2);
    }
}

__global__ void k_adler32_fin(const uint8_t *__restrict__ src, const uint64_t *__restrict__ off,
                              const uint64_t *__restrict__ len, const uint32_t *__restrict__ init,
                              uint32_t *__restrict__ out, const unsigned long long *__restrict__ acc,
                              uint32_t count) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= count) return;
    const uint64_t L = len[b];
    const uint32_t a0 = init ? init[b] : 1u;
    uint64_t A0 = a0 & 0xffffu, B0 = (a0 >> 16) & 0xffffu;
    if (L < 16) {                                      // adler32.c:71-94
        const uint8_t *buf = src + off[b];
        uint32_t a = (uint32_t)A0, s2 = (uint32_t)B0;
        if (L == 1) {
            a += buf[0];
            if (a >= kAdlerBase) a -= kAdlerBase;
            s2 += a;
            if (s2 >= kAdlerBase) s2 -= kAdlerBase;
        } else {
            for (uint64_t i = 0; i < L; i++) { a += buf[i]; s2 += a; }
            if (a >= kAdlerBase) a -= kAdlerBase;
            s2 %= kAdlerBase;
        }
        out[b] = a | (s2 << 16);
        return;
    }
    const uint64_t A = (A0 + acc[2 * b] % kAdlerBase) % kAdlerBase;
    const uint64_t B = (B0 + (L % kAdlerBase) * A0 + acc[2 * b + 1] % kAdlerBase) % kAdlerBase;
    out[b] = (uint32_t)A | ((uint32_t)B << 16);
}

// crc32.c:155-170 (reflected GF(2) product mod the CRC-32 polynomial)
__device__ inline uint32_t d_multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = b & 1 ? (b >> 1) ^ 0xedb88320u : b >> 1;
    }
    return p;
}
// x^(8n) mod p (crc32.c:176-187 with k = 3), squaring x^(2^k) as it goes
__device__ inline uint32_t d_x8nmodp(uint64_t n) {
    uint32_t p = 1u << 31, sq = 1u << 30;             // x^0, x^1
    for (int k = 0; k < 3; k++) sq = d_multmodp(sq, sq);
    while (n) {
        if (n & 1) p = d_multmodp(sq, p);
        n >>= 1;
        if (n) sq = d_multmodp(sq, sq);
    }
    return p;
}

constexpr uint64_t kCpRow = kCrcRow;                   // k_crc32s<64> row: 64 lanes x 64 B

__global__ __launch_bounds__(kCsBlock) void k_crc32_part(const uint8_t *__restrict__ src,
                                                         const uint64_t *__restrict__ off,
                                                         const uint64_t *__restrict__ len,
                                                         const uint32_t *__restrict__ init,
                                                         uint32_t *__restrict__ part_out, uint32_t count,
                                                         uint32_t parts, const CrcTables *__restrict__ tab) {
    __shared__ __attribute__((aligned(16))) uint32_t s_t[4 * 256 << kCsCopyLog];
    __shared__ uint32_t s_sh[kCrcSh64Tabs][8][16];
    for (int i = threadIdx.x; i < (4 * 256 << kCsCopyLog); i += kCsBlock) s_t[i] = (&tab->s4[0][0])[i >> kCsCopyLog];
    for (int i = threadIdx.x; i < kCrcSh64Tabs * 8 * 16; i += kCsBlock) (&s_sh[0][0][0])[i] = (&tab->sh64[0][0][0])[i];
    __syncthreads();
    const uint8_t *T = reinterpret_cast<const uint8_t *>(s_t);
    const uint32_t loff = (threadIdx.x & ((1u << kCsCopyLog) - 1u)) << 2;
    const int lane = threadIdx.x & 63;
    const uint64_t items = (uint64_t)count * parts;
    for (uint64_t item = (uint64_t)blockIdx.x * (kCsBlock / 64) + (threadIdx.x >> 6); item < items;
         item += (uint64_t)gridDim.x * (kCsBlock / 64)) {
        const uint32_t b = (uint32_t)(item / parts), p = (uint32_t)(item % parts);
        const uint64_t L = len[b];
        if (L < 4) continue;                           // k_crc32_fin's byte loop
        const uint8_t *buf = src + off[b];
        const uint64_t V = (L + kCpRow - 1) & ~(kCpRow - 1), rows = V / kCpRow, per = (rows + parts - 1) / parts;
        const uint64_t r0 = (uint64_t)p * per, r1 = r0 + per < rows ? r0 + per : rows;
        const int64_t pad = (int64_t)(V - L);
        const uint32_t xv = ~(init ? init[b] : 0u);
        uint32_t acc = 0;
        for (uint64_t row = r0; row < r1; row++) {
            const int64_t x = (int64_t)(row * kCpRow) + 64 * lane - pad;
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; q++) load_chunk16(buf, x + 16 * q, L, w + 4 * q);
            if (x < 4 && x + 64 > 0) {                 // fold ~init into data bytes 0..3
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const int64_t o = x + j;
                    if (o >= 0 && o < 4) w[j >> 2] ^= ((xv >> (8 * o)) & 0xffu) << (8 * (j & 3));
                }
            }
            acc = crc_word(acc, &s_sh[7][0][0]);       // advance over the other lanes' 63*64 bytes
#pragma unroll
            for (int k = 0; k < 16; k++) acc = s4_step(acc, w[k], T, loff);
        }
#pragma unroll
        for (int l = 0; l < 6; l++) {
            const uint32_t other = __shfl_down(acc, 1 << l, 64);
            acc = crc_word(acc, &s_sh[l][0][0], other);
        }
        if (lane == 0) part_out[item] = acc;
    }
}

// d_multmodp(a, b) for a = x^e, e >= 0 given by its powers x^(2^i) (tp[i]):
// the product of the powers of e's set bits
__device__ inline uint32_t d_xpow(const uint32_t *tp, uint64_t e, uint32_t b) {
    for (int i = 0; e; i++, e >>= 1)
        if (e & 1) b = d_multmodp(tp[i], b);
    return b;
}

// One wave per buffer.  The parts are counted from the end: part p = last - 1
// - r (r >= 0) is followed by r full parts and the last one, so its term is
// part_p * x^(8 kCpRow (rows_last + r per)) = X * F^r * part_p with F =
// x^(8 kCpRow per), X = x^(8 kCpRow rows_last).  Lane l sums r in [l q, (l+1) q)
// by Horner in F, scales by F^(l q), and the lanes' sums are xor-reduced
// (crc32_combine's linearity, crc32.c:1002-1010): no lane-to-lane ordering.
// (One lane folding the parts in order took ~0.46 ms for 1024 parts.)
__global__ __launch_bounds__(64) void k_crc32_fin(const uint8_t *__restrict__ src, const uint64_t *__restrict__ off,
                                                  const uint64_t *__restrict__ len, const uint32_t *__restrict__ init,
                                                  uint32_t *__restrict__ out, const uint32_t *__restrict__ part_out,
                                                  uint32_t count, uint32_t parts, const CrcTables *__restrict__ tab) {
    const uint32_t *tp = tab->xrow;                    // x^(8 kCpRow 2^i)
    const uint32_t b = blockIdx.x;
    const int lane = threadIdx.x;
    if (b >= count) return;
    const uint64_t L = len[b];
    const uint32_t c0 = init ? init[b] : 0u;
    if (L < 4) {                                       // crc32.c byte loop (tiny input)
        if (lane == 0) {
            const uint8_t *buf = src + off[b];
            uint32_t c = ~c0;
            for (uint64_t i = 0; i < L; i++) c = (c >> 8) ^ tab->byte[(c ^ buf[i]) & 0xffu];
            out[b] = ~c;
        }
        return;
    }
    const uint64_t V = (L + kCpRow - 1) & ~(kCpRow - 1), rows = V / kCpRow, per = (rows + parts - 1) / parts;
    const uint32_t np = (uint32_t)((rows + per - 1) / per);          // parts holding rows
    const uint64_t rows_last = rows - (uint64_t)(np - 1) * per;
    const uint32_t *pp = part_out + (uint64_t)b * parts;
    const uint32_t nr = np - 1;                        // parts before the last
    const uint32_t q = (nr + 63) / 64;
    const uint32_t one = 1u << 31;                     // x^0
    const uint32_t F = d_xpow(tp, per, one);
    uint32_t acc = 0;
    for (uint32_t j = q; j-- > 0;) {                   // Horner over r = lane q + j, highest first
        const uint32_t r = (uint32_t)lane * q + j;
        acc = d_multmodp(F, acc);
        if (r < nr) acc ^= pp[nr - 1 - r];
    }
    acc = d_xpow(tp, per * (uint64_t)lane * q, acc);  // F^(l q)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o, 64);
    if (lane == 0) out[b] = ~(d_xpow(tp, rows_last, acc) ^ pp[np - 1]);
}

// parts per buffer for a split launch: enough waves to fill the chip
static uint32_t split_parts(uint32_t count, size_t scratch, size_t per_part_bytes, size_t fixed_per_buf) {
    if (count == 0 || count >= 4096) return 1;
    uint32_t parts = (16384u + count - 1) / count;
    if (parts > 1024) parts = 1024;
    while (parts > 1 && (size_t)count * (fixed_per_buf + per_part_bytes * parts) > scratch) parts >>= 1;
    return parts;
}

static int grid_for(uint32_t count, uint32_t per_wave = 1) {
    uint32_t waves = (count + per_wave - 1) / per_wave;
    uint32_t blocks = (waves + (kCkBlock / 64) - 1) / (kCkBlock / 64);
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    return (int)blocks;
}

int launch_crc32(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                 const uint32_t *init, uint32_t *out, uint32_t count,
                 void *scratch, size_t scratch_bytes, hipStream_t st) {
    if (count == 0) return 0;
    if (const uint32_t parts = scratch ? split_parts(count, scratch_bytes, 4, 0) : 1; parts > 1) {
        uint32_t *po = static_cast<uint32_t *>(scratch);
        const uint64_t items = (uint64_t)count * parts;
        uint64_t blocks = (items + (kCsBlock / 64) - 1) / (kCsBlock / 64);
        if (blocks > 512) blocks = 512;
        hipLaunchKernelGGL(k_crc32_part, dim3((uint32_t)blocks), dim3(kCsBlock), 0, st, src, off, len, init, po,
                           count, parts, device_crc_tables());
        hipLaunchKernelGGL(k_crc32_fin, dim3(count), dim3(64), 0, st, src, off, len, init, out, po, count, parts,
                           device_crc_tables());
        return (int)hipGetLastError();
    }
    static const bool nibble = std::getenv("ZGPU_CRC_NIBBLE") != nullptr;   // A/B: the nibble kernel
    if (nibble) {
        // 16-lane groups once there are enough buffers to fill the chip 4x over
        if (count >= 4u * 256u * (kCkBlock / 64) * 4u)
            hipLaunchKernelGGL(k_crc32<16>, dim3(grid_for(count, 4)), dim3(kCkBlock), 0, st, src, off,
                               len, init, out, count, device_crc_tables());
        else
            hipLaunchKernelGGL(k_crc32<64>, dim3(grid_for(count)), dim3(kCkBlock), 0, st, src, off,
                               len, init, out, count, device_crc_tables());
        return (int)hipGetLastError();
    }
    // one 1024-thread block per CU (128 KiB of tables), persistent over buffers;
    // 16-lane groups when there are many buffers
    auto blocks = [&](uint32_t per_wave) {
        uint32_t waves = (count + per_wave - 1) / per_wave;
        uint32_t b = (waves + (kCsBlock / 64) - 1) / (kCsBlock / 64);
        return b > 512u ? 512u : (b ? b : 1u);
    };
    if (count >= 256u * (kCsBlock / 64) * 4u * 2u)
        hipLaunchKernelGGL(k_crc32s<16>, dim3(blocks(4)), dim3(kCsBlock), 0, st, src, off, len, init, out,
                           count, device_crc_tables());
    else
        hipLaunchKernelGGL(k_crc32s<64>, dim3(blocks(1)), dim3(kCsBlock), 0, st, src, off, len, init, out,
                           count, device_crc_tables());
    return (int)hipGetLastError();
}

int launch_adler32(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                   const uint32_t *init, uint32_t *out, uint32_t count,
                   void *scratch, size_t scratch_bytes, hipStream_t st) {
    if (count == 0) return 0;
    if (const uint32_t parts = scratch ? split_parts(count, scratch_bytes, 0, 16) : 1; parts > 1) {
        auto *acc = static_cast<unsigned long long *>(scratch);
        if (hipMemsetAsync(acc, 0, 16ull * count, st) != hipSuccess) return (int)hipErrorInvalidValue;
        const uint64_t items = (uint64_t)count * parts;
        hipLaunchKernelGGL(k_adler32_part, dim3((uint32_t)((items + (kCkBlock / 64) - 1) / (kCkBlock / 64))),
                           dim3(kCkBlock), 0, st, src, off, len, acc, count, parts);
        hipLaunchKernelGGL(k_adler32_fin, dim3((count + 63) / 64), dim3(64), 0, st, src, off, len, init, out, acc,
                           count);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(k_adler32, dim3(grid_for(count)), dim3(kCkBlock), 0, st, src, off, len,
                       init, out, count);
    return (int)hipGetLastError();
}

// scratch that lets a launch of `count` buffers split them (launch_crc32/adler32)
size_t checksum_scratch_bytes(uint32_t count) { return count >= 4096 ? 0 : 16ull * 16384 + 64ull * count; }

}  // namespace zgpu
