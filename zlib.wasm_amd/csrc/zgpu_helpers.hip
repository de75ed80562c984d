// zgpu_helpers.hip — the four kernels of src/zlib_simd_optimized.c that have no
// caller in the reference, kept as C-ABI names with
// zlib-correct semantics and run on the GPU:
//   k_slide_hash     slide_hash (deflate.c:187-209): every head[]/prev[] entry
//                    m -> m >= wsize ? m - wsize : NIL, all entries (the
//                    reference's loop leaves a remainder of < 16 untouched)
//   k_compare256     leading equal bytes of two 256-byte strings
//   k_longest_match  longest_match (deflate.c:1356-1497) over a caller's window
//                    and prev[]: one wave, 64 bytes compared per round trip
//   k_chunkmemset    the LZ77 copy dest[i] = src[i % dist] (the reference's
//                    pattern splat is wrong for dist not in {1, 2, 4, 8, >= 16})
#include "zgpu_internal.h"

namespace zgpu {

__global__ void k_slide_hash(uint16_t *head, uint16_t *prev, uint32_t hash_size, uint32_t window_size,
                             uint32_t wsize) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < hash_size) { const uint32_t m = head[i]; head[i] = (uint16_t)(m >= wsize ? m - wsize : 0u); }
    if (i < window_size) { const uint32_t m = prev[i]; prev[i] = (uint16_t)(m >= wsize ? m - wsize : 0u); }
}

// leading equal bytes of a[0..max) and b[0..max), one byte per lane, 64 per round
__device__ __attribute__((always_inline)) inline uint32_t wave_common(const uint8_t *a, const uint8_t *b,
                                                                      uint32_t from, uint32_t max) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t k0 = from; k0 < max; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool diff = k < max && a[k] != b[k];
        const uint64_t m = __ballot(diff);
        if (m) return k0 + (uint32_t)__builtin_ctzll(m);
    }
    return max;
}

__global__ __launch_bounds__(64) void k_compare256(const uint8_t *a, const uint8_t *b, uint32_t *out) {
    const uint32_t r = wave_common(a, b, 0, 256);
    if (threadIdx.x == 0) *out = r;
}

// zlib's loop: quick reject on scan[best-1..best] and scan[0..1], byte 2 not
// compared (equal hashes imply it in zlib; the caller's prev[] decides here),
// bytes 3.. compared up to MAX_MATCH, first strictly longer candidate kept,
// stop at nice (min(258, lookahead)), chain quartered when prev_length >=
// good, limit strstart - MAX_DIST, result capped at lookahead.
__global__ __launch_bounds__(64) void k_longest_match(const uint8_t *window, uint32_t strstart,
                                                      uint32_t prev_length, uint32_t good, uint32_t chain,
                                                      uint32_t lookahead, const uint16_t *prev, uint32_t wmask,
                                                      uint32_t *out) {
    const uint32_t wsize = wmask + 1;
    const uint32_t max_dist = wsize - (uint32_t)kMinLookahead;
    const uint8_t *scan = window + strstart;
    uint32_t best = prev_length;
    uint32_t nice = (uint32_t)kMaxMatch < lookahead ? (uint32_t)kMaxMatch : lookahead;
    if (prev_length >= good) chain >>= 2;
    const uint32_t limit = strstart > max_dist ? strstart - max_dist : 0u;
    uint32_t cur = prev[strstart & wmask];
    uint32_t start = 0, found = 0;
    if (cur > limit && chain != 0) {
        do {
            const uint8_t *m = window + cur;
            if (m[best] == scan[best] && m[best - 1] == scan[best - 1] && m[0] == scan[0] && m[1] == scan[1]) {
                const uint32_t len = wave_common(scan, m, 3, (uint32_t)kMaxMatch);
                if (len > best) {
                    start = cur;
                    found = 1;
                    best = len;
                    if (len >= nice) break;
                }
            }
            cur = prev[cur & wmask];
        } while (cur > limit && --chain != 0);
    }
    if (threadIdx.x == 0) {
        out[0] = best <= lookahead ? best : lookahead;
        out[1] = start;
        out[2] = found;                                // match_start written
    }
}

__global__ void k_chunkmemset(uint8_t *dest, const uint8_t *src, uint32_t dist, uint32_t len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) dest[i] = src[i % dist];
}

int launch_slide_hash(uint16_t *head, uint16_t *prev, uint32_t hash_size, uint32_t window_size, uint32_t wsize,
                      hipStream_t st) {
    const uint32_t n = hash_size > window_size ? hash_size : window_size;
    if (n) hipLaunchKernelGGL(k_slide_hash, dim3((n + 255) / 256), dim3(256), 0, st, head, prev, hash_size,
                              window_size, wsize);
    return (int)hipGetLastError();
}
int launch_compare256(const uint8_t *a, const uint8_t *b, uint32_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_compare256, dim3(1), dim3(64), 0, st, a, b, out);
    return (int)hipGetLastError();
}
int launch_longest_match(const uint8_t *window, uint32_t strstart, uint32_t prev_length, uint32_t good,
                         uint32_t chain, uint32_t lookahead, const uint16_t *prev, uint32_t wmask, uint32_t *out,
                         hipStream_t st) {
    hipLaunchKernelGGL(k_longest_match, dim3(1), dim3(64), 0, st, window, strstart, prev_length, good, chain,
                       lookahead, prev, wmask, out);
    return (int)hipGetLastError();
}
int launch_chunkmemset(uint8_t *dest, const uint8_t *src, uint32_t dist, uint32_t len, hipStream_t st) {
    if (len) hipLaunchKernelGGL(k_chunkmemset, dim3((len + 255) / 256), dim3(256), 0, st, dest, src, dist, len);
    return (int)hipGetLastError();
}

}  // namespace zgpu
