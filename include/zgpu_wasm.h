/*
 * zgpu_wasm.h — the reference's WASM front-end exports, re-exported by
 * libzgpu.so with the same names and C signatures so the existing
 * compress()/decompress()/compressSIMD() callers (src/lib/index.ts:120,170,
 * 250,267) bind unchanged.  All of them route to the GPU path.
 */
#ifndef ZGPU_WASM_H
#define ZGPU_WASM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/wasm_module.c:34-46 — compress2 with level clamp; NULL/empty -> Z_STREAM_ERROR */
int zlib_compress_buffer(const unsigned char *src, unsigned long src_len,
                         unsigned char *dest, unsigned long *dest_len, int level);
/* src/wasm_module.c:53-60 — uncompress; NULL/empty -> Z_STREAM_ERROR */
int zlib_decompress_buffer(const unsigned char *src, unsigned long src_len,
                           unsigned char *dest, unsigned long *dest_len);
/* src/wasm_module_simd.c:425-456 — the same under the SIMD module's names */
int zlib_decompress_optimized(const unsigned char *input, unsigned long input_len,
                              unsigned char *output, unsigned long *output_len);
int zlib_decompress(const unsigned char *input, unsigned long input_len,
                    unsigned char *output, unsigned long *output_len);
int zlib_compress_optimized(const unsigned char *input, unsigned long input_len,
                            unsigned char *output, unsigned long *output_len, int level);
int zlib_compress(const unsigned char *input, unsigned long input_len,
                  unsigned char *output, unsigned long *output_len, int level);

/* src/wasm_module.c:160-291 — stream contexts over deflate() / inflate() */
typedef struct zlib_stream_s zlib_stream_t;
zlib_stream_t *zlib_deflate_init(int level, int window_bits, int mem_level, int strategy);
int zlib_deflate_process(zlib_stream_t *ctx, const unsigned char *input, unsigned int input_len,
                         unsigned char *output, unsigned int output_len, int flush);
void zlib_deflate_end(zlib_stream_t *ctx);
zlib_stream_t *zlib_inflate_init(int window_bits);
int zlib_inflate_process(zlib_stream_t *ctx, const unsigned char *input, unsigned int input_len,
                         unsigned char *output, unsigned int output_len);
void zlib_inflate_end(zlib_stream_t *ctx);
unsigned int zlib_stream_avail_in(zlib_stream_t *ctx);
unsigned int zlib_stream_avail_out(zlib_stream_t *ctx);
unsigned long zlib_stream_total_in(zlib_stream_t *ctx);
unsigned long zlib_stream_total_out(zlib_stream_t *ctx);

/* src/wasm_module.c:65-84 */
unsigned long zlib_crc32(unsigned long crc, const unsigned char *buf, unsigned int len);
unsigned long zlib_adler32(unsigned long adler, const unsigned char *buf, unsigned int len);
unsigned long zlib_compress_bound(unsigned long source_len);
const char *zlib_get_version(void);

/* src/zlib_simd_compression.c:280 and src/zlib_simd_optimized.c:354-383:
 * raw deflate (windowBits -15).  Deviation: a too-small output returns
 * Z_BUF_ERROR instead of the reference's Z_OK-with-unchanged-length. */
int zlib_compress_simd(const uint8_t *input, size_t input_len,
                       uint8_t *output, size_t *output_len, int level);
int zlib_compress_simd_full(const uint8_t *input, size_t input_len,
                            uint8_t *output, size_t *output_len, int level);
/* src/wasm_module_side.c:61-70: raw deflate for src_len >= 8192, else compress2 */
int zlib_compress_simd_buffer(const uint8_t *src, size_t src_len,
                              uint8_t *dest, size_t *dest_len, int level);
/* src/zlib_simd_compression.c:342, src/zlib_simd_optimized.c:387 */
uint32_t zlib_crc32_simd_optimized(uint32_t crc, const uint8_t *data, size_t len);
uint32_t zlib_crc32_simd_enhanced(uint32_t crc, const uint8_t *data, size_t len);
/* src/zlib_simd_optimized.c:116, with zlib-correct Adler-32 semantics */
uint32_t zlib_adler32_simd(uint32_t adler, const uint8_t *buf, size_t len);

/* src/zlib_simd_optimized.c:27,74,210,296 — the build's kernels that have no
 * caller in the reference, with zlib-correct semantics, run on
 * the GPU over the caller's host arrays:
 *  slide_hash: every entry m of head[hash_size] and prev[window_size] becomes
 *    m >= wsize ? m - wsize : 0 (deflate.c:187-209; the reference leaves a
 *    remainder of < 16 entries untouched);
 *  compare256: number of leading equal bytes of src0[0..256) and src1[0..256);
 *  longest_match: deflate.c:1356-1497 over window[0 .. 2*(wmask+1)) and
 *    prev[0 .. wmask+1), chain head prev[strstart & wmask], nice = min(258,
 *    lookahead), limit strstart - (wmask+1-262); returns min(best, lookahead),
 *    writes *match_start only when a candidate beat prev_length; invalid
 *    arguments return prev_length;
 *  chunkmemset: dest[i] = src[i % dist] for i < len (the LZ77 copy; the
 *    reference's splat is wrong for dist in 3, 5..7, 9..15). */
void zlib_slide_hash_simd(uint16_t *hash_table, uint16_t *prev_table, uint32_t hash_size,
                          uint32_t window_size, uint16_t wsize);
uint32_t zlib_compare256_simd(const uint8_t *src0, const uint8_t *src1);
uint32_t zlib_longest_match_simd(const uint8_t *window, uint32_t strstart, uint32_t prev_length,
                                 uint32_t good_match, uint32_t max_chain_length, uint32_t lookahead,
                                 const uint16_t *prev_table, uint32_t wmask, uint32_t *match_start);
void zlib_chunkmemset_simd(uint8_t *dest, uint8_t *src, uint32_t dist, uint32_t len);

#ifdef __cplusplus
}
#endif
#endif /* ZGPU_WASM_H */
