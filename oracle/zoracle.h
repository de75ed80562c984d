/*
 * zoracle.h — TEST INFRASTRUCTURE ONLY (never linked into the product path).
 *
 * Plain-C restatement of the reference's compression hot path
 * (discere-os/zlib.wasm @ zlib 1.3.1.1-motley: deflate.c, trees.c, crc32.c,
 * adler32.c, compress.c).  Two formulations of deflate live here:
 *
 *   zo_compress()     sequential restatement of deflate_fast/deflate_slow over
 *                     absolute input positions (the reference's algorithm);
 *   zo_pp_*()         the position-parallel formulation the GPU kernels
 *                     implement: per-position hash links,
 *                     per-position longest_match results for both chain budgets,
 *                     then a sequential parse.  Used to check each GPU stage.
 *
 * Parity of this oracle is pinned against the compiled reference
 * (oracle/_ref/libzref.so, built in the build container only) by
 * tests/test_oracle.py and by the committed fixtures in tests/golden/.
 */
#ifndef ZORACLE_H
#define ZORACLE_H
#include <stddef.h>
#include <stdint.h>

#define ZO_OK            0
#define ZO_STREAM_ERROR (-2)
#define ZO_DATA_ERROR   (-3)
#define ZO_MEM_ERROR    (-4)
#define ZO_BUF_ERROR    (-5)

/* wrap: 0 = raw deflate (windowBits -15), 1 = zlib (windowBits 15),
 *       2 = gzip (windowBits 31) */
unsigned long zo_compress_bound(unsigned long n);
int zo_compress(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                int level, int wrap);
/* strategies (zlib.h:197-201): deflateInit2_(strategy) semantics */
#define ZO_FILTERED     1
#define ZO_HUFFMAN_ONLY 2
#define ZO_RLE          3
#define ZO_FIXED        4
int zo_compress2(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                 int level, int wrap, int strategy);

uint32_t zo_crc32(uint32_t crc, const uint8_t *buf, size_t len);
uint32_t zo_adler32(uint32_t adler, const uint8_t *buf, size_t len);
uint32_t zo_crc32_combine(uint32_t crc1, uint32_t crc2, int64_t len2);
uint32_t zo_adler32_combine(uint32_t adler1, uint32_t adler2, int64_t len2);

/* ---- position-parallel formulation (GPU spec) ---- */
/* link[p] = p - q for the most recent q < p (q <= n-3, q != 0) with
 * hash3(q) == hash3(p) and p - q <= 32767; 0 when there is none or p > n-3. */
void zo_pp_links(const uint8_t *src, size_t n, uint16_t *link);
/* For every p <= n-3 whose head link is within MAX_DIST: the longest_match
 * result for the level's full chain budget and for the quartered budget,
 * packed (len << 16) | dist; 0 when no candidate survives the quick reject
 * or there is no valid head.  Levels 4..9 (all positions inserted). */
void zo_pp_match(const uint8_t *src, size_t n, int level, const uint16_t *link,
                 uint32_t *full, uint32_t *quarter);
/* Whole-stream compression through the position-parallel formulation
 * (levels 1..9; levels 1..3 use the inserted-set walk of Appendix B.2). */
int zo_pp_compress(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                   int level, int wrap);

int zo_pp_compress2(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n,
                    int level, int wrap, int strategy);
/* deflate() over a sequence of calls: the input is [0, n); call i ended at
 * fpos[i] (ascending) with flush ftype[i] in {Z_PARTIAL_FLUSH 1, Z_SYNC_FLUSH 2,
 * Z_FULL_FLUSH 3, Z_BLOCK 5} (calls zlib turns away, a repeated flush with no
 * input and no higher rank, are not listed); Z_NO_FLUSH calls in between do not
 * change the stream.  finish = 1: the last call was Z_FINISH at n (final block,
 * trailer); finish = 0: fpos[nf-1] == n and the output is every complete byte
 * written so far (header included).  Levels 1..9 (level 0's stored blocks
 * follow the caller's avail_out).  deflate.c:954-1263,1923-2043, trees.c:887. */
int zo_deflate_flushes(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n, int level,
                       int wrap, int strategy, const size_t *fpos, const int *ftype, int nf,
                       int finish);
/* level 0 over a deflate() call sequence (take[i] input bytes, flush[i]), each
 * call's output space large enough: the whole stream, and per call the status
 * and the total output length after it (deflate.c:763-1265, :1635-1815) */
int zo_deflate_stored_calls(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t n, int wrap,
                            const size_t *take, const int *flush, int ncalls, int *status, size_t *out_len);
/* ---- the a18 helper kernels (src/zlib_simd_optimized.c:27,74,210,296) with
 * zlib-correct semantics: slide_hash (deflate.c:187-209), a 256-byte common
 * prefix, longest_match over a caller's window/prev (deflate.c:1356-1497, nice
 * = min(258, lookahead)), the LZ77 copy dest[i] = src[i % dist]. */
void zo_slide_hash(uint16_t *head, uint16_t *prev, uint32_t hash_size, uint32_t window_size,
                   uint32_t wsize);
uint32_t zo_compare256(const uint8_t *a, const uint8_t *b);
uint32_t zo_longest_match(const uint8_t *window, uint32_t strstart, uint32_t prev_length,
                          uint32_t good, uint32_t chain, uint32_t lookahead, const uint16_t *prev,
                          uint32_t wmask, uint32_t *match_start);
void zo_chunkmemset(uint8_t *dest, const uint8_t *src, uint32_t dist, uint32_t len);
/* ---- inflate (zinflate.c): inflate.c / inftrees.c / uncompr.c ----
 * wrap: 0 raw, 1 zlib, 2 gzip, 3 zlib or gzip (windowBits 15+32).
 * zo_inflate_run stops at the stream end (0), a data error (1), a preset
 * dictionary request (2), a full output (3) or the end of the input (4);
 * out_len = bytes written, consumed = input bytes inflate() has taken. */
int zo_inflate_run(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, int wrap,
                   size_t *out_len, size_t *consumed);
/* uncompress2 (uncompr.c:24-80) for any wrapper: ZO_OK / ZO_DATA_ERROR /
 * ZO_BUF_ERROR; *dst_len in: capacity, out: bytes written; *src_len in: input
 * length, out: bytes consumed */
int zo_uncompress3(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t *src_len, int wrap);
int zo_uncompress2(uint8_t *dst, size_t *dst_len, const uint8_t *src, size_t *src_len);
#endif
