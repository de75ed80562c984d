/*
 * zgpu.h — C ABI of libzgpu.so, the MI355X (gfx950) deflate / CRC-32 / Adler-32
 * hot path.  Plain pointers and sizes only; no torch, no HIP types.
 *
 * Three layers, all exported from one library:
 *
 *  1. Batched API (new; no reference equivalent, SURVEY §8b "New batched
 *     extension").  One independent stream per buffer; per-buffer semantics are
 *     exactly compress2() / crc32() / adler32() of the reference
 *     (compress.c:22-59, crc32.c:1015, adler32.c:128).
 *       *_dev   : inputs and outputs already resident in HBM (device pointers),
 *                 enqueued on the caller's HIP stream (`stream`, a hipStream_t,
 *                 NULL = default stream).
 *       host    : host buffers; staged over PCIe by the library.
 *
 *  2. zlib.h drop-in names (zgpu_zlib.h): compress2, compress, compressBound,
 *     deflateInit_/deflateInit2_/deflate/deflateEnd/deflateBound, uncompress,
 *     uncompress2, inflateInit_/inflateInit2_/inflate/inflateEnd/inflateReset,
 *     crc32, crc32_z, crc32_combine*, adler32, adler32_z, adler32_combine*,
 *     zlibVersion — replacing zlib.h:224-1836 of the reference.
 *
 *  3. The reference's WASM front-end exports (src/wasm_module.c:34-84,
 *     src/zlib_simd_compression.c:280,342, src/zlib_simd_optimized.c:27-409):
 *     zlib_compress_buffer, zlib_crc32, ... (zgpu_wasm.h).
 *
 * Every compute entry point runs on the GPU; there is no CPU fallback.  With no
 * usable GPU the calls return ZGPU_ENODEV (or Z_MEM_ERROR through the zlib
 * names) and print a diagnostic once.
 */
#ifndef ZGPU_H
#define ZGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: the zlib ones (zlib.h:181-190) plus one for "no GPU" */
#define ZGPU_OK            0
#define ZGPU_STREAM_ERROR (-2)
#define ZGPU_MEM_ERROR    (-4)
#define ZGPU_BUF_ERROR    (-5)
#define ZGPU_ENODEV      (-100)

/* stream wrappers: same meaning as windowBits -15 / 15 / 31 */
#define ZGPU_WRAP_RAW  0
#define ZGPU_WRAP_ZLIB 1
#define ZGPU_WRAP_GZIP 2

/* Library / device bring-up.  Idempotent; called implicitly by every entry
 * point.  Returns ZGPU_OK or ZGPU_ENODEV. */
int zgpu_init(void);
/* Human-readable build / device description (static storage). */
const char *zgpu_info(void);
/* Bytes of input processed per deflate sub-batch (workspace ≈ 16 B per input
 * byte).  Default 1 GiB.  Returns the previous value. */
size_t zgpu_set_inflight_bytes(size_t bytes);

/* Per-stage device timing for profiling: HIP events recorded on the launch
 * stream around every kernel of zgpu_deflate_batch_dev.  enable != 0 resets the
 * totals and starts collecting; enable == 0 stops.  zgpu_stage_timing_read
 * copies total milliseconds and launch counts for up to `nstages` stages:
 * 0 checksum (trailer), 1 links, 2 match, 3 lazy parse, 4 greedy parse,
 * 5 encode; for zgpu_inflate_batch_dev 3 decode, 4 match copy, 5 finish.
 * Returns the number of stages written. */
void zgpu_stage_timing(int enable);
int zgpu_stage_timing_read(double *ms, uint64_t *launches, int nstages);

/* ---------------- batched, device-resident ---------------- */

/* Compress `count` independent buffers.  Buffer i is src[src_off[i] ..
 * src_off[i]+src_len[i]) and is written to dst[dst_off[i] .. +dst_cap[i]).
 * On completion dst_len[i] = bytes written and status[i] = Z_OK, or
 * Z_BUF_ERROR with dst_len[i] = dst_cap[i] and the stream prefix written
 * (compress2 semantics, compress.c:44-58).  level: -1 (=6) or 0..9.
 * All arrays are device pointers; `stream` orders the work, and the call returns
 * once it is complete (the sub-batch planning reads src_len to the host). */
int zgpu_deflate_batch_dev(const uint8_t *src, const uint64_t *src_off,
                           const uint64_t *src_len, uint8_t *dst,
                           const uint64_t *dst_off, const uint64_t *dst_cap,
                           uint64_t *dst_len, int32_t *status, uint32_t count,
                           int level, int wrap, void *stream);

/* zgpu_deflate_batch_dev with a deflateInit2_ strategy (zlib.h:197-201):
 * 0 default, 1 Z_FILTERED, 2 Z_HUFFMAN_ONLY, 3 Z_RLE, 4 Z_FIXED; per buffer the
 * output equals deflateInit2_(level, Z_DEFLATED, windowBits of `wrap`, 8,
 * strategy) + deflate(Z_FINISH). */
int zgpu_deflate_batch_dev_ex(const uint8_t *src, const uint64_t *src_off,
                              const uint64_t *src_len, uint8_t *dst,
                              const uint64_t *dst_off, const uint64_t *dst_cap,
                              uint64_t *dst_len, int32_t *status, uint32_t count,
                              int level, int wrap, int strategy, void *stream);

/* zgpu_deflate_batch_dev with all of deflateInit2_'s parameters (zlib.h:
 * 553-626, deflate.c:379-524): per buffer the output equals
 * deflateInit2_(level, Z_DEFLATED, window_bits, mem_level, strategy) +
 * deflate(Z_FINISH).  window_bits 8..15 (zlib wrapper; 8 is coded as 9),
 * -15..-9 (raw), 25..31 (gzip); mem_level 1..9 (hash_bits = mem_level + 7,
 * lit_bufsize = 1 << (mem_level + 6)).  Others: ZGPU_STREAM_ERROR. */
int zgpu_deflate_batch_dev2(const uint8_t *src, const uint64_t *src_off,
                            const uint64_t *src_len, uint8_t *dst,
                            const uint64_t *dst_off, const uint64_t *dst_cap,
                            uint64_t *dst_len, int32_t *status, uint32_t count,
                            int level, int window_bits, int mem_level, int strategy,
                            void *stream);

/* crc32(init[i], buffer i) for each buffer (init == NULL: 0).  Device ptrs. */
int zgpu_crc32_batch_dev(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                         const uint32_t *init, uint32_t *out, uint32_t count,
                         void *stream);
/* adler32(init[i], buffer i) for each buffer (init == NULL: 1).  Device ptrs. */
int zgpu_adler32_batch_dev(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                           const uint32_t *init, uint32_t *out, uint32_t count,
                           void *stream);

/* Decompress `count` independent streams (the other half of the wire format,
 * SURVEY §8f row 2).  Stream i is src[src_off[i] .. +src_len[i]) and is
 * inflated into dst[dst_off[i] .. +dst_cap[i]).  Per stream the result is what
 * the reference's uncompress2 (uncompr.c:24-85) returns for that input and
 * capacity, for wrap 1 (zlib) exactly, and for the other wrappers with
 * inflateInit2_(-15 raw / 31 gzip / 47 zlib-or-gzip) in the same loop:
 *   status[i]   Z_OK, Z_DATA_ERROR (corrupt, truncated, preset dictionary) or
 *               Z_BUF_ERROR (the output filled up before the stream ended);
 *   dst_len[i]  bytes written (the decodable prefix on errors; 0 when
 *               dst_cap[i] == 0, uncompress2's 1-byte probe);
 *   src_used[i] input bytes consumed (may be NULL).
 * wrap: ZGPU_WRAP_RAW / _ZLIB / _GZIP, or ZGPU_WRAP_AUTO (zlib or gzip header).
 * Each stream's src_len and dst_cap must be < 4 GiB (else ZGPU_STREAM_ERROR).
 * Device pointers, ordered on `stream`; returns when complete. */
#define ZGPU_WRAP_AUTO 3
int zgpu_inflate_batch_dev(const uint8_t *src, const uint64_t *src_off,
                           const uint64_t *src_len, uint8_t *dst,
                           const uint64_t *dst_off, const uint64_t *dst_cap,
                           uint64_t *dst_len, uint64_t *src_used, int32_t *status,
                           uint32_t count, int wrap, void *stream);

/* ---------------- batched, host buffers ---------------- */

/* Host-memory form of zgpu_deflate_batch_dev; dst_len[i] is in: capacity,
 * out: bytes written; status[i] as above.  Synchronous. */
int zgpu_compress_batch(const uint8_t *const *src, const size_t *src_len,
                        uint8_t *const *dst, size_t *dst_len, int *status,
                        size_t count, int level, int wrap);
/* Host-memory form with a strategy (see zgpu_deflate_batch_dev_ex). */
int zgpu_compress_batch_ex(const uint8_t *const *src, const size_t *src_len,
                           uint8_t *const *dst, size_t *dst_len, int *status,
                           size_t count, int level, int wrap, int strategy);
/* Host-memory form of zgpu_deflate_batch_dev2. */
int zgpu_compress_batch2(const uint8_t *const *src, const size_t *src_len,
                         uint8_t *const *dst, size_t *dst_len, int *status,
                         size_t count, int level, int window_bits, int mem_level,
                         int strategy);
/* Host-memory form of zgpu_inflate_batch_dev: dst_len[i] in: capacity, out:
 * bytes written; src_used may be NULL.  Synchronous. */
int zgpu_uncompress_batch(const uint8_t *const *src, const size_t *src_len,
                          uint8_t *const *dst, size_t *dst_len, size_t *src_used,
                          int *status, size_t count, int wrap);
int zgpu_crc32_batch(const uint8_t *const *src, const size_t *len,
                     const uint32_t *init, uint32_t *out, size_t count);
int zgpu_adler32_batch(const uint8_t *const *src, const size_t *len,
                       const uint32_t *init, uint32_t *out, size_t count);

/* The zlib.h checksums crc32()/crc32_z()/adler32()/adler32_z() have no error
 * return.  When their GPU call fails they return 0, set errno = EIO and keep
 * the library's error code (ZGPU_ENODEV, ZGPU_MEM_ERROR, ...) for this thread:
 * zgpu_checksum_error() returns it (ZGPU_OK when none failed since the last
 * reset; reset != 0 clears it).  ZGPU_CHECKSUM_ERROR=abort ends the process
 * instead. */
int zgpu_checksum_error(int reset);

/* ---------------- synthetic workloads (benchmark inputs) ---------------- */

/* Fill `count` buffers of `len` bytes each, laid out back to back at dst
 * (device pointer), with the seeded generator of DESIGN.md §"Workloads":
 * kind 0 = uniform random bytes (C2), 1 = Silesia-style 64 KiB-segment mix
 * (C4), 2 = enwik-style text/markup (C3), 3 = small-vocabulary text (C5).
 * Buffer i is a pure function of (kind, seed, first_index + i, len). */
int zgpu_generate_dev(uint8_t *dst, uint64_t len, uint32_t count, int kind,
                      uint64_t seed, uint64_t first_index, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* ZGPU_H */
