/*
 * zgpu_zlib.h — zlib.h-compatible compression ABI exported by libzgpu.so.
 *
 * A program built against the reference's zlib.h (zlib 1.3.1.1-motley) for the
 * compression side can link libzgpu.so instead of libz: same symbol names, same
 * signatures, same z_stream layout, same return codes.  Each declaration cites
 * the reference prototype it replaces.
 *
 * uncompress()/uncompress2() return what the reference returns for every input
 * (valid, corrupt, truncated, short output), with the same output and the same
 * consumed length.  inflate() decodes whenever input arrives and hands out
 * every byte decoded so far; each attempt resumes at a block boundary with the
 * 32 KiB window carried (linear in the stream), and the trailer is checked as
 * inflate.c does.  A call whose output space ends first consumes the input
 * inflate.c would (up to the codes of the symbol it has no room for) and hands
 * the rest back in next_in / avail_in.  inflateSetDictionary() answers Z_NEED_DICT
 * (zlib streams) or presets a raw stream's window before its first input.
 *
 * deflate() semantics: deflateInit2_ accepts windowBits 8..15 (zlib), -9..-15
 * (raw), 25..31 (gzip), memLevel 1..9 and every strategy (Z_DEFAULT_STRATEGY,
 * Z_FILTERED, Z_HUFFMAN_ONLY, Z_RLE, Z_FIXED); the stream is allocated through
 * zalloc/zfree.  Every call does what the reference's call does, levels 1..9:
 * the header on the first call, the blocks completed before a Z_NO_FLUSH call's
 * need_more point, a flush call's blocks and marker (Z_PARTIAL_FLUSH,
 * Z_SYNC_FLUSH, Z_FULL_FLUSH, Z_BLOCK; refused repeats with Z_BUF_ERROR), the
 * last block and trailer at Z_FINISH -- and it stops after a block when
 * avail_out is used up, consuming only the input the reference had read by
 * then (avail_in / total_in).  The parse runs on the GPU, one job per call that
 * can complete a block, resumed at the last block cut handed out.  Level 0:
 * deflate_stored's blocks as the reference cuts them, by min_block and by the
 * output space of each call (a small avail_out gives shorter blocks through the
 * pending buffer, deflate.c:1635-1815; tests/golden/stream_golden.json holds
 * 28 level-0 sessions with output buffers from 1 byte up).  After Z_FINISH the
 * caller continues with Z_FINISH until Z_STREAM_END (zlib.h); a flush call
 * that ran out of output space and is given more input instead of the same
 * flush again goes on as the reference does (tests/test_gpu_fuzz.py).  A first
 * call whose output space is exactly the header goes as the reference's does,
 * with a preset dictionary too, except a flush call whose input's first string
 * is in the dictionary (refused, below).
 * deflateSetDictionary, deflateSetHeader, deflatePrime, deflateTune and
 * deflateParams give the reference's stream: deflateParams flushes with Z_BLOCK
 * itself when the level's function or the strategy changes (as deflate.c does)
 * and switches between level 0, deflate_fast and deflate_slow levels, and
 * between deflate_slow or deflate_fast levels and Z_HUFFMAN_ONLY / Z_RLE
 * (gzsetparams' pattern; back to the function the stretch began from); a level
 * change within one function, and deflateTune, take effect at the next decision
 * even with input pending.  What the model cannot place returns Z_STREAM_ERROR
 * with strm->msg set, never a different stream (zgpu_api.cpp, `unsupported`):
 *   - deflateParams to or from Z_HUFFMAN_ONLY / Z_RLE after data other than
 *     between deflate_slow levels (4..9, memLevel <= 8) or deflate_fast
 *     levels (1..3) and those strategies and back to the same function, and
 *     back after a first call of a single byte;
 *   - deflatePrime after a call that stopped on a full output buffer (or with
 *     output pending) when its bits complete a byte: the reference writes
 *     that byte inside its pending output (put_byte at pending_buf[pending])
 *     and ends the stream with a stale buffer byte; bits that complete none
 *     are modelled.  Also after a flush call that did not reach its marker,
 *     and after Z_STREAM_END;
 *   - deflateSetDictionary after the stream has ended;
 *   - deflateResetKeep on a stream that has taken input, except after a
 *     stream that deflate_slow (levels 4..9, not Z_HUFFMAN_ONLY / Z_RLE) ran
 *     from its part start to a point with no input pending (the end of
 *     Z_FINISH, or a flush that took all its input): that window is carried
 *     into the next stream as the reference carries it; then a preset
 *     dictionary, or a switch to level 0 or to a deflate_fast level before the
 *     next input, is refused;
 *   - a first deflate() flush call whose output space is exactly a preset
 *     dictionary's 6-byte header, with the input's first three bytes in the
 *     dictionary (or a Z_NO_FLUSH one whose first read could fill a block
 *     before its first literal);
 *   - inflatePrime other than on a raw stream before its first input.
 * inflateUndermine returns Z_DATA_ERROR (as a reference built without
 * INFLATE_ALLOW_INVALID_DISTANCE_TOOFAR_ARRR does).  inflateBack reports a
 * distance beyond its window at the first such distance; where out() fails,
 * the input left in next_in / avail_in may differ from the reference's (whose
 * bit buffer has pulled bytes ahead).
 */
#ifndef ZGPU_ZLIB_H
#define ZGPU_ZLIB_H

#include "zgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned char Bytef;
typedef unsigned int uInt;
typedef unsigned long uLong;
typedef uLong uLongf;
typedef void *voidpf;
typedef voidpf (*alloc_func)(voidpf opaque, uInt items, uInt size);
typedef void (*free_func)(voidpf opaque, voidpf address);

/* z_stream, field for field as zlib.h:90-110 */
typedef struct z_stream_s {
    const Bytef *next_in;
    uInt avail_in;
    uLong total_in;
    Bytef *next_out;
    uInt avail_out;
    uLong total_out;
    const char *msg;
    struct internal_state *state;
    alloc_func zalloc;
    free_func zfree;
    voidpf opaque;
    int data_type;
    uLong adler;
    uLong reserved;
} z_stream;
typedef z_stream *z_streamp;

/* zlib.h:172-204 */
#define Z_NO_FLUSH      0
#define Z_PARTIAL_FLUSH 1
#define Z_SYNC_FLUSH    2
#define Z_FULL_FLUSH    3
#define Z_FINISH        4
#define Z_BLOCK         5
#define Z_TREES         6
#define Z_OK            0
#define Z_STREAM_END    1
#define Z_NEED_DICT     2                                                  /* zlib.h:183 */
#define Z_DATA_ERROR   (-3)
#define Z_STREAM_ERROR (-2)
#define Z_MEM_ERROR    (-4)
#define Z_BUF_ERROR    (-5)
#define Z_VERSION_ERROR (-6)
#define Z_DEFAULT_COMPRESSION (-1)
#define Z_FILTERED            1                                        /* zlib.h:197-201 */
#define Z_HUFFMAN_ONLY        2
#define Z_RLE                 3
#define Z_FIXED               4
#define Z_DEFAULT_STRATEGY    0
#define Z_DEFLATED 8
#define Z_UNKNOWN 2

#define ZGPU_ZLIB_VERSION "1.3.1.1-motley"

const char *zlibVersion(void);                                          /* zlib.h:224 */
int deflateInit_(z_streamp strm, int level, const char *version,
                 int stream_size);                                      /* zlib.h:1803 */
int deflateInit2_(z_streamp strm, int level, int method, int windowBits,
                  int memLevel, int strategy, const char *version,
                  int stream_size);                                     /* zlib.h:1807 */
int deflate(z_streamp strm, int flush);                                 /* zlib.h:254 */
int deflateEnd(z_streamp strm);                                         /* zlib.h:367 */
uLong deflateBound(z_streamp strm, uLong sourceLen);                    /* zlib.h:694 */
int deflateReset(z_streamp strm);                                       /* zlib.h:621 */
int deflateCopy(z_streamp dest, z_streamp source);                      /* zlib.h:603 */
int deflatePending(z_streamp strm, unsigned *pending, int *bits);       /* zlib.h:746 */
int deflateUsed(z_streamp strm, int *bits);                             /* zlib.h deflateUsed; deflate.c:723 */
int deflateGetDictionary(z_streamp strm, Bytef *dictionary,
                         uInt *dictLength);                             /* zlib.h deflateGetDictionary; deflate.c:616 */
int deflateResetKeep(z_streamp strm);                                   /* zlib.h deflateResetKeep; deflate.c:635 */

/* gzip header (zlib.h gz_header) for deflateSetHeader / inflateGetHeader */
typedef struct gz_header_s {
    int text;
    uLong time;
    int xflags;
    int os;
    Bytef *extra;
    uInt extra_len;
    uInt extra_max;
    Bytef *name;
    uInt name_max;
    Bytef *comment;
    uInt comm_max;
    int hcrc;
    int done;
} gz_header;
typedef gz_header *gz_headerp;

int deflateSetDictionary(z_streamp strm, const Bytef *dictionary,
                         uInt dictLength);                              /* zlib.h deflateSetDictionary; deflate.c */
int deflateParams(z_streamp strm, int level, int strategy);            /* zlib.h deflateParams; deflate.c */
int deflateTune(z_streamp strm, int good_length, int max_lazy,
                int nice_length, int max_chain);                        /* zlib.h deflateTune; deflate.c */
int deflatePrime(z_streamp strm, int bits, int value);                 /* zlib.h deflatePrime; deflate.c */
int deflateSetHeader(z_streamp strm, gz_headerp head);                 /* zlib.h deflateSetHeader; deflate.c */
int inflateSetDictionary(z_streamp strm, const Bytef *dictionary,
                         uInt dictLength);                              /* zlib.h inflateSetDictionary; inflate.c */
int compress(Bytef *dest, uLongf *destLen, const Bytef *source,
             uLong sourceLen);                                          /* zlib.h:1251 */
int compress2(Bytef *dest, uLongf *destLen, const Bytef *source,
              uLong sourceLen, int level);                              /* zlib.h:1266 */
uLong compressBound(uLong sourceLen);                                   /* zlib.h:1282 */
/* crc32 / crc32_z / adler32 / adler32_z run on the GPU.  A failed GPU call
 * returns 0 with errno = EIO; zgpu_checksum_error() (zgpu.h) names the
 * error.  ZGPU_CHECKSUM_ERROR=abort ends the process instead. */
uLong adler32(uLong adler, const Bytef *buf, uInt len);                 /* zlib.h:1711 */
uLong adler32_z(uLong adler, const Bytef *buf, size_t len);             /* zlib.h:1731 */
uLong adler32_combine(uLong adler1, uLong adler2, long len2);           /* zlib.h:1738 */
uLong adler32_combine64(uLong adler1, uLong adler2, int64_t len2);
uLong crc32(uLong crc, const Bytef *buf, uInt len);                     /* zlib.h:1749 */
uLong crc32_z(uLong crc, const Bytef *buf, size_t len);                 /* zlib.h:1767 */
uLong crc32_combine(uLong crc1, uLong crc2, long len2);                 /* zlib.h:1774 */
uLong crc32_combine64(uLong crc1, uLong crc2, int64_t len2);
uLong crc32_combine_gen(long len2);                                     /* zlib.h:1784 */
uLong crc32_combine_gen64(int64_t len2);
uLong crc32_combine_op(uLong crc1, uLong crc2, uLong op);               /* zlib.h:1790 */
const char *zError(int err);                                            /* zlib.h zError; zutil.c:131 */
uLong zlibCompileFlags(void);                                           /* zlib.h zlibCompileFlags; zutil.c:31 */
const uint32_t *get_crc_table(void);                                    /* zlib.h get_crc_table; crc32.c:549 */

int uncompress(Bytef *dest, uLongf *destLen, const Bytef *source,
               uLong sourceLen);                                        /* zlib.h:1289 */
int uncompress2(Bytef *dest, uLongf *destLen, const Bytef *source,
                uLong *sourceLen);                                      /* zlib.h:1307 */
int inflateInit_(z_streamp strm, const char *version, int stream_size); /* zlib.h:1805 */
/* windowBits 8..15 zlib, -8..-15 raw, +16 gzip, +32 zlib or gzip (zlib.h:853) */
int inflateInit2_(z_streamp strm, int windowBits, const char *version,
                  int stream_size);                                     /* zlib.h:1811 */
int inflate(z_streamp strm, int flush);                                 /* zlib.h:405 */
int inflateEnd(z_streamp strm);                                         /* zlib.h:525 */
int inflateReset(z_streamp strm);                                       /* zlib.h:980 */
int inflateGetHeader(z_streamp strm, gz_headerp head);                  /* zlib.h inflateGetHeader; inflate.c:1330 */
int inflateSync(z_streamp strm);                                        /* zlib.h inflateSync; inflate.c:1375 */
int inflateCopy(z_streamp dest, z_streamp source);                      /* zlib.h inflateCopy; inflate.c:1439 */
/* inflate(flush): Z_NO_FLUSH, Z_SYNC_FLUSH, Z_FINISH (Z_BUF_ERROR short of the
 * stream end), Z_BLOCK (stop at the next block boundary, or after a zlib / gzip
 * header; strm->data_type as inflate.c sets it there) and Z_TREES (also after
 * each block header, data_type + 256).  inflateSync searches the whole bytes
 * the reference holds in its bit buffer first (inflate.c:1388-1398). */
int inflateReset2(z_streamp strm, int windowBits);                      /* zlib.h inflateReset2; inflate.c:153 */
int inflateResetKeep(z_streamp strm);                                   /* zlib.h inflateResetKeep; inflate.c:105 */
int inflatePrime(z_streamp strm, int bits, int value);                  /* zlib.h inflatePrime; inflate.c:223
                                                                           (raw streams before their first input) */
int inflateGetDictionary(z_streamp strm, Bytef *dictionary,
                         uInt *dictLength);                             /* zlib.h inflateGetDictionary; inflate.c:1278 */
int inflateSyncPoint(z_streamp strm);                                   /* zlib.h inflateSyncPoint; inflate.c:1431 */
int inflateUndermine(z_streamp strm, int subvert);                      /* zlib.h inflateUndermine; inflate.c:1483 */
int inflateValidate(z_streamp strm, int check);                         /* zlib.h inflateValidate; inflate.c:1498 */
long inflateMark(z_streamp strm);                                       /* zlib.h inflateMark; inflate.c:1510 */
unsigned long inflateCodesUsed(z_streamp strm);                         /* zlib.h inflateCodesUsed; inflate.c:1521 */
typedef unsigned (*in_func)(void *, const unsigned char **);            /* zlib.h in_func */
typedef int (*out_func)(void *, unsigned char *, unsigned);             /* zlib.h out_func */
int inflateBackInit_(z_streamp strm, int windowBits, unsigned char *window,
                     const char *version, int stream_size);             /* zlib.h inflateBackInit_; infback.c:25 */
int inflateBack(z_streamp strm, in_func in, void *in_desc,
                out_func out, void *out_desc);                          /* zlib.h inflateBack; infback.c:250 */
int inflateBackEnd(z_streamp strm);                                     /* zlib.h inflateBackEnd; infback.c:632 */
#define inflateBackInit(strm, windowBits, window) \
    inflateBackInit_((strm), (windowBits), (window), ZGPU_ZLIB_VERSION, (int)sizeof(z_stream))

#define inflateInit(strm) \
    inflateInit_((strm), ZGPU_ZLIB_VERSION, (int)sizeof(z_stream))
#define inflateInit2(strm, windowBits) \
    inflateInit2_((strm), (windowBits), ZGPU_ZLIB_VERSION, (int)sizeof(z_stream))
#define deflateInit(strm, level) \
    deflateInit_((strm), (level), ZGPU_ZLIB_VERSION, (int)sizeof(z_stream))
#define deflateInit2(strm, level, method, windowBits, memLevel, strategy) \
    deflateInit2_((strm), (level), (method), (windowBits), (memLevel), \
                  (strategy), ZGPU_ZLIB_VERSION, (int)sizeof(z_stream))

#ifdef __cplusplus
}
#endif
#endif /* ZGPU_ZLIB_H */
