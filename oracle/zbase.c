/*
 * zbase.c — TEST/BENCH INFRASTRUCTURE ONLY (never linked into the product path).
 *
 * The CPU baselines bench.py reports: the host's system zlib
 * (the upstream zlib the reference vendors; its level-6 streams are checked
 * byte-identical to the reference's on the sample before they are timed) run
 * over a bounded sample on T threads for a fixed time, with no Python in the
 * timed loop.
 *   zb_compress_rate   compress2() of whole buffers (compress.c:22-59), the
 *                      per-buffer work of a batched deflate
 *   zb_crc32_rate      crc32() of `chunk`-byte pieces (crc32.c:694-1010)
 *   zb_adler32_rate    adler32() of `chunk`-byte pieces (adler32.c:61-127)
 * Each returns MB/s (1e6 B/s) over the wall time of all threads and stores the
 * bytes processed in *done.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>
#include <zlib.h>

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

typedef struct {
    int kind;                       /* 0 compress2, 1 crc32, 2 adler32 */
    const uint8_t *const *bufs;
    const size_t *lens;
    int nbuf, level, tid, threads;
    size_t chunk;
    double deadline;
    uint64_t done;
    uint32_t sink;
    int err;
} zb_job;

static void *zb_run(void *arg) {
    zb_job *j = (zb_job *)arg;
    uint8_t *out = NULL;
    uLong cap = 0;
    if (j->kind == 0) {
        size_t mx = 0;
        for (int i = 0; i < j->nbuf; i++) if (j->lens[i] > mx) mx = j->lens[i];
        cap = compressBound((uLong)mx);
        out = (uint8_t *)malloc(cap);
        if (!out) { j->err = 1; return NULL; }
    }
    int k = j->tid;
    size_t off = 0;
    while (now_s() < j->deadline) {
        if (j->kind == 0) {
            const int b = k % j->nbuf;
            uLongf dl = cap;
            if (compress2(out, &dl, j->bufs[b], (uLong)j->lens[b], j->level) != Z_OK) { j->err = 1; break; }
            j->done += j->lens[b];
            j->sink ^= (uint32_t)dl;
            k += j->threads;
        } else {
            /* 64 pieces per deadline test; piece i of thread t at (t + i*T) * chunk */
            const size_t total = j->lens[0], pieces = total / j->chunk;
            for (int r = 0; r < 64; r++) {
                const size_t p = (size_t)(k % (int)pieces) * j->chunk;
                uint32_t v = j->kind == 1 ? (uint32_t)crc32(0L, j->bufs[0] + p, (uInt)j->chunk)
                                          : (uint32_t)adler32(1L, j->bufs[0] + p, (uInt)j->chunk);
                j->sink ^= v;
                j->done += j->chunk;
                k += j->threads;
            }
            (void)off;
        }
    }
    free(out);
    return NULL;
}

static double zb_rate(int kind, const uint8_t *const *bufs, const size_t *lens, int nbuf, int level,
                      size_t chunk, int threads, double seconds, uint64_t *done) {
    if (threads < 1) threads = 1;
    zb_job *jobs = (zb_job *)calloc((size_t)threads, sizeof(zb_job));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1.0; }
    const double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        jobs[t] = (zb_job){kind, bufs, lens, nbuf, level, t, threads, chunk, t0 + seconds, 0, 0, 0};
        pthread_create(&th[t], NULL, zb_run, &jobs[t]);
    }
    uint64_t tot = 0;
    int err = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        tot += jobs[t].done;
        err |= jobs[t].err;
    }
    const double el = now_s() - t0;
    free(jobs);
    free(th);
    if (done) *done = tot;
    return err ? -1.0 : (double)tot / el / 1e6;
}

double zb_compress_rate(const uint8_t *const *bufs, const size_t *lens, int nbuf, int level, int threads,
                        double seconds, uint64_t *done) {
    return zb_rate(0, bufs, lens, nbuf, level, 0, threads, seconds, done);
}

double zb_crc32_rate(const uint8_t *buf, size_t len, size_t chunk, int threads, double seconds, uint64_t *done) {
    const uint8_t *b[1] = {buf};
    size_t l[1] = {len};
    return zb_rate(1, b, l, 1, 0, chunk, threads, seconds, done);
}

double zb_adler32_rate(const uint8_t *buf, size_t len, size_t chunk, int threads, double seconds, uint64_t *done) {
    const uint8_t *b[1] = {buf};
    size_t l[1] = {len};
    return zb_rate(2, b, l, 1, 0, chunk, threads, seconds, done);
}

const char *zb_zlib_version(void) { return zlibVersion(); }
