// zgpu_api.cpp — host side of libzgpu.so: device bring-up, static tables,
// sub-batch orchestration of the deflate pipeline, and the three exported
// C ABIs (batched zgpu_*, zlib.h names, the reference's WASM front-end names).
//
// Every compute path runs on the GPU.  There is deliberately no CPU fallback:
// with no usable device every entry point fails (ZGPU_ENODEV / Z_MEM_ERROR)
// after printing one diagnostic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cerrno>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "zgpu_internal.h"
#include "../../include/zgpu.h"
#include "../../include/zgpu_zlib.h"
#include "../../include/zgpu_wasm.h"
#include "../../include/zgpu_debug.h"

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

// debug (ZGPU_SEGV_TRACE): a host backtrace of the library on SIGSEGV
namespace {
void segv_backtrace(int sig) {
    void *a[64];
    const int n = backtrace(a, 64);
    backtrace_symbols_fd(a, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
__attribute__((constructor)) void install_segv_backtrace() {
    if (std::getenv("ZGPU_SEGV_TRACE")) signal(SIGSEGV, segv_backtrace);
}
}  // namespace

using namespace zgpu;

namespace {

// ------------------------------------------------------------------------
// host restatement of the table derivations (trees.c:303-396, crc32.c)
// ------------------------------------------------------------------------
constexpr uint32_t kPoly = 0xedb88320u;

uint32_t multmodp(uint32_t a, uint32_t b) {                  // crc32.c:155-170
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) { p ^= b; if ((a & (m - 1)) == 0) break; }
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}
uint32_t x2nmodp(int64_t n, unsigned k) {                     // crc32.c:176-187
    static uint32_t x2n[32];
    static std::once_flag once;
    std::call_once(once, [] {
        uint32_t p = 1u << 30;
        x2n[0] = p;
        for (int i = 1; i < 32; i++) x2n[i] = p = multmodp(p, p);
    });
    uint32_t p = 1u << 31;
    while (n) {
        if (n & 1) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}

// configuration_table (deflate.c:112-125): good, lazy, nice, chain
const LevelCfg kLevelCfg[10] = {{0, 0, 0, 0},      {4, 4, 8, 4},       {4, 5, 16, 8},
                                {4, 6, 32, 32},    {4, 4, 16, 16},    {8, 16, 32, 32},
                                {8, 16, 128, 128}, {8, 32, 128, 256}, {32, 128, 258, 1024},
                                {32, 258, 258, 4096}};

unsigned bitrev(unsigned code, int len) {
    unsigned r = 0;
    while (len-- > 0) { r = (r << 1) | (code & 1u); code >>= 1; }
    return r;
}

void build_code_tables(CodeTables &t) {
    std::memset(&t, 0, sizeof t);
    static const uint8_t xl[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
    static const uint8_t xd[30] = {0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};
    static const uint8_t xb[19] = {0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,2,3,7};
    static const uint8_t bo[19] = {16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15};
    std::memcpy(t.xlbits, xl, 29);
    std::memcpy(t.xdbits, xd, 30);
    std::memcpy(t.xblbits, xb, 19);
    std::memcpy(t.bl_order, bo, 19);
    int length = 0, code;
    for (code = 0; code < 28; code++) {
        t.len_base[code] = (uint16_t)length;
        for (int k = 0; k < (1 << xl[code]); k++) t.len_code[length++] = (uint8_t)code;
    }
    t.len_code[255] = 28;
    t.len_base[28] = 0;
    int dist = 0;
    for (code = 0; code < 16; code++) {
        t.dist_base[code] = (uint16_t)dist;
        for (int k = 0; k < (1 << xd[code]); k++) t.dist_code[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < 30; code++) {
        t.dist_base[code] = (uint16_t)(dist << 7);
        for (int k = 0; k < (1 << (xd[code] - 7)); k++) t.dist_code[256 + dist++] = (uint8_t)code;
    }
    uint16_t cnt[16] = {0};
    for (int n = 0; n < 288; n++) {
        t.stat_llen[n] = (uint8_t)(n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8);
        cnt[t.stat_llen[n]]++;
    }
    uint16_t next[16];
    unsigned c = 0;
    for (int b = 1; b <= 15; b++) { c = (c + cnt[b - 1]) << 1; next[b] = (uint16_t)c; }
    for (int n = 0; n < 288; n++) t.stat_lcode[n] = (uint16_t)bitrev(next[t.stat_llen[n]]++, t.stat_llen[n]);
    for (int n = 0; n < 30; n++) t.stat_dcode[n] = (uint16_t)bitrev((unsigned)n, 5);
    for (int n = 0; n < 30; n++) t.stat_dlen[n] = 5;
    std::memcpy(t.cfg, kLevelCfg, sizeof kLevelCfg);
}

void build_crc_tables(CrcTables &t) {
    for (uint32_t v = 0; v < 256; v++) {
        uint32_t c = v;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? kPoly ^ (c >> 1) : c >> 1;
        t.byte[v] = c;
    }
    auto raw_crc = [&](const uint8_t *m, int len) {
        uint32_t c = 0;
        for (int i = 0; i < len; i++) c = (c >> 8) ^ t.byte[(c ^ m[i]) & 0xffu];
        return c;
    };
    for (int j = 0; j < 32; j++)
        for (uint32_t v = 0; v < 16; v++) {
            uint8_t msg[16] = {0};
            msg[j >> 1] = (uint8_t)(v << (4 * (j & 1)));
            t.nib[j][v] = raw_crc(msg, 16);
        }
    const uint64_t amounts[kCrcShiftTabs] = {16, 32, 64, 128, 256, 512, 1024, kCrcSegment};
    for (int k = 0; k < kCrcShiftTabs; k++) {
        const uint32_t op = x2nmodp((int64_t)amounts[k], 3);
        for (int j = 0; j < 8; j++)
            for (uint32_t v = 0; v < 16; v++) t.shift[k][j][v] = multmodp(op, v << (4 * j));
    }
    for (uint32_t v = 0; v < 256; v++) t.s4[0][v] = t.byte[v];
    for (int k = 1; k < 4; k++)
        for (uint32_t v = 0; v < 256; v++) {
            const uint32_t c = t.s4[k - 1][v];
            t.s4[k][v] = (c >> 8) ^ t.byte[c & 0xffu];
        }
    for (int i = 0; i < 48; i++) t.xrow[i] = x2nmodp((int64_t)(kCrcRow << i), 3);
    const uint64_t a64[kCrcSh64Tabs] = {64, 128, 256, 512, 1024, 2048, 64 * 15, 64 * 63};
    for (int k = 0; k < kCrcSh64Tabs; k++) {
        const uint32_t op = x2nmodp((int64_t)a64[k], 3);
        for (int j = 0; j < 8; j++)
            for (uint32_t v = 0; v < 16; v++) t.sh64[k][j][v] = multmodp(op, v << (4 * j));
    }
}

// ------------------------------------------------------------------------
// device context
// ------------------------------------------------------------------------
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    bool ensure(size_t bytes) {
        if (bytes <= cap) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 8 + 4096;
        if (hipMalloc(&p, want) != hipSuccess) { p = nullptr; return false; }
        cap = want;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
};

constexpr int kStages = 6;

struct StageTimer {
    bool on = false;
    double ms[kStages] = {0};
    uint64_t n[kStages] = {0};
    std::vector<hipEvent_t> pool;
    std::vector<std::pair<int, int>> pending;   // (stage, event pair index)
    size_t used = 0;
    hipEvent_t ev(size_t i) {
        while (pool.size() <= i) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[i];
    }
    // wraps one launch; returns the launcher's result
    template <typename F> int run(int stage, hipStream_t st, F &&launch) {
        if (!on) return launch();
        hipEvent_t a = ev(used), b = ev(used + 1);
        if (a) (void)hipEventRecord(a, st);
        int rc = launch();
        if (b) (void)hipEventRecord(b, st);
        if (a && b) pending.push_back({stage, (int)used});
        used += 2;
        return rc;
    }
    void collect() {     // after the stream has been synchronised
        for (auto &pe : pending) {
            float t = 0;
            if (hipEventElapsedTime(&t, pool[pe.second], pool[pe.second + 1]) == hipSuccess) {
                ms[pe.first] += t;
                n[pe.first]++;
            }
        }
        pending.clear();
        used = 0;
    }
};

struct Ctx {
    bool busy = false;
    int device = 0;
    hipStream_t own = nullptr;   // the stream of the host-buffer entry points
    StageTimer timer;
    uint64_t timer_epoch = 0;
    size_t inflight = size_t(1) << 30;
    DevBuf ws_link, ws_rf, ws_rq, ws_sym, ws_blk, ws_meta, ws_heads, ws_io, ws_io2, ws_small, ws_state;
    // second workspace slot and stream for the L4-9 pipeline (k_match of
    // sub-batch i+1 runs on `aux` while links/parse/encode run on the caller's
    // stream)
    DevBuf ws_link2, ws_rf2, ws_rq2, ws_state2;
    DevBuf ws_sym2, ws_blk2;  // k_lzp (the walks and the parse of slot 1 beside the encode of slot 0)
    DevBuf ws_key, ws_key2;   // k_count's walk-length keys (one byte per position)
    DevBuf ws_stg;            // k_parse_seg's symbol staging (caller's stream only)
    DevBuf ws_help;           // the a18 helpers' staging (zlib_*_simd)
    DevBuf ws_seg;            // k_match segments of sub-batches of few large buffers
    // few large buffers: k_pbig* lane groups and records, k_enc_* block plans
    DevBuf ws_pg, ws_plane, ws_pbuf, ws_eplan, ws_wind, ws_tl, ws_pron;
    DevBuf ws_ck;             // split checksum partials (few large buffers)
    DevBuf ws_srec, ws_snap;  // a streaming job's block records and head[] snapshot
    DevBuf ws_srt, ws_boff, ws_work, ws_bblk;   // the sorted-run parse of levels 2..3 (k_bsort / k_bwork / k_parse_srt)
    // inflate: match records, per-stream results, checks, offsets, stop codes
    DevBuf ws_mrec, ws_irec, ws_ick, ws_imeta, ws_istop;
    DevBuf ws_iidx;           // the streaming inflate()'s consumption index (InflateJob::eidx / bidx)
    // the block-parallel decode of a lone stream (inflate_par): candidate lists,
    // per-block jobs and records, output symbols
    DevBuf ws_par1, ws_par2, ws_pjob, ws_psym, ws_pslot;
    hipStream_t aux = nullptr;
    hipEvent_t ev_links[2] = {nullptr, nullptr}, ev_match[2] = {nullptr, nullptr};
    // pinned host staging of single small crc32()/adler32() calls (checksum_small)
    uint8_t *pin = nullptr;
};

// One entry per HIP device: its static tables and a pool of contexts.  A call
// leases a free context of the caller's current device (creating one, up to
// kMaxCtx, when all are busy), so host threads run side by side on their own
// streams and workspaces instead of queueing on one lock (zlib.h:150-151:
// zlib is thread-safe).
constexpr int kMaxDevices = 64;
constexpr size_t kMaxCtx = 8;
struct Device {
    std::mutex mu;
    std::condition_variable cv;
    int state = 0;            // 0 uninit, 1 ok, -1 failed
    std::string info;
    CrcTables *d_crc = nullptr;
    std::vector<std::unique_ptr<Ctx>> pool;
};
Device g_dev[kMaxDevices];
std::atomic<size_t> g_inflight{size_t(1) << 30};
std::atomic<bool> g_timing{false};
std::atomic<uint64_t> g_timing_epoch{0};
std::atomic<bool> g_nodev_said{false};

int nodev(const char *why) {
    if (!g_nodev_said.exchange(true))
        std::fprintf(stderr, "libzgpu: %s; the GPU path cannot run (no CPU fallback)\n", why);
    return ZGPU_ENODEV;
}

int current_device(int *d) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return nodev("no HIP device available");
    if (hipGetDevice(d) != hipSuccess || *d < 0 || *d >= kMaxDevices) return nodev("no current HIP device");
    return ZGPU_OK;
}

// first use of device d (D.mu held, d current)
int init_device_locked(Device &D, int d) {
    if (D.state == 1) return ZGPU_OK;
    if (D.state == -1) return ZGPU_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess) { D.state = -1; return nodev("device query failed"); }
    D.info = std::string("libzgpu gfx950 build; device ") + std::to_string(d) + ": " + prop.name + " (" +
             prop.gcnArchName + "), " + std::to_string(prop.multiProcessorCount) + " CUs";
    CodeTables ct;
    build_code_tables(ct);
    static CrcTables crc;
    static std::once_flag crc_once;
    std::call_once(crc_once, [] { build_crc_tables(crc); });
    if (launch_tables_upload(&ct, &crc) != 0 || hipMalloc(&D.d_crc, sizeof(CrcTables)) != hipSuccess ||
        hipMemcpy(D.d_crc, &crc, sizeof(CrcTables), hipMemcpyHostToDevice) != hipSuccess) {
        D.state = -1;
        return nodev("table upload failed");
    }
    static std::once_flag env_once;
    std::call_once(env_once, [] {
        if (const char *e = std::getenv("ZGPU_INFLIGHT_MB")) g_inflight = size_t(std::atoll(e)) << 20;
    });
    D.state = 1;
    return ZGPU_OK;
}

// RAII lease of a context on the caller's current device; rc != 0: no context
struct Lease {
    Ctx *c = nullptr;
    Device *D = nullptr;
    int rc = ZGPU_ENODEV;
    Lease() {
        int d = 0;
        if ((rc = current_device(&d))) return;
        D = &g_dev[d];
        std::unique_lock<std::mutex> g(D->mu);
        if ((rc = init_device_locked(*D, d))) return;
        for (;;) {
            for (auto &p : D->pool)
                if (!p->busy) { c = p.get(); break; }
            if (c) break;
            if (D->pool.size() < kMaxCtx) {
                auto p = std::make_unique<Ctx>();
                p->device = d;
                if (hipStreamCreateWithFlags(&p->own, hipStreamNonBlocking) != hipSuccess) {
                    rc = ZGPU_MEM_ERROR;
                    return;
                }
                D->pool.push_back(std::move(p));
                c = D->pool.back().get();
                break;
            }
            D->cv.wait(g);
        }
        c->busy = true;
        c->inflight = g_inflight;
        const uint64_t ep = g_timing_epoch;
        if (c->timer_epoch != ep) {        // zgpu_stage_timing(1) since this context last ran
            for (int i = 0; i < kStages; i++) { c->timer.ms[i] = 0; c->timer.n[i] = 0; }
            c->timer.pending.clear();
            c->timer.used = 0;
            c->timer_epoch = ep;
        }
        c->timer.on = g_timing;
        rc = ZGPU_OK;
    }
    ~Lease() {
        if (!c) return;
        std::lock_guard<std::mutex> g(D->mu);
        c->busy = false;
        D->cv.notify_one();
    }
    Lease(const Lease &) = delete;
    Lease &operator=(const Lease &) = delete;
};

int ensure_init() {
    int d = 0;
    if (int rc = current_device(&d)) return rc;
    std::lock_guard<std::mutex> g(g_dev[d].mu);
    return init_device_locked(g_dev[d], d);
}

// blocking copy on the context's stream (the stream is non-blocking, so a
// plain hipMemcpy on the null stream would not wait for its kernels)
inline bool copy_sync_ok(void *d, const void *src, size_t n, hipMemcpyKind k, hipStream_t st) {
    return hipMemcpyAsync(d, src, n, k, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
}
#define copy_sync(d, src, n, k, st) (copy_sync_ok((d), (src), (n), (k), (st)) ? hipSuccess : hipErrorUnknown)

inline int hip_ok(hipError_t e) { return e == hipSuccess ? ZGPU_OK : ZGPU_MEM_ERROR; }

// ------------------------------------------------------------------------
// deflate orchestration (caller holds a Lease on c)
// ------------------------------------------------------------------------
// The deflate(flush) calls of a streaming job (device arrays, see DeflateJob).
struct FlushSpec {
    const uint64_t *pos;
    const uint32_t *type;
    uint32_t n;
    int open_end;
    uint32_t start, bit0, byte0;   // a resumed job (DeflateJob::start/bit0/byte0)
    uint64_t *out;                 // DeflateJob::flush_out
    // levels 1..3 resumed (host arrays): k_parse_fast's head[hash_size], rebased to
    // the job's buffer, and the prev links of its positions [0, prev_n)
    const uint32_t *head_in;
    const uint16_t *prev_in;
    size_t prev_n;
    // level 0 (host array): the stored blocks and markers, made on the host the
    // way deflate_stored cuts them (see deflate_stored_call)
    const BlockRec *plan;
    uint32_t nplan;
    int dict;                      // DeflateJob::dict / pre_ins (a preset dictionary)
    uint32_t pre_ins;
    // Z_NO_FLUSH stops (DeflateJob::mlim .. snap, fl_aux, device arrays)
    const uint64_t *mlim;
    uint32_t nmlim;
    uint64_t *srec;
    uint32_t *ev_blk;
    uint32_t e0;
    int cut;
    uint32_t *snap;
    const uint64_t *aux;
    // configuration changes (DeflateJob::cfg_pos / cfg_tab / ncfg / cfg_q, device arrays)
    const uint64_t *cfg_pos = nullptr;
    const LevelCfg *cfg_tab = nullptr;
    uint32_t ncfg = 0;
    int cfg_q = 0;
    // a window parsed partly by deflate_fast (DeflateJob::lk_n, pre_from, keep_head)
    uint32_t lk_n = 0, pre_from = 0;
    int keep_head = 0;
    int zp0 = kMinMatch - 1, zm0 = kMinMatch - 1;   // DeflateJob::zp0 / zm0
    int seg_parse = 0;             // the job's stops are all Z_NO_FLUSH: k_pbig* may parse it (k_pbig6s)
    SkipSpec sk{};                 // DeflateJob::sk
};

// deflateInit2_'s windowBits / memLevel rules (deflate.c:400-425): negative
// windowBits raw deflate, 16 + windowBits gzip, 8 made 9 (zlib wrapper only)
int parse_window(int windowBits, int memLevel, int *wrap, int *wbits) {
    int w = 1;
    if (windowBits < 0) {
        w = 0;
        if (windowBits < -15) return ZGPU_STREAM_ERROR;
        windowBits = -windowBits;
    } else if (windowBits > 15) {
        w = 2;
        windowBits -= 16;
    }
    if (memLevel < 1 || memLevel > 9 || windowBits < 8 || windowBits > 15 || (windowBits == 8 && w != 1))
        return ZGPU_STREAM_ERROR;
    *wrap = w;
    *wbits = windowBits == 8 ? 9 : windowBits;
    return ZGPU_OK;
}

// wbits 9..15 (deflateInit2_'s windowBits with 8 already made 9), mem_level
// 1..9 (hash_bits = mem_level + 7, lit_bufsize = 1 << (mem_level + 6))
// a failed device step of a deflate launch (ZGPU_STREAM_TRACE names its line)
static int zfail(int line) {
    static const bool on = std::getenv("ZGPU_STREAM_TRACE") != nullptr;
    if (on) std::fprintf(stderr, "deflate_dev_locked: failed at zgpu_api.cpp:%d (%s)\n", line,
                         hipGetErrorString(hipGetLastError()));
    return ZGPU_MEM_ERROR;
}

int deflate_dev_locked(Ctx &c, const uint8_t *src, const uint64_t *src_off, const uint64_t *src_len,
                       uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap,
                       uint64_t *dst_len, int32_t *status, uint32_t count, int level, int wrap,
                       int strategy, hipStream_t st, const FlushSpec *fs = nullptr, int wbits = 15,
                       int mem_level = 8, const LevelCfg *tune = nullptr, uint8_t *d_wind = nullptr,
                       const uint64_t *host_len = nullptr) {
    if (level == -1) level = 6;
    if (level < 0 || level > 9 || wrap < 0 || wrap > 2 || strategy < 0 || strategy > 4 || wbits < 9 ||
        wbits > 15 || mem_level < 1 || mem_level > 9)
        return ZGPU_STREAM_ERROR;
    const int hbits = mem_level + 7;
    const WinP wp = win_params(wbits, hbits);
    const uint64_t hsize = 1ull << hbits;
    if (fs && (count != 1 || (level == 0) != (fs->plan != nullptr))) return ZGPU_STREAM_ERROR;
    if (count == 0) return ZGPU_OK;
    // the lengths plan the sub-batches: the host path passes its own copy (a
    // lone call saves a device-to-host copy and a stream synchronisation)
    std::vector<uint64_t> lens(count);
    if (host_len) {
        std::memcpy(lens.data(), host_len, 8ull * count);
    } else if (hipMemcpyAsync(lens.data(), src_len, 8ull * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipStreamSynchronize(st) != hipSuccess) {
        return zfail(__LINE__);
    }
    for (uint32_t i = 0; i < count; i++)
        if (lens[i] >= kMaxBuffer) return ZGPU_STREAM_ERROR;   // 32-bit positions in the kernels

    // plan sub-batches: Σ n <= budget (a single larger buffer runs alone).  L1-3
    // keep ~6 B of workspace per in-flight byte (L4-9: ~25) and their parse is
    // one sequential lane per buffer, so they get 4x the budget: more buffers
    // in flight is what their throughput scales with.
    // (levels 1..3 from the sorted runs keep ~28 B per byte: the plain budget, at most 4 GiB)
    // By default only few buffers at levels 2..3 take it (a lone 1 MiB buffer:
    // 4.2-4.8 MB/s against 1.1-1.4 on k_parse_fast's one lane; at level 1 and
    // for batches the chain walk is as fast or faster);
    // ZGPU_FAST_SRT=1 / 0: always / never
    static const int fsrt_env0 = [] { const char *e = std::getenv("ZGPU_FAST_SRT"); return e ? std::atoi(e) : -1; }();
    uint64_t total_in = 0;
    for (uint32_t i = 0; i < count; i++) total_in += lens[i];
    // (k_parse_srt takes a search's chain whole: good_match above prev_length 2, as
    // configuration_table's L1-3 rows have it, and at most 64 strings inserted per match)
    const LevelCfg fcfg = tune ? *tune : kLevelCfg[level];
    const bool fsrt_ok = level >= 1 && level <= 3 && strategy != 2 && strategy != 3 && !fs && hbits <= 15 &&
                         fcfg.good > kMinMatch - 1 && fcfg.lazy <= 64;
    const bool fsrt_want = fsrt_ok && (fsrt_env0 == 1 || (fsrt_env0 == -1 && level >= 2 && count <= 16 &&
                                                           total_in <= (256ull << 20)));
    const uint64_t budget = fsrt_want ? std::min<uint64_t>(c.inflight, 4ull << 30)
                            : (level >= 1 && level <= 3) || strategy == 2 || strategy == 3
                                ? 4 * (uint64_t)c.inflight : (uint64_t)c.inflight;
    std::vector<uint32_t> cuts{0};
    {
        uint64_t acc = 0;
        for (uint32_t i = 0; i < count; i++) {
            if (acc > 0 && acc + lens[i] > budget) { cuts.push_back(i); acc = 0; }
            acc += lens[i];
        }
        cuts.push_back(count);
    }
    uint64_t max_pos = 0, max_blk = 0;
    uint32_t max_cnt = 0;
    std::vector<uint64_t> meta(2ull * count);   // [ws_off | blk_off] per buffer, sub-batch relative
    for (size_t s = 0; s + 1 < cuts.size(); s++) {
        uint64_t pos = 0, blk = 0;
        const uint32_t a = cuts[s], b = cuts[s + 1];
        for (uint32_t i = a; i < b; i++) {
            meta[i] = pos;
            meta[count + i] = blk;
            // n + 1 rounded up: k_parse_seg may stage a buffer's final pending
            // literal at index n (a run of literals up to the end), which must
            // not land in the next buffer's region
            pos += (lens[i] + 64) & ~63ull;
            blk += lens[i] / wp.sym_limit + 2 + (fs ? 2ull * fs->n + fs->nplan : 0);   // a flush: a block and a marker
        }
        max_pos = std::max(max_pos, pos);
        max_blk = std::max(max_blk, blk);
        max_cnt = std::max(max_cnt, b - a);
    }
    // deflate.c:1190-1193: level 0 stores; Z_HUFFMAN_ONLY / Z_RLE replace the
    // level's parser; the other strategies change the lazy parse / tree choice
    const bool huff = level >= 1 && strategy == 2, rle = level >= 1 && strategy == 3;
    const bool slow = level >= 4 && !huff && !rle;
    const size_t nsub = cuts.size() - 1;
    static const bool no_pipe = std::getenv("ZGPU_NO_PIPELINE") != nullptr;
    const bool piped = slow && nsub > 1 && !no_pipe;
    // k_match per segment where a sub-batch has too few buffers to fill the GPU
    // one workgroup per buffer (a single zlib.h buffer, say).  The segment is
    // the sub-batch's bytes over the 256 CUs, in whole 4 KiB tiles, at most
    // 256 KiB: a lone 64 KiB compress2 walks 16 one-tile segments side by side
    // instead of 16 tiles in a row (each segment stages <= 32 KiB it does not walk).
    constexpr uint64_t kSegMax = 256 * 1024, kSegTile = kMatchTile, kSegCUs = 256;
    static_assert(kSegMax % kSegTile == 0, "segments are whole k_match tiles");
    std::vector<uint32_t> segs;
    std::vector<size_t> seg_at(nsub + 1, 0), seg_len(nsub, kSegMax);
    for (size_t sb = 0; sb < nsub; sb++) {
        seg_at[sb] = segs.size() / 2;
        const uint32_t a = cuts[sb], b = cuts[sb + 1];
        uint64_t big = 0, tot = 0;
        for (uint32_t i = a; i < b; i++) big = std::max(big, lens[i]), tot += lens[i];
        uint64_t seg = (tot / kSegCUs + kSegTile - 1) / kSegTile * kSegTile;
        seg = seg < kSegTile ? kSegTile : seg > kSegMax ? kSegMax : seg;
        seg_len[sb] = seg;
        if (!slow || b - a >= 512 || big <= seg) continue;
        for (uint32_t i = a; i < b; i++)
            for (uint64_t o = 0; o < lens[i]; o += seg) {
                segs.push_back(i - a);
                segs.push_back((uint32_t)o);
            }
    }
    seg_at[nsub] = segs.size() / 2;
    if (!segs.empty() && (!c.ws_seg.ensure(4 * segs.size()) ||
                          hipMemcpyAsync(c.ws_seg.p, segs.data(), 4 * segs.size(), hipMemcpyHostToDevice, st) !=
                              hipSuccess))
        return zfail(__LINE__);
    // k_lzp (round 6, the A/B build only): the walks only where deflate_slow
    // asks for them, and the parse, in one kernel per buffer, for batch jobs of
    // levels whose chain is at most kLzpMaxChain (levels 4..7) and no
    // per-segment match.  Exact, and slower than k_match + k_parse_seg
    // (DESIGN.md 4.15); ZGPU_LZP=1 in a library built with it.
    static const int lzp_env = [] { const char *e = std::getenv("ZGPU_LZP"); return e && lzp_built() ? std::atoi(e) : 0; }();
    const LevelCfg jcfg = tune ? *tune : kLevelCfg[level];
    const bool lzp = lzp_env && slow && !fs && jcfg.chain >= 4 && jcfg.chain <= kLzpMaxChain && segs.empty();
    if (!c.ws_meta.ensure(16ull * count + 8ull * max_cnt * 2)) return zfail(__LINE__);
    const size_t ckb = checksum_scratch_bytes(max_cnt);     // trailer checksums of few large buffers
    void *ck = ckb && c.ws_ck.ensure(ckb) ? c.ws_ck.p : nullptr;
    if (!c.ws_link.ensure(2 * max_pos + 64)) return zfail(__LINE__);
    if (!c.ws_sym.ensure(4 * max_pos + 64)) return zfail(__LINE__);
    if (!c.ws_blk.ensure(sizeof(BlockRec) * max_blk)) return zfail(__LINE__);
    if ((slow || huff || rle) && !c.ws_rf.ensure(4 * max_pos + 64)) return zfail(__LINE__);
    // rquart: quarter-budget results (L5-9; k_lzp: every level)
    if (slow && !c.ws_rq.ensure(4 * max_pos + 64)) return zfail(__LINE__);
    if (slow && !lzp && !c.ws_state.ensure(max_pos / 4 + 64)) return zfail(__LINE__);
    if (slow && !c.ws_key.ensure(max_pos + 64)) return zfail(__LINE__);
    if (slow && !lzp && !c.ws_stg.ensure(4 * max_pos + 64)) return zfail(__LINE__);
    if (piped) {
        if (!c.ws_key2.ensure(max_pos + 64)) return zfail(__LINE__);
        if (!c.ws_link2.ensure(2 * max_pos + 64) || !c.ws_rq2.ensure(4 * max_pos + 64)) return zfail(__LINE__);
        if (!c.ws_rf2.ensure(4 * max_pos + 64)) return zfail(__LINE__);
        if (!lzp && !c.ws_state2.ensure(max_pos / 4 + 64)) return zfail(__LINE__);
        if (lzp && (!c.ws_sym2.ensure(4 * max_pos + 64) || !c.ws_blk2.ensure(sizeof(BlockRec) * max_blk)))
            return zfail(__LINE__);
        if (!c.aux && hipStreamCreateWithFlags(&c.aux, hipStreamNonBlocking) != hipSuccess) {
            c.aux = nullptr;
            return zfail(__LINE__);
        }
        for (int k = 0; k < 2; k++) {
            if (!c.ev_links[k] && hipEventCreateWithFlags(&c.ev_links[k], hipEventDisableTiming) != hipSuccess)
                return zfail(__LINE__);
            if (!c.ev_match[k] && hipEventCreateWithFlags(&c.ev_match[k], hipEventDisableTiming) != hipSuccess)
                return zfail(__LINE__);
        }
    }
    if (level >= 1 && level <= 3 && !huff && !rle && !c.ws_heads.ensure(4ull * hsize * max_cnt))
        return zfail(__LINE__);
    // levels 1..3 of a batch job from the same sorted runs (k_bwork<true> +
    // k_parse_srt; ZGPU_FAST_SRT=1)
    bool fsrt = fsrt_want;
    std::vector<uint32_t> bblk;
    std::vector<size_t> bblk_at(nsub + 1, 0);
    uint64_t max_sblk = 0;
    // the sorted-run workspace (~22 B per input byte: work items 16, entries 2,
    // block tables ~4) goes back when the call ends if it exceeds the in-flight
    // budget, instead of staying pinned for the context's life
    struct SrtBack {
        Ctx &c;
        ~SrtBack() {
            for (DevBuf *b : {&c.ws_work, &c.ws_srt, &c.ws_boff})
                if (b->cap > c.inflight) b->release();
        }
    } srt_back{c};
    if (fsrt) {
        for (size_t sb = 0; sb < nsub; sb++) {
            bblk_at[sb] = bblk.size();
            uint32_t acc = 0;
            for (uint32_t i = cuts[sb]; i < cuts[sb + 1]; i++) {
                bblk.push_back(acc);
                acc += (uint32_t)((lens[i] + kSortBlock - 1) / kSortBlock);
            }
            bblk.push_back(acc);
            max_sblk = std::max<uint64_t>(max_sblk, acc);
        }
        bblk_at[nsub] = bblk.size();
        if (!c.ws_srt.ensure(2 * max_pos + 64) || !c.ws_work.ensure(16 * max_pos + 64) ||
            !c.ws_boff.ensure(2ull * kSortOffStride * max_sblk + 64) || !c.ws_bblk.ensure(4 * bblk.size() + 64) ||
            hipMemcpyAsync(c.ws_bblk.p, bblk.data(), 4 * bblk.size(), hipMemcpyHostToDevice, st) != hipSuccess) {
            (void)hipGetLastError();
            fsrt = false;                               // no room: the chain-walk parse
        }
    }
    // ... and, for a batch (no streaming job), the lazy parse and the encoder
    // too: k_pbig* over segments of pseg bytes (>= 1 KiB; ~64 Ki lanes per
    // sub-batch), kParseLanes lanes per workgroup, k_enc_* per block.  One
    // table holds every sub-batch's (buffer, first lane) pairs, then the
    // per-buffer lane bases.
    static const bool no_big = std::getenv("ZGPU_NO_BIGBUF") != nullptr;   // A/B: the one-workgroup stages
    std::vector<uint32_t> pg, plb;
    std::vector<size_t> pg_at(nsub + 1, 0), plb_at(nsub + 1, 0);
    std::vector<uint32_t> pseg_of(nsub, 0), maxblk_of(nsub, 0), preach_of(nsub, 1);
    uint64_t max_lanes = 0;
    // A sub-batch of small buffers (a lone 64 KiB compress2, say) parses in
    // 256-byte segments, each buffer one workgroup of at most kParseLanes
    // lanes, and a lane's run-on may cross kSmallReach segments before it must
    // meet a later lane's pass 1 (k_pbig3 joins the chain of meets): four times
    // the lanes of 1 KiB segments, so a quarter of each lane's serial parse,
    // without the stitch failures short segments would give long matches
    static const int small_seg = [] { const char *e = std::getenv("ZGPU_PSEG_SMALL"); return e ? std::atoi(e) : 1; }();
    for (size_t sb = 0; sb < nsub; sb++) {
        pg_at[sb] = pg.size() / 2;
        plb_at[sb] = plb.size();
        if ((fs && !fs->seg_parse) || no_big || seg_at[sb + 1] == seg_at[sb]) continue;
        const uint32_t a = cuts[sb], b = cuts[sb + 1];
        const uint64_t st0 = fs ? fs->start : 0;            // a streaming job parses from its resume point
        uint64_t tot = 0;
        for (uint32_t i = a; i < b; i++) tot += lens[i] - st0;
        uint64_t ps = ((tot + 65535) / 65536 + 15) & ~15ull;
        ps = ps < 1024 ? 1024 : ps > 65536 ? 65536 : ps;
        uint64_t maxlen = 0;
        for (uint32_t i = a; i < b; i++) maxlen = std::max<uint64_t>(maxlen, lens[i] - st0);
        if (small_seg && !fs && tot <= (4ull << 20) && maxlen <= kSmallSeg * kParseLanesHost) {
            ps = kSmallSeg;
            preach_of[sb] = (uint32_t)kSmallReach;
        }
        uint64_t lanes = 0;
        for (uint32_t i = a; i < b; i++) {
            const uint64_t nl = std::max<uint64_t>(1, (lens[i] - st0 + ps - 1) / ps);
            plb.push_back((uint32_t)lanes);
            for (uint64_t j = 0; j < nl; j += kParseLanesHost) {
                pg.push_back(i - a);
                pg.push_back((uint32_t)j);
            }
            lanes += nl;
        }
        max_lanes = std::max(max_lanes, lanes);
        pseg_of[sb] = (uint32_t)ps;
    }
    pg_at[nsub] = pg.size() / 2;
    plb_at[nsub] = plb.size();
    // k_pbig6s's timeline: a slide per window and two entries per stop at most
    uint32_t ntl = 0;
    if (fs && !pg.empty()) {
        ntl = (uint32_t)(lens[0] / wp.wsize + 2ull * fs->n + 8);
        if (!c.ws_tl.ensure(16ull * ntl + 4ull * fs->n + 64)) return zfail(__LINE__);
    }
    // The block-parallel encoder (k_enc_plan / scan / emit, §4.6b) for every
    // batch job at levels 1..9: one workgroup per block instead of one per
    // buffer (a 4096 x 1 MiB L6 sub-batch: 42 -> ~10 ms), and for streaming
    // jobs with Z_NO_FLUSH stops only (resumed at a partial byte, records from
    // k_enc_rec).  Other streaming jobs (markers) and level 0 keep k_encode.
    bool block_enc = (!fs || fs->seg_parse) && level >= 1 && !no_big;
    for (size_t sb = 0; sb < nsub; sb++) {            // (k_pbig6's grid too: set for every path)
        uint64_t mb = 0;
        for (uint32_t i = cuts[sb]; i < cuts[sb + 1]; i++) mb = std::max<uint64_t>(mb, lens[i] / wp.sym_limit + 2);
        maxblk_of[sb] = (uint32_t)mb;
    }
    // The plans take sizeof(EncPlan) (~1 KiB) per possible block: at memLevel 1
    // (a block per 127 symbols) a 1 GiB buffer needs ~8.7 GB of them.  When that
    // allocation fails the job encodes with k_encode instead (one workgroup per
    // buffer, no plan workspace) rather than failing.
    // (ZGPU_EPLAN_LIMIT_MB, tests: treat a larger plan workspace as unavailable)
    const char *eplan_lim = std::getenv("ZGPU_EPLAN_LIMIT_MB");
    if (block_enc && eplan_lim && sizeof(EncPlan) * max_blk > (uint64_t)std::atoll(eplan_lim) << 20) block_enc = false;
    if (block_enc && !c.ws_eplan.ensure(sizeof(EncPlan) * max_blk)) {
        (void)hipGetLastError();
        block_enc = false;
    }
    if (!pg.empty()) {
        const size_t npg = pg.size();
        pg.insert(pg.end(), plb.begin(), plb.end());
        if (!c.ws_pg.ensure(4 * pg.size()) ||
            hipMemcpyAsync(c.ws_pg.p, pg.data(), 4 * pg.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
            !c.ws_plane.ensure(sizeof(PLane) * max_lanes) || !c.ws_pbuf.ensure(sizeof(PBuf) * max_cnt) ||
            !c.ws_pron.ensure(4ull * kRonCap * max_lanes))
            return zfail(__LINE__);
        pg.resize(npg);
    }
    const size_t plb_base = pg.size();
    uint64_t *d_meta = c.ws_meta.as<uint64_t>();
    uint32_t *d_nblk = reinterpret_cast<uint32_t *>(d_meta + 2ull * count);
    uint32_t *d_check = d_nblk + max_cnt;
    uint32_t *d_nblk2 = d_check + max_cnt;                   // k_lzp's slot 1 (ws_meta holds 4 x max_cnt words)
    if (hipMemcpyAsync(d_meta, meta.data(), 16ull * count, hipMemcpyHostToDevice, st) != hipSuccess)
        return zfail(__LINE__);
    // ZGPU_POISON (debug): fill every workspace with a per-call byte pattern so
    // a kernel that reads a word it did not write shows up as a mismatch
    static const bool poison = std::getenv("ZGPU_POISON") != nullptr;
    if (poison) {
        static int round = 0;
        const int v = 0x5a ^ (round++ * 0x3b);
        for (DevBuf *b : {&c.ws_link, &c.ws_sym, &c.ws_stg, &c.ws_blk, &c.ws_rf, &c.ws_rq, &c.ws_state, &c.ws_heads,
                          &c.ws_link2, &c.ws_rf2, &c.ws_rq2, &c.ws_state2})
            if (b->p && hipMemsetAsync(b->p, v & 0xff, b->cap, st) != hipSuccess) return zfail(__LINE__);
        if (hipMemsetAsync(d_nblk, v & 0xff, 8ull * max_cnt, st) != hipSuccess) return zfail(__LINE__);
    }
    if (fs && fs->plan &&
        (hipMemcpyAsync(c.ws_blk.p, fs->plan, sizeof(BlockRec) * fs->nplan, hipMemcpyHostToDevice, st) != hipSuccess ||
         hipMemcpyAsync(d_nblk, &fs->nplan, 4, hipMemcpyHostToDevice, st) != hipSuccess))
        return zfail(__LINE__);
    if (fs && fs->head_in) {
        if (!c.ws_heads.ensure(4ull * hsize) ||
            hipMemcpyAsync(c.ws_heads.p, fs->head_in, 4ull * hsize, hipMemcpyHostToDevice, st) != hipSuccess ||
            (fs->prev_n && hipMemcpyAsync(c.ws_link.p, fs->prev_in, 2ull * fs->prev_n, hipMemcpyHostToDevice, st) !=
                               hipSuccess))
            return zfail(__LINE__);
    }

    StageTimer &T = c.timer;
    auto make_job = [&](size_t s) {
        const uint32_t a = cuts[s], b = cuts[s + 1];
        const int slot = piped ? (int)(s & 1) : 0;
        DeflateJob job{};
        job.src = src; job.src_off = src_off; job.src_len = src_len;
        job.dst = dst; job.dst_off = dst_off; job.dst_cap = dst_cap;
        job.dst_len = dst_len; job.status = status;
        job.first = a; job.count = b - a; job.level = level; job.wrap = wrap; job.strategy = strategy;
        job.wbits = wbits; job.hbits = hbits;
        job.cfg = tune ? *tune : kLevelCfg[level];
        job.ws_off = d_meta + a;
        job.blk_off = d_meta + count + a;
        job.link = (slot ? c.ws_link2 : c.ws_link).as<uint16_t>();
        job.key = slow ? (slot ? c.ws_key2 : c.ws_key).as<uint8_t>() : nullptr;
        job.rfull = (slow || huff || rle) ? (slot ? c.ws_rf2 : c.ws_rf).as<uint32_t>() : nullptr;
        job.rquart = slow ? (slot ? c.ws_rq2 : c.ws_rq).as<uint32_t>() : nullptr;
        job.sym = c.ws_sym.as<uint32_t>();
        job.stage = slow && !lzp ? c.ws_stg.as<uint32_t>() : nullptr;
        job.pstate = slow && !lzp ? (slot ? c.ws_state2 : c.ws_state).as<uint32_t>() : nullptr;
        job.blocks = c.ws_blk.as<BlockRec>();
        job.nblocks = d_nblk;
        static const int lzp_flags = [] { const char *e = std::getenv("ZGPU_LZP_FLAGS"); return e ? std::atoi(e) : 1; }();
        job.lzp_flags = lzp_flags;
        if (lzp) {                                      // k_lzp writes the symbols beside the encode: two slots
            if (slot) {
                job.sym = c.ws_sym2.as<uint32_t>();
                job.blocks = c.ws_blk2.as<BlockRec>();
                job.nblocks = d_nblk2;
            }
        }
        job.pos31 = 1;
        for (uint32_t i = a; i < b; i++)
            if (lens[i] >= (1ull << 31) - (1ull << 16)) job.pos31 = 0;
        static const int lgh_env = [] { const char *e = std::getenv("ZGPU_LINKS_GH"); return e ? std::atoi(e) : 1; }();
        // not in the pipeline: there k_links runs beside k_match, and two
        // k_links_gh workgroups per CU slow the walks by what they save
        job.links_gh = lgh_env && slow && hbits <= 15 && !piped;
        for (uint32_t i = a; i < b && job.links_gh; i++)
            if (lens[i] < kLinksGhMin) job.links_gh = 0;
        job.check = d_check;
        job.wind = d_wind ? d_wind + a : nullptr;
        if (seg_at[s + 1] > seg_at[s]) {
            job.seg = c.ws_seg.as<uint32_t>() + 2 * seg_at[s];
            job.nseg = (uint32_t)(seg_at[s + 1] - seg_at[s]);
            job.seg_len = (uint32_t)seg_len[s];
        }
        if (pg_at[s + 1] > pg_at[s]) {
            job.pgrp = c.ws_pg.as<uint32_t>() + 2 * pg_at[s];
            job.npgrp = (uint32_t)(pg_at[s + 1] - pg_at[s]);
            job.plbase = c.ws_pg.as<uint32_t>() + plb_base + plb_at[s];
            job.pseg = pseg_of[s];
            job.preach = preach_of[s];
            job.pron = c.ws_pron.as<uint32_t>();
            job.plane = c.ws_plane.as<PLane>();
            job.pbuf = c.ws_pbuf.as<PBuf>();
            if (ntl) {
                job.tl = c.ws_tl.as<uint32_t>();
                job.ntl = ntl;
            }
        }
        job.maxblk = maxblk_of[s];
        if (fsrt) {
            job.bblk = c.ws_bblk.as<uint32_t>() + bblk_at[s];
            job.srt = c.ws_srt.as<uint16_t>();
            job.boff = c.ws_boff.as<uint16_t>();
            job.work = c.ws_work.as<uint4>();
            job.nsblk = bblk[bblk_at[s + 1] - 1];
        }
        static const int fcmp64 = std::getenv("ZGPU_FAST_CMP64") != nullptr;   // A/B: k_parse_fast's compare
        job.fcmp = fcmp64;
        if (block_enc) job.eplan = c.ws_eplan.as<EncPlan>();
        if (fs) {
            job.fl_pos = fs->pos;
            job.fl_type = fs->type;
            job.nfl = fs->n;
            job.open_end = fs->open_end;
            job.start = fs->start;
            job.bit0 = fs->bit0;
            job.byte0 = fs->byte0;
            job.flush_out = fs->out;
            job.plan = fs->plan != nullptr;
            job.dict = fs->dict;
            job.pre_ins = fs->pre_ins;
            job.mlim = fs->mlim;
            job.nmlim = fs->nmlim;
            job.srec = fs->srec;
            job.ev_blk = fs->ev_blk;
            job.e0 = fs->e0;
            job.cut = fs->cut;
            job.snap = fs->snap;
            job.fl_aux = fs->aux;
            job.cfg_pos = fs->cfg_pos;
            job.cfg_tab = fs->cfg_tab;
            job.ncfg = fs->ncfg;
            job.cfg_q = fs->cfg_q;
            job.pre_from = fs->pre_from;
            job.keep_head = fs->keep_head;
            job.zp0 = fs->zp0;
            job.zm0 = fs->zm0;
            job.sk = fs->sk;
            if (slow && fs->head_in) {                  // k_links resumes deflate_fast's chains
                job.lk_n = fs->lk_n;
                job.lk_head = c.ws_heads.as<uint32_t>();
            }
        }
        return job;
    };
    // trailer check value, parse, encode of sub-batch s on the caller's stream
    auto tail = [&](size_t s, const DeflateJob &job) -> int {
        const uint32_t a = cuts[s], b = cuts[s + 1];
        int rc = 0;
        if (wrap == 1)
            rc = T.run(0, st, [&] { return launch_adler32(src, src_off + a, src_len + a, nullptr, d_check, b - a, ck, ckb, st); });
        else if (wrap == 2)
            rc = T.run(0, st, [&] { return launch_crc32(src, src_off + a, src_len + a, nullptr, d_check, b - a, ck, ckb, st); });
        if (rc) return zfail(__LINE__);
        if ((huff || rle) && fs) {
            if (T.run(4, st, [&] { return launch_deflate_stage(10, job, nullptr, st); })) return zfail(__LINE__);
        } else if (huff) {
            if (T.run(4, st, [&] { return launch_deflate_stage(7, job, nullptr, st); })) return zfail(__LINE__);
        } else if (rle) {
            if (T.run(4, st, [&] { return launch_deflate_stage(8, job, nullptr, st); })) return zfail(__LINE__);
        } else if (level >= 4 && fs && job.pgrp) {
            // a streaming job with Z_NO_FLUSH stops only: the segmented parse,
            // fill_window's bookkeeping and the stops replayed over its blocks
            // (k_pbig6s); what it cannot place goes to the sequential parse
            if (T.run(3, st, [&] { return launch_deflate_stage(13, job, nullptr, st); })) return zfail(__LINE__);
            if (T.run(3, st, [&] { return launch_deflate_stage(6, job, nullptr, st); })) return zfail(__LINE__);
        } else if (level >= 4 && fs) {
            // flush jobs: the sequential lazy parse (the segmented one does not
            // model a flush's effect on the parse)
            if (T.run(3, st, [&] { return launch_deflate_stage(2, job, nullptr, st); })) return zfail(__LINE__);
        } else if (level >= 4 && lzp) {
            // parsed by k_lzp with the walks
        } else if (level >= 4) {
            const int ps = job.pgrp ? 11 : 5;                  // few large buffers: k_pbig*
            if (T.run(3, st, [&] { return launch_deflate_stage(ps, job, nullptr, st); })) return zfail(__LINE__);
            if (T.run(3, st, [&] { return launch_deflate_stage(6, job, nullptr, st); })) return zfail(__LINE__);
        } else if (level >= 1 && fsrt) {
            if (T.run(1, st, [&] { return launch_deflate_stage(14, job, nullptr, st); })) return zfail(__LINE__);
            if (T.run(4, st, [&] { return launch_deflate_stage(16, job, nullptr, st); })) return zfail(__LINE__);
        } else if (level >= 1) {
            uint32_t *heads = c.ws_heads.as<uint32_t>();
            if (T.run(4, st, [&] { return launch_deflate_stage(3, job, heads, st); })) return zfail(__LINE__);
        }
        const int es = job.eplan ? 12 : 4;                      // batch jobs: k_enc_* (§4.6b)
        if (T.run(5, st, [&] { return launch_deflate_stage(es, job, nullptr, st); })) return zfail(__LINE__);
        return ZGPU_OK;
    };

    if (!piped) {
        for (size_t s = 0; s < nsub; s++) {
            const DeflateJob job = make_job(s);
            if (slow) {
                if (T.run(1, st, [&] { return launch_deflate_stage(0, job, nullptr, st); })) return zfail(__LINE__);
                if (T.run(2, st, [&] { return launch_deflate_stage(lzp ? 17 : 1, job, nullptr, st); }))
                    return zfail(__LINE__);
            }
            if (int rc = tail(s, job)) return rc;
        }
    } else {
        // caller's stream: links(0), then per s: links(s+1), [wait match(s)] tail(s)
        // aux stream:      per s: [wait links(s)] match(s)
        // Slot s%2 is reused by s+2: links(s+2) follows tail(s) on the caller's
        // stream, and match(s+2) waits for links(s+2), so neither overwrites a
        // slot still being read.
        hipStream_t ax = c.aux;
        auto links = [&](size_t s) -> int {
            const DeflateJob job = make_job(s);
            if (T.run(1, st, [&] { return launch_deflate_stage(0, job, nullptr, st); })) return zfail(__LINE__);
            if (hipEventRecord(c.ev_links[s & 1], st) != hipSuccess) return zfail(__LINE__);
            if (hipStreamWaitEvent(ax, c.ev_links[s & 1], 0) != hipSuccess) return zfail(__LINE__);
            if (T.run(2, ax, [&] { return launch_deflate_stage(lzp ? 17 : 1, job, nullptr, ax); }))
                return zfail(__LINE__);
            if (hipEventRecord(c.ev_match[s & 1], ax) != hipSuccess) return zfail(__LINE__);
            return ZGPU_OK;
        };
        if (int rc = links(0)) return rc;
        for (size_t s = 0; s < nsub; s++) {
            if (s + 1 < nsub) if (int rc = links(s + 1)) return rc;
            if (hipStreamWaitEvent(st, c.ev_match[s & 1], 0) != hipSuccess) return zfail(__LINE__);
            if (int rc = tail(s, make_job(s))) return rc;
        }
    }
    const hipError_t se = hipStreamSynchronize(st);
    int rc = hip_ok(se);
    if (rc) { static const bool on = std::getenv("ZGPU_STREAM_TRACE") != nullptr;
              if (on) std::fprintf(stderr, "deflate_dev_locked: sync %s\n", hipGetErrorString(se)); }
    if (piped && rc == ZGPU_OK) rc = hip_ok(hipStreamSynchronize(c.aux));
    c.timer.collect();
    return rc;
}

// host-buffer batch: pack, upload, run, download
// host-side flush calls of one streaming job (positions ascending, see FlushSpec)
struct FlushHost {
    const uint64_t *pos;
    const uint32_t *type;
    uint32_t n;
    int open_end;
    uint32_t start, bit0, byte0;   // in: a resumed job (see DeflateJob)
    uint64_t out[8];               // out: DeflateJob::flush_out
    // levels 1..3 (see FlushSpec): the chains the job starts from, and where
    // it leaves them: head[32768] and the prev links of [S, last flush), S = out[2]
    const uint32_t *head_in = nullptr;
    const uint16_t *prev_in = nullptr;
    size_t prev_n = 0;
    std::vector<uint32_t> *head_out = nullptr;
    std::vector<uint16_t> *prev_out = nullptr;
    const BlockRec *plan = nullptr;    // level 0: see FlushSpec
    uint32_t nplan = 0;
    int dict = 0;                      // see FlushSpec
    uint32_t pre_ins = 0;
    // Z_NO_FLUSH stops (events of kind 0): in, a job resumed at a block cut;
    // out, the records (DeflateJob::srec), the records before each event, and
    // for levels 1..3 head[] at the last cut with that record's index and the
    // prev links of [its S, its end)
    uint32_t e0 = 0;
    int cut = 0;
    const uint64_t *aux = nullptr;     // DeflateJob::fl_aux (pause events), n entries
    std::vector<uint64_t> *rec_out = nullptr;
    std::vector<uint32_t> *evb_out = nullptr;
    std::vector<uint32_t> *snap_head = nullptr;
    std::vector<uint16_t> *snap_prev = nullptr;
    uint32_t snap_rec = 0xffffffffu;
    // configuration changes (host arrays, see DeflateJob::cfg_pos)
    const uint64_t *cfg_pos = nullptr;
    const LevelCfg *cfg_tab = nullptr;
    uint32_t ncfg = 0;
    // a window parsed partly by deflate_fast: see FlushSpec
    uint32_t lk_n = 0, pre_from = 0;
    int keep_head = 0;
    int zp0 = kMinMatch - 1, zm0 = kMinMatch - 1;   // DeflateJob::zp0 / zm0
    int seg_parse = 0;                 // see FlushSpec
    SkipSpec sk{};                     // see FlushSpec
};

// streaming jobs on the segmented parse (FlushHost::seg_parse): at least this
// much input to parse, and at most this many window slides (k_pbig6s replays
// them one by one on one lane)
constexpr uint64_t kSegStreamMin = 1ull << 20;
constexpr uint64_t kSegStreamSlides = 1ull << 18;

// debug trace of the streaming deflate() engine (ZGPU_STREAM_TRACE)
#define ZTRACE(...) do { static const bool on_ = std::getenv("ZGPU_STREAM_TRACE") != nullptr; \
    if (on_) { std::fprintf(stderr, __VA_ARGS__); std::fflush(stderr); } } while (0)
int compress_host_locked(Ctx &c, const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                         size_t *dst_len, int *status, size_t count, int level, int wrap, int strategy,
                         FlushHost *fh = nullptr, int wbits = 15, int mem_level = 8,
                         const LevelCfg *tune = nullptr, uint8_t *wind_out = nullptr) {
    if (count == 0) return ZGPU_OK;
    for (size_t i = 0; i < count; i++)
        if (src_len[i] >= kMaxBuffer) return ZGPU_STREAM_ERROR;
    std::vector<uint64_t> so(count), sl(count), dofs(count), dcap(count);
    uint64_t in_total = 0, out_total = 0;
    for (size_t i = 0; i < count; i++) {
        so[i] = in_total;
        sl[i] = src_len[i];
        in_total += (src_len[i] + 15) & ~15ull;
        dofs[i] = out_total;
        dcap[i] = dst_len[i];
        out_total += (dst_len[i] + 15) & ~15ull;
    }
    const size_t ev_bytes = fh ? 32ull * fh->n + 192 + (8 + sizeof(LevelCfg)) * fh->ncfg + 16 : 0;
    const size_t meta_bytes = 8 * 4 * count + 16 * count + ev_bytes;
    if (!c.ws_io.ensure(in_total + 64) || !c.ws_io2.ensure(out_total + 64) ||
        !c.ws_small.ensure(meta_bytes + 64))
        return ZGPU_MEM_ERROR;
    uint8_t *d_in = c.ws_io.as<uint8_t>(), *d_out = c.ws_io2.as<uint8_t>();
    uint64_t *d_so = c.ws_small.as<uint64_t>();
    uint64_t *d_sl = d_so + count, *d_do = d_sl + count, *d_dc = d_do + count, *d_dl = d_dc + count;
    int32_t *d_st = reinterpret_cast<int32_t *>(d_dl + count);
    hipStream_t st = c.own;
    static const bool poison = std::getenv("ZGPU_POISON") != nullptr;   // debug, see deflate_dev_locked
    if (poison) {
        static int round = 0;
        const int v = (0xc3 ^ (round++ * 0x29)) & 0xff;
        if (hipMemsetAsync(d_in, v, c.ws_io.cap, st) != hipSuccess ||
            hipMemsetAsync(d_out, v ^ 0xff, c.ws_io2.cap, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
    }
    for (size_t i = 0; i < count; i++)
        if (src_len[i] && hipMemcpyAsync(d_in + so[i], src[i], src_len[i], hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
    std::vector<uint64_t> m4;                          // alive until the call returns (the upload's source)
    {   // d_so, d_sl, d_do, d_dc are consecutive: one upload (a lone call's latency is its copies)
        m4.reserve(4 * count);
        m4.insert(m4.end(), so.begin(), so.end());
        m4.insert(m4.end(), sl.begin(), sl.end());
        m4.insert(m4.end(), dofs.begin(), dofs.end());
        m4.insert(m4.end(), dcap.begin(), dcap.end());
        (void)d_sl; (void)d_dc;
        if (hipMemcpyAsync(d_so, m4.data(), 32 * count, hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
    }
    FlushSpec fs{};
    if (fh) {
        uint64_t *d_fp = reinterpret_cast<uint64_t *>(d_st + 2 * count);   // 8-aligned
        uint32_t *d_ft = reinterpret_cast<uint32_t *>(d_fp + fh->n);
        if (fh->n && (hipMemcpyAsync(d_fp, fh->pos, 8ull * fh->n, hipMemcpyHostToDevice, st) != hipSuccess ||
                      hipMemcpyAsync(d_ft, fh->type, 4ull * fh->n, hipMemcpyHostToDevice, st) != hipSuccess))
            return ZGPU_MEM_ERROR;
        uint64_t *d_mb = d_fp + fh->n + (fh->n + 1) / 2;
        if (hipMemsetAsync(d_mb, 0, 64, st) != hipSuccess) return ZGPU_MEM_ERROR;
        // k_match's clamps: the flush events only (not the Z_NO_FLUSH stops)
        std::vector<uint64_t> ml;
        for (uint32_t i = 0; i < fh->n; i++)
            if (fh->type[i] != 0 && fh->type[i] != kEvPause && fh->type[i] != kEvPrime) ml.push_back(fh->pos[i]);
        uint64_t *d_ml = d_mb + 8;
        uint64_t *d_aux = d_ml + fh->n;
        uint32_t *d_evb = reinterpret_cast<uint32_t *>(d_aux + fh->n);
        if (!ml.empty() && hipMemcpyAsync(d_ml, ml.data(), 8 * ml.size(), hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
        if (fh->n && hipMemsetAsync(d_evb, 0xff, 4ull * fh->n, st) != hipSuccess) return ZGPU_MEM_ERROR;
        if (fh->aux && fh->n && hipMemcpyAsync(d_aux, fh->aux, 8ull * fh->n, hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
        fs = FlushSpec{d_fp, d_ft, fh->n, fh->open_end, fh->start, fh->bit0, fh->byte0, d_mb,
                       fh->head_in, fh->prev_in, fh->prev_n, fh->plan, fh->nplan, fh->dict, fh->pre_ins,
                       d_ml, (uint32_t)ml.size(), nullptr, d_evb, fh->e0, fh->cut, nullptr,
                       fh->aux ? d_aux : nullptr};
        if (fh->ncfg) {                                  // configuration changes after the events
            uint64_t *d_cp = reinterpret_cast<uint64_t *>(d_evb + fh->n + (fh->n & 1));
            LevelCfg *d_ct = reinterpret_cast<LevelCfg *>(d_cp + fh->ncfg);
            if (hipMemcpyAsync(d_cp, fh->cfg_pos, 8ull * fh->ncfg, hipMemcpyHostToDevice, st) != hipSuccess ||
                hipMemcpyAsync(d_ct, fh->cfg_tab, sizeof(LevelCfg) * fh->ncfg, hipMemcpyHostToDevice, st) !=
                    hipSuccess)
                return ZGPU_MEM_ERROR;
            fs.cfg_pos = d_cp;
            fs.cfg_tab = d_ct;
            fs.ncfg = fh->ncfg;
            for (uint32_t k = 0; k < fh->ncfg; k++) fs.cfg_q |= (int)(fh->cfg_tab[k].good < fh->cfg_tab[k].lazy);
        }
        fs.lk_n = fh->lk_n;
        fs.pre_from = fh->pre_from;
        fs.keep_head = fh->keep_head;
        fs.zp0 = fh->zp0;
        fs.zm0 = fh->zm0;
        fs.seg_parse = fh->seg_parse;
        fs.sk = fh->sk;
        if (fh->rec_out) {
            const size_t sym_limit = (size_t(1) << (mem_level + 6)) - 1;         // lit_bufsize - 1
            const size_t nrec = src_len[0] / sym_limit + 4 + 2ull * fh->n + fh->nplan;
            if (!c.ws_srec.ensure(32 * nrec)) return ZGPU_MEM_ERROR;
            fs.srec = c.ws_srec.as<uint64_t>();
        }
        if (fh->snap_head) {
            const size_t hsize = size_t(1) << (mem_level + 7);
            if (!c.ws_snap.ensure(4 * (hsize + 1)) ||
                hipMemsetAsync(c.ws_snap.p, 0xff, 4 * (hsize + 1), st) != hipSuccess)
                return ZGPU_MEM_ERROR;
            fs.snap = c.ws_snap.as<uint32_t>();
        }
    }
    if (fh) ZTRACE("chl: launch n %u open %d\n", fh->n, fh->open_end);
    if (wind_out && !c.ws_wind.ensure(count + 64)) return ZGPU_MEM_ERROR;
    int rc = deflate_dev_locked(c, d_in, d_so, d_sl, d_out, d_do, d_dc, d_dl, d_st, (uint32_t)count,
                                level, wrap, strategy, st, fh ? &fs : nullptr, wbits, mem_level, tune,
                                wind_out ? c.ws_wind.as<uint8_t>() : nullptr, sl.data());
    if (fh) ZTRACE("chl: ran rc %d\n", rc);
    if (rc) return rc;
    if (wind_out && copy_sync(wind_out, c.ws_wind.p, count, hipMemcpyDeviceToHost, st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    if (fh && copy_sync(fh->out, fs.out, 64, hipMemcpyDeviceToHost, st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    // Every count and length the device reports is checked against the host
    // buffer it sizes before anything is copied into host memory: a kernel
    // fault must end in an error code, never in a write past a host buffer
    // (the r04c run's heap corruption had this signature).
    if (fh && fh->rec_out) {
        uint32_t nb = 0;
        if (copy_sync(&nb, c.ws_meta.as<uint64_t>() + 2, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
        ZTRACE("chl: nb %u\n", nb);
        if ((size_t)nb > c.ws_srec.cap / 32) {
            ZTRACE("chl: %u records reported, %zu fit\n", nb, c.ws_srec.cap / 32);
            return ZGPU_MEM_ERROR;
        }
        fh->rec_out->resize(4ull * nb);
        fh->evb_out->resize(fh->n);
        if ((nb && copy_sync(fh->rec_out->data(), fs.srec, 32ull * nb, hipMemcpyDeviceToHost, st) != hipSuccess) ||
            (fh->n && copy_sync(fh->evb_out->data(), fs.ev_blk, 4ull * fh->n, hipMemcpyDeviceToHost, st) != hipSuccess))
            return ZGPU_MEM_ERROR;
        fh->snap_rec = 0xffffffffu;
        if (fh->snap_head) {
            const size_t hsize = size_t(1) << (mem_level + 7);
            uint32_t k = 0xffffffffu;
            if (copy_sync(&k, fs.snap + hsize, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return ZGPU_MEM_ERROR;
            if (k < nb) {
                const uint64_t S = (*fh->rec_out)[4ull * k + 2] >> 32, x = (*fh->rec_out)[4ull * k + 2] & 0xffffffffu;
                if (x > src_len[0] || S > x || 2 * x > c.ws_link.cap) return ZGPU_MEM_ERROR;
                fh->snap_head->resize(hsize);
                fh->snap_prev->resize(x > S ? x - S : 0);
                if (copy_sync(fh->snap_head->data(), fs.snap, 4ull * hsize, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    (x > S && copy_sync(fh->snap_prev->data(), c.ws_link.as<uint16_t>() + S, 2 * (x - S),
                                        hipMemcpyDeviceToHost, st) != hipSuccess))
                    return ZGPU_MEM_ERROR;
                fh->snap_rec = k;
            }
        }
    }
    if (fh && fh->head_out && fh->n) {
        const uint64_t S = fh->out[2], end = fh->pos[fh->n - 1];
        const size_t hsize = size_t(1) << (mem_level + 7);
        if (end > src_len[0] || S > end || 2 * end > c.ws_link.cap || 4 * hsize > c.ws_heads.cap)
            return ZGPU_MEM_ERROR;
        fh->head_out->resize(hsize);
        fh->prev_out->resize(end > S ? end - S : 0);
        if (copy_sync(fh->head_out->data(), c.ws_heads.p, 4ull * hsize, hipMemcpyDeviceToHost, st) != hipSuccess ||
            (end > S && copy_sync(fh->prev_out->data(), c.ws_link.as<uint16_t>() + S, 2 * (end - S),
                                  hipMemcpyDeviceToHost, st) != hipSuccess))
            return ZGPU_MEM_ERROR;
    }
    std::vector<uint64_t> ol(count);
    std::vector<int32_t> os(count);
    // the lengths and statuses are consecutive (d_dl, d_st): one copy.  A lone buffer of at most 256 KiB
    // of output space comes back whole in the same wait (a few KiB more over PCIe against a second round
    // trip of copy and stream synchronisation; only its reported length is handed on)
    const bool whole = count == 1 && dcap[0] > 0 && dcap[0] <= (uint64_t(256) << 10);
    std::vector<uint8_t> lsb(12 * count), stage(whole ? dcap[0] : 0);
    if (hipMemcpyAsync(lsb.data(), d_dl, 12 * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        (whole && hipMemcpyAsync(stage.data(), d_out + dofs[0], dcap[0], hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    std::memcpy(ol.data(), lsb.data(), 8 * count);
    std::memcpy(os.data(), lsb.data() + 8 * count, 4 * count);
    for (size_t i = 0; i < count; i++)
        if (ol[i] > dcap[i]) {
            ZTRACE("chl: buffer %zu: %lu bytes reported, capacity %lu\n", i, (unsigned long)ol[i],
                   (unsigned long)dcap[i]);
            return ZGPU_MEM_ERROR;
        }
    for (size_t i = 0; i < count; i++) {
        if (whole) {
            if (ol[i]) std::memcpy(dst[i], stage.data(), ol[i]);
        } else if (ol[i] && copy_sync(dst[i], d_out + dofs[i], ol[i], hipMemcpyDeviceToHost, st) != hipSuccess) {
            return ZGPU_MEM_ERROR;
        }
        dst_len[i] = ol[i];
        if (status) status[i] = os[i];
    }
    return ZGPU_OK;
}

// ------------------------------------------------------------------------
// inflate orchestration (caller holds a Lease on c).  Sub-batches keep the sum of
// output capacities within the in-flight budget; each stream gets cap/3 + 2
// match records (a match writes >= 3 bytes, the last one may be cut short).
// stop_out (device, optional): InflateStop per stream.
// ------------------------------------------------------------------------
constexpr uint64_t kParInflateMin = 32 * 1024;    // inflate_par: lone streams from this many compressed bytes (tools/par_threshold.py)
struct InflateResumeDev {          // InflateJob's resume arrays (device, per stream)
    const uint64_t *res_bit;
    const uint32_t *res_hist;
    uint64_t *blk_out;
    uint32_t stop_mode;            // InflateJob::stop_mode
    uint64_t *zstate_out;          // InflateJob::zstate_out
    uint32_t dmax = 0;             // InflateJob::dmax
    uint64_t trees_after = 0;      // InflateJob::trees_after
    uint64_t *eidx = nullptr, *bidx = nullptr;   // InflateJob::eidx / bidx / icnt (null: no index)
    uint32_t *icnt = nullptr;
    uint32_t ecap = 0, bcap = 0;
};

// ------------------------------------------------------------------------
// The block-parallel decode of a lone stream (a large uncompress, say): a
// stream decodes on one wave at about 8 MB/s, and a lone one leaves the rest of
// the GPU idle.  Its dynamic and stored blocks are found by trying every bit
// offset as a block header (k_infl_scan1 / k_infl_scan2: inftrees.c's rules
// on the header and both codes); every candidate is decoded count-only for its
// end and output length (k_inflate_decode, InflateJob::count_only); the chain
// of ends is followed from the first block (a fixed-code block, which no scan
// can tell from noise, is decoded count-only when the chain reaches it).  Then
// all blocks of the chain decode at once at their output offsets, k_infl_sym
// resolves each block's matches with the bytes before it as references, and
// one k_infl_resolve launch per block, in stream order, turns the references
// into bytes.  The check value and the trailer are compared last.  Anything
// else -- an error anywhere, FDICT, a gzip FHCRC, output beyond the capacity,
// a candidate list overflow -- returns 0 and the caller runs the exact
// sequential path, which reports what uncompress2 would.
// Returns 1 (done: out_len, used), 0 (not taken), < 0 a device error.
// ------------------------------------------------------------------------
int inflate_dev_locked(Ctx &c, const uint8_t *src, const uint64_t *src_off, const uint64_t *src_len,
                       uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap, uint64_t *dst_len,
                       uint64_t *src_used, int32_t *status, uint32_t *stop_out, uint32_t count, int wrap,
                       int wbits, hipStream_t st, const InflateResumeDev *rs = nullptr);

std::atomic<uint64_t> g_par_inflates{0};          // streams the block-parallel decode finished (zgpu_debug.h)

int inflate_par_locked(Ctx &c, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, int wrap, int wbits,
                       hipStream_t st, uint64_t &out_len, uint64_t &used) {
    if (n < 64 || n >= (1ull << 31) || cap >= (1ull << 31)) return 0;
    // ---- the stream header, on the host (inflate.c HEAD .. gzip header)
    std::vector<uint8_t> h((size_t)std::min<uint64_t>(n, 65536));
    if (copy_sync(h.data(), in, h.size(), hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
    uint64_t hb = 0;
    int kind = 0;                                   // 0 raw, 1 zlib, 2 gzip
    if (wrap) {
        if ((wrap & 2) && h[0] == 0x1f && h[1] == 0x8b) {
            const uint32_t flags = h[3];
            if (h[2] != 8 || (flags & 0xe0) || (flags & 0x02)) return 0;   // FHCRC: the exact path checks it
            size_t p = 10;
            if (flags & 0x04) {
                if (p + 2 > h.size()) return 0;
                p += 2 + (h[p] | ((size_t)h[p + 1] << 8));
            }
            for (uint32_t f = 0x08; f <= 0x10; f <<= 1) {
                if (!(flags & f)) continue;
                while (p < h.size() && h[p] != 0) p++;
                if (p >= h.size()) return 0;
                p++;
            }
            if (p >= h.size()) return 0;
            hb = p;
            kind = 2;
        } else {
            const uint32_t cmf = h[0], flg = h[1], wlen = (cmf >> 4) + 8;
            if (!(wrap & 1) || ((cmf << 8) + flg) % 31 || (cmf & 15) != 8 || wlen > 15 ||
                (wbits && wlen > (uint32_t)wbits) || (flg & 0x20))
                return 0;
            hb = 2;
            kind = 1;
        }
    }
    // ---- candidate block headers
    const uint64_t b0 = 8 * hb, b1 = 8 * n;
    const uint32_t lcap = (uint32_t)std::min<uint64_t>((b1 - b0) / 16 + 65536, 1ull << 26);
    // A workspace this path cannot get is no error: the exact sequential decode
    // runs instead.  `nomem` clears the failed allocation's error.
    auto nomem = [] { (void)hipGetLastError(); return 0; };
    if (!c.ws_par1.ensure(8ull * lcap + 64) || !c.ws_par2.ensure(8ull * lcap + 64) || !c.ws_imeta.ensure(64))
        return nomem();
    uint64_t *l1 = c.ws_par1.as<uint64_t>(), *l2 = c.ws_par2.as<uint64_t>();
    uint32_t *cnt = reinterpret_cast<uint32_t *>(c.ws_imeta.as<uint64_t>() + 4);   // two list counters
    uint32_t k1 = 0, k2 = 0;
    if (hipMemsetAsync(cnt, 0, 8, st) != hipSuccess || launch_infl_scan1(in, n, b0, b1, l1, lcap, cnt, st) ||
        copy_sync(&k1, cnt, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return -1;
    if (k1 > lcap) return 0;
    if (launch_infl_scan2(in, n, l1, k1, l2, lcap, cnt + 1, st) ||
        copy_sync(&k2, cnt + 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return -1;
    if (k2 > lcap) return 0;
    std::vector<uint64_t> cand(k2);
    if (k2 && copy_sync(cand.data(), l2, 8ull * k2, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
    std::sort(cand.begin(), cand.end());
    // ---- every candidate decoded once, each in a slot of its own: where it ends, what it makes.
    // Slot k holds the block's literals at [k * kSlot + 32 KiB, +kSlot) behind a pretend 32 KiB
    // window (so no distance stops it; k_infl_sym checks them against the real output) and its
    // matches as records.  A block longer than its slot, or one the scan missed, is measured
    // count-only and decoded in place below.
    constexpr uint64_t kSlot = 256 * 1024, kSlotRec = kSlot / 3 + 2;
    struct Span { uint64_t end, out; uint32_t stop, last, nm; int64_t slot; };
    uint8_t *slots = nullptr;
    uint64_t *mrec = nullptr;
    auto spans = [&](const std::vector<uint64_t> &bits, std::vector<Span> &res, bool write) -> int {
        const uint32_t K = (uint32_t)bits.size();
        res.assign(K, Span{0, 0, kIData, 0, 0, -1});
        if (K == 0) return 0;
        // per job: src_off src_len res_bit dst_off dst_cap dst_len blk_out[2] zstate[2] mrec_off | res_hist |
        // status | rec
        const size_t bytes = 8ull * K * 11 + 4ull * K * 2 + sizeof(InflateRec) * K + 256;
        if (!c.ws_pjob.ensure(bytes)) return 1;
        uint64_t *d = c.ws_pjob.as<uint64_t>();
        uint64_t *soff = d, *slen = d + K, *rbit = d + 2 * K, *doff = d + 3 * K, *dcap = d + 4 * K, *dlen = d + 5 * K;
        uint64_t *blk = d + 6 * K, *zs = d + 8 * K, *mo = d + 10 * K;
        uint32_t *hist = reinterpret_cast<uint32_t *>(d + 11 * K);
        int32_t *stv = reinterpret_cast<int32_t *>(hist + K);
        InflateRec *rec = reinterpret_cast<InflateRec *>((reinterpret_cast<uintptr_t>(stv + K) + 63) & ~(uintptr_t)63);
        std::vector<uint64_t> zero(K, 0), nn(K, n), dof(K), cp(K, 32768 + kSlot), mof(K);
        std::vector<uint32_t> hh(K, 32768u);
        for (uint32_t k = 0; k < K; k++) { dof[k] = write ? k * kSlot : 0; mof[k] = write ? k * kSlotRec : 0; }
        if (hipMemcpyAsync(soff, zero.data(), 8ull * K, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(slen, nn.data(), 8ull * K, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(rbit, bits.data(), 8ull * K, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(doff, dof.data(), 8ull * K, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(dcap, cp.data(), 8ull * K, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(mo, mof.data(), 8ull * K, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(hist, hh.data(), 4ull * K, hipMemcpyHostToDevice, st) != hipSuccess)
            return -1;
        InflateJob job{};
        job.src = in; job.src_off = soff; job.src_len = slen;
        job.dst = write ? slots : out; job.dst_off = doff; job.dst_cap = dcap; job.dst_len = dlen;
        job.status = stv; job.first = 0; job.count = K; job.wrap = 0;
        job.mrec_off = mo; job.mrec = write ? mrec : nullptr;
        job.rec = rec;
        job.res_bit = rbit; job.res_hist = hist; job.blk_out = blk;
        job.stop_mode = 2 | 4;                   // stop at the block's end (the last one's too), start in TYPE
        job.zstate_out = zs;                     // bit 32: BFINAL of the block
        job.count_only = write ? 0 : 1;
        if (c.timer.run(3, st, [&] { return launch_inflate_stage(0, job, st); })) return -1;
        std::vector<InflateRec> r(K);
        std::vector<uint64_t> bo(2ull * K), z(2ull * K);
        if (copy_sync(r.data(), rec, sizeof(InflateRec) * K, hipMemcpyDeviceToHost, st) != hipSuccess ||
            copy_sync(bo.data(), blk, 16ull * K, hipMemcpyDeviceToHost, st) != hipSuccess ||
            copy_sync(z.data(), zs, 16ull * K, hipMemcpyDeviceToHost, st) != hipSuccess)
            return -1;
        for (uint32_t k = 0; k < K; k++) {
            res[k].stop = r[k].stop;
            res[k].last = (z[2ull * k] >> 32) & 1u;
            res[k].out = r[k].put >= 32768 ? r[k].put - 32768 : 0;
            res[k].end = bo[2ull * k];           // the bit after its END_BLOCK code
            res[k].nm = r[k].nmatch;
            res[k].slot = write ? (int64_t)k : -1;
        }
        return 0;
    };
    // slots (and their match records, 2.7 B per slot byte) for every candidate
    // when they fit 4x the in-flight budget; otherwise, or when the allocation
    // fails, every candidate is measured count-only and decoded in place
    bool write = (uint64_t)cand.size() * (kSlot + 8 * kSlotRec) <= 4 * (uint64_t)c.inflight;
    struct SlotsBack {            // slots beyond the in-flight budget go back when the call ends
        Ctx &c;
        ~SlotsBack() {
            for (DevBuf *b : {&c.ws_pslot, &c.ws_mrec, &c.ws_par2, &c.ws_psym})
                if (b->cap > c.inflight) b->release();
        }
    } slots_back{c};
    if (write) {
        if (!c.ws_pslot.ensure(cand.size() * kSlot + 32768 + 64) || !c.ws_mrec.ensure(8 * cand.size() * kSlotRec + 64)) {
            (void)hipGetLastError();
            write = false;
        } else {
            slots = c.ws_pslot.as<uint8_t>();
            mrec = c.ws_mrec.as<uint64_t>();
        }
    }
    std::vector<Span> sp;
    if (int e = spans(cand, sp, write)) return e > 0 ? nomem() : -1;
    // ---- the chain of blocks from the first one
    struct Blk { uint64_t bit, o0, out; bool last; uint32_t nm; int64_t slot; };
    std::vector<Blk> chain;
    uint64_t b = b0, total = 0;
    int misses = 0;
    for (;;) {
        const auto it = std::lower_bound(cand.begin(), cand.end(), b);
        Span s;
        if (it != cand.end() && *it == b) s = sp[(size_t)(it - cand.begin())];
        if (!(it != cand.end() && *it == b) || s.stop == kIFull) {
            // a fixed-code block (or a stored one the scan missed), or one longer than its slot
            if (++misses > 16) return 0;
            std::vector<Span> one;
            if (int e = spans(std::vector<uint64_t>{b}, one, false)) return e > 0 ? nomem() : -1;
            s = one[0];
        }
        if (s.stop != kIBlock || s.end <= b) return 0;
        chain.push_back(Blk{b, total, s.out, s.last != 0, s.nm, s.slot});
        total += s.out;
        if (total > cap) return 0;
        b = s.end;
        if (s.last) break;
    }
    const uint64_t tb = (b + 7) >> 3;               // the trailer's first byte (inflate.c CHECK: BYTEBITS)
    const uint64_t tlen = kind == 1 ? 4 : kind == 2 ? 8 : 0;
    if (tb + tlen > n) return 0;
    // ---- blocks without a slot: decoded at their output offset, literals in place, matches as records
    // after the slots' records
    std::vector<uint32_t> ip;                        // chain indexes of those blocks
    for (uint32_t k = 0; k < (uint32_t)chain.size(); k++)
        if (chain[k].slot < 0) ip.push_back(k);
    const uint32_t NB = (uint32_t)ip.size();
    std::vector<uint64_t> moff(NB), hist(NB);
    uint64_t mtot = 0;
    for (uint32_t j = 0; j < NB; j++) {
        hist[j] = std::min<uint64_t>(32768, chain[ip[j]].o0);
        moff[j] = mtot;
        mtot += chain[ip[j]].out / 3 + 2;
    }
    // their records in a buffer of their own (the slots' stay where the candidates' decode put them)
    if (!c.ws_par2.ensure(8 * mtot + 64) || !c.ws_psym.ensure(4 * total + 64)) return nomem();
    uint64_t *mrec_ip = c.ws_par2.as<uint64_t>();
    if (NB) {
        std::vector<uint64_t> soff(NB, 0), slen(NB, n), rbit(NB), doff(NB), dcap(NB);
        std::vector<uint32_t> h32(NB);
        for (uint32_t j = 0; j < NB; j++) {
            const Blk &B = chain[ip[j]];
            h32[j] = (uint32_t)hist[j];
            rbit[j] = B.bit;
            doff[j] = B.o0 - hist[j];
            dcap[j] = hist[j] + B.out;
        }
        const size_t jb = 8ull * NB * 9 + 4ull * NB * 2 + sizeof(InflateRec) * NB + 256;
        if (!c.ws_pjob.ensure(jb)) return nomem();
        uint64_t *d = c.ws_pjob.as<uint64_t>();
        uint64_t *d_soff = d, *d_slen = d + NB, *d_rbit = d + 2 * NB, *d_doff = d + 3 * NB, *d_dcap = d + 4 * NB;
        uint64_t *d_dlen = d + 5 * NB, *d_blk = d + 6 * NB, *d_moff = d + 8 * NB;
        uint32_t *d_hist = reinterpret_cast<uint32_t *>(d + 9 * NB);
        int32_t *d_stv = reinterpret_cast<int32_t *>(d_hist + NB);
        InflateRec *d_rec = reinterpret_cast<InflateRec *>((reinterpret_cast<uintptr_t>(d_stv + NB) + 63) & ~(uintptr_t)63);
        if (hipMemcpyAsync(d_soff, soff.data(), 8ull * NB, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_slen, slen.data(), 8ull * NB, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_rbit, rbit.data(), 8ull * NB, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_doff, doff.data(), 8ull * NB, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_dcap, dcap.data(), 8ull * NB, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_moff, moff.data(), 8ull * NB, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_hist, h32.data(), 4ull * NB, hipMemcpyHostToDevice, st) != hipSuccess)
            return -1;
        InflateJob job{};
        job.src = in; job.src_off = d_soff; job.src_len = d_slen;
        job.dst = out; job.dst_off = d_doff; job.dst_cap = d_dcap; job.dst_len = d_dlen;
        job.status = d_stv; job.first = 0; job.count = NB; job.wrap = 0;
        job.mrec_off = d_moff; job.mrec = mrec_ip;
        job.rec = d_rec;
        job.res_bit = d_rbit; job.res_hist = d_hist; job.blk_out = d_blk;
        job.stop_mode = 2 | 4;
        if (c.timer.run(3, st, [&] { return launch_inflate_stage(0, job, st); })) return -1;
        std::vector<InflateRec> r(NB);
        if (copy_sync(r.data(), d_rec, sizeof(InflateRec) * NB, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
        for (uint32_t j = 0; j < NB; j++) {
            Blk &B = chain[ip[j]];
            if (r[j].put != hist[j] + B.out || r[j].stop != (uint32_t)kIBlock) return 0;
            B.nm = r[j].nmatch;
        }
    }
    // ---- matches: symbols per block, then references block by block
    std::vector<ParBlkHost> pb;
    size_t j = 0;
    for (const Blk &B : chain) {
        if (B.slot >= 0) {                           // from its slot (copied even when literal-only)
            pb.push_back(ParBlkHost{B.o0, B.o0 + B.out, B.o0 - 32768, (uint64_t)B.slot * kSlotRec,
                                    (uint64_t)B.slot * kSlot + 32768, B.nm, 0});
        } else {
            if (B.nm) pb.push_back(ParBlkHost{B.o0, B.o0 + B.out, B.o0 - hist[j], moff[j], ~0ull, B.nm, 0});
            j++;
        }
    }
    if (!pb.empty()) {
        if (!c.ws_par1.ensure(sizeof(ParBlkHost) * pb.size() + 64) || !c.ws_imeta.ensure(64)) return nomem();
        uint32_t *sym = c.ws_psym.as<uint32_t>();
        uint32_t *err = reinterpret_cast<uint32_t *>(c.ws_imeta.as<uint64_t>() + 5);
        uint32_t e_host = 0;
        if (hipMemcpyAsync(c.ws_par1.p, pb.data(), sizeof(ParBlkHost) * pb.size(), hipMemcpyHostToDevice, st) !=
                hipSuccess ||
            hipMemsetAsync(err, 0, 4, st) != hipSuccess ||
            c.timer.run(4, st, [&] {
                int e = launch_infl_sym(out, slots, sym, c.ws_par1.p, (uint32_t)pb.size(), mrec, mrec_ip, err, st);
                for (size_t k = 0; !e && k < pb.size(); k++)
                    if (pb[k].nm) e = launch_infl_resolve(out, sym, pb[k].o0, pb[k].o1, st);
                return e;
            }) ||
            copy_sync(&e_host, err, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
            return -1;
        if (e_host) return 0;                        // a distance before the stream's start: the exact path reports it
    }
    // ---- the check value against the trailer
    uint8_t t[8] = {0};
    if (tlen && copy_sync(t, in + tb, tlen, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
    if (kind) {
        uint64_t *m = c.ws_imeta.ensure(64) ? c.ws_imeta.as<uint64_t>() : nullptr;
        if (!m) return -1;
        const uint64_t ol[2] = {0, total};
        uint32_t *ck = reinterpret_cast<uint32_t *>(m + 2);
        const size_t ckb = checksum_scratch_bytes(1);
        void *scr = ckb && c.ws_ck.ensure(ckb) ? c.ws_ck.p : nullptr;
        uint32_t got = 0;
        if (hipMemcpyAsync(m, ol, 16, hipMemcpyHostToDevice, st) != hipSuccess ||
            c.timer.run(0, st, [&] {
                return kind == 1 ? launch_adler32(out, m, m + 1, nullptr, ck, 1, scr, ckb, st)
                                 : launch_crc32(out, m, m + 1, nullptr, ck, 1, scr, ckb, st);
            }) ||
            copy_sync(&got, ck, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
            return -1;
        if (kind == 1) {
            const uint32_t want = (uint32_t)t[0] << 24 | (uint32_t)t[1] << 16 | (uint32_t)t[2] << 8 | t[3];
            if (got != want) return 0;
        } else {
            const uint32_t want = t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
            const uint32_t isz = t[4] | (uint32_t)t[5] << 8 | (uint32_t)t[6] << 16 | (uint32_t)t[7] << 24;
            if (got != want || isz != (uint32_t)total) return 0;
        }
    }
    out_len = total;
    used = tb + tlen;
    g_par_inflates.fetch_add(1);
    return 1;
}

int inflate_dev_locked(Ctx &c, const uint8_t *src, const uint64_t *src_off, const uint64_t *src_len,
                       uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap, uint64_t *dst_len,
                       uint64_t *src_used, int32_t *status, uint32_t *stop_out, uint32_t count, int wrap,
                       int wbits, hipStream_t st, const InflateResumeDev *rs) {
    if (wrap < 0 || wrap > 3) return ZGPU_STREAM_ERROR;
    if (count == 0) return ZGPU_OK;
    std::vector<uint64_t> lens(count), caps(count);
    if (hipMemcpyAsync(lens.data(), src_len, 8ull * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(caps.data(), dst_cap, 8ull * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    for (uint32_t i = 0; i < count; i++)
        if (lens[i] >= (1ull << 32) || caps[i] >= (1ull << 32)) return ZGPU_STREAM_ERROR;   // per-stream limit
    // a lone large stream: the block-parallel decode when it applies
    static const bool no_par = std::getenv("ZGPU_NO_PAR_INFLATE") != nullptr;    // A/B
    static const uint64_t par_min = [] {                 // ZGPU_PAR_INFLATE_MIN (tests): compressed bytes
        const char *e = std::getenv("ZGPU_PAR_INFLATE_MIN");
        return e ? (uint64_t)std::atoll(e) : (uint64_t)kParInflateMin;
    }();
    if (count == 1 && !rs && !no_par && lens[0] >= par_min && caps[0] > 0) {
        uint64_t so = 0, dof = 0;
        if (copy_sync(&so, src_off, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            copy_sync(&dof, dst_off, 8, hipMemcpyDeviceToHost, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
        uint64_t olen = 0, used = 0;
        const int pr = inflate_par_locked(c, src + so, lens[0], dst + dof, caps[0], wrap, wbits, st, olen, used);
        if (pr < 0) return ZGPU_MEM_ERROR;
        if (pr == 1) {
            const int32_t zok = 0;
            const uint32_t send = kIEnd;
            if (hipMemcpyAsync(dst_len, &olen, 8, hipMemcpyHostToDevice, st) != hipSuccess ||
                (src_used && hipMemcpyAsync(src_used, &used, 8, hipMemcpyHostToDevice, st) != hipSuccess) ||
                (status && hipMemcpyAsync(status, &zok, 4, hipMemcpyHostToDevice, st) != hipSuccess) ||
                (stop_out && hipMemcpyAsync(stop_out, &send, 4, hipMemcpyHostToDevice, st) != hipSuccess))
                return ZGPU_MEM_ERROR;
            const int rc = hip_ok(hipStreamSynchronize(st));
            c.timer.collect();
            return rc;
        }
    }
    const uint64_t budget = c.inflight;
    std::vector<uint32_t> cuts{0};
    {
        uint64_t acc = 0;
        for (uint32_t i = 0; i < count; i++) {
            const uint64_t w = caps[i] + lens[i];
            if (acc > 0 && acc + w > budget) { cuts.push_back(i); acc = 0; }
            acc += w;
        }
        cuts.push_back(count);
    }
    std::vector<uint64_t> moff(count);
    uint64_t max_rec = 0;
    uint32_t max_cnt = 0;
    for (size_t s = 0; s + 1 < cuts.size(); s++) {
        uint64_t acc = 0;
        for (uint32_t i = cuts[s]; i < cuts[s + 1]; i++) { moff[i] = acc; acc += caps[i] / 3 + 2; }
        max_rec = std::max(max_rec, acc);
        max_cnt = std::max(max_cnt, cuts[s + 1] - cuts[s]);
    }
    const size_t ckb = checksum_scratch_bytes(max_cnt);
    void *ck = ckb && c.ws_ck.ensure(ckb) ? c.ws_ck.p : nullptr;
    if (!c.ws_mrec.ensure(8 * max_rec + 64) || !c.ws_irec.ensure(sizeof(InflateRec) * max_cnt + 64) ||
        !c.ws_ick.ensure(8ull * max_cnt + 64) || !c.ws_imeta.ensure(8ull * count + 64))
        return ZGPU_MEM_ERROR;
    uint64_t *d_moff = c.ws_imeta.as<uint64_t>();
    if (hipMemcpyAsync(d_moff, moff.data(), 8ull * count, hipMemcpyHostToDevice, st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    StageTimer &T = c.timer;
    for (size_t s = 0; s + 1 < cuts.size(); s++) {
        const uint32_t a = cuts[s], b = cuts[s + 1];
        InflateJob job{};
        job.src = src; job.src_off = src_off; job.src_len = src_len;
        job.dst = dst; job.dst_off = dst_off; job.dst_cap = dst_cap; job.dst_len = dst_len;
        job.src_used = src_used; job.status = status; job.stop_out = stop_out;
        job.first = a; job.count = b - a; job.wrap = wrap; job.wbits = wbits;
        job.mrec_off = d_moff + a;
        job.mrec = c.ws_mrec.as<uint64_t>();
        job.rec = c.ws_irec.as<InflateRec>();
        job.adler = c.ws_ick.as<uint32_t>();
        job.crc = job.adler + max_cnt;
        job.crc_byte = device_crc_tables()->byte;
        if (rs) {
            job.res_bit = rs->res_bit;
            job.res_hist = rs->res_hist;
            job.blk_out = rs->blk_out;
            job.stop_mode = rs->stop_mode;
            job.zstate_out = rs->zstate_out;
            job.zcodes = rs->zstate_out != nullptr;
            job.dmax = rs->dmax;
            job.trees_after = rs->trees_after;
            job.eidx = rs->eidx;
            job.bidx = rs->bidx;
            job.icnt = rs->icnt;
            job.ecap = rs->ecap;
            job.bcap = rs->bcap;
        }
        if (T.run(3, st, [&] { return launch_inflate_stage(0, job, st); })) return ZGPU_MEM_ERROR;
        if (T.run(4, st, [&] { return launch_inflate_stage(1, job, st); })) return ZGPU_MEM_ERROR;
        if ((wrap & 1) && T.run(0, st, [&] {
                return launch_adler32(dst, dst_off + a, dst_len + a, nullptr, job.adler, b - a, ck, ckb, st); }))
            return ZGPU_MEM_ERROR;
        if ((wrap & 2) && T.run(0, st, [&] {
                return launch_crc32(dst, dst_off + a, dst_len + a, nullptr, job.crc, b - a, ck, ckb, st); }))
            return ZGPU_MEM_ERROR;
        if (T.run(5, st, [&] { return launch_inflate_stage(2, job, st); })) return ZGPU_MEM_ERROR;
    }
    int rc = hip_ok(hipStreamSynchronize(st));
    c.timer.collect();
    return rc;
}

// host-buffer inflate batch: pack, upload, run, download.  dst_len in:
// capacity, out: bytes written; src_used / stop optional.
int uncompress_host_locked(Ctx &c, const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                           size_t *dst_len, size_t *src_used, int *status, int *stop, size_t count, int wrap,
                           int wbits) {
    if (count == 0) return ZGPU_OK;
    std::vector<uint64_t> so(count), sl(count), dofs(count), dcap(count);
    uint64_t in_total = 0, out_total = 0;
    for (size_t i = 0; i < count; i++) {
        so[i] = in_total;
        sl[i] = src_len[i];
        in_total += (src_len[i] + 15) & ~15ull;
        dofs[i] = out_total;
        dcap[i] = dst_len[i];
        out_total += (dst_len[i] + 15) & ~15ull;
    }
    const size_t meta_bytes = 8 * 6 * count + 8 * count;
    if (!c.ws_io.ensure(in_total + 64) || !c.ws_io2.ensure(out_total + 64) ||
        !c.ws_small.ensure(meta_bytes + 64) || !c.ws_istop.ensure(4ull * count + 64))
        return ZGPU_MEM_ERROR;
    uint8_t *d_in = c.ws_io.as<uint8_t>(), *d_out = c.ws_io2.as<uint8_t>();
    uint64_t *d_so = c.ws_small.as<uint64_t>();
    uint64_t *d_sl = d_so + count, *d_do = d_sl + count, *d_dc = d_do + count, *d_dl = d_dc + count;
    uint64_t *d_used = d_dl + count;
    int32_t *d_st = reinterpret_cast<int32_t *>(d_used + count);
    uint32_t *d_stop = c.ws_istop.as<uint32_t>();
    hipStream_t st = c.own;
    for (size_t i = 0; i < count; i++)
        if (src_len[i] && hipMemcpyAsync(d_in + so[i], src[i], src_len[i], hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
    std::vector<uint64_t> m4;                          // alive until the call returns (the upload's source)
    {   // d_so, d_sl, d_do, d_dc are consecutive: one upload (a lone call's latency is its copies)
        m4.reserve(4 * count);
        m4.insert(m4.end(), so.begin(), so.end());
        m4.insert(m4.end(), sl.begin(), sl.end());
        m4.insert(m4.end(), dofs.begin(), dofs.end());
        m4.insert(m4.end(), dcap.begin(), dcap.end());
        (void)d_sl; (void)d_dc;
        if (hipMemcpyAsync(d_so, m4.data(), 32 * count, hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
    }
    int rc = inflate_dev_locked(c, d_in, d_so, d_sl, d_out, d_do, d_dc, d_dl, d_used, d_st, d_stop,
                                (uint32_t)count, wrap, wbits, st);
    if (rc) return rc;
    std::vector<uint64_t> ol(count), ou(count);
    std::vector<int32_t> os(count);
    std::vector<uint32_t> ostop(count);
    // the four result arrays in one wait, and a lone stream of at most 256 KiB of output space whole in
    // the same one (as compress_host_locked)
    const bool whole = count == 1 && dcap[0] > 0 && dcap[0] <= (uint64_t(256) << 10);
    std::vector<uint8_t> stage(whole ? dcap[0] : 0);
    if (hipMemcpyAsync(ol.data(), d_dl, 8 * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(ou.data(), d_used, 8 * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(os.data(), d_st, 4 * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(ostop.data(), d_stop, 4 * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        (whole && hipMemcpyAsync(stage.data(), d_out + dofs[0], dcap[0], hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    for (size_t i = 0; i < count; i++)
        if (ol[i] > dcap[i] || ou[i] > sl[i]) return ZGPU_MEM_ERROR;   // device-reported sizes (see compress_host_locked)
    for (size_t i = 0; i < count; i++) {
        if (whole) {
            if (ol[i]) std::memcpy(dst[i], stage.data(), ol[i]);
        } else if (ol[i] && copy_sync(dst[i], d_out + dofs[i], ol[i], hipMemcpyDeviceToHost, st) != hipSuccess) {
            return ZGPU_MEM_ERROR;
        }
        dst_len[i] = ol[i];
        if (src_used) src_used[i] = ou[i];
        if (status) status[i] = os[i];
        if (stop) stop[i] = (int)ostop[i];
    }
    return ZGPU_OK;
}

// One attempt of the streaming inflate(): the stream's input `in` (n bytes)
// decoded from its start (resume == false: header, blocks, trailer) or, raw,
// from the block header at bit start_bit with the window `hist` already in
// front of the output.  out receives hist + the new output (at most cap bytes
// in all); t the stop reason, the bytes used and the last block boundary.
struct InflateTry {
    uint32_t stop;
    int status;
    uint64_t put, used, blk_bit, blk_put;
    uint64_t zstate;               // InflateJob::zstate_out
    int64_t zmark;                 // inflateMark where the input ran out
    uint32_t zcodes;               // inflateCodesUsed of the last dynamic block decoded (~0: none)
};
// The consumption index of one streaming attempt (InflateJob::eidx / bidx),
// relative to the attempt's input and output arrays: e[2k], e[2k + 1] per
// symbol (output end | stored << 32 | BFINAL << 33; the input bit after its
// codes, a stored run's first byte); b = (bit, output) of each block
// boundary; ne / nb = those met (ne > e.size() / 2: the index stops short of
// the decode's end)
struct InflateIndex {
    std::vector<uint64_t> e, b;
    uint32_t ne = 0, nb = 0;
};
constexpr uint32_t kIdxCap = 1u << 20, kIdxBCap = 1u << 14;

int inflate_try_locked(Ctx &c, const uint8_t *in, size_t n, bool resume, uint64_t start_bit, const uint8_t *hist,
                       size_t hist_len, size_t cap, int wrap, int wbits, std::vector<uint8_t> &out, InflateTry &t,
                       uint32_t stop_mode = 0, uint32_t dmax = 0, InflateIndex *ix = nullptr,
                       uint64_t trees_after = 0) {
    if (!c.ws_io.ensure(n + 64) || !c.ws_io2.ensure(cap + 64) || !c.ws_small.ensure(8 * 16 + 64) ||
        !c.ws_istop.ensure(64))
        return ZGPU_MEM_ERROR;
    if (ix && !c.ws_iidx.ensure(16ull * kIdxCap + 16ull * kIdxBCap + 64)) ix = nullptr;
    uint8_t *d_in = c.ws_io.as<uint8_t>(), *d_out = c.ws_io2.as<uint8_t>();
    uint64_t *m = c.ws_small.as<uint64_t>();          // so sl do dc dl used | st | rbit hist | blk[2]
    int32_t *d_st = reinterpret_cast<int32_t *>(m + 6);
    uint64_t *d_rbit = m + 7;
    uint32_t *d_hist = reinterpret_cast<uint32_t *>(m + 8);
    uint64_t *d_blk = m + 9;
    uint64_t *d_zs = m + 11;
    uint32_t *d_stop = c.ws_istop.as<uint32_t>();
    hipStream_t st = c.own;
    const uint64_t meta[4] = {0, (uint64_t)n, 0, (uint64_t)cap};
    const uint64_t rbit = start_bit;
    const uint32_t hl = (uint32_t)hist_len;
    if ((n && hipMemcpyAsync(d_in, in, n, hipMemcpyHostToDevice, st) != hipSuccess) ||
        (hist_len && hipMemcpyAsync(d_out, hist, hist_len, hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipMemcpyAsync(m, meta, sizeof meta, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_rbit, &rbit, 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_hist, &hl, 4, hipMemcpyHostToDevice, st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    InflateResumeDev rs{resume ? d_rbit : nullptr, resume ? d_hist : nullptr, d_blk, stop_mode, d_zs, dmax};
    rs.trees_after = trees_after;
    if (ix) {
        rs.eidx = c.ws_iidx.as<uint64_t>();
        rs.bidx = rs.eidx + 2ull * kIdxCap;
        rs.icnt = reinterpret_cast<uint32_t *>(rs.bidx + 2ull * kIdxBCap);
        rs.ecap = kIdxCap;
        rs.bcap = kIdxBCap;
    }
    int rc = inflate_dev_locked(c, d_in, m, m + 1, d_out, m + 2, m + 3, m + 4, m + 5, d_st, d_stop, 1,
                                resume ? 0 : wrap, wbits, st, &rs);
    if (rc) return rc;
    uint64_t res[2], blk[4];
    int32_t status = 0;
    uint32_t stop = 0;
    if (copy_sync(res, m + 4, 16, hipMemcpyDeviceToHost, st) != hipSuccess ||
        copy_sync(blk, d_blk, 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
        copy_sync(&status, d_st, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        copy_sync(&stop, d_stop, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    if (res[0] > cap || res[1] > n) return ZGPU_MEM_ERROR;      // device-reported sizes (see compress_host_locked)
    out.resize(res[0]);
    if (res[0] && copy_sync(out.data(), d_out, res[0], hipMemcpyDeviceToHost, st) != hipSuccess) return ZGPU_MEM_ERROR;
    t.stop = stop;
    t.status = status;
    t.put = res[0];
    t.used = res[1];
    t.blk_bit = blk[0];
    t.blk_put = blk[1];
    t.zstate = blk[2];
    t.zmark = (int32_t)(uint32_t)blk[3];
    t.zcodes = (uint32_t)(blk[3] >> 32);
    if (ix) {
        uint32_t cnt[2];
        if (copy_sync(cnt, rs.icnt, 8, hipMemcpyDeviceToHost, st) != hipSuccess) return ZGPU_MEM_ERROR;
        ix->ne = cnt[0];
        ix->nb = cnt[1];
        ix->e.resize(2ull * std::min(cnt[0], kIdxCap));
        ix->b.resize(2ull * std::min(cnt[1], kIdxBCap));
        if ((!ix->e.empty() &&
             copy_sync(ix->e.data(), rs.eidx, 8 * ix->e.size(), hipMemcpyDeviceToHost, st) != hipSuccess) ||
            (!ix->b.empty() &&
             copy_sync(ix->b.data(), rs.bidx, 8 * ix->b.size(), hipMemcpyDeviceToHost, st) != hipSuccess))
            return ZGPU_MEM_ERROR;
        for (size_t k = 0; k < ix->e.size(); k += 2)          // device-reported positions (compress_host_locked)
            if ((uint32_t)ix->e[k] > cap + 258 || ix->e[k + 1] > ((ix->e[k] >> 32) & 1u ? n : 8ull * n))
                return ZGPU_MEM_ERROR;
    }
    return ZGPU_OK;
}

// host-buffer checksum batch.  Large buffers are cut into 1 MiB pieces so a
// single huge buffer still spreads over the whole GPU; pieces are joined with
// crc32_combine / adler32_combine (crc32.c:1021, adler32.c:133).
uint32_t adler_combine(uint32_t a1, uint32_t a2, int64_t len2);
uint32_t crc_combine(uint32_t c1, uint32_t c2, int64_t len2) {
    return multmodp(x2nmodp(len2, 3), c1) ^ c2;
}

int checksum_host_locked(Ctx &c, bool is_crc, const uint8_t *const *src, const size_t *len,
                         const uint32_t *init, uint32_t *out, size_t count) {
    constexpr uint64_t kPiece = 1ull << 20;
    struct Piece { size_t buf; uint64_t off, len; };
    std::vector<Piece> pieces;
    std::vector<size_t> first(count + 1);
    for (size_t i = 0; i < count; i++) {
        first[i] = pieces.size();
        uint64_t L = len[i];
        if (L == 0) { pieces.push_back({i, 0, 0}); continue; }
        for (uint64_t o = 0; o < L; o += kPiece) pieces.push_back({i, o, std::min(kPiece, L - o)});
    }
    first[count] = pieces.size();
    const size_t np = pieces.size();
    std::vector<uint64_t> po(np), pl(np);
    uint64_t total = 0;
    for (size_t k = 0; k < np; k++) {
        po[k] = total;
        pl[k] = pieces[k].len;
        total += (pieces[k].len + 15) & ~15ull;
    }
    if (!c.ws_io.ensure(total + 64) || !c.ws_small.ensure(8 * 2 * np + 8 * np + 64)) return ZGPU_MEM_ERROR;
    uint8_t *d_in = c.ws_io.as<uint8_t>();
    uint64_t *d_po = c.ws_small.as<uint64_t>(), *d_pl = d_po + np;
    uint32_t *d_init = reinterpret_cast<uint32_t *>(d_pl + np), *d_out = d_init + np;
    std::vector<uint32_t> pinit(np, is_crc ? 0u : 1u);
    for (size_t i = 0; i < count; i++)
        if (init) pinit[first[i]] = init[i];
    hipStream_t st = c.own;
    for (size_t k = 0; k < np; k++)
        if (pieces[k].len &&
            hipMemcpyAsync(d_in + po[k], src[pieces[k].buf] + pieces[k].off, pieces[k].len,
                           hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
    if (hipMemcpyAsync(d_po, po.data(), 8 * np, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_pl, pl.data(), 8 * np, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_init, pinit.data(), 4 * np, hipMemcpyHostToDevice, st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    const size_t ckb = checksum_scratch_bytes((uint32_t)np);
    void *ck = ckb && c.ws_ck.ensure(ckb) ? c.ws_ck.p : nullptr;
    int rc = is_crc ? launch_crc32(d_in, d_po, d_pl, d_init, d_out, (uint32_t)np, ck, ckb, st)
                    : launch_adler32(d_in, d_po, d_pl, d_init, d_out, (uint32_t)np, ck, ckb, st);
    if (rc) return ZGPU_MEM_ERROR;
    std::vector<uint32_t> res(np);
    if (copy_sync(res.data(), d_out, 4 * np, hipMemcpyDeviceToHost, st) != hipSuccess) return ZGPU_MEM_ERROR;
    for (size_t i = 0; i < count; i++) {
        uint32_t v = res[first[i]];
        for (size_t k = first[i] + 1; k < first[i + 1]; k++)
            v = is_crc ? crc_combine(v, res[k], (int64_t)pieces[k].len)
                       : adler_combine(v, res[k], (int64_t)pieces[k].len);
        out[i] = v;
    }
    return ZGPU_OK;
}

constexpr uint32_t kBase = 65521u;
uint32_t adler_combine(uint32_t adler1, uint32_t adler2, int64_t len2) {   // adler32.c:133-155
    if (len2 < 0) return 0xffffffffu;
    uint32_t rem = (uint32_t)(len2 % kBase);
    uint32_t s1 = adler1 & 0xffffu;
    uint32_t s2 = (uint32_t)(((uint64_t)rem * s1) % kBase);
    s1 += (adler2 & 0xffffu) + kBase - 1;
    s2 += ((adler1 >> 16) & 0xffffu) + ((adler2 >> 16) & 0xffffu) + kBase - rem;
    if (s1 >= kBase) s1 -= kBase;
    if (s1 >= kBase) s1 -= kBase;
    if (s2 >= (kBase << 1)) s2 -= (kBase << 1);
    if (s2 >= kBase) s2 -= kBase;
    return s1 | (s2 << 16);
}

uint64_t compress_bound64(uint64_t n) {                      // compress.c:72-75
    return n + (n >> 12) + (n >> 14) + (n >> 25) + 13;
}

}  // namespace

namespace zgpu {
const CrcTables *device_crc_tables() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDevices) return nullptr;
    return g_dev[d].d_crc;
}
}  // namespace zgpu

// ==========================================================================
// exported C ABI
// ==========================================================================
extern "C" {

int zgpu_init(void) { return ensure_init(); }

const char *zgpu_info(void) {
    int d = 0;
    if (current_device(&d)) return "libzgpu: no GPU";
    Device &D = g_dev[d];
    std::lock_guard<std::mutex> g(D.mu);
    if (init_device_locked(D, d) != ZGPU_OK) return "libzgpu: no GPU";
    return D.info.c_str();
}

size_t zgpu_set_inflight_bytes(size_t bytes) {
    size_t old = g_inflight;
    if (bytes >= (1u << 20)) g_inflight = bytes;
    return old;
}

void zgpu_stage_timing(int enable) {
    if (enable) g_timing_epoch++;
    g_timing = enable != 0;
}

// sums over every context of every device (read after the timed work ended)
int zgpu_stage_timing_read(double *ms, uint64_t *launches, int nstages) {
    int k = nstages < kStages ? nstages : kStages;
    for (int i = 0; i < k; i++) {
        if (ms) ms[i] = 0;
        if (launches) launches[i] = 0;
    }
    const uint64_t ep = g_timing_epoch;
    for (auto &D : g_dev) {
        std::lock_guard<std::mutex> g(D.mu);
        for (auto &p : D.pool) {
            if (p->timer_epoch != ep) continue;
            for (int i = 0; i < k; i++) {
                if (ms) ms[i] += p->timer.ms[i];
                if (launches) launches[i] += p->timer.n[i];
            }
        }
    }
    return k;
}

int zgpu_deflate_batch_dev_ex(const uint8_t *src, const uint64_t *src_off, const uint64_t *src_len,
                              uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap,
                              uint64_t *dst_len, int32_t *status, uint32_t count, int level, int wrap,
                              int strategy, void *stream) {
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    return deflate_dev_locked(c, src, src_off, src_len, dst, dst_off, dst_cap, dst_len, status,
                              count, level, wrap, strategy, static_cast<hipStream_t>(stream));
}

int zgpu_deflate_batch_dev2(const uint8_t *src, const uint64_t *src_off, const uint64_t *src_len,
                            uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap,
                            uint64_t *dst_len, int32_t *status, uint32_t count, int level, int window_bits,
                            int mem_level, int strategy, void *stream) {
    int wrap = 0, wbits = 0;
    if (parse_window(window_bits, mem_level, &wrap, &wbits)) return ZGPU_STREAM_ERROR;
    Lease L;
    if (L.rc) return L.rc;
    return deflate_dev_locked(*L.c, src, src_off, src_len, dst, dst_off, dst_cap, dst_len, status, count, level,
                              wrap, strategy, static_cast<hipStream_t>(stream), nullptr, wbits, mem_level);
}

int zgpu_deflate_batch_dev(const uint8_t *src, const uint64_t *src_off, const uint64_t *src_len,
                           uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap,
                           uint64_t *dst_len, int32_t *status, uint32_t count, int level, int wrap,
                           void *stream) {
    return zgpu_deflate_batch_dev_ex(src, src_off, src_len, dst, dst_off, dst_cap, dst_len, status,
                                     count, level, wrap, 0, stream);
}

int zgpu_crc32_batch_dev(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                         const uint32_t *init, uint32_t *out, uint32_t count, void *stream) {
    Lease L;
    if (L.rc) return L.rc;
    const size_t ckb = checksum_scratch_bytes(count);
    void *ck = ckb && L.c->ws_ck.ensure(ckb) ? L.c->ws_ck.p : nullptr;
    return launch_crc32(src, off, len, init, out, count, ck, ckb, static_cast<hipStream_t>(stream))
               ? ZGPU_MEM_ERROR : ZGPU_OK;
}

int zgpu_adler32_batch_dev(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                           const uint32_t *init, uint32_t *out, uint32_t count, void *stream) {
    Lease L;
    if (L.rc) return L.rc;
    const size_t ckb = checksum_scratch_bytes(count);
    void *ck = ckb && L.c->ws_ck.ensure(ckb) ? L.c->ws_ck.p : nullptr;
    return launch_adler32(src, off, len, init, out, count, ck, ckb, static_cast<hipStream_t>(stream))
               ? ZGPU_MEM_ERROR : ZGPU_OK;
}

int zgpu_compress_batch_ex(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                           size_t *dst_len, int *status, size_t count, int level, int wrap, int strategy) {
    for (size_t i = 0; i < count; i++)          // checked before any GPU work (and testable without one)
        if (src_len && src_len[i] >= kMaxBuffer) return ZGPU_STREAM_ERROR;
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    return compress_host_locked(c, src, src_len, dst, dst_len, status, count, level, wrap, strategy);
}

int zgpu_compress_batch2(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                         size_t *dst_len, int *status, size_t count, int level, int window_bits, int mem_level,
                         int strategy) {
    int wrap = 0, wbits = 0;
    if (parse_window(window_bits, mem_level, &wrap, &wbits)) return ZGPU_STREAM_ERROR;
    for (size_t i = 0; i < count; i++)
        if (src_len && src_len[i] >= kMaxBuffer) return ZGPU_STREAM_ERROR;
    Lease L;
    if (L.rc) return L.rc;
    return compress_host_locked(*L.c, src, src_len, dst, dst_len, status, count, level, wrap, strategy, nullptr,
                                wbits, mem_level);
}

int zgpu_compress_batch(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                        size_t *dst_len, int *status, size_t count, int level, int wrap) {
    return zgpu_compress_batch_ex(src, src_len, dst, dst_len, status, count, level, wrap, 0);
}

int zgpu_inflate_batch_dev(const uint8_t *src, const uint64_t *src_off, const uint64_t *src_len,
                           uint8_t *dst, const uint64_t *dst_off, const uint64_t *dst_cap,
                           uint64_t *dst_len, uint64_t *src_used, int32_t *status, uint32_t count,
                           int wrap, void *stream) {
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    return inflate_dev_locked(c, src, src_off, src_len, dst, dst_off, dst_cap, dst_len, src_used, status,
                              nullptr, count, wrap, 15, static_cast<hipStream_t>(stream));
}

int zgpu_uncompress_batch(const uint8_t *const *src, const size_t *src_len, uint8_t *const *dst,
                          size_t *dst_len, size_t *src_used, int *status, size_t count, int wrap) {
    if (wrap < 0 || wrap > 3) return ZGPU_STREAM_ERROR;
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    return uncompress_host_locked(c, src, src_len, dst, dst_len, src_used, status, nullptr, count, wrap, 15);
}

int zgpu_crc32_batch(const uint8_t *const *src, const size_t *len, const uint32_t *init,
                     uint32_t *out, size_t count) {
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    return checksum_host_locked(c, true, src, len, init, out, count);
}

int zgpu_adler32_batch(const uint8_t *const *src, const size_t *len, const uint32_t *init,
                       uint32_t *out, size_t count) {
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    return checksum_host_locked(c, false, src, len, init, out, count);
}

int zgpu_generate_dev(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed,
                      uint64_t first_index, void *stream) {
    int rc = ensure_init();
    if (rc) return rc;
    return launch_generate(dst, len, count, kind, seed, first_index, static_cast<hipStream_t>(stream))
               ? ZGPU_STREAM_ERROR : ZGPU_OK;
}

uint64_t zgpu_debug_par_inflates(void) { return g_par_inflates.load(); }

int zgpu_debug_parse_fallbacks(uint64_t *out) {
    Lease L;
    if (L.rc) return L.rc;
    return zgpu::parse_fallback_counts(out) ? ZGPU_STREAM_ERROR : ZGPU_OK;
}

int zgpu_debug_stages(const uint8_t *src, size_t n, int level, uint16_t *link, uint32_t *rfull,
                      uint32_t *rquart) {
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    if (level < 4 || level > 9) return ZGPU_STREAM_ERROR;
    const size_t nn = n ? n : 1;
    if (!c.ws_io.ensure(nn + 64) || !c.ws_link.ensure(2 * nn + 64) || !c.ws_rf.ensure(4 * nn + 64) ||
        !c.ws_rq.ensure(4 * nn + 64) || !c.ws_key.ensure(nn + 64) || !c.ws_small.ensure(64))
        return ZGPU_MEM_ERROR;
    uint64_t *d_meta = c.ws_small.as<uint64_t>();   // off, len, ws_off
    const uint64_t meta[3] = {0, (uint64_t)n, 0};
    hipStream_t st = c.own;
    if (copy_sync(d_meta, meta, sizeof meta, hipMemcpyHostToDevice, st) != hipSuccess ||
        (n && copy_sync(c.ws_io.p, src, n, hipMemcpyHostToDevice, st) != hipSuccess))
        return ZGPU_MEM_ERROR;
    DeflateJob job{};
    job.src = c.ws_io.as<uint8_t>(); job.src_off = d_meta; job.src_len = d_meta + 1;
    job.first = 0; job.count = 1; job.level = level; job.wrap = 1;
    job.wbits = 15; job.hbits = 15;                   // deflateInit_ defaults (deflate.c:444)
    job.cfg = kLevelCfg[level];
    job.ws_off = d_meta + 2;
    job.link = c.ws_link.as<uint16_t>();
    job.rfull = c.ws_rf.as<uint32_t>();
    job.rquart = c.ws_rq.as<uint32_t>();
    job.key = c.ws_key.as<uint8_t>();
    job.links_gh = n >= kLinksGhMin;                  // as the batch path picks k_links' head[] place
    // ZGPU_DEBUG_SEG=<bytes> (tests): run the stages per segment of that many
    // bytes (a multiple of kMatchTile), as a sub-batch of few large buffers does
    if (const char *dseg = std::getenv("ZGPU_DEBUG_SEG"); dseg && n) {
        const uint64_t sl = (uint64_t)std::atoll(dseg);
        if (sl == 0 || sl % kMatchTile) return ZGPU_STREAM_ERROR;
        std::vector<uint32_t> segs;
        for (uint64_t o = 0; o < n; o += sl) { segs.push_back(0); segs.push_back((uint32_t)o); }
        if (!c.ws_seg.ensure(4 * segs.size()) ||
            copy_sync(c.ws_seg.p, segs.data(), 4 * segs.size(), hipMemcpyHostToDevice, st) != hipSuccess)
            return ZGPU_MEM_ERROR;
        job.seg = c.ws_seg.as<uint32_t>();
        job.nseg = (uint32_t)(segs.size() / 2);
        job.seg_len = (uint32_t)sl;
        job.links_gh = 0;
    }
    if (launch_deflate_stage(0, job, nullptr, st) || launch_deflate_stage(1, job, nullptr, st) ||
        hipStreamSynchronize(st) != hipSuccess)
        return ZGPU_MEM_ERROR;
    if (link && n && copy_sync(link, job.link, 2 * n, hipMemcpyDeviceToHost, st) != hipSuccess) return ZGPU_MEM_ERROR;
    // k_match keeps the quartered budget's result only where it differs from
    // the full one (bit 31 of rfull); the debug view gives both in full
    std::vector<uint32_t> rf(n), rq(n);
    if (n && (copy_sync(rf.data(), job.rfull, 4 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
              copy_sync(rq.data(), job.rquart, 4 * n, hipMemcpyDeviceToHost, st) != hipSuccess))
        return ZGPU_MEM_ERROR;
    for (size_t p = 0; p < n; p++) {
        const uint32_t f = rf[p] & 0x7fffffffu;
        if (rfull) rfull[p] = f;
        if (rquart && level >= 5) rquart[p] = (rf[p] >> 31) ? rq[p] : f;
    }
    return ZGPU_OK;
}

// ---------------------------- zlib.h names ----------------------------

const char *zlibVersion(void) { return ZGPU_ZLIB_VERSION; }

uLong compressBound(uLong sourceLen) { return (uLong)compress_bound64(sourceLen); }

// compress2 of kMaxBuffer bytes or more.  compress.c:22-59 feeds the source
// through deflate() in uInt-sized pieces: Z_NO_FLUSH calls of 2^32 - 1 bytes,
// then Z_FINISH with the rest, the output in pieces of at most 2^32 - 1 bytes.
// Here the same calls go through the streaming engine, each piece further cut
// at every 1 GiB of input, so that no job spans 4 GiB (its kernels address a
// buffer with 32-bit positions).  Such an extra Z_NO_FLUSH call changes
// nothing in the stream: its only effect in the reference is fill_window calls
// at the decision points within MIN_LOOKAHEAD of its end, and at a window
// offset S (a multiple of w_size) those slide only when the end lies in
// (S + 2 w_size - 262, S + 2 w_size - 1] -- never for an end at a multiple of
// w_size.  Level 0 cuts its stored blocks by the input each call
// offers, so it gets the reference's pieces unchanged.
static int compress2_big(Bytef *dest, uLongf *destLen, const Bytef *source, uLong sourceLen, int level) {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    int err = deflateInit_(&zs, level, ZGPU_ZLIB_VERSION, (int)sizeof(z_stream));
    if (err != Z_OK) { *destLen = 0; return err; }
    const uint64_t kUIntMax = 0xffffffffull, kStep = 1ull << 30, n = sourceLen;
    uint64_t left = *destLen, pos = 0, piece_end = 0;
    zs.next_out = dest;
    zs.avail_out = 0;
    int flush = Z_NO_FLUSH;
    do {
        if (zs.avail_out == 0) {
            zs.avail_out = (uInt)(left > kUIntMax ? kUIntMax : left);
            left -= zs.avail_out;
        }
        if (zs.avail_in == 0) {
            if (pos == piece_end) piece_end = std::min(n, piece_end + kUIntMax);   // the reference's next piece
            // level 0: exactly the reference's pieces (its stored blocks follow
            // each call's input; the level-0 path cuts its own device jobs)
            const uint64_t end = level == 0 ? piece_end : std::min(piece_end, (pos / kStep + 1) * kStep);
            zs.next_in = const_cast<Bytef *>(source) + pos;
            zs.avail_in = (uInt)(end - pos);
            pos = end;
            flush = pos == n ? Z_FINISH : Z_NO_FLUSH;
        }
        err = deflate(&zs, flush);
    } while (err == Z_OK);
    *destLen = zs.total_out;
    deflateEnd(&zs);
    return err == Z_STREAM_END ? Z_OK : err;
}

static int compress2_body(Bytef *dest, uLongf *destLen, const Bytef *source, uLong sourceLen, int level) {
    if (!destLen) return Z_STREAM_ERROR;
    if (level != Z_DEFAULT_COMPRESSION && (level < 0 || level > 9)) { *destLen = 0; return Z_STREAM_ERROR; }
    if (!dest || (sourceLen && !source)) { *destLen = 0; return Z_STREAM_ERROR; }
    if ((uint64_t)sourceLen >= kMaxBuffer) return compress2_big(dest, destLen, source, sourceLen, level);
    size_t cap = *destLen;
    const uint8_t *s = source;
    uint8_t *d = dest;
    size_t sl = sourceLen;
    int st = 0;
    int rc = zgpu_compress_batch(&s, &sl, &d, &cap, &st, 1, level, ZGPU_WRAP_ZLIB);
    if (rc == ZGPU_ENODEV) { *destLen = 0; return Z_MEM_ERROR; }
    if (rc) { *destLen = 0; return rc; }
    *destLen = cap;
    return st;
}

int compress(Bytef *dest, uLongf *destLen, const Bytef *source, uLong sourceLen) {
    return compress2(dest, destLen, source, sourceLen, Z_DEFAULT_COMPRESSION);
}

// A single call of up to kSmallCk bytes (zlib users checksum chunk by chunk):
// the bytes are copied into the context's pinned staging buffer, the kernel
// reads them there over the host link and writes the result back into it --
// one launch and one synchronisation, no DMA copies or device metadata.
constexpr size_t kSmallCk = 64 * 1024;
constexpr size_t kPinBytes = kSmallCk + 64;
int checksum_small(bool is_crc, uint32_t init, const uint8_t *buf, size_t len, uint32_t *res) {
    Lease L;
    if (L.rc) return L.rc;
    Ctx &c = *L.c;
    if (!c.pin && hipHostMalloc(reinterpret_cast<void **>(&c.pin), kPinBytes, hipHostMallocDefault) != hipSuccess) {
        c.pin = nullptr;
        return ZGPU_MEM_ERROR;
    }
    uint64_t *meta = reinterpret_cast<uint64_t *>(c.pin);   // offset, length, init | result
    uint32_t *w = reinterpret_cast<uint32_t *>(meta + 2);
    meta[0] = 0;
    meta[1] = len;
    w[0] = init;
    w[1] = 0;
    if (len) std::memcpy(c.pin + 64, buf, len);
    // splitting one buffer over many waves pays from ~16 KiB on
    const size_t ckb = len > 16384 ? checksum_scratch_bytes(1) : 0;
    void *ck = ckb && c.ws_ck.ensure(ckb) ? c.ws_ck.p : nullptr;
    const int rc = is_crc ? launch_crc32(c.pin + 64, meta, meta + 1, w, w + 1, 1, ck, ckb, c.own)
                          : launch_adler32(c.pin + 64, meta, meta + 1, w, w + 1, 1, ck, ckb, c.own);
    if (rc || hipStreamSynchronize(c.own) != hipSuccess) return ZGPU_MEM_ERROR;
    *res = reinterpret_cast<volatile uint32_t *>(w)[1];
    return ZGPU_OK;
}

// The last failure of this thread's public crc32() / adler32() calls
// (zgpu_checksum_error): ZGPU_OK, or the library's error code.
thread_local int t_ck_error = ZGPU_OK;

static uint32_t checksum_one(bool is_crc, uint32_t init, const Bytef *buf, size_t len) {
    const uint8_t *p = buf;
    uint32_t out = 0;
    const int rc = len <= kSmallCk ? checksum_small(is_crc, init, p, len, &out)
                   : is_crc      ? zgpu_crc32_batch(&p, &len, &init, &out, 1)
                                 : zgpu_adler32_batch(&p, &len, &init, &out, 1);
    if (rc) {
        // zlib's crc32()/adler32() have no error return and there is no CPU
        // path.  A failed GPU call returns 0 (crc32(0, Z_NULL, 0)'s value) with
        // errno = EIO and the error code kept for zgpu_checksum_error(), and
        // says so on stderr (first failure of the process, then every 1000th).
        // ZGPU_CHECKSUM_ERROR=abort ends the process instead.
        static const bool abort_on = [] {
            const char *e = std::getenv("ZGPU_CHECKSUM_ERROR");
            return e && std::strcmp(e, "abort") == 0;
        }();
        static std::atomic<uint64_t> fails{0};
        const uint64_t k = fails.fetch_add(1);
        if (abort_on || k % 1000 == 0)
            std::fprintf(stderr, "libzgpu: %s of %zu bytes failed on the GPU (rc %d)%s\n", is_crc ? "crc32" : "adler32",
                         len, rc, abort_on ? "" : "; returned 0, errno EIO (zgpu_checksum_error)");
        if (abort_on) std::abort();
        t_ck_error = rc;
        errno = EIO;
        return 0;
    }
    return out;
}

int zgpu_checksum_error(int reset) {
    const int e = t_ck_error;
    if (reset) t_ck_error = ZGPU_OK;
    return e;
}

// The check values deflate() / inflate() and the dictionary calls compute for
// themselves (running checks, trailers, gzip header CRCs) go through these
// instead of the public crc32_z / adler32_z: a failed GPU call there is an
// error code of the call (Z_MEM_ERROR through the entry points' existing
// std::bad_alloc handlers), never the end of the host process.  (The public
// crc32() / adler32() have no error return: errno and zgpu_checksum_error.)
struct GpuCheckFailed : std::bad_alloc {
    const char *what() const noexcept override { return "libzgpu: GPU checksum failed"; }
};
static uint32_t ck_internal(bool is_crc, uint32_t init, const Bytef *buf, size_t len) {
    if (buf == nullptr) return is_crc ? 0u : 1u;
    const uint8_t *p = buf;
    uint32_t out = 0;
    const int rc = len <= kSmallCk ? checksum_small(is_crc, init, p, len, &out)
                   : is_crc      ? zgpu_crc32_batch(&p, &len, &init, &out, 1)
                                 : zgpu_adler32_batch(&p, &len, &init, &out, 1);
    if (rc) {
        // ZGPU_TEST_CHECKSUM_ZERO=1: tests/conftest.py's host-side tests on a
        // machine without a GPU (z_stream bookkeeping such as deflateBound after
        // deflateSetDictionary) take 0 here instead of the call's error
        static const bool test_zero = std::getenv("ZGPU_TEST_CHECKSUM_ZERO") != nullptr;
        if (test_zero) return 0;
        throw GpuCheckFailed();
    }
    return out;
}
static inline uint32_t ck_crc32(uint32_t crc, const Bytef *buf, size_t len) { return ck_internal(true, crc, buf, len); }
static inline uint32_t ck_adler32(uint32_t a, const Bytef *buf, size_t len) { return ck_internal(false, a, buf, len); }

uLong crc32_z(uLong crc, const Bytef *buf, size_t len) {
    if (buf == nullptr) return 0;                      // crc32.c:700
    return checksum_one(true, (uint32_t)crc, buf, len);
}
uLong crc32(uLong crc, const Bytef *buf, uInt len) { return crc32_z(crc, buf, len); }
uLong adler32_z(uLong adler, const Bytef *buf, size_t len) {
    if (buf == nullptr) return 1;                      // adler32.c:83-84
    return checksum_one(false, (uint32_t)adler, buf, len);
}
uLong adler32(uLong adler, const Bytef *buf, uInt len) { return adler32_z(adler, buf, len); }

uLong crc32_combine64(uLong crc1, uLong crc2, int64_t len2) {
    return crc_combine((uint32_t)crc1, (uint32_t)crc2, len2);
}
uLong crc32_combine(uLong crc1, uLong crc2, long len2) { return crc32_combine64(crc1, crc2, len2); }
uLong crc32_combine_gen64(int64_t len2) { return x2nmodp(len2, 3); }
uLong crc32_combine_gen(long len2) { return crc32_combine_gen64(len2); }
uLong crc32_combine_op(uLong crc1, uLong crc2, uLong op) {
    return multmodp((uint32_t)op, (uint32_t)crc1) ^ (uint32_t)crc2;
}
uLong adler32_combine64(uLong adler1, uLong adler2, int64_t len2) {
    return adler_combine((uint32_t)adler1, (uint32_t)adler2, len2);
}
uLong adler32_combine(uLong adler1, uLong adler2, long len2) { return adler32_combine64(adler1, adler2, len2); }

// zutil.c:131 zError: z_errmsg[Z_NEED_DICT - err] (zutil.c:12-23); a code
// outside Z_VERSION_ERROR..Z_NEED_DICT gets "" here instead of a read past the table
const char *zError(int err) {
    static const char *const msg[10] = {"need dictionary", "stream end", "", "file error", "stream error",
                                        "data error", "insufficient memory", "buffer error",
                                        "incompatible version", ""};
    return err <= 2 && err >= -6 ? msg[2 - err] : "";
}

// zutil.c:31 zlibCompileFlags: type sizes in bits 0..7 (uInt, uLong, voidpf,
// z_off_t: 0 = 16-bit, 1 = 32, 2 = 64), no debug / assembler / dynamic-table /
// FASTEST options.  The reference compiled here reports 0xa9.
uLong zlibCompileFlags(void) {
    auto sz = [](size_t b) -> uLong { return b == 2 ? 0 : b == 4 ? 1 : b == 8 ? 2 : 3; };
    return sz(sizeof(uInt)) | sz(sizeof(uLong)) << 2 | sz(sizeof(voidpf)) << 4 | sz(sizeof(int64_t)) << 6;
}

// crc32.c:549 get_crc_table: the byte-wise table of the reflected polynomial
// 0xedb88320 (the one crc32_z's byte loop uses); built once, never freed
const uint32_t *get_crc_table(void) {
    static CrcTables t;
    static std::once_flag once;
    std::call_once(once, [] { build_crc_tables(t); });
    return t.byte;
}

// The stream state and its buffers are allocated through the caller's
// zalloc / zfree, as deflateInit2_ / inflateInit2_ do (deflate.c:393-406,
// zutil.c:286-294): ZAlloc is a std allocator over them (malloc / free when
// the stream gives none).  An allocation that fails throws std::bad_alloc,
// which every entry point turns into Z_MEM_ERROR.
extern "C++" {
template <class T> struct ZAlloc {
    using value_type = T;
    alloc_func za = nullptr;
    free_func zf = nullptr;
    voidpf op = nullptr;
    ZAlloc() = default;
    ZAlloc(alloc_func a, free_func f, voidpf o) : za(a), zf(f), op(o) {}
    template <class U> ZAlloc(const ZAlloc<U> &o) : za(o.za), zf(o.zf), op(o.op) {}
    T *allocate(size_t n) {
        if (n == 0) n = 1;
        if (n > 0xffffffffull / sizeof(T)) throw std::bad_alloc();
        void *p = za ? za(op, (uInt)n, (uInt)sizeof(T)) : std::malloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return static_cast<T *>(p);
    }
    void deallocate(T *p, size_t) {
        if (zf) zf(op, p);
        else std::free(p);
    }
    template <class U> bool operator==(const ZAlloc<U> &o) const { return za == o.za && zf == o.zf && op == o.op; }
    template <class U> bool operator!=(const ZAlloc<U> &o) const { return !(*this == o); }
};
template <class T> using zvec = std::vector<T, ZAlloc<T>>;
}  // extern "C++"

// the defaults deflateInit2_ / inflateInit2_ store in the stream (zutil.c:286-294)
voidpf zgpu_zcalloc(voidpf, uInt items, uInt size) { return std::calloc(items, size); }
void zgpu_zcfree(voidpf, voidpf ptr) { std::free(ptr); }

// z_stream deflate: gather input, compress on the GPU at a flush call or at
// Z_FINISH, drain.
// one step of a streaming deflate job's timeline (see deflate_part)
struct StreamItem {
    uint64_t end_bit;        // part output bit after it
    uint64_t in_end, S, E;   // part positions: where it ends, the window offset, fill_window's end of input read
    uint32_t ev;             // a stop's or marker's event index (internal_state::ev_*), else ~0u
    uint32_t rec;            // the job's record index (blocks, markers)
    uint8_t kind, pbyte, res;
    uint8_t wu;              // bi_used at the record's last bi_windup, 0: none (deflateUsed)
};
enum : uint8_t { kItStop = 0, kItBlock = 1, kItMarker = 2, kItFinal = 3 };

struct internal_state {
    ZAlloc<uint8_t> al;
    explicit internal_state(const ZAlloc<uint8_t> &a = {})
        : al(a), in(a), out(a), ev_pos(a), ev_type(a), ev_aux(a), fast_head(a), fast_prev(a), l0_hist(a), hist(a), body(a),
          items(ZAlloc<StreamItem>(a)), evb(ZAlloc<uint32_t>(a)), iwin(a), cfg_pos(a), cfg_row(ZAlloc<LevelCfg>(a)),
          hr(ZAlloc<HrStretch>(a)) {}
    int level, wrap, strategy;
    zvec<uint8_t> in, out;          // deflate: the input since the last Z_FULL_FLUSH; output queue
    size_t out_pos;
    int finished;     // 0 gathering, 1 compressed / decoded
    // deflate(flush) calls (Z_PARTIAL_FLUSH, Z_SYNC_FLUSH, Z_FULL_FLUSH, Z_BLOCK):
    // the stream is the header, then one raw "part" per Z_FULL_FLUSH-separated
    // stretch of input (each starts from an empty window and byte aligned,
    // deflate.c:1225-1231), then the trailer
    int last_flush = -2;            // deflate.c: s->last_flush (deflateReset)
    bool flushed = false;           // a flush call was acted on
    bool header_done = false;
    zvec<uint64_t> ev_pos;          // the current part's flush calls (part-relative)
    zvec<uint32_t> ev_type;
    zvec<uint64_t> ev_aux;          // kEvPause events: the end of the block the call stopped after
    size_t part_out = 0;            // bytes of the current part already queued
    size_t in_base = 0;             // part position of in[0] (input behind the resume point is dropped)
    uint32_t check = 0;             // adler32 / crc32 of the stream's input before ck_pos
    size_t ck_pos = 0;              // part position the running check has reached
    // resume point: the state right after the last flush acted on in this part.
    // The next job compresses from there (its buffer starts at the window
    // offset S, the parse at the flush, the output at its bit) instead of from
    // the part start, so a stream with many flush calls costs linear work.
    // Levels 1..3 keep exact hash chains sequentially (deflate_fast inserts
    // selectively, deflate.c:1873-1897) and restart at the part start.
    size_t res_S = 0, res_pos = 0, res_ev = 0;
    uint64_t res_bits = 0;
    uint32_t res_byte = 0;
    // levels 1..3: k_parse_fast's hash chains at the resume point (head[] as
    // part positions, prev links of [res_S, res_pos)) and as the last job left them
    zvec<uint64_t> fast_head;       // level 1-3 head[] at the resume point: 64-bit part positions
    zvec<uint16_t> fast_prev;       // the prev links of part positions [fast_S, fast_at)
    uint64_t fast_at = 0, fast_S = 0;   // the snapshot's part position and its window offset
    uint32_t fast_pend = 0;             // strings a flush left unhashed there (s->insert)
    // level 0 (deflate_stored_call): the window's bytes (the last st_strstart
    // input bytes) and the part position of the input consumed, for a
    // deflateParams switch to a level that searches the window
    zvec<uint8_t> l0_hist;
    uint64_t l0_pos = 0;
    // inflate streams
    int inflating = 0;
    int wbits = 15;         // deflate: w_bits (9..15); inflate: inflateInit2_'s windowBits
    int mem_level = 8;      // deflate: memLevel (hash_bits = memLevel + 7)
    size_t tried = 0;       // input end (absolute) at the last decode attempt that ran out of input
    size_t cap = 0;         // output capacity of the next attempt (beyond the window)
    int result = Z_OK;      // once decoded: Z_STREAM_END, Z_DATA_ERROR or Z_NEED_DICT
    // inflate resume point: once a block of the stream is complete, every later
    // attempt decodes raw from the last block boundary (res_bit, absolute
    // input bit; res_put, absolute output byte) with the 32 KiB of output
    // before it (hist) as the window, so a stream fed in pieces costs linear
    // work.  in_base: absolute input offset of in[0]; ideliv: output bytes
    // handed out; out holds the decoded bytes not handed out yet.
    int imode = 0;          // 0: decode from the stream start, 1: resume
    int igz = 0;            // the stream has a gzip header (CRC-32 + ISIZE trailer)
    uint64_t res_bit = 0, res_put = 0, ideliv = 0;
    uint32_t icheck = 0;    // Adler-32 / CRC-32 of the output before res_put
    zvec<uint8_t> hist;
    // exact input accounting (inflate.c inf_leave: a call whose output space
    // ends first stops reading after the symbol it has no room for): cons =
    // absolute input consumed as the caller was told; in's bytes from cons on
    // were handed back and are expected again (held_at: the next_in they were
    // handed back at).  ix: the last decode's symbol index (InflateIndex::e)
    // with its input / output origins, the output it starts at and whether it
    // reaches the decode's end; fin_used: a finished stream's input end (the
    // trailer included); acct_done: the attempt set next_in / total_in itself
    uint64_t cons = 0, fin_used = 0;
    const Bytef *held_at = nullptr;
    std::vector<uint64_t> ix, ix2;                       // ix2: an earlier index that starts lower
    uint64_t ix_ibase = 0, ix_obase = 0, ix_o0 = 0, ix2_ibase = 0, ix2_obase = 0, ix2_o0 = 0;
    bool ix_all = false, acct_done = false;
    bool hdr_stop_now = false;                           // this call's decode stopped after a block header (Z_TREES)
    bool after_hdr = false;                              // the reference stands after a block header (LEN_ / COPY_)
    std::vector<uint64_t> bx;                            // the last decode's block boundaries (absolute bit, output)
    uint64_t bx_last = ~0ull;                            // the bit of the one that ends the last block (a Z_BLOCK stop)
    std::vector<uint64_t> hx;                            // its block headers' ends (absolute bit | BFINAL << 63, output)
    uint64_t out_at = 0;                                 // absolute output of out[0] (out_pos = ideliv - out_at)
    // the bits inflate.c holds in its bit buffer after the last call: where the
    // input ran out (iheld_end, from the last decode), or below 8 at a stop for
    // room (inflateSync searches the whole bytes among them first)
    uint32_t iheld = 0, iheld_end = 0;
    // deflateTune (deflate.c:805-820): the jobs' good/lazy/nice/chain
    bool tuned = false;
    LevelCfg tune{};
    // the timeline of the last streaming job (deflate_part): its output bytes
    // from part byte body_at on, its items, the next one to hand out (t) and
    // the one the resume point stands at (res_item, -1: before the first)
    zvec<uint8_t> body;
    size_t body_at = 0;
    std::vector<StreamItem, ZAlloc<StreamItem>> items;
    size_t t = 0;
    long res_item = -1;
    zvec<uint32_t> evb;                  // per event from job_ev on: the job's records before it
    size_t job_ev = 0;                   // the last job's first event
    bool trailer_due = false;            // Z_FINISH: the last block is out, the trailer not yet queued
    bool stale = true;                   // events changed since the last job
    bool job_closed = false;             // the last job ran to Z_FINISH
    bool tentative = false;              // the last event is a stop its call did not reach
    size_t rd = 0;                       // part position the reference's fill_window has read up to
    size_t rd_seen = 0;                  // ... as next_in / total_in show it
    size_t ev_done = 0;                  // events whose call got to them (stop reached, marker handed out)
    size_t flush_done = 0;               // part position of the last flush handed out
    uint64_t proc_bits = 0;              // part output bit after the last item handed out
    uint64_t res_E = 0;                  // the resume point's E (fill_window's end of input read)
    int res_cut = 0;                     // the resume point is a block cut (not a flush)
    int64_t st_strstart = 0, st_block_start = 0;   // level 0: deflate_stored's window offsets
    size_t job_base = 0;                 // res_S of the last job (snapshots are relative to it)
    uint32_t snap_rec = 0xffffffffu;     // levels 1..3: the record whose head[] the last job kept
    std::vector<uint32_t> snap_head;
    std::vector<uint16_t> snap_prev;
    const gz_header *gzhead = nullptr;   // deflateSetHeader: written by the first deflate() call
    bool dict_set = false;               // deflateSetDictionary: the zlib header's FDICT + DICTID
    uint32_t dict_id = 0;
    size_t dict_len = 0;                 // the dictionary bytes in the window (<= w_size), just before rd
                                         // (deflateResetKeep: the window carried over, < w_size + MAX_DIST)
    bool carried = false;                // deflateResetKeep carried the last stream's window into this one
    bool fn_mixed = false;               // deflateParams changed the compress function after data
    bool need_dict = false;              // inflate: Z_NEED_DICT answered, waiting for the dictionary
    uint32_t want_dict = 0;              // its DICTID
    gz_header *ihead = nullptr;          // inflateGetHeader: filled as the gzip header arrives
    // inflateSync (inflate.c:1375-1437): the search's progress (bytes of
    // 00 00 ff ff seen), and after a sync point was found the stream's tail
    // rule: 1 the trailer is read but not checked, 2 no trailer (no header had
    // been read: the rest is raw)
    bool isyncing = false;
    uint32_t isync_have = 0;
    int isync = 0;
    int idt = 0;                         // strm->data_type at the last inflate(Z_BLOCK) stop
    bool itype = false;                  // the resume point is a block boundary (inflate.c mode TYPE)
    bool itail = false;                  // Z_BLOCK stopped after the last block: the trailer is next
    uint64_t iadj = 0;                   // input consumed that total_in does not count (Z_NEED_DICT's call)
    // inflate's sliding window as inflate.c keeps it (updatewindow, inflate.c:391-434): created by
    // the first call that writes output unless that call ends the stream under Z_FINISH (or stops
    // on an error), then fed every call's output; inflateSetDictionary presets it.  What
    // inflateGetDictionary returns and inflateResetKeep carries into a raw stream.
    zvec<uint8_t> iwin;
    bool iwin_on = false;
    bool ivalid = true;                  // inflateValidate: the check values are verified (wrap & 4)
    // strm->adler as inflate.c keeps it on a zlib / gzip stream: 1 (zlib, after DICT) or 0 (gzip,
    // after its header), then the check of every byte written (inflate.c inf_leave UPDATE_CHECK)
    bool iadl_on = false;
    uint32_t iadl = 0;
    // where the last decode left inflate.c's state (InflateJob::zstate_out): mode STORED with no bits
    // held (inflateSyncPoint), inflateMark's value, inflateCodesUsed of the last dynamic block
    bool isyncpt = false;
    int64_t imark = -65536;
    uint32_t icodes = 0;
    uint32_t iprime_n = 0;               // inflatePrime's bits before the stream's first input
    unsigned char *iback_win = nullptr;  // inflateBackInit_: the caller's window (1 << wbits bytes)
    uint64_t iprime_v = 0;
    // configuration rows changed with input pending (deflateParams within the
    // same function, deflateTune; deflate.c:760-820): row cfg_row[k] governs
    // the current part's decision points from part position cfg_pos[k] on,
    // cfg0 the ones before cfg_pos[0]
    zvec<uint64_t> cfg_pos;
    std::vector<LevelCfg, ZAlloc<LevelCfg>> cfg_row;
    LevelCfg cfg0{};
    // deflate_state's prev_length / match_length across a function switch
    // (DeflateJob::zp0 / zm0): as the last job left them (exit_*), and as they
    // stand at the last switch (zl_*, part position zl_pos; ~0: none in this part)
    uint32_t exit_p = kMinMatch - 1, exit_m = kMinMatch - 1;
    uint32_t zl_p = kMinMatch - 1, zl_m = kMinMatch - 1;
    uint64_t zl_pos = ~0ull;
    bool prime_due = false;              // a deflatePrime event no job has written yet
    int bi_used = 0;                     // deflateUsed: ((bi_valid - 1) & 7) + 1 at the last bi_windup, 0: none
    // Stretches of the current part parsed by deflate_huff / deflate_rle between
    // deflate_slow stretches (deflateParams after data, deflate.c:760-803):
    // [a, b) part positions, b = ~0 while open.  Neither function inserts
    // strings, so the chains after b leave [a, b) out (DeflateJob::sk); the
    // first fill_window of the stretch still hashes the two s->insert strings
    // before a that deflate_slow's flush left (deflate.c:306-325), when it
    // reads at least 2 bytes (first_end: where the first call after a ended),
    // and the rolling ins_h is set afresh by every fill_window that reads
    // (deflate.c:307-310), so the strings after b hash as usual.
    struct HrStretch { uint64_t a, b, first_end; int fn; };   // fn: fn_of() before the stretch (1 fast, 2 slow)
    std::vector<HrStretch, ZAlloc<HrStretch>> hr;
    bool hr_lost = false;                // an open stretch's part ended (Z_FULL_FLUSH)
};

namespace {
// a state in the stream's memory (ZALLOC, deflate.c:406); nullptr when it fails
internal_state *new_state(z_streamp strm, const internal_state *copy = nullptr) {
    if (!strm->zalloc) { strm->zalloc = zgpu_zcalloc; strm->opaque = nullptr; }   // deflate.c:393-401
    if (!strm->zfree) strm->zfree = zgpu_zcfree;
    void *mem = strm->zalloc(strm->opaque, 1, (uInt)sizeof(internal_state));
    if (!mem) return nullptr;
    try {
        return copy ? new (mem) internal_state(*copy)
                    : new (mem) internal_state(ZAlloc<uint8_t>(strm->zalloc, strm->zfree, strm->opaque));
    } catch (const std::bad_alloc &) {
        strm->zfree(strm->opaque, mem);
        return nullptr;
    }
}
void free_state(z_streamp strm, internal_state *s) {
    s->~internal_state();
    strm->zfree(strm->opaque, s);
}
}  // namespace

int deflateInit2_(z_streamp strm, int level, int method, int windowBits, int memLevel, int strategy,
                  const char *version, int stream_size) {
    if (!version || version[0] != ZGPU_ZLIB_VERSION[0] || stream_size != (int)sizeof(z_stream))
        return Z_VERSION_ERROR;                         // deflate.c:386-389
    if (!strm) return Z_STREAM_ERROR;
    strm->msg = nullptr;
    if (level == Z_DEFAULT_COMPRESSION) level = 6;
    int wrap = 1, wbits = 15;
    if (parse_window(windowBits, memLevel, &wrap, &wbits) || method != Z_DEFLATED || strategy < 0 ||
        strategy > Z_FIXED || level < 0 || level > 9)
        return Z_STREAM_ERROR;                          // deflate.c:400-425
    internal_state *s = new_state(strm);
    if (!s) return Z_MEM_ERROR;
    s->level = level;
    s->wrap = wrap;
    s->wbits = wbits;
    s->mem_level = memLevel;
    s->strategy = strategy;
    s->out_pos = 0;
    s->finished = 0;
    s->check = wrap == 2 ? 0 : 1;
    strm->state = s;
    strm->total_in = strm->total_out = 0;
    strm->data_type = Z_UNKNOWN;
    strm->adler = wrap == 2 ? 0 : 1;
    return Z_OK;
}

int deflateInit_(z_streamp strm, int level, const char *version, int stream_size) {
    return deflateInit2_(strm, level, Z_DEFLATED, 15, 8, Z_DEFAULT_STRATEGY, version, stream_size);
}

namespace {
// ---------------------------------------------------------------------------
// Streaming deflate() at levels 1..9.  Every call that offers input or asks
// for a flush records an event: the end of the input it offers and its flush
// kind (0: Z_NO_FLUSH).  A job compresses the current part (the input since
// the last Z_FULL_FLUSH) from its resume point, with every event since, as
// one raw stream on the GPU: the parse stands still at each Z_NO_FLUSH call's
// need_more point and acts on each flush there, as deflate_slow /
// deflate_fast / deflate_rle / deflate_huff do.  It returns a timeline: its
// blocks and markers with the output bit after each and the input
// fill_window had read when each was flushed, and its stops.  deflate() hands
// out what the reference's call hands out -- every block flushed before the
// call's own stop, marker or final block -- and pauses after a block when
// avail_out is used up (FLUSH_BLOCK's need_more, deflate.c:1685-1690), having
// consumed only the input read by then.  A later job resumes at the last
// block cut handed out whose state a new job starts in (the lazy parse's
// simple state; for levels 1..3 with head[] as it stood there).
// ---------------------------------------------------------------------------
int deflate_part(internal_state *s, bool closed) {
    // a pause at the block the resume point stands at is behind it already
    while (s->res_ev < s->ev_pos.size() && s->ev_type[s->res_ev] == kEvPause && s->ev_aux[s->res_ev] <= s->res_pos)
        s->res_ev++;
    const size_t base = s->res_S, nev = s->ev_pos.size() - s->res_ev;
    std::vector<uint64_t> pos(nev + 1), aux(nev + 1, 0);
    for (size_t i = 0; i < nev; i++) {
        pos[i] = s->ev_pos[s->res_ev + i] - base;
        if (s->ev_type[s->res_ev + i] == kEvPause) aux[i] = s->ev_aux[s->res_ev + i] - base;
        if (s->ev_type[s->res_ev + i] == kEvPrime) aux[i] = s->ev_aux[s->res_ev + i];   // value | bits << 16
    }
    const uint8_t *sp = s->in.data() + (base - s->in_base);
    size_t sl = s->in_base + s->in.size() - base;
    // any windowBits / memLevel: blocks may be fixed-code where stored would
    // not fit the window (up to 9 bits a literal), plus headers and markers
    size_t cap = sl + (sl >> 2) + 1024 + 16ull * nev;
    s->body.resize(cap);
    uint8_t *dp = s->body.data();
    int st = 0;
    FlushHost fh{pos.data(), s->ev_type.data() + s->res_ev, (uint32_t)nev, closed ? 0 : 1,
                 (uint32_t)(s->res_pos - base), (uint32_t)(s->res_bits & 7),
                 s->res_byte & ((1u << (s->res_bits & 7)) - 1u), {0, 0, 0, 0}};
    fh.e0 = s->res_E > base ? (uint32_t)(s->res_E - base) : 0;
    fh.cut = s->res_cut;
    fh.aux = aux.data();
    std::vector<uint64_t> rec;
    std::vector<uint32_t> evb;
    fh.rec_out = &rec;
    fh.evb_out = &evb;
    // the configuration row at the resume point, and the changes after it
    LevelCfg job_cfg = s->tuned ? s->tune : kLevelCfg[s->level];
    std::vector<uint64_t> cpos;
    std::vector<LevelCfg> crow;
    if (!s->cfg_pos.empty()) {
        job_cfg = s->cfg0;
        for (size_t k = 0; k < s->cfg_pos.size(); k++) {
            if (s->cfg_pos[k] <= s->res_pos) {
                job_cfg = s->cfg_row[k];
            } else {
                cpos.push_back(s->cfg_pos[k] - base);
                crow.push_back(s->cfg_row[k]);
            }
        }
        fh.cfg_pos = cpos.data();
        fh.cfg_tab = crow.data();
        fh.ncfg = (uint32_t)cpos.size();
    }
    // The hash chains the job starts from.  deflate_fast inserts selectively
    // (deflate.c:1873-1897): where it parsed, its chains come from the snapshot
    // of its last resume point (fast_head / fast_prev at part position fast_at,
    // fast_pend strings still to be hashed there).  Everything after that -- or
    // everything, with no deflate_fast region in reach -- was inserted string by
    // string (deflate_slow, a dictionary, a stored stretch's s->insert strings
    // that fill_window hashes, deflate.c:318-335), the last two of a flush late.
    std::vector<uint32_t> head_in;
    const bool fast = s->level >= 1 && s->level <= 3 && s->strategy != Z_HUFFMAN_ONLY && s->strategy != Z_RLE;
    const bool slow = s->level >= 4 && s->strategy != Z_HUFFMAN_ONLY && s->strategy != Z_RLE;
    const uint64_t wsize = 1ull << s->wbits;
    const bool have_fast = !s->fast_head.empty() && s->fast_S <= base && base <= s->fast_at &&
                           s->fast_at + wsize > s->res_pos;
    if ((fast || slow) && have_fast && s->res_pos > base) {     // rebase the saved chains to this buffer
        head_in.resize(s->fast_head.size());
        for (size_t i = 0; i < head_in.size(); i++)
            head_in[i] = s->fast_head[i] > base ? (uint32_t)(s->fast_head[i] - base) : 0;
        fh.head_in = head_in.data();
        fh.prev_in = s->fast_prev.data() + (base - s->fast_S);
        fh.prev_n = (size_t)(s->fast_at - base);
    }
    const uint32_t snap_end = have_fast ? (uint32_t)(s->fast_at - s->fast_pend - base) : 0;
    if (fast && s->res_pos > base && !(have_fast && s->fast_at == s->res_pos)) {
        // the window's strings are inserted first, all but the last two (a preset
        // dictionary, deflateSetDictionary; or a window another function parsed):
        // from the snapshot's end on, or all of them with no snapshot
        const uint32_t d = (uint32_t)(s->res_pos - base);
        fh.dict = 1;
        fh.keep_head = have_fast ? 1 : 0;
        fh.pre_from = snap_end;
        fh.pre_ins = d >= kMinMatch ? d - (kMinMatch - 1) : 0;
        if (fh.pre_ins < fh.pre_from) fh.pre_ins = fh.pre_from;
    }
    if (slow && have_fast && snap_end > 0) fh.lk_n = snap_end;   // k_links: deflate_fast's links below snap_end
    // prev_length / match_length: the state a function switch left at its flush, else the clean one
    const bool at_switch = s->res_pos == s->zl_pos;
    fh.zp0 = fast ? (int)s->zl_p : (at_switch ? (int)s->zl_p : kMinMatch - 1);
    fh.zm0 = at_switch ? (int)s->zl_m : kMinMatch - 1;
    if (fast) {
        fh.snap_head = &s->snap_head;
        fh.snap_prev = &s->snap_prev;
    }
    // deflate_huff / deflate_rle stretches in this job's window: slow jobs
    // leave them out of k_links; fast jobs out of the strings k_parse_fast
    // inserts before it starts (pre_from .. pre_ins)
    if (slow || (fast && fh.dict)) {
        const uint64_t end = base + sl;
        for (const internal_state::HrStretch &h : s->hr) {
            if (h.b == ~0ull) continue;                          // open: this job is no slow job then
            const uint64_t a = std::max(h.a, (uint64_t)base), b = std::min(h.b, end);
            if (a >= b) continue;
            if (fh.sk.n == kMaxSkip) return Z_STREAM_ERROR;
            fh.sk.a[fh.sk.n] = (uint32_t)(a - base);
            fh.sk.b[fh.sk.n] = (uint32_t)(b - base);
            fh.sk.n++;
        }
    }
    // With Z_NO_FLUSH stops only (a large deflate() call and its Z_FINISH,
    // compress2 over 4 GiB) the lazy parse is the whole-input one from the
    // resume point -- a stop only holds fill_window back -- so the segmented
    // parse runs it and k_pbig6s places the stops and window offsets
    static const bool no_seg_stream = std::getenv("ZGPU_NO_SEGSTREAM") != nullptr;   // A/B
    static const uint64_t seg_min = [] {      // ZGPU_SEG_STREAM_MIN (tests): a smaller minimum
        const char *e = std::getenv("ZGPU_SEG_STREAM_MIN");
        return e ? (uint64_t)std::atoll(e) : kSegStreamMin;
    }();
    bool stops_only = slow && !no_seg_stream && cpos.empty() && !fh.head_in && fh.lk_n == 0 &&
                      fh.zp0 == kMinMatch - 1 && fh.zm0 == kMinMatch - 1 && sl - fh.start >= seg_min &&
                      ((sl - fh.start) >> s->wbits) <= kSegStreamSlides;
    if (!closed && nev == 0) stops_only = false;
    for (size_t i = 0; stops_only && i < nev; i++) stops_only = s->ev_type[s->res_ev + i] == 0;
    fh.seg_parse = stops_only ? 1 : 0;
    ZTRACE("part: base %zu nev %zu sl %zu cap %zu start %u bit0 %u e0 %u cut %d fast %d\n", base, nev, sl, cap,
           fh.start, fh.bit0, fh.e0, fh.cut, (int)fast);
    {
        Lease L;
        int rc = L.rc;
        if (!rc) rc = compress_host_locked(*L.c, &sp, &sl, &dp, &cap, &st, 1, s->level, ZGPU_WRAP_RAW, s->strategy,
                                           &fh, s->wbits, s->mem_level, &job_cfg);
        ZTRACE("part: rc %d st %d out %zu recs %zu evb %zu snap %u\n", rc, st, cap, rec.size() / 4, evb.size(),
               fh.snap_rec);
        if (rc || st) return rc == ZGPU_ENODEV ? Z_MEM_ERROR : (rc ? rc : st);
    }
    s->body.resize(cap);
    s->body_at = (size_t)(s->res_bits >> 3);
    s->job_base = base;
    s->exit_p = (uint32_t)(fh.out[4] & 0xffffu);     // the parse's state after the job's last event
    s->exit_m = (uint32_t)((fh.out[4] >> 16) & 0xffffu);
    s->snap_rec = fast ? fh.snap_rec : 0xffffffffu;
    // the timeline: records in order, each stop before the first record
    // flushed after it, each flush event's marker as its record
    const uint32_t nb = (uint32_t)(rec.size() / 4);
    const uint64_t bit0 = (uint64_t)s->body_at << 3;
    {
        // what the device reported must describe this job's input and output
        uint64_t lb = s->res_bits & 7, le = 0;
        bool ok = evb.size() == nev;
        for (uint32_t j = 0; ok && j < nb; j++) {
            const uint64_t eb = rec[4ull * j], x = rec[4ull * j + 2] & 0xffffffffu, S = rec[4ull * j + 2] >> 32,
                           E = rec[4ull * j + 3] & 0xffffffffu;
            ok = eb >= lb && eb <= 8ull * cap + 7 && x >= le && x <= sl && S <= x && E >= x && E <= sl;
            if (!ok) ZTRACE("part: bad record %u: bit %lu (last %lu, cap %zu) end %lu (last %lu) S %lu E %lu sl %zu\n",
                            j, (unsigned long)eb, (unsigned long)lb, cap, (unsigned long)x, (unsigned long)le,
                            (unsigned long)S, (unsigned long)E, sl);
            lb = eb;
            le = x;
        }
        for (size_t i = 0; ok && i < nev; i++) ok = evb[i] <= nb || evb[i] == 0xffffffffu;
        if (!ok) {
            ZTRACE("part: bad job (nb %u nev %zu evb %zu)\n", nb, nev, evb.size());
            return Z_STREAM_ERROR;
        }
    }
    s->items.clear();
    uint64_t last_bit = s->res_bits;
    size_t e = 0;
    for (uint32_t j = 0;; j++) {
        while (e < nev && evb[e] == j && (s->ev_type[s->res_ev + e] == 0 || s->ev_type[s->res_ev + e] == kEvPause)) {
            if (s->ev_type[s->res_ev + e] == kEvPause) {        // no item: the next fill reads further
                e++;
                continue;
            }
            StreamItem it{};
            it.kind = kItStop;
            it.end_bit = last_bit;
            it.in_end = it.E = s->ev_pos[s->res_ev + e];
            it.ev = (uint32_t)(s->res_ev + e);
            it.rec = ~0u;
            s->items.push_back(it);
            e++;
        }
        if (j == nb) break;
        StreamItem it{};
        it.end_bit = bit0 + rec[4ull * j];
        it.pbyte = (uint8_t)rec[4ull * j + 1];
        it.wu = (uint8_t)((rec[4ull * j + 1] >> 8) & 15u);
        it.in_end = base + (rec[4ull * j + 2] & 0xffffffffu);
        it.S = base + (rec[4ull * j + 2] >> 32);
        it.E = base + (rec[4ull * j + 3] & 0xffffffffu);
        it.res = (uint8_t)(rec[4ull * j + 3] >> 63);
        it.rec = j;
        it.ev = ~0u;
        if (e < nev && evb[e] == j) {
            it.kind = kItMarker;
            it.ev = (uint32_t)(s->res_ev + e);
            e++;
        } else {
            it.kind = closed && j + 1 == nb ? kItFinal : kItBlock;
        }
        s->items.push_back(it);
        last_bit = it.end_bit;
    }
    ZTRACE("part: items %zu\n", s->items.size());
    s->evb.assign(evb.begin(), evb.end());
    s->job_ev = s->res_ev;
    s->job_closed = closed;
    s->stale = false;
    s->prime_due = false;
    // the items before the resume point were handed out by earlier calls
    s->t -= (size_t)(s->res_item + 1);
    s->res_item = -1;
    return Z_OK;
}

// the running Adler-32 / CRC-32 up to part position `end`
void advance_check(internal_state *s, size_t end) {
    if (!s->wrap || s->ck_pos >= end) return;
    const uint8_t *p = s->in.data() + (s->ck_pos - s->in_base);
    const size_t n = end - s->ck_pos;
    s->check = s->wrap == 2 ? ck_crc32(s->check, p, n) : ck_adler32(s->check, p, n);
    s->ck_pos = end;
}

// a Z_FULL_FLUSH closes the part: the next starts with an empty window
void close_part(internal_state *s) {
    if (!s->hr.empty() && s->hr.back().b == ~0ull) s->hr_lost = true;   // ins_h now stale from another part
    s->hr.clear();
    s->in.clear();
    s->in_base = 0;
    s->ck_pos = 0;
    s->ev_pos.clear();
    s->ev_type.clear();
    s->ev_aux.clear();
    s->evb.clear();
    s->job_ev = 0;
    s->trailer_due = false;
    s->part_out = 0;
    s->res_S = s->res_pos = s->res_ev = 0;
    s->res_bits = 0;
    s->res_byte = 0;
    s->res_E = 0;
    s->res_cut = 0;
    s->fast_head.clear();
    s->fast_prev.clear();
    s->items.clear();
    s->t = 0;
    s->res_item = -1;
    s->stale = true;
    s->tentative = false;
    s->rd = s->rd_seen = 0;
    s->ev_done = 0;
    s->flush_done = 0;
    s->proc_bits = 0;
    s->body.clear();
    s->body_at = 0;
    s->cfg_pos.clear();                 // the current row goes on (s->level, s->tune)
    s->cfg_row.clear();
    s->zl_pos = ~0ull;                  // prev_length (zl_p) goes on: deflate_fast never resets it
}

// after a call: the latest item handed out that a new job can start at
void choose_resume(internal_state *s) {
    const bool fast = s->level >= 1 && s->level <= 3 && s->strategy != Z_HUFFMAN_ONLY && s->strategy != Z_RLE;
    for (long r = (long)s->t - 1; r > s->res_item; r--) {
        const StreamItem &it = s->items[(size_t)r];
        if (it.kind == kItStop || it.kind == kItFinal || !it.res) continue;
        if (fast && it.rec != s->snap_rec) continue;
        s->res_S = it.S;
        s->res_pos = it.in_end;
        s->res_bits = it.end_bit;
        s->res_byte = it.pbyte;
        s->res_E = it.E;
        s->res_cut = it.kind == kItBlock;
        // the events after it: a stop or marker comes after record `rec` when
        // its record index is above it; a pause applies after the record before
        // its index, so one at this record is behind the resume point already
        s->res_ev = s->ev_pos.size();
        for (size_t k = s->job_ev; k < s->ev_pos.size() && k - s->job_ev < s->evb.size(); k++) {
            const uint32_t b = s->evb[k - s->job_ev];
            if (b > it.rec + (s->ev_type[k] == kEvPause ? 1u : 0u)) { s->res_ev = k; break; }
        }
        if (fast) {
            // job-relative heads -> part positions in 64 bits: a part may run past 4 GiB
            // (in_base moves with every resume), a job never does (its input is < kMaxBuffer)
            const uint64_t b = s->job_base;
            s->fast_head.resize(s->snap_head.size());
            for (size_t i = 0; i < s->snap_head.size(); i++)
                s->fast_head[i] = s->snap_head[i] ? (uint64_t)s->snap_head[i] + b : 0;
            s->fast_prev.assign(s->snap_prev.begin(), s->snap_prev.end());
            s->fast_at = s->res_pos;
            s->fast_S = s->res_S;
            s->fast_pend = it.kind == kItBlock ? 0u : (uint32_t)std::min<uint64_t>(s->res_pos - s->res_S, kMinMatch - 1);
        }
        if (s->res_S > s->in_base) {                 // the input before the window is not needed again
            s->in.erase(s->in.begin(), s->in.begin() + (std::ptrdiff_t)(s->res_S - s->in_base));
            s->in_base = s->res_S;
        }
        size_t k = 0;                                 // rows behind the resume point: the job's first row
        while (k < s->cfg_pos.size() && s->cfg_pos[k] <= s->res_pos) s->cfg0 = s->cfg_row[k++];
        s->cfg_pos.erase(s->cfg_pos.begin(), s->cfg_pos.begin() + (std::ptrdiff_t)k);
        s->cfg_row.erase(s->cfg_row.begin(), s->cfg_row.begin() + (std::ptrdiff_t)k);
        s->res_item = r;
        return;
    }
}

void queue_header(internal_state *s) {                          // deflate.c:1002-1073
    if (s->header_done) return;
    s->header_done = true;
    if (s->wrap == 1) {
        uint32_t header = (8u + ((uint32_t)(s->wbits - 8) << 4)) << 8;
        const uint32_t flags = (s->strategy >= 2 || s->level < 2) ? 0u : s->level < 6 ? 1u : s->level == 6 ? 2u : 3u;
        header |= flags << 6;
        if (s->dict_set) header |= 0x20;                        // PRESET_DICT
        header += 31 - (header % 31);
        s->out.push_back((uint8_t)(header >> 8));
        s->out.push_back((uint8_t)header);
        if (s->dict_set)                                        // DICTID, most significant byte first
            for (int i = 3; i >= 0; i--) s->out.push_back((uint8_t)(s->dict_id >> (8 * i)));
    } else if (s->wrap == 2) {
        const uint8_t xfl = s->level == 9 ? 2 : (s->strategy >= 2 || s->level < 2) ? 4 : 0;
        const gz_header *h = s->gzhead;
        if (!h) {
            const uint8_t g[10] = {31, 139, 8, 0, 0, 0, 0, 0, xfl, 3};   // OS_CODE 3 (Unix)
            s->out.insert(s->out.end(), g, g + 10);
            return;
        }
        // deflateSetHeader's fields (deflate.c GZIP_STATE .. HCRC_STATE)
        std::vector<uint8_t> g = {31, 139, 8,
                                  (uint8_t)((h->text ? 1 : 0) + (h->hcrc ? 2 : 0) + (h->extra ? 4 : 0) +
                                            (h->name ? 8 : 0) + (h->comment ? 16 : 0)),
                                  (uint8_t)(h->time & 0xff), (uint8_t)((h->time >> 8) & 0xff),
                                  (uint8_t)((h->time >> 16) & 0xff), (uint8_t)((h->time >> 24) & 0xff), xfl,
                                  (uint8_t)(h->os & 0xff)};
        if (h->extra) {
            g.push_back((uint8_t)(h->extra_len & 0xff));
            g.push_back((uint8_t)((h->extra_len >> 8) & 0xff));
            g.insert(g.end(), h->extra, h->extra + (h->extra_len & 0xffff));
        }
        if (h->name)
            for (const Bytef *p = h->name;; p++) { g.push_back(*p); if (!*p) break; }
        if (h->comment)
            for (const Bytef *p = h->comment;; p++) { g.push_back(*p); if (!*p) break; }
        if (h->hcrc) {                                          // the header's CRC-32, low 16 bits
            const uint32_t c = ck_crc32(0, g.data(), g.size());
            g.push_back((uint8_t)(c & 0xff));
            g.push_back((uint8_t)((c >> 8) & 0xff));
        }
        s->out.insert(s->out.end(), g.begin(), g.end());
    }
}

// input given to deflate() since the last point where the whole stream is
// known (the start, or a flush that compressed everything)
bool pending_input(const internal_state *s) {
    if (s->last_flush == -2 || s->finished) return false;
    if (s->level == 0) return !s->in.empty();
    return s->in_base + s->in.size() > s->flush_done || s->ev_done < s->ev_type.size() || s->t < s->items.size();
}

void drain(z_streamp strm, internal_state *s) {
    size_t take = std::min<size_t>(strm->avail_out, s->out.size() - s->out_pos);
    std::memcpy(strm->next_out, s->out.data() + s->out_pos, take);
    s->out_pos += take;
    strm->next_out += take;
    strm->avail_out -= (uInt)take;
    strm->total_out += take;
    if (s->out_pos == s->out.size() && !s->finished) {
        s->out.clear();
        s->out_pos = 0;
    }
}

inline int flush_rank(int f) { return f * 2 - (f > 4 ? 9 : 0); }   // deflate.c: RANK

// Level 0: one deflate() call of deflate_stored (deflate.c:1635-1815), its
// block cuts made here exactly as the reference makes them -- its first loop
// sends stored blocks straight to next_out while the output space holds a
// whole worthy (min_block) or flushed block, the rest of the input fills the
// window, and a worthy or flushed block goes through the pending buffer --
// with the window offsets (strstart, block_start), the pending buffer size and
// the output space it sees.  The blocks and deflate()'s markers are written by
// k_encode on the GPU from a host-made block list (DeflateJob::plan).  s->in
// holds the window's unsent bytes [block_start, strstart).
int deflate_stored_call(z_streamp strm, internal_state *s, int flush) {
    // deflate.c:1192: deflate_stored runs when there is input or a flush
    if (strm->avail_in == 0 && flush == Z_NO_FLUSH) return Z_OK;
    const uint64_t w_size = 1ull << s->wbits, window_size = 2 * w_size;
    const uint64_t pbs = 1ull << (s->mem_level + 8);          // pending_buf_size = lit_bufsize * 4
    constexpr uint64_t kMaxStored = 65535;
    int64_t &strstart = s->st_strstart, &block_start = s->st_block_start;
    uint64_t aout = strm->avail_out;                            // the output space as the reference sees it
    uint32_t bits = (uint32_t)(s->res_bits & 7);                // bi_valid
    std::vector<BlockRec> plan;
    std::vector<uint8_t> buf(s->in.begin(), s->in.end());      // the job's input: unsent window bytes, then reads
    uint64_t bpos = 0;                                          // buf position of the next byte to send
    auto read = [&](uint64_t n) {                               // read_buf (deflate.c:218-239)
        if (!n) return;
        buf.insert(buf.end(), strm->next_in, strm->next_in + n);   // (the check: once per call, below)
        strm->next_in += n;
        strm->avail_in -= (uInt)n;
        strm->total_in += n;
    };
    auto block = [&](uint64_t len, bool last) {                 // _tr_stored_block + flush_pending
        BlockRec r{};
        r.in_start = bpos;
        r.in_end = bpos + len;
        r.flags = last ? kBlkLast : 0u;
        plan.push_back(r);
        const uint64_t bytes = (bits + 3 + 7) / 8 + 4 + len;
        aout -= std::min(aout, bytes);
        bits = 0;
        bpos += len;
    };
    uint64_t min_block = std::min(pbs - 5, w_size);
    const uint64_t used0 = strm->avail_in;
    const Bytef *const in0 = strm->next_in;                     // this call's reads start here
    bool last = false;
    do {                                                        // deflate.c:1652-1725
        uint64_t len = kMaxStored;
        uint64_t have = (bits + 42) >> 3;
        if (aout < have) break;
        have = aout - have;
        const uint64_t left = (uint64_t)(strstart - block_start);
        if (len > left + strm->avail_in) len = left + strm->avail_in;
        if (len > have) len = have;
        if (len < min_block && ((len == 0 && flush != Z_FINISH) || flush == Z_NO_FLUSH || len != left + strm->avail_in))
            break;
        last = flush == Z_FINISH && len == left + strm->avail_in;
        const uint64_t from_win = std::min(left, len);
        block_start += (int64_t)from_win;
        read(len - from_win);                                   // straight from next_in
        block(len, last);
    } while (!last);
    const uint64_t used = used0 - strm->avail_in;
    if (used) {                                                 // deflate.c:1733-1760
        if (used >= w_size) {
            strstart = (int64_t)w_size;
        } else {
            if (window_size - (uint64_t)strstart <= used) strstart -= (int64_t)w_size;
            strstart += (int64_t)used;
        }
        block_start = strstart;
    }
    int bstate;                                                 // 0 need_more, 1 block_done, 2 finish_started, 3 finish_done
    if (last) {
        bstate = 3;
    } else if (flush != Z_NO_FLUSH && flush != Z_FINISH && strm->avail_in == 0 && strstart == block_start) {
        bstate = 1;
    } else {
        uint64_t have = window_size - (uint64_t)strstart;       // fill the window (deflate.c:1770-1790)
        if (strm->avail_in > have && block_start >= (int64_t)w_size) {
            block_start -= (int64_t)w_size;
            strstart -= (int64_t)w_size;
            have += w_size;
        }
        if (have > strm->avail_in) have = strm->avail_in;
        read(have);
        strstart += (int64_t)have;
        have = (bits + 42) >> 3;                                // a block through pending (deflate.c:1792-1813)
        have = std::min(pbs - have, kMaxStored);
        min_block = std::min(have, w_size);
        const uint64_t left = (uint64_t)(strstart - block_start);
        if (left >= min_block ||
            ((left || flush == Z_FINISH) && flush != Z_NO_FLUSH && strm->avail_in == 0 && left <= have)) {
            const uint64_t len = std::min(left, have);
            last = flush == Z_FINISH && strm->avail_in == 0 && len == left;
            block(len, last);
            block_start += (int64_t)len;
        }
        bstate = last ? 2 : 0;
    }
    if (bstate == 1) {                                          // deflate.c:1211-1233: the flush's marker
        BlockRec r{};
        r.in_start = r.in_end = bpos;
        r.flags = kBlkMarker | ((uint32_t)flush << 4);
        plan.push_back(r);
        if (flush == Z_FULL_FLUSH) strstart = block_start = 0;
    }
    {   // deflateUsed: _tr_stored_block winds up after each header, the final block once more
        uint32_t b = (uint32_t)(s->res_bits & 7);
        for (const BlockRec &r : plan) {
            const uint32_t mk = (r.flags & kBlkMarker) ? blk_marker_kind(r.flags) : 0;
            if (!(r.flags & kBlkMarker) || mk == 2 || mk == 3) {
                s->bi_used = (int)((b + 2) & 7) + 1;
                b = 0;
                if (r.flags & kBlkLast) s->bi_used = 8;
            } else if (mk == 1) {
                b = (b + 10) & 7;                          // _tr_align: a static empty block, bi_flush
            }
        }
    }
    // The call's blocks go to the device as jobs of at most kL0Job input bytes
    // (the kernels address a job's input with 32-bit positions; a compress2 of
    // 4 GiB and more offers 2^32 - 1 bytes to one call, compress.c:44-54).  A
    // stored block ends byte-aligned, so a job after the first starts at a
    // whole byte and the jobs' outputs simply follow each other.
    constexpr uint64_t kL0Job = 1ull << 30;
    for (size_t i0 = 0; i0 < plan.size();) {
        const uint64_t base = plan[i0].in_start;
        size_t i1 = i0 + 1;
        while (i1 < plan.size() && plan[i1].in_end - base <= kL0Job) i1++;
        std::vector<BlockRec> sub(plan.begin() + (std::ptrdiff_t)i0, plan.begin() + (std::ptrdiff_t)i1);
        for (BlockRec &r : sub) r.in_start -= base, r.in_end -= base;
        const uint64_t jn = sub.back().in_end;
        std::vector<uint8_t> body((size_t)compress_bound64(jn) + 64 + 8 * sub.size());
        const uint8_t *sp = buf.data() + base;
        uint8_t *dp = body.data();
        size_t sl = jn, cap = body.size();
        int st = 0;
        FlushHost fh{nullptr, nullptr, 0, 1, 0, (uint32_t)(s->res_bits & 7),
                     s->res_byte & ((1u << (s->res_bits & 7)) - 1u), {0, 0, 0, 0}};
        fh.plan = sub.data();
        fh.nplan = (uint32_t)sub.size();
        {
            Lease L;
            int rc = L.rc;
            if (!rc) rc = compress_host_locked(*L.c, &sp, &sl, &dp, &cap, &st, 1, 0, ZGPU_WRAP_RAW, s->strategy, &fh,
                                               s->wbits, s->mem_level);
            if (rc || st) return rc == ZGPU_ENODEV ? Z_MEM_ERROR : (rc ? rc : st);
        }
        const size_t jb = (size_t)(s->res_bits >> 3);
        s->out.insert(s->out.end(), body.begin() + (std::ptrdiff_t)(s->part_out - jb),
                      body.begin() + (std::ptrdiff_t)cap);
        s->part_out = jb + cap;
        s->res_bits = ((uint64_t)jb << 3) + fh.out[1];
        s->res_byte = (uint32_t)fh.out[3];
        // hand the job's bytes out now: the plan fits the caller's space (aout),
        // and the queue stays one job's size (a zalloc'd buffer is under 4 GiB)
        drain(strm, s);
        i0 = i1;
    }
    s->in.assign(buf.begin() + (std::ptrdiff_t)bpos, buf.end());   // the window's unsent bytes
    {   // read_buf's running check over everything this call read (one contiguous run from in0)
        const uint64_t rd = used0 - strm->avail_in;
        if (rd && s->wrap == 1) s->check = ck_adler32(s->check, in0, rd);
        else if (rd && s->wrap == 2) s->check = ck_crc32(s->check, in0, rd);
    }
    {   // the window: the last strstart bytes read (deflate.c:1733-1790 keep them contiguous)
        const uint64_t rd = used0 - strm->avail_in, keep = (uint64_t)strstart;
        if (rd >= keep) {
            s->l0_hist.assign(in0 + (rd - keep), in0 + rd);
        } else {
            s->l0_hist.insert(s->l0_hist.end(), in0, in0 + rd);
            if (s->l0_hist.size() > keep) s->l0_hist.erase(s->l0_hist.begin(), s->l0_hist.end() - (std::ptrdiff_t)keep);
        }
        s->l0_pos += rd;
        if (bstate == 1 && flush == Z_FULL_FLUSH) s->l0_hist.clear(), s->l0_pos = 0;   // a new part
    }
    if (s->wrap) strm->adler = s->check;
    drain(strm, s);
    if (bstate == 1 && flush == Z_FULL_FLUSH) s->part_out = 0, s->res_bits = 0;   // a new part: byte aligned
    if (bstate == 3) {                                          // finish_done: the trailer now
        s->finished = 1;
        if (s->wrap) {
            const uint32_t ck = s->check;
            if (s->wrap == 1) {
                for (int i = 3; i >= 0; i--) s->out.push_back((uint8_t)(ck >> (8 * i)));
            } else {
                const uint32_t isz = (uint32_t)strm->total_in;
                for (int i = 0; i < 4; i++) s->out.push_back((uint8_t)(ck >> (8 * i)));
                for (int i = 0; i < 4; i++) s->out.push_back((uint8_t)(isz >> (8 * i)));
            }
        }
        drain(strm, s);
        return s->out_pos == s->out.size() ? Z_STREAM_END : Z_OK;
    }
    if (bstate == 2) {                                          // finish_started: the trailer with a later call
        s->finished = 1;
        s->trailer_due = true;
    }
    if (strm->avail_out == 0) s->last_flush = -1;
    return Z_OK;
}

// part output bytes [part_out, to) of the last job into the output queue
void queue_to(internal_state *s, size_t to) {
    if (to <= s->part_out) return;
    s->out.insert(s->out.end(), s->body.begin() + (std::ptrdiff_t)(s->part_out - s->body_at),
                  s->body.begin() + (std::ptrdiff_t)(to - s->body_at));
    s->part_out = to;
}

// the input the reference has read by now (s->rd) out of next_in / avail_in
void sync_input(z_streamp strm, internal_state *s) {
    if (s->rd <= s->rd_seen) return;
    const size_t d = s->rd - s->rd_seen;
    strm->next_in += d;
    strm->avail_in -= (uInt)d;
    strm->total_in += d;
    s->rd_seen = s->rd;
}

void queue_trailer(z_streamp strm, internal_state *s) {        // deflate.c:1236-1262
    if (!s->wrap) return;
    advance_check(s, s->in_base + s->in.size());
    const uint32_t ck = s->check;
    strm->adler = ck;
    if (s->wrap == 1) {
        for (int i = 3; i >= 0; i--) s->out.push_back((uint8_t)(ck >> (8 * i)));
    } else {
        const uint32_t isz = (uint32_t)strm->total_in;
        for (int i = 0; i < 4; i++) s->out.push_back((uint8_t)(ck >> (8 * i)));
        for (int i = 0; i < 4; i++) s->out.push_back((uint8_t)(isz >> (8 * i)));
    }
}

// Hands out the timeline from s->t on, as the reference's call does, until
// the call's own event `own` (its stop or its marker; ~0u: Z_FINISH, the
// final block) or until avail_out is used up after a block.  *full: a
// Z_FULL_FLUSH marker was handed out (the part ends).
int run_items(z_streamp strm, internal_state *s, uint32_t own, bool *full) {
    while (s->t < s->items.size()) {
        const StreamItem it = s->items[s->t];
        s->t++;
        if (it.kind == kItStop) {                 // need_more (deflate.c:1941-1944)
            s->rd = it.E;
            if (it.ev == own) {
                s->ev_done = own + 1;
                s->tentative = false;
                return Z_OK;
            }
            continue;
        }
        if (it.E > s->rd) s->rd = it.E;
        s->proc_bits = it.end_bit;
        if (it.wu) s->bi_used = it.wu;
        if (it.kind == kItFinal) {                // FLUSH_BLOCK(s, 1), then the trailer
            queue_to(s, s->body_at + s->body.size());
            s->rd = s->in_base + s->in.size();
            sync_input(strm, s);
            s->finished = 1;
            drain(strm, s);
            if (strm->avail_out == 0) {           // finish_started: the trailer comes with a later call
                s->trailer_due = true;
                s->last_flush = -1;
                return Z_OK;
            }
            queue_trailer(strm, s);               // finish_done (deflate.c:1236-1262)
            drain(strm, s);
            return s->out_pos == s->out.size() ? Z_STREAM_END : Z_OK;
        }
        queue_to(s, (size_t)(it.end_bit >> 3));
        drain(strm, s);
        if (it.kind == kItMarker) {               // block_done: the flush's marker (deflate.c:1211-1233)
            if (s->ev_type[it.ev] == kEvPrime) continue;   // a deflatePrime's bits (the parse stands behind them)
            s->rd = it.in_end;
            if (it.ev != own) continue;           // an earlier flush left without bits (Z_BLOCK)
            s->ev_done = own + 1;
            s->flush_done = it.in_end;
            *full = s->ev_type[own] == Z_FULL_FLUSH;
            if (strm->avail_out == 0) s->last_flush = -1;
            return Z_OK;
        }
        if (strm->avail_out == 0) {               // FLUSH_BLOCK's need_more (deflate.c:1685-1690)
            s->last_flush = -1;
            if (own != ~0u && s->ev_type[own] == 0) s->tentative = true;
            return Z_OK;
        }
    }
    return Z_OK;
}
}  // namespace

// A stop turned into a pause (more input after a call that paused inside a block) applies after the paused
// block's record.  When the resume point chosen at the end of that call is that record itself, the pause is
// behind it -- choose_resume's rule for pauses (a pause at the resume record is behind it), which could not
// see this one, as it was still a stop then -- and the next job must not carry it: the window's read state
// at the resume point is the record's own (res_E).  A job starting at the pause's block end with the pause
// among its events produced no records and the stream made no progress (round 6, tools/header_first_probe.py).
static void drop_pause_behind_resume(internal_state *s, size_t le) {
    if (s->res_item < 0 || le + 1 != s->ev_type.size() || s->res_pos < s->ev_aux[le]) return;
    s->ev_pos.pop_back();
    s->ev_type.pop_back();
    s->ev_aux.pop_back();
    s->ev_done = s->ev_type.size();
    if (s->res_ev > s->ev_type.size()) s->res_ev = s->ev_type.size();
}

static void stream_trace(const char *where, z_streamp strm, const internal_state *s, int flush) {
    static const bool on = std::getenv("ZGPU_STREAM_TRACE") != nullptr;
    if (!on) return;
    std::fprintf(stderr, "[%s] flush %d in %u out %u total_in %lu rd %zu seen %zu C %zu in_base %zu ev %zu done %zu "
                 "items %zu t %zu res_item %ld res_S %zu res_pos %zu part_out %zu body_at %zu body %zu q %zu/%zu\n",
                 where, flush, strm->avail_in, strm->avail_out, (unsigned long)strm->total_in, s->rd, s->rd_seen,
                 s->in_base + s->in.size(), s->in_base, s->ev_pos.size(), s->ev_done, s->items.size(), s->t,
                 s->res_item, s->res_S, s->res_pos, s->part_out, s->body_at, s->body.size(), s->out_pos, s->out.size());
}

static int deflate_body(z_streamp strm, int flush) {
    if (!strm || !strm->state || strm->state->inflating || flush < 0 || flush > Z_BLOCK) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (!strm->next_out || (strm->avail_in && !strm->next_in) || (s->finished && flush != Z_FINISH))
        return Z_STREAM_ERROR;
    if (s->job_closed && flush != Z_FINISH) {
        // zlib.h: after Z_FINISH, deflate() is called with Z_FINISH until Z_STREAM_END
        strm->msg = const_cast<char *>("deflate: Z_FINISH is pending, call with Z_FINISH until Z_STREAM_END");
        return Z_STREAM_ERROR;
    }
    if (strm->avail_out == 0) return Z_BUF_ERROR;
    const int old_flush = s->last_flush;
    s->last_flush = flush;
    if (s->out_pos < s->out.size()) {                           // deflate.c:983-1005
        drain(strm, s);
        if (strm->avail_out == 0) {
            s->last_flush = -1;
            return Z_OK;
        }
    } else if (strm->avail_in == 0 && flush_rank(flush) <= flush_rank(old_flush) && flush != Z_FINISH) {
        return Z_BUF_ERROR;
    }
    if (s->finished && strm->avail_in) return Z_BUF_ERROR;
    if (s->finished) {                                          // FINISH_STATE
        if (s->trailer_due) {
            s->trailer_due = false;
            queue_trailer(strm, s);
            drain(strm, s);
            return s->out_pos == s->out.size() ? Z_STREAM_END : Z_OK;
        }
        return Z_STREAM_END;
    }
    const size_t C = s->in_base + s->in.size();                // part position of the input copied so far
    size_t P = s->rd + strm->avail_in;                         // the input this call offers ends here
    // 32-bit kernel positions (level 0 cuts its own jobs: deflate_stored_call)
    if (s->level != 0 && P > C && (uint64_t)(P - s->in_base) >= kMaxBuffer) return Z_MEM_ERROR;

    // the first call asks for Z_FINISH with everything and has room for any
    // result (deflateBound): one batch job straight into next_out (ADVICE r2:
    // with less room the timeline below pauses like zlib, without a job whose
    // result might not fit and would be thrown away)
    if (flush == Z_FINISH && !s->header_done && !s->flushed && C == 0 && s->level != 0 &&
        strm->avail_out >= deflateBound(strm, strm->avail_in)) {
        size_t cap = strm->avail_out;
        const uint8_t *sp = strm->next_in;
        uint8_t *dp = strm->next_out;
        size_t sl = strm->avail_in;
        int st = 0;
        int rc;
        {
            Lease L;
            rc = L.rc;
            uint8_t wind = 0;
            if (!rc) rc = compress_host_locked(*L.c, &sp, &sl, &dp, &cap, &st, 1, s->level, s->wrap, s->strategy,
                                               nullptr, s->wbits, s->mem_level, s->tuned ? &s->tune : nullptr,
                                               &wind);
            s->bi_used = wind;
        }
        if (rc || st) return rc == ZGPU_ENODEV ? Z_MEM_ERROR : (rc ? rc : st);
        {
            // the window as the reference leaves it, for deflateGetDictionary: all
            // input read (E = n) and the window offset of the final fill_window,
            // which with all input present depends on n alone: the k-th slide
            // happens once strstart - S >= w_size + MAX_DIST (deflate.c:277)
            const uint64_t w = uint64_t(1) << s->wbits, maxd = w - kMinLookahead;
            uint64_t S = 0;
            while (S + w + maxd <= sl) S += w;
            const size_t keep = (size_t)std::min<uint64_t>(sl, w);
            s->in.assign(sp + (sl - keep), sp + sl);
            s->in_base = sl - keep;
            s->rd = s->rd_seen = sl;
            s->res_S = S;
            strm->next_out += cap;
            strm->avail_out -= (uInt)cap;
            strm->total_out += cap;
            strm->adler = s->wrap == 2 ? ck_crc32(0, sp, sl) : (s->wrap == 1 ? ck_adler32(1, sp, sl) : strm->adler);
            strm->next_in += sl;
            strm->total_in += sl;
            strm->avail_in = 0;
            s->header_done = true;
            s->finished = 1;
            return Z_STREAM_END;
        }
    }
    bool force_skip = false;
    const bool slow_fn = s->level >= 4 && s->strategy != Z_HUFFMAN_ONLY && s->strategy != Z_RLE;
    if (!s->header_done) {                                      // deflate.c:1002-1073
        const size_t before = s->out.size();
        queue_header(s);
        // a first call whose output space is exactly the header (below) that is not modelled is refused
        // here, before any output
        if (s->out_pos == before && strm->avail_out == s->out.size() - before && s->level != 0 && slow_fn &&
            P - s->rd >= 2) {
            const char *why = nullptr;
            // the first fill_window's read: window_size - strstart
            const size_t first = std::min<size_t>(P - s->rd, (size_t(2) << s->wbits) - s->dict_len);
            const size_t sym_limit = ((size_t)1 << (s->mem_level + 6)) - 1;
            if (s->dict_len > 0 && P - s->rd >= 3 && (flush != Z_NO_FLUSH || first >= 3 * sym_limit)) {
                // With a dictionary the first decision may find a match (history), and the stop at the
                // first lazy literal moves with the parse.  Under Z_NO_FLUSH that does not matter: the
                // call stops at that literal or at need_more, whichever comes first, and the loop goes on
                // from there in the next call with the same state -- the model's stop at need_more -- as
                // long as no block fills first (less than 3 bytes a symbol for a whole symbol buffer).
                // A flush call whose input the dictionary covers to its end would act on its flush
                // instead; without a match at the first decision (the input's first three bytes nowhere
                // in the dictionary) the literal comes at the second decision, as with no history.
                const uint8_t *d0 = s->in.data() + (s->rd - s->dict_len - s->in_base);
                const uint8_t *x = strm->next_in;
                for (size_t k = 0; k + 3 <= s->dict_len && !why; k++)
                    if (d0[k] == x[0] && d0[k + 1] == x[1] && d0[k + 2] == x[2])
                        why = "deflate: a first flush call whose output space is exactly a preset dictionary's "
                              "header, with the input's first string in the dictionary, is not modelled";
            }
            if (why) {
                s->out.resize(before);
                s->header_done = false;
                strm->msg = const_cast<char *>(why);
                return Z_STREAM_ERROR;
            }
        }
        drain(strm, s);
        if (s->out_pos < s->out.size()) {
            s->last_flush = -1;
            return Z_OK;
        }
        // The header took the last byte of output space, so the compress
        // function runs with avail_out == 0 (a call that starts with none gets
        // Z_BUF_ERROR, and pending output that fills it returns before; only the
        // header's call gets here).  deflate_slow stops at its first lazy literal
        // (need_more, at strstart 2 with no history): the call's flush never
        // happens, and fill_window has read at most window_size bytes.  With one
        // byte, and for deflate_fast / _huff / _rle, the input's end is reached:
        // FLUSH_BLOCK cuts the block and returns need_more before the flush's
        // marker.  Without input the flush goes ahead (its marker waits).
        const size_t avail = P - s->rd;
        if (strm->avail_out == 0 && s->level != 0) {
            // whatever the compress function returns then (need_more, or a marker
            // left pending), deflate() leaves with last_flush = -1: the next call
            // with no input is no Z_BUF_ERROR
            if (avail > 0 || flush != Z_NO_FLUSH) s->last_flush = -1;
            if (avail > 0 && slow_fn && avail >= 2) {
                // fill_window's first read: window_size - strstart (a dictionary's bytes stand before it)
                P = std::min<size_t>(P, s->rd + (size_t(2) << s->wbits) - s->dict_len);
                flush = Z_NO_FLUSH;
                force_skip = true;
            } else if (avail > 0 && flush != Z_NO_FLUSH && flush != Z_FINISH) {
                flush = Z_BLOCK;
            }
        }
    }
    if (s->level == 0) return deflate_stored_call(strm, s, flush);
    s->flushed = true;
    if (P > C) {                                                // copy what is new
        s->in.insert(s->in.end(), strm->next_in + (C - s->rd), strm->next_in + (P - s->rd));
        if (!s->hr.empty() && s->hr.back().b == ~0ull && !s->hr.back().first_end && P > s->hr.back().a)
            s->hr.back().first_end = P;                              // an open huff/rle stretch's first call
    } else if (P < C) {                                         // offered less than before: drop the rest
        s->in.resize(P - s->in_base);
        s->stale = true;
    }

    // the call's event
    uint32_t own = ~0u;
    if (s->ev_done < s->ev_type.size()) {                       // the last call did not get to its event
        const size_t le = s->ev_type.size() - 1;
        if (s->ev_type[le] == 0 && P != s->ev_pos[le] && le >= 1 && s->ev_type[le - 1] == kEvPrime &&
            s->ev_pos[le - 1] == s->ev_pos[le] && s->ev_done == le) {
            // the stop deflatePrime left due behind its bits (a pause before them stands for the block the
            // call stopped after): more input, and the reference reads on from there (deflatePrime)
            s->ev_pos.pop_back();
            s->ev_type.pop_back();
            s->ev_aux.pop_back();
            s->ev_done = s->ev_type.size();
            s->stale = true;
        } else if (s->ev_type[le] == 0) {                       // a stop it paused before
            if (P != s->ev_pos[le]) {
                // more input: the reference goes on from the paused block
                // reading up to the new end, the stop never comes
                if (s->t == 0 || s->items[s->t - 1].kind != kItBlock) return Z_STREAM_ERROR;   // not paused
                s->ev_type[le] = kEvPause;
                s->ev_aux[le] = s->items[s->t - 1].in_end;
                s->ev_done = le + 1;
                drop_pause_behind_resume(s, le);
                s->stale = true;
            } else if (flush == Z_NO_FLUSH) {
                own = (uint32_t)le;
            }
        } else {                                                // a flush whose marker is still due
            const bool at_marker = s->t < s->items.size() && s->items[s->t].kind == kItMarker &&
                                   s->items[s->t].ev == (uint32_t)le;
            if (P == s->ev_pos[le] && flush != Z_NO_FLUSH && flush != Z_FINISH) {
                // the repeated flush call: its own kind of marker (deflate.c:1211-1233)
                s->ev_type[le] = (uint32_t)flush;
                own = (uint32_t)le;
            } else if (at_marker) {
                s->ev_type[le] = Z_BLOCK;                       // the cut stays, no marker bits
                s->ev_done = le + 1;
            } else if (P != s->ev_pos[le] || flush == Z_NO_FLUSH) {
                // more input, or no flush: the reference goes on from the
                // paused block reading up to the new end, no marker (zlib.h asks
                // for the same flush until it completes; k_match keeps no clamp)
                if (s->t == 0 || s->items[s->t - 1].kind != kItBlock) return Z_STREAM_ERROR;   // not paused
                s->ev_type[le] = kEvPause;
                s->ev_aux[le] = s->items[s->t - 1].in_end;
                s->ev_done = le + 1;
                drop_pause_behind_resume(s, le);
            } else {                                            // Z_FINISH's drain takes over
                s->ev_pos.pop_back();
                s->ev_type.pop_back();
                s->ev_aux.pop_back();
            }
            s->stale = true;
        }
    }
    if (own == ~0u && flush != Z_FINISH) {
        const size_t last = s->ev_pos.empty() ? s->res_pos : (size_t)s->ev_pos.back();   // a pause's: its call's end
        if (flush != Z_NO_FLUSH || P > last) {
            s->ev_pos.push_back(P);
            s->ev_type.push_back((uint32_t)flush);
            s->ev_aux.push_back(0);
            own = (uint32_t)(s->ev_pos.size() - 1);
            s->stale = true;
        }
    }
    int rc = Z_OK;
    bool full = false;
    stream_trace("event", strm, s, flush);
    if (own != ~0u || flush == Z_FINISH) {
        // a Z_NO_FLUSH call that cannot complete a block before its stop (a
        // block holds lit_bufsize - 1 symbols, each covering >= 1 input byte
        // below P) hands out nothing: no job
        bool skip = false;
        if (flush == Z_NO_FLUSH && s->t == s->items.size() && !s->job_closed && !s->prime_due) {
            size_t x0 = s->res_pos;
            for (size_t k = s->t; k-- > 0;)
                if (s->items[k].kind != kItStop) { x0 = (size_t)s->items[k].in_end; break; }
            const size_t sym_limit = ((size_t)1 << (s->mem_level + 6)) - 1;
            skip = force_skip || P < x0 + sym_limit;
        }
        if (skip) {
            s->rd = P;
            s->ev_done = own + 1;
            s->tentative = false;
        } else {
            if (s->stale || (flush == Z_FINISH && !s->job_closed)) {
                if (int e = deflate_part(s, flush == Z_FINISH)) return e;
            }
            stream_trace("job", strm, s, flush);
            rc = run_items(strm, s, own, &full);
        }
    }
    stream_trace("ran", strm, s, flush);
    sync_input(strm, s);
    if (!s->finished) {
        advance_check(s, s->rd);
        if (s->wrap) strm->adler = s->check;
    }
    if (full) {
        close_part(s);
    } else if (!s->finished) {
        choose_resume(s);
    }
    return rc;
}

int deflateReset(z_streamp strm) {                              // deflate.c:560-620
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    const int level = s->level, wrap = s->wrap, strategy = s->strategy, wbits = s->wbits, mem = s->mem_level;
    const gz_header *gzhead = s->gzhead;                       // deflateResetKeep keeps it
    *s = internal_state(s->al);
    s->gzhead = gzhead;
    s->level = level;
    s->wrap = wrap;
    s->strategy = strategy;
    s->wbits = wbits;
    s->mem_level = mem;
    s->out_pos = 0;
    s->finished = 0;
    s->check = wrap == 2 ? 0 : 1;
    strm->total_in = strm->total_out = 0;
    strm->msg = nullptr;
    strm->data_type = Z_UNKNOWN;
    strm->adler = wrap == 2 ? 0 : 1;
    return Z_OK;
}

int deflateCopy(z_streamp dest, z_streamp source) {             // deflate.c:1270-1311
    if (!dest || !source || !source->state || source->state->inflating) return Z_STREAM_ERROR;
    *dest = *source;
    internal_state *s = new_state(dest, source->state);
    if (!s) return Z_MEM_ERROR;
    dest->state = s;
    return Z_OK;
}

// Bytes generated and not yet handed out; bits: those of a partial last byte
// after the last block or marker handed out (deflate.c:739-747).
// deflateUsed (deflate.c:723-728): bi_used, the bits of the last output byte
// the most recent bi_windup completed (1..8; trees.c winds up after a stored
// block's header and after the final block), 0 before any.  Taken from the
// encoder's records (k_encode / k_enc_scan report it).
int deflateUsed(z_streamp strm, int *bits) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    if (bits) *bits = strm->state->bi_used;
    return Z_OK;
}

// deflateGetDictionary (deflate.c:616-633): the window's last
// min(strstart + lookahead, w_size) bytes -- the input fill_window has read
// (s->rd) back to the window offset S where the reference stands: the last
// record handed out (a stop, block or marker), or the resume point.  Level 0:
// deflate_stored's window.  After a Z_FULL_FLUSH the part starts anew here (its
// window empty), so bytes from before the flush are not returned.
int deflateGetDictionary(z_streamp strm, Bytef *dictionary, uInt *dictLength) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    const internal_state *s = strm->state;
    const uint64_t wsize = uint64_t(1) << s->wbits;
    const uint8_t *src = nullptr;
    size_t len = 0;
    if (s->level == 0) {
        len = (size_t)std::min<uint64_t>(std::min<uint64_t>((uint64_t)s->st_strstart, s->l0_hist.size()), wsize);
        src = s->l0_hist.data() + (s->l0_hist.size() - len);
    } else {
        const uint64_t S = s->t > 0 ? s->items[s->t - 1].S : s->res_S;
        const uint64_t E = std::min<uint64_t>(s->rd, s->in_base + s->in.size());
        const uint64_t lo = std::max<uint64_t>(S, s->in_base);
        len = E > lo ? (size_t)std::min<uint64_t>(E - lo, wsize) : 0;
        src = s->in.data() + (E - len - s->in_base);
    }
    if (dictionary && len) std::memcpy(dictionary, src, len);
    if (dictLength) *dictLength = (uInt)len;
    return Z_OK;
}

int deflatePending(z_streamp strm, unsigned *pending, int *bits) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (pending) *pending = (unsigned)(s->out.size() - s->out_pos);
    if (bits) {
        uint64_t b = s->level == 0 ? s->res_bits : s->proc_bits;
        if (s->prime_due && s->level != 0 && !s->ev_type.empty()) {
            // deflatePrime's bits no job has written yet are in bi_buf already (deflate.c:745-755)
            size_t k = s->ev_type.size() - 1;
            if (s->ev_type[k] == 0 && k > 0 && s->ev_type[k - 1] == kEvPrime) k--;   // its call's stop, due again
            for (; s->ev_type[k] == kEvPrime; k--) {
                b += s->ev_aux[k] >> 16;
                if (k == 0) break;
            }
        }
        *bits = s->finished ? 0 : (int)(b & 7);
    }
    return Z_OK;
}

namespace {
int unsupported(z_streamp strm, const char *why) {
    strm->msg = const_cast<char *>(why);
    return Z_STREAM_ERROR;
}
int deflate_fn(int level) { return level == 0 ? 0 : level <= 3 ? 1 : 2; }   // stored, fast, slow
// the function deflate() runs (deflate.c:1190-1193): stored, fast, slow, huff 3, rle 4
int fn_of(int level, int strategy) {
    return level == 0 ? 0 : strategy == Z_HUFFMAN_ONLY ? 3 : strategy == Z_RLE ? 4 : deflate_fn(level);
}
}  // namespace

// deflateResetKeep (deflate.c:635-671): deflateReset without lm_init, so the
// next stream keeps the window, the hash chains and strstart of this one and
// may refer back into it.  Where that state is the initial one (nothing
// compressed or preset since deflateInit / deflateReset) it is exactly
// deflateReset.  After a stream that deflate_slow (levels 4-9, not
// Z_HUFFMAN_ONLY / Z_RLE) ran from its part start (deflateInit, deflateReset or
// its last Z_FULL_FLUSH) to a point with nothing left in the lookahead -- the
// end of Z_FINISH, or a flush call that took all its input -- the carried
// state is a preset dictionary in all but its bookkeeping:
//  - deflate_slow hashed every string of the part but the last two, which wait
//    as s->insert (deflate.c:1941-2027, :2030-2032), as deflateSetDictionary
//    leaves them (deflate.c:593-605);
//  - prev_length = match_length = MIN_MATCH-1 and match_available = 0 there
//    (the flush tail, deflate.c:2030-2040), as after deflateSetDictionary;
//  - the window holds the part's bytes from the window offset on, strstart =
//    block_start = their count P (< w_size + MAX_DIST: fill_window slides at
//    the loop top that ended the parse), so the next stream's part is those P
//    bytes then its input, in window coordinates, and its slides fall where
//    the reference's do;
//  - strm->adler restarts (1, or 0 for gzip) and covers only the new input; a
//    zlib header carries FDICT with that start value as DICTID, since
//    deflate.c:1030-1036 tests strstart != 0.
// Other carried states (deflate_fast's selective hashing, deflate_stored's
// window, a huffman-only / RLE stretch, input still in the lookahead) are not
// modelled (Z_STREAM_ERROR with strm->msg, never a different stream).
int deflateResetKeep(z_streamp strm) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    const bool fresh = s->in_base + s->in.size() == 0 && s->rd == 0 && !s->flushed && !s->dict_set &&
                       s->l0_hist.empty() && s->st_strstart == 0 && strm->total_in == 0;
    if (fresh) return deflateReset(strm);
    const char *why = "deflateResetKeep: a window carried into the next stream is modelled after deflate_slow "
                      "(levels 4-9) ran the whole part to a point with no input pending only";
    if (s->level < 4 || fn_of(s->level, s->strategy) != 2 || s->fn_mixed || !s->hr.empty() || s->level == 0 ||
        (!s->finished && pending_input(s)) || s->tentative)
        return unsupported(strm, why);
    // the window: the part's bytes from the window offset S to the end E.  The parse ended at a loop top
    // whose fill_window slid once more if strstart >= w_size + MAX_DIST (deflate.c:1535-1545), and every
    // slide found strstart at least that, so strstart = E below w_size + MAX_DIST, else the one value
    // in [MAX_DIST, w_size + MAX_DIST) that E reaches by whole slides: a function of E alone
    const uint64_t W = uint64_t(1) << s->wbits, maxd = W - kMinLookahead;
    const uint64_t E = std::min<uint64_t>(s->rd, s->in_base + s->in.size());
    const uint64_t S = E - (E < W + maxd ? E : maxd + (E - maxd) % W);
    // a one-call stream keeps its last w_size bytes: the older part of the window lies beyond MAX_DIST of
    // every later position (no candidate, no byte compared; a chain walk stops at the first link below the
    // limit, whatever string it is), so it only has to hold its place
    const uint64_t lo = std::max<uint64_t>(S, s->in_base);
    if (E - lo < std::min<uint64_t>(E - S, W)) return unsupported(strm, why);
    try {
        zvec<uint8_t> win(s->al);
        win.resize((size_t)(lo - S), 0);
        win.insert(win.end(), s->in.begin() + (std::ptrdiff_t)(lo - s->in_base),
                   s->in.begin() + (std::ptrdiff_t)(E - s->in_base));
        const size_t P = win.size();
        const int rc = deflateReset(strm);
        if (rc != Z_OK || P == 0) return rc;
        s = strm->state;
        s->in.assign(win.begin(), win.end());
        s->in_base = s->res_S = 0;
        s->dict_len = P;
        s->carried = true;
        s->res_pos = s->rd = s->rd_seen = s->flush_done = s->ck_pos = P;
        s->res_E = P;
        s->res_cut = 0;                                 // the last two strings wait as s->insert
        s->zl_p = s->zl_m = kMinMatch - 1;
        s->zl_pos = ~0ull;
        if (s->wrap == 1) {                             // strstart != 0: FDICT, DICTID = adler32 start value
            s->dict_set = true;
            s->dict_id = (uint32_t)strm->adler;
        }
        s->stale = true;
        s->flushed = true;                              // the part path (bit and parse offsets)
        return Z_OK;
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}

// deflateSetDictionary (deflate.c:550-613).  Accepted on a zlib stream
// before its first deflate() call and on a raw stream whenever the window holds
// no unprocessed input (lookahead == 0: before any data, after a flush, and at
// level 0, which keeps no lookahead).  The dictionary (its last w_size bytes; a
// raw stream's longer dictionary replaces the history, strings and all) goes
// into the window as if it were input that is never sent: every string of it is
// hashed but the last two, which wait as s->insert, and block_start moves past
// it (so a level-0 stream's unsent window bytes are dropped, as the reference's
// are).  Here the part's input gets the bytes and the resume point moves to
// their end; at level 0 deflate_stored's window offsets move as fill_window
// moves them.  A zlib stream's header then carries FDICT and the DICTID.
int deflateSetDictionary(z_streamp strm, const Bytef *dictionary, uInt dictLength) {
    if (!strm || !strm->state || strm->state->inflating || !dictionary) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (s->wrap == 2 || (s->wrap == 1 && s->last_flush != -2)) return Z_STREAM_ERROR;
    if (s->level != 0 && pending_input(s)) return Z_STREAM_ERROR;        // s->lookahead != 0
    if (s->finished) return unsupported(strm, "deflateSetDictionary: the stream has ended");
    if (s->carried && dictLength > 0)
        return unsupported(strm, "deflateSetDictionary: after deflateResetKeep carried a window, not modelled");
    try {
        if (s->wrap == 1) strm->adler = ck_adler32(strm->adler, dictionary, dictLength);
        const uint64_t wsize = uint64_t(1) << s->wbits;
        bool reset = false;
        if (dictLength >= wsize) {                      // the tail replaces the history
            reset = s->wrap == 0;                       // a zlib stream's window is empty anyway
            dictionary += dictLength - wsize;
            dictLength = (uInt)wsize;
        }
        s->zl_p = s->zl_m = kMinMatch - 1;               // match_length = prev_length = MIN_MATCH-1
        s->zl_pos = ~0ull;
        if (s->wrap == 1 && dictLength) {               // strstart != 0: FDICT + DICTID (deflate.c:1027-1036)
            s->dict_set = true;
            s->dict_id = (uint32_t)strm->adler;
        }
        if (s->level == 0) {
            // deflate_stored's window: fill_window's reads and slides as the
            // reference's deflateSetDictionary drives them (deflate.c:582-605)
            int64_t ss = reset ? 0 : s->st_strstart, bs = reset ? 0 : s->st_block_start;
            const int64_t W = (int64_t)wsize, maxd = W - kMinLookahead;
            uint64_t look = 0, avail = dictLength;
            auto fill = [&] {
                do {
                    if (ss >= W + maxd) { ss -= W; bs -= W; }
                    const uint64_t more = (uint64_t)(2 * W - (int64_t)look - ss), take = std::min(avail, more);
                    avail -= take;
                    look += take;
                } while (look < (uint64_t)kMinLookahead && avail != 0);
            };
            fill();
            while (look >= (uint64_t)kMinMatch) {
                ss += (int64_t)look - (kMinMatch - 1);
                look = kMinMatch - 1;
                fill();
            }
            ss += (int64_t)look;
            s->st_strstart = s->st_block_start = ss;
            (void)bs;
            if (reset) s->l0_hist.clear();
            s->l0_hist.insert(s->l0_hist.end(), dictionary, dictionary + dictLength);
            if (s->l0_hist.size() > (uint64_t)ss)
                s->l0_hist.erase(s->l0_hist.begin(), s->l0_hist.end() - (std::ptrdiff_t)ss);
            s->l0_pos += dictLength;
            s->in.clear();                              // block_start = strstart: unsent bytes dropped
            return Z_OK;
        }
        if (dictLength == 0) return Z_OK;
        const size_t X = s->in_base + s->in.size();     // the part position everything is processed to
        if (reset) {                                    // CLEAR_HASH, strstart = block_start = 0
            s->in.clear();
            s->in_base = s->res_S = X;
        }
        s->in.insert(s->in.end(), dictionary, dictionary + dictLength);
        s->dict_len = dictLength;
        s->res_pos = s->rd = s->rd_seen = s->flush_done = s->ck_pos = X + dictLength;
        s->res_E = X + dictLength;
        s->res_cut = 0;                                 // the last two strings wait as s->insert
        s->res_ev = s->ev_pos.size();
        s->ev_done = s->ev_type.size();
        s->items.clear();
        s->t = 0;
        s->res_item = -1;
        s->stale = true;
        s->flushed = true;                              // the part path (bit and parse offsets)
        return Z_OK;
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}

// The decision point the parse stands at between two deflate() calls (part
// position): after a call that stopped on a full output buffer, the end of the
// last block it handed out (the reference's strstart there); after need_more,
// the first point with less than MIN_LOOKAHEAD of the input read ahead of it
// (deflate_slow / deflate_fast decide no position closer to the end of the
// input without a flush, deflate.c:1841-1844, :1941-1944), or the last flush.
size_t parse_point(const internal_state *s) {
    if (s->ev_done < s->ev_type.size() && s->t > 0 && s->items[s->t - 1].kind == kItBlock)
        return (size_t)s->items[s->t - 1].in_end;
    const size_t x = s->rd > (size_t)(kMinLookahead - 1) ? s->rd - (kMinLookahead - 1) : 0;
    return std::max(x, s->flush_done);
}

// A configuration row changed with input pending (deflate.c:760-820 rewrite
// max_lazy_match, good_match, nice_match, max_chain_length in the state): the
// decisions from the point the parse stands at on read the new row.  A later
// job carries it as a change at that part position (DeflateJob::cfg_pos).
// Z_HUFFMAN_ONLY / Z_RLE read no row.
void cfg_change(internal_state *s, const LevelCfg &before) {
    if (!pending_input(s) || s->level == 0 || s->strategy == Z_HUFFMAN_ONLY || s->strategy == Z_RLE) return;
    const LevelCfg now = s->tuned ? s->tune : kLevelCfg[s->level];
    const size_t x = parse_point(s);
    if (s->cfg_pos.empty()) s->cfg0 = before;
    if (!s->cfg_pos.empty() && s->cfg_pos.back() >= x) {   // a second change at the same point
        s->cfg_row.back() = now;
        return;
    }
    s->cfg_pos.push_back(x);
    s->cfg_row.push_back(now);
}

// deflateTune (deflate.c:805-820): good_length, max_lazy, nice_length,
// max_chain for the decisions from here on (unsigned as deflate_state holds
// them; a chain of 0 never runs out in longest_match's unsigned count).
int deflateTune(z_streamp strm, int good_length, int max_lazy, int nice_length, int max_chain) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    try {
        const LevelCfg before = s->tuned ? s->tune : kLevelCfg[s->level];
        s->tune = LevelCfg{(uint32_t)good_length, (uint32_t)max_lazy,
                           nice_length < 0 ? 0xffffffffu : (uint32_t)nice_length,
                           max_chain == 0 ? 0xffffffffu : (uint32_t)max_chain};
        s->tuned = true;
        cfg_change(s, before);
        return Z_OK;
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}

// Level 0 <-> a searching level after deflateParams' Z_BLOCK flush (everything
// given so far is out).  deflate_stored keeps the window (its last strstart
// bytes) and s->insert (deflate.c:1733-1760); the function after it hashes
// those strings in fill_window (deflate.c:318-335) and searches the window, so
// the part goes on with the window as its history.  The other way, deflate_stored
// starts with strstart = block_start at the window position of the flush.
void enter_stored(internal_state *s) {
    const size_t X = s->in_base + s->in.size();                 // == s->rd after the flush
    s->st_strstart = s->st_block_start = (int64_t)(X - s->res_S);
    s->l0_hist.assign(s->in.begin() + (std::ptrdiff_t)(s->res_S - s->in_base), s->in.end());
    s->l0_pos = X;
    s->in.clear();                                              // the window's unsent bytes: none
}

void leave_stored(internal_state *s) {
    const size_t X = (size_t)s->l0_pos, S = X - s->l0_hist.size();
    s->in.assign(s->l0_hist.begin(), s->l0_hist.end());
    s->in_base = s->res_S = S;
    s->res_pos = s->rd = s->rd_seen = s->flush_done = s->ck_pos = X;
    s->res_E = X;
    s->res_cut = 0;                                             // s->insert strings wait for the next fill
    s->res_ev = 0;
    s->ev_pos.clear();
    s->ev_type.clear();
    s->ev_aux.clear();
    s->evb.clear();
    s->job_ev = 0;
    s->ev_done = 0;
    s->items.clear();
    s->t = 0;
    s->res_item = -1;
    s->stale = true;
    s->tentative = false;
    s->job_closed = false;
    s->proc_bits = s->res_bits;
    s->body.clear();
    s->body_at = 0;
    s->cfg_pos.clear();
    s->cfg_row.clear();
    s->zl_pos = X;                                              // deflate_stored kept prev/match_length
}

// deflateParams (deflate.c:760-803): flushes with Z_BLOCK when the level's
// function or the strategy changes and deflate() has run, then switches; a
// level change within the same function takes effect at the next decision.
int deflateParams(z_streamp strm, int level, int strategy) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (level == Z_DEFAULT_COMPRESSION) level = 6;
    if (level < 0 || level > 9 || strategy < 0 || strategy > Z_FIXED) return Z_STREAM_ERROR;
    const bool started = s->last_flush != -2;
    // deflate_slow <-> deflate_huff / deflate_rle after data: the stretch the
    // latter parse is left out of the chains (internal_state::hr)
    const int of = fn_of(s->level, s->strategy), nf = fn_of(level, strategy);
    // deflate_stored after a preset dictionary or a carried window (the bytes wait in the part's input as
    // history, where deflate_stored_call would take them for data) is not modelled
    if (!started && level == 0 && s->level != 0 && s->dict_len > 0)
        return unsupported(strm, "deflateParams: level 0 after a preset dictionary or a carried window is not "
                                 "modelled");
    // deflate_fast's longest_match starts from prev_length, which deflate_slow left at 0 when its last
    // symbol was a match (deflate.c:2008-2015): not known here for a carried window
    if (!started && s->carried && nf == 1 && of != 1)
        return unsupported(strm, "deflateParams: a deflate_fast level after deflateResetKeep carried a window is "
                                 "not modelled");
    const bool enter_hr = started && !s->finished && of < 3 && nf >= 3 && level != 0 && s->level != 0;
    const bool leave_hr = started && !s->finished && of >= 3 && nf < 3 && level != 0 && s->level != 0;
    if (enter_hr) {
        // from deflate_slow (k_links keys the stretch past every hash: memLevel
        // <= 8) or from deflate_fast (its chains resume from the snapshot at the
        // flush, the stretch left out of the strings inserted there)
        const uint64_t X = s->in_base + s->in.size();           // where the Z_BLOCK flush will stand
        if ((of != 2 && of != 1) || (of == 2 && s->mem_level > 8) || X < 2)
            return unsupported(strm, "deflateParams: a switch to Z_HUFFMAN_ONLY / Z_RLE after data is modelled "
                                     "from deflate_fast and deflate_slow levels (memLevel <= 8 for the latter) only");
    }
    if (leave_hr) {
        const bool ok = !s->hr_lost && !s->hr.empty() && s->hr.back().b == ~0ull && nf == s->hr.back().fn &&
                        (s->hr.back().first_end == 0 || s->hr.back().first_end >= s->hr.back().a + 2);
        if (!ok)
            return unsupported(strm, "deflateParams: a switch from Z_HUFFMAN_ONLY / Z_RLE after data is modelled "
                                     "back to the function the stretch began from (deflate_fast or deflate_slow "
                                     "levels), after a first call of at least 2 bytes");
    }
    if ((strategy != s->strategy || deflate_fn(level) != deflate_fn(s->level)) && started) {
        const int err = deflate(strm, Z_BLOCK);
        if (err == Z_STREAM_ERROR) return err;
        if (strm->avail_in || pending_input(s)) return Z_BUF_ERROR;
    }
    try {
        if (started && of != nf) s->fn_mixed = true;
        if (enter_hr) {
            internal_state::HrStretch h{};
            h.a = s->in_base + s->in.size();
            h.b = ~0ull;
            h.fn = of;
            s->hr.push_back(h);
            s->hr_lost = false;
        }
        if (leave_hr) {
            internal_state::HrStretch &h = s->hr.back();
            h.b = s->in_base + s->in.size();
            if (h.b == h.a) s->hr.pop_back();                    // no input in between: nothing skipped, ins_h fresh
        }
        if (started && !s->finished && (deflate_fn(level) != deflate_fn(s->level) || enter_hr || leave_hr)) {
            // the parse state the next function inherits (deflate_slow rewrites
            // prev_length at every decision, deflate_fast only match_length,
            // deflate_stored neither)
            if (s->level >= 4 && s->strategy != Z_HUFFMAN_ONLY && s->strategy != Z_RLE) s->zl_p = s->exit_p;
            if (s->level != 0) s->zl_m = s->exit_m;
            s->zl_pos = s->level != 0 ? s->res_pos : s->zl_pos;
        }
        if (started && !s->finished && (level == 0) != (s->level == 0)) {
            if (level == 0) enter_stored(s);
            else leave_stored(s);
        }
        if (s->level != level) {
            const LevelCfg before = s->tuned ? s->tune : kLevelCfg[s->level];
            s->level = level;
            s->tuned = false;                  // configuration_table's row again
            cfg_change(s, before);
        }
        s->strategy = strategy;
        return Z_OK;
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}

// deflatePrime (deflate.c): bits in front of what deflate() writes next.
// Whole bytes are queued at once (pending, ahead of a header not written
// yet), the rest starts the part's first byte.
int deflatePrime(z_streamp strm, int bits, int value) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (bits < 0 || bits > 16) return Z_BUF_ERROR;
    // deflate.c:741-744: no room ahead of the symbol buffer for more bits (the
    // pending output handed out so far reaches into it)
    const size_t lit_bufsize = size_t(1) << (s->mem_level + 6);
    if (s->out_pos < s->out.size() && s->out_pos + 2 > lit_bufsize) return Z_BUF_ERROR;
    if (!s->finished && pending_input(s)) {
        // With input pending the reference writes the bits into bi_buf at
        // once: after the blocks flushed so far, ahead of the block in
        // progress.  The parse stands at the last call's stop there; the bits
        // become an event at that stop (kEvPrime), which the next job's parse
        // turns into a marker record that k_encode writes.
        //
        // After a call that stopped on a full output buffer inside its input
        // (FLUSH_BLOCK's need_more, its stop still due) the reference stands
        // right after the block it flushed last: the bits go after that block
        // and ahead of the next.  The stop becomes the pause the next deflate()
        // would make of it (the block's end; the parse reads on from there),
        // the bits an event right after it, which the parse writes as the
        // pause passes, and the stop is due again behind them (round 6).
        const size_t le = s->ev_type.empty() ? 0 : s->ev_type.size() - 1;
        const bool due_stop = s->level != 0 && !s->ev_type.empty() && s->ev_type[le] == 0 && s->ev_done == le;
        const bool after_pause_prime = due_stop && le >= 1 && s->ev_type[le - 1] == kEvPrime &&
                                       s->ev_pos[le - 1] == s->ev_pos[le];
        const bool paused = due_stop && s->t > 0 && s->t <= s->items.size() && s->items[s->t - 1].kind == kItBlock;
        if (due_stop && (after_pause_prime || paused)) {
            if (bits == 0) return Z_OK;
            // The call left output pending with pending_out moved past pending_buf.  deflatePrime's
            // _tr_flush_bits puts whole bytes at pending_buf[pending] (put_byte indexes by the pending
            // count, deflate.h), inside the bytes still to go out, and the stream's last pending byte
            // becomes whatever the buffer held there: only bits that complete no byte keep the stream whole
            uint32_t held = (uint32_t)(s->proc_bits & 7);
            for (size_t k = le; k-- > 0 && s->ev_type[k] == kEvPrime && s->ev_pos[k] == s->ev_pos[le];)
                held += (uint32_t)(s->ev_aux[k] >> 16);
            if (held + (uint32_t)bits >= 8)
                return unsupported(strm, "deflatePrime: after a call that stopped on a full output buffer, bits "
                                         "that complete a byte (the reference writes it into its pending output at "
                                         "the pending count's offset) are not modelled");
            try {
                const uint32_t v = (uint32_t)value & ((1u << bits) - 1u);
                const uint64_t P0 = s->ev_pos[le];
                const uint64_t arg = (uint64_t)v | ((uint64_t)bits << 16);
                if (after_pause_prime) {                        // another deflatePrime there: in front of the stop
                    s->ev_pos.insert(s->ev_pos.begin() + (std::ptrdiff_t)le, P0);
                    s->ev_type.insert(s->ev_type.begin() + (std::ptrdiff_t)le, kEvPrime);
                    s->ev_aux.insert(s->ev_aux.begin() + (std::ptrdiff_t)le, arg);
                } else {
                    s->ev_type[le] = kEvPause;
                    s->ev_aux[le] = s->items[s->t - 1].in_end;
                    s->ev_pos.push_back(P0);
                    s->ev_type.push_back(kEvPrime);
                    s->ev_aux.push_back(arg);
                    s->ev_pos.push_back(P0);
                    s->ev_type.push_back(0);
                    s->ev_aux.push_back(0);
                    // a pause at the resume point's own block is behind it (drop_pause_behind_resume)
                    if (s->res_item >= 0 && s->res_pos >= s->ev_aux[le]) {
                        s->ev_pos.erase(s->ev_pos.begin() + (std::ptrdiff_t)le);
                        s->ev_type.erase(s->ev_type.begin() + (std::ptrdiff_t)le);
                        s->ev_aux.erase(s->ev_aux.begin() + (std::ptrdiff_t)le);
                        if (s->res_ev > le) s->res_ev = le;
                    }
                }
                s->ev_done = s->ev_type.size() - 1;             // the stop is due again
                s->stale = true;
                s->prime_due = true;
                return Z_OK;
            } catch (const std::bad_alloc &) {
                return Z_MEM_ERROR;
            }
        }
        if (s->level == 0 || s->ev_type.empty() || s->ev_done != s->ev_type.size() || s->tentative ||
            (s->ev_type.back() != 0 && s->ev_type.back() != kEvPrime))
            return unsupported(strm, "deflatePrime: input pending after a call that did not reach its end");
        if (bits == 0) return Z_OK;
        try {
            const uint32_t v = (uint32_t)value & ((1u << bits) - 1u);
            s->ev_pos.push_back(s->ev_pos.back());
            s->ev_type.push_back(kEvPrime);
            s->ev_aux.push_back((uint64_t)v | ((uint64_t)bits << 16));
            s->ev_done = s->ev_type.size();
            s->stale = true;
            s->prime_due = true;
            return Z_OK;
        } catch (const std::bad_alloc &) {
            return Z_MEM_ERROR;
        }
    }
    if (s->finished) return unsupported(strm, "deflatePrime: after Z_STREAM_END");
    // output still pending after a call that filled its buffer: a completed byte would go to
    // pending_buf[pending], inside that output (put_byte, as in the paused case above)
    if (s->out_pos < s->out.size() && (uint32_t)(s->res_bits & 7) + (uint32_t)bits >= 8)
        return unsupported(strm, "deflatePrime: with output pending, bits that complete a byte (the reference "
                                 "writes it into its pending output at the pending count's offset) are not "
                                 "modelled");
    try {
        uint32_t nb = (uint32_t)(s->res_bits & 7);
        uint64_t acc = (s->res_byte & ((1u << nb) - 1u)) | ((uint64_t)((uint32_t)value & ((1u << bits) - 1u)) << nb);
        nb += (uint32_t)bits;
        uint64_t whole = 0;
        while (nb >= 8) {
            s->out.push_back((uint8_t)acc);
            acc >>= 8;
            nb -= 8;
            whole++;
        }
        if (s->header_done) {              // part bytes
            s->part_out += whole;
            s->res_bits = ((s->res_bits >> 3) + whole) * 8 + nb;
        } else {                           // ahead of the header: the part starts at the partial byte
            s->res_bits = nb;
        }
        s->res_byte = (uint32_t)acc & 0xffu;
        s->proc_bits = s->res_bits;
        s->flushed = true;
        return Z_OK;
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}

// deflateSetHeader (deflate.c): the gzip header the first deflate() call writes
int deflateSetHeader(z_streamp strm, gz_headerp head) {
    if (!strm || !strm->state || strm->state->inflating || strm->state->wrap != 2) return Z_STREAM_ERROR;
    strm->state->gzhead = head;
    if (head) strm->state->flushed = true;   // the header is written on the host (queue_header)
    return Z_OK;
}

int deflateEnd(z_streamp strm) {
    if (!strm || !strm->state || strm->state->inflating) return Z_STREAM_ERROR;
    free_state(strm, strm->state);
    strm->state = nullptr;
    return Z_OK;
}

// deflate_state's strstart != 0 (deflateBound's DICTID allowance): a preset
// dictionary or a flush put positions behind the parse, or the parse has
// decided a position -- which a Z_NO_FLUSH call does once the lookahead it
// leaves (below MIN_LOOKAHEAD, at most MAX_MATCH for Z_RLE, 0 for
// Z_HUFFMAN_ONLY) is less than what it has read.  A Z_FULL_FLUSH resets it
// (deflate.c:1225-1229), as it resets the part.
static bool strstart_nonzero(const z_stream *strm, const internal_state *s) {
    if (s->level == 0) return s->st_strstart != 0;
    if (s->finished)                       // the part since the last Z_FULL_FLUSH, or the one-call stream
        return s->flushed ? s->in_base + s->in.size() > 0 : strm->total_in > 0;
    if (s->flush_done > 0) return true;
    const size_t need = s->strategy == Z_HUFFMAN_ONLY ? 1 : s->strategy == Z_RLE ? kMaxMatch + 1 : kMinLookahead;
    return s->rd >= need;
}

uLong deflateBound(z_streamp strm, uLong sourceLen) {          // deflate.c:842-905
    const uLong fixedlen = sourceLen + (sourceLen >> 3) + (sourceLen >> 8) + (sourceLen >> 9) + 4;
    const uLong storelen = sourceLen + (sourceLen >> 5) + (sourceLen >> 7) + (sourceLen >> 11) + 7;
    if (!strm || !strm->state || strm->state->inflating) return (fixedlen > storelen ? fixedlen : storelen) + 18;
    const internal_state *s = strm->state;
    // the wrapper's row also after Z_STREAM_END (the reference's bound does not
    // change once the trailer is written: tests/golden/zstream_golden.json)
    const int w = s->wrap;
    uLong wraplen = 6;
    if (w == 0) {
        wraplen = 0;
    } else if (w == 1) {
        wraplen = 6 + (strstart_nonzero(strm, s) ? 4 : 0);
    } else if (w == 2) {
        wraplen = 18;
        if (const gz_header *h = s->gzhead) {                      // the caller's header, read now
            if (h->extra) wraplen += 2 + h->extra_len;
            if (const Bytef *str = h->name) do wraplen++; while (*str++);
            if (const Bytef *str = h->comment) do wraplen++; while (*str++);
            if (h->hcrc) wraplen += 2;
        }
    }
    if (s->wbits != 15 || s->mem_level + 7 != 8 + 7)   // not the default parameters: a conservative bound
        return (s->wbits <= s->mem_level + 7 && s->level ? fixedlen : storelen) + wraplen;
    return sourceLen + (sourceLen >> 12) + (sourceLen >> 14) + (sourceLen >> 25) + 13 - 6 + wraplen;
}

// ------------------------------- inflate -------------------------------

static int uncompress2_body(Bytef *dest, uLongf *destLen, const Bytef *source, uLong *sourceLen) {
    if (!destLen || !sourceLen || (*sourceLen && !source) || (*destLen && !dest)) return Z_STREAM_ERROR;
    const uint8_t *s = source;
    uint8_t *d = dest;
    size_t sl = *sourceLen, cap = *destLen, used = 0;
    int st = 0;
    int rc = zgpu_uncompress_batch(&s, &sl, &d, &cap, &used, &st, 1, ZGPU_WRAP_ZLIB);
    if (rc == ZGPU_ENODEV) return Z_MEM_ERROR;
    if (rc) return rc;
    *destLen = cap;
    *sourceLen = used;
    return st;
}

int uncompress(Bytef *dest, uLongf *destLen, const Bytef *source, uLong sourceLen) {    // uncompr.c:82-85
    return uncompress2(dest, destLen, source, &sourceLen);
}

// z_stream inflate: gather input, decode on the GPU once the gathered input
// holds a whole stream, drain.
int inflateInit2_(z_streamp strm, int windowBits, const char *version, int stream_size) {
    if (!version || version[0] != ZGPU_ZLIB_VERSION[0] || stream_size != (int)sizeof(z_stream))
        return Z_VERSION_ERROR;                                       // inflate.c:203-206
    if (!strm) return Z_STREAM_ERROR;
    int wrap;                                                         // inflateReset2, inflate.c:161-185
    if (windowBits < 0) {
        if (windowBits < -15) return Z_STREAM_ERROR;
        wrap = 0;
        windowBits = -windowBits;
    } else {
        wrap = ((windowBits >> 4) + 5) & 3;                           // 1 zlib, 2 gzip, 3 either
        if (windowBits < 48) windowBits &= 15;
    }
    if (windowBits && (windowBits < 8 || windowBits > 15)) return Z_STREAM_ERROR;
    internal_state *s = new_state(strm);
    if (!s) return Z_MEM_ERROR;
    s->inflating = 1;
    s->wrap = wrap;
    s->wbits = windowBits;
    s->out_pos = 0;
    s->finished = 0;
    strm->msg = nullptr;
    strm->state = s;
    strm->total_in = strm->total_out = 0;
    strm->adler = wrap & 1;
    return Z_OK;
}

int inflateInit_(z_streamp strm, const char *version, int stream_size) {
    return inflateInit2_(strm, 15, version, stream_size);
}

int inflateReset(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    s->in.clear(); s->out.clear(); s->hist.clear();
    s->out_pos = 0; s->finished = 0; s->tried = 0; s->cap = 0; s->result = Z_OK;
    s->in_base = 0; s->imode = 0; s->igz = 0; s->res_bit = s->res_put = s->ideliv = 0; s->icheck = 0;
    s->need_dict = false; s->want_dict = 0;
    s->ihead = nullptr;                                                // inflateResetKeep: head = Z_NULL
    s->isyncing = false; s->isync_have = 0; s->isync = 0; s->idt = 0; s->itype = false; s->itail = false;
    s->iadj = 0;
    s->iwin.clear(); s->iwin_on = false;                               // wsize = whave = wnext = 0
    s->isyncpt = false; s->imark = -65536; s->icodes = 0; s->iprime_n = 0; s->iprime_v = 0;
    s->iadl_on = false; s->iadl = 0;
    s->cons = s->fin_used = 0; s->held_at = nullptr; s->ix.clear(); s->ix2.clear(); s->ix_all = false;
    s->bx.clear(); s->hx.clear(); s->out_at = 0; s->after_hdr = false;
    s->iheld = s->iheld_end = 0;
    strm->total_in = strm->total_out = 0;
    strm->msg = nullptr;
    if (s->wrap) strm->adler = s->wrap & 1;                           // inflateResetKeep: only when wrapped
    return Z_OK;
}

// the window size updatewindow allocates: 1 << wbits (inflateInit2_'s, or the
// zlib header's CINFO + 8 when that was 0, 15 for gzip)
static size_t inflate_wsize(const internal_state *s) {
    int wb = s->wbits;
    if (!wb) wb = s->igz || s->in.empty() || s->in_base ? 15 : (s->in[0] >> 4) + 8;
    return size_t(1) << wb;
}

// inflateResetKeep (inflate.c:105-128): inflateReset without forgetting the
// window.  A raw stream then decodes with it in front of its output, as it
// would after inflateSetDictionary; a zlib / gzip stream decodes from its header
// (a valid one never reaches back past its own start).
int inflateResetKeep(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    try {
        zvec<uint8_t> win(s->iwin);
        const bool on = s->iwin_on;
        inflateReset(strm);
        s->iwin.swap(win);
        s->iwin_on = on;
        if (s->wrap == 0 && !s->iwin.empty()) {
            s->hist.assign(s->iwin.begin(), s->iwin.end());
            s->res_bit = 0;
            s->res_put = s->ideliv = s->hist.size();
            s->icheck = 1;
            s->imode = 1;
        }
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
    return Z_OK;
}

// inflateReset2 (inflate.c:153-191): new windowBits (same rules as
// inflateInit2_), the window dropped when its size changes, then inflateReset
int inflateReset2(z_streamp strm, int windowBits) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    int wrap;
    if (windowBits < 0) {
        if (windowBits < -15) return Z_STREAM_ERROR;
        wrap = 0;
        windowBits = -windowBits;
    } else {
        wrap = ((windowBits >> 4) + 5) & 3;
        if (windowBits < 48) windowBits &= 15;
    }
    if (windowBits && (windowBits < 8 || windowBits > 15)) return Z_STREAM_ERROR;
    s->wrap = wrap;
    s->wbits = windowBits;
    // inflate.c:157's wrap = (windowBits >> 4) + 5 carries bit 4 (check the
    // trailer) again: an earlier inflateValidate(strm, 0) ends here
    s->ivalid = wrap != 0;
    return inflateReset(strm);
}

// inflateUndermine (inflate.c:1483-1496): the reference is built without
// INFLATE_ALLOW_INVALID_DISTANCE_TOOFAR_ARRR, so it refuses to subvert the
// distance check and answers Z_DATA_ERROR
int inflateUndermine(z_streamp strm, int subvert) {
    (void)subvert;
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    return Z_DATA_ERROR;
}

// inflateValidate (inflate.c:1498-1508): check != 0 verifies the trailer's
// Adler-32 / CRC-32 + ISIZE (the default); 0 reads them unchecked, and
// strm->adler keeps its start value as inflate.c then computes no check
int inflateValidate(z_streamp strm, int check) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    s->ivalid = check && s->wrap;
    return Z_OK;
}

// inflateGetDictionary (inflate.c:1278-1296): the window's bytes, oldest first
int inflateGetDictionary(z_streamp strm, Bytef *dictionary, uInt *dictLength) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (dictionary && !s->iwin.empty()) std::memcpy(dictionary, s->iwin.data(), s->iwin.size());
    if (dictLength) *dictLength = (uInt)s->iwin.size();
    return Z_OK;
}

// inflateSyncPoint (inflate.c:1431-1437): 1 when inflate stands in mode STORED
// with no bits held -- the input ran out right after a stored block's header
// byte (a Z_SYNC_FLUSH / Z_FULL_FLUSH point whose 00 00 ff ff is not here yet)
int inflateSyncPoint(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    const internal_state *s = strm->state;
    return !s->finished && s->out_pos == s->out.size() && s->isyncpt ? 1 : 0;
}

// inflateMark (inflate.c:1510-1519): where the input ran out, (back << 16) +
// (a stored block's bytes still to copy): back = -1 at a block boundary, in a
// header or a stored block, else the bits of the length / distance symbol
// already consumed (0 in mode LEN).  A call that stopped on a full output
// buffer (the reference then stands in mode LIT / MATCH / COPY mid-output) is
// not modelled: the value is the one at the end of the input decoded so far.
long inflateMark(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating) return -(1L << 16);
    const internal_state *s = strm->state;
    return s->finished ? -(1L << 16) : (long)s->imark;
}

// inflateCodesUsed (inflate.c:1521-1527): the code-table entries the last
// dynamic block's literal/length and distance tables took (inftrees.c
// inflate_table at lenbits 9 / distbits 6); 0 after a reset.  Reported by the
// decode (zgpu_inflate.hip codes_used).
unsigned long inflateCodesUsed(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating) return (unsigned long)-1;
    return strm->state->icodes;
}

// inflatePrime (inflate.c:223-239): bits inserted ahead of the input.  Taken
// on a raw stream before its first input (zran.c's pattern: inflateReset2(-15),
// inflatePrime, inflateSetDictionary, then the stream from a byte offset): the
// bits lead the decode as a virtual prefix that total_in does not count.  Bits
// primed in the middle of a stream or ahead of a zlib / gzip header are not
// modelled (Z_STREAM_ERROR with strm->msg).
int inflatePrime(z_streamp strm, int bits, int value) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (bits == 0) return Z_OK;
    const bool start = s->in.empty() && s->in_base == 0 && !s->finished && s->res_bit == 0 && strm->total_in == 0;
    if (bits < 0) {                                   // hold = bits = 0
        if (!start) return unsupported(strm, "inflatePrime: clearing the bit buffer mid-stream is not modelled");
        s->iprime_n = 0;
        s->iprime_v = 0;
        return Z_OK;
    }
    if (bits > 16 || s->iprime_n + (uint32_t)bits > 32) return Z_STREAM_ERROR;
    if (!start || s->wrap != 0) return unsupported(strm, "inflatePrime: raw streams before their first input only");
    s->iprime_v |= (uint64_t)((uint32_t)value & ((1u << bits) - 1u)) << s->iprime_n;
    s->iprime_n += (uint32_t)bits;
    return Z_OK;
}

namespace {
uint32_t stream_check(const internal_state *s, uint32_t init, const uint8_t *p, size_t n) {
    return s->igz ? ck_crc32(init, p, n) : ck_adler32(init, p, n);
}

// the symbol index and block boundaries of a decode whose output array starts
// at absolute output obase, hist_len bytes of window in front (InflateIndex,
// InflateTry::blk_*: the last boundary); `whole`: the decode ran to its own
// end (not cut at its output capacity).  Of the two earlier indexes the one
// that starts lower stays as ix2: after a Z_BLOCK stop the resume point (where
// later decodes start) can lie past the output handed out.
void keep_index(internal_state *s, InflateIndex &ix, const InflateTry &t, uint64_t obase, size_t hist_len,
                bool whole) {
    // the second index: the previous one, unless only the older one reaches
    // the output handed out so far
    auto covers = [&](const std::vector<uint64_t> &e, uint64_t eobase, uint64_t o0) {
        return !e.empty() && o0 <= s->ideliv && (uint32_t)e[e.size() - 2] + eobase > s->ideliv;
    };
    if (!s->ix.empty() && (covers(s->ix, s->ix_obase, s->ix_o0) || !covers(s->ix2, s->ix2_obase, s->ix2_o0))) {
        s->ix2.swap(s->ix);
        s->ix2_ibase = s->ix_ibase;
        s->ix2_obase = s->ix_obase;
        s->ix2_o0 = s->ix_o0;
    }
    s->ix.swap(ix.e);
    s->ix_ibase = s->in_base;
    s->ix_obase = obase;
    s->ix_o0 = obase + hist_len;
    s->ix_all = whole && 2ull * ix.ne <= s->ix.size();
    const uint64_t ib = 8ull * s->in_base;                        // the decode's in[0] is in_base (0 from the start)
    s->bx.clear();
    s->bx_last = ~0ull;
    auto add = [&](uint64_t b, uint64_t p, bool abs) {
        if (!abs) { b += ib; p += obase; }
        if (b && (s->bx.empty() || b > s->bx[s->bx.size() - 2])) {
            s->bx.push_back(b);
            s->bx.push_back(p);
        }
    };
    if (s->imode == 1) add(s->res_bit, s->res_put, true);           // where the decode started
    s->hx.clear();
    for (size_t k = 0; k + 1 < ix.b.size(); k += 2) {
        const uint64_t b = ix.b[k] & ~(3ull << 62);
        if ((ix.b[k] >> 62) & 1u) {                                  // a header's end (Z_TREES stops)
            s->hx.push_back((b + ib) | (ix.b[k] & (1ull << 63)));
            s->hx.push_back(ix.b[k + 1] + obase);
            continue;
        }
        add(b, ix.b[k + 1], false);
        if (ix.b[k] >> 63) s->bx_last = b + ib;
    }
    add(t.blk_bit, t.blk_put, false);
    if (t.stop == kIBlock && ((t.zstate >> 32) & 1u)) s->bx_last = t.blk_bit + ib;
}

// the resume point (res_bit, res_put, hist, icheck) moved to the last block
// boundary of the last decode at or before output xlim and input bit blim
// (where the reference stands), when that is past the current one.  The check
// and the window come from s->out, which keeps the output from the window
// before the resume point on; input before the boundary's byte is dropped.
void advance_resume(internal_state *s, uint64_t xlim, uint64_t blim, bool last_ok = false) {
    uint64_t bb = 0, bp = 0;
    for (size_t k = 0; k + 1 < s->bx.size(); k += 2)      // (the last block's end only for its trailer: itail)
        if (s->bx[k] <= blim && s->bx[k + 1] <= xlim && s->bx[k] > bb && (last_ok || s->bx[k] != s->bx_last)) {
            bb = s->bx[k];
            bp = s->bx[k + 1];
        }
    if (!bb || bb <= s->res_bit || bp < s->res_put) return;
    const uint64_t h0 = bp > 32768 ? bp - 32768 : 0;              // the window before the new point
    if (h0 < s->out_at || s->res_put < s->out_at || bp > s->out_at + s->out.size() ||
        (bb >> 3) < s->in_base || (bb >> 3) > s->in_base + s->in.size())
        return;
    if (s->imode == 0) {
        s->igz = (s->wrap & 2) && s->in.size() >= 2 && s->in[0] == 0x1f && s->in[1] == 0x8b;
        s->icheck = s->igz ? 0u : 1u;
    }
    const uint8_t *o = s->out.data();                              // o[x - out_at]: absolute output byte x
    if (s->wrap != 0)
        s->icheck = stream_check(s, s->icheck, o + (s->res_put - s->out_at), (size_t)(bp - s->res_put));
    s->hist.assign(o + (h0 - s->out_at), o + (bp - s->out_at));
    s->res_bit = bb;
    s->res_put = bp;
    s->imode = 1;
    s->itype = true;
    const uint64_t drop = (bb >> 3) - s->in_base;                 // input before the boundary's byte
    s->in.erase(s->in.begin(), s->in.begin() + (std::ptrdiff_t)drop);
    s->in_base += drop;
    if (h0 > s->out_at && h0 <= s->ideliv) {                      // output before the window is not needed again
        s->out.erase(s->out.begin(), s->out.begin() + (std::ptrdiff_t)(h0 - s->out_at));
        s->out_at = h0;
        s->out_pos = (size_t)(s->ideliv - s->out_at);
    }
}

// One decode attempt of the streaming inflate() over the input gathered so
// far: from the stream start until a block is complete, then from the last
// block boundary.  Sets s->out (bytes not handed out yet), s->finished and
// s->result; `took` input bytes of this call may be handed back past the end.
int inflate_attempt(z_streamp strm, internal_state *s, size_t took, bool block = false, bool trees = false) {
    const uint64_t in_end = s->in_base + s->in.size();
    if (s->cap == 0) s->cap = std::max<size_t>(4 * s->in.size(), 1 << 16);
    const bool is_check = s->wrap != 0;
    auto check_of = [&](uint32_t init, const uint8_t *p, size_t n) -> uint32_t {
        return s->igz ? ck_crc32(init, p, n) : ck_adler32(init, p, n);
    };
    if (s->itail) {
        // the last block is out (an inflate(Z_BLOCK) stopped after it): the
        // trailer, byte aligned after it (inflate.c TYPEDO .. LENGTH), read
        // once the block's output is all handed out
        if (s->out_pos < s->out.size()) return Z_OK;
        const uint64_t tpos = (s->res_bit + 7) >> 3;
        const uint64_t need = !s->wrap || s->isync == 2 ? 0 : s->igz ? 8 : 4;
        if (in_end < tpos + need) {
            s->tried = in_end;
            return Z_OK;
        }
        const uint8_t *tr = s->in.data() + (tpos - s->in_base);
        bool ok = true;
        if (!s->isync && s->ivalid && need == 4) {
            ok = ((uint32_t)tr[0] << 24 | (uint32_t)tr[1] << 16 | (uint32_t)tr[2] << 8 | tr[3]) == s->icheck;
            if (!ok) strm->msg = const_cast<char *>("incorrect data check");
        } else if (!s->isync && s->ivalid && need == 8) {
            const uint32_t c = tr[0] | (uint32_t)tr[1] << 8 | (uint32_t)tr[2] << 16 | (uint32_t)tr[3] << 24;
            const uint32_t z = tr[4] | (uint32_t)tr[5] << 8 | (uint32_t)tr[6] << 16 | (uint32_t)tr[7] << 24;
            ok = c == s->icheck && z == (uint32_t)s->res_put;
            if (!ok) strm->msg = const_cast<char *>(c != s->icheck ? "incorrect data check" : "incorrect length check");
        }
        s->finished = 1;
        s->itail = false;
        s->acct_done = true;
        if (ok) {
            const uint64_t used = tpos + need;
            const size_t back = (size_t)std::min<uint64_t>(in_end - used, took);
            strm->next_in -= back;
            strm->avail_in += (uInt)back;
            strm->total_in = used - s->iadj;
            if (s->wrap && !s->isync && s->ivalid) strm->adler = s->icheck;
            s->result = Z_STREAM_END;
        } else {
            s->result = Z_DATA_ERROR;
        }
        s->in.clear();
        return Z_OK;
    }
    for (;;) {
        const bool resume = s->imode == 1;
        // inflateValidate(strm, 0) on a zlib / gzip stream: the decode stops after
        // the header and goes on raw from there, so that the trailer is read on
        // the host, unchecked
        const bool hdr_stop = !s->ivalid && s->wrap && !resume && !block;
        const size_t hl = resume ? s->hist.size() : 0;
        // inflate(Z_BLOCK) stops after the header only in the call that reads
        // its last byte (inflate.c: mode TYPE is reached there); when an earlier
        // call already took the whole header, the decode is mid-block and this
        // call runs to the end of the first block
        bool hdr_done = false;
        if (block && !resume && s->wrap && s->in.size() >= took) {
            const size_t before = s->in.size() - took;          // input the earlier calls gave
            const uint8_t *h = s->in.data();
            size_t hlen = 0;                                    // 0: not complete in `before` bytes
            if (before >= 2 && (s->wrap & 2) && h[0] == 0x1f && h[1] == 0x8b) {
                if (before >= 10) {
                    const uint32_t fl = h[3];
                    size_t p = 10;
                    bool ok = true;
                    if (fl & 0x04) {
                        ok = before >= p + 2;
                        if (ok) p += 2 + (h[p] | ((size_t)h[p + 1] << 8));
                    }
                    for (uint32_t f = 0x08; ok && f <= 0x10; f <<= 1) {
                        if (!(fl & f)) continue;
                        while (p < before && h[p] != 0) p++;
                        ok = p < before;
                        p++;
                    }
                    if (ok && (fl & 0x02)) p += 2;
                    if (ok && p <= before) hlen = p;
                }
            } else if (before >= 2) {
                hlen = (h[1] & 0x20) ? 6 : 2;                   // FDICT: the DICTID too
                if (hlen > before) hlen = 0;
            }
            hdr_done = hlen != 0;
        }
        // inflate(Z_TREES) also stops after a block header (inflate.c STORED,
        // fixed TYPEDO, CODELENS: LEN_ / COPY_) that the reference has not
        // finished reading: one ending past where it stands
        const uint64_t pref = 8 * s->cons - s->iheld;            // the reference's bit position
        const uint64_t ib = resume ? 8ull * s->in_base : 0;
        const uint64_t trees_after = pref > ib ? pref - ib : 0;
        std::vector<uint8_t> o;
        InflateTry t{};
        InflateIndex ixo;
        int rc;
        {
            Lease L;
            rc = L.rc;
            // inflate(Z_BLOCK): stop after the header (zlib / gzip, from the
            // start) or at the end of the next block
            const uint32_t mode = hdr_stop ? 1u
                                  : !block ? 0u
                                           : ((!resume && s->wrap && !hdr_done) ? 1u : 2u) | (resume && s->itype ? 4u : 0u) |
                                                 (trees ? 8u : 0u);
            if (!rc) rc = inflate_try_locked(*L.c, s->in.data(), s->in.size(), resume,
                                             resume ? s->res_bit - 8ull * s->in_base : 0, s->hist.data(), hl,
                                             hl + s->cap, s->wrap, s->wbits, o, t, mode,
                                             s->iback_win ? 1u << s->wbits : 0u, &ixo, trees_after);
        }
        if (rc) return rc == ZGPU_ENODEV ? Z_MEM_ERROR : rc;
        if (t.stop != kIFull) {
            if (t.zcodes != 0xffffffffu) s->icodes = t.zcodes;
            const bool in_end_stop = t.stop == kIInEnd;
            s->isyncpt = in_end_stop && ((t.zstate >> 34) & 1u);
            s->imark = in_end_stop ? t.zmark : -65536;
            s->iheld_end = in_end_stop ? (uint32_t)t.zstate : 0;
        }
        if (t.stop == kIFull) {                                  // grow the output and decode again
            if (s->cap >= (size_t(1) << 31)) return Z_MEM_ERROR;
            s->cap *= 2;
            continue;
        }
        const uint64_t obase = resume ? s->res_put - hl : 0;     // absolute output byte of o[0]
        if (t.stop != kITrees) keep_index(s, ixo, t, obase, hl, t.stop != kIFull);   // (a header stop adds nothing)
        auto append_new = [&](uint64_t upto) {                   // s->out from out_at: o's bytes replace those it covers
            if (obase <= s->out_at) {
                s->out.assign(o.begin() + (std::ptrdiff_t)(s->out_at - obase), o.begin() + (std::ptrdiff_t)(upto - obase));
            } else {
                s->out.resize((size_t)(obase - s->out_at));
                s->out.insert(s->out.end(), o.begin(), o.begin() + (std::ptrdiff_t)(upto - obase));
            }
            s->out_pos = (size_t)(s->ideliv - s->out_at);
        };
        const uint64_t put_abs = obase + t.put;
        if (t.stop == kIBlock && hdr_stop) {                     // the header read: resume raw after it
            uint64_t bb = t.blk_bit;
            s->igz = (s->wrap & 2) && s->in.size() >= 2 && s->in[0] == 0x1f && s->in[1] == 0x8b;
            s->icheck = s->igz ? 0u : 1u;
            s->hist.clear();
            s->res_bit = bb;
            s->res_put = 0;
            s->imode = 1;
            s->itype = true;
            const uint64_t drop = (bb >> 3) - s->in_base;
            s->in.erase(s->in.begin(), s->in.begin() + (std::ptrdiff_t)drop);
            s->in_base += drop;
            s->tried = 0;
            continue;
        }
        if (t.stop == kIBlock) {
            // inflate(Z_BLOCK) at a block boundary (or before the first block):
            // the output through it, the resume point there, and the input after
            // the byte holding the boundary handed back -- the reference stops
            // there with that byte's unused bits in its bit buffer
            // (strm->data_type = bits + 128, inflate.c:1267-1269)
            append_new(put_abs);
            uint64_t bb = t.blk_bit, bp = t.blk_put;
            if (resume) { bb += 8ull * s->in_base; bp += obase; }
            if (!resume) {
                s->igz = (s->wrap & 2) && s->in.size() >= 2 && s->in[0] == 0x1f && s->in[1] == 0x8b;
                s->icheck = s->igz ? 0u : 1u;
            }
            if (is_check && !s->isync)
                s->icheck = check_of(s->icheck, o.data() + (s->res_put - obase), (size_t)(bp - s->res_put));
            const uint64_t h0 = bp > 32768 ? bp - 32768 : 0;
            s->hist.assign(o.begin() + (std::ptrdiff_t)(h0 - obase), o.begin() + (std::ptrdiff_t)(bp - obase));
            s->res_bit = bb;
            s->res_put = bp;
            s->imode = 1;
            const uint64_t used_abs = (bb + 7) >> 3;              // the input after it goes back (inflate_body)
            const size_t back = (size_t)std::min<uint64_t>(in_end - used_abs, took);
            s->in.resize(s->in.size() - back);
            const uint64_t drop = (bb >> 3) - s->in_base;         // input before the boundary's byte
            s->in.erase(s->in.begin(), s->in.begin() + (std::ptrdiff_t)drop);
            s->in_base += drop;
            s->tried = 0;
            s->itype = true;
            const bool last = (t.zstate >> 32) & 1u;
            s->itail = last;                                     // only the trailer is left
            s->idt = (int)((8 - (bb & 7)) & 7) + (last ? 64 : 0) + 128;
            s->iheld_end = (uint32_t)((8 - (bb & 7)) & 7);
            return Z_OK;
        }
        if (t.stop == kITrees) {
            // inflate(Z_TREES) after a block header: the header read (up to its
            // byte), no output; the decode resumes at the block's start, which
            // the reference has read past (the next Z_TREES / Z_BLOCK call runs
            // to the block's end), data_type + 256 (inflate.c:1267-1270); the
            // output an earlier decode left beyond stays
            const uint64_t hb = t.blk_bit + 8ull * (resume ? s->in_base : 0);
            const uint64_t used_abs = (hb + 7) >> 3;              // the input after it goes back (inflate_body)
            s->in.resize(s->in.size() - (size_t)std::min<uint64_t>(in_end - used_abs, took));
            s->tried = 0;
            s->itype = false;
            s->hdr_stop_now = true;
            const bool last = (t.zstate >> 32) & 1u;
            s->iheld_end = (uint32_t)(8 * used_abs - hb);
            s->idt = (int)s->iheld_end + (last ? 64 : 0) + 256;
            return Z_OK;
        }
        if (!resume && t.stop == kIDict) {
            // a zlib header with FDICT: Z_NEED_DICT with the header (2 bytes +
            // DICTID) consumed and the rest handed back (inflate.c DICTID/DICT);
            // inflateSetDictionary resumes after it
            s->acct_done = true;
            const size_t keep = 6, back = std::min<size_t>(s->in.size() - keep, took);
            strm->next_in -= back;
            strm->avail_in += (uInt)back;
            // inflate.c returns Z_NEED_DICT from DICT straight after RESTORE(),
            // not through inf_leave: what this call consumed is never added to
            // total_in (here, or later)
            strm->total_in -= took;
            s->iadj += took - back;
            s->in.resize(s->in.size() - back);
            s->need_dict = true;
            s->want_dict = ((uint32_t)s->in[2] << 24) | ((uint32_t)s->in[3] << 16) | ((uint32_t)s->in[4] << 8) | s->in[5];
            strm->adler = s->want_dict;
            return Z_OK;
        }
        if (!resume && t.stop != kIInEnd) {                      // the whole stream in one attempt
            append_new(put_abs);
            s->finished = 1;
            s->igz = (s->wrap & 2) && s->in.size() >= 2 && s->in[0] == 0x1f && s->in[1] == 0x8b;
            s->fin_used = t.used;                               // the input past it goes back (inflate_body)
            if (t.stop == kIEnd) {
                s->result = Z_STREAM_END;
                if (s->wrap) strm->adler = s->in.size() >= 2 && s->in[0] == 0x1f && s->in[1] == 0x8b
                                               ? ck_crc32(0, o.data(), o.size())
                                               : ck_adler32(1, o.data(), o.size());
            } else {
                s->result = Z_DATA_ERROR;
                strm->msg = const_cast<char *>("invalid or corrupt deflate stream");
            }
            return Z_OK;
        }
        if (resume && t.stop == kIData) {
            append_new(put_abs);
            s->finished = 1;
            s->result = Z_DATA_ERROR;
            strm->msg = const_cast<char *>("invalid or corrupt deflate stream");
            s->fin_used = s->in_base + t.used;
            return Z_OK;
        }
        if (resume && t.stop == kIEnd) {                         // the final block: check the trailer
            const uint64_t tpos = s->in_base + t.used;
            const uint64_t need = !s->wrap || s->isync == 2 ? 0 : s->igz ? 8 : 4;
            if (in_end >= tpos + need) {
                append_new(put_abs);
                s->finished = 1;
                s->result = Z_STREAM_END;
                uint32_t ck = s->icheck;
                if (is_check) ck = check_of(ck, o.data() + (s->res_put - obase), (size_t)(put_abs - s->res_put));
                const uint8_t *tr = s->in.data() + (tpos - s->in_base);
                bool ok = true;
                if (s->isync || !s->ivalid) {
                    // after inflateSync, or with inflateValidate(strm, 0), the trailer
                    // is read, not checked (wrap &= ~4)
                } else if (s->wrap && !s->igz) {
                    ok = ((uint32_t)tr[0] << 24 | (uint32_t)tr[1] << 16 | (uint32_t)tr[2] << 8 | tr[3]) == ck;
                    if (!ok) strm->msg = const_cast<char *>("incorrect data check");
                } else if (s->igz) {
                    const uint32_t c = tr[0] | (uint32_t)tr[1] << 8 | (uint32_t)tr[2] << 16 | (uint32_t)tr[3] << 24;
                    const uint32_t z = tr[4] | (uint32_t)tr[5] << 8 | (uint32_t)tr[6] << 16 | (uint32_t)tr[7] << 24;
                    ok = c == ck && z == (uint32_t)put_abs;
                    if (!ok) strm->msg = const_cast<char *>(c != ck ? "incorrect data check" : "incorrect length check");
                }
                if (ok) {
                    s->fin_used = tpos + need;
                    if (s->wrap && !s->isync && s->ivalid) strm->adler = ck;
                    s->idt = 64;                                 // the last block, done
                } else {
                    s->fin_used = in_end;
                    s->result = Z_DATA_ERROR;
                }
                return Z_OK;
            }
            // the trailer is not all here: wait at the last block boundary
        }
        // the stream goes on: hand out its prefix, move the resume point
        append_new(put_abs);
        s->tried = in_end;
        if (!resume) s->igz = (s->wrap & 2) && s->in.size() >= 2 && s->in[0] == 0x1f && s->in[1] == 0x8b;
        // where the input ran out (inflate.c:1267-1269): what a later Z_BLOCK
        // call reports once the output is all handed out
        s->idt = (int)(t.zstate & 0xffffffffu) + ((t.zstate >> 32) & 1u ? 64 : 0) + ((t.zstate >> 33) & 1u ? 128 : 0);
        // the resume point moves after the output is handed out (inflate_body):
        // to the last block boundary the reference has passed
        return Z_OK;
    }
}
}  // namespace

// The gzip header as far as it has arrived, into inflateGetHeader's gz_header
// (inflate.c HEAD .. HCRC: text, time, xflags, os, extra_len, extra / name /
// comment up to their max, hcrc, done = 1 once complete; done = -1 for a zlib
// stream; extra / name / comment set to Z_NULL when the flag is absent).
void gz_header_fill(internal_state *s) {
    gz_header *h = s->ihead;
    if (!h || h->done != 0 || s->in_base != 0) return;
    const uint8_t *b = s->in.data();
    const size_t m = s->in.size();
    if (m < 2) return;
    if (!(b[0] == 0x1f && b[1] == 0x8b)) { h->done = -1; return; }
    if (m < 4) return;
    const unsigned flags = b[2] | (unsigned)b[3] << 8;
    if ((flags & 0xffu) != Z_DEFLATED || (flags & 0xe000u)) return;   // BAD: no more fields
    h->text = (int)((flags >> 8) & 1u);
    if (m < 8) return;
    h->time = (uLong)b[4] | (uLong)b[5] << 8 | (uLong)b[6] << 16 | (uLong)b[7] << 24;
    if (m < 10) return;
    h->xflags = b[8];
    h->os = b[9];
    size_t p = 10;
    if (flags & 0x0400u) {
        if (m < 12) return;
        const unsigned xlen = b[10] | (unsigned)b[11] << 8;
        h->extra_len = xlen;
        p = 12;
        const size_t have = std::min<size_t>(xlen, m - p);
        if (h->extra) std::memcpy(h->extra, b + p, std::min<size_t>(have, h->extra_max));
        if (have < xlen) return;
        p += xlen;
    } else {
        h->extra = nullptr;
    }
    for (int k = 0; k < 2; k++) {                               // FNAME, FCOMMENT
        Bytef *&dst = k ? h->comment : h->name;
        const uInt max = k ? h->comm_max : h->name_max;
        if (!(flags & (k ? 0x1000u : 0x0800u))) { dst = nullptr; continue; }
        size_t q = p;
        while (q < m && b[q]) q++;
        const bool end = q < m;
        if (dst) std::memcpy(dst, b + p, std::min<size_t>((end ? q + 1 : q) - p, max));
        if (!end) return;
        p = q + 1;
    }
    if (flags & 0x0200u) {                                      // FHCRC: a mismatch is BAD (the decode says so)
        if (m < p + 2) return;
        const uint32_t c = ck_crc32(0, b, p);
        if ((c & 0xffffu) != (uint32_t)(b[p] | b[p + 1] << 8)) return;
    }
    h->hcrc = (int)((flags >> 9) & 1u);
    h->done = 1;
}

// a zlib / gzip header has been read (inflate.c's state->flags != -1)
bool inflate_header_seen(const internal_state *s) {
    if (!s->wrap) return false;
    if (s->imode == 1 || s->ideliv || s->finished || s->in_base) return true;
    const uint8_t *b = s->in.data();
    const size_t m = s->in.size();
    if (m < 2) return false;
    if (!((s->wrap & 2) && b[0] == 0x1f && b[1] == 0x8b)) return true;   // a zlib header (checked by the decode)
    return m >= 4;                                              // gzip: FLAGS read (inflate.c FLAGS sets state->flags)
}

// Where the reference stops reading when its output space ends at absolute
// output X with more output due: inflate.c's LIT, MATCH and COPY wait for room
// only after the symbol's codes are read (a stored block: after the bytes
// copied), and inf_leave returns the bytes pulled so far, the bit position
// rounded up (inflate_fast returns the whole bytes it holds; the slow path pulls
// a byte only when a code needs it).  From the last decode's symbol index
// (InflateIndex); ~0 when X lies outside it.  dt: the data_type inflate.c
// reports there (the bits it holds, + 64 in the last block; mode LIT / MATCH /
// COPY).
static uint64_t stall_in(const std::vector<uint64_t> &e, uint64_t ibase, uint64_t obase, uint64_t o0, uint64_t X,
                         int *dt, uint32_t *held) {
    if (X < o0) return ~0ull;
    size_t lo = 0, hi = e.size() / 2;                           // the first symbol whose output ends past X
    while (lo < hi) {
        const size_t m = (lo + hi) / 2;
        if ((uint32_t)e[2 * m] + obase > X) hi = m;
        else lo = m + 1;
    }
    if (2 * lo == e.size()) return ~0ull;
    const uint64_t a = e[2 * lo], v = e[2 * lo + 1];
    const int last = (a >> 33) & 1u ? 64 : 0;
    if ((a >> 32) & 1u) {                                       // a stored run: the bytes copied before X
        const uint64_t start = lo ? (uint32_t)e[2 * lo - 2] + obase : o0;
        if (dt) *dt = last;
        if (held) *held = 0;
        return ibase + v + (X - start);
    }
    const uint64_t c = (v + 7) >> 3;
    if (dt) *dt = (int)(8 * c - v) + last;
    if (held) *held = (uint32_t)(8 * c - v);
    return ibase + c;
}
static uint64_t stall_from_index(const internal_state *s, uint64_t X, int *dt = nullptr, uint32_t *held = nullptr) {
    const uint64_t c = stall_in(s->ix, s->ix_ibase, s->ix_obase, s->ix_o0, X, dt, held);
    return c != ~0ull ? c : stall_in(s->ix2, s->ix2_ibase, s->ix2_obase, s->ix2_o0, X, dt, held);
}

// the symbol index rebuilt from the resume point (at or before X) to 4 MiB of
// output past X, the resume point moved up to X (the index of the last attempt
// stops kIdxCap symbols after its start)
static int refresh_index(internal_state *s, uint64_t X) {
    const bool resume = s->imode == 1;
    const size_t hl = resume ? s->hist.size() : 0;
    const uint64_t from = resume ? s->res_put : 0;
    const uint64_t cap = hl + std::min<uint64_t>(X - from + (4u << 20), 1ull << 31);
    if (from > X) return Z_OK;                                  // a Z_BLOCK stop's resume point: past X
    std::vector<uint8_t> o;
    InflateTry t{};
    InflateIndex ixo;
    int rc;
    {
        Lease L;
        rc = L.rc;
        if (!rc) rc = inflate_try_locked(*L.c, s->in.data(), s->in.size(), resume,
                                         resume ? s->res_bit - 8ull * s->in_base : 0, s->hist.data(), hl, cap,
                                         s->wrap, s->wbits, o, t, 0, s->iback_win ? 1u << s->wbits : 0u, &ixo);
    }
    if (rc) return rc == ZGPU_ENODEV ? Z_MEM_ERROR : rc;
    keep_index(s, ixo, t, from - hl, hl, t.stop != kIFull);
    return Z_OK;
}

static int inflate_body(z_streamp strm, int flush) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (!strm->next_out || (strm->avail_in && !strm->next_in)) return Z_STREAM_ERROR;   // inflate.c:610-612
    if (s->need_dict) return Z_NEED_DICT;                      // inflate.c DICT: until the dictionary is set
    // Z_TREES: Z_BLOCK's stops and one after each block header (inflate.c)
    const bool trees = flush == Z_TREES;
    const bool block = flush == Z_BLOCK || trees;
    const Bytef *const next0 = strm->next_in;
    const uInt avail0 = strm->avail_in;
    const uLong total0 = strm->total_in;
    // Z_BLOCK: while the block the last call stopped at is still being handed
    // out, the reference reads no more input
    // Z_BLOCK after a stop at a block's end whose output is still being handed
    // out (the resume point past it): the reference reads no more input
    const bool taking = !(s->finished || (block && s->res_put > s->ideliv));
    const uint64_t pref0 = 8 * s->cons - s->iheld;             // the reference's bit position
    s->acct_done = false;
    s->hdr_stop_now = false;
    size_t took = 0;                 // bytes new to the engine
    bool redo = false;               // decode again: the bytes handed back came back different
    if (taking) {
        // the bytes the last call handed back (in from cons on) are expected
        // first; when they come back as they went (the same next_in, or equal
        // bytes) what they decoded to stands, else the decode goes again from
        // the resume point (at or before the output handed out) with what came
        const uint64_t I = s->in_base + s->in.size();
        uint64_t held = I > s->cons ? I - s->cons : 0;
        if (held) {
            // (after a Z_BLOCK stop the engine may have dropped input up to the
            // block boundary's byte, past cons: those bytes are taken as they were)
            const bool same = avail0 >= held &&
                              (next0 == s->held_at || s->cons < s->in_base ||
                               std::memcmp(next0, s->in.data() + (s->cons - s->in_base), (size_t)held) == 0);
            if (!same && s->res_put <= s->ideliv && s->cons >= s->in_base) {
                s->in.resize((size_t)(s->cons - s->in_base));
                s->out.resize(s->out_pos);                      // what was handed out stays (the window)
                s->tried = 0;
                s->ix.clear();
                s->ix2.clear();
                s->ix_all = false;
                held = 0;
                redo = true;
            }
        }
        took = avail0 > held ? (size_t)(avail0 - held) : 0;
    }
    if (took && s->iprime_n) {
        // inflatePrime's bits: P virtual bytes in front of the input, the primed
        // bits their last ones (a decode reads each byte from bit 0 up), the
        // decode resumed raw from there; total_in does not count the P bytes
        const uint32_t P = (s->iprime_n + 7) / 8;
        const uint64_t v = s->iprime_v << (8 * P - s->iprime_n);
        for (uint32_t k = 0; k < P; k++) s->in.push_back((uint8_t)(v >> (8 * k)));
        s->iadj += P;
        s->cons += P;
        s->res_bit = 8ull * P - s->iprime_n;
        s->res_put = s->ideliv;
        if (!s->imode) s->hist.clear();
        s->imode = 1;
        s->icheck = 1;
        s->iprime_n = 0;
        s->iprime_v = 0;
    }
    const uint64_t T = s->cons;      // absolute input position of next0[0]
    if (took) s->in.insert(s->in.end(), next0 + (avail0 - took), next0 + avail0);
    if (taking) {                    // all of it for now; the accounting below hands back what the reference leaves
        strm->next_in = next0 + avail0;
        strm->avail_in = 0;
        strm->total_in = total0 + avail0;
    }
    gz_header_fill(s);
    // Decode what has arrived whenever input arrives: a stream that is still
    // open (a sync-flushed connection, a file read in pieces) hands out every
    // byte its input decodes to so far, as inflate() does (inflate.c:622-1221).
    // Each attempt resumes at a block boundary (inflate_attempt).
    const uint64_t in_end = s->in_base + s->in.size();
    // (the trailer after a Z_BLOCK stop at the last block is read once its
    // output is all handed out)
    const bool tail_due = s->itail && s->out_pos >= s->out.size();
    // Z_TREES with the reference at a block's start: the header stop needs a
    // decode even when no new input came (the index knows no header ends)
    const bool trees_due = trees && !s->finished && s->imode == 1 && pref0 == s->res_bit;
    bool decoded = false;
    if (!s->finished && (took || redo || tail_due || trees_due || (flush == Z_FINISH && s->tried != in_end))) {
        decoded = true;
        if (block) s->idt = 0;
        if (int rc = inflate_attempt(strm, s, taking ? avail0 : 0, block, trees)) return rc;
        if (s->need_dict) {
            s->cons = strm->total_in + s->iadj;
            s->held_at = strm->next_in;
            return Z_NEED_DICT;
        }
    }
    if (block) strm->data_type = s->idt;
    // Z_BLOCK with output of an earlier call still to hand out: the reference
    // decodes on only to the end of the block it is in (inflate.c TYPE), the
    // first boundary past the output handed out
    uint64_t cap_put = ~0ull, cap_bit = 0;
    bool cap_hdr = false, cap_last = false;             // Z_TREES: the stop is a header's end (BFINAL of its block)
    if (block && s->out_pos < s->out.size() && !s->hdr_stop_now) {
        for (size_t k = 0; k + 1 < s->bx.size(); k += 2)
            // (past a header stop the block's end may be where the reference stands: an empty stored block)
            if ((s->bx[k] > pref0 || (s->after_hdr && s->bx[k] == pref0)) && s->bx[k + 1] >= s->ideliv) {
                cap_bit = s->bx[k];
                cap_put = s->bx[k + 1];
                break;
            }
        if (trees)                                      // ... or the end of a header the reference has not read
            for (size_t k = 0; k + 1 < s->hx.size(); k += 2) {
                const uint64_t hb = s->hx[k] & ~(1ull << 63);
                if (hb > pref0 && s->hx[k + 1] >= s->ideliv) {
                    if (cap_put == ~0ull || hb <= cap_bit) {    // (an empty stored block: its header stop comes first)
                        cap_bit = hb;
                        cap_put = s->hx[k + 1];
                        cap_hdr = true;
                        cap_last = s->hx[k] >> 63;
                    }
                    break;
                }
            }
    }
    size_t give = 0;
    if (s->out_pos < s->out.size() && !s->hdr_stop_now) {      // (stopped after a header: no output)
        give = std::min<size_t>(strm->avail_out, s->out.size() - s->out_pos);
        if (cap_put != ~0ull) give = (size_t)std::min<uint64_t>(give, cap_put - s->ideliv);
        std::memcpy(strm->next_out, s->out.data() + s->out_pos, give);
        s->out_pos += give;
        s->ideliv += give;
        strm->next_out += give;
        strm->avail_out -= (uInt)give;
        strm->total_out += give;
    }
    // the last block's output all handed out after a Z_BLOCK stop at its end:
    // a call that does not stop at block ends reads the trailer too (inflate.c
    // TYPEDO .. CHECK .. DONE)
    if (!block && s->itail && !s->finished && !s->acct_done && s->out_pos >= s->out.size())
        if (int rc = inflate_attempt(strm, s, taking ? avail0 : 0, false)) return rc;
    // the input this call consumed (inflate.c inf_leave): all of it unless the
    // output space ended first, then up to the reference's stop at the output
    // handed out (stall_from_index); a finished stream's up to its end
    const bool pending = s->out_pos < s->out.size() && !s->hdr_stop_now;
    if (s->acct_done) {
        s->cons = strm->total_in + s->iadj;
    } else {
        uint64_t C;
        s->iheld = s->iheld_end;
        if (s->ideliv == cap_put && cap_hdr) {
            // after a block header, mode LEN_ / COPY_ (Z_TREES)
            C = (cap_bit + 7) >> 3;
            s->iheld = (uint32_t)(8 * C - cap_bit);
            strm->data_type = (int)s->iheld + 256 + (cap_last ? 64 : 0);
        } else if (s->ideliv == cap_put) {
            // at the block's end, mode TYPE: the bits after its end-of-block code held
            C = (cap_bit + 7) >> 3;
            s->iheld = (uint32_t)(8 * C - cap_bit);
            strm->data_type = (int)s->iheld + 128 + (cap_bit == s->bx_last ? 64 : 0);
            if (cap_bit == s->bx_last && !s->finished) s->itail = true;   // the trailer next
        } else if (pending) {
            int dt = -1;
            C = stall_from_index(s, s->ideliv, &dt, &s->iheld);
            if (C == ~0ull) {
                if (int rc = refresh_index(s, s->ideliv)) return rc;
                C = stall_from_index(s, s->ideliv, &dt, &s->iheld);
            }
            if (C == ~0ull) C = s->finished ? s->fin_used : s->in_base + s->in.size();
            if (block && dt >= 0) strm->data_type = dt;        // stopped for room, not at a block boundary
        } else {
            C = s->finished ? s->fin_used : s->in_base + s->in.size();
        }
        const uint64_t used = std::min<uint64_t>(C > T ? C - T : 0, avail0);
        strm->next_in = next0 + used;
        strm->avail_in = avail0 - (uInt)used;
        strm->total_in = total0 + used;
        s->cons = T + used;
        if (s->finished && !pending) {
            s->in.clear();
            s->in.shrink_to_fit();
        } else if (!s->finished) {
            // the resume point to the last boundary the reference has passed
            advance_resume(s, s->ideliv, 8 * s->cons - s->iheld, s->itail);
        }
        // the reference stands after a header: it stopped there this call, or
        // stood there before and nothing moved it
        s->after_hdr = s->hdr_stop_now || (s->ideliv == cap_put && cap_hdr) ||
                       (s->after_hdr && !decoded && give == 0 && s->ideliv != cap_put &&
                        8 * s->cons - s->iheld == pref0);
    }
    s->held_at = strm->next_in;
    if (s->finished && !pending && s->ideliv != cap_put) return s->result;
    // inflate.c:1261-1262: no progress, or Z_FINISH short of the stream end
    if ((strm->next_in == next0 && give == 0) || flush == Z_FINISH) return Z_BUF_ERROR;
    return Z_OK;
}

// inflateSetDictionary (inflate.c): a zlib stream that answered Z_NEED_DICT
// goes on with the dictionary as its window (its Adler-32 must equal the
// header's DICTID, else Z_DATA_ERROR); a raw stream takes it as the window
// before its first input.  The decode resumes after the 6 header bytes with the
// window's last 1 << CINFO+8 bytes in front of the output (inflate_attempt).
int inflateSetDictionary(z_streamp strm, const Bytef *dictionary, uInt dictLength) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (s->wrap != 0 && !s->need_dict) return Z_STREAM_ERROR;
    if (dictLength && !dictionary) return Z_STREAM_ERROR;
    try {
        if (s->need_dict) {
            if (ck_adler32(1, dictionary, dictLength) != s->want_dict) return Z_DATA_ERROR;
        } else if (!s->in.empty() || s->ideliv || s->imode) {
            strm->msg = const_cast<char *>("inflateSetDictionary: raw streams before their first input only");
            return Z_STREAM_ERROR;
        }
        // updatewindow keeps 1 << state->wbits bytes: inflateInit2_'s windowBits,
        // or, when that is 0, the zlib header's CINFO + 8 (inflate.c HEAD)
        const int wb = s->wbits ? s->wbits : s->need_dict ? (s->in[0] >> 4) + 8 : 15;
        const size_t wsize = size_t(1) << wb, keep = std::min<size_t>(dictLength, wsize);
        s->hist.assign(dictionary + (dictLength - keep), dictionary + dictLength);
        s->iwin.assign(s->hist.begin(), s->hist.end());        // updatewindow(dictionary + dictLength, dictLength)
        s->iwin_on = true;
        s->res_bit = s->need_dict ? 48 : 0;                    // after CMF, FLG and DICTID
        s->res_put = s->ideliv = s->hist.size();               // the window counts as handed out
        s->icheck = 1;
        s->igz = 0;
        s->imode = 1;
        s->need_dict = false;
        s->tried = 0;
        return Z_OK;
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}

// inflateBackInit_ / inflateBack / inflateBackEnd (infback.c:25-640): a raw
// deflate stream pulled through in() and pushed through out() in pieces of at
// most the caller's window (1 << windowBits bytes).  The decode is the
// streaming inflate() above, fed whatever in() returns; its output is staged
// in the caller's window and handed to out() whenever the window is full, at
// the stream end and before any error return, as infback.c's inf_leave does.
// Unused input is left in strm->next_in / avail_in; total_in / total_out are
// not touched.  Returns Z_STREAM_END, Z_DATA_ERROR, Z_MEM_ERROR or Z_BUF_ERROR
// (in() gave no input: strm->next_in is then Z_NULL; or out() returned nonzero).
int inflateBackInit_(z_streamp strm, int windowBits, unsigned char *window, const char *version, int stream_size) {
    if (!version || version[0] != ZGPU_ZLIB_VERSION[0] || stream_size != (int)sizeof(z_stream))
        return Z_VERSION_ERROR;                                       // infback.c:30-32
    if (!strm || !window || windowBits < 8 || windowBits > 15) return Z_STREAM_ERROR;
    strm->msg = nullptr;
    internal_state *s = new_state(strm);
    if (!s) return Z_MEM_ERROR;
    s->inflating = 1;
    s->wrap = 0;
    s->wbits = windowBits;
    s->iback_win = window;
    s->out_pos = 0;
    s->finished = 0;
    strm->state = s;
    return Z_OK;
}

int inflateBack(z_streamp strm, in_func in, void *in_desc, out_func out, void *out_desc) {
    if (!strm || !strm->state || !strm->state->inflating || !strm->state->iback_win || !in || !out)
        return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    const uLong tin = strm->total_in, tout = strm->total_out, adl = strm->adler;
    if (int rc = inflateReset(strm)) return rc;                          // mode = TYPE, whave = 0
    unsigned char *win = s->iback_win;
    const unsigned wsize = 1u << s->wbits;
    const unsigned char *next = strm->next_in;
    unsigned have = next ? strm->avail_in : 0;
    unsigned left = wsize;                                               // window bytes still free
    int ret = Z_BUF_ERROR;
    for (;;) {
        // in() only when the decode has nothing left to hand out (infback.c
        // pulls input when a code needs bits; a full window goes to out() first)
        if (have == 0 && s->out_pos >= s->out.size()) {
            have = in(in_desc, &next);
            if (have == 0) { next = nullptr; ret = Z_BUF_ERROR; break; }
        }
        strm->next_in = next;
        strm->avail_in = have;
        strm->next_out = win + (wsize - left);
        strm->avail_out = left;
        const int r = inflate(strm, Z_NO_FLUSH);
        next = strm->next_in;
        have = strm->avail_in;
        left = strm->avail_out;
        if (r == Z_STREAM_END) { ret = Z_STREAM_END; break; }
        if (r == Z_DATA_ERROR || r == Z_MEM_ERROR || r == Z_STREAM_ERROR) { ret = r; break; }
        if (left == 0) {                                                 // the window is full
            if (out(out_desc, win, wsize)) { ret = Z_BUF_ERROR; left = wsize; break; }
            left = wsize;
        }
    }
    // inf_leave: the window's leftover output, then the unused input
    if (left < wsize && out(out_desc, win, wsize - left) && ret == Z_STREAM_END) ret = Z_BUF_ERROR;
    strm->next_in = next;
    strm->avail_in = next ? have : 0;
    strm->total_in = tin;
    strm->total_out = tout;
    strm->adler = adl;
    return ret;
}

int inflateBackEnd(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating || !strm->state->iback_win) return Z_STREAM_ERROR;
    free_state(strm, strm->state);
    strm->state = nullptr;
    return Z_OK;
}

int inflateEnd(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    free_state(strm, strm->state);
    strm->state = nullptr;
    return Z_OK;
}

// inflateGetHeader (inflate.c:1330-1340): gzip streams only; the fields are
// filled as the header arrives (gz_header_fill)
int inflateGetHeader(z_streamp strm, gz_headerp head) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if ((s->wrap & 2) == 0 || !head) return Z_STREAM_ERROR;
    s->ihead = head;
    head->done = 0;
    gz_header_fill(s);
    return Z_OK;
}

// inflateSync (inflate.c:1375-1437): skip input up to and through the next
// 00 00 ff ff (a Z_SYNC_FLUSH / Z_FULL_FLUSH point; a search split over calls
// goes on where it stopped), then restart on a new block with no window and
// no check value: a stream whose header was read keeps its trailer, unchecked;
// one without (raw, or no header yet) ends with its last block.  The bits
// the reference may hold in its bit buffer are not searched: this engine
// holds none between calls.
int inflateSync(z_streamp strm) {
    if (!strm || !strm->state || !strm->state->inflating) return Z_STREAM_ERROR;
    internal_state *s = strm->state;
    if (strm->avail_in == 0 && (s->isyncing || s->iheld < 8)) return Z_BUF_ERROR;   // inflate.c:1385
    uint32_t got = s->isync_have;
    if (!s->isyncing) {
        // inflate.c:1388-1398: the whole bytes in the bit buffer (the last input
        // consumed, after its oldest bits & 7 are dropped) are searched first
        s->isyncing = true;
        got = 0;
        const uint64_t k = s->iheld / 8;
        if (k && s->cons >= s->in_base + k && s->cons - s->in_base <= s->in.size())
            for (const uint8_t *b = s->in.data() + (s->cons - k - s->in_base), *e = b + k; b < e && got < 4; b++) {
                if (*b == (got < 2 ? 0 : 0xff)) got++;
                else if (*b) got = 0;
                else got = 4 - got;
            }
        s->iheld = 0;
    }
    uInt len = 0;
    while (len < strm->avail_in && got < 4) {                   // syncsearch (inflate.c:1352-1373)
        const uint8_t c = strm->next_in[len];
        if (c == (got < 2 ? 0 : 0xff)) got++;
        else if (c) got = 0;
        else got = 4 - got;
        len++;
    }
    s->isync_have = got;
    strm->next_in += len;
    strm->avail_in -= len;
    strm->total_in += len;
    if (got != 4) return Z_DATA_ERROR;
    const bool hdr = inflate_header_seen(s);
    if (hdr && s->imode == 0 && s->in.size() >= 2)
        s->igz = (s->wrap & 2) && s->in[0] == 0x1f && s->in[1] == 0x8b;
    s->isync = hdr ? 1 : 2;
    try {
        s->in.clear();
        s->out.clear();
        s->hist.clear();
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
    s->out_pos = 0;
    s->out_at = s->ideliv;
    s->bx.clear();
    s->hx.clear();
    s->ix2.clear();
    s->after_hdr = false;
    s->in_base = strm->total_in + s->iadj;                     // absolute input position
    s->cons = s->in_base;
    s->held_at = strm->next_in;
    s->ix.clear();
    s->ix_all = false;
    s->finished = 0;
    s->result = Z_OK;
    s->tried = 0;
    s->imode = 1;
    s->res_bit = 8ull * s->in_base;
    s->res_put = s->ideliv;
    s->icheck = s->igz ? 0u : 1u;
    s->need_dict = false;
    s->isyncing = false;
    s->itype = true;                                            // mode TYPE
    s->itail = false;
    // inflate.c:1410-1416: wrap &= ~4, then inflateReset's adler = wrap & 1 --
    // the stream's wrap setting (1 zlib, 2 gzip, 3 auto-detect), not the header
    // found: an auto-detecting stream reports 1 after a gzip header too
    if (hdr) strm->adler = (uLong)(s->wrap & 1);
    return Z_OK;
}

// inflateCopy (inflate.c:1439-1485): a deep copy of the stream and its state
int inflateCopy(z_streamp dest, z_streamp source) {
    if (!dest || !source || !source->state || !source->state->inflating) return Z_STREAM_ERROR;
    *dest = *source;
    internal_state *s = new_state(dest, source->state);
    if (!s) return Z_MEM_ERROR;
    dest->state = s;
    return Z_OK;
}

// the entry points that allocate: an allocation failure is Z_MEM_ERROR
int deflate(z_streamp strm, int flush) {
    try {
        return deflate_body(strm, flush);
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}
int inflate(z_streamp strm, int flush) {
    try {
        const bool ok = strm && strm->state && strm->state->inflating;
        const Bytef *next0 = ok ? strm->next_out : nullptr;
        const uInt out0 = ok ? strm->avail_out : 0;
        const int rc = inflate_body(strm, flush);
        if (ok && strm->state) {
            // updatewindow's condition (inflate.c:1249-1256): the window exists, or
            // this call wrote output, did not stop on an error and did not end the
            // stream under Z_FINISH
            internal_state *s = strm->state;
            const size_t n = out0 - strm->avail_out;
            const bool bad = rc == Z_DATA_ERROR || rc == Z_MEM_ERROR || rc == Z_STREAM_ERROR;
            // the check value of a zlib / gzip stream as each call leaves it: the
            // running check of the bytes written, from 1 (zlib) / 0 (gzip) once the
            // header is in; none after inflateSync or with inflateValidate(0)
            if (s->wrap && !s->isync && !s->iback_win && !s->need_dict) {
                if (!s->iadl_on && (n || s->imode == 1 || s->finished)) {
                    s->iadl_on = true;
                    s->iadl = s->igz ? 0u : 1u;
                }
                if (s->iadl_on) {
                    if (n && s->ivalid)
                        s->iadl = s->igz ? ck_crc32(s->iadl, next0, n) : ck_adler32(s->iadl, next0, n);
                    strm->adler = s->iadl;
                }
            }
            // inflate.c CHECK resets its output count (out = left) before inf_leave's
            // updatewindow: the call that completes a zlib / gzip stream adds
            // nothing to the window
            const bool checked = rc == Z_STREAM_END && s->wrap != 0;
            if (!checked && (s->iwin_on || (n && !bad && (rc != Z_STREAM_END || flush != Z_FINISH)))) {
                s->iwin_on = true;
                const size_t ws = inflate_wsize(s);
                if (n >= ws) {
                    s->iwin.assign(next0 + (n - ws), next0 + n);
                } else {
                    s->iwin.insert(s->iwin.end(), next0, next0 + n);
                    if (s->iwin.size() > ws) s->iwin.erase(s->iwin.begin(), s->iwin.end() - (std::ptrdiff_t)ws);
                }
            }
        }
        return rc;
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}
int compress2(Bytef *dest, uLongf *destLen, const Bytef *source, uLong sourceLen, int level) {
    try {
        return compress2_body(dest, destLen, source, sourceLen, level);
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}
int uncompress2(Bytef *dest, uLongf *destLen, const Bytef *source, uLong *sourceLen) {
    try {
        return uncompress2_body(dest, destLen, source, sourceLen);
    } catch (const std::bad_alloc &) {
        return Z_MEM_ERROR;
    }
}

// ----------------------- reference WASM front-end -----------------------

int zlib_decompress_buffer(const unsigned char *src, unsigned long src_len, unsigned char *dest,
                           unsigned long *dest_len) {                // src/wasm_module.c:53-60
    if (!src || !dest || !dest_len || src_len == 0) return Z_STREAM_ERROR;
    return uncompress(dest, dest_len, src, src_len);
}
int zlib_decompress_optimized(const unsigned char *input, unsigned long input_len, unsigned char *output,
                              unsigned long *output_len) {           // src/wasm_module_simd.c:425-428
    return zlib_decompress_buffer(input, input_len, output, output_len);
}
int zlib_decompress(const unsigned char *input, unsigned long input_len, unsigned char *output,
                    unsigned long *output_len) {                     // src/wasm_module_simd.c:453-456
    return zlib_decompress_buffer(input, input_len, output, output_len);
}

struct zlib_stream_s {                                                // src/wasm_module.c:160-163
    z_stream stream;
    int initialized;
};

zlib_stream_t *zlib_deflate_init(int level, int window_bits, int mem_level, int strategy) {
    if (level < 0 || level > 9) level = Z_DEFAULT_COMPRESSION;        // src/wasm_module.c:168-186
    if (window_bits < 8 || window_bits > 15) window_bits = 15;
    if (mem_level < 1 || mem_level > 9) mem_level = 8;
    zlib_stream_t *ctx = static_cast<zlib_stream_t *>(std::calloc(1, sizeof(zlib_stream_t)));
    if (!ctx) return nullptr;
    if (deflateInit2_(&ctx->stream, level, Z_DEFLATED, window_bits, mem_level, strategy, ZGPU_ZLIB_VERSION,
                      (int)sizeof(z_stream)) != Z_OK) {
        std::free(ctx);                                               // windowBits < 15 / memLevel != 8
        return nullptr;
    }
    ctx->initialized = 1;
    return ctx;
}
int zlib_deflate_process(zlib_stream_t *ctx, const unsigned char *input, unsigned int input_len,
                         unsigned char *output, unsigned int output_len, int flush) {
    if (!ctx || !ctx->initialized) return Z_STREAM_ERROR;             // src/wasm_module.c:192-203
    ctx->stream.next_in = const_cast<Bytef *>(input);
    ctx->stream.avail_in = input_len;
    ctx->stream.next_out = output;
    ctx->stream.avail_out = output_len;
    return deflate(&ctx->stream, flush);
}
void zlib_deflate_end(zlib_stream_t *ctx) {                           // src/wasm_module.c:209-215
    if (!ctx) return;
    if (ctx->initialized) deflateEnd(&ctx->stream);
    std::free(ctx);
}
zlib_stream_t *zlib_inflate_init(int window_bits) {                  // src/wasm_module.c:209-226
    if (window_bits < 8 || window_bits > 15) window_bits = 15;
    zlib_stream_t *ctx = static_cast<zlib_stream_t *>(std::calloc(1, sizeof(zlib_stream_t)));
    if (!ctx) return nullptr;
    if (inflateInit2_(&ctx->stream, window_bits, ZGPU_ZLIB_VERSION, (int)sizeof(z_stream)) != Z_OK) {
        std::free(ctx);
        return nullptr;
    }
    ctx->initialized = 1;
    return ctx;
}
int zlib_inflate_process(zlib_stream_t *ctx, const unsigned char *input, unsigned int input_len,
                         unsigned char *output, unsigned int output_len) {   // src/wasm_module.c:232-243
    if (!ctx || !ctx->initialized) return Z_STREAM_ERROR;
    ctx->stream.next_in = const_cast<Bytef *>(input);
    ctx->stream.avail_in = input_len;
    ctx->stream.next_out = output;
    ctx->stream.avail_out = output_len;
    return inflate(&ctx->stream, Z_NO_FLUSH);
}
void zlib_inflate_end(zlib_stream_t *ctx) {                           // src/wasm_module.c:249-255
    if (!ctx) return;
    if (ctx->initialized) inflateEnd(&ctx->stream);
    std::free(ctx);
}
unsigned int zlib_stream_avail_in(zlib_stream_t *ctx) { return ctx ? ctx->stream.avail_in : 0; }
unsigned int zlib_stream_avail_out(zlib_stream_t *ctx) { return ctx ? ctx->stream.avail_out : 0; }
unsigned long zlib_stream_total_in(zlib_stream_t *ctx) { return ctx ? ctx->stream.total_in : 0; }
unsigned long zlib_stream_total_out(zlib_stream_t *ctx) { return ctx ? ctx->stream.total_out : 0; }
int zlib_compress_optimized(const unsigned char *input, unsigned long input_len, unsigned char *output,
                            unsigned long *output_len, int level) {  // src/wasm_module_simd.c:419-422
    return zlib_compress_buffer(input, input_len, output, output_len, level);
}
int zlib_compress(const unsigned char *input, unsigned long input_len, unsigned char *output,
                  unsigned long *output_len, int level) {            // src/wasm_module_simd.c:447-450
    return zlib_compress_buffer(input, input_len, output, output_len, level);
}

int zlib_compress_buffer(const unsigned char *src, unsigned long src_len, unsigned char *dest,
                         unsigned long *dest_len, int level) {         // src/wasm_module.c:34-46
    if (!src || !dest || !dest_len || src_len == 0) return Z_STREAM_ERROR;
    if (level < 0 || level > 9) level = Z_DEFAULT_COMPRESSION;
    return compress2(dest, dest_len, src, src_len, level);
}
unsigned long zlib_crc32(unsigned long crc, const unsigned char *buf, unsigned int len) {
    return crc32(crc, buf, len);                                      // src/wasm_module.c:65-68
}
unsigned long zlib_adler32(unsigned long adler, const unsigned char *buf, unsigned int len) {
    return adler32(adler, buf, len);                                  // src/wasm_module.c:73-76
}
unsigned long zlib_compress_bound(unsigned long source_len) { return compressBound(source_len); }
const char *zlib_get_version(void) { return zlibVersion(); }

int zlib_compress_simd_full(const uint8_t *input, size_t input_len, uint8_t *output,
                            size_t *output_len, int level) {         // src/zlib_simd_optimized.c:354-383
    if (!input || !output || !output_len) return Z_STREAM_ERROR;
    if (level < 0 || level > 9) level = Z_DEFAULT_COMPRESSION;
    size_t cap = *output_len;
    int st = 0;
    int rc = zgpu_compress_batch(&input, &input_len, &output, &cap, &st, 1, level, ZGPU_WRAP_RAW);
    if (rc) return rc == ZGPU_ENODEV ? Z_MEM_ERROR : rc;
    if (st) return st;      // Z_BUF_ERROR (documented deviation: the reference returns Z_OK)
    *output_len = cap;
    return Z_OK;
}
int zlib_compress_simd(const uint8_t *input, size_t input_len, uint8_t *output, size_t *output_len,
                       int level) {                                   // src/zlib_simd_compression.c:280
    return zlib_compress_simd_full(input, input_len, output, output_len, level);
}
uint32_t zlib_crc32_simd_enhanced(uint32_t crc, const uint8_t *data, size_t len) {
    return (uint32_t)crc32_z(crc, data, len);                         // src/zlib_simd_optimized.c:387
}
uint32_t zlib_crc32_simd_optimized(uint32_t crc, const uint8_t *data, size_t len) {
    return (uint32_t)crc32_z(crc, data, len);                         // src/zlib_simd_compression.c:342
}
uint32_t zlib_adler32_simd(uint32_t adler, const uint8_t *buf, size_t len) {
    return (uint32_t)adler32_z(adler, buf, len);   // zlib-correct, unlike src/zlib_simd_optimized.c:116
}
int zlib_compress_simd_buffer(const uint8_t *src, size_t src_len, uint8_t *dest, size_t *dest_len,
                              int level) {                            // src/wasm_module_side.c:61-70
    if (src_len >= 8192) return zlib_compress_simd(src, src_len, dest, dest_len, level);
    unsigned long dl = *dest_len;
    int rc = compress2(dest, &dl, src, src_len, level);
    *dest_len = dl;
    return rc;
}

// ---- src/zlib_simd_optimized.c kernels without a caller, zlib-
// correct, on the GPU: the caller's host arrays are staged, the kernel runs,
// the results come back.  With no GPU they leave their outputs unchanged (and
// return 0) after libzgpu's one-time diagnostic.
void zlib_slide_hash_simd(uint16_t *hash_table, uint16_t *prev_table, uint32_t hash_size,
                          uint32_t window_size, uint16_t wsize) {    // src/zlib_simd_optimized.c:27
    if ((!hash_table && hash_size) || (!prev_table && window_size)) return;
    Lease L;
    if (L.rc) return;
    Ctx &c = *L.c;
    const size_t hb = 2ull * hash_size, pb = 2ull * window_size;
    if (!c.ws_help.ensure(hb + pb + 64)) return;
    uint16_t *dh = c.ws_help.as<uint16_t>(), *dp = dh + hash_size;
    if ((hb && hipMemcpy(dh, hash_table, hb, hipMemcpyHostToDevice) != hipSuccess) ||
        (pb && hipMemcpy(dp, prev_table, pb, hipMemcpyHostToDevice) != hipSuccess) ||
        launch_slide_hash(dh, dp, hash_size, window_size, wsize, nullptr) ||
        (hb && hipMemcpy(hash_table, dh, hb, hipMemcpyDeviceToHost) != hipSuccess) ||
        (pb && hipMemcpy(prev_table, dp, pb, hipMemcpyDeviceToHost) != hipSuccess))
        std::fprintf(stderr, "libzgpu: zlib_slide_hash_simd failed\n");
}
uint32_t zlib_compare256_simd(const uint8_t *src0, const uint8_t *src1) {   // src/zlib_simd_optimized.c:74
    if (!src0 || !src1) return 0;
    Lease L;
    if (L.rc || !L.c->ws_help.ensure(512 + 64)) return 0;
    Ctx &c = *L.c;
    uint8_t *d = c.ws_help.as<uint8_t>();
    uint32_t *dr = reinterpret_cast<uint32_t *>(d + 512), r = 0;
    if (hipMemcpy(d, src0, 256, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + 256, src1, 256, hipMemcpyHostToDevice) != hipSuccess ||
        launch_compare256(d, d + 256, dr, nullptr) ||
        hipMemcpy(&r, dr, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    return r;
}
uint32_t zlib_longest_match_simd(const uint8_t *window, uint32_t strstart, uint32_t prev_length,
                                 uint32_t good_match, uint32_t max_chain_length, uint32_t lookahead,
                                 const uint16_t *prev_table, uint32_t wmask,
                                 uint32_t *match_start) {            // src/zlib_simd_optimized.c:210
    // zlib's window is 2 * wsize bytes and prev[] wsize entries (wsize = wmask + 1,
    // a power of two); strstart <= 2 * wsize - MIN_LOOKAHEAD as deflate keeps it
    const uint64_t wsize = (uint64_t)wmask + 1;
    if (!window || !prev_table || !match_start || (wsize & wmask) || wsize < 512 || wsize > 32768 ||
        prev_length < 2 || prev_length > (uint32_t)kMaxMatch ||
        (uint64_t)strstart + kMinLookahead > 2 * wsize || lookahead > 2 * wsize - strstart)
        return prev_length;
    Lease L;
    if (L.rc || !L.c->ws_help.ensure(2 * wsize + 2 * wsize + 64)) return prev_length;
    Ctx &c = *L.c;
    uint8_t *dw = c.ws_help.as<uint8_t>();
    uint16_t *dp = reinterpret_cast<uint16_t *>(dw + 2 * wsize);
    uint32_t *dr = reinterpret_cast<uint32_t *>(dw + 4 * wsize), r[3] = {prev_length, 0, 0};
    if (hipMemcpy(dw, window, 2 * wsize, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dp, prev_table, 2 * wsize, hipMemcpyHostToDevice) != hipSuccess ||
        launch_longest_match(dw, strstart, prev_length, good_match, max_chain_length, lookahead, dp, wmask, dr,
                             nullptr) ||
        hipMemcpy(r, dr, sizeof r, hipMemcpyDeviceToHost) != hipSuccess)
        return prev_length;
    if (r[2]) *match_start = r[1];
    return r[0];
}
void zlib_chunkmemset_simd(uint8_t *dest, uint8_t *src, uint32_t dist,
                           uint32_t len) {                           // src/zlib_simd_optimized.c:296
    if (!dest || !src || dist == 0 || len == 0) return;
    const uint32_t sn = dist < len ? dist : len;
    Lease L;
    if (L.rc || !L.c->ws_help.ensure((size_t)sn + len + 64)) return;
    Ctx &c = *L.c;
    uint8_t *ds = c.ws_help.as<uint8_t>(), *dd = ds + ((sn + 15) & ~15u);
    if (hipMemcpy(ds, src, sn, hipMemcpyHostToDevice) != hipSuccess ||
        launch_chunkmemset(dd, ds, dist, len, nullptr) ||
        hipMemcpy(dest, dd, len, hipMemcpyDeviceToHost) != hipSuccess)
        std::fprintf(stderr, "libzgpu: zlib_chunkmemset_simd failed\n");
}

}  // extern "C"
