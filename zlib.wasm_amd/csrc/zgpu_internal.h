// zgpu_internal.h — constants, tables and launch entry points shared by the
// HIP translation units of libzgpu.so.  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace zgpu {

// ---- deflate constants (zutil.h:77-89, deflate.h:33-55,293-303) ----
constexpr int kWSize = 32768;
constexpr int kMinMatch = 3;
constexpr int kMaxMatch = 258;
constexpr int kMinLookahead = kMaxMatch + kMinMatch + 1;   // 262
constexpr int kMaxDist = kWSize - kMinLookahead;            // 32506
constexpr int kTooFar = 4096;                               // deflate.c:88-90
constexpr int kSymLimit = 16383;                            // lit_bufsize - 1
// k_match's tile: positions walked per LDS window load.  A segmented k_match
// (few large buffers) must start every segment on a tile boundary, so the
// host's segment sizes are whole multiples of it.
constexpr uint32_t kMatchTile = 4096;
// k_lzp (match + lazy parse in one kernel) serves batch jobs whose chain budget is at most this (levels 4..7)
constexpr uint32_t kLzpMaxChain = 256;
// k_links keeps head[] in the key[] region (32 Ki x 4 B) for buffers this long
constexpr uint64_t kLinksGhMin = 131072;
// Buffers are addressed with 32-bit positions inside the kernels: deflate
// refuses buffers of kMaxBuffer bytes or more (Z_STREAM_ERROR / Z_MEM_ERROR).
constexpr uint64_t kMaxBuffer = (1ull << 32) - (1ull << 16);
constexpr int kLCodes = 286, kDCodes = 30, kBLCodes = 19;
constexpr int kHeapSize = 2 * kLCodes + 1;                  // 573
constexpr int kMaxBits = 15, kMaxBLBits = 7;
constexpr int kEndBlock = 256;

// configuration_table (deflate.c:112-125)
// configuration_table (deflate.c:112-125) or deflateTune's values
// (deflate.c:805-820); chain 0xffffffff: no budget (deflateTune's 0, which
// longest_match's unsigned count never reaches again)
struct LevelCfg { uint32_t good, lazy, nice, chain; };

// Static code tables (RFC 1951 §3.2.5-3.2.6), derived on the host at init the
// way tr_static_init (trees.c:303-396) derives them, copied to __constant__.
struct CodeTables {
    uint8_t  len_code[256];     // normalized match length -> length code 0..28
    uint8_t  dist_code[512];    // d<256: [d]; else [256 + (d>>7)]
    uint16_t len_base[29];
    uint16_t dist_base[30];
    uint8_t  xlbits[29];
    uint8_t  xdbits[30];
    uint8_t  xblbits[19];
    uint8_t  bl_order[19];
    uint16_t stat_lcode[288];
    uint8_t  stat_llen[288];
    uint16_t stat_dcode[30];
    uint8_t  stat_dlen[30];     // all 5 (static_dtree, trees.c:292)
    LevelCfg cfg[10];
};

// CRC-32 tables (reflected poly 0xedb88320, crc32.c), built on the host:
//   nib[j][v]  raw CRC (zero init, no final xor) of a 16-byte chunk whose
//              nibble j (byte j/2, low nibble first) is v, all else zero;
//   shift[k][j][v] advance-by-zero-bytes operators as 8 nibble tables:
//              k = 0..5 -> 16<<k bytes, k = 6 -> 1024 bytes,
//              k = 7 -> kCrcSegment bytes (segment Horner);
//   byte[v]    the classic byte table (tiny-buffer path).
constexpr int kCrcShiftTabs = 8;
//   s4[k][v]   slice-by-4 tables: s4[0] = byte, s4[k][v] = s4[k-1][v] advanced
//              by one zero byte;
//   sh64[k][j][v] nibble operators advancing by {64,128,...,2048, 960, 4032}
//              bytes (k_crc32s: the gaps between a lane's chunks and the
//              lane-combine tree).
constexpr int kCrcSh64Tabs = 8;
struct CrcTables {
    uint32_t nib[32][16];
    uint32_t shift[kCrcShiftTabs][8][16];
    uint32_t byte[256];
    uint32_t s4[4][256];
    uint32_t sh64[kCrcSh64Tabs][8][16];
    uint32_t xrow[48];        // x^(8 kCrcRow 2^i) mod P: k_crc32_fin's shifts over whole rows
};
constexpr uint64_t kCrcRow = 64 * 64;           // k_crc32_part's row: 64 lanes x 64 bytes
constexpr uint64_t kCrcSegment = 64 * 1024;   // bytes per checksum work item

// Per-buffer deflate block record written by the parse, read by the encoder.
struct BlockRec {
    uint32_t sym_start;   // index of first symbol (relative to buffer's sym base)
    uint32_t nsym;
    uint64_t in_start;    // block_start (absolute input position)
    uint64_t in_end;      // strstart at flush
    uint32_t flags;       // kBlk* below
    uint32_t pad;
};
constexpr uint32_t kBlkLast = 1u;     // BFINAL
constexpr uint32_t kBlkStored = 2u;   // stored-eligible (block_start still in the window)
// A marker record is no block: it stands for the bits a deflate(flush) call
// appends after its blocks (deflate.c:1211-1233), its kind in bits 4..6:
// Z_PARTIAL_FLUSH 1 (_tr_align), Z_SYNC_FLUSH 2 / Z_FULL_FLUSH 3 (an empty
// stored block), Z_BLOCK 5 (nothing).
constexpr uint32_t kBlkMarker = 8u;
constexpr uint32_t kEvPause = 8u;      // DeflateJob::fl_aux
// a deflatePrime call with input pending (deflate.c:731-757): an event at the
// stop of the deflate() call before it, fl_aux = value | bits << 16; the parse
// writes a marker of kind kMarkPrime there (its bits in BlockRec::pad), which
// k_encode turns into the bits, ahead of the block in progress
constexpr uint32_t kEvPrime = 16u;
constexpr uint32_t kMarkPrime = 6u;
__host__ __device__ constexpr uint32_t blk_marker_kind(uint32_t flags) { return (flags >> 4) & 7u; }

// k_pbig1..6 (a sub-batch of few large buffers): the segmented lazy parse's
// per-lane state between its kernels, and per buffer
struct PLane {
    uint32_t e_p, e_ml, e_ms, e_av;   // where pass 1 stopped (position, match length/start, literal pending)
    uint32_t k1;                      // pass-1 symbols staged
    uint32_t y, sig;                  // pass 2: where the parse meets the next lane's (~0: the end), pending literal
    uint32_t kstart, rcnt, cnt, base; // pass-1 symbols before y(i-1), run-on symbols, the lane's count, first index
    uint32_t p0;                      // first input position the lane's symbols cover (k_pbig5)
};
constexpr uint32_t kRonCap = 64;      // run-on symbols per lane when preach > 1
// sub-batches of small buffers (zgpu_api.cpp): 256-byte segments whose run-ons may cross 8 segments;
// k_pbig1s stages 64 such segments in LDS
constexpr uint32_t kSmallSeg = 256, kSmallReach = 8;
struct PBuf { uint32_t fail, first_end, fin, total; };
constexpr uint32_t kParseLanesHost = 256;   // lanes (segments) per k_pbig* / k_parse_seg workgroup

// k_enc_plan -> k_enc_scan -> k_enc_emit (few large buffers): one block's
// header fields and code tables, and where its bits start
struct EncPlan {
    uint16_t lcode[kLCodes], dcode[kDCodes], bcode[kBLCodes];
    uint8_t llen[kLCodes], dlen[kDCodes], blen[kBLCodes];
    uint8_t type, pad0;
    uint16_t lmax, dmax, blmax;
    uint64_t bits;           // static / dynamic: the block's bits from its 3-bit header through END_BLOCK
    uint64_t start;          // the output bit where the block's header starts; [nblocks]: the stream's end
};

// k_links for a streaming job whose window holds deflate_huff / deflate_rle
// stretches (zgpu_api.cpp internal_state::hr): positions [a[k], b[k]) are not
// inserted (no link, head[] untouched).  Buffer-relative.
constexpr int kMaxSkip = 8;
struct SkipSpec {
    uint32_t n;
    uint32_t a[kMaxSkip], b[kMaxSkip];
};

// Per-buffer workspace layout for one deflate sub-batch (device arrays).
struct DeflateJob {
    const uint8_t *src;      // batch input base
    const uint64_t *src_off;
    const uint64_t *src_len;
    uint8_t *dst;
    const uint64_t *dst_off;
    const uint64_t *dst_cap;
    uint64_t *dst_len;
    int32_t *status;
    uint32_t first;          // first buffer index of this sub-batch
    uint32_t count;          // buffers in this sub-batch
    int level, wrap;
    int strategy;            // deflateInit2_ strategy: 0 default, 1 filtered, 2 huffman only, 3 rle, 4 fixed
    // workspace, indexed by position relative to ws_off[i]
    const uint64_t *ws_off;  // per sub-batch buffer: start in the position-indexed arrays
    const uint64_t *blk_off; // per sub-batch buffer: start in the block array
    uint16_t *link;          // [Σn]
    uint8_t *key;            // [Σn] k_count's walk-length keys (k_match's position order)
    uint32_t *rfull;         // [Σn]
    uint32_t *rquart;        // [Σn] (levels 5..9)
    uint32_t *pstate;        // [Σn/16] lazy-parse sync states, 2 bits per position
    uint32_t *sym;           // [Σn]
    uint32_t *stage;         // [Σn] k_parse_seg's pass-1 symbol staging (levels 4..9)
    BlockRec *blocks;        // [Σ(n/16383 + 2)]
    uint32_t *nblocks;       // [count]
    uint32_t *check;         // [count] adler32 / crc32 of the input (trailer)
    uint8_t *wind;           // [count] or null: bi_used at the stream's last bi_windup (deflateUsed)
    // deflate(flush) calls of a streaming job (count == 1, zgpu_api.cpp deflate()):
    // the input position where each flush call ended (ascending) and its kind
    // (Z_PARTIAL_FLUSH 1, Z_SYNC_FLUSH 2, Z_FULL_FLUSH 3 -- only as the job's
    // last event --, Z_BLOCK 5); open_end: the stream goes on after the last
    // flush (no final block, complete bytes only).  nfl == 0 for batch jobs.
    const uint64_t *fl_pos;
    const uint32_t *fl_type;
    uint32_t nfl;
    int open_end;
    // a resumed flush job (zgpu_api.cpp deflate_part): the buffer starts at the
    // window offset S of the last flush acted on, the parse at that flush
    // (`start`), and the output at bit `bit0` of a byte whose low bits are byte0
    uint32_t start, bit0, byte0;
    // flush jobs' results or null: [0] output bits before the last marker,
    // [1] output bits at the end, [2] the window offset S at the last flush
    // (buffer-relative), [3] the last, partial output byte
    uint64_t *flush_out;
    int plan;                // level 0 streaming: the block records were made on the host (stored blocks)
    // k_match over segments (a sub-batch of few large buffers): nseg pairs
    // (buffer, start) of seg_len-byte segments, one workgroup each; null: one
    // workgroup per buffer
    const uint32_t *seg;
    uint32_t nseg, seg_len;
    // every buffer of the sub-batch is under 2^31 bytes: k_parse_fast runs on
    // 32-bit positions
    int pos31;
    // every buffer of the sub-batch has >= kLinksGhMin bytes: k_links keeps its
    // head[] table (32-bit positions) in the buffer's key[] region, which
    // k_count overwrites after it, instead of in LDS (two workgroups per CU)
    int links_gh;
    // deflateInit2_'s windowBits (9..15; 8 is stored as 9, deflate.c:395) and
    // memLevel + 7 = hash_bits (8..16): w_size = 1 << wbits, MAX_DIST = w_size
    // - 262, hash_shift = (hash_bits + 2) / 3, lit_bufsize = 1 << (memLevel + 6)
    // and the block cut at lit_bufsize - 1 symbols (deflate.c:440-455)
    int wbits, hbits;
    // good_match, max_lazy_match, nice_match, max_chain_length of the job
    // (the level's configuration_table row, or deflateTune's)
    LevelCfg cfg;
    // deflateSetDictionary (levels 1..3): the buffer starts with the
    // dictionary, the parse at `start`; the hash chains start empty and
    // positions [0, pre_ins) are inserted first (deflate.c deflateSetDictionary
    // inserts all but the last two, which wait as s->insert)
    int dict;
    uint32_t pre_ins;
    // Z_NO_FLUSH calls of a streaming job: an event of kind 0 is the end of
    // such a call's input.  The parse stops there once the lookahead is below
    // MIN_LOOKAHEAD (deflate_slow, deflate_fast), at most MAX_MATCH
    // (deflate_rle) or 0 (deflate_huff) with that input used up -- need_more
    // (deflate.c:1941-1944, :1841-1844, :2065-2068, :2129-2134) -- and goes on
    // with the next call's input.  Only events of other kinds clamp k_match
    // (mlim: their positions), since a position decided before a need_more
    // return has MIN_LOOKAHEAD bytes after it.
    const uint64_t *mlim;
    uint32_t nmlim;
    // an event of kind kEvPause: the call before stopped on a full output
    // buffer right after the block that ends at fl_aux[i], and the next call
    // offered more input: from there on fill_window reads up to the next
    // event's end instead of stopping at this one's (fl_pos[i])
    const uint64_t *fl_aux;
    // per block / marker record j of a streaming job (or null): srec[4j] the
    // output bit after it and srec[4j + 1] the partial byte there (k_encode),
    // srec[4j + 2] = S << 32 | in_end and srec[4j + 3] = E | resumable << 63 as
    // the parse flushed it (window offset, fill_window's end of input read,
    // whether the lazy state there is the simple one a new job starts in)
    uint64_t *srec;
    uint32_t *ev_blk;        // per event: the records before it when it was acted on
    uint32_t e0;             // a job resumed at a block cut: E there (0: the start, nothing read ahead)
    int cut;                 // resumed at a block cut, not after a flush (no s->insert strings)
    uint32_t *snap;          // levels 1..3: head[] at the last cut; snap[hash_size] = its record
    // configuration changes of a streaming job (deflateParams within the same
    // function, deflateTune, with input pending: deflate.c:760-820): cfg_tab[k]
    // applies to the decision points at or after cfg_pos[k] (ascending,
    // buffer-relative); before cfg_pos[0], `cfg`.  Each decision reads its
    // row when it is made (deflate_slow / deflate_fast / longest_match read
    // max_lazy, good, nice and chain from the state each time).
    const uint64_t *cfg_pos;
    const LevelCfg *cfg_tab;
    uint32_t ncfg;
    int cfg_q;               // some row of cfg_tab has good < lazy: k_match computes rquart
    // a streaming job whose window was (partly) parsed by deflate_fast, which
    // inserts selectively (deflate.c:1873-1897), while this job's function
    // inserts every position (deflateParams switched it after a Z_BLOCK flush):
    //  k_links: positions [0, lk_n) keep the links already in `link` (the
    //           deflate_fast chains, uploaded), the chunk holding lk_n starts
    //           from lk_head[hash] (buffer positions, 0 none) instead of empty;
    //  k_parse_fast (keep_head): head[] and prev[] as uploaded, then positions
    //           [pre_from, pre_ins) inserted in order before the parse starts
    uint32_t lk_n;
    const uint32_t *lk_head;
    uint32_t pre_from;
    int keep_head;
    // deflate_state's prev_length / match_length where the job starts (a
    // function switch carries them over: deflate_fast never writes
    // prev_length and both parsers leave 0 behind a match, so the first
    // searches after a switch may start from best_len 0, whose quick reject
    // also tests the byte before the string, deflate.c:1356-1497).  zp0: the
    // prev_length every deflate_fast search starts from; zm0: deflate_slow's
    // match_length before its first decision.  2 (MIN_MATCH-1) is the clean
    // state.  A streaming job reports both as the parse leaves them in
    // flush_out[4] (prev_length | match_length << 16).
    int zp0, zm0;
    // a batch sub-batch of few large buffers (levels 4..9, job.seg set):
    // the lazy parse and the encoder spread each buffer over many workgroups
    // (k_pbig*, k_enc_plan/scan/emit).  pgrp: npgrp pairs (buffer, first lane)
    // of kParseLanes lanes, one workgroup each; a buffer has ceil(n / pseg)
    // lanes, its lane 0 is plane[plbase[buffer]]; maxblk: the most block
    // records a buffer may have
    const uint32_t *pgrp;
    uint32_t npgrp, pseg, maxblk;
    // preach: segments a lane's run-on may cross before it must meet a later
    // lane's pass 1 (1: the next one).  Above 1 only when every buffer has at
    // most kParseLanes lanes (one workgroup each), which k_pbig3 then joins
    // along the chain of meets; run-on symbols go to pron (kRonCap per lane)
    uint32_t preach;
    uint32_t *pron;
    const uint32_t *plbase;
    PLane *plane;
    PBuf *pbuf;
    EncPlan *eplan;
    // a streaming job parsed by k_pbig1..5 (Z_NO_FLUSH stops only, see
    // k_pbig6s): workspace for fill_window's timeline, ntl entries of 4 words
    // (first decision point, S, E, -) and then one trigger point per event
    uint32_t *tl;
    uint32_t ntl;
    int fcmp;                // k_parse_fast: load 64 candidate bytes per chain step (A/B; 0: 16 first)
    SkipSpec sk;             // k_links: huff/rle stretches of a streaming job (n = 0: none)
    // The sorted-run longest_match (k_bsort / k_bwork / k_match2, batch jobs at
    // levels 4..9, hash_bits <= 15).  Each buffer is cut into blocks of
    // kSortBlock positions; bblk[i] is buffer i's first block in the
    // sub-batch's flat block numbering (count + 1 entries).
    //  srt  [Σn] u16, position-indexed: block b's inserted positions (p <=
    //       n-3), block-relative, sorted by (hash, position): the candidates of
    //       a position in its block are the entries just before its own
    //       within its hash's run;
    //  boff [blocks * kSortOffStride] u16: per block, off[h] = the entries
    //       with a hash below h (h = 0 .. hash_size), i.e. hash h's run;
    //  work [Σn] uint4, position-indexed: per block, one work item per
    //       sorted entry (its index, position, and its hash's runs in the
    //       block and the two before it), each 4096-entry slice ordered by
    //       candidate count so that walks of similar length share a wave.
    const uint32_t *bblk;
    uint32_t nsblk;          // blocks in the sub-batch (k_bsort / k_bwork grid)
    uint16_t *srt;
    uint16_t *boff;
    uint4 *work;
    int lzp_flags;           // k_lzp A/B switches (ZGPU_LZP_FLAGS): bit 0 the parser wave at raised priority
};
// k_bsort's block (positions) and the stride of its per-block hash table
constexpr int kSortBlock = 16384;
constexpr int kSortOffStride = 32776;          // >= 32768 + 1, a multiple of 8

// the per-job window/hash parameters (deflate.c:440-455)
struct WinP {
    int64_t wsize, max_dist;
    uint32_t shift, mask, sym_limit;
};
__host__ __device__ inline WinP win_params(int wbits, int hbits) {
    WinP w;
    w.wsize = (int64_t)1 << wbits;
    w.max_dist = w.wsize - kMinLookahead;
    w.shift = (uint32_t)(hbits + kMinMatch - 1) / kMinMatch;
    w.mask = (1u << hbits) - 1u;
    w.sym_limit = (1u << (hbits - 7 + 6)) - 1u;
    return w;
}

// ---- inflate ----
// where k_inflate_decode stopped (zo_inflate_run's codes)
// (kIBlock: inflate(Z_BLOCK)'s stop at a block boundary, InflateJob::stop_mode)
enum InflateStop : uint32_t { kIEnd = 0, kIData = 1, kIDict = 2, kIFull = 3, kIInEnd = 4, kIBlock = 5, kITrees = 6 };

struct InflateRec {          // per stream, written by k_inflate_decode
    uint64_t put;            // output bytes produced
    uint64_t used;           // input bytes consumed at the stop (check passed)
    uint64_t used_bad;       // consumed when the trailer check fails
    uint32_t stop;           // InflateStop; kIEnd may still fail its check
    uint32_t nmatch;         // match records for k_inflate_copy
    uint32_t chk_kind;       // 0 none, 1 Adler-32 (zlib), 2 CRC-32 (gzip)
    uint32_t chk_want;       // trailer value
    uint32_t isize;          // gzip ISIZE: 0 n/a, 1 equal, 2 differs, 3 input ended
    uint32_t pbyte;          // probe mode (capacity 0): the byte produced, if any
};

struct InflateJob {
    const uint8_t *src;
    const uint64_t *src_off;
    const uint64_t *src_len;
    uint8_t *dst;
    const uint64_t *dst_off;
    const uint64_t *dst_cap;
    uint64_t *dst_len;
    uint64_t *src_used;      // may be null
    int32_t *status;
    uint32_t *stop_out;      // may be null: InflateStop after the checks
    uint32_t first, count;
    int wrap;                // 0 raw, 1 zlib, 2 gzip, 3 zlib or gzip
    int wbits;               // inflateInit2_ window bits (8..15; 0: the header's)
    const uint64_t *mrec_off;   // per sub-batch stream: first match record
    uint64_t *mrec;          // match records: pos | len << 32 | dist << 41
    InflateRec *rec;         // [count]
    uint32_t *adler, *crc;   // [count] checks of the produced output
    const uint32_t *crc_byte;   // CRC-32 byte table (device)
    // resuming a stream at a block boundary (the streaming inflate()), all
    // optional: res_bit[g] = bit position of a block header in the stream's
    // input (the job is then raw: no header, no trailer); res_hist[g] = bytes
    // of earlier output already at dst (<= 32 KiB, the window), decoding
    // appends after them; blk_out[2g], [2g+1] = bit position and output
    // position of the last block boundary the decode reached (0, 0: none)
    const uint64_t *res_bit;
    const uint32_t *res_hist;
    uint64_t *blk_out;
    // inflate(Z_BLOCK) (inflate.c TYPE: "if (flush == Z_BLOCK) goto inf_leave"):
    // bit 0 stop right after a zlib / gzip header, bit 1 at the end of the
    // first block that is not the last; the stop (kIBlock) is the boundary in
    // blk_out.  bit 3 (inflate(Z_TREES), inflate.c STORED / TABLE .. LEN_):
    // stop after the first block header that ends past trees_after, before its
    // first code (kITrees, the header's end in blk_out)
    uint32_t stop_mode;
    // the state inflate.c would report in strm->data_type where the decode
    // stopped (or null): input bits it would hold (inbits - the bit after the
    // last symbol part decoded) | BFINAL of the current block << 32 | waiting
    // at a block header (mode TYPE) << 33.  stop_mode bit 2: the decode starts
    // in mode TYPE (resumed at a boundary), not TYPEDO / HEAD
    uint64_t *zstate_out;
    // [2g + 1] of zstate_out: inflateMark's value where the input ran out (low 32 bits, signed) and
    // inflateCodesUsed of the last dynamic block (high 32 bits; ~0: none in this decode), computed
    // only when zcodes is set
    int zcodes;
    uint32_t dmax;           // inflateBack: distances beyond its window (1 << windowBits) are errors; 0: none
    // stop_mode bit 3: only a header that ends past this input bit (where the
    // reference stands: a header it has begun but not finished, or one after it)
    uint64_t trees_after;
    // count only (the block-parallel decode's dry run): no output, no match
    // records, no capacity limit; dst_len / rec / blk_out report where the
    // decode ended and how much it would have produced
    int count_only;
    // the streaming inflate()'s consumption index (one-stream jobs; null: off): per symbol that
    // writes output, eidx[2k] = its output end (low 32 bits) | stored run << 32 | BFINAL of its
    // block << 33, eidx[2k + 1] = the input bit position once its codes are read (a stored run:
    // its first input byte).  bidx[2k], [2k + 1] = bit and output position of each block's
    // end (the last block's: bit | 1 << 63).  icnt[0], [1] = entries / ends met (may exceed
    // ecap / bcap)
    uint64_t *eidx, *bidx;
    uint32_t *icnt;
    uint32_t ecap, bcap;
};
int launch_inflate_stage(int stage, const InflateJob &job, hipStream_t st);
// the block-parallel decode of a lone stream (zgpu_inflate.hip, zgpu_api.cpp inflate_par)
struct ParBlkHost { uint64_t o0, o1, base, moff, lit; uint32_t nm, pad; };   // = zgpu_inflate.hip ParBlk
int launch_infl_scan1(const uint8_t *in, uint64_t n, uint64_t b0, uint64_t b1, uint64_t *list, uint32_t cap,
                      uint32_t *cnt, hipStream_t st);
int launch_infl_scan2(const uint8_t *in, uint64_t n, const uint64_t *list, uint32_t count, uint64_t *out,
                      uint32_t cap, uint32_t *cnt, hipStream_t st);
int launch_infl_sym(uint8_t *out, const uint8_t *slots, uint32_t *sym, const void *blks, uint32_t nblk,
                    const uint64_t *mrec_slots, const uint64_t *mrec_inplace, uint32_t *err, hipStream_t st);
int launch_infl_resolve(uint8_t *out, const uint32_t *sym, uint64_t o0, uint64_t o1, hipStream_t st);

// launchers (return hipError_t as int)
int launch_tables_upload(const CodeTables *ct, const CrcTables *crc);
const CrcTables *device_crc_tables();
int launch_crc32(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                 const uint32_t *init, uint32_t *out, uint32_t count,
                 void *scratch, size_t scratch_bytes, hipStream_t st);
int launch_adler32(const uint8_t *src, const uint64_t *off, const uint64_t *len,
                   const uint32_t *init, uint32_t *out, uint32_t count,
                   void *scratch, size_t scratch_bytes, hipStream_t st);
size_t checksum_scratch_bytes(uint32_t count);
// stage: 0 links, 1 match, 2 lazy parse (sequential), 3 greedy parse (heads: 128 KiB/buffer),
//        4 encode, 5 lazy parse (segmented), 6 lazy parse fallback for buffers flagged by 5,
//        7 huffman-only parse, 8 rle parse, 9 walk-length keys (k_count),
//        10 huffman-only / rle parse of a flush job (sequential),
//        11 lazy parse of few large buffers (k_pbig*; 6 handles its fallbacks),
//        12 encode of few large buffers (k_enc_plan, k_enc_scan, k_enc_emit)
int launch_deflate_stage(int stage, const DeflateJob &job, uint32_t *heads, hipStream_t st);
// k_parse_seg's fallback counters (zgpu_debug_parse_fallbacks): out[0..1]
int parse_fallback_counts(uint64_t *out);
// 1 when k_lzp is compiled in (the A/B build, -DZGPU_LZP)
int lzp_built();
// a18 helpers (zgpu_helpers.hip)
int launch_slide_hash(uint16_t *head, uint16_t *prev, uint32_t hash_size, uint32_t window_size, uint32_t wsize,
                      hipStream_t st);
int launch_compare256(const uint8_t *a, const uint8_t *b, uint32_t *out, hipStream_t st);
int launch_longest_match(const uint8_t *window, uint32_t strstart, uint32_t prev_length, uint32_t good,
                         uint32_t chain, uint32_t lookahead, const uint16_t *prev, uint32_t wmask, uint32_t *out,
                         hipStream_t st);
int launch_chunkmemset(uint8_t *dest, const uint8_t *src, uint32_t dist, uint32_t len, hipStream_t st);
int launch_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed,
                    uint64_t first_index, hipStream_t st);

}  // namespace zgpu
