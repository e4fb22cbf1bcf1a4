// Internal definitions shared by the host orchestration and the gfx950 kernels.
#pragma once
#include <stdint.h>

namespace mm2g {

constexpr uint64_t U64MAX = ~0ULL;
constexpr int WAVE = 64;
// chain DP segment classes (DESIGN.md "Chain DP"): <= CHAIN_TINY anchors one
// lane in registers, <= CHAIN_MED one lane (state machine), longer one wave
constexpr int CHAIN_TINY = 8;
constexpr int CHAIN_MED = 128;

// Anchor key packing (DESIGN.md "Anchor key").  The reference anchor is
// (x, y) = (rev<<63 | rid<<32 | rpos, span<<32 | qpos) sorted by (x, y)
// (src/seeds.rs:58,73-76).  For queries span == k for every minimizer, so the
// order of (x, y) equals the order of
//      key = group << (RB+QB) | p << QB | q
// with group = rid (forward), n_seq + rid (reverse), 2*n_seq for the Q19
// pseudo-group (odd rid: rpos bit 31 set and `rpos as u64` sign-extended,
// so x = 0xffffffff_8xxxxxxx for both strands), p = rpos & 0x7fffffff.
struct KeyLayout {
    uint32_t qb, rb, gb;   // bit widths
    uint32_t n_seq;
};

// Per-read device outputs of the chain kernels (mirrors mm2g_read_result).
struct ReadOut {
    int32_t flags;
    int32_t n_anchors;
    int32_t score;
    int32_t cm;
    int32_t qs, qe, ts, te;
    int32_t group;
    int32_t best_i;
    int32_t n_match;
    int32_t dv_st, dv_en;
    int32_t m_dv;
    int32_t qlen;
    int32_t m_kept;        // minimizers kept by the query filter
    uint64_t dp_pairs;     // inner-loop j evaluations (all passes)
    // chain-kernel statistics (mm2g_debug_chain_stats): wall-clock ticks
    // (100 MHz) of pass 0 / pass 1, non-isolated anchors, j-steps, HBM j-steps
    uint32_t t_pass[2];
    uint32_t n_noniso, n_steps, n_deep;
    uint32_t pad2;
};
static_assert(sizeof(ReadOut) == 96, "ReadOut layout");

enum : int32_t {
    RF_MAPPED = 1, RF_RESCUED = 2, RF_DV_FOUND = 4, RF_PANIC = 8, RF_EMPTY = 16,
};

struct ChainKParams {
    int32_t max_dist_x, max_dist_y, bw, max_iter, max_skip, span;
    int32_t rescue_size;
    float rescue_ratio_f;   // (1.0f - rmq_rescue_ratio), computed on the host in f32
    int32_t pass;           // 0 = first DP, 1 = rescue DP (only RF_RESCUED reads)
    int32_t lut_n;          // entries in the pen LUT (bw + 1)
    int32_t multi;          // -n <= 1, -m <= k: chains[0] is one anchor, the rescue test sees coverage = span
};

// Device index layout: open-addressed table of distinct minimizer hashes.
// A Single (one occurrence) keeps its position in the entry itself, so the
// anchor pass needs no gather for it: n = IX_INLINE | (pos >> 32), off = the
// low 32 bits of pos (pos = rid<<32 | rpos<<1 | strand, Index p/h values).
struct IxEntry {
    uint64_t key;   // minimizer hash (key_span >> 8); U64MAX = empty
    uint32_t off;   // first position in ix_pos (Multi), low word of the position (Single)
    uint32_t n;     // occurrences (Multi), IX_INLINE | high word of the position (Single)
};
constexpr uint32_t IX_INLINE = 0x80000000u;
__host__ __device__ inline uint32_t ix_count(uint32_t n) { return (n & IX_INLINE) ? 1u : n; }

__host__ __device__ inline uint32_t ix_slot(uint64_t h, uint32_t log2cap) {
    return (uint32_t)((h * 0x9E3779B97F4A7C15ULL) >> (64 - log2cap));
}


// ---- kernel arguments (mm2g_kernels.hip) --------------------------------
// Batch status word (u32 at the start of the context's status block, copied
// back with the results): a workspace that was too small for this batch.  The
// host grows it and maps the batch again (mm2g_batch_results).
enum : uint32_t { BS_SKETCH = 1, BS_TAB = 2, BS_ANCHORS = 4, BS_SKETCH_DV = 8 };
struct SketchArgs {
    const uint8_t* seq;
    const uint64_t* rd_off;     // n+1 offsets into seq
    uint32_t n;
    int w, k;
    const uint64_t* out_base;   // per sequence: first output slot
    const uint64_t* out_end;    // per sequence: one past the last slot (capacity)
    uint64_t* mz_x;             // key_span = hash<<8 | span
    uint32_t* mz_y;             // i<<1 | z   (rid is implicit / added by caller)
    uint32_t* mz_cnt;           // per sequence
    int32_t* overflow;
    uint64_t* prof;             // MM2G_SKETCH_PROF: per sequence 8 phase-time sums (else null)
    // Index build (mm2g_ixbuild.hip): sequence r is a view [view_off, +view_len)
    // into a contig with view_pre bases of that contig before it; steps before
    // emit_from are warm-up (no emissions); view_last = the view ends its contig
    // (final flush, sketch.rs:99).  Null view_off: sequences are rd_off ranges.
    const uint64_t* view_off = nullptr;
    const uint32_t* view_len = nullptr;
    const uint32_t* view_pre = nullptr;
    const uint32_t* emit_from = nullptr;
    const uint8_t* view_last = nullptr;
    // HPC index build (flag & 1): per base of seq, the TinyQueue span of the
    // k-mer ending there (src/sketch.rs:51-64; 256 = too long, no info).
    // Null: every span is k (non-HPC, sketch.rs:66-70).
    const uint16_t* hpc_span = nullptr;
    // Query reads in the device nt4 format (include/mm2g.h, "nt4 read batch"):
    // read r's 2-bit codes start at pk_words[pk_off[r]], its ambiguity bitmap
    // (if any) at pk_words[amb_off[r]] (U64MAX = none).  Null: ASCII `seq`.
    const uint64_t* pk_words = nullptr;
    const uint64_t* pk_off = nullptr;
    const uint64_t* amb_off = nullptr;
    uint32_t* mz_need = nullptr;   // per sequence: the unclamped minimizer count (mz_cnt is clamped to the slot)
    // Query views (views of nt4 reads, odd k; DESIGN.md "Query sketch views"):
    // view r is [view_off[r], + view_len[r]) of read view_read[r] (view_off a
    // multiple of 8), with the same view_pre / emit_from / view_last meaning.
    const uint32_t* view_read = nullptr;
    uint32_t x64 = 0;              // k <= 15: keep the 64-bit LDS window (MM2G_KNOB_SKETCH_X32 = 0) instead of the hash-only one
};
struct FilterArgs {
    uint32_t n;
    const uint64_t* mz_base; const uint32_t* mz_cnt; const uint64_t* mz_x;
    const uint64_t* tab_off;   // per read (n+1), exclusive scan of table sizes
    uint64_t* tab_key; uint32_t* tab_cnt;
    uint8_t* keep;
    int q_occ_max; float q_occ_frac;
    uint64_t cap_tab;          // entries of tab_key/tab_cnt: a read whose table would end beyond it is skipped (batch flagged)
};
struct SeedArgs {
    uint32_t n;
    const uint64_t* rd_off;
    const uint64_t* mz_base; const uint32_t* mz_cnt; const uint64_t* mz_x; const uint32_t* mz_y; const uint8_t* keep;
    const IxEntry* tab; uint32_t log2cap; int32_t mid_occ;
    const uint64_t* ix_pos;
    uint32_t* mz_n; uint32_t* mz_poff;
    uint32_t* a_cnt;
    const uint64_t* a_off;
    uint64_t* keys;
    KeyLayout kl; int span;
    uint64_t cap_keys, cap_pos, cap_mz;   // bounds for the MM2G_CHECKED build
    ReadOut* out;                         // m_kept
    uint32_t* a_part;                     // per read, SEED_PARTS-1 entries: anchors before part k (k = 1..)
    const uint32_t* abort = nullptr;      // batch status word (BS_*): kernels after the anchor scan exit on BS_ANCHORS
    const uint32_t* order = nullptr;      // k_seed_write: reads heaviest first (null = batch order)
    // fused seeding: reads with small_max < A <= 65535 anchors and at most fuse_mmax minimizers
    // get their keys from k_sort_read's first pass instead (0 = off; SortArgs::fuse_mmax)
    uint32_t fuse_mmax = 0, small_max = 0;
    // fused seeding of the whole-read sort: reads over 65535 anchors get their keys from k_sort_big's
    // first pass (SortArgs::fuse_big; 0 = off)
    uint32_t fuse_big = 0;
};
// seed_write splits each read's minimizers into this many contiguous parts
// (whole 64-minimizer chunks), one wave each; seed_count records where they start
constexpr int SEED_PARTS = 16;   // (round 5: 4 -> 16; C5's 1,000-read units then give 16 k waves instead of 4 k)
// per-read anchor sort + singleton filter (k_sort_small / k_sort_read)
constexpr int32_t SEG_CHUNK = 4096;     // anchors per work item of the streaming chain kernels
constexpr uint32_t SEG_THREAD = 1024;   // cell segments up to this length: one thread per anchor (default seg_small)
constexpr int CELL_SHIFT = 15;   // 32 kb reference cells (>= every max_dist_x the filter is used with)
constexpr uint32_t MAX_CELLS = 320 * 1024;   // more cells: singleton filter off (the sorts' two LDS bitmaps must fit)
struct SortArgs {
    uint32_t n;
    const uint64_t* a_off;
    uint64_t* keys; uint64_t* tmp;
    uint32_t qb, rb, n_seq;
    uint64_t cap_keys;
    const uint32_t* goff;   // per group incl. the Q19 pseudo-group 2*n_seq: first cell (guard cell on either side); [2*n_seq+1] = cells
    uint32_t cells;         // 0 = singleton filter off
    uint32_t* cnt2;         // per read: anchors kept (sorted at keys[a_off[r] ..])
    uint64_t* smax;         // per read: 1 + largest dropped (singleton) key, 0 = none
    uint32_t small_max;     // reads with more anchors go to k_sort_read (LDS bitonic below)
    uint64_t* prof;         // MM2G_SORT_PROF: per read 8 wall-clock stamps of k_sort_read's phases (else null)
    uint32_t lds_words;     // dynamic LDS of k_sort_read: requested (0 = SORT_LDS), set by launch_sort_read
    uint32_t seg_small;     // cell segments up to this length (<= 1024) are ranked one thread per anchor
    uint32_t* meta;         // per anchor scratch (the DP's f buffer): u16 kept-cell rank of each key (k_sort_read)
    const uint32_t* abort = nullptr;
    uint32_t* rlist = nullptr;   // reads k_sort_read leaves to k_sort_radix ([n]), and their count (zeroed by k_sort_small)
    uint32_t* rcount = nullptr;
    const uint32_t* order = nullptr;   // k_sort_read: block b sorts read order[b] (heaviest first); null = b
    uint32_t* rwork = nullptr;         // k_sort_big: next list entry to take (zeroed by k_sort_small)
    uint32_t big_wnd = 1u << 30;       // k_sort_big: most windows its P3 appends to (0: per-key scatter by bucket)
    // fused seeding (k_sort_read P1 writes the keys of the reads k_seed_write skipped; SeedArgs)
    uint32_t fuse_mmax = 0;
    const uint64_t* rd_off = nullptr; const uint64_t* mz_base = nullptr; const uint32_t* mz_cnt = nullptr;
    const uint32_t* mz_y = nullptr; const uint32_t* mz_n = nullptr; const uint32_t* mz_poff = nullptr;
    const uint64_t* ix_pos = nullptr; KeyLayout kl{}; int span = 0; uint64_t cap_pos = 0;
    // fused seeding in k_sort_big (reads over 65535 anchors, k_seed_write skipped them): its first
    // pass runs k_seed_write's parts, one wave each, from k_seed_count's part starts
    uint32_t fuse_big = 0;
    const uint32_t* a_part = nullptr;
    // segments up to this many keys are ranked by a linear scan, longer ones chunk-sorted first
    // (k_sort_read / k_sort_big; MM2G_KNOB_READ_TINY / MM2G_KNOB_BIG_TINY)
    uint32_t read_tiny = 16, big_tiny = 16;
    uint32_t small_reg = 1;   // k_sort_small: reads of 257..4096 anchors sorted with the keys in registers (MM2G_KNOB_SMALL_REG)
};
struct ChainArgs {
    uint32_t n;
    const uint64_t* rd_off;
    const uint64_t* a_off;
    const uint64_t* keys;
    int32_t* f; int32_t* pp; uint32_t* chain;
    const int16_t* lut;
    ChainKParams P; KeyLayout kl;
    ReadOut* out;
    uint32_t* work;
    uint64_t cap_keys;
    uint32_t* trace;    // MM2G_CHECKED: host-mapped per-wave progress {read, i, phase, aux}
    const uint32_t* order;   // reads in hand-out order (heaviest first); null = identity
    uint64_t a_total;        // anchors in the batch; chain[a_total + a_off[r] ...] = segment scratch
    int32_t n_prio;          // order[0 .. n_prio) run at raised wave priority
    int32_t* tmark;          // per-anchor scratch: the reference's t[] for one-lane segments
    uint4* lseg;             // long-segment queue: (read, s, e, -)
    uint32_t* lseg_n;        // its length (atomic counter)
    uint32_t lseg_cap;
    uint32_t* lseg_order;    // long segments, longest first
    unsigned long long* rbest;   // per read: packed (f, index) of the last argmax f
    const uint32_t* cnt2;    // anchors kept per read (k_sort_read's singleton filter)
    const uint64_t* smax;    // 1 + largest dropped key per read, 0 = none
    uint4* mseg;             // medium-segment queue: (read, s, e, -)
    uint32_t* mseg_n;        // its length (atomic counter)
    uint32_t* mseg_take;     // next entry to hand out (atomic counter)
    uint32_t mseg_cap;
    int32_t* fmin;           // per read: a lower bound of max f (k_chain_lb); null = no segment pruning
    uint32_t lseg_prof;      // MM2G_LSEG_PROF: k_chain_long stores each long segment's wall-clock ticks in lseg[].w
    uint32_t lazy;           // k_chain_long: skip deep windows no predecessor of which can beat max_f (not in debug mode)
    uint32_t* item_off;      // k_seg_items: first work item (chunk) of order[t]; [n] = total
    uint32_t* item_read = nullptr;   // k_seg_items: per work item its position t in order (null: search item_off)
    uint32_t item_cap = 0;           // entries of item_read
    uint32_t seg_chunk;      // anchors per work item (multiple of 64; SEG_CHUNK)
    uint32_t giant_min;      // long segments of at least this many anchors try k_chain_giant first (rescue: 128)
    uint32_t giant_lcap;     // tests: cap of the LDS variant below its LDS capacity (0 = none)
    uint32_t giant_gmax;     // global variant: anchors per workgroup scratch slice (0 = off)
    void* giant_scr;         // global variant scratch: grid x giant_gmax x 42 B
    uint32_t spec_rounds = 3; // k_chain_long: speculative rounds per 64-anchor block (MM2G_KNOB_SPEC_ROUNDS)
    uint32_t spec_eval = 1;   // k_chain_long: next-round guesses evaluated along the round's predecessors (MM2G_KNOB_SPEC_EVAL)
    uint32_t spec_batch = 4;  // k_chain_long: predecessors per step of a speculative round, 4 or 8 (MM2G_KNOB_SPEC_BATCH)
    uint32_t cands_longw = 1024;         // k_seg_cands: reads over this many segment-start words take a whole workgroup
    const uint32_t* mz_cnt = nullptr;    // with bsum: k_seg_items writes bsum[3] = sum mz_cnt, bsum[4] = sum cnt2
    unsigned long long* bsum = nullptr;
    int32_t est_lane = 0;    // k_chain_seg (production): estimated DP pairs up to which a segment takes one lane
    uint32_t full_dp = 0;    // debug mode (exact f/pprev everywhere): pass 0 uses EST_LANE instead of est_lane
    uint32_t giant_exact;    // 1: policy iteration on the reference loop itself (pass 0's real chains)
    const uint32_t* abort = nullptr;
    unsigned long long* gprof = nullptr;   // MM2G_LSEG_PROF: k_chain_giant phase sums (16 counters)
    unsigned long long* seg_stat = nullptr;   // k_lseg_order: anchors in long (< / >= giant_min) and medium segments
    // Pass 0 (production, pruning on): segment starts of the sorted kept anchors, one bit per
    // anchor (k_chain_lb writes them, k_chain_seg's sparse items read them); read r's words
    // start at (a_off[r] >> 6) + r.  Null: every item streams its keys.
    uint64_t* isob = nullptr;
    unsigned long long* seg_streamed = nullptr;   // anchors of the items k_chain_seg streamed in this pass (counter)
    // k_seg_cands -> k_chain_seg (pass 0 with isob): the (read, chunk) items left to streaming
    uint2* sq = nullptr;
    uint32_t* sq_n = nullptr;
    uint32_t sq_cap = 0;
    uint32_t zero_fmin = 0;   // k_seg_items clears fmin[0, n) (the pass's LB starts from 0)
};
struct DvArgs {
    uint32_t n;
    const uint64_t* a_off; const uint64_t* keys; const uint32_t* chain;
    const uint64_t* mz_base; const uint32_t* mz_cnt; const uint32_t* mz_y;
    KeyLayout kl; int span;
    ReadOut* out;
    uint64_t cap_keys, cap_mz;
    const uint32_t* abort = nullptr;
    uint32_t strict = 0;      // the dv sketch's k is odd: its minimizer positions strictly increase (parallel match)
    uint32_t long_m = 0;      // strict: reads with more minimizers than k_dv stages (<= long_m) go to k_dv_long (0 = none)
};

}  // namespace mm2g

// ---- launchers (return 0 or a hipError_t) --------------------------------
typedef struct ihipStream_t* hipStream_t;
int launch_sketch(const mm2g::SketchArgs& a, int n_blocks, hipStream_t st);
int launch_filter(const mm2g::FilterArgs& a, int k, int n_blocks, hipStream_t st);
int launch_seed_count(const mm2g::SeedArgs& a, int n_blocks, hipStream_t st);
int launch_seed_write(const mm2g::SeedArgs& a, int n_blocks, hipStream_t st);
// per-read MSD bucket sort on (group, rpos) + per-bucket full-key sort (qb = query bits of the key)
int launch_sort_read(int stage, const mm2g::SortArgs& a, hipStream_t st);
// dynamic LDS words k_sort_read runs with (launch_sort_read; the host sizes fuse_mmax from it)
uint32_t sort_read_lds_words(const mm2g::SortArgs& a);   // 0 small reads, 1 large
// MM2G_CHECKED builds: first recorded bounds violation {line, index, cap}; 0 = none
int mm2g_checked_read(unsigned long long out[4], hipStream_t st);
// chain DP of one pass, stage 0..4: k_chain_seg, k_chain_med, k_lseg_order, k_chain_long, k_chain_fin
int launch_chain_stage(int stage, const mm2g::ChainArgs& a, int blocks, hipStream_t st);
int chain_max_blocks(int lut_n, int which);   // co-resident workgroups (0 = k_chain_seg, 1 = k_chain_long, 2 = k_chain_med)
int launch_read_order(uint32_t n, const uint32_t* a_cnt, uint32_t* order, hipStream_t st);
int launch_dv(const mm2g::DvArgs& a, hipStream_t st);
// out[i] = exclusive prefix of f(in[t]); mode 0 identity, mode 1 the global filter
// table size of a read with in[t] minimizers (0 when it fits k_filter_lds).  When
// cap > 0 and the total exceeds it, `bit` is OR-ed into status[0]; status[slot]
// receives the total.
// order (mode 0 over anchor counts): also the heaviest-first read order (k_read_order's)
int launch_excl_scan(const uint32_t* in, uint32_t n, uint64_t* out, int mode, int q_occ_max, int k, uint64_t cap, uint32_t* status,
                     uint32_t bit, int slot, hipStream_t st, uint32_t* order = nullptr);
// per-batch sums for the counters: status64[3] = sum mz_cnt, status64[4] = sum cnt2
int launch_batch_sums(uint32_t n, const uint32_t* mz_cnt, const uint32_t* cnt2, unsigned long long* status64, hipStream_t st);
// minimizer slots: read r gets [rd_off[r] + 16r, rd_off[r+1] + 16(r+1)), or `slot` entries each when non-zero (tests)
// (zout / zst: also zero out[0, n] and zst[0, zst_words) -- the map's first kernel)
int launch_mz_base(uint32_t n, const uint64_t* rd_off, uint64_t* base, uint64_t* end, uint32_t slot, hipStream_t st,
                   mm2g::ReadOut* zout = nullptr, unsigned long long* zst = nullptr, int zst_words = 0);
// query sketch views: the view table (per-read view counts, their exclusive scan vo, the views) in one
// single-workgroup launch, plus launch_mz_base's work when base is given; per-read concatenation
int launch_view_plan(uint32_t n, const uint64_t* rd_off, uint32_t V, uint32_t W0, uint64_t nvmax, uint64_t* vo, uint32_t* v_read,
                     uint64_t* v_off, uint32_t* v_len, uint32_t* v_pre, uint32_t* v_from, uint8_t* v_last, uint64_t* v_base, uint64_t* v_end,
                     uint64_t* base, uint64_t* end, mm2g::ReadOut* zout, unsigned long long* zst, int zst_words, hipStream_t st);
int launch_view_compact(uint32_t n, const uint64_t* vo, const uint64_t* v_off, const uint64_t* v_base, const uint32_t* v_cnt,
                        const uint32_t* v_need, const uint64_t* vx, const uint32_t* vy, const uint64_t* base, const uint64_t* end, uint64_t* x,
                        uint32_t* y, uint32_t* cnt, uint32_t* need, int32_t* overflow, hipStream_t st);
int launch_mid_hist(const mm2g::IxEntry* tab, uint64_t cap, uint32_t nbins, unsigned long long* hist, uint32_t* ovf, uint32_t ovf_cap,
                    uint32_t* ovf_n, hipStream_t st);
int launch_ix_build(const uint64_t* keys, const uint32_t* offs, const uint32_t* ns, uint64_t nk, mm2g::IxEntry* tab, uint32_t log2cap, hipStream_t st);
