/*
 * mm2g.h — C ABI of the MI355X-native sketch -> seed -> chain path of mm2rs.
 *
 * This is the drop-in boundary for the reference crate's hot path
 * (xuzhougeng/minimap2_rs, src/{sketch,seeds,index,lchain,paf}.rs).  The
 * reference has no FFI layer of its own; every entry point
 * below names the Rust function it replaces (file:line under
 * /root/reference) and keeps its argument meaning.  A Rust host would bind
 * these with a plain `extern "C"` block.
 *
 * Conventions
 *   - Status: 0 = ok, negative = MM2G_E_* ; mm2g_last_error() gives text
 *     (thread-local).  No C++ exception crosses this boundary.
 *   - Ownership: the caller owns every host buffer it passes; the library
 *     owns device memory behind opaque handles, released by *_free/_destroy.
 *   - Threading: one mm2g_ctx per (host thread, device).  Calls on one
 *     context are serialised on its HIP stream; distinct contexts (and
 *     devices) run concurrently — that is how reads shard over GPUs.
 *   - Argument checks mirror the reference asserts: 0 < w < 256,
 *     0 < k <= 28, non-empty sequence (src/sketch.rs:30-32).
 *   - Nothing on the mapping path reads the environment: tuning and test
 *     switches are explicit per-context knobs (mm2g_ctx_set_knob).
 */
#ifndef MM2G_H
#define MM2G_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MM2G_OK 0
#define MM2G_E_ARG -1      /* invalid argument (reference: assert!/panic)   */
#define MM2G_E_IO -2       /* file I/O or format error (reference: anyhow)   */
#define MM2G_E_HIP -3      /* HIP runtime error                              */
#define MM2G_E_NOMEM -4    /* host or device allocation failed               */
#define MM2G_E_STATE -5    /* call sequence error (e.g. no index uploaded)  */
#define MM2G_E_UNSUP -6    /* outside the supported parity envelope          */

typedef struct mm2g_index mm2g_index; /* host index: Index (src/index.rs:33-42) */
typedef struct mm2g_ctx mm2g_ctx;     /* one device: stream, device index, batch workspaces */

int mm2g_version(void);
const char* mm2g_last_error(void);
/* Number of visible HIP devices (0 when none / no driver). */
int mm2g_device_count(void);

/* ---------------------------------------------------------------- index
 * build_index_from_fasta(path, w, k, b, flag) (src/index.rs:427-475). */
int mm2g_index_build_fasta(const char* path, int w, int k, int b, int flag, int n_threads, mm2g_index** out);
/* Same from in-memory sequences (names may be NULL -> no name). */
int mm2g_index_build_seqs(uint32_t n_seq, const char* const* names, const uint8_t* const* seqs, const uint64_t* lens,
                          int w, int k, int b, int flag, int n_threads, mm2g_index** out);
/* The same builds on a GPU (reference sketching, a
 * hand-written radix sort by (bucket, hash, position) and the p/h construction
 * on `device`; S packed by host threads meanwhile); the
 * result is identical to the host build (same .mmi bytes).  Odd and even k
 * (per-view warm-ups sized on the host) and HPC (flag & 1: TinyQueue spans,
 * src/sketch.rs:51-64, computed per base on the device) are built on the
 * device; a device failure the build cannot handle (minimizer slot overflow)
 * falls back to the host build inside the call unless MM2G_IKNOB_GPU_STRICT. */
int mm2g_index_build_fasta_gpu(const char* path, int w, int k, int b, int flag, int device, int n_threads, mm2g_index** out);
int mm2g_index_build_seqs_gpu(uint32_t n_seq, const char* const* names, const uint8_t* const* seqs, const uint64_t* lens,
                              int w, int k, int b, int flag, int device, int n_threads, mm2g_index** out);
/* Index::load_from_mmi (src/index.rs:361-424) / Index::save_to_mmi (:233-307).
 * Hash entries are written in ascending key order (the reference writes
 * HashMap iteration order, which is random per process). */
int mm2g_index_load_mmi(const char* path, mm2g_index** out);
int mm2g_index_save_mmi(const mm2g_index* idx, const char* path);
void mm2g_index_free(mm2g_index* idx);
/* Index::stats (src/index.rs:111-122). */
int mm2g_index_stats(const mm2g_index* idx, uint64_t* n_keys, double* avg_occ, double* avg_spacing, uint64_t* total_len);
/* Index::calc_mid_occ (src/index.rs:124-141); INT32_MAX when the index is empty. */
int mm2g_index_calc_mid_occ(const mm2g_index* idx, float frac, int32_t* out);
int mm2g_index_params(const mm2g_index* idx, int32_t* w, int32_t* k, int32_t* b, int32_t* flag, uint32_t* n_seq);
int mm2g_index_seq(const mm2g_index* idx, uint32_t rid, const char** name, uint32_t* len);
/* Index::get (src/index.rs:143-154): *kind = 0 none, 1 Single, 2 Multi;
 * returns the number of positions (copies up to cap into out). */
int64_t mm2g_index_get(const mm2g_index* idx, uint64_t minier, int* kind, uint64_t* out, int64_t cap);
/* How this index came to be (the reference has one path, build_index_from_fasta
 * src/index.rs:427-475, or load_from_mmi :361-424): returns an MM2G_IX_* value;
 * *note (may be NULL) receives why a GPU build ran on the host, else NULL. */
#define MM2G_IX_HOST 1          /* mm2g_index_build_fasta / _seqs                      */
#define MM2G_IX_GPU 2           /* mm2g_index_build_*_gpu, built on the device          */
#define MM2G_IX_GPU_FALLBACK 3  /* a GPU build the device could not do, built on the host */
#define MM2G_IX_MMI 4           /* mm2g_index_load_mmi                                  */
int mm2g_index_origin(const mm2g_index* idx, const char** note);
/* Free the host hash tables and S of an index whose device copies are made
 * (per GPU process only names, lengths and (w, k) are needed afterwards, for
 * PAF and dv).  Later save/get/calc_mid_occ/upload calls fail with
 * MM2G_E_STATE; stats keep their values. */
int mm2g_index_release_tables(mm2g_index* idx);

/* ---------------------------------------------------------------- device
 * One context per (host thread, device). */
int mm2g_ctx_create(int device, mm2g_ctx** out);
void mm2g_ctx_destroy(mm2g_ctx* ctx);
/* Copies the index into HBM as an open-addressed key table + position
 * array (DESIGN.md "Index layout").  mid_occ as computed by the caller
 * (main.rs:196-197: max(calc_mid_occ(-f), 10)). */
int mm2g_ctx_upload_index(mm2g_ctx* ctx, const mm2g_index* idx, int32_t mid_occ);
/* The same for n contexts (normally one per GPU: `mm2rs align --devices`):
 * the host layout is built once and the devices' copies are made in parallel
 * host threads.  All or nothing: on an error no context changes its index
 * (each keeps the one it had). */
int mm2g_ctx_upload_index_many(mm2g_ctx* const* ctxs, int n, const mm2g_index* idx, int32_t mid_occ);
/* Use the device index of `src` (same device) in `dst` without another copy:
 * several contexts — one per host thread, each with its own stream and batch
 * buffers — map concurrently against one index in HBM. */
int mm2g_ctx_share_index(mm2g_ctx* dst, const mm2g_ctx* src, int32_t mid_occ);
/* Index::calc_mid_occ (src/index.rs:124-141) computed on the uploaded device
 * table by a count histogram; equals
 * mm2g_index_calc_mid_occ on the same index.  INT32_MAX when empty. */
int mm2g_ctx_index_mid_occ(mm2g_ctx* ctx, float frac, int32_t* out);
/* Replace the mid_occ given at upload/share (main.rs:196-197 clamp is the caller's). */
int mm2g_ctx_set_mid_occ(mm2g_ctx* ctx, int32_t mid_occ);

/* Mapping options: `mm2rs align` flags (src/main.rs:55-89) and the chain
 * parameters they drive (default_chain_params, src/main.rs:105-123). */
typedef struct {
    int32_t w, k;            /* query sketch (CLI -w/-k after -x preset)        */
    int32_t max_gap;         /* -g  -> max_dist_x = max_dist_y                  */
    int32_t bw, bw_long;     /* -r bw[,bw_long]  (500, 20000)                   */
    int32_t min_cnt;         /* -n  (3)                                         */
    int32_t min_chain_score; /* -m  (40)                                        */
    float mask_level;        /* -M  (0.5)                                       */
    float pri_ratio;         /* -p  (0.8)                                       */
    int32_t best_n;          /* -N  (5)                                         */
} mm2g_map_opts;
void mm2g_map_opts_default(mm2g_map_opts* o);

/* Per-read result (the integer PAF columns; dv inputs).  flags: */
#define MM2G_R_MAPPED 1    /* a chain exists -> one PAF line                  */
#define MM2G_R_RESCUED 2   /* rescue_long_join re-ran the DP with bw_long     */
#define MM2G_R_DV_FOUND 4  /* first chain position found among minimizers     */
#define MM2G_R_PANIC 8     /* reference panics: chain on an odd-rid contig (Q19) */
#define MM2G_R_EMPTY 16    /* empty read (reference asserts, src/sketch.rs:30) */
typedef struct {
    int32_t flags;
    int32_t n_anchors;
    int32_t score;        /* s1: f[best_i]                                     */
    int32_t cm;           /* chain length                                      */
    int32_t qs, qe;       /* chain_qrange (forward-of-anchor coordinates)      */
    int32_t ts, te;       /* chain_trange                                      */
    int32_t rid;          /* target id (0x7fffffff for a Q19 chain)            */
    int32_t rev;          /* strand '-'                                        */
    int32_t n_match;      /* paf.rs:178-186 greedy match                       */
    int32_t dv_st, dv_en; /* minimizer-index range of the match                */
    int32_t m_dv;         /* #minimizers of the dv sketch (idx.w, idx.k)       */
    int64_t sum_k;        /* sum of their spans                                */
    int32_t qlen;
    float dv;             /* filled by the host (glibc powf)                   */
} mm2g_read_result;

/* ---------------------------------------------------------------- reads
 * nt4 read batch: the input format of query reads on the device.  Reads cross
 * PCIe and sit in HBM as nt4 codes (src/nt4.rs:2-10: A/a 0, C/c 1, G/g 2,
 * T/t 3, anything else 4) packed 2 bits per base:
 *   base i of read r: bits 2*(i%32) of words[pk_off[r] + i/32]  (code & 3;
 *                     an ambiguous base stores 0)
 *   a read with an ambiguous base (code 4) also has a bitmap:
 *                     bit i%64 of words[amb_off[r] + i/64] = base i is ambiguous;
 *                     amb_off[r] = UINT64_MAX for a read without one. */
typedef struct {
    uint32_t n_reads;
    const uint64_t* lens;      /* bases per read                               */
    const uint64_t* pk_off;    /* word offset of each read's codes             */
    const uint64_t* amb_off;   /* word offset of its bitmap, or UINT64_MAX     */
    const uint64_t* words;
    uint64_t n_words;
} mm2g_nt4_batch;
/* Words mm2g_nt4_pack may need for these reads (codes plus worst-case bitmaps). */
uint64_t mm2g_nt4_words_bound(const uint64_t* offs, uint32_t n_reads);
/* Pack ASCII reads (seq[offs[r] .. offs[r+1])) into the nt4 format on
 * n_threads host threads; fills pk_off/amb_off (n_reads each).  Returns the
 * words written or a negative status.  The reference applies nt4 base by base
 * inside sketch_sequence (src/sketch.rs:62). */
int64_t mm2g_nt4_pack(const uint8_t* seq, const uint64_t* offs, uint32_t n_reads, uint64_t* pk_off, uint64_t* amb_off,
                      uint64_t* words, uint64_t cap_words, int n_threads);

/* Stage a batch of ASCII reads (concatenated; offs has n_reads+1 entries):
 * packed to nt4 on host threads into pinned memory (double-buffered per
 * context) and copied to HBM asynchronously on the context stream.  Returns
 * before the copy ends; the caller may reuse its buffers at once.  A batch
 * whose results were not collected is dropped. */
int mm2g_batch_set_reads(mm2g_ctx* ctx, const uint8_t* seq, const uint64_t* offs, uint32_t n_reads);
/* The same for reads the caller already packed (copied into pinned staging). */
int mm2g_batch_set_reads_nt4(mm2g_ctx* ctx, const mm2g_nt4_batch* batch);
/* Queue sketch -> filter -> lookup -> anchors -> sort -> chain DP (+rescue) ->
 * chain epilogue -> dv counts for the resident batch on the context stream and
 * return without waiting (no host synchronisation inside).  Equivalent to the
 * Align flow (src/main.rs:189-230) applied to every read. */
int mm2g_batch_map(mm2g_ctx* ctx, const mm2g_map_opts* opts);
/* Wait for the batch, copy per-read results to the caller and finish dv
 * (paf.rs:189-199).  Batch workspaces are sized from the previous batches; if
 * one was too small (the device flags it) it is grown and the batch mapped
 * again here, transparently. */
int mm2g_batch_results(mm2g_ctx* ctx, mm2g_read_result* out, uint32_t n_reads);
/* Format PAF lines (write_paf, src/paf.rs:224-236) for n results; names
 * are the read names. Returns bytes written (or negative status); lines
 * for reads without a chain are omitted. */
int64_t mm2g_format_paf(const mm2g_index* idx, const mm2g_read_result* res, const char* const* names, uint32_t n,
                        char* out, int64_t cap);

/* PAF lines of the batch mm2g_batch_results collected last, for its first n
 * reads in read order (names[r] = read r's name): write_paf_many_with_scores
 * (src/paf.rs:238-248) of main.rs:209-218's chains -- one line per mapped read
 * under -n >= 2 (the same text as mm2g_format_paf), several with tp:A:P/S and
 * s2 under -n <= 1 -m <= k.  Reads on which the reference panics print nothing.
 * Returns bytes written; out = NULL only sizes. */
int64_t mm2g_batch_paf(mm2g_ctx* ctx, const char* const* names, uint32_t n, char* out, int64_t cap);

/* One line of the multi-chain output (paf_from_chain_with_primary, src/paf.rs:130-222). */
typedef struct {
    int32_t qs, qe, ts, te;  /* chain ranges (forward-of-anchor query coordinates)  */
    int32_t rid, rev, cm;
    int32_t primary;         /* tp:A:P (1) or S (0)                                 */
    float dv;
    int32_t s1, s2;
} mm2g_chain_line;
/* The host epilogue of one read under -n <= 1 -m <= k (what mm2g_batch_results
 * runs per read; DESIGN.md §2 "-n <= 1"), on the caller's sorted anchors
 * (xy pairs as build_anchors_filtered returns them) and the final chain_dp_all
 * pass's f / pprev (after rescue_long_join when it re-ran the DP): the
 * backtrack (src/lchain.rs:92-175; z ordered by rustc 1.81+ sort_unstable),
 * merge_adjacent_chains_with_gap (:288-314, max_gap = opts->max_gap),
 * select_and_filter_chains (:237-260) and the PAF records with dv
 * (paf.rs:155-199; mini_pos = the read's minimizer positions of the index's
 * (w, k) sketch, avg_k their mean span in f32; tlen[rid] per target).  Host
 * only.  Returns the number of lines (written up to cap), 0 for none, or
 * MM2G_E_STATE when the reference panics on the read (*panic = 1). */
int64_t mm2g_multi_chain_lines(const uint64_t* xy, const int32_t* f, const int32_t* pprev, int64_t n, int32_t qlen,
                               const int32_t* mini_pos, int64_t n_mini, float avg_k, const uint32_t* tlen, uint32_t n_seq,
                               const mm2g_map_opts* opts, mm2g_chain_line* out, int64_t cap, int32_t* panic);

/* ---------------------------------------------------------------- stages
 * Stage-level access for parity tests (each replaces one reference fn). */
/* sketch_sequence(seq, w, k, rid, false, out) (src/sketch.rs:29-100) on the
 * device for every read of the batch: out_ks/out_rps receive the minimizers
 * of read r at [out_off[r], out_off[r+1]).  Pass NULL buffers to size. */
int mm2g_batch_sketch(mm2g_ctx* ctx, int w, int k, uint32_t rid, uint64_t* out_off, uint64_t* out_ks, uint64_t* out_rps,
                      uint64_t cap);
/* build_anchors_filtered(idx, mv, qlen, mid_occ) (src/seeds.rs:42-60) for every
 * read of the resident batch, with the query minimizers collected and filtered
 * as the Align flow does (collect_query_minimizers with opts->w/k, seeds.rs:7-11;
 * filter_query_minimizers(10, 0.01), seeds.rs:13-36; main.rs:194-195) and the
 * context's mid_occ.  Read r's anchors, sorted by (x, y) (seeds.rs:58), are the
 * Anchor {x, y} pairs xy[2*a_off[r] ..] up to xy[2*a_off[r+1]]; a_off has
 * n_reads+1 entries.  Returns the number of anchors; xy = NULL only sizes. */
int64_t mm2g_seed_batch(mm2g_ctx* ctx, const mm2g_map_opts* opts, uint64_t* a_off, uint64_t* xy, uint64_t cap);

/* ChainParams (src/lchain.rs:36-52). */
typedef struct {
    int32_t max_dist_x, max_dist_y, bw, max_chain_iter, min_chain_score, min_cnt;
    float chn_pen_gap, chn_pen_skip;
    int32_t max_chain_skip, max_drop, bw_long, rmq_rescue_size;
    float rmq_rescue_ratio;
} mm2g_chain_params;
/* default_chain_params(k) (src/main.rs:105-123). */
void mm2g_chain_params_default(mm2g_chain_params* p, int k);
/* One read's chain: chain_dp_all's chains[0]/scores[0] (src/lchain.rs:59-176;
 * the fallback chain under min_cnt >= 2), after rescue_long_join
 * when requested (:321-330), with chain_qrange/chain_trange (:178-200). */
typedef struct {
    int32_t flags;        /* MM2G_R_MAPPED, MM2G_R_RESCUED, MM2G_R_PANIC (Q19 rid) */
    int32_t n_anchors, score, cm;
    int32_t qs, qe, ts, te;
    int32_t rid, rev;     /* of the chain's last anchor; 0x7fffffff/1 for Q19 */
} mm2g_chain_result;
/* chain_dp_all(&anchors, &p) (src/lchain.rs:59) on the device for n_reads
 * caller-owned anchor sets: read r's anchors are xy[2*(a_off[r]-a_off[0]) ..]
 * ({x, y} pairs sorted by (x, y) as build_anchors_filtered returns them; one
 * span for all), qlen[r] its query length.  rescue != 0 also runs
 * rescue_long_join(anchors, chains, scores, p, qlen) (:321-330).  Optional
 * outputs (NULL to skip), indexed like the anchors: f and pprev of the final
 * DP pass (lchain.rs:67-91), and chain = the anchor indices of chains[0]
 * (ascending, res[r].cm of them, relative to the read's first anchor).
 * Unsupported (MM2G_E_UNSUP): chn_pen_skip != 0, min_cnt < 2, unsorted or
 * mixed-span anchors. */
int mm2g_chain_batch(mm2g_ctx* ctx, const mm2g_chain_params* p, uint32_t n_reads, const uint64_t* a_off, const uint64_t* xy,
                     const int32_t* qlen, int rescue, mm2g_chain_result* res, int32_t* f, int32_t* pprev, uint32_t* chain);

/* After mm2g_batch_map with debug enabled: the sorted anchors of read r
 * (build_anchors_filtered, src/seeds.rs:42-60) as (x, y) pairs, and the DP
 * arrays f/pprev of the final chain_dp_all pass (src/lchain.rs:59-91).
 * With debug off, mm2g_debug_anchors returns the sorted anchors the DP ran on
 * (those kept by the sort's singleton filter). */
int mm2g_ctx_set_debug(mm2g_ctx* ctx, int on);
int64_t mm2g_debug_anchors(mm2g_ctx* ctx, uint32_t r, uint64_t* xy, int64_t cap);
int64_t mm2g_debug_dp(mm2g_ctx* ctx, uint32_t r, int32_t* f, int32_t* pprev, int64_t cap);
int64_t mm2g_debug_keep(mm2g_ctx* ctx, uint32_t r, uint8_t* keep, int64_t cap);

/* After mm2g_batch_results: per read [pass-0 ticks, pass-1 ticks (100 MHz
 * wall clock), anchors in long segments, DP j-steps, j-steps reading HBM,
 * longest segment | #long segments << 16 (pass 0)] of the chain kernel
 * (6 values per read).  Returns the batch size. */
int64_t mm2g_debug_chain_stats(mm2g_ctx* ctx, uint32_t* out6, uint32_t n);

/* ---------------------------------------------------------------- knobs
 * Tuning and test switches of one context (defaults in brackets).  The
 * production path reads no environment variable; tests and A/B runs set these. */
enum {
    MM2G_KNOB_SORT_SMALL = 1,    /* reads with <= this many anchors: LDS bitonic sort, max 4096 [4096]        */
    MM2G_KNOB_SEG_SMALL = 2,     /* sort cell segments ranked one thread per anchor up to this length [1024]  */
    MM2G_KNOB_SEG_CHUNK = 3,     /* anchors per chain work item (multiple of 64) [4096]                       */
    MM2G_KNOB_GIANT_MIN = 4,     /* rescue-pass segments of >= this many anchors try k_chain_giant [128]      */
    MM2G_KNOB_GIANT_MIN0 = 5,    /* the same for pass 0 (exact mode); <= 0 = off [0]                          */
    MM2G_KNOB_GIANT_LCAP = 6,    /* tests: cap of the LDS giant variant; 0 = its LDS capacity [0]             */
    MM2G_KNOB_GIANT_GMAX = 7,    /* anchors per workgroup slice of the HBM giant variant; 0 = off [65536]     */
    MM2G_KNOB_GIANT_GBLOCKS = 8, /* workgroups of the HBM giant variant [256]                                 */
    MM2G_KNOB_FILTER = 9,        /* the sort's singleton filter [1]                                           */
    MM2G_KNOB_LAZY = 10,         /* k_chain_long skips windows that cannot beat max_f, and its simple paths;
                                    2: also in debug mode (exact f/pprev either way; tests) [1]               */
    MM2G_KNOB_PRUNE = 11,        /* pass-0 segment pruning by the best-f lower bound [1]                      */
    MM2G_KNOB_GIANT = 12,        /* the giant-segment kernels [1]                                             */
    MM2G_KNOB_SKETCH_PROF = 13,  /* phase profile of k_sketch to stderr [0]                                   */
    MM2G_KNOB_SORT_PROF = 14,    /* phase profile of k_sort_read to stderr [0]                                */
    MM2G_KNOB_LSEG_PROF = 15,    /* slowest long segments to stderr [0]                                       */
    MM2G_KNOB_MIDHIST_BINS = 16, /* bins of the device mid_occ histogram, 2..16384 [4096]                     */
    MM2G_KNOB_SYNC_EACH = 17,    /* synchronise after every stage and report faults [0]                       */
    MM2G_KNOB_HOST_THREADS = 18, /* host threads packing reads to nt4 [min(8, cores)]                         */
    MM2G_KNOB_WS_MIN = 19,       /* tests: a batch's first map starts with minimizer slots, filter-table and
                                    anchor workspaces of this many entries, forcing the re-map; 0 = off [0]   */
    MM2G_KNOB_SORT_LDS_KB = 20,  /* dynamic LDS of the large-read sort in KiB (at most 157; up to 76: 512-thread workgroups, two per CU); 0 = 157 [0] */
    MM2G_KNOB_STOP_AT = 21,      /* measurement only (results invalid): 1 stop after the anchors, 2 after the
                                    sort, 3 no rescue pass, 4 no dv kernel; 0 = full path [0]                 */
    MM2G_KNOB_SPEC_ROUNDS = 22,  /* speculative 64-anchor rounds of k_chain_long per block, 0..16 [3]            */
    MM2G_KNOB_MED_PAIRS = 23,    /* pass 0 (production): segments of up to this many estimated DP pairs take one
                                    lane (k_chain_med), longer ones a wave (k_chain_long); 0 = every segment
                                    over 8 anchors to a wave [0]                                                 */
    MM2G_KNOB_MED_PAIRS_RESCUE = 24, /* the same for the rescue pass [0]                                          */
    MM2G_KNOB_WS_FAIL = 25,      /* tests: the next this-many up-front anchor-workspace reservations fail as if
                                    HBM were full, forcing the exact-size fallback; 0 = off [0]              */
    /* 26: retired (round 5; the sort's fused LB pass, measured slower and removed) */
    MM2G_KNOB_SKETCH_VIEW = 27,  /* odd k: reads longer than this are sketched as views of this many bases,
                                    one wave each; 0 = one wave per read [2560]                             */
    /* 28: retired (round 5; k_chain_long_mw, measured 2x slower and removed) */
    MM2G_KNOB_PRUNE_RESCUE = 29, /* the rescue pass prunes segments by pass 0's best-f lower bound [1]         */
    MM2G_KNOB_VIEW_READS = 30,   /* sketch views (MM2G_KNOB_SKETCH_VIEW) only for batches of fewer reads [2048]  */
    MM2G_KNOB_SEG_SPARSE = 31,   /* pass 0: work items whose reads' best-f bound rules out every segment of <= 8
                                    anchors find their candidate segments from k_chain_lb's segment-start bits
                                    instead of streaming their keys [1]                                       */
    MM2G_KNOB_SPEC_BATCH = 32,   /* predecessors per step of k_chain_long's speculative rounds: 4 or 8 [4]     */
    MM2G_KNOB_DV_PAR = 33,       /* odd index k: k_dv matches the chain against the minimizer positions by one
                                    parallel search per chain anchor instead of the sequential walk [1]     */
    /* 34, 35: retired (round 5: k_chain_long guess sweeps before the speculative rounds, measured no faster) */
    MM2G_KNOB_SEED_FUSE = 36,    /* reads the cell sort takes (k_sort_read) get their anchor keys from its first
                                    pass instead of k_seed_write (no separate write-then-read of the keys) [1] */
    MM2G_KNOB_SKETCH_X32 = 37,   /* k <= 15: k_sketch keeps the 32-bit hash alone in its LDS window [1]           */
    MM2G_KNOB_BIG_WND = 38,      /* k_sort_big (reads over 65535 anchors): most windows its bucket pass appends
                                    the kept keys to, <= 126; 0 = the per-key scatter to bucket slots [126]   */
    MM2G_KNOB_CANDS_LONGW = 39,  /* k_seg_cands: reads over this many 64-anchor segment-start words are walked
                                    by a whole workgroup instead of one wave; 0 = never [1024]               */
    MM2G_KNOB_SEED_FUSE_BIG = 40, /* reads over 65535 anchors (k_sort_big) get their anchor keys from its first
                                    pass instead of k_seed_write [1]                                          */
    MM2G_KNOB_READ_TINY = 41,    /* k_sort_read: cell segments up to this many keys are ranked by a linear scan
                                    (longer: 64-key chunk sort first), 1..1024 [16]                          */
    MM2G_KNOB_BIG_TINY = 42,     /* the same for k_sort_big's buckets, 1..2048 [16]                              */
    MM2G_KNOB_SPEC_EVAL = 43,    /* k_chain_long: a block's next-round guesses are evaluated along the predecessors
                                    the round chose (pointer doubling) instead of taken as computed [1]        */
    MM2G_KNOB_SMALL_REG = 44,    /* k_sort_small: reads of 257..4096 anchors are sorted with the keys in registers
                                    (lane and wave exchanges; LDS only across waves) [1]                     */
    MM2G_KNOB_COUNT = 45
};
int mm2g_ctx_set_knob(mm2g_ctx* ctx, int knob, int64_t value);
int64_t mm2g_ctx_get_knob(const mm2g_ctx* ctx, int knob);
/* Process-wide switches of the index build and .mmi load. */
enum {
    MM2G_IKNOB_IXCHUNK = 1,      /* GPU index build: bases per sketch view [65536]                            */
    MM2G_IKNOB_IXPROF = 2,       /* GPU index build: phase times to stderr [0]                                */
    MM2G_IKNOB_LOAD_THREADS = 3, /* .mmi load threads; 0 = min(32, cores) [0]                                 */
    MM2G_IKNOB_GPU_STRICT = 4,   /* tests: a GPU index build the device cannot do fails instead of falling
                                    back to the host build [0]                                               */
    MM2G_IKNOB_FORCE_FALLBACK = 5, /* tests: GPU index builds take the host fallback (MM2G_IX_GPU_FALLBACK) [0] */
    MM2G_IKNOB_IXSORTV = 6,      /* tests: the GPU index build sorts by value even when the pairs arrive sorted [0] */
    MM2G_IKNOB_COUNT = 7
};
int mm2g_set_index_knob(int knob, int64_t value);

/* Per-kernel device time (HIP events on the context stream) accumulated over
 * mm2g_batch_map calls since the last reset: names[i], ms[i], calls[i]. */
int mm2g_prof_enable(mm2g_ctx* ctx, int on);
int mm2g_prof_get(mm2g_ctx* ctx, int i, const char** name, double* ms, int64_t* calls);
int mm2g_prof_reset(mm2g_ctx* ctx);
/* Batch counters for roofline accounting: [0]=bases [1]=minimizers
 * [2]=kept minimizers [3]=anchors [4]=rescued anchors [5]=dp pair evaluations
 * [6]=anchors entering the DP (after the sort's singleton filter); anchors in
 * the DP's long segments below the giant-kernel size [7] / from it on [8] and
 * in its medium segments [9] of pass 0, and [10], [11], [12] of the rescue pass;
 * DP anchors whose keys k_chain_seg streams in pass 0 (k_seg_cands finds the
 * other reads' candidate segments without reading keys) [13], that k_chain_lb
 * streams [14] (0 when it did not run: debug, multi-chain or pruning off), and
 * rescued anchors k_chain_seg streams in the rescue pass [15]; the anchors [16]
 * and minimizers [17] of the reads whose keys k_sort_read makes itself (fused
 * seeding: k_seed_write skips them); the anchors of the reads the sort hands
 * to k_sort_small [18], to k_sort_read's cell path [19] and to the whole-read
 * kernel (k_sort_big with the singleton filter on, k_sort_radix without) [20];
 * the anchors [21] and minimizers [22] of the reads whose keys k_sort_big makes
 * itself (MM2G_KNOB_SEED_FUSE_BIG).
 * Copies min(n, MM2G_N_COUNTERS) values; returns how many. */
#define MM2G_N_COUNTERS 23
int mm2g_batch_counters(mm2g_ctx* ctx, uint64_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* MM2G_H */
