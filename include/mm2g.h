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
 *     0 < k <= 28, non-empty sequence (src/sketch.rs:40-42).
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
/* The same builds on a GPU (reference sketching, bucket
 * sort by hash and p/h construction on `device`, S packed there too); the
 * result is identical to the host build (same .mmi bytes).  HPC (flag & 1) and
 * even k fall back to the host build inside the call. */
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

/* ---------------------------------------------------------------- device
 * One context per (host thread, device). */
int mm2g_ctx_create(int device, mm2g_ctx** out);
void mm2g_ctx_destroy(mm2g_ctx* ctx);
/* Copies the index into HBM as an open-addressed key table + position
 * array (DESIGN.md "Index layout").  mid_occ as computed by the caller
 * (main.rs:196-197: max(calc_mid_occ(-f), 10)). */
int mm2g_ctx_upload_index(mm2g_ctx* ctx, const mm2g_index* idx, int32_t mid_occ);
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
#define MM2G_R_EMPTY 16    /* empty read (reference asserts, src/sketch.rs:40) */
typedef struct {
    int32_t flags;
    int32_t n_anchors;
    int32_t score;        /* s1: f[best_i]                                     */
    int32_t cm;           /* chain length                                      */
    int32_t qs, qe;       /* chain_qrange (forward-of-anchor coordinates)      */
    int32_t ts, te;       /* chain_trange                                      */
    int32_t rid;          /* target id (0x7fffffff for a Q19 chain)            */
    int32_t rev;          /* strand '-'                                        */
    int32_t n_match;      /* paf.rs:414-421 greedy match                       */
    int32_t dv_st, dv_en; /* minimizer-index range of the match                */
    int32_t m_dv;         /* #minimizers of the dv sketch (idx.w, idx.k)       */
    int64_t sum_k;        /* sum of their spans                                */
    int32_t qlen;
    float dv;             /* filled by the host (glibc powf)                   */
} mm2g_read_result;

/* Upload a batch of reads (ASCII, concatenated; offs has n_reads+1 entries). */
int mm2g_batch_set_reads(mm2g_ctx* ctx, const uint8_t* seq, const uint64_t* offs, uint32_t n_reads);
/* Run sketch -> filter -> lookup -> anchors -> sort -> chain DP (+rescue) ->
 * chain epilogue -> dv counts on the device for the resident batch; the
 * results stay on the device until mm2g_batch_results.  Equivalent to the
 * Align flow (src/main.rs:189-230) applied to every read. */
int mm2g_batch_map(mm2g_ctx* ctx, const mm2g_map_opts* opts);
/* Copy per-read results to the host and finish dv (paf.rs:156-199). */
int mm2g_batch_results(mm2g_ctx* ctx, mm2g_read_result* out, uint32_t n_reads);
/* Format PAF lines (write_paf, src/paf.rs:224-236) for n results; names
 * are the read names. Returns bytes written (or negative status); lines
 * for reads without a chain are omitted. */
int64_t mm2g_format_paf(const mm2g_index* idx, const mm2g_read_result* res, const char* const* names, uint32_t n,
                        char* out, int64_t cap);

/* ---------------------------------------------------------------- stages
 * Stage-level access for parity tests (each replaces one reference fn). */
/* sketch_sequence(seq, w, k, rid, false, out) (src/sketch.rs:29-100) on the
 * device for every read of the batch: out_ks/out_rps receive the minimizers
 * of read r at [out_off[r], out_off[r+1]).  Pass NULL buffers to size. */
int mm2g_batch_sketch(mm2g_ctx* ctx, int w, int k, uint32_t rid, uint64_t* out_off, uint64_t* out_ks, uint64_t* out_rps,
                      uint64_t cap);
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

/* Per-kernel device time (HIP events on the context stream) accumulated over
 * mm2g_batch_map calls since the last reset: names[i], ms[i], calls[i]. */
int mm2g_prof_enable(mm2g_ctx* ctx, int on);
int mm2g_prof_get(mm2g_ctx* ctx, int i, const char** name, double* ms, int64_t* calls);
int mm2g_prof_reset(mm2g_ctx* ctx);
/* Batch counters for roofline accounting: [0]=bases [1]=minimizers
 * [2]=kept minimizers [3]=anchors [4]=rescued anchors [5]=dp pair evaluations
 * [6]=anchors entering the DP (after the sort's singleton filter).
 * Copies min(n, MM2G_N_COUNTERS) values; returns how many. */
#define MM2G_N_COUNTERS 7
int mm2g_batch_counters(mm2g_ctx* ctx, uint64_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* MM2G_H */
