// Host orchestration of the MI355X path and the C ABI declared in
// include/mm2g.h.  One mm2g_ctx = one device + one HIP stream + the device
// index + batch workspaces sized for 288 GB of HBM3E (buffers grow on demand,
// never shrink).  A batch is: host nt4 packing into pinned staging + async H2D
// (mm2g_batch_set_reads), a fixed sequence of kernel launches with no host
// synchronisation (mm2g_batch_map), and one wait for the results
// (mm2g_batch_results).  Workspaces are sized from earlier batches; the
// device flags one that was too small and the batch is mapped again.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/mm2g.h"
#include "mm2g_index.h"
#include "mm2g_internal.h"
#include "mm2g_multi.h"
#include "mm2g_reads.h"

using namespace mm2g;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;
static int set_err(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap; va_start(ap, fmt); vsnprintf(buf, sizeof buf, fmt, ap); va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return set_err(MM2G_E_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); } while (0)
#define LCHK(x) do { int e_ = (x); if (e_ != 0) return set_err(MM2G_E_HIP, "kernel launch %s: %s", #x, hipGetErrorString((hipError_t)e_)); } while (0)

struct mm2g_index {
    HostIndex h;
    int origin = 0;              // MM2G_IX_* (mm2g_index_origin)
    std::string origin_note;     // why a GPU build ran on the host instead
    bool released = false;       // mm2g_index_release_tables: the hash tables and S are freed
    uint64_t st_keys = 0, st_total = 0; double st_occ = 0, st_spacing = 0;   // stats kept across the release
};
static int need_tables(const mm2g_index* idx) {
    if (idx->released) return set_err(MM2G_E_STATE, "index tables were released (mm2g_index_release_tables)");
    return 0;
}

// ------------------------------------------------------------------ device buffers
struct DevBuf {
    void* p = nullptr; size_t cap = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
};
template <typename T>
static int ensure(DevBuf& b, size_t n, T** out) {
    size_t need = std::max<size_t>(n, 1) * sizeof(T);
    if (need > b.cap) {
        if (b.p) { (void)hipFree(b.p); b.p = nullptr; b.cap = 0; }
        size_t nc = need + need / 4;
        if (hipMalloc(&b.p, nc) != hipSuccess) { b.p = nullptr; return set_err(MM2G_E_NOMEM, "hipMalloc(%zu bytes) failed", nc); }
        b.cap = nc;
    }
    *out = (T*)b.p;
    return 0;
}
#define ENSURE(buf, T, n, ptr) do { int e_ = ensure<T>(buf, (n), &(ptr)); if (e_) return e_; } while (0)

struct ProfSlot { std::string name; double ms = 0; int64_t calls = 0; };
// Batch status block (u64 words, device + pinned copy): [0] BS_* bits | dv
// overflow, [1] filter-table entries, [2] anchors, [3] minimizers, [4] anchors
// in the DP, [5] / [6] of them in reads k_chain_seg streams / k_chain_lb runs
// on, [8 + 3 pass ..] anchors in long (< / >= giant_min) and medium
// segments of each DP pass (k_lseg_order)
constexpr int STAT_WORDS = 18;

// pinned host staging of one read batch (header + nt4 words), double-buffered
struct Stage { uint64_t* p = nullptr; uint64_t cap = 0; hipEvent_t ev = nullptr; bool pending = false; };
// minimizer slots of one sketch of the batch
struct SketchBufs {
    DevBuf base, end, x, y, cnt, need;
    bool exact = false;    // slots sized by the true counts (after an overflow)
    uint64_t cap = 0;      // minimizer slots allocated
};
// query sketch views (run_sketch): the view table, per-view slots, per-read view offsets
struct ViewBufs { DevBuf read, len, pre, from, cnt, need, off, base, end, last, vo, x, y; };

static int64_t knob_default(int k) {
    switch (k) {
    case MM2G_KNOB_SORT_SMALL: return 4096;
    case MM2G_KNOB_SEG_SMALL: return SEG_THREAD;
    case MM2G_KNOB_SEG_CHUNK: return SEG_CHUNK;
    case MM2G_KNOB_GIANT_MIN: return 128;
    case MM2G_KNOB_GIANT_GMAX: return 65536;
    case MM2G_KNOB_GIANT_GBLOCKS: return 256;
    case MM2G_KNOB_FILTER: case MM2G_KNOB_LAZY: case MM2G_KNOB_PRUNE: case MM2G_KNOB_GIANT: return 1;
    case MM2G_KNOB_MIDHIST_BINS: return 4096;
    case MM2G_KNOB_SPEC_ROUNDS: return 3;
    case MM2G_KNOB_MED_PAIRS: return 0;
    case MM2G_KNOB_MED_PAIRS_RESCUE: return 0;
    case MM2G_KNOB_SKETCH_VIEW: return 2560;
    case MM2G_KNOB_PRUNE_RESCUE: return 1;
    case MM2G_KNOB_VIEW_READS: return 2048;
    case MM2G_KNOB_SEG_SPARSE: return 1;
    case MM2G_KNOB_SPEC_BATCH: return 4;
    case MM2G_KNOB_DV_PAR: return 1;
    case MM2G_KNOB_SEED_FUSE: return 1;
    case MM2G_KNOB_SEED_FUSE_BIG: return 1;
    case MM2G_KNOB_READ_TINY: return 16;
    case MM2G_KNOB_BIG_TINY: return 16;
    case MM2G_KNOB_SPEC_EVAL: return 1;
    case MM2G_KNOB_SMALL_REG: return 1;
    case MM2G_KNOB_SKETCH_X32: return 1;
    case MM2G_KNOB_BIG_WND: return 126;
    case MM2G_KNOB_CANDS_LONGW: return 1024;
    case MM2G_KNOB_HOST_THREADS: return (int64_t)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    default: return 0;
    }
}

struct mm2g_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t knob[MM2G_KNOB_COUNT] = {};
    // index (device copy shared by every context it was shared with, same device)
    const HostIndex* hidx = nullptr;
    struct DevIndex { DevBuf tab, ix_pos, goff; uint32_t cells = 0; };
    std::shared_ptr<DevIndex> dix;
    uint32_t log2cap = 0;
    int32_t mid_occ = 10;
    bool have_index = false;
    // batch: reads (device: rd_off[n+1] | pk_off[n] | amb_off[n] | nt4 words)
    uint32_t n_reads = 0;
    uint64_t total_bases = 0;
    uint32_t max_read_len = 0;
    std::vector<uint64_t> h_rd_off;
    Stage stage[2]; int st_next = 0;
    DevBuf rd_dev;
    const uint64_t *d_rd_off = nullptr, *d_pk_off = nullptr, *d_amb_off = nullptr, *d_words = nullptr;
    SketchBufs sk1, sk2;                   // CLI (w, k) sketch; index (w, k) sketch for dv when they differ
    ViewBufs vw;                           // query views of both sketches (one at a time on the stream)
    bool views_off = false;                // a re-map after a minimizer-slot overflow: whole-read sketch
    DevBuf keep, mz_n, mz_poff;
    DevBuf tab_off, tab_key, tab_cnt;
    DevBuf a_part;                         // seed_write part starts (SEED_PARTS - 1 per read)
    DevBuf giant_scr;                      // k_chain_giant<true> scratch (allocated on first use)
    DevBuf a_cnt, a_off, keys, keys_tmp, fbuf, ppbuf, fmin, item_off, item_read, outb, lut, work, order, tmark, lseg, lseg_order, lseg_n, rbest, mseg, cnt2, smax, rlist, isob, sq, sq_n;
    DevBuf dstat;                          // batch status block (BS_* word, workspace needs, counters)
    DevBuf chain_rdoff;                    // mm2g_chain_batch: prefix sums of the caller's qlen
    uint64_t cap_tab = 0, cap_A = 0;       // filter-table entries / anchors the workspaces hold
    uint64_t* h_stat = nullptr;            // pinned copy of dstat (STAT_WORDS u64)
    hipEvent_t ev_done = nullptr;          // end of the queued batch
    ReadOut* h_out = nullptr; size_t h_out_cap = 0;   // pinned
    unsigned char* h_multi = nullptr; size_t h_multi_cap = 0;   // pinned: the multi-chain epilogue's keys, f, pprev (16 B per anchor)
    bool mapped = false, collected = false, stop_after_sort = false, dv_separate = false;
    bool redo = false;                     // inside wait_batch's re-map (MM2G_KNOB_WS_MIN applies to first maps only)
    bool ws_exact = false;                 // anchor workspace sized to the batches' exact counts (HBM was short)
    bool lb_ran0 = false;                  // the last map launched pass 0's k_chain_lb (counter 14)
    uint64_t n_anchors = 0;
    KeyLayout kl{};
    mm2g_map_opts last_opts{};
    std::vector<int16_t> h_lut; float lut_gap = -1; int lut_n = 0; bool lut_dirty = true; void* lut_dev = nullptr;
    bool debug = false;
    bool full_last = false;                // the last map kept every anchor (debug mode or multi-chain output)
    bool filt_last = false;                // the last map's sort ran the singleton-filter cell path
    uint32_t small_last = 0;               // ... and handed reads of 2..small_last anchors to k_sort_small
    bool multi_last = false;               // ... and its results come from the multi-chain epilogue (-n <= 1, -m <= k)
    std::vector<mm2g::MultiRead> multi;    // per read of the last collected multi-chain batch
    std::vector<mm2g_read_result> h_res;   // per-read results of the last collected batch (mm2g_batch_paf)
    // profiling
    bool prof = false;
    std::vector<ProfSlot> slots;
    std::map<std::string, int> slot_ix;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::vector<hipEvent_t> ev_pool; size_t ev_next = 0;
    uint64_t counters[MM2G_N_COUNTERS] = {};

    hipEvent_t ev() {
        if (ev_next == ev_pool.size()) { hipEvent_t e; (void)hipEventCreate(&e); ev_pool.push_back(e); }
        return ev_pool[ev_next++];
    }
    int prof_begin(const char* name, hipEvent_t& e0) {
        if (!prof) return -1;
        auto it = slot_ix.find(name);
        int i;
        if (it == slot_ix.end()) { i = (int)slots.size(); slots.push_back(ProfSlot{name}); slot_ix[name] = i; } else i = it->second;
        e0 = ev(); (void)hipEventRecord(e0, stream);
        return i;
    }
    void prof_end(int i, hipEvent_t e0) {
        if (i < 0) return;
        hipEvent_t e1 = ev(); (void)hipEventRecord(e1, stream);
        pending.push_back({i, {e0, e1}});
    }
    void prof_collect() {
        if (pending.empty()) { ev_next = 0; return; }
        (void)hipEventSynchronize(pending.back().second.second);
        for (auto& p : pending) {
            float ms = 0; (void)hipEventElapsedTime(&ms, p.second.first, p.second.second);
            slots[p.first].ms += ms; slots[p.first].calls += 1;
        }
        pending.clear(); ev_next = 0;
    }
};

// MM2G_KNOB_SYNC_EACH: synchronise after every stage and report the first
// failing stage (and, in MM2G_CHECKED builds, the first out-of-range index).
struct ProfScope {
    mm2g_ctx* c; int i; hipEvent_t e0{}; const char* name;
    ProfScope(mm2g_ctx* c_, const char* n) : c(c_), name(n) { i = c->prof_begin(n, e0); }
    ~ProfScope() {
        c->prof_end(i, e0);
        if (c->knob[MM2G_KNOB_SYNC_EACH]) {
            unsigned long long ck[4] = {0, 0, 0, 0};
            int e = mm2g_checked_read(ck, c->stream);
            if (e != 0 || ck[0] != 0) {
                fprintf(stderr, "[mm2g] stage %s: hip=%d (%s) check line=%llu idx=%llu cap=%llu\n", name, e,
                        hipGetErrorString((hipError_t)e), ck[0], ck[1], ck[2]);
                fflush(stderr);
            }
        }
    }
};

// MM2G_KNOB_SORT_PROF: phase times of k_sort_read (wall clock, 100 MHz) to stderr
static void dump_sort_prof(mm2g_ctx* c, uint64_t* d, uint32_t n) {
    std::vector<uint64_t> h((size_t)n * 24);
    if (hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) return;
    (void)hipFree(d);
    double ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tot = 0, a0 = 0, a2 = 0, np = 0, nleg = 0, nbigp = 0, ktiny = 0, klong = 0, ksrch = 0;
    uint64_t t_lo = ~0ULL, t_hi = 0;
    uint32_t m = 0;
    std::vector<uint32_t> q0, q2, q3;
    for (uint32_t r = 0; r < n; ++r) {
        const uint64_t* p = &h[(size_t)r * 24];
        if (!p[11]) continue;
        q3.push_back((uint32_t)p[13]);
        ++m;
        for (int k = 0; k < 8; ++k) ph[k] += (double)p[k];
        tot += (double)(p[11] - p[10]);
        a0 += (double)p[8]; a2 += (double)(uint32_t)p[9];
        if ((p[9] >> 32) == 0xffffu) nleg += 1;
        else if ((p[9] >> 32) == 0xfffeu) nbigp += 1;
        else np += (double)(p[9] >> 32);
        t_lo = std::min(t_lo, p[10]); t_hi = std::max(t_hi, p[11]);
        q0.push_back((uint32_t)p[8]); q2.push_back((uint32_t)p[9]);
        ktiny += (double)(uint32_t)p[14]; klong += (double)(p[14] >> 32); ksrch += (double)p[15];
    }
    if (!m) return;
    std::sort(q0.begin(), q0.end()); std::sort(q2.begin(), q2.end()); std::sort(q3.begin(), q3.end());
    auto Q = [](const std::vector<uint32_t>& v, double f) { return v[std::min(v.size() - 1, (size_t)(f * v.size()))]; };
    fprintf(stderr, "[sort_prof] A0 q10/50/90/99/max=%u/%u/%u/%u/%u  A q10/50/90/99/max=%u/%u/%u/%u/%u  kept cells q10/50/90/99/max=%u/%u/%u/%u/%u\n",
            Q(q0, .1), Q(q0, .5), Q(q0, .9), Q(q0, .99), q0.back(), Q(q2, .1), Q(q2, .5), Q(q2, .9), Q(q2, .99), q2.back(),
            Q(q3, .1), Q(q3, .5), Q(q3, .9), Q(q3, .99), q3.back());
    fprintf(stderr, "[sort_prof] reads=%u (whole-read radix %.0f, bucket path %.0f) A0=%.0f A=%.0f nbig=%.2f windows=%.2f us/read: p1+kc=%.1f p2=%.1f gather=%.1f fuse_stage=%.1f chunk=%.1f rank=%.1f p4b/radix=%.1f total=%.1f span_us=%.1f concurrency=%.1f\n",
            m, nleg, nbigp, a0 / m, a2 / m, np / m, ph[7] / m, ph[0] / m / 100, ph[1] / m / 100, ph[2] / m / 100, ph[3] / m / 100, ph[4] / m / 100,
            ph[5] / m / 100, ph[6] / m / 100, tot / m / 100, (double)(t_hi - t_lo) / 100, tot / (double)(t_hi - t_lo));
    fprintf(stderr, "[sort_prof] keys per read in segments <= %u: %.0f, 17..64: %.0f, > 64: %.0f (%.2f other-chunk searches each)\n",
            16u, ktiny / m, (a2 - ktiny - klong) / m, klong / m, klong > 0 ? ksrch / klong : 0.0);
}

// MM2G_SKETCH_PROF: phase times of k_sketch summed over each read's tiles
static void dump_sketch_prof(mm2g_ctx* c, uint64_t* d, uint32_t n) {
    std::vector<uint64_t> h((size_t)n * 8);
    if (hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) return;
    (void)hipFree(d);
    double ph[5] = {0, 0, 0, 0, 0}, L = 0;
    uint32_t m = 0;
    uint64_t t_hi = 0, tiles = 0, slow = 0;
    for (uint32_t r = 0; r < n; ++r) {
        const uint64_t* p = &h[(size_t)r * 8];
        if (!p[5]) continue;
        ++m;
        tiles += p[7] >> 32; slow += p[7] & 0xffffffffULL;
        for (int k = 0; k < 5; ++k) ph[k] += (double)p[k];
        L += (double)p[5];
        t_hi = std::max(t_hi, p[6]);
    }
    if (!m) return;
    double tot = ph[0] + ph[1] + ph[2] + ph[3] + ph[4];
    fprintf(stderr, "[sketch_prof] reads=%u len=%.0f us/read: stage=%.1f warmup=%.1f phase1=%.1f phase2=%.1f tail=%.1f total=%.1f; exact-path tiles %.1f%%\n",
            m, L / m, ph[0] / m / 100, ph[1] / m / 100, ph[2] / m / 100, ph[3] / m / 100, ph[4] / m / 100, tot / m / 100,
            tiles ? 100.0 * (double)slow / (double)tiles : 0.0);
}

static inline uint32_t bit_width(uint64_t x) { uint32_t b = 0; while (x) { ++b; x >>= 1; } return b; }
static inline int grid_for(uint32_t n) { int b = (int)((n + 3) / 4); return std::max(1, std::min(b, 4096)); }

template <size_t N>
static inline char* put_lit(char* p, const char (&lit)[N]) {
    memcpy(p, lit, N - 1);
    return p + (N - 1);
}

extern "C" {

int mm2g_version(void) { return 1; }
const char* mm2g_last_error(void) { return g_err.c_str(); }
int mm2g_device_count(void) { int n = 0; if (hipGetDeviceCount(&n) != hipSuccess) return 0; return n; }

// ------------------------------------------------------------------ index API
int mm2g_index_build_fasta(const char* path, int w, int k, int b, int flag, int n_threads, mm2g_index** out) {
    if (!path || !out) return set_err(MM2G_E_ARG, "null argument");
    std::vector<FastaRecord> recs; std::string err;
    if (!read_fasta(path, recs, false, err)) return set_err(MM2G_E_IO, "%s", err.c_str());
    std::vector<const uint8_t*> seqs; std::vector<uint64_t> lens; std::vector<std::string> names;
    for (auto& r : recs) { seqs.push_back((const uint8_t*)r.seq.data()); lens.push_back(r.seq.size()); names.push_back(r.name); }
    std::unique_ptr<mm2g_index> I(new mm2g_index());
    if (!build_index(seqs, lens, &names, w, k, b, flag, n_threads, I->h, err)) return set_err(MM2G_E_ARG, "%s", err.c_str());
    I->origin = MM2G_IX_HOST;
    *out = I.release();
    return 0;
}

int mm2g_index_build_seqs(uint32_t n_seq, const char* const* names, const uint8_t* const* seqs, const uint64_t* lens,
                          int w, int k, int b, int flag, int n_threads, mm2g_index** out) {
    if (!out || (n_seq && (!seqs || !lens))) return set_err(MM2G_E_ARG, "null argument");
    std::vector<const uint8_t*> s(seqs, seqs + n_seq);
    std::vector<uint64_t> l(lens, lens + n_seq);
    std::vector<std::string> nm;
    if (names) for (uint32_t i = 0; i < n_seq; ++i) nm.push_back(names[i] ? names[i] : "");
    std::unique_ptr<mm2g_index> I(new mm2g_index());
    std::string err;
    if (!build_index(s, l, names ? &nm : nullptr, w, k, b, flag, n_threads, I->h, err)) return set_err(MM2G_E_ARG, "%s", err.c_str());
    I->origin = MM2G_IX_HOST;
    *out = I.release();
    return 0;
}

// The GPU index build; where the device cannot do it (minimizer slot overflow,
// or MM2G_IKNOB_FORCE_FALLBACK in tests) the host builds the same index and the
// index records it (mm2g_index_origin: MM2G_IX_GPU_FALLBACK and the reason).
static int build_gpu_or_host(int device, const std::vector<const uint8_t*>& seqs, const std::vector<uint64_t>& lens,
                             const std::vector<std::string>* names, int w, int k, int b, int flag, int n_threads, mm2g_index** out) {
    std::unique_ptr<mm2g_index> I(new mm2g_index());
    std::string err;
    bool unsupported = false;
    bool ok;
    if (g_index_knob[MM2G_IKNOB_FORCE_FALLBACK].load()) {
        ok = false; unsupported = true; err = "GPU index build: host fallback forced (MM2G_IKNOB_FORCE_FALLBACK)";
    } else {
        ok = build_index_gpu(device, seqs, lens, names, w, k, b, flag, I->h, err, unsupported);
    }
    I->origin = MM2G_IX_GPU;
    if (!ok) {
        if (!unsupported) return set_err(MM2G_E_HIP, "%s", err.c_str());
        if (g_index_knob[MM2G_IKNOB_GPU_STRICT].load()) return set_err(MM2G_E_UNSUP, "%s", err.c_str());
        const std::string why = err;
        if (!build_index(seqs, lens, names, w, k, b, flag, n_threads, I->h, err)) return set_err(MM2G_E_ARG, "%s", err.c_str());
        I->origin = MM2G_IX_GPU_FALLBACK;
        I->origin_note = why;
    }
    *out = I.release();
    return 0;
}

int mm2g_index_build_fasta_gpu(const char* path, int w, int k, int b, int flag, int device, int n_threads, mm2g_index** out) {
    if (!path || !out) return set_err(MM2G_E_ARG, "null argument");
    std::vector<FastaRecord> recs; std::string err;
    if (!read_fasta(path, recs, false, err)) return set_err(MM2G_E_IO, "%s", err.c_str());
    std::vector<const uint8_t*> seqs; std::vector<uint64_t> lens; std::vector<std::string> names;
    for (auto& r : recs) { seqs.push_back((const uint8_t*)r.seq.data()); lens.push_back(r.seq.size()); names.push_back(r.name); }
    return build_gpu_or_host(device, seqs, lens, &names, w, k, b, flag, n_threads, out);
}

int mm2g_index_build_seqs_gpu(uint32_t n_seq, const char* const* names, const uint8_t* const* seqs, const uint64_t* lens,
                              int w, int k, int b, int flag, int device, int n_threads, mm2g_index** out) {
    if (!out || (n_seq && (!seqs || !lens))) return set_err(MM2G_E_ARG, "null argument");
    std::vector<const uint8_t*> s(seqs, seqs + n_seq);
    std::vector<uint64_t> l(lens, lens + n_seq);
    std::vector<std::string> nm;
    if (names) for (uint32_t i = 0; i < n_seq; ++i) nm.push_back(names[i] ? names[i] : "");
    return build_gpu_or_host(device, s, l, names ? &nm : nullptr, w, k, b, flag, n_threads, out);
}

int mm2g_index_load_mmi(const char* path, mm2g_index** out) {
    if (!path || !out) return set_err(MM2G_E_ARG, "null argument");
    std::unique_ptr<mm2g_index> I(new mm2g_index());
    std::string err;
    if (!load_mmi(path, I->h, err)) return set_err(MM2G_E_IO, "%s", err.c_str());
    I->origin = MM2G_IX_MMI;
    *out = I.release();
    return 0;
}
int mm2g_index_save_mmi(const mm2g_index* idx, const char* path) {
    if (!idx || !path) return set_err(MM2G_E_ARG, "null argument");
    if (int e = need_tables(idx)) return e;
    std::string err;
    if (!save_mmi(idx->h, path, err)) return set_err(MM2G_E_IO, "%s", err.c_str());
    return 0;
}
void mm2g_index_free(mm2g_index* idx) { delete idx; }
int mm2g_index_stats(const mm2g_index* idx, uint64_t* n_keys, double* avg_occ, double* avg_spacing, uint64_t* total_len) {
    if (!idx) return set_err(MM2G_E_ARG, "null index");
    uint64_t a, d; double b, c;
    if (idx->released) { a = idx->st_keys; b = idx->st_occ; c = idx->st_spacing; d = idx->st_total; }
    else idx->h.stats(a, b, c, d);
    if (n_keys) *n_keys = a; if (avg_occ) *avg_occ = b; if (avg_spacing) *avg_spacing = c; if (total_len) *total_len = d;
    return 0;
}
int mm2g_index_calc_mid_occ(const mm2g_index* idx, float frac, int32_t* out) {
    if (!idx || !out) return set_err(MM2G_E_ARG, "null argument");
    if (int e = need_tables(idx)) return e;
    *out = idx->h.calc_mid_occ(frac);
    return 0;
}
int mm2g_index_params(const mm2g_index* idx, int32_t* w, int32_t* k, int32_t* b, int32_t* flag, uint32_t* n_seq) {
    if (!idx) return set_err(MM2G_E_ARG, "null index");
    if (w) *w = idx->h.w; if (k) *k = idx->h.k; if (b) *b = idx->h.b; if (flag) *flag = idx->h.flag; if (n_seq) *n_seq = idx->h.n_seq;
    return 0;
}
int mm2g_index_seq(const mm2g_index* idx, uint32_t rid, const char** name, uint32_t* len) {
    if (!idx || rid >= idx->h.seq.size()) return set_err(MM2G_E_ARG, "rid out of range");
    if (name) *name = idx->h.seq[rid].has_name ? idx->h.seq[rid].name.c_str() : nullptr;
    if (len) *len = idx->h.seq[rid].len;
    return 0;
}
int64_t mm2g_index_get(const mm2g_index* idx, uint64_t minier, int* kind, uint64_t* out, int64_t cap) {
    if (!idx || !kind) return set_err(MM2G_E_ARG, "null argument");
    if (int e = need_tables(idx)) return e;
    const uint64_t* pos; size_t n; uint64_t single;
    idx->h.get(minier, *kind, pos, n, single);
    for (size_t i = 0; i < n && (int64_t)i < cap; ++i) out[i] = pos[i];
    return (int64_t)n;
}

int mm2g_index_origin(const mm2g_index* idx, const char** note) {
    if (!idx) return set_err(MM2G_E_ARG, "null index");
    if (note) *note = idx->origin_note.empty() ? nullptr : idx->origin_note.c_str();
    return idx->origin;
}
int mm2g_index_release_tables(mm2g_index* idx) {
    if (!idx) return set_err(MM2G_E_ARG, "null index");
    if (idx->released) return 0;
    idx->h.stats(idx->st_keys, idx->st_occ, idx->st_spacing, idx->st_total);
    std::vector<HostBucket>().swap(idx->h.B);
    SVec().swap(idx->h.S);
    idx->released = true;
    return 0;
}

// ------------------------------------------------------------------ context
int mm2g_ctx_create(int device, mm2g_ctx** out) {
    if (!out) return set_err(MM2G_E_ARG, "null argument");
    int nd = 0;
    HIPCHK(hipGetDeviceCount(&nd));
    if (device < 0 || device >= nd) return set_err(MM2G_E_ARG, "device %d out of range (%d devices)", device, nd);
    HIPCHK(hipSetDevice(device));
    std::unique_ptr<mm2g_ctx> c(new mm2g_ctx());
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipHostMalloc((void**)&c->h_stat, STAT_WORDS * sizeof(uint64_t), hipHostMallocDefault));
    HIPCHK(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
    for (auto& S : c->stage) HIPCHK(hipEventCreateWithFlags(&S.ev, hipEventDisableTiming));
    for (int k = 0; k < MM2G_KNOB_COUNT; ++k) c->knob[k] = knob_default(k);
    *out = c.release();
    return 0;
}
void mm2g_ctx_destroy(mm2g_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->h_stat) (void)hipHostFree(c->h_stat);
    for (auto& S : c->stage) { if (S.p) (void)hipHostFree(S.p); if (S.ev) (void)hipEventDestroy(S.ev); }
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->h_out) (void)hipHostFree(c->h_out);
    if (c->h_multi) (void)hipHostFree(c->h_multi);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

// The index in the device layout's input form: per distinct key (key, off, n)
// with Singles inline (IxEntry), and the positions of the Multis.  Built once
// per upload call, however many devices receive it.
struct FlatIndex { std::vector<uint64_t> keys, pos; std::vector<uint32_t> offs, ns; };
static int flatten_index(const mm2g_index* idx, FlatIndex& F) {
    if (int e = need_tables(idx)) return e;
    const HostIndex& H = idx->h;
    if (H.max_len >= (1u << 31)) return set_err(MM2G_E_UNSUP, "reference sequences must be shorter than 2^31");
    if (H.n_seq >= IX_INLINE) return set_err(MM2G_E_UNSUP, "2^31 or more reference sequences");
    H.flatten(F.keys, F.offs, F.ns, F.pos);
    if (F.pos.size() >= (1ULL << 32)) return set_err(MM2G_E_UNSUP, "more than 2^32 index positions");
    for (size_t t = 0; t < F.keys.size(); ++t)          // Singles: the position inline (IxEntry)
        if (F.ns[t] == 1) { const uint64_t p = F.pos[F.offs[t]]; F.offs[t] = (uint32_t)p; F.ns[t] = IX_INLINE | (uint32_t)(p >> 32); }
    return 0;
}

// The device copy is built into a staged DevIndex; the context switches to it
// (commit_flat) only once it is complete, so a failed upload leaves the context
// on its previous index.
struct StagedIndex { std::shared_ptr<mm2g_ctx::DevIndex> dix; uint32_t l2 = 0; };

static int stage_flat(mm2g_ctx* c, const HostIndex& H, const FlatIndex& F, StagedIndex& S) {
    HIPCHK(hipSetDevice(c->device));
    const uint64_t nk = F.keys.size();
    uint32_t l2 = 2;                                               // >= one 4-slot probe group (k_seed_count)
    while ((1ULL << l2) < 2 * std::max<uint64_t>(nk, 1)) ++l2;     // load factor <= 0.5
    if (l2 > 31) return set_err(MM2G_E_UNSUP, "index too large for the device table");
    IxEntry* tab; uint64_t* dpos;
    S.dix = std::make_shared<mm2g_ctx::DevIndex>();     // a fresh copy (contexts sharing the old one keep it)
    S.l2 = l2;
    ENSURE(S.dix->tab, IxEntry, (size_t)1 << l2, tab);
    ENSURE(S.dix->ix_pos, uint64_t, F.pos.size(), dpos);
    HIPCHK(hipMemsetAsync(tab, 0xff, sizeof(IxEntry) << l2, c->stream));
    if (!F.pos.empty()) HIPCHK(hipMemcpyAsync(dpos, F.pos.data(), F.pos.size() * 8, hipMemcpyHostToDevice, c->stream));
    DevBuf dk, doff, dn;
    uint64_t* k_; uint32_t* o_; uint32_t* n_;
    ENSURE(dk, uint64_t, nk, k_); ENSURE(doff, uint32_t, nk, o_); ENSURE(dn, uint32_t, nk, n_);
    if (nk) {
        HIPCHK(hipMemcpyAsync(k_, F.keys.data(), nk * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(o_, F.offs.data(), nk * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(n_, F.ns.data(), nk * 4, hipMemcpyHostToDevice, c->stream));
    }
    LCHK(launch_ix_build(k_, o_, n_, nk, tab, l2, c->stream));
    // singleton-filter cells: per group (fwd, rev) a guard cell, ceil(len / 2^CELL_SHIFT) cells, a guard cell
    {
        std::vector<uint32_t> goff(2 * (size_t)H.n_seq + 2);
        uint64_t run = 0;
        for (uint32_t g = 0; g < 2 * H.n_seq; ++g) {
            goff[g] = (uint32_t)std::min<uint64_t>(run, 0xffffffffu);
            run += ((uint64_t)H.seq[g % H.n_seq].len >> CELL_SHIFT) + 3;
        }
        // the Q19 pseudo-group 2 * n_seq (odd rids, both strands, rpos = pos)
        goff[2 * H.n_seq] = (uint32_t)std::min<uint64_t>(run, 0xffffffffu);
        run += ((uint64_t)H.max_len >> CELL_SHIFT) + 3;
        goff[2 * H.n_seq + 1] = (uint32_t)std::min<uint64_t>(run, 0xffffffffu);
        // two bitmaps must fit the LDS budget of k_sort_read next to its static arrays
        S.dix->cells = (run <= (uint64_t)MAX_CELLS) ? (uint32_t)run : 0u;
        uint32_t* dg;
        ENSURE(S.dix->goff, uint32_t, goff.size(), dg);
        HIPCHK(hipMemcpyAsync(dg, goff.data(), goff.size() * 4, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

static void commit_flat(mm2g_ctx* c, const HostIndex& H, StagedIndex& S, int32_t mid_occ) {
    c->mapped = false;
    c->dix = std::move(S.dix);
    c->log2cap = S.l2;
    c->hidx = &H;
    c->mid_occ = mid_occ;
    c->have_index = true;
}

int mm2g_ctx_upload_index(mm2g_ctx* c, const mm2g_index* idx, int32_t mid_occ) {
    if (!c || !idx) return set_err(MM2G_E_ARG, "null argument");
    FlatIndex F;
    if (int e = flatten_index(idx, F)) return e;
    StagedIndex S;
    if (int e = stage_flat(c, idx->h, F, S)) return e;
    commit_flat(c, idx->h, S, mid_occ);
    return 0;
}

// One flatten, then every context's copy (normally one per GPU) in its own
// host thread: the H2D copies and table builds of the devices overlap.  All or
// nothing: the contexts switch to the new index only when every copy is done.
int mm2g_ctx_upload_index_many(mm2g_ctx* const* ctxs, int n, const mm2g_index* idx, int32_t mid_occ) {
    if (!ctxs || n < 0 || !idx) return set_err(MM2G_E_ARG, "null argument");
    for (int i = 0; i < n; ++i) if (!ctxs[i]) return set_err(MM2G_E_ARG, "null context %d", i);
    FlatIndex F;
    if (int e = flatten_index(idx, F)) return e;
    std::vector<int> rc(n, 0);
    std::vector<std::string> msg(n);
    std::vector<StagedIndex> S(n);
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i)
        th.emplace_back([&, i] { rc[i] = stage_flat(ctxs[i], idx->h, F, S[i]); if (rc[i]) msg[i] = g_err; });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[i]) return set_err(rc[i], "device %d: %s", ctxs[i]->device, msg[i].c_str());
    for (int i = 0; i < n; ++i) commit_flat(ctxs[i], idx->h, S[i], mid_occ);
    return 0;
}

int mm2g_ctx_share_index(mm2g_ctx* dst, const mm2g_ctx* src, int32_t mid_occ) {
    if (!dst || !src) return set_err(MM2G_E_ARG, "null argument");
    if (!src->have_index) return set_err(MM2G_E_STATE, "source context has no index");
    if (dst->device != src->device) return set_err(MM2G_E_ARG, "contexts are on different devices");
    dst->mapped = false;
    dst->dix = src->dix;
    dst->log2cap = src->log2cap;
    dst->hidx = src->hidx;
    dst->mid_occ = mid_occ;
    dst->have_index = true;
    return 0;
}

// Index::calc_mid_occ (src/index.rs:124-141) from the uploaded device table
// (SURVEY.md §8f row 2): a histogram of per-key occurrence counts instead of the
// reference's sort of all of them; counts at or above the last bin are gathered
// and sorted only if the quantile lands among them.
int mm2g_ctx_index_mid_occ(mm2g_ctx* c, float frac, int32_t* out) {
    if (!c || !out) return set_err(MM2G_E_ARG, "null argument");
    if (!c->have_index) return set_err(MM2G_E_STATE, "no index uploaded");
    HIPCHK(hipSetDevice(c->device));
    uint32_t nbins = 4096;
    nbins = (uint32_t)std::max<int64_t>(2, std::min<int64_t>(16384, c->knob[MM2G_KNOB_MIDHIST_BINS]));
    const uint64_t cap = 1ULL << c->log2cap;
    const IxEntry* tab = (const IxEntry*)c->dix->tab.p;
    DevBuf dh, dn, dv;
    unsigned long long* hist; uint32_t* n_ovf;
    ENSURE(dh, unsigned long long, nbins, hist);
    ENSURE(dn, uint32_t, 1, n_ovf);
    HIPCHK(hipMemsetAsync(hist, 0, (size_t)nbins * 8, c->stream));
    HIPCHK(hipMemsetAsync(n_ovf, 0, 4, c->stream));
    LCHK(launch_mid_hist(tab, cap, nbins, hist, nullptr, 0, n_ovf, c->stream));
    std::vector<unsigned long long> h(nbins);
    uint32_t no = 0;
    HIPCHK(hipMemcpyAsync(h.data(), hist, (size_t)nbins * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&no, n_ovf, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    uint64_t n = no;
    for (auto v : h) n += v;
    if (n == 0) { *out = INT32_MAX; return 0; }
    const double f = (1.0 - (double)frac) * (double)n;
    uint64_t i = f <= 0.0 ? 0 : (uint64_t)f;
    if (i > n - 1) i = n - 1;
    uint64_t run = 0;
    for (uint32_t v = 0; v < nbins; ++v) {
        if (i < run + h[v]) { *out = (int32_t)v + 1; return 0; }
        run += h[v];
    }
    uint32_t* ovf;
    ENSURE(dv, uint32_t, no, ovf);
    HIPCHK(hipMemsetAsync(hist, 0, (size_t)nbins * 8, c->stream));
    HIPCHK(hipMemsetAsync(n_ovf, 0, 4, c->stream));
    LCHK(launch_mid_hist(tab, cap, nbins, hist, ovf, no, n_ovf, c->stream));
    std::vector<uint32_t> ov(no);
    if (no) HIPCHK(hipMemcpyAsync(ov.data(), ovf, (size_t)no * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    std::nth_element(ov.begin(), ov.begin() + (i - run), ov.end());
    *out = (int32_t)ov[i - run] + 1;
    return 0;
}

int mm2g_ctx_set_mid_occ(mm2g_ctx* c, int32_t mid_occ) {
    if (!c) return set_err(MM2G_E_ARG, "null argument");
    c->mid_occ = mid_occ;
    c->mapped = false;      // a mapped batch's anchors used the old mid_occ
    return 0;
}

// ------------------------------------------------------------------ batch
void mm2g_map_opts_default(mm2g_map_opts* o) {
    o->w = 10; o->k = 15; o->max_gap = 5000; o->bw = 500; o->bw_long = 20000;
    o->min_cnt = 3; o->min_chain_score = 40; o->mask_level = 0.5f; o->pri_ratio = 0.8f; o->best_n = 5;
}

uint64_t mm2g_nt4_words_bound(const uint64_t* offs, uint32_t n_reads) { return offs ? nt4_words_bound(offs, n_reads) : 0; }
int64_t mm2g_nt4_pack(const uint8_t* seq, const uint64_t* offs, uint32_t n_reads, uint64_t* pk_off, uint64_t* amb_off, uint64_t* words,
                      uint64_t cap_words, int n_threads) {
    if (n_reads && (!seq || !offs || !pk_off || !amb_off || !words)) return set_err(MM2G_E_ARG, "null argument");
    for (uint32_t i = 0; i < n_reads; ++i)
        if (offs[i + 1] < offs[i]) return set_err(MM2G_E_ARG, "offsets must be non-decreasing");
    const int64_t w = nt4_pack(seq, offs, n_reads, pk_off, amb_off, words, cap_words, std::max(1, n_threads));
    if (w < 0) return set_err(MM2G_E_ARG, "output capacity too small (%lld words needed at least)", (long long)-w);
    return w;
}

// Record the batch geometry and queue the H2D copy of the staged buffer
// (header + nt4 words) on the context stream.
static int stage_commit(mm2g_ctx* c, Stage& S, uint32_t n, uint64_t total_words, std::vector<uint64_t>& ro, uint32_t mx) {
    c->mapped = false;
    uint64_t* d;
    ENSURE(c->rd_dev, uint64_t, total_words, d);
    HIPCHK(hipMemcpyAsync(d, S.p, total_words * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipEventRecord(S.ev, c->stream));
    S.pending = true;
    c->st_next ^= 1;
    c->h_rd_off.swap(ro);
    c->max_read_len = mx;
    c->d_rd_off = d; c->d_pk_off = d + n + 1; c->d_amb_off = d + 2 * (size_t)n + 1; c->d_words = d + 3 * (size_t)n + 1;
    c->n_reads = n; c->total_bases = c->h_rd_off[n];
    c->sk1.exact = c->sk2.exact = false;
    return 0;
}

// The next free pinned staging buffer with room for `words` u64 (waits for its last H2D).
static int stage_acquire(mm2g_ctx* c, uint64_t words, Stage** out) {
    Stage& S = c->stage[c->st_next];
    if (S.pending) { HIPCHK(hipEventSynchronize(S.ev)); S.pending = false; }
    if (S.cap < words) {
        if (S.p) (void)hipHostFree(S.p);
        S.p = nullptr; S.cap = 0;
        const uint64_t nc = words + words / 4 + 1024;
        HIPCHK(hipHostMalloc((void**)&S.p, nc * 8, hipHostMallocDefault));
        S.cap = nc;
    }
    *out = &S;
    return 0;
}

// Validates the offsets into `ro` (relative, n+1) and the longest read; the
// context takes them only in stage_commit, so a failed call leaves the
// previous batch's geometry intact.
static int check_offsets(const uint64_t* offs, uint32_t n, std::vector<uint64_t>& ro, uint32_t& mx) {
    ro.assign((size_t)n + 1, 0);
    mx = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (offs[i + 1] < offs[i]) return set_err(MM2G_E_ARG, "offsets must be non-decreasing");
        const uint64_t L = offs[i + 1] - offs[i];
        if (L >= (1ULL << 31)) return set_err(MM2G_E_UNSUP, "reads must be shorter than 2^31");
        mx = std::max<uint32_t>(mx, (uint32_t)L);
        ro[i + 1] = ro[i] + L;
    }
    return 0;
}

int mm2g_batch_set_reads(mm2g_ctx* c, const uint8_t* seq, const uint64_t* offs, uint32_t n_reads) {
    if (!c || (n_reads && (!seq || !offs))) return set_err(MM2G_E_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    static const uint64_t zero = 0;
    if (!n_reads) offs = &zero;
    std::vector<uint64_t> ro; uint32_t mx;
    if (int e = check_offsets(offs, n_reads, ro, mx)) return e;
    const uint64_t hdr = 3 * (uint64_t)n_reads + 1;
    Stage* S;
    if (int e = stage_acquire(c, hdr + nt4_words_bound(offs, n_reads), &S)) return e;
    uint64_t* h = S->p;
    memcpy(h, ro.data(), ((size_t)n_reads + 1) * 8);
    const int64_t nw = nt4_pack(seq, offs, n_reads, h + n_reads + 1, h + 2 * (size_t)n_reads + 1, h + hdr, S->cap - hdr,
                                (int)c->knob[MM2G_KNOB_HOST_THREADS]);
    if (nw < 0) return set_err(MM2G_E_NOMEM, "nt4 staging too small");
    return stage_commit(c, *S, n_reads, hdr + (uint64_t)nw, ro, mx);
}

int mm2g_batch_set_reads_nt4(mm2g_ctx* c, const mm2g_nt4_batch* b) {
    if (!c || !b || (b->n_reads && (!b->lens || !b->pk_off || !b->amb_off || !b->words)))
        return set_err(MM2G_E_ARG, "null argument");
    HIPCHK(hipSetDevice(c->device));
    const uint32_t n = b->n_reads;
    std::vector<uint64_t> offs((size_t)n + 1, 0);
    for (uint32_t r = 0; r < n; ++r) {
        const uint64_t L = b->lens[r];
        if (b->pk_off[r] + (L + 31) / 32 > b->n_words) return set_err(MM2G_E_ARG, "read %u: codes beyond n_words", r);
        if (b->amb_off[r] != ~0ULL && b->amb_off[r] + (L + 63) / 64 > b->n_words) return set_err(MM2G_E_ARG, "read %u: bitmap beyond n_words", r);
        offs[r + 1] = offs[r] + L;
    }
    std::vector<uint64_t> ro; uint32_t mx;
    if (int e = check_offsets(offs.data(), n, ro, mx)) return e;
    const uint64_t hdr = 3 * (uint64_t)n + 1;
    Stage* S;
    if (int e = stage_acquire(c, hdr + b->n_words, &S)) return e;
    uint64_t* h = S->p;
    memcpy(h, ro.data(), ((size_t)n + 1) * 8);
    if (n) {
        memcpy(h + n + 1, b->pk_off, (size_t)n * 8);
        memcpy(h + 2 * (size_t)n + 1, b->amb_off, (size_t)n * 8);
    }
    if (b->n_words) memcpy(h + hdr, b->words, b->n_words * 8);
    return stage_commit(c, *S, n, hdr + b->n_words, ro, mx);
}

// Sketch the resident batch into sk's slots (one slot of L+16 per read, or the
// exact layout a previous overflow recorded).  A read whose minimizers do not
// fit is clamped and flagged in *ovf; mm2g_batch_results re-runs the batch.
static int run_sketch(mm2g_ctx* c, int w, int k, SketchBufs& B, int32_t* ovf, ReadOut* zout = nullptr, unsigned long long* zst = nullptr) {
    const uint32_t n = c->n_reads;
    uint64_t *base, *end, *x; uint32_t *y, *cnt, *need;
    ENSURE(B.base, uint64_t, n + 1, base); ENSURE(B.end, uint64_t, n + 1, end);
    ENSURE(B.cnt, uint32_t, n + 1, cnt); ENSURE(B.need, uint32_t, n + 1, need);
    const uint32_t slot = c->redo ? 0u : (uint32_t)std::max<int64_t>(0, std::min<int64_t>(c->knob[MM2G_KNOB_WS_MIN], 1 << 30));
    if (!B.exact) B.cap = slot ? (uint64_t)slot * n + 16 : c->total_bases + 16ull * n + 16;
    ENSURE(B.x, uint64_t, B.cap, x); ENSURE(B.y, uint32_t, B.cap, y);
    // query views (odd k only: the fixed warm-up is exact there; a re-run
    // after a slot overflow has them off, so the exact per-read layout needs one pass)
    const uint32_t V = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(c->knob[MM2G_KNOB_SKETCH_VIEW], 1 << 30));
    // ... and only for batches too small to fill the GPU with one wave per read
    // (C2's 500-read units; C3's 5,000-read units measured 4 % slower with views)
    const bool few = (int64_t)n < c->knob[MM2G_KNOB_VIEW_READS];
    const bool views = V >= 64 && (k & 1) && few && !c->views_off && c->max_read_len > V && !c->knob[MM2G_KNOB_SKETCH_PROF] && !slot;
    if (!B.exact) {   // (zout / zst: the batch's outputs and status block are cleared here too)
        if (!views) {   // (with views: k_view_plan does it)
            ProfScope ps(c, "mz_base");
            LCHK(launch_mz_base(n, c->d_rd_off, base, end, slot, c->stream, zout, zst, STAT_WORDS));
        }
    } else {
        if (zout) HIPCHK(hipMemsetAsync(zout, 0, sizeof(ReadOut) * ((size_t)n + 1), c->stream));
        if (zst) HIPCHK(hipMemsetAsync(zst, 0, STAT_WORDS * 8, c->stream));
    }
    SketchArgs a{nullptr, c->d_rd_off, n, w, k, base, end, x, y, cnt, ovf};
    a.x64 = c->knob[MM2G_KNOB_SKETCH_X32] ? 0u : 1u;
    a.pk_words = c->d_words; a.pk_off = c->d_pk_off; a.amb_off = c->d_amb_off; a.mz_need = need;
    if (views) {
        const uint32_t W0 = (uint32_t)((2 * (w + k) + 64 + 7) & ~7);
        const uint64_t nvmax = (uint64_t)n + c->total_bases / V + 1;
        uint32_t *v_read, *v_len, *v_pre, *v_from, *v_cnt, *v_need; uint64_t *v_off, *v_base, *v_end, *vo, *vx; uint8_t* v_last; uint32_t* vy;
        ViewBufs& Vb = c->vw;
        ENSURE(Vb.read, uint32_t, nvmax, v_read); ENSURE(Vb.len, uint32_t, nvmax, v_len); ENSURE(Vb.pre, uint32_t, nvmax, v_pre);
        ENSURE(Vb.from, uint32_t, nvmax, v_from); ENSURE(Vb.cnt, uint32_t, nvmax, v_cnt); ENSURE(Vb.need, uint32_t, nvmax, v_need);
        ENSURE(Vb.off, uint64_t, nvmax, v_off); ENSURE(Vb.base, uint64_t, nvmax, v_base); ENSURE(Vb.end, uint64_t, nvmax, v_end);
        ENSURE(Vb.last, uint8_t, nvmax, v_last); ENSURE(Vb.vo, uint64_t, n + 1, vo);
        const uint64_t vcap = c->total_bases + 16 * nvmax + 16;
        ENSURE(Vb.x, uint64_t, vcap, vx); ENSURE(Vb.y, uint32_t, vcap, vy);
        {
            ProfScope ps(c, "sketch_views");
            LCHK(launch_view_plan(n, c->d_rd_off, V, W0, nvmax, vo, v_read, v_off, v_len, v_pre, v_from, v_last, v_base, v_end,
                                  B.exact ? nullptr : base, end, zout, zst, STAT_WORDS, c->stream));
        }
        SketchArgs va = a;
        va.n = (uint32_t)nvmax; va.out_base = v_base; va.out_end = v_end; va.mz_x = vx; va.mz_y = vy; va.mz_cnt = v_cnt; va.mz_need = v_need;
        va.view_off = v_off; va.view_len = v_len; va.view_pre = v_pre; va.emit_from = v_from; va.view_last = v_last; va.view_read = v_read;
        {
            ProfScope ps(c, "sketch");
            LCHK(launch_sketch(va, grid_for((uint32_t)nvmax), c->stream));
        }
        ProfScope ps(c, "sketch_views");
        LCHK(launch_view_compact(n, vo, v_off, v_base, v_cnt, v_need, vx, vy, base, end, x, y, cnt, need, ovf, c->stream));
        return 0;
    }
    ProfScope ps(c, "sketch");
    uint64_t* skp = nullptr;
    if (c->knob[MM2G_KNOB_SKETCH_PROF]) { HIPCHK(hipMalloc(&skp, (size_t)n * 64)); HIPCHK(hipMemsetAsync(skp, 0, (size_t)n * 64, c->stream)); a.prof = skp; }
    LCHK(launch_sketch(a, grid_for(n), c->stream));
    if (skp) dump_sketch_prof(c, skp, n);
    return 0;
}

// After an overflow: slots sized by each read's true minimizer count.
static int sketch_exact_layout(mm2g_ctx* c, SketchBufs& B) {
    const uint32_t n = c->n_reads;
    std::vector<uint32_t> need(n);
    if (n) HIPCHK(hipMemcpyAsync(need.data(), B.need.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    std::vector<uint64_t> hb((size_t)n + 1), he((size_t)n + 1);
    uint64_t run = 0;
    for (uint32_t i = 0; i < n; ++i) { hb[i] = run; run += need[i]; he[i] = run; }
    B.cap = run + 1;
    B.exact = true;
    uint64_t *base, *end;
    ENSURE(B.base, uint64_t, n + 1, base); ENSURE(B.end, uint64_t, n + 1, end);
    if (n) {
        HIPCHK(hipMemcpyAsync(base, hb.data(), (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(end, he.data(), (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

static void build_lut(mm2g_ctx* c, float gap, int n) {
    // comput_sc penalty (src/lchain.rs:28-31) for chn_pen_skip == 0 (main.rs:116):
    // (gap*dd + 0*dg + 0.5*log2(dd+1)) as i32, f32 op by op, glibc logf.
    // gap = chn_pen_gap = 0.01f * 0.8f * k (main.rs:106-107)
    if (gap == c->lut_gap && n <= c->lut_n) return;
    c->h_lut.assign(n, 0);
    for (int dd = 0; dd < n; ++dd) {
        const float lin = gap * (float)dd + 0.0f * 1.0f;
        float lg = 0.0f;
        if (dd >= 1) { const int x = dd + 1; lg = x <= 1 ? 0.0f : logf((float)x) / 0.693147180559945309417232121458176568f; }
        const float v = lin + 0.5f * lg;
        c->h_lut[dd] = (int16_t)(int32_t)v;
    }
    c->lut_gap = gap; c->lut_n = n;
    c->lut_dirty = true;
}

// The pen LUT on the device (n entries, whole 16-B words for load_lut): it
// stays resident and is copied only when it changes.
static int upload_lut(mm2g_ctx* c, float gap, int n, int16_t** out) {
    build_lut(c, gap, n);
    int16_t* lut;
    ENSURE(c->lut, int16_t, (c->h_lut.size() + 7) & ~(size_t)7, lut);
    if (c->lut_dirty || c->lut_dev != c->lut.p) {
        HIPCHK(hipMemcpyAsync(lut, c->h_lut.data(), c->h_lut.size() * 2, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->lut_dirty = false; c->lut_dev = c->lut.p;
    }
    *out = lut;
    return 0;
}

// -n <= 1 with -m <= k (the query span): several chains reach the output (DESIGN.md "-n <= 1")
static bool multi_chain_opts(const mm2g_map_opts* o) { return o->min_cnt < 2 && o->min_chain_score <= o->k; }

// Argument checks of the Align flow (main.rs:189-230) shared by map and the stage entry points.
static int check_opts(mm2g_ctx* c, const mm2g_map_opts* o, int32_t& mdx0, int32_t& mdx1) {
    if (!(o->w > 0 && o->w < 256 && o->k > 0 && o->k <= 28)) return set_err(MM2G_E_ARG, "invalid w/k (0 < w < 256, 0 < k <= 28)");
    if (o->bw < 0 || o->bw_long < 0) return set_err(MM2G_E_ARG, "negative bandwidth");
    mdx0 = std::max(o->max_gap, o->bw); mdx1 = std::max(o->max_gap, o->bw_long);
    if (std::max(o->bw, o->bw_long) + 1 > 60000) return set_err(MM2G_E_UNSUP, "bandwidth > 59999 not supported");
    // rpos_j + max_dist_x is i32 in the reference; keep it from wrapping (DESIGN.md Q-envelope)
    if (c->hidx && (uint64_t)c->hidx->max_len + (uint64_t)std::max(mdx0, mdx1) >= (1ULL << 31))
        return set_err(MM2G_E_UNSUP, "reference length + max gap must stay below 2^31");
    return 0;
}

// Chain DP + fallback + rescue (lchain.rs:59-176, 321-330; main.rs:209-215)
// over the sorted keys of the batch (cnt2/smax: the sort's singleton filter).
// full: exact f/pprev for every anchor (debug mode, mm2g_chain_batch with DP
// arrays requested): no segment pruning, no lazy windows.
static int run_chain(mm2g_ctx* c, uint32_t n, const uint64_t* rd_off, const ChainKParams& P0, float gap, int npass, int32_t mdx1,
                     int32_t mdy1, int32_t bw_long, uint64_t A_cap, const uint64_t* a_off, const uint32_t* a_cnt, uint64_t* keys,
                     uint64_t* ktmp, const uint32_t* cnt2, const uint64_t* smax, ReadOut* out, const uint32_t* abort, bool full,
                     unsigned long long* stat = nullptr, bool order_ready = false, const uint32_t* sum_mz = nullptr) {
    int32_t *fb, *pb;
    ENSURE(c->fbuf, int32_t, A_cap, fb); ENSURE(c->ppbuf, int32_t, A_cap, pb);
    int16_t* lut; uint32_t* work;
    if (int e = upload_lut(c, gap, std::max(P0.bw, npass > 1 ? bw_long : 0) + 1, &lut)) return e;
    ENSURE(c->work, uint32_t, 4, work);
    // work: [0..1] k_chain_giant hand-out per pass (k_seg_items of pass 0 clears it)
    uint32_t* order;
    ENSURE(c->order, uint32_t, n, order);
    int32_t* tmark;
    ENSURE(c->tmark, int32_t, A_cap, tmark);
    // every segment over CHAIN_TINY anchors may take a wave (med_pairs 0), and they are disjoint
    const uint32_t lcap = (uint32_t)std::min<uint64_t>(A_cap / (CHAIN_TINY + 1) + 64, 0xffffffffu);
    uint4* lseg; uint32_t *lseg_n, *lseg_order; unsigned long long* rbest;
    ENSURE(c->lseg, uint4, lcap, lseg);
    ENSURE(c->lseg_order, uint32_t, lcap, lseg_order);
    ENSURE(c->lseg_n, uint32_t, 4, lseg_n);
    ENSURE(c->rbest, unsigned long long, n, rbest);
    const uint32_t mcap2 = (uint32_t)std::min<uint64_t>(A_cap / (CHAIN_TINY + 1) + 64, 0xffffffffu);
    uint4* mseg;
    ENSURE(c->mseg, uint4, mcap2, mseg);
    if (!order_ready) LCHK(launch_read_order(n, a_cnt, order, c->stream));   // map_enqueue made the same order
    const int64_t* K = c->knob;
    const bool lazy = (!full && K[MM2G_KNOB_LAZY]) || K[MM2G_KNOB_LAZY] == 2;   // 2: also with full DP arrays (tests)
    ChainArgs ca{n, rd_off, a_off, keys, fb, pb, (uint32_t*)ktmp, lut, P0, c->kl, out, work,
                 std::min(c->keys.cap, c->fbuf.cap / 4 * 8) / 8, nullptr, order, A_cap, std::min<int32_t>((int32_t)n, 4 * 256), tmark,
                 lseg, lseg_n, lcap, lseg_order, rbest, cnt2, smax, mseg, lseg_n + 2, lseg_n + 3, mcap2, nullptr, 0u,
                 lazy ? 1u : 0u, nullptr, 0u};
    ca.abort = abort;
    ca.full_dp = full ? 1u : 0u;   // not "no fmin": with pruning off, production still follows the med_pairs knobs
    int32_t* fmin_buf = nullptr;
    if (!full && K[MM2G_KNOB_PRUNE]) ENSURE(c->fmin, int32_t, n, fmin_buf);
    // pass 0's segment-start words (k_chain_lb -> k_chain_seg's sparse items): read r at (a_off[r] >> 6) + r
    uint64_t* isob = nullptr;
    uint2* sq = nullptr;
    uint32_t* sq_n = nullptr;
    const uint32_t sq_cap = (uint32_t)std::min<uint64_t>(A_cap / 64 + n + 16, 0xffffffffu);
    if (fmin_buf && K[MM2G_KNOB_SEG_SPARSE] && K[MM2G_KNOB_MED_PAIRS] == 0) {
        ENSURE(c->isob, uint64_t, A_cap / 64 + n + 2, isob);
        ENSURE(c->sq, uint2, sq_cap, sq);
        ENSURE(c->sq_n, uint32_t, 1, sq_n);
    }
    uint32_t* item_off;
    ENSURE(c->item_off, uint32_t, n + 1, item_off);
    ca.item_off = item_off;
    {   // items per read <= max(ceil(A / seg_chunk), the sort's candidate budget A / 32 + 8)
        const uint64_t icap = std::min<uint64_t>(A_cap / 32 + 8ull * n + 1024, 0xffffffffull);
        uint32_t* ir;
        ENSURE(c->item_read, uint32_t, icap, ir);
        ca.item_read = ir; ca.item_cap = (uint32_t)icap;
    }
    ca.seg_chunk = std::max<uint32_t>(64u, (uint32_t)K[MM2G_KNOB_SEG_CHUNK] & ~63u);
    ca.spec_rounds = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(16, K[MM2G_KNOB_SPEC_ROUNDS]));
    ca.spec_eval = K[MM2G_KNOB_SPEC_EVAL] ? 1u : 0u;
    ca.spec_batch = K[MM2G_KNOB_SPEC_BATCH] == 8 ? 8u : 4u;
    ca.cands_longw = K[MM2G_KNOB_CANDS_LONGW] > 0 ? (uint32_t)std::min<int64_t>(K[MM2G_KNOB_CANDS_LONGW], 0x7fffffff) : 0x7fffffffu;
    // Giant segments (k_chain_giant): the rescue pass's pseudo-group clusters
    // settle in a few no-break policy-iteration rounds.  Pass 0's long segments
    // are real chains whose windows carry many mark sources: k_chain_long is
    // faster on the usual few-hundred-anchor ones; its
    // exact mode is off by default (measured 15x (C3) and 6x (C5) slower).
    uint32_t giant_min[2] = {K[MM2G_KNOB_GIANT_MIN0] > 0 ? (uint32_t)std::max<int64_t>(2, K[MM2G_KNOB_GIANT_MIN0]) : 0xffffffffu,
                             (uint32_t)std::max<int64_t>(2, K[MM2G_KNOB_GIANT_MIN])};
    for (int pass = 0; pass < npass; ++pass) {
        if (pass == 1) {
            ca.P.pass = 1; ca.P.bw = bw_long; ca.P.max_dist_x = mdx1; ca.P.max_dist_y = mdy1;
            ca.P.lut_n = bw_long + 1; ca.lseg_n = lseg_n + 1;
        }
        int sb = chain_max_blocks(ca.P.lut_n, 0), lb = chain_max_blocks(ca.P.lut_n, 1), mb = chain_max_blocks(ca.P.lut_n, 2);
        if (sb <= 0) sb = 1024;
        if (lb <= 0) lb = 1024;
        if (mb <= 0) mb = 1024;
        sb = std::max(1, std::min((int)((n * 4 + 3) / 4), sb));   // items: up to ~4 chunks per read
        static const char* names[2][5] = {{"chain_seg", "chain_med", "chain_lorder", "chain_long", "chain_fin"},
                                          {"chain_seg_rescue", "chain_med_rescue", "chain_lorder_rescue", "chain_long_rescue", "chain_fin_rescue"}};
        const int blocks[5] = {sb, mb, 1, lb, 0};
        // Lower bound of each read's best f (k_chain_lb, this pass's parameters): prunes
        // segments (not in debug mode).  In the rescue pass (rescued reads only) the bound
        // is LB_1, raised by pass 0's LB_0 when the rescue's comput_sc limits are all at
        // least pass 0's (bw_long >= bw, max_dist_x/y no smaller): every pass-0 transition
        // is then accepted there with the same score, so its best f >= LB_0.  The reference
        // accepts -r A,B with B < A (main.rs:205-206): then pass-0 steps with dd in
        // (bw_long, bw] are rejected in the rescue and LB_0 does not bound it.
        const bool rescue_wider = bw_long >= P0.bw && mdx1 >= P0.max_dist_x && mdy1 >= P0.max_dist_y;
        ca.fmin = (pass == 0 || K[MM2G_KNOB_PRUNE_RESCUE]) ? fmin_buf : nullptr;
        if (pass == 0) c->lb_ran0 = ca.fmin != nullptr;
        ca.isob = isob;
        ca.seg_streamed = stat ? stat + 5 + pass : nullptr;   // status words 5 / 6
        ca.zero_fmin = ca.fmin && (pass == 0 || !rescue_wider) ? 1u : 0u;   // cleared by k_seg_items
        ca.sq = nullptr; ca.sq_cap = 0;
        ca.sq_n = (ca.fmin && isob) ? sq_n : nullptr;                      // ... as is the item counter
        // the last pass's k_seg_items also writes the batch sums (status words 3 and 4): one launch less
        ca.bsum = (sum_mz && stat && pass == npass - 1) ? stat : nullptr;
        ca.mz_cnt = sum_mz;
        {
            ProfScope ps(c, pass ? "chain_items_rescue" : "chain_items");
            LCHK(launch_chain_stage(6, ca, 1, c->stream));
        }
        if (ca.fmin) {
            {
                ProfScope ps(c, pass ? "chain_lb_rescue" : "chain_lb");
                LCHK(launch_chain_stage(5, ca, 2048, c->stream));
            }
            if (ca.isob) {   // candidate segments per read; k_chain_seg streams only the reads left over
                ca.sq = sq; ca.sq_cap = sq_cap;
                ProfScope ps(c, pass ? "chain_cands_rescue" : "chain_cands");
                // one workgroup per 16 reads; with long reads (over ~64 kb) also one per read (up to
                // 1024), since each such read takes a whole workgroup
                // (the kernel's criterion, cnt2 > cands_longw * 64: at most A_cap / (64 cands_longw) such reads)
                const uint64_t nlong = std::min<uint64_t>(n, A_cap / (64ull * ca.cands_longw) + 1);
                const uint32_t cb = std::max<uint32_t>((n + 15) / 16, (uint32_t)nlong);
                LCHK(launch_chain_stage(10, ca, (int)std::min<uint32_t>(cb, 1024), c->stream));
            }
        }
        ca.lseg_prof = K[MM2G_KNOB_LSEG_PROF] ? 1u : 0u;
        unsigned long long* gprof = nullptr;
        if (ca.lseg_prof) {
            HIPCHK(hipMalloc(&gprof, 32 * 8));
            HIPCHK(hipMemsetAsync(gprof, 0, 32 * 8, c->stream));
        }
        ca.gprof = gprof;
        ca.seg_stat = stat ? stat + 8 + 3 * pass : nullptr;
        for (int stg = 0; stg < 5; ++stg) {
            ca.giant_min = giant_min[pass];
            ca.giant_exact = pass == 0 ? 1u : 0u;
            ca.est_lane = (int32_t)std::max<int64_t>(0, std::min<int64_t>(1 << 20, K[pass ? MM2G_KNOB_MED_PAIRS_RESCUE : MM2G_KNOB_MED_PAIRS]));
            if (stg == 2) {   // longest-first order of the long segments (k_chain_giant and k_chain_long)
                ProfScope ps(c, names[pass][stg]);
                LCHK(launch_chain_stage(2, ca, 1, c->stream));
            }
            // production only; the pin bitmap and the lo field bound the window (max_iter <= 5120)
            if (stg == 2 && ca.lazy && ca.giant_min != 0xffffffffu && ca.P.max_iter <= 5120 && K[MM2G_KNOB_GIANT]) {
                ProfScope ps(c, pass ? "chain_giant_rescue" : "chain_giant");
                if (K[MM2G_KNOB_GIANT_LCAP] > 0) ca.giant_lcap = (uint32_t)std::max<int64_t>(16, K[MM2G_KNOB_GIANT_LCAP]) & ~15u;
                LCHK(launch_chain_stage(7, ca, 0, c->stream));   // workgroups: as many as fit (giant_lcap sets their LDS)
                // longer segments from a per-workgroup HBM slice (100 kb reads' rescue)
                const uint32_t gmax = (uint32_t)std::max<int64_t>(0, K[MM2G_KNOB_GIANT_GMAX]) & ~15u;
                if (gmax) {
                    const int gblocks = (int)std::max<int64_t>(1, K[MM2G_KNOB_GIANT_GBLOCKS]);
                    unsigned char* scr;
                    ENSURE(c->giant_scr, unsigned char, (size_t)gblocks * gmax * 42, scr);
                    ca.giant_scr = scr;
                    ca.giant_gmax = gmax;
                    LCHK(launch_chain_stage(8, ca, gblocks, c->stream));
                }
            }
            if (stg == 2) continue;   // launched above
            // k_chain_seg routes a segment to k_chain_med only when its estimated pairs stay
            // under est_lane (EST_LANE for pass 0 with full DP arrays): at 0 the queue stays
            // empty and the launch would only add its latency (C2 is launch-bound)
            if (stg == 1 && ca.est_lane == 0 && !(pass == 0 && full)) continue;
            ProfScope ps(c, names[pass][stg]);
            LCHK(launch_chain_stage(stg, ca, blocks[stg], c->stream));
        }
        if (gprof) {   // k_chain_giant phase sums (wall clock, 100 MHz); k_chain_long per-anchor cycles
            unsigned long long g[32];
            HIPCHK(hipMemcpyAsync(g, gprof, sizeof g, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            (void)hipFree(gprof);
            ca.gprof = nullptr;
            fprintf(stderr, "[giant_prof] pass %d: %llu segments, %llu anchors, %llu iterations, %llu pins, %llu fallbacks; block-us: total %.0f "
                            "setup %.0f eval %.0f changed %.0f improve %.0f children %.0f markcheck %.0f pin %.0f write %.0f\n",
                    pass, g[8], g[9], g[10], g[11], g[13], g[12] / 100.0, g[0] / 100.0, g[1] / 100.0, g[2] / 100.0, g[3] / 100.0,
                    g[4] / 100.0, g[5] / 100.0, g[6] / 100.0, g[7] / 100.0);
            const double np_ = (double)std::max<unsigned long long>(g[17] + g[19], 1);
            fprintf(stderr, "[long_prof] pass %d: %llu anchors in long segments, %llu committed by the speculative block pass in %llu rounds; "
                            "per-anchor path: %llu settled by the simple/shortcut step, %llu exact (%llu 64-lane window steps in all); "
                            "shader cycles per per-anchor-path anchor: st %.0f simple %.0f exact %.0f tail %.0f\n",
                    pass, g[16], g[24], g[25], g[17], g[19], g[18], g[20] / np_, g[21] / np_, g[22] / np_, g[23] / np_);
            fprintf(stderr, "[long_prof] pass %d heaviest segment: %llu anchors committed speculatively in %llu rounds, %llu by the per-anchor path; "
                            "shader cycles: speculative %llu, per-anchor path %llu, segment %llu\n",
                    pass, g[26], g[27], g[28], g[30], g[29], g[31]);
        }
        if (ca.lseg_prof) {   // the slowest long segments of this pass
            uint32_t nl = 0;
            HIPCHK(hipMemcpyAsync(&nl, ca.lseg_n, 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            nl = std::min(nl, lcap);
            std::vector<uint4> ls(nl);
            if (nl) HIPCHK(hipMemcpy(ls.data(), lseg, (size_t)nl * 16, hipMemcpyDeviceToHost));
            // lseg[].w: wall-clock ticks (100 MHz) of the kernel that ran the segment; bit 31 = k_chain_giant's
            const uint32_t GBIT = 0x80000000u;
            std::sort(ls.begin(), ls.end(), [&](const uint4& x, const uint4& y) { return (x.w & ~GBIT) > (y.w & ~GBIT); });
            double tot = 0, tot_g = 0; uint32_t ng = 0;
            for (auto& v : ls) { tot += v.w & ~GBIT; if (v.w & GBIT) { tot_g += v.w & ~GBIT; ++ng; } }
            fprintf(stderr, "[lseg_prof] pass %d: %u long segments (%u by k_chain_giant), sum %.0f us (giant %.0f us); slowest:", pass, nl, ng,
                    tot / 100, tot_g / 100);
            for (size_t i = 0; i < ls.size() && i < 8; ++i) {
                ReadOut ro;
                HIPCHK(hipMemcpy(&ro, out + ls[i].x, sizeof ro, hipMemcpyDeviceToHost));
                fprintf(stderr, " (read %u len %u %s %.0f us, read j-steps %u pairs %llu)", ls[i].x, ls[i].z - ls[i].y,
                        (ls[i].w & GBIT) ? "giant" : "long", (ls[i].w & ~GBIT) / 100.0, ro.n_steps, (unsigned long long)ro.dp_pairs);
            }
            fprintf(stderr, "\n");
        }
    }
    return 0;
}

// The anchor workspace of a batch: keys, sorted keys, f (the sort's tags
// first), pprev and the DP marks, 28 B per anchor (x 1.25 slack), kept across
// batches.  The first estimate is 3 anchors per base (C3 has 2): about 10 GB
// per context for a 100 Mb batch.  When HBM cannot hold that, the batch's exact
// anchor count (the scan's total; one synchronisation) is used instead, so a
// batch whose anchors fit is never refused for the estimate.  The
// fallback first frees all five buffers (a partial grab of the estimate must
// not keep HBM from the exact one), clears the failed hipMalloc's error, and
// leaves the context in exact-size mode: later batches keep the exact
// capacity (grown by wait_batch's re-map when a batch needs more) instead of
// re-inflating to the estimate and paying hipFree + a failed hipMalloc + a
// stream synchronisation every batch.
static int reserve_anchor_ws(mm2g_ctx* c, const unsigned long long* st, uint64_t& A_cap) {
    DevBuf* bufs[5] = {&c->keys, &c->keys_tmp, &c->fbuf, &c->ppbuf, &c->tmark};
    auto grab = [&](uint64_t n) -> int {
        uint64_t* p64; int32_t* p32;
        if (int e = ensure<uint64_t>(c->keys, n, &p64)) return e;
        if (int e = ensure<uint64_t>(c->keys_tmp, n, &p64)) return e;
        if (int e = ensure<int32_t>(c->fbuf, n, &p32)) return e;
        if (int e = ensure<int32_t>(c->ppbuf, n, &p32)) return e;
        if (int e = ensure<int32_t>(c->tmark, n, &p32)) return e;
        return 0;
    };
    if (c->knob[MM2G_KNOB_WS_FAIL] > 0) {   // tests: a partial grab (keys at the estimate), then HBM "full"
        --c->knob[MM2G_KNOB_WS_FAIL];
        uint64_t* p64;
        if (int e = ensure<uint64_t>(c->keys, A_cap, &p64)) return e;
    } else if (grab(A_cap) == 0) {
        return 0;
    }
    (void)hipGetLastError();                  // the failed hipMalloc must not surface as a launch error
    unsigned long long tot = 0;
    HIPCHK(hipMemcpyAsync(&tot, st + 2, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));  // also: nothing queued still uses the buffers freed below
    const uint64_t need = std::max<uint64_t>((uint64_t)tot, 1);
    for (DevBuf* b : bufs) if (b->cap < need * (b == &c->keys || b == &c->keys_tmp ? 8 : 4)) {
        for (DevBuf* d : bufs) { if (d->p) (void)hipFree(d->p); d->p = nullptr; d->cap = 0; }
        break;
    }
    c->ws_exact = true;
    c->cap_A = A_cap = need;
    const int e = grab(A_cap);
    if (e) (void)hipGetLastError();
    return e;
}

// Queue the whole path for the resident batch on the context stream (no host
// synchronisation): sketch -> filter -> lookup -> anchors -> sort -> chain ->
// dv, then the per-read results and the status block to pinned host memory.
// `stop_after_sort`: the seed stage entry point (mm2g_seed_batch).
static int map_enqueue(mm2g_ctx* c, const mm2g_map_opts* o, bool stop_after_sort) {
    int32_t mdx0, mdx1;
    if (int e = check_opts(c, o, mdx0, mdx1)) return e;
    // -n <= 1 with -m <= k: one-anchor backtrack chains pass (the backtrack leaves mg_chain_bk_end after one
    // step, lchain.rs:110,114), so every anchor's f / pprev matters: full arrays, no singleton filter, and the
    // host epilogue (mm2g_multi.cpp) runs the backtrack, merge and selection (DESIGN.md "-n <= 1")
    const bool multi = !stop_after_sort && multi_chain_opts(o);
    const bool full = c->debug || multi;
    c->full_last = full || stop_after_sort;
    c->multi_last = multi;
    HIPCHK(hipSetDevice(c->device));
    const HostIndex& H = *c->hidx;
    const uint32_t n = c->n_reads;
    const int64_t* K = c->knob;
    c->mapped = false;
    c->collected = false;
    c->stop_after_sort = stop_after_sort;
    c->last_opts = *o;
    // key layout
    KeyLayout kl;
    kl.n_seq = H.n_seq;
    kl.qb = std::max<uint32_t>(1, bit_width(c->max_read_len));
    kl.rb = std::max<uint32_t>(1, bit_width(H.max_len));
    kl.gb = std::max<uint32_t>(1, bit_width(2ull * H.n_seq));
    if (kl.qb + kl.rb + kl.gb > 64) return set_err(MM2G_E_UNSUP, "anchor key needs %u bits (> 64)", kl.qb + kl.rb + kl.gb);
    c->kl = kl;
    ReadOut* out;
    ENSURE(c->outb, ReadOut, n + 1, out);
    unsigned long long* st;
    ENSURE(c->dstat, unsigned long long, STAT_WORDS, st);
    uint32_t* st32 = (uint32_t*)st;
    if (n == 0) {
        HIPCHK(hipMemsetAsync(out, 0, sizeof(ReadOut), c->stream));
        HIPCHK(hipMemsetAsync(st, 0, STAT_WORDS * 8, c->stream));
    }
    if (c->h_out_cap < (size_t)n + 1) {
        HIPCHK(hipStreamSynchronize(c->stream));   // a previous batch's copy may still target it
        if (c->h_out) (void)hipHostFree(c->h_out);
        c->h_out = nullptr; c->h_out_cap = 0;
        HIPCHK(hipHostMalloc((void**)&c->h_out, ((size_t)n + 1) * sizeof(ReadOut), hipHostMallocDefault));
        c->h_out_cap = (size_t)n + 1;
    }
    if (n == 0) {
        HIPCHK(hipMemcpyAsync(c->h_stat, st, STAT_WORDS * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipEventRecord(c->ev_done, c->stream));
        c->mapped = true;
        return 0;
    }
    // 1. sketch (CLI w/k, rid 0: seeds.rs:7-11)
    if (int e = run_sketch(c, o->w, o->k, c->sk1, (int32_t*)st32, out, st)) return e;   // clears out[] and st[] first
    const uint64_t mcap = c->sk1.cap;
    uint64_t* mz_base = (uint64_t*)c->sk1.base.p; uint32_t* mz_cnt = (uint32_t*)c->sk1.cnt.p;
    // 2. query filter (seeds.rs:13-36; (10, 0.01) hard-wired at main.rs:195).  Only
    //    reads whose count table outgrows LDS use the global table; its size is
    //    estimated from the read lengths and checked on the device.
    {
        uint64_t est = 0;
        for (uint32_t r = 0; r < n; ++r) {
            const uint64_t m = 2 * (c->h_rd_off[r + 1] - c->h_rd_off[r]) / (uint64_t)(o->w + 1) + 64;
            uint64_t ts = 1;
            while (ts < 2 * m) ts <<= 1;
            if (m > 10 && (ts > 4096 || o->k > 16)) est += ts;
        }
        c->cap_tab = std::max(c->cap_tab, est);
        if (c->knob[MM2G_KNOB_WS_MIN] > 0 && !c->redo) c->cap_tab = (uint64_t)c->knob[MM2G_KNOB_WS_MIN];   // tests: force the re-map
    }
    uint64_t* tab_off; uint8_t* keep;
    ENSURE(c->tab_off, uint64_t, n + 1, tab_off);
    ENSURE(c->keep, uint8_t, mcap, keep);
    {
        ProfScope ps(c, "scan");
        LCHK(launch_excl_scan(mz_cnt, n, tab_off, 1, 10, o->k, std::max<uint64_t>(c->cap_tab, 1), st32, BS_TAB, 1, c->stream));
    }
    uint64_t* tkey; uint32_t* tcnt;
    ENSURE(c->tab_key, uint64_t, c->cap_tab, tkey);
    ENSURE(c->tab_cnt, uint32_t, c->cap_tab, tcnt);
    {
        FilterArgs fa{n, mz_base, mz_cnt, (const uint64_t*)c->sk1.x.p, tab_off, tkey, tcnt, keep, 10, 0.01f, c->cap_tab};
        ProfScope ps(c, "filter");
        LCHK(launch_filter(fa, o->k, grid_for(n), c->stream));
    }
    // 3. lookup + anchor count (index.rs:143-154, seeds.rs:42-57); the anchor
    //    workspace keeps its capacity across batches, checked on the device
    uint32_t *mz_n, *mz_poff, *a_cnt; uint64_t* a_off;
    ENSURE(c->mz_n, uint32_t, mcap, mz_n); ENSURE(c->mz_poff, uint32_t, mcap, mz_poff);
    ENSURE(c->a_cnt, uint32_t, n + 1, a_cnt); ENSURE(c->a_off, uint64_t, n + 1, a_off);
    uint32_t* a_part;
    ENSURE(c->a_part, uint32_t, (size_t)n * (SEED_PARTS - 1), a_part);
    SeedArgs sa{n, c->d_rd_off, mz_base, mz_cnt, (const uint64_t*)c->sk1.x.p, (const uint32_t*)c->sk1.y.p, keep,
                (const IxEntry*)c->dix->tab.p, c->log2cap, c->mid_occ, (const uint64_t*)c->dix->ix_pos.p, mz_n, mz_poff, a_cnt, a_off, nullptr, kl, o->k,
                0, c->dix->ix_pos.cap / 8, mcap, out, a_part};
    sa.abort = st32;
    {
        ProfScope ps(c, "seed_count");
        LCHK(launch_seed_count(sa, grid_for(n), c->stream));
    }
    if (!c->ws_exact) c->cap_A = std::max<uint64_t>(c->cap_A, 3 * c->total_bases + 65536);   // exact-size mode: see reserve_anchor_ws
    if (c->knob[MM2G_KNOB_WS_MIN] > 0 && !c->redo) c->cap_A = (uint64_t)c->knob[MM2G_KNOB_WS_MIN];   // tests: force the re-map
    uint64_t A_cap = c->cap_A;
    // reads heaviest first (anchor counts from seed_count): the hand-out order of
    // seed_write, the sort and the chain work items; made by the anchor scan's block
    uint32_t* rorder;
    ENSURE(c->order, uint32_t, n, rorder);
    {
        ProfScope ps(c, "scan");
        LCHK(launch_excl_scan(a_cnt, n, a_off, 0, 0, o->k, A_cap, st32, BS_ANCHORS, 2, c->stream, rorder));
    }
    if (int e = reserve_anchor_ws(c, st, A_cap)) return e;
    uint64_t* keys = (uint64_t*)c->keys.p;
    uint64_t* ktmp = (uint64_t*)c->keys_tmp.p;
    int32_t* fb = (int32_t*)c->fbuf.p;      // the sort's per-key tags live here before the DP needs it
    sa.keys = keys; sa.cap_keys = c->keys.cap / 8;
    sa.order = rorder;
    // 4. anchor sort (seeds.rs:58).  The singleton filter needs every max_dist_x
    //    of both DP passes within one 2^CELL_SHIFT cell (DESIGN.md "Anchor sort");
    //    it is off in debug mode (full anchor/DP arrays for the parity tests).
    const bool filt = !full && !stop_after_sort && K[MM2G_KNOB_FILTER] && std::max(mdx0, mdx1) <= (1 << CELL_SHIFT);
    const uint32_t sort_small_max = (uint32_t)std::min<int64_t>(K[MM2G_KNOB_SORT_SMALL], 4096);
    // fused seeding: k_sort_read's first pass makes the keys of the reads it sorts when their
    // minimizers (16 B each) fit in its LDS above the two cell bitmaps
    uint32_t fuse_mmax = 0;
    if (filt && K[MM2G_KNOB_SEED_FUSE]) {
        SortArgs t{};
        t.cells = c->dix->cells;
        t.lds_words = (uint32_t)(std::max<int64_t>(0, K[MM2G_KNOB_SORT_LDS_KB]) * 256);
        const uint32_t LW = sort_read_lds_words(t), nw = (t.cells + 31) / 32;
        if (LW > 2 * nw + 64 + 2048) fuse_mmax = std::min<uint32_t>((LW - 2 * nw - 64 - 2048) / 4, 0xffffu);   // 4 words per minimizer + 4096 u16 owner starts
    }
    const uint32_t fuse_big = (filt && K[MM2G_KNOB_SEED_FUSE_BIG]) ? 1u : 0u;   // k_sort_big seeds the reads over 65535 anchors
    sa.fuse_mmax = fuse_mmax; sa.small_max = sort_small_max; sa.fuse_big = fuse_big;
    c->filt_last = filt; c->small_last = sort_small_max;
    {
        ProfScope ps(c, "seed_write");
        LCHK(launch_seed_write(sa, grid_for(n), c->stream));
    }
    uint32_t* cnt2; uint64_t* smax; uint32_t* rlist;
    ENSURE(c->cnt2, uint32_t, n, cnt2);
    ENSURE(c->rlist, uint32_t, n + 2, rlist);
    ENSURE(c->smax, uint64_t, n, smax);
    const int64_t stop_at = K[MM2G_KNOB_STOP_AT];   // measurement only: later stages skipped, results invalid
    // pass-0 chain parameters (main.rs:201-214): the sort's LB pass uses them too
    ChainKParams P{};
    P.max_dist_x = mdx0; P.max_dist_y = std::max(o->max_gap, o->bw); P.bw = o->bw; P.max_iter = 5000; P.max_skip = 25;
    P.span = o->k; P.rescue_size = 1000; P.rescue_ratio_f = 1.0f - 0.1f; P.pass = 0; P.lut_n = o->bw + 1;
    P.multi = multi ? 1 : 0;
    const float gap = 0.01f * 0.8f * (float)o->k;
    const int npass = stop_at == 3 ? 1 : 2;
    const bool chain = !stop_after_sort && stop_at != 1 && stop_at != 2;
    SortArgs so{n, a_off, keys, ktmp, kl.qb, kl.rb, kl.n_seq, c->keys.cap / 8, (const uint32_t*)c->dix->goff.p,
                filt ? c->dix->cells : 0u, cnt2, smax, sort_small_max, nullptr, 0u,
                (uint32_t)std::max<int64_t>(1, std::min<int64_t>(K[MM2G_KNOB_SEG_SMALL], SEG_THREAD)), nullptr};
    so.abort = st32;
    so.meta = (uint32_t*)fb;
    so.rlist = rlist; so.rcount = rlist + n; so.rwork = rlist + n + 1;
    so.order = rorder;
    so.lds_words = (uint32_t)(std::max<int64_t>(0, K[MM2G_KNOB_SORT_LDS_KB]) * 256);
    so.fuse_mmax = fuse_mmax;
    so.fuse_big = fuse_big; so.a_part = a_part;
    so.read_tiny = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(K[MM2G_KNOB_READ_TINY], 1024));
    so.big_tiny = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(K[MM2G_KNOB_BIG_TINY], 2048));
    so.small_reg = K[MM2G_KNOB_SMALL_REG] ? 1u : 0u;
    so.big_wnd = (uint32_t)std::max<int64_t>(0, K[MM2G_KNOB_BIG_WND]);
    so.rd_off = c->d_rd_off; so.mz_base = mz_base; so.mz_cnt = mz_cnt; so.mz_y = (const uint32_t*)c->sk1.y.p;
    so.mz_n = mz_n; so.mz_poff = mz_poff; so.ix_pos = (const uint64_t*)c->dix->ix_pos.p; so.kl = kl; so.span = o->k;
    so.cap_pos = c->dix->ix_pos.cap / 8;
    uint64_t* sprof = nullptr;
    if (K[MM2G_KNOB_SORT_PROF]) { HIPCHK(hipMalloc(&sprof, (size_t)n * 192)); HIPCHK(hipMemsetAsync(sprof, 0, (size_t)n * 192, c->stream)); so.prof = sprof; }
    if (stop_at != 1) {
    {
        ProfScope ps(c, "sort_small");
        LCHK(launch_sort_read(0, so, c->stream));
    }
    {
        ProfScope ps(c, "sort_large");
        LCHK(launch_sort_read(1, so, c->stream));
    }
    {
        ProfScope ps(c, so.cells ? "sort_big" : "sort_radix");   // reads k_sort_read listed: buckets (filter on) or radix
        LCHK(launch_sort_read(2, so, c->stream));
    }
    if (sprof) dump_sort_prof(c, sprof, n);
    // the sorted anchors are in the tmp buffer: swap the roles for everything downstream
    std::swap(c->keys.p, c->keys_tmp.p); std::swap(c->keys.cap, c->keys_tmp.cap);
    std::swap(keys, ktmp);
    }
    if (chain) {
        // 5. chain DP + fallback + rescue
        if (int e = run_chain(c, n, c->d_rd_off, P, gap, npass, mdx1, std::max(o->max_gap, o->bw_long), o->bw_long, A_cap,
                              a_off, a_cnt, keys, ktmp, cnt2, smax, out, st32, full, st, true, mz_cnt))
            return e;
        // 6. dv inputs (paf.rs:156-199): sketch with the INDEX w/k (Q3)
        const bool sep = (H.w != o->w || H.k != o->k);
        c->dv_separate = sep;
        if (sep) {
            if (!(H.w > 0 && H.w < 256 && H.k > 0 && H.k <= 28)) return set_err(MM2G_E_ARG, "index w/k invalid for the dv sketch");
            if (int e = run_sketch(c, H.w, H.k, c->sk2, (int32_t*)(st32 + 1))) return e;
        }
        SketchBufs& D = sep ? c->sk2 : c->sk1;
        DvArgs da{n, a_off, keys, (const uint32_t*)ktmp, (const uint64_t*)D.base.p, (const uint32_t*)D.cnt.p, (const uint32_t*)D.y.p, kl, o->k,
                  out, c->keys.cap / 8, D.y.cap / 4};
        da.abort = st32;
        da.strict = (H.k & 1) && c->knob[MM2G_KNOB_DV_PAR] ? 1u : 0u;   // odd k: positions strictly increase
        // reads whose dv sketch outgrows k_dv's 4096 staged positions (~2 per w+1 bases): a workgroup each
        da.long_m = da.strict && 2ull * c->max_read_len / (uint64_t)(H.w + 1) + 64 > 4096 ? 0xffffffffu : 0u;
        ProfScope ps(c, "dv");
        if (stop_at != 4) LCHK(launch_dv(da, c->stream));
    }
    if (!chain) LCHK(launch_batch_sums(n, mz_cnt, cnt2, st, c->stream));   // (else the last chain pass's k_seg_items)
    HIPCHK(hipMemcpyAsync(c->h_out, out, (size_t)n * sizeof(ReadOut), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_stat, st, STAT_WORDS * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipEventRecord(c->ev_done, c->stream));
    c->mapped = true;
    return 0;
}

// Wait for the queued batch; when a workspace was too small, grow it and map
// the batch again (reads are still resident), at most a few times.
static int wait_batch(mm2g_ctx* c) {
    if (!c->mapped) return set_err(MM2G_E_STATE, "batch not mapped");
    if (c->collected) return 0;
    for (int it = 0;; ++it) {
        HIPCHK(hipEventSynchronize(c->ev_done));
        const uint32_t* s32 = (const uint32_t*)c->h_stat;
        const uint32_t bits = s32[0], dv_ovf = s32[1];
        if (!bits && !dv_ovf) break;
        if (it >= 4) return set_err(MM2G_E_STATE, "batch workspaces did not converge (status %u)", bits);
        if (bits & BS_SKETCH) { if (int e = sketch_exact_layout(c, c->sk1)) return e; }
        if (dv_ovf) { if (int e = sketch_exact_layout(c, c->sk2)) return e; }
        if ((bits & BS_SKETCH) || dv_ovf) c->views_off = true;   // a view may have overflowed its own slot
        if (bits & BS_TAB) c->cap_tab = std::max(c->cap_tab, c->h_stat[1] + c->h_stat[1] / 4 + 1024);
        if (bits & BS_ANCHORS) c->cap_A = std::max(c->cap_A, c->h_stat[2] + c->h_stat[2] / 4 + 65536);
        const mm2g_map_opts o = c->last_opts;
        c->redo = true;
        const int e = map_enqueue(c, &o, c->stop_after_sort);
        c->redo = false;
        if (e) return e;
    }
    c->n_anchors = c->h_stat[2];
    c->prof_collect();
    c->collected = true;
    c->views_off = false;
    return 0;
}

int mm2g_batch_map(mm2g_ctx* c, const mm2g_map_opts* o) {
    if (!c || !o) return set_err(MM2G_E_ARG, "null argument");
    if (!c->have_index) return set_err(MM2G_E_STATE, "no index uploaded");
    return map_enqueue(c, o, false);
}

static void unpack_keys(const KeyLayout& kl, uint64_t span, const uint64_t* k, int64_t A, uint64_t* xy);

// -n <= 1 with -m <= k: the backtrack, merge, selection and PAF records of every
// read on the host (mm2g_multi.cpp) from the full sorted anchors and the final
// DP pass's f / pprev; the read's result describes its first (primary) line.
static int multi_epilogue(mm2g_ctx* c) {
    const uint32_t n = c->n_reads;
    const HostIndex& H = *c->hidx;
    const mm2g_map_opts& o = c->last_opts;
    std::vector<uint64_t> aoff((size_t)n + 1);
    HIPCHK(hipMemcpy(aoff.data(), c->a_off.p, ((size_t)n + 1) * 8, hipMemcpyDeviceToHost));
    const uint64_t A = aoff[n];
    // keys, f and pprev into the context's pinned buffer (DMA at full PCIe rate, kept across
    // batches); the keys are unpacked per read by the workers below
    if (c->h_multi_cap < A * 16) {
        if (c->h_multi) (void)hipHostFree(c->h_multi);
        c->h_multi = nullptr; c->h_multi_cap = 0;
        const size_t want = std::max<size_t>(A * 16 + A * 4, 1 << 20);   // 25 % slack for the next batches
        if (hipHostMalloc((void**)&c->h_multi, want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            c->h_multi = nullptr;
            return set_err(MM2G_E_NOMEM, "multi-chain epilogue: %zu B of pinned host memory", want);
        }
        c->h_multi_cap = want;
    }
    const uint64_t* keys = (const uint64_t*)c->h_multi;
    const int32_t* f = (const int32_t*)(c->h_multi + A * 8);
    const int32_t* pp = (const int32_t*)(c->h_multi + A * 12);
    if (A) {
        HIPCHK(hipMemcpy(c->h_multi, c->keys.p, A * 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(c->h_multi + A * 8, c->fbuf.p, A * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(c->h_multi + A * 12, c->ppbuf.p, A * 4, hipMemcpyDeviceToHost));
    }
    // query minimizer positions of the dv sketch (idx.w, idx.k; paf.rs:155-160)
    const SketchBufs& D = c->dv_separate ? c->sk2 : c->sk1;
    std::vector<uint64_t> mb(n);
    std::vector<uint32_t> mc(n);
    if (n) {
        HIPCHK(hipMemcpy(mb.data(), D.base.p, (size_t)n * 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(mc.data(), D.cnt.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    }
    uint64_t yend = 0;
    for (uint32_t i = 0; i < n; ++i) yend = std::max<uint64_t>(yend, mb[i] + mc[i]);
    std::vector<uint32_t> my(yend);
    if (yend) HIPCHK(hipMemcpy(my.data(), D.y.p, yend * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> tlen(H.n_seq);
    for (uint32_t t = 0; t < H.n_seq; ++t) tlen[t] = H.seq[t].len;
    const int32_t kdv = c->dv_separate ? H.k : o.k;
    mm2g::MultiParams P{o.min_cnt, o.min_chain_score, 500, o.max_gap, o.mask_level, o.pri_ratio, o.best_n};
    c->multi.assign(n, mm2g::MultiRead{});
    // reads are independent: blocks of 64 handed out to the host_threads pool.  A worker
    // that throws (std::bad_alloc on a 100 kb read's vectors) records the first error and stops the
    // others; every started thread is joined and the call returns an MM2G error
    std::atomic<uint32_t> next{0};
    std::atomic<int> failed{0};
    std::mutex err_mu;
    std::string err_msg;
    auto work = [&]() {
    try {
    std::vector<int32_t> mp;
    std::vector<uint64_t> xy;
    for (;;) {
    const uint32_t b0 = next.fetch_add(64);
    if (b0 >= n) break;
    for (uint32_t i = b0; i < std::min(n, b0 + 64); ++i) {
        mm2g_read_result& r = c->h_res[i];
        if (!(r.flags & MM2G_R_MAPPED)) continue;
        const uint64_t a0 = aoff[i], na = aoff[i + 1] - aoff[i];
        mp.resize(mc[i]);
        for (uint32_t t = 0; t < mc[i]; ++t) mp[t] = (int32_t)(my[mb[i] + t] >> 1);
        xy.resize(2 * na);
        unpack_keys(c->kl, (uint64_t)o.k, keys + a0, (int64_t)na, xy.data());
        // avg_k = sum of spans / count in f32 (query spans are all k, non-HPC)
        const float avg_k = mc[i] ? (float)((uint64_t)mc[i] * (uint64_t)kdv) / (float)mc[i] : (float)H.k;
        mm2g::MultiRead& M = c->multi[i];
        mm2g::multi_chain_read(xy.data(), f + a0, pp + a0, (int64_t)na, r.qlen, mp.data(), (int64_t)mc[i],
                               avg_k, kdv, tlen.data(), H.n_seq, P, M);
        const int32_t keep = r.flags & MM2G_R_RESCUED;
        const int32_t qlen = r.qlen, nanc = r.n_anchors;
        memset(&r, 0, sizeof r);
        r.qlen = qlen; r.n_anchors = nanc;
        r.m_dv = (int32_t)mc[i]; r.sum_k = (int64_t)mc[i] * kdv;
        if (M.panic) { r.flags = MM2G_R_MAPPED | MM2G_R_PANIC | keep; continue; }
        if (M.lines.empty()) continue;
        const mm2g::MultiLine& L = M.lines[0];
        r.flags = MM2G_R_MAPPED | keep | (L.dv_found ? MM2G_R_DV_FOUND : 0);
        r.score = M.s1; r.cm = L.cm; r.qs = L.qs; r.qe = L.qe; r.ts = L.ts; r.te = L.te; r.rid = L.rid; r.rev = L.rev;
        r.n_match = L.n_match; r.dv_st = L.dv_st; r.dv_en = L.dv_en; r.dv = L.dv;
    }
    if (failed.load()) break;
    }
    } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(err_mu);
        if (!failed.exchange(1)) err_msg = e.what();
        next.store(n);
    }
    };
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(c->knob[MM2G_KNOB_HOST_THREADS], (n + 63) / 64));
    std::vector<std::thread> th;
    try {
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
    } catch (const std::exception&) {}    // fewer threads than asked: the started ones and this one finish the work
    work();
    for (auto& t : th) t.join();
    if (failed.load()) return set_err(MM2G_E_NOMEM, "multi-chain epilogue: %s", err_msg.c_str());
    return 0;
}

int mm2g_batch_results(mm2g_ctx* c, mm2g_read_result* res, uint32_t n) {
    if (!c) return set_err(MM2G_E_ARG, "null context");
    if (!c->mapped || c->stop_after_sort) return set_err(MM2G_E_STATE, "batch not mapped");
    if (n > c->n_reads) return set_err(MM2G_E_ARG, "n exceeds the batch size");
    HIPCHK(hipSetDevice(c->device));
    if (int e = wait_batch(c)) return e;
    const HostIndex& H = *c->hidx;
    const int kdv = c->dv_separate ? H.k : c->last_opts.k;
    uint64_t cnt[6] = {c->total_bases, c->h_stat[3], 0, c->n_anchors, 0, 0};
    uint64_t scls[3] = {0, 0, 0};   // anchors per sort class (counters 18-20, launch_sort_read)
    c->h_res.resize(c->n_reads);
    for (uint32_t i = 0; i < c->n_reads; ++i) {
        const ReadOut& o = c->h_out[i];
        cnt[4] += (o.flags & RF_RESCUED) ? (uint64_t)o.n_anchors : 0;
        cnt[5] += o.dp_pairs;
        cnt[2] += (uint64_t)o.m_kept;
        mm2g_read_result& r = c->h_res[i];
        memset(&r, 0, sizeof r);
        const uint64_t L = c->h_rd_off[i + 1] - c->h_rd_off[i];
        r.qlen = (int32_t)L;
        if (L == 0) { r.flags = MM2G_R_EMPTY; continue; }
        r.n_anchors = o.n_anchors;
        {
            const uint32_t na = (uint32_t)o.n_anchors;
            if (na > 1) scls[na <= c->small_last ? 0 : (c->filt_last && na <= 65535u) ? 1 : 2] += na;
        }
        if (!(o.flags & RF_MAPPED)) continue;
        r.flags = MM2G_R_MAPPED | ((o.flags & RF_RESCUED) ? MM2G_R_RESCUED : 0) | ((o.flags & RF_DV_FOUND) ? MM2G_R_DV_FOUND : 0) |
                  ((o.flags & RF_PANIC) ? MM2G_R_PANIC : 0);
        r.score = o.score; r.cm = o.cm; r.qs = o.qs; r.qe = o.qe; r.ts = o.ts; r.te = o.te;
        const uint32_t g = (uint32_t)o.group;
        if (g == 2u * H.n_seq) { r.rid = 0x7fffffff; r.rev = 1; }
        else if (g >= H.n_seq) { r.rid = (int32_t)(g - H.n_seq); r.rev = 1; }
        else { r.rid = (int32_t)g; r.rev = 0; }
        r.n_match = o.n_match; r.dv_st = o.dv_st; r.dv_en = o.dv_en; r.m_dv = o.m_dv;
        r.sum_k = (int64_t)o.m_dv * kdv;      // query spans are all k (non-HPC)
        // dv (paf.rs:189-199): f32 op by op, glibc powf
        r.dv = 0.0f;
        if ((o.flags & RF_DV_FOUND) && !(o.flags & RF_PANIC)) {
            const float avg_k = r.m_dv ? (float)(uint64_t)r.sum_k / (float)(uint64_t)r.m_dv : (float)H.k;
            int32_t n_tot = o.dv_en - o.dv_st + 1;
            const int32_t qlen = r.qlen;
            const int32_t rqs = r.rev ? qlen - r.qe : r.qs, rqe = r.rev ? qlen - r.qs : r.qe;
            const int32_t ak = (int32_t)avg_k;
            const int32_t tlen = (int32_t)H.seq[r.rid].len;
            if (rqs > ak && r.ts > ak) n_tot += 1;
            if (qlen - rqe > ak && tlen - r.te > ak) n_tot += 1;
            const float frac = (float)r.n_match / (float)n_tot;
            r.dv = frac >= 1.0f ? 0.0f : 1.0f - powf(frac, 1.0f / fmaxf(avg_k, 1.0f));
        }
    }
    if (c->multi_last) { if (int e = multi_epilogue(c)) return e; }
    else c->multi.clear();
    if (res && n) memcpy(res, c->h_res.data(), (size_t)n * sizeof(mm2g_read_result));
    for (int t = 0; t < 6; ++t) c->counters[t] = cnt[t];
    c->counters[6] = c->h_stat[4];    // anchors left after the sort's singleton filter (the DP input)
    for (int t = 0; t < 6; ++t) c->counters[7 + t] = c->h_stat[8 + t];   // anchors per chain kernel class and pass
    c->counters[13] = c->h_stat[5];   // DP anchors whose keys k_chain_seg streams (pass 0; the rest: sparse items)
    c->counters[14] = c->lb_ran0 ? c->h_stat[4] : 0;   // ... that k_chain_lb streams (pass 0; 0 when it did not run)
    c->counters[15] = c->h_stat[6];   // rescued anchors whose keys k_chain_seg streams (pass 1)
    c->counters[16] = c->h_stat[7];   // anchors of the reads k_sort_read seeds itself (fused seeding)
    c->counters[17] = c->h_stat[14];  // ... and their minimizers
    for (int t = 0; t < 3; ++t) c->counters[18 + t] = scls[t];
    c->counters[21] = c->h_stat[15];  // anchors of the reads k_sort_big seeds itself
    c->counters[22] = c->h_stat[16];  // ... and their minimizers
    return 0;
}

static inline char* put_u(char* p, uint64_t v) {
    char tmp[24]; int n = 0;
    do { tmp[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (n) *p++ = tmp[--n];
    return p;
}

static int64_t format_paf(const HostIndex& H, const mm2g_read_result* res, const char* const* names, uint32_t n, char* out, int64_t cap) {
    int64_t o = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const mm2g_read_result& r = res[i];
        if (!(r.flags & MM2G_R_MAPPED) || (r.flags & MM2G_R_PANIC)) continue;
        const HostSeq& s = H.seq[r.rid];
        const char* tname = s.has_name ? s.name.c_str() : "*";
        const size_t qn = strlen(names[i]), tn = strlen(tname);
        char line[512];
        char* p = line;
        const uint32_t qlen = (uint32_t)r.qlen, qs = (uint32_t)r.qs, qe = (uint32_t)r.qe;
        const uint32_t pqs = r.rev ? qlen - qe : qs, pqe = r.rev ? qlen - qs : qe;   // write_paf (paf.rs:225-227)
        *p++ = '\t'; p = put_u(p, qlen); *p++ = '\t'; p = put_u(p, pqs); *p++ = '\t'; p = put_u(p, pqe);
        *p++ = '\t'; *p++ = r.rev ? '-' : '+'; *p++ = '\t';
        char* q = line + 256;
        *q++ = '\t'; q = put_u(q, s.len); *q++ = '\t'; q = put_u(q, (uint32_t)r.ts); *q++ = '\t'; q = put_u(q, (uint32_t)r.te);
        *q++ = '\t'; q = put_u(q, (uint32_t)std::max(r.qe - r.qs, 0)); *q++ = '\t'; q = put_u(q, (uint32_t)std::max(r.te - r.ts, 0));
        q = put_lit(q, "\t60\ttp:A:P\tcm:i:"); q = put_u(q, (uint32_t)r.cm);
        q = put_lit(q, "\ts1:i:"); q = put_u(q, (uint32_t)std::max(r.score, 0));
        q = put_lit(q, "\ts2:i:0\tdv:f:");
        q += snprintf(q, 32, "%.4f", (double)r.dv);
        q = put_lit(q, "\trl:i:0\n");
        const int64_t len = (int64_t)qn + (p - line) + (int64_t)tn + (q - (line + 256));
        if (out) {
            if (o + len > cap) return set_err(MM2G_E_NOMEM, "PAF output buffer too small");
            memcpy(out + o, names[i], qn); o += (int64_t)qn;
            memcpy(out + o, line, (size_t)(p - line)); o += p - line;
            memcpy(out + o, tname, tn); o += (int64_t)tn;
            memcpy(out + o, line + 256, (size_t)(q - (line + 256))); o += q - (line + 256);
        } else o += len;
    }
    return o;
}

int64_t mm2g_multi_chain_lines(const uint64_t* xy, const int32_t* f, const int32_t* pprev, int64_t n, int32_t qlen,
                               const int32_t* mini_pos, int64_t n_mini, float avg_k, const uint32_t* tlen, uint32_t n_seq,
                               const mm2g_map_opts* o, mm2g_chain_line* out, int64_t cap, int32_t* panic) {
    if (!o || n < 0 || n_mini < 0 || (n && (!xy || !f || !pprev)) || (n_mini && !mini_pos) || (n_seq && !tlen) || (cap && !out))
        return set_err(MM2G_E_ARG, "null argument");
    mm2g::MultiParams P{o->min_cnt, o->min_chain_score, 500, o->max_gap, o->mask_level, o->pri_ratio, o->best_n};
    mm2g::MultiRead M;
    mm2g::multi_chain_read(xy, f, pprev, n, qlen, mini_pos, n_mini, avg_k, 0, tlen, n_seq, P, M);
    if (panic) *panic = M.panic ? 1 : 0;
    if (M.panic) return set_err(MM2G_E_STATE, "the reference panics on this read");
    for (size_t i = 0; i < M.lines.size() && (int64_t)i < cap; ++i) {
        const mm2g::MultiLine& L = M.lines[i];
        out[i] = mm2g_chain_line{L.qs, L.qe, L.ts, L.te, L.rid, L.rev, L.cm, L.primary ? 1 : 0, L.dv, M.s1, M.s2};
    }
    return (int64_t)M.lines.size();
}

int64_t mm2g_format_paf(const mm2g_index* idx, const mm2g_read_result* res, const char* const* names, uint32_t n, char* out, int64_t cap) {
    if (!idx || (n && (!res || !names))) return set_err(MM2G_E_ARG, "null argument");
    return format_paf(idx->h, res, names, n, out, cap);
}

int64_t mm2g_batch_paf(mm2g_ctx* c, const char* const* names, uint32_t n, char* out, int64_t cap) {
    if (!c || (n && !names)) return set_err(MM2G_E_ARG, "null argument");
    if (!c->mapped || !c->collected || c->h_res.size() != c->n_reads) return set_err(MM2G_E_STATE, "call mm2g_batch_results first");
    if (n > c->n_reads) return set_err(MM2G_E_ARG, "n exceeds the batch size");
    const HostIndex& H = *c->hidx;
    if (!c->multi_last) return format_paf(H, c->h_res.data(), names, n, out, cap);
    // several lines per read: write_paf_many_with_scores (paf.rs:238-248) -> write_paf (:224-236)
    int64_t o = 0;
    std::string line;
    for (uint32_t i = 0; i < n; ++i) {
        const mm2g::MultiRead& M = c->multi[i];
        if (M.panic) continue;                       // the reference panics before printing (main.rs:218-226)
        const uint32_t qlen = (uint32_t)c->h_res[i].qlen;
        for (const mm2g::MultiLine& L : M.lines) {
            const HostSeq& sq = H.seq[L.rid];
            const uint32_t qs = (uint32_t)L.qs, qe = (uint32_t)L.qe;
            const uint32_t pqs = L.rev ? qlen - qe : qs, pqe = L.rev ? qlen - qs : qe;
            char buf[320];
            line.assign(names[i]);
            snprintf(buf, sizeof buf, "\t%u\t%u\t%u\t%c\t", qlen, pqs, pqe, L.rev ? '-' : '+');
            line += buf;
            line += sq.has_name ? sq.name.c_str() : "*";
            snprintf(buf, sizeof buf, "\t%u\t%u\t%u\t%u\t%u\t60\ttp:A:%c\tcm:i:%u\ts1:i:%u\ts2:i:%u\tdv:f:%.4f\trl:i:0\n",
                     sq.len, (uint32_t)L.ts, (uint32_t)L.te, (uint32_t)std::max(L.qe - L.qs, 0), (uint32_t)std::max(L.te - L.ts, 0),
                     L.primary ? 'P' : 'S', (uint32_t)L.cm, (uint32_t)std::max(M.s1, 0), (uint32_t)std::max(M.s2, 0), (double)L.dv);
            line += buf;
            if (out) {
                if (o + (int64_t)line.size() > cap) return set_err(MM2G_E_NOMEM, "PAF output buffer too small");
                memcpy(out + o, line.data(), line.size());
            }
            o += (int64_t)line.size();
        }
    }
    return o;
}

// ------------------------------------------------------------------ stages
int mm2g_batch_sketch(mm2g_ctx* c, int w, int k, uint32_t rid, uint64_t* out_off, uint64_t* out_ks, uint64_t* out_rps, uint64_t cap) {
    if (!c) return set_err(MM2G_E_ARG, "null context");
    if (!(w > 0 && w < 256 && k > 0 && k <= 28)) return set_err(MM2G_E_ARG, "invalid w/k (0 < w < 256, 0 < k <= 28)");
    HIPCHK(hipSetDevice(c->device));
    const uint32_t n = c->n_reads;
    for (uint32_t i = 0; i < n; ++i)
        if (c->h_rd_off[i + 1] == c->h_rd_off[i]) return set_err(MM2G_E_ARG, "empty sequence (src/sketch.rs:30-32)");
    c->mapped = false;                      // the sketch reuses the dv sketch's slots
    SketchBufs& B = c->sk2;
    B.exact = false;
    int32_t* ovf;
    unsigned long long* st;
    ENSURE(c->dstat, unsigned long long, STAT_WORDS, st);
    ovf = (int32_t*)st + 1;
    for (int it = 0;; ++it) {
        HIPCHK(hipMemsetAsync(st, 0, STAT_WORDS * 8, c->stream));
        if (int e = run_sketch(c, w, k, B, ovf)) return e;
        int32_t o = 0;
        HIPCHK(hipMemcpyAsync(&o, ovf, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (!o) break;
        if (it) { c->views_off = false; return set_err(MM2G_E_STATE, "sketch slots did not converge"); }
        if (int e = sketch_exact_layout(c, B)) return e;
        c->views_off = true;   // a view may have overflowed its own slot: whole-read sketch for the re-run
    }
    c->views_off = false;
    std::vector<uint32_t> hc(n); std::vector<uint64_t> hb(n);
    if (n) {
        HIPCHK(hipMemcpyAsync(hc.data(), B.cnt.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(hb.data(), B.base.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    uint64_t run = 0;
    for (uint32_t i = 0; i < n; ++i) { if (out_off) out_off[i] = run; run += hc[i]; }
    if (out_off) out_off[n] = run;
    if (!out_ks && !out_rps) return 0;
    if (run > cap) return set_err(MM2G_E_ARG, "output capacity too small");
    std::vector<uint64_t> x; std::vector<uint32_t> y;
    for (uint32_t i = 0; i < n; ++i) {
        x.resize(hc[i]); y.resize(hc[i]);
        if (hc[i]) {
            HIPCHK(hipMemcpy(x.data(), (uint64_t*)B.x.p + hb[i], hc[i] * 8, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(y.data(), (uint32_t*)B.y.p + hb[i], hc[i] * 4, hipMemcpyDeviceToHost));
        }
        const uint64_t o0 = out_off ? out_off[i] : 0;
        for (uint32_t t = 0; t < hc[i]; ++t) {
            if (out_ks) out_ks[o0 + t] = x[t];
            if (out_rps) out_rps[o0 + t] = ((uint64_t)rid << 32) | y[t];
        }
    }
    return 0;
}

// Sorted device keys of one read -> the reference's Anchor (x, y) (seeds.rs:62-79).
static void unpack_keys(const KeyLayout& kl, uint64_t span, const uint64_t* k, int64_t A, uint64_t* xy) {
    const uint64_t qm = (1ULL << kl.qb) - 1, rm = (1ULL << kl.rb) - 1;
    for (int64_t i = 0; i < A; ++i) {
        const uint64_t g = k[i] >> (kl.rb + kl.qb), p = (k[i] >> kl.qb) & rm, q = k[i] & qm;
        uint64_t x;
        if (g == 2ull * kl.n_seq) x = 0xffffffff80000000ULL | p;
        else if (g >= kl.n_seq) x = (1ULL << 63) | ((g - kl.n_seq) << 32) | p;
        else x = (g << 32) | p;
        xy[2 * i] = x; xy[2 * i + 1] = (span << 32) | q;
    }
}

int64_t mm2g_seed_batch(mm2g_ctx* c, const mm2g_map_opts* o, uint64_t* a_off, uint64_t* xy, uint64_t cap) {
    if (!c || !o || !a_off) return set_err(MM2G_E_ARG, "null argument");
    if (!c->have_index) return set_err(MM2G_E_STATE, "no index uploaded");
    HIPCHK(hipSetDevice(c->device));
    const mm2g_map_opts& L = c->last_opts;    // field by field: no struct padding in the comparison
    const bool same = c->mapped && c->stop_after_sort && L.w == o->w && L.k == o->k && L.max_gap == o->max_gap && L.bw == o->bw &&
                      L.bw_long == o->bw_long && L.min_cnt == o->min_cnt && L.min_chain_score == o->min_chain_score &&
                      L.mask_level == o->mask_level && L.pri_ratio == o->pri_ratio && L.best_n == o->best_n;
    if (!same)
        if (int e = map_enqueue(c, o, true)) return e;
    if (int e = wait_batch(c)) return e;
    const uint32_t n = c->n_reads;
    HIPCHK(hipMemcpyAsync(a_off, c->a_off.p, ((size_t)n + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint64_t A = n ? a_off[n] : 0;
    if (!n) a_off[0] = 0;
    if (!xy) return (int64_t)A;
    if (A > cap) return set_err(MM2G_E_ARG, "output capacity too small (%llu anchors)", (unsigned long long)A);
    std::vector<uint64_t> k(A);
    if (A) HIPCHK(hipMemcpy(k.data(), c->keys.p, A * 8, hipMemcpyDeviceToHost));
    unpack_keys(c->kl, (uint64_t)o->k, k.data(), (int64_t)A, xy);
    return (int64_t)A;
}

void mm2g_chain_params_default(mm2g_chain_params* p, int k) {
    // default_chain_params (src/main.rs:105-123)
    p->max_dist_x = 5000; p->max_dist_y = 5000; p->bw = 500; p->max_chain_iter = 5000; p->min_chain_score = 40; p->min_cnt = 3;
    p->chn_pen_gap = 0.01f * 0.8f * (float)k; p->chn_pen_skip = 0.0f; p->max_chain_skip = 25; p->max_drop = 500;
    p->bw_long = 20000; p->rmq_rescue_size = 1000; p->rmq_rescue_ratio = 0.1f;
}

int mm2g_chain_batch(mm2g_ctx* c, const mm2g_chain_params* p, uint32_t n, const uint64_t* a_off, const uint64_t* xy, const int32_t* qlen,
                     int rescue, mm2g_chain_result* res, int32_t* f, int32_t* pprev, uint32_t* chain) {
    if (!c || !p || !a_off || (n && !qlen) || !res) return set_err(MM2G_E_ARG, "null argument");
    const uint64_t A = a_off[n] - a_off[0];
    if (A && !xy) return set_err(MM2G_E_ARG, "null anchors");
    if (p->chn_pen_skip != 0.0f) return set_err(MM2G_E_UNSUP, "chn_pen_skip != 0 (the reference fixes it at 0, main.rs:116)");
    if (p->bw < 0 || p->bw_long < 0 || p->max_chain_iter < 1 || p->max_chain_skip < 0) return set_err(MM2G_E_ARG, "invalid chain parameters");
    if (std::max(p->bw, p->bw_long) + 1 > 60000) return set_err(MM2G_E_UNSUP, "bandwidth > 59999 not supported");
    HIPCHK(hipSetDevice(c->device));
    // key layout from the anchors themselves: groups by (rev, rid), the Q19
    // pseudo-group (x>>32 == 0xffffffff) last; order-preserving, so the caller's
    // (x, y) order must be the key order (checked)
    uint64_t max_rid = 0, max_p = 0, max_q = 0;
    int64_t span = -1;
    for (uint64_t i = 0; i < A; ++i) {
        const uint64_t x = xy[2 * i], y = xy[2 * i + 1];
        const uint32_t hi = (uint32_t)(x >> 32);
        if (hi != 0xffffffffu) {
            if (x & 0x80000000ULL) return set_err(MM2G_E_UNSUP, "anchor %llu: rpos >= 2^31 outside the Q19 group", (unsigned long long)i);
            max_rid = std::max<uint64_t>(max_rid, hi & 0x7fffffffu);
        }
        max_p = std::max<uint64_t>(max_p, x & 0x7fffffffULL);
        max_q = std::max<uint64_t>(max_q, y & 0xffffffffULL);
        const int64_t sp = (int64_t)((y >> 32) & 0xff);
        if ((y >> 40) != 0) return set_err(MM2G_E_UNSUP, "anchor %llu: y above the span byte", (unsigned long long)i);
        if (span < 0) span = sp;
        else if (sp != span) return set_err(MM2G_E_UNSUP, "anchors of different spans (the device DP keeps one span)");
    }
    if (span < 0) span = 15;
    if (p->min_cnt < 2 && A && p->min_chain_score <= span)   // see check_opts: one-anchor backtrack chains can pass
        return set_err(MM2G_E_UNSUP, "min_cnt %d with min_chain_score %d <= span %lld: Rust sort_unstable tie order (DESIGN.md \"-n <= 1\")",
                       p->min_cnt, p->min_chain_score, (long long)span);
    KeyLayout kl;
    kl.n_seq = (uint32_t)max_rid + 1;
    kl.qb = std::max<uint32_t>(1, bit_width(max_q));
    kl.rb = std::max<uint32_t>(1, bit_width(max_p));
    kl.gb = std::max<uint32_t>(1, bit_width(2ull * kl.n_seq));
    if (kl.qb + kl.rb + kl.gb > 64) return set_err(MM2G_E_UNSUP, "anchor key needs %u bits (> 64)", kl.qb + kl.rb + kl.gb);
    std::vector<uint64_t> keys(A), ho(n + 1), hro(n + 1, 0);
    std::vector<uint32_t> hcnt(n);
    for (uint32_t r = 0; r < n; ++r) {
        if (a_off[r + 1] < a_off[r]) return set_err(MM2G_E_ARG, "a_off must be non-decreasing");
        if (qlen[r] < 0) return set_err(MM2G_E_ARG, "negative qlen");
        ho[r] = a_off[r] - a_off[0]; hcnt[r] = (uint32_t)(a_off[r + 1] - a_off[r]);
        hro[r + 1] = hro[r] + (uint64_t)qlen[r];
        for (uint64_t i = a_off[r]; i < a_off[r + 1]; ++i) {
            const uint64_t x = xy[2 * (i - a_off[0])], y = xy[2 * (i - a_off[0]) + 1];
            const uint32_t hi = (uint32_t)(x >> 32);
            const uint64_t rid = hi & 0x7fffffffu;
            const uint64_t g = hi == 0xffffffffu ? 2ull * kl.n_seq : (x >> 63) ? kl.n_seq + rid : rid;
            const uint64_t key = (g << (kl.rb + kl.qb)) | ((x & 0x7fffffffULL) << kl.qb) | (y & 0xffffffffULL);
            if (i > a_off[r] && key < keys[i - 1 - a_off[0]])
                return set_err(MM2G_E_UNSUP, "read %u: anchors are not sorted by (x, y) (build_anchors_filtered order, seeds.rs:58)", r);
            keys[i - a_off[0]] = key;
        }
    }
    ho[n] = A;
    c->mapped = false;      // the batch workspaces are reused
    c->kl = kl;
    const uint64_t A_cap = std::max<uint64_t>(A, 1);
    uint64_t *dk, *dt, *doff, *dro, *smax; uint32_t *dcnt, *cnt2; ReadOut* out;
    ENSURE(c->keys, uint64_t, A_cap, dk); ENSURE(c->keys_tmp, uint64_t, A_cap, dt);
    ENSURE(c->a_off, uint64_t, n + 1, doff); ENSURE(c->a_cnt, uint32_t, n + 1, dcnt);
    ENSURE(c->cnt2, uint32_t, n + 1, cnt2); ENSURE(c->smax, uint64_t, n + 1, smax);
    ENSURE(c->chain_rdoff, uint64_t, n + 1, dro);
    ENSURE(c->outb, ReadOut, n + 1, out);
    HIPCHK(hipMemcpyAsync(dk, keys.data(), A * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(doff, ho.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(dro, hro.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if (n) {
        HIPCHK(hipMemcpyAsync(dcnt, hcnt.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(cnt2, hcnt.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));   // every anchor enters the DP
    }
    HIPCHK(hipMemsetAsync(smax, 0, ((size_t)n + 1) * 8, c->stream));
    HIPCHK(hipMemsetAsync(out, 0, sizeof(ReadOut) * ((size_t)n + 1), c->stream));
    ChainKParams P{};
    P.max_dist_x = std::max(p->max_dist_x, p->bw); P.max_dist_y = std::max(p->max_dist_y, p->bw);   // lchain.rs:63-66
    P.bw = p->bw; P.max_iter = p->max_chain_iter; P.max_skip = p->max_chain_skip;
    P.span = (int32_t)span; P.rescue_size = p->rmq_rescue_size; P.rescue_ratio_f = 1.0f - p->rmq_rescue_ratio; P.pass = 0; P.lut_n = p->bw + 1;
    const int32_t mdx1 = std::max(p->max_dist_x, p->bw_long), mdy1 = std::max(p->max_dist_y, p->bw_long);
    if (int e = run_chain(c, n, dro, P, p->chn_pen_gap, rescue ? 2 : 1, mdx1, mdy1, p->bw_long, A_cap, doff, dcnt, dk, dt, cnt2, smax, out,
                          nullptr, c->debug || f || pprev))
        return e;
    std::vector<ReadOut> ho2(n);
    if (n) HIPCHK(hipMemcpyAsync(ho2.data(), out, (size_t)n * sizeof(ReadOut), hipMemcpyDeviceToHost, c->stream));
    if (f && A) HIPCHK(hipMemcpyAsync(f, c->fbuf.p, A * 4, hipMemcpyDeviceToHost, c->stream));
    if (pprev && A) HIPCHK(hipMemcpyAsync(pprev, c->ppbuf.p, A * 4, hipMemcpyDeviceToHost, c->stream));
    std::vector<uint32_t> cb;
    if (chain && A) { cb.resize(A); HIPCHK(hipMemcpyAsync(cb.data(), dt, A * 4, hipMemcpyDeviceToHost, c->stream)); }
    HIPCHK(hipStreamSynchronize(c->stream));
    c->prof_collect();
    for (uint32_t r = 0; r < n; ++r) {
        const ReadOut& o = ho2[r];
        mm2g_chain_result& R = res[r];
        memset(&R, 0, sizeof R);
        R.n_anchors = (int32_t)hcnt[r];
        if (!(o.flags & RF_MAPPED)) continue;
        R.flags = MM2G_R_MAPPED | ((rescue && (o.flags & RF_RESCUED)) ? MM2G_R_RESCUED : 0) | ((o.flags & RF_PANIC) ? MM2G_R_PANIC : 0);
        R.score = o.score; R.cm = o.cm; R.qs = o.qs; R.qe = o.qe; R.ts = o.ts; R.te = o.te;
        const uint32_t g = (uint32_t)o.group;
        if (g == 2u * kl.n_seq) { R.rid = 0x7fffffff; R.rev = 1; }
        else if (g >= kl.n_seq) { R.rid = (int32_t)(g - kl.n_seq); R.rev = 1; }
        else { R.rid = (int32_t)g; R.rev = 0; }
        // chain_dp_all's chains[0]: the pprev walk from best_i, reversed to ascending (lchain.rs:162-173)
        if (chain)
            for (int32_t t = 0; t < o.cm; ++t) chain[ho[r] + t] = cb[ho[r] + (uint64_t)(o.cm - 1 - t)];
    }
    return 0;
}

int mm2g_ctx_set_debug(mm2g_ctx* c, int on) { if (!c) return set_err(MM2G_E_ARG, "null context"); c->debug = on != 0; return 0; }

int mm2g_ctx_set_knob(mm2g_ctx* c, int knob, int64_t value) {
    if (!c) return set_err(MM2G_E_ARG, "null context");
    if (knob <= 0 || knob >= MM2G_KNOB_COUNT) return set_err(MM2G_E_ARG, "unknown knob %d", knob);
    c->knob[knob] = value;
    return 0;
}
int64_t mm2g_ctx_get_knob(const mm2g_ctx* c, int knob) {
    if (!c) return set_err(MM2G_E_ARG, "null context");
    if (knob <= 0 || knob >= MM2G_KNOB_COUNT) return set_err(MM2G_E_ARG, "unknown knob %d", knob);
    return c->knob[knob];
}
int mm2g_set_index_knob(int knob, int64_t value) {
    if (knob <= 0 || knob >= MM2G_IKNOB_COUNT) return set_err(MM2G_E_ARG, "unknown index knob %d", knob);
    g_index_knob[knob].store(value);
    return 0;
}

// The debug accessors read what the last mm2g_batch_map left on the device:
// they wait for it first (the context stream is non-blocking).
static int debug_ready(mm2g_ctx* c, uint32_t r) {
    if (!c || !c->mapped || r >= c->n_reads) return set_err(MM2G_E_STATE, "no mapped batch / bad read index");
    HIPCHK(hipSetDevice(c->device));
    if (int e = wait_batch(c)) return e;
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

// Unpack the sorted keys of read r back into the reference's (x, y).
int64_t mm2g_debug_anchors(mm2g_ctx* c, uint32_t r, uint64_t* xy, int64_t cap) {
    if (int e = debug_ready(c, r)) return e;
    uint64_t off[2];
    HIPCHK(hipMemcpy(off, (uint64_t*)c->a_off.p + r, 16, hipMemcpyDeviceToHost));
    int64_t A = (int64_t)(off[1] - off[0]);
    if (!c->full_last) {   // production sort: only the anchors kept by the singleton filter are sorted
        uint32_t kept = 0;
        HIPCHK(hipMemcpy(&kept, (uint32_t*)c->cnt2.p + r, 4, hipMemcpyDeviceToHost));
        A = kept;
    }
    if (!xy) return A;
    std::vector<uint64_t> k((size_t)A);
    if (A) HIPCHK(hipMemcpy(k.data(), (uint64_t*)c->keys.p + off[0], A * 8, hipMemcpyDeviceToHost));
    const int64_t m = std::min<int64_t>(A, cap);
    unpack_keys(c->kl, (uint64_t)c->last_opts.k, k.data(), m, xy);
    return A;
}
int64_t mm2g_debug_dp(mm2g_ctx* c, uint32_t r, int32_t* f, int32_t* pprev, int64_t cap) {
    if (int e = debug_ready(c, r)) return e;
    uint64_t off[2];
    HIPCHK(hipMemcpy(off, (uint64_t*)c->a_off.p + r, 16, hipMemcpyDeviceToHost));
    const int64_t A = (int64_t)(off[1] - off[0]);
    const int64_t m = std::min<int64_t>(A, cap);
    if (f && m) HIPCHK(hipMemcpy(f, (int32_t*)c->fbuf.p + off[0], m * 4, hipMemcpyDeviceToHost));
    if (pprev && m) HIPCHK(hipMemcpy(pprev, (int32_t*)c->ppbuf.p + off[0], m * 4, hipMemcpyDeviceToHost));
    return A;
}
int64_t mm2g_debug_keep(mm2g_ctx* c, uint32_t r, uint8_t* keep, int64_t cap) {
    if (int e = debug_ready(c, r)) return e;
    uint64_t b; uint32_t m;
    HIPCHK(hipMemcpy(&b, (uint64_t*)c->sk1.base.p + r, 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&m, (uint32_t*)c->sk1.cnt.p + r, 4, hipMemcpyDeviceToHost));
    if (keep && m) HIPCHK(hipMemcpy(keep, (uint8_t*)c->keep.p + b, std::min<int64_t>(m, cap), hipMemcpyDeviceToHost));
    return m;
}

int mm2g_prof_enable(mm2g_ctx* c, int on) { if (!c) return set_err(MM2G_E_ARG, "null context"); c->prof = on != 0; return 0; }
int mm2g_prof_get(mm2g_ctx* c, int i, const char** name, double* ms, int64_t* calls) {
    if (!c) return set_err(MM2G_E_ARG, "null context");
    c->prof_collect();
    if (i < 0 || i >= (int)c->slots.size()) return MM2G_E_ARG;
    if (name) *name = c->slots[i].name.c_str();
    if (ms) *ms = c->slots[i].ms;
    if (calls) *calls = c->slots[i].calls;
    return 0;
}
int mm2g_prof_reset(mm2g_ctx* c) {
    if (!c) return set_err(MM2G_E_ARG, "null context");
    c->prof_collect();
    for (auto& s : c->slots) { s.ms = 0; s.calls = 0; }
    return 0;
}
int64_t mm2g_debug_chain_stats(mm2g_ctx* c, uint32_t* out6, uint32_t n) {
    if (!c) return set_err(MM2G_E_ARG, "null context");
    if (!c->mapped || !c->h_out) return set_err(MM2G_E_STATE, "call mm2g_batch_results first");
    HIPCHK(hipSetDevice(c->device));
    if (int e = wait_batch(c)) return e;        // h_out is filled by an async copy
    if (out6)
        for (uint32_t i = 0; i < n && i < c->n_reads; ++i) {
            const ReadOut& o = c->h_out[i];
            out6[6 * i + 0] = o.t_pass[0]; out6[6 * i + 1] = o.t_pass[1];
            out6[6 * i + 2] = o.n_noniso; out6[6 * i + 3] = o.n_steps; out6[6 * i + 4] = o.n_deep; out6[6 * i + 5] = o.pad2;
        }
    return (int64_t)c->n_reads;
}
int mm2g_batch_counters(mm2g_ctx* c, uint64_t* out, int n) {
    if (!c || !out || n < 0) return set_err(MM2G_E_ARG, "null argument");
    for (int t = 0; t < n && t < MM2G_N_COUNTERS; ++t) out[t] = c->counters[t];
    return n < MM2G_N_COUNTERS ? n : MM2G_N_COUNTERS;
}

}  // extern "C"
