// GPU index build: `mm2rs index` = build_index_from_fasta
// (src/index.rs:427-475) with the reference sketch, bucketing and post_process
// (src/index.rs:69-109) run on the device.
//
//   1. contigs -> HBM; each contig is cut into views of IX_CHUNK bases plus a
//      warm-up before them (view_warmup below).  k_sketch runs one wave per view
//      (SketchArgs view_*): the k-mer registers walk back into the contig (the
//      reference never resets them), l and the w-slot window converge inside
//      the warm-up, and only steps >= the view's own first base emit, so the
//      views' emissions partition the contig's.
//   2. k_ix_compact: (hash, rid<<32 | pos<<1 | strand) pairs, contig order.
//   3. two stable LSD radix sorts (rocPRIM): by value, then by hash -> sorted by
//      (hash, value), which is post_process's order: per hash a run; runs of
//      one are singletons, longer runs sorted position slices.
//   4. the host distributes runs to buckets (hash & (2^b-1)) in hash order:
//      exactly finish_bucket's h / p, so .mmi, stats, mid_occ and the device
//      table are byte-identical with the host build (tests/test_gpu_parity.py).
//   5. S, the 4-bit packed reference (src/index.rs:14-19), is packed on the
//      device (k_pack4).
//   HPC (flag & 1, src/sketch.rs:51-64): the reference never advances i past a
//      homopolymer run, so k-mers are the plain ones and only the
//      spans change: span(i) = sum of skip_len over the last k ACGT bases since
//      the last ambiguous base (TinyQueue), skip_len(j) = the run of base j's
//      code starting at j, to the contig end.  k_hpc_skip / k_hpc_span compute
//      them per base (u16, capped at 256: a span >= 256 gives no info) before
//      the sketch, which reads them (SketchArgs::hpc_span).
#include <hip/hip_runtime.h>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "mm2g_index.h"
#include "mm2g_internal.h"

using namespace mm2g;

namespace {

constexpr int64_t IX_CHUNK = 1 << 16;

__device__ __forceinline__ uint32_t nt4_dev(uint32_t b) {   // src/nt4.rs:2-10
    const uint32_t c = b | 0x20u;
    return c == 'a' ? 0u : c == 'c' ? 1u : c == 'g' ? 2u : c == 't' ? 3u : 4u;
}

// one wave per view: its minimizers -> (hash, rid_pos_strand) at out_off[v]
__global__ __launch_bounds__(256) void k_ix_compact(uint32_t n_views, const uint64_t* mz_base, const uint32_t* mz_cnt,
                                                    const uint64_t* mz_x, const uint32_t* mz_y, const uint32_t* view_rid,
                                                    const uint32_t* view_pre, const uint64_t* out_off, uint64_t* hash, uint64_t* val) {
    const uint32_t v = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= n_views) return;
    const int lane = threadIdx.x & 63;
    const uint64_t b = mz_base[v], o = out_off[v];
    const uint32_t n = mz_cnt[v];
    const uint64_t rid = view_rid[v], pre = view_pre[v];
    for (uint32_t i = lane; i < n; i += 64) {
        const uint64_t x = mz_x[b + i];
        const uint32_t y = mz_y[b + i];
        hash[o + i] = x >> 8;
        val[o + i] = (rid << 32) | ((pre + (y >> 1)) << 1) | (uint64_t)(y & 1u);   // src/sketch.rs:72 (i not truncated)
    }
}

// contig of global position i: the last r with coff[r] <= i (coff: n+1 offsets)
__device__ __forceinline__ uint32_t contig_of(const uint64_t* coff, uint32_t n, uint64_t i) {
    uint32_t lo = 0, hi = n;              // coff[lo] <= i < coff[hi]
    while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (coff[mid] <= i) lo = mid; else hi = mid; }
    return lo;
}

// HPC skip_len (src/sketch.rs:53-58): the run of seq[i]'s code from i on, to
// the contig end, capped at 256 (0 for an ambiguous base)
__global__ __launch_bounds__(256) void k_hpc_skip(const uint8_t* seq, uint64_t total, const uint64_t* coff, uint32_t n,
                                                  uint16_t* skip) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = nt4_dev(seq[i]);
        if (c >= 4) { skip[i] = 0; continue; }
        const uint64_t e = coff[contig_of(coff, n, i) + 1];
        const uint64_t lim = e < i + 256 ? e : i + 256;
        uint64_t t = i + 1;
        while (t < lim && nt4_dev(seq[t]) == c) ++t;
        skip[i] = (uint16_t)(t - i);
    }
}

// HPC span (src/sketch.rs:59-61): TinyQueue holds the last k skip_lens since
// the last ambiguous base (cleared there, :64), so span(i) is their sum over
// j in (i-k, i] back to that base or the contig start; capped at 256
__global__ __launch_bounds__(256) void k_hpc_span(const uint8_t* seq, uint64_t total, const uint64_t* coff, uint32_t n, int k,
                                                  const uint16_t* skip, uint16_t* span) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        if (nt4_dev(seq[i]) >= 4) { span[i] = 0; continue; }
        const uint64_t s0 = coff[contig_of(coff, n, i)];
        uint32_t sum = 0;
        for (uint64_t j = i, m = 0; m < (uint64_t)k && j >= s0; --j, ++m) {
            if (nt4_dev(seq[j]) >= 4) break;
            sum += skip[j];
            if (j == 0) break;
        }
        span[i] = (uint16_t)(sum < 256u ? sum : 256u);
    }
}

// S (src/index.rs:14-19): 8 bases per u32 word, base j of the concatenation in
// bits 4(j%8)..; words past the sequence stay 0 (kroundup64 padding)
__global__ void k_pack4(const uint8_t* seq, uint64_t total, uint64_t n_words, uint32_t* S) {
    const uint64_t wd = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (wd >= n_words) return;
    uint32_t v = 0;
    for (int j = 0; j < 8; ++j) {
        const uint64_t p = wd * 8 + j;
        if (p < total) v |= (nt4_dev(seq[p]) & 0xFu) << (4 * j);
    }
    S[wd] = v;
}

struct Dev {
    std::vector<void*> ptrs;
    ~Dev() { for (void* p : ptrs) (void)hipFree(p); }
    template <typename T>
    T* alloc(size_t n) {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return (T*)p;
    }
};

// Warm-up start of a view whose emissions begin at contig position c0.  The
// sketch starts the view with l = 0 (src/sketch.rs:44,66-70: l counts the
// non-symmetric ACGT k-mers since the last ambiguous base); the reference's l
// there is unknown.  Both agree from the first ambiguous base on, and -- for
// every comparison the reference makes, against k, w+k-1 and w+k -- from the
// (w+k)-th non-symmetric k-mer on.  info and the w-slot window then follow
// after w more steps.  Odd k has no symmetric k-mers, so a fixed 2(w+k)+64
// bases always suffice; with even k a palindromic run ((AT)n, (ACGT)n, ...)
// produces symmetric k-mers only, so the warm-up grows (doubling, down to the
// contig start, where the sketch is exact) until it converges early enough.
// The k-mer registers at vs come from the k-1 ACGT bases before it, as the
// kernel's own walk-back computes them.
int64_t view_warmup(const uint8_t* seq, int64_t c0, int w, int k) {
    const int64_t cap = w + k;
    int64_t warm = 2 * (w + k) + 64;
    const uint64_t mask = (1ULL << (2 * k)) - 1;
    const uint32_t shift1 = 2u * (uint32_t)(k - 1);
    auto nt4h = [](uint8_t b) -> uint32_t {
        const uint32_t c = b | 0x20u;
        return c == 'a' ? 0u : c == 'c' ? 1u : c == 'g' ? 2u : c == 't' ? 3u : 4u;
    };
    for (;;) {
        const int64_t vs = c0 > warm ? c0 - warm : 0;
        if (vs == 0) return 0;
        int64_t p = vs;
        int need = k - 1;
        while (need > 0 && p > 0) { --p; if (nt4h(seq[p]) < 4) --need; }
        uint64_t kf = 0, kr = 0;
        for (; p < vs; ++p) {
            const uint32_t c = nt4h(seq[p]);
            if (c < 4) { kf = ((kf << 2) | c) & mask; kr = (kr >> 2) | ((uint64_t)(3 ^ c) << shift1); }
        }
        int64_t n = 0, conv = -1;
        for (p = vs; p < c0 && conv < 0; ++p) {
            const uint32_t c = nt4h(seq[p]);
            if (c >= 4) { conv = p; break; }
            kf = ((kf << 2) | c) & mask; kr = (kr >> 2) | ((uint64_t)(3 ^ c) << shift1);
            if (kf != kr && ++n >= cap) conv = p;
        }
        if (conv >= 0 && conv + w + 2 <= c0) return vs;
        warm *= 2;
    }
}

inline int bit_width64(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }
inline size_t kroundup64(size_t x) { --x; x |= x >> 1; x |= x >> 2; x |= x >> 4; x |= x >> 8; x |= x >> 16; x |= x >> 32; return x + 1; }

}  // namespace

namespace mm2g {

#define IXCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); return false; } } while (0)

bool build_index_gpu(int device, const std::vector<const uint8_t*>& seqs, const std::vector<uint64_t>& lens,
                     const std::vector<std::string>* names, int w, int k, int b, int flag, HostIndex& idx, std::string& err,
                     bool& unsupported) {
    unsupported = false;
    const bool prof = g_index_knob[2].load() != 0;   // MM2G_IKNOB_IXPROF
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[ixbuild] %-28s %8.3f s\n", what, std::chrono::duration<double>(t - t_last).count());
        t_last = t;
    };
    if (w <= 0 || w >= 256 || k <= 0 || k > 28) { err = "invalid w/k (0 < w < 256, 0 < k <= 28)"; return false; }
    if (b < 1 || b > 30) { err = "invalid bucket bits"; return false; }
    const size_t n = seqs.size();
    for (size_t i = 0; i < n; ++i)
        if (lens[i] >= (1ULL << 31)) { err = "sequences must be shorter than 2^31"; return false; }
    IXCHK(hipSetDevice(device));
    hipStream_t st;
    IXCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{st};
    Dev D;
    idx = HostIndex();
    idx.w = w; idx.k = k; idx.b = b; idx.flag = flag; idx.n_seq = (uint32_t)n;
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        HostSeq s;
        s.has_name = names != nullptr;
        if (names) s.name = (*names)[i];
        s.offset = total; s.len = (uint32_t)lens[i];
        idx.seq.push_back(s);
        idx.max_len = std::max(idx.max_len, s.len);
        total += lens[i];
    }
    // ---- 1. contigs to HBM, views
    uint8_t* d_seq = D.alloc<uint8_t>(total + 64);
    if (!d_seq) { err = "hipMalloc(reference) failed"; return false; }
    for (size_t i = 0; i < n; ++i)
        if (lens[i]) IXCHK(hipMemcpyAsync(d_seq + idx.seq[i].offset, seqs[i], lens[i], hipMemcpyHostToDevice, st));
    int64_t chunk = IX_CHUNK;
    if (const int64_t v = g_index_knob[1].load()) chunk = std::max<int64_t>(256, v);   // MM2G_IKNOB_IXCHUNK (tests)
    std::vector<uint64_t> v_off, v_base, v_end;
    std::vector<uint32_t> v_len, v_pre, v_from, v_rid;
    std::vector<uint8_t> v_last;
    uint64_t cap = 0;
    for (size_t r = 0; r < n; ++r) {
        const int64_t L = (int64_t)lens[r];
        for (int64_t c0 = 0; c0 < L; c0 += chunk) {
            const int64_t vs = c0 ? view_warmup(seqs[r], c0, w, k) : 0, ve = std::min<int64_t>(L, c0 + chunk);
            v_off.push_back(idx.seq[r].offset + (uint64_t)vs);
            v_len.push_back((uint32_t)(ve - vs)); v_pre.push_back((uint32_t)vs); v_from.push_back((uint32_t)(c0 - vs));
            v_last.push_back(ve == L ? 1 : 0); v_rid.push_back((uint32_t)r);
            v_base.push_back(cap); cap += (uint64_t)(ve - vs) + 16; v_end.push_back(cap);
        }
    }
    const uint32_t nv = (uint32_t)v_off.size();
    std::vector<uint32_t> S_host;
    idx.S.assign(kroundup64((size_t)((total + 7) / 8)), 0u);
    if (nv == 0) { idx.B.assign((size_t)1 << b, HostBucket()); return true; }
    uint64_t* d_voff = D.alloc<uint64_t>(nv); uint32_t* d_vlen = D.alloc<uint32_t>(nv); uint32_t* d_vpre = D.alloc<uint32_t>(nv);
    uint32_t* d_vfrom = D.alloc<uint32_t>(nv); uint8_t* d_vlast = D.alloc<uint8_t>(nv); uint32_t* d_vrid = D.alloc<uint32_t>(nv);
    uint64_t* d_vbase = D.alloc<uint64_t>(nv); uint64_t* d_vend = D.alloc<uint64_t>(nv);
    uint64_t* d_mx = D.alloc<uint64_t>(cap); uint32_t* d_my = D.alloc<uint32_t>(cap); uint32_t* d_cnt = D.alloc<uint32_t>(nv);
    int32_t* d_ovf = D.alloc<int32_t>(4);
    if (!d_voff || !d_vlen || !d_vpre || !d_vfrom || !d_vlast || !d_vrid || !d_vbase || !d_vend || !d_mx || !d_my || !d_cnt || !d_ovf) {
        err = "hipMalloc(index views) failed"; return false;
    }
    IXCHK(hipMemcpyAsync(d_voff, v_off.data(), nv * 8, hipMemcpyHostToDevice, st));
    IXCHK(hipMemcpyAsync(d_vlen, v_len.data(), nv * 4, hipMemcpyHostToDevice, st));
    IXCHK(hipMemcpyAsync(d_vpre, v_pre.data(), nv * 4, hipMemcpyHostToDevice, st));
    IXCHK(hipMemcpyAsync(d_vfrom, v_from.data(), nv * 4, hipMemcpyHostToDevice, st));
    IXCHK(hipMemcpyAsync(d_vlast, v_last.data(), nv, hipMemcpyHostToDevice, st));
    IXCHK(hipMemcpyAsync(d_vrid, v_rid.data(), nv * 4, hipMemcpyHostToDevice, st));
    IXCHK(hipMemcpyAsync(d_vbase, v_base.data(), nv * 8, hipMemcpyHostToDevice, st));
    IXCHK(hipMemcpyAsync(d_vend, v_end.data(), nv * 8, hipMemcpyHostToDevice, st));
    IXCHK(hipMemsetAsync(d_ovf, 0, 16, st));
    // ---- 2. S on the device (overlaps nothing on the host; small)
    {
        uint32_t* d_S = D.alloc<uint32_t>(idx.S.size());
        if (!d_S) { err = "hipMalloc(S) failed"; return false; }
        const uint64_t nw = idx.S.size();
        hipLaunchKernelGGL(k_pack4, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, d_seq, total, nw, d_S);
        IXCHK(hipGetLastError());
        IXCHK(hipMemcpyAsync(idx.S.data(), d_S, nw * 4, hipMemcpyDeviceToHost, st));
    }
    // ---- 3. HPC spans (flag & 1), then sketch every view (one wave each)
    uint16_t* d_span = nullptr;
    if (flag & 1) {
        std::vector<uint64_t> coff(n + 1, 0);
        for (size_t i = 0; i < n; ++i) coff[i + 1] = coff[i] + lens[i];
        uint64_t* d_coff = D.alloc<uint64_t>(n + 1);
        uint16_t* d_skip = D.alloc<uint16_t>(total);
        d_span = D.alloc<uint16_t>(total);
        if (!d_coff || !d_skip || !d_span) { err = "hipMalloc(HPC spans) failed"; return false; }
        IXCHK(hipMemcpyAsync(d_coff, coff.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
        const unsigned nb = (unsigned)std::min<uint64_t>((total + 255) / 256, 65536);
        hipLaunchKernelGGL(k_hpc_skip, dim3(nb), dim3(256), 0, st, d_seq, total, d_coff, (uint32_t)n, d_skip);
        IXCHK(hipGetLastError());
        hipLaunchKernelGGL(k_hpc_span, dim3(nb), dim3(256), 0, st, d_seq, total, d_coff, (uint32_t)n, k, d_skip, d_span);
        IXCHK(hipGetLastError());
    }
    SketchArgs sa{d_seq, nullptr, nv, w, k, d_vbase, d_vend, d_mx, d_my, d_cnt, d_ovf};
    sa.view_off = d_voff; sa.view_len = d_vlen; sa.view_pre = d_vpre; sa.emit_from = d_vfrom; sa.view_last = d_vlast;
    sa.hpc_span = d_span;
    if (launch_sketch(sa, (int)std::min<uint32_t>((nv + 3) / 4, 4096u), st) != 0) { err = "k_sketch launch failed"; return false; }
    std::vector<uint32_t> cnt(nv);
    int32_t ovf = 0;
    IXCHK(hipMemcpyAsync(cnt.data(), d_cnt, nv * 4, hipMemcpyDeviceToHost, st));
    IXCHK(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, st));
    IXCHK(hipStreamSynchronize(st));
    if (ovf) { unsupported = true; err = "GPU index build: minimizer slot overflow (host build)"; return false; }
    lap("H2D + S + sketch");
    std::vector<uint64_t> ooff(nv);
    uint64_t M = 0;
    for (uint32_t v = 0; v < nv; ++v) { ooff[v] = M; M += cnt[v]; }
    // ---- 4. pairs, then sort by (hash, value)
    uint64_t* d_ooff = D.alloc<uint64_t>(nv);
    uint64_t* h0 = D.alloc<uint64_t>(M); uint64_t* v0 = D.alloc<uint64_t>(M);
    uint64_t* h1 = D.alloc<uint64_t>(M); uint64_t* v1 = D.alloc<uint64_t>(M);
    if (!d_ooff || !h0 || !v0 || !h1 || !v1) { err = "hipMalloc(index pairs) failed"; return false; }
    IXCHK(hipMemcpyAsync(d_ooff, ooff.data(), nv * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_ix_compact, dim3((nv + 3) / 4), dim3(256), 0, st, nv, d_vbase, d_cnt, d_mx, d_my, d_vrid, d_vpre, d_ooff, h0, v0);
    IXCHK(hipGetLastError());
    const int vbits = 32 + std::max(1, bit_width64(n ? n - 1 : 0)), hbits = 2 * k;
    size_t tb1 = 0, tb2 = 0;
    IXCHK(rocprim::radix_sort_pairs(nullptr, tb1, v0, v1, h0, h1, (size_t)M, 0, vbits, st));
    IXCHK(rocprim::radix_sort_pairs(nullptr, tb2, h1, h0, v1, v0, (size_t)M, 0, hbits, st));
    void* tmp = D.alloc<uint8_t>(std::max(tb1, tb2));
    if (!tmp) { err = "hipMalloc(sort scratch) failed"; return false; }
    size_t tb = std::max(tb1, tb2);
    IXCHK(rocprim::radix_sort_pairs(tmp, tb, v0, v1, h0, h1, (size_t)M, 0, vbits, st));   // by value (stable)
    tb = std::max(tb1, tb2);
    IXCHK(rocprim::radix_sort_pairs(tmp, tb, h1, h0, v1, v0, (size_t)M, 0, hbits, st));   // then by hash
    // pinned staging: the two sorted arrays come back at PCIe rate
    uint64_t *hh = nullptr, *vv = nullptr;
    IXCHK(hipHostMalloc((void**)&hh, std::max<uint64_t>(M, 1) * 8, hipHostMallocDefault));
    struct PinGuard { uint64_t* p; ~PinGuard() { if (p) (void)hipHostFree(p); } } g1{hh};
    IXCHK(hipHostMalloc((void**)&vv, std::max<uint64_t>(M, 1) * 8, hipHostMallocDefault));
    PinGuard g2{vv};
    IXCHK(hipStreamSynchronize(st));
    lap("pairs + 2 radix sorts");
    IXCHK(hipMemcpyAsync(hh, h0, M * 8, hipMemcpyDeviceToHost, st));
    IXCHK(hipMemcpyAsync(vv, v0, M * 8, hipMemcpyDeviceToHost, st));
    IXCHK(hipStreamSynchronize(st));
    lap("D2H pairs (pinned)");
    // ---- 5. runs -> buckets (finish_bucket's h and p, src/index.rs:77-108).
    // Threads take contiguous hash ranges cut at run starts; per (thread, bucket)
    // counts give every thread its slice of each bucket's h and p, so runs land
    // in hash order exactly as the serial distribution would place them.
    const size_t nb = (size_t)1 << b;
    const uint64_t bmask = nb - 1;
    int nt = (int)std::min<uint64_t>(std::max(1u, std::thread::hardware_concurrency()), 32);
    if (M < (1u << 16)) nt = 1;
    std::vector<uint64_t> cut(nt + 1, M);
    cut[0] = 0;
    for (int t = 1; t < nt; ++t) {
        uint64_t c = M * (uint64_t)t / (uint64_t)nt;
        while (c > 0 && c < M && hh[c] == hh[c - 1]) ++c;
        cut[t] = std::max(c, cut[t - 1]);
    }
    std::vector<std::vector<uint64_t>> cnt_h(nt, std::vector<uint64_t>(nb, 0)), cnt_p(nt, std::vector<uint64_t>(nb, 0));
    auto run_threads = [&](auto fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(fn, t);
        for (auto& x : th) x.join();
    };
    run_threads([&](int t) {
        for (uint64_t s = cut[t]; s < cut[t + 1];) {
            uint64_t e = s + 1;
            while (e < cut[t + 1] && hh[e] == hh[s]) ++e;
            const size_t bk = (size_t)(hh[s] & bmask);
            cnt_h[t][bk] += 1; if (e - s > 1) cnt_p[t][bk] += e - s;
            s = e;
        }
    });
    idx.B.assign(nb, HostBucket());
    for (size_t bk = 0; bk < nb; ++bk) {   // exclusive offsets per (thread, bucket)
        uint64_t oh = 0, op = 0;
        for (int t = 0; t < nt; ++t) {
            const uint64_t ch = cnt_h[t][bk], cp = cnt_p[t][bk];
            cnt_h[t][bk] = oh; cnt_p[t][bk] = op; oh += ch; op += cp;
        }
        idx.B[bk].h.resize(oh); idx.B[bk].p.resize(op);
        idx.B[bk].has_h = oh > 0;
    }
    run_threads([&](int t) {
        std::vector<uint64_t>& oh = cnt_h[t];
        std::vector<uint64_t>& op = cnt_p[t];
        for (uint64_t s = cut[t]; s < cut[t + 1];) {
            uint64_t e = s + 1;
            while (e < cut[t + 1] && hh[e] == hh[s]) ++e;
            const size_t bk = (size_t)(hh[s] & bmask);
            HostBucket& B = idx.B[bk];
            const uint64_t key_top = (hh[s] >> b) << 1;
            if (e - s == 1) B.h[oh[bk]++] = {key_top | 1, vv[s]};
            else {
                B.h[oh[bk]++] = {key_top, (op[bk] << 32) | (uint64_t)(e - s)};
                std::copy(vv + s, vv + e, B.p.begin() + (ptrdiff_t)op[bk]);
                op[bk] += e - s;
            }
            s = e;
        }
    });
    lap("host bucket distribution");
    return true;
}

}  // namespace mm2g
