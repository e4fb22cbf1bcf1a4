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
//   3. a hand-written stable LSD radix sort (8-bit digits, ballot-ranked tiles)
//      by the bucket-major key (hash & (2^b-1), hash >> b) -- after a stable sort
//      by value when the values arrive out of order (even k only) -> sorted by
//      (bucket, hash, value): per hash a run (post_process's order); runs of one
//      are singletons, longer runs sorted position slices.
//   4. runs -> finish_bucket's h / p on the device (scans of run starts and of
//      multi-run members), bucket by bucket; host threads copy each bucket's
//      slices through pinned buffers.  .mmi, stats, mid_occ and the device table
//      are byte-identical with the host build (tests/test_gpu_parity.py).
//   5. S, the 4-bit packed reference (src/index.rs:14-19), is packed by host
//      threads while the device sketches and sorts.
//   HPC (flag & 1, src/sketch.rs:51-64): the reference never advances i past a
//      homopolymer run, so k-mers are the plain ones and only the
//      spans change: span(i) = sum of skip_len over the last k ACGT bases since
//      the last ambiguous base (TinyQueue), skip_len(j) = the run of base j's
//      code starting at j, to the contig end.  k_hpc_skip / k_hpc_span compute
//      them per base (u16, capped at 256: a span >= 256 gives no info) before
//      the sketch, which reads them (SketchArgs::hpc_span).
#include <hip/hip_runtime.h>

#include <cstring>

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

// The contigs in the device nt4 format of the query reads (include/mm2g.h "nt4
// read batch"), so the build's sketch runs the query kernel's tuned SeqNt4 path
// with views: contig r's 2-bit codes at u64 word pk_off[r] (base i at bits
// 2(i%8) of u16 word i/8), its ambiguity bitmap at amb_off[r] (bit i%8 of byte
// i/8).  One thread per 8 bases; gs[r] = the first 8-base group of contig r.
__global__ __launch_bounds__(256) void k_pack_nt4(const uint8_t* seq, const uint64_t* coff, const uint64_t* gs, uint32_t n,
                                                  uint64_t n_groups, const uint64_t* pk_off, const uint64_t* amb_off,
                                                  uint64_t* words) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups; g += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = n;          // gs[lo] <= g < gs[hi]
        while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (gs[mid] <= g) lo = mid; else hi = mid; }
        const uint64_t j = g - gs[lo], p0 = coff[lo] + 8 * j, e = coff[lo + 1];
        uint32_t code = 0, amb = 0;
        for (int u = 0; u < 8; ++u) {
            const uint64_t p = p0 + (uint64_t)u;
            const uint32_t c = p < e ? nt4_dev(seq[p]) : 4u;
            if (c < 4) code |= c << (2 * u); else if (p < e) amb |= 1u << u;
        }
        ((uint16_t*)(words + pk_off[lo]))[j] = (uint16_t)code;
        ((uint8_t*)(words + amb_off[lo]))[j] = (uint8_t)amb;
    }
}

// ---- device-wide scans and the LSD radix sort of the build's (hash, position) pairs
// (post_process's sort, src/index.rs:74-109), hand-written for gfx950: 8-bit digits,
// tiles of RS_TILE pairs per 256-thread block, stable ranks from wave ballots.
constexpr int SC_T = 1024, SC_PER = 16;            // scan: 16,384 elements per block
constexpr uint64_t SC_CHUNK = (uint64_t)SC_T * SC_PER;
constexpr int RS_ROWS = 16;                        // radix: rows of 256 pairs per tile
constexpr uint64_t RS_TILE = 256ull * RS_ROWS;

template <typename T>
__device__ __forceinline__ T block_excl_scan1024(T v, T& total, T* sh) {   // 1024 threads, sh: 16 T
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { const T o = __shfl_up(x, d, 64); if (lane >= d) x += o; }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    T wbase = 0, tot = 0;
    for (int t = 0; t < 16; ++t) { const T c = sh[t]; if (t < wv) wbase += c; tot += c; }
    __syncthreads();
    total = tot;
    return wbase + x - v;
}

// per-chunk sums
template <typename T>
__global__ __launch_bounds__(SC_T) void k_scan_reduce(const T* in, uint64_t n, T* part) {
    __shared__ T sh[16];
    const uint64_t c0 = (uint64_t)blockIdx.x * SC_CHUNK;
    T s = 0;
#pragma unroll
    for (int j = 0; j < SC_PER; ++j) { const uint64_t i = c0 + (uint64_t)j * SC_T + threadIdx.x; if (i < n) s += in[i]; }
    T tot;
    (void)block_excl_scan1024<T>(s, tot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}
// exclusive scan of the chunk sums in place (one block)
template <typename T>
__global__ __launch_bounds__(SC_T) void k_scan_parts(T* part, uint32_t np) {
    __shared__ T sh[16];
    T carry = 0;
    for (uint32_t b0 = 0; b0 < np; b0 += SC_T) {
        const uint32_t i = b0 + threadIdx.x;
        const T v = i < np ? part[i] : 0;
        T tot;
        const T ex = block_excl_scan1024<T>(v, tot, sh);
        if (i < np) part[i] = carry + ex;
        carry += tot;
    }
}
// exclusive scan of each chunk from its base; out may alias in
template <typename T>
__global__ __launch_bounds__(SC_T) void k_scan_down(const T* in, T* out, uint64_t n, const T* part) {
    __shared__ T sh[16];
    const uint64_t c0 = (uint64_t)blockIdx.x * SC_CHUNK;
    T carry = part[blockIdx.x];
    for (int j = 0; j < SC_PER; ++j) {
        const uint64_t i = c0 + (uint64_t)j * SC_T + threadIdx.x;
        const T v = i < n ? in[i] : 0;
        T tot;
        const T ex = block_excl_scan1024<T>(v, tot, sh);
        if (i < n) out[i] = carry + ex;
        carry += tot;
    }
}

// digit counts of one tile: cnt[d * nb + tile]
__global__ __launch_bounds__(256) void k_rs_count(const uint64_t* key, uint64_t n, int shift, uint32_t* cnt, uint32_t nb) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll
    for (int j = 0; j < RS_ROWS; ++j) {
        const uint64_t i = t0 + (uint64_t)j * 256 + threadIdx.x;
        if (i < n) atomicAdd(&h[(uint32_t)(key[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    cnt[(uint64_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// stable scatter of one tile: rows of 256 pairs in index order; inside a row a
// pair's rank among the equal digits of lower lanes comes from digit ballots,
// across the row's four waves from their per-digit counts
__global__ __launch_bounds__(256) void k_rs_scatter(const uint64_t* kin, const uint64_t* vin, uint64_t* kout, uint64_t* vout,
                                                    uint64_t n, int shift, const uint32_t* off, uint32_t nb) {
    __shared__ uint32_t base[256];
    __shared__ uint32_t wc[4][256];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    base[tid] = off[(uint64_t)tid * nb + blockIdx.x];
    for (int w = 0; w < 4; ++w) wc[w][tid] = 0;
    const uint64_t t0 = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t lt = (1ULL << lane) - 1ULL;
    __syncthreads();
    for (int j = 0; j < RS_ROWS; ++j) {
        const uint64_t i = t0 + (uint64_t)j * 256 + tid;
        const bool valid = i < n;
        const uint64_t k = valid ? kin[i] : 0ULL, v = valid ? vin[i] : 0ULL;
        const uint32_t d = (uint32_t)(k >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const bool on = (d >> bit) & 1u;
            const uint64_t bb = __ballot(on);
            peers &= on ? bb : ~bb;
        }
        const uint32_t r = (uint32_t)__popcll(peers & lt);
        if (valid && r == 0) wc[wv][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        uint32_t pos = 0;
        if (valid) {
            pos = base[d] + r;
            for (int w = 0; w < wv; ++w) pos += wc[w][d];
        }
        __syncthreads();
        base[tid] += wc[0][tid] + wc[1][tid] + wc[2][tid] + wc[3][tid];
        wc[0][tid] = 0; wc[1][tid] = 0; wc[2][tid] = 0; wc[3][tid] = 0;
        __syncthreads();
        if (valid) { kout[pos] = k; vout[pos] = v; }
    }
}

// 1 iff the values are not in ascending order (the pairs come in contig order, so odd k
// never needs the value sort: its minimizer positions strictly increase)
__global__ __launch_bounds__(256) void k_unsorted(const uint64_t* v, uint64_t n, int32_t* flag) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (v[i - 1] > v[i]) { *flag = 1; return; }
}
// bucket-major sort key: (hash & (2^b-1)) << sh | hash >> b, sh = max(2k - b, 0)
__global__ __launch_bounds__(256) void k_rot_keys(uint64_t* h, uint64_t n, int b, int sh) {
    const uint64_t bm = (1ULL << b) - 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        h[i] = ((h[i] & bm) << sh) | (h[i] >> b);
}
// per pair: run start (1) in the low word, member of a run of >= 2 (1) in the high word
__global__ __launch_bounds__(256) void k_run_flags(const uint64_t* rk, uint64_t n, uint64_t* fl) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t x = rk[i];
        const bool st = i == 0 || rk[i - 1] != x, en = i + 1 == n || rk[i + 1] != x;
        fl[i] = (st ? 1ULL : 0ULL) | ((st && en) ? 0ULL : (1ULL << 32));
    }
}
// scanned flags -> positions of multi runs (P, bucket order) and run starts / their P index
__global__ __launch_bounds__(256) void k_run_emit(const uint64_t* rk, const uint64_t* val, const uint64_t* sc, uint64_t n,
                                                  uint64_t* P, uint64_t* rs, uint64_t* rq) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t x = rk[i], e = sc[i];
        const uint64_t r = e & 0xffffffffULL, q = e >> 32;
        const bool st = i == 0 || rk[i - 1] != x, en = i + 1 == n || rk[i + 1] != x;
        if (!(st && en)) P[q] = val[i];
        if (st) { rs[r] = i; rq[r] = q; }
    }
}
// first run of every bucket (rf[nbk] = R); buckets are the rotated key's top bits
__global__ __launch_bounds__(256) void k_bucket_first(const uint64_t* rk, const uint64_t* rs, uint64_t R, int sh, uint64_t nbk, uint64_t* rf) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= R; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t bk = r < R ? rk[rs[r]] >> sh : nbk;
        const uint64_t pb = r ? rk[rs[r - 1]] >> sh : 0;
        for (uint64_t t = r ? pb + 1 : 0; t <= bk; ++t) rf[t] = r;
    }
}
__global__ __launch_bounds__(256) void k_gather_u64(const uint64_t* src, const uint64_t* ix, uint64_t n, uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[ix[i]];
}
// finish_bucket's h entries (src/index.rs:77-108), bucket by bucket: (key>>b)<<1 | 1 -> position
// for a run of one, (key>>b)<<1 -> (offset in the bucket's p) << 32 | n otherwise
__global__ __launch_bounds__(256) void k_run_entries(const uint64_t* rk, const uint64_t* val, const uint64_t* rs, const uint64_t* rq,
                                                     uint64_t R, uint64_t n, int sh, const uint64_t* rf, uint64_t* H) {
    const uint64_t tm = (1ULL << sh) - 1;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = rs[r], len = (r + 1 < R ? rs[r + 1] : n) - i;
        const uint64_t x = rk[i], bk = x >> sh, top = x & tm;
        const uint64_t pbase = rq[rf[bk]];
        H[2 * r] = (top << 1) | (len == 1 ? 1ULL : 0ULL);
        H[2 * r + 1] = len == 1 ? val[i] : ((rq[r] - pbase) << 32) | len;
    }
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


// exclusive scan of n values (in place allowed); part: scratch of ceil(n / SC_CHUNK) T
template <typename T>
hipError_t dev_excl_scan(const T* in, T* out, uint64_t n, T* part, hipStream_t st) {
    const uint32_t np = (uint32_t)((n + SC_CHUNK - 1) / SC_CHUNK);
    if (np == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_reduce<T>, dim3(np), dim3(SC_T), 0, st, in, n, part);
    hipLaunchKernelGGL(k_scan_parts<T>, dim3(1), dim3(SC_T), 0, st, part, np);
    hipLaunchKernelGGL(k_scan_down<T>, dim3(np), dim3(SC_T), 0, st, in, out, n, (const T*)part);
    return hipGetLastError();
}

// stable LSD radix sort of (k, v) pairs by the low `bits` bits of k, ping-ponging between
// (k0, v0) and (k1, v1); returns in `flip` whether the result is in (k1, v1)
hipError_t dev_radix_sort(uint64_t* k0, uint64_t* v0, uint64_t* k1, uint64_t* v1, uint64_t n, int bits, uint32_t* cnt,
                          uint32_t* part, hipStream_t st, bool& flip) {
    flip = false;
    const uint32_t nb = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    for (int sh = 0; sh < bits; sh += 8) {
        hipLaunchKernelGGL(k_rs_count, dim3(nb), dim3(256), 0, st, (const uint64_t*)k0, n, sh, cnt, nb);
        if (hipError_t e = dev_excl_scan<uint32_t>(cnt, cnt, 256ull * nb, part, st)) return e;
        hipLaunchKernelGGL(k_rs_scatter, dim3(nb), dim3(256), 0, st, (const uint64_t*)k0, (const uint64_t*)v0, k1, v1, n, sh,
                           (const uint32_t*)cnt, nb);
        if (hipError_t e = hipGetLastError()) return e;
        std::swap(k0, k1); std::swap(v0, v1);
        flip = !flip;
    }
    return hipSuccess;
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
    if (prof) { IXCHK(hipStreamSynchronize(st)); lap("H2D reference"); }
    int64_t chunk = IX_CHUNK;
    if (const int64_t v = g_index_knob[1].load()) chunk = std::max<int64_t>(256, v);   // MM2G_IKNOB_IXCHUNK (tests)
    // non-HPC builds sketch the contigs in the query reads' nt4 format (k_pack_nt4): views then
    // start at a multiple of 8 bases (the warm-up only grows) and view_off is contig-relative
    const bool nt4 = !(flag & 1);
    std::vector<uint64_t> v_off, v_base, v_end;
    std::vector<uint32_t> v_len, v_pre, v_from, v_rid;
    std::vector<uint8_t> v_last;
    uint64_t cap = 0;
    for (size_t r = 0; r < n; ++r) {
        const int64_t L = (int64_t)lens[r];
        for (int64_t c0 = 0; c0 < L; c0 += chunk) {
            int64_t vs = c0 ? view_warmup(seqs[r], c0, w, k) : 0;
            const int64_t ve = std::min<int64_t>(L, c0 + chunk);
            if (nt4) vs &= ~(int64_t)7;
            v_off.push_back(nt4 ? (uint64_t)vs : idx.seq[r].offset + (uint64_t)vs);
            v_len.push_back((uint32_t)(ve - vs)); v_pre.push_back((uint32_t)vs); v_from.push_back((uint32_t)(c0 - vs));
            v_last.push_back(ve == L ? 1 : 0); v_rid.push_back((uint32_t)r);
            // minimizer slots: ~2/(w+1) per base is the usual density; a quarter per base (+256) holds
            // it, and a view that needs more (homopolymer runs emit at every base) is re-run exactly
            v_base.push_back(cap); cap += (uint64_t)((ve - vs) >> 2) + 256; v_end.push_back(cap);
        }
    }
    const uint32_t nv = (uint32_t)v_off.size();
    if (nv == 0) { idx.S.assign(kroundup64((size_t)((total + 7) / 8)), 0u); idx.B.assign((size_t)1 << b, HostBucket()); return true; }
    uint64_t* d_voff = D.alloc<uint64_t>(nv); uint32_t* d_vlen = D.alloc<uint32_t>(nv); uint32_t* d_vpre = D.alloc<uint32_t>(nv);
    uint32_t* d_vfrom = D.alloc<uint32_t>(nv); uint8_t* d_vlast = D.alloc<uint8_t>(nv); uint32_t* d_vrid = D.alloc<uint32_t>(nv);
    uint64_t* d_vbase = D.alloc<uint64_t>(nv); uint64_t* d_vend = D.alloc<uint64_t>(nv);
    uint64_t* d_mx = D.alloc<uint64_t>(cap); uint32_t* d_my = D.alloc<uint32_t>(cap); uint32_t* d_cnt = D.alloc<uint32_t>(nv);
    uint32_t* d_need = D.alloc<uint32_t>(nv);
    int32_t* d_ovf = D.alloc<int32_t>(4);
    if (!d_voff || !d_vlen || !d_vpre || !d_vfrom || !d_vlast || !d_vrid || !d_vbase || !d_vend || !d_mx || !d_my || !d_cnt || !d_need || !d_ovf) {
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
    // ---- 2. S (src/index.rs:14-19) on host threads, overlapping the device work below: 8 bases
    // per u32 word, base j of the concatenation in bits 4(j%8); words past the sequence stay 0
    struct Joiner { std::thread t; ~Joiner() { if (t.joinable()) t.join(); } } s_pack;
    {
        const uint64_t nw = (total + 7) / 8;
        SVec* Sv = &idx.S;
        s_pack.t = std::thread([&seqs, &lens, Sv, nw, n]() {
            const size_t nall = kroundup64((size_t)nw);
            Sv->resize(nall);                           // uninitialised (SVec): the threads write every word
            uint32_t* S = Sv->data();
            std::fill(S + nw, S + nall, 0u);            // kroundup64 padding
            static const uint8_t T4[256] = {
                4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,
                4,0,4,1,4,4,4,2,4,4,4,4,4,4,4,4, 4,4,4,4,3,4,4,4,4,4,4,4,4,4,4,4, 4,0,4,1,4,4,4,2,4,4,4,4,4,4,4,4, 4,4,4,4,3,4,4,4,4,4,4,4,4,4,4,4,
                4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,
                4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4};
            std::vector<uint64_t> coff(n + 1, 0);
            for (size_t i = 0; i < n; ++i) coff[i + 1] = coff[i] + lens[i];
            const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>(16, nw / (1u << 20)));
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() {
                const uint64_t w0 = nw * t / nt, w1 = nw * (t + 1) / nt;
                size_t r = (size_t)(std::upper_bound(coff.begin(), coff.end(), w0 * 8) - coff.begin()) - 1;
                for (uint64_t wd = w0; wd < w1; ++wd) {
                    uint32_t v = 0;
                    for (int j = 0; j < 8; ++j) {
                        const uint64_t p = wd * 8 + (uint64_t)j;
                        while (r < n && p >= coff[r + 1]) ++r;
                        if (r >= n) break;
                        v |= (uint32_t)(T4[seqs[r][p - coff[r]]] & 0xFu) << (4 * j);
                    }
                    S[wd] = v;
                }
            });
            for (auto& x : th) x.join();
        });
    }
    if (prof) { IXCHK(hipStreamSynchronize(st)); lap("views (S packs on the host)"); }
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
    if (nt4) {   // contig r = "read" r of an nt4 batch; view r reads contig v_rid[r]
        std::vector<uint64_t> coff(n + 1, 0), gs(n + 1, 0), pko(n), ambo(n);
        uint64_t nwords = 0;
        for (size_t i = 0; i < n; ++i) {
            coff[i + 1] = coff[i] + lens[i];
            const uint64_t ng = (lens[i] + 7) / 8;
            gs[i + 1] = gs[i] + ng;
            pko[i] = nwords; nwords += (ng + 3) / 4;       // 4 u16 code words per u64
            ambo[i] = nwords; nwords += (ng + 7) / 8;      // 8 bitmap bytes per u64
        }
        uint64_t* d_coff = D.alloc<uint64_t>(n + 1); uint64_t* d_gs = D.alloc<uint64_t>(n + 1);
        uint64_t* d_pko = D.alloc<uint64_t>(n); uint64_t* d_ambo = D.alloc<uint64_t>(n);
        uint64_t* d_words = D.alloc<uint64_t>(nwords + 1);
        if (!d_coff || !d_gs || !d_pko || !d_ambo || !d_words) { err = "hipMalloc(nt4 reference) failed"; return false; }
        IXCHK(hipMemcpyAsync(d_coff, coff.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
        IXCHK(hipMemcpyAsync(d_gs, gs.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
        IXCHK(hipMemcpyAsync(d_pko, pko.data(), n * 8, hipMemcpyHostToDevice, st));
        IXCHK(hipMemcpyAsync(d_ambo, ambo.data(), n * 8, hipMemcpyHostToDevice, st));
        const unsigned nb = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((gs[n] + 255) / 256, 65536));
        hipLaunchKernelGGL(k_pack_nt4, dim3(nb), dim3(256), 0, st, d_seq, d_coff, d_gs, (uint32_t)n, gs[n], d_pko, d_ambo, d_words);
        IXCHK(hipGetLastError());
        sa.pk_words = d_words; sa.pk_off = d_pko; sa.amb_off = d_ambo; sa.view_read = d_vrid;
    }
    sa.mz_need = d_need;
    std::vector<uint32_t> cnt(nv);
    for (int pass = 0;; ++pass) {
        if (launch_sketch(sa, (int)std::min<uint32_t>((nv + 3) / 4, 4096u), st) != 0) { err = "k_sketch launch failed"; return false; }
        int32_t ovf = 0;
        IXCHK(hipMemcpyAsync(cnt.data(), d_cnt, nv * 4, hipMemcpyDeviceToHost, st));
        IXCHK(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, st));
        IXCHK(hipStreamSynchronize(st));
        if (!ovf) break;
        if (pass) { unsupported = true; err = "GPU index build: minimizer slot overflow (host build)"; return false; }
        // a view outgrew its slot: every view again with exactly its own count (mz_need)
        IXCHK(hipMemcpy(cnt.data(), d_need, nv * 4, hipMemcpyDeviceToHost));
        cap = 0;
        for (uint32_t v = 0; v < nv; ++v) { v_base[v] = cap; cap += (uint64_t)cnt[v] + 16; v_end[v] = cap; }
        d_mx = D.alloc<uint64_t>(cap); d_my = D.alloc<uint32_t>(cap);
        if (!d_mx || !d_my) { err = "hipMalloc(index minimizers) failed"; return false; }
        IXCHK(hipMemcpyAsync(d_vbase, v_base.data(), nv * 8, hipMemcpyHostToDevice, st));
        IXCHK(hipMemcpyAsync(d_vend, v_end.data(), nv * 8, hipMemcpyHostToDevice, st));
        IXCHK(hipMemsetAsync(d_ovf, 0, 16, st));
        sa.mz_x = d_mx; sa.mz_y = d_my;
    }
    lap("sketch");
    std::vector<uint64_t> ooff(nv);
    uint64_t M = 0;
    for (uint32_t v = 0; v < nv; ++v) { ooff[v] = M; M += cnt[v]; }
    if (M >= (1ULL << 32)) { unsupported = true; err = "GPU index build: 2^32 or more minimizers (host build)"; return false; }
    if (M == 0) { idx.B.assign((size_t)1 << b, HostBucket()); return true; }
    // ---- 4. pairs (contig order), then sorted by (bucket, hash, value) on the device
    uint64_t* d_ooff = D.alloc<uint64_t>(nv);
    uint64_t* h0 = D.alloc<uint64_t>(M); uint64_t* v0 = D.alloc<uint64_t>(M);
    uint64_t* h1 = D.alloc<uint64_t>(M); uint64_t* v1 = D.alloc<uint64_t>(M);
    const uint32_t rnb = (uint32_t)((M + RS_TILE - 1) / RS_TILE);
    uint32_t* d_cnt8 = D.alloc<uint32_t>(256ull * rnb);
    uint32_t* d_part32 = D.alloc<uint32_t>(256ull * rnb / SC_CHUNK + 2);
    uint64_t* d_part64 = D.alloc<uint64_t>(M / SC_CHUNK + 2);
    int32_t* d_flag = D.alloc<int32_t>(1);
    if (!d_ooff || !h0 || !v0 || !h1 || !v1 || !d_cnt8 || !d_part32 || !d_part64 || !d_flag) { err = "hipMalloc(index pairs) failed"; return false; }
    IXCHK(hipMemcpyAsync(d_ooff, ooff.data(), nv * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_ix_compact, dim3((nv + 3) / 4), dim3(256), 0, st, nv, d_vbase, d_cnt, d_mx, d_my, d_vrid, d_vpre, d_ooff, h0, v0);
    IXCHK(hipGetLastError());
    if (prof) { IXCHK(hipStreamSynchronize(st)); lap("pairs"); }
    const int vbits = 32 + std::max(1, bit_width64(n ? n - 1 : 0)), hbits = 2 * k;
    const unsigned gs = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((M + 255) / 256, 65536));
    // post_process orders each hash's positions; the pairs arrive in contig order, so only a
    // value out of order (possible for even k) needs the stable sort by value first
    int32_t unsorted = 0;
    IXCHK(hipMemsetAsync(d_flag, 0, 4, st));
    hipLaunchKernelGGL(k_unsorted, dim3(gs), dim3(256), 0, st, (const uint64_t*)v0, M, d_flag);
    IXCHK(hipMemcpyAsync(&unsorted, d_flag, 4, hipMemcpyDeviceToHost, st));
    IXCHK(hipStreamSynchronize(st));
    if (g_index_knob[6].load()) unsorted = 1;   // MM2G_IKNOB_IXSORTV (tests)
    bool flip = false;
    if (unsorted) {
        IXCHK(dev_radix_sort(v0, h0, v1, h1, M, vbits, d_cnt8, d_part32, st, flip));
        if (flip) { std::swap(h0, h1); std::swap(v0, v1); }
    }
    // bucket-major key: the .mmi and the host index keep every bucket's keys in hash order
    const int rsh = hbits > b ? hbits - b : 0;
    const uint64_t nbk = (uint64_t)1 << b;
    hipLaunchKernelGGL(k_rot_keys, dim3(gs), dim3(256), 0, st, h0, M, b, rsh);
    IXCHK(dev_radix_sort(h0, v0, h1, v1, M, hbits, d_cnt8, d_part32, st, flip));
    if (flip) { std::swap(h0, h1); std::swap(v0, v1); }
    if (prof) { IXCHK(hipStreamSynchronize(st)); lap(unsorted ? "radix sorts (value, hash)" : "radix sort (hash)"); }
    // ---- 5. runs -> finish_bucket's h and p (src/index.rs:77-108), bucket by bucket, on the device
    uint64_t* fl = h1;                // free after the sort
    uint64_t* sc = v1;
    hipLaunchKernelGGL(k_run_flags, dim3(gs), dim3(256), 0, st, (const uint64_t*)h0, M, fl);
    IXCHK(hipGetLastError());
    IXCHK(dev_excl_scan<uint64_t>(fl, sc, M, d_part64, st));
    uint64_t lastf = 0, lasts = 0;
    IXCHK(hipMemcpyAsync(&lastf, fl + (M - 1), 8, hipMemcpyDeviceToHost, st));
    IXCHK(hipMemcpyAsync(&lasts, sc + (M - 1), 8, hipMemcpyDeviceToHost, st));
    IXCHK(hipStreamSynchronize(st));
    const uint64_t R = (lasts & 0xffffffffULL) + (lastf & 0xffffffffULL), PT = (lasts >> 32) + (lastf >> 32);
    uint64_t* dP = D.alloc<uint64_t>(PT); uint64_t* rs = D.alloc<uint64_t>(R); uint64_t* rq = D.alloc<uint64_t>(R + 1);
    uint64_t* rf = D.alloc<uint64_t>(nbk + 1); uint64_t* pb = D.alloc<uint64_t>(nbk + 1); uint64_t* dH = D.alloc<uint64_t>(2 * R);
    if (!dP || !rs || !rq || !rf || !pb || !dH) { err = "hipMalloc(index buckets) failed"; return false; }
    IXCHK(hipMemcpyAsync(rq + R, &PT, 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_run_emit, dim3(gs), dim3(256), 0, st, (const uint64_t*)h0, (const uint64_t*)v0, (const uint64_t*)sc, M, dP, rs, rq);
    const unsigned gr = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((R + 256) / 256, 65536));
    hipLaunchKernelGGL(k_bucket_first, dim3(gr), dim3(256), 0, st, (const uint64_t*)h0, (const uint64_t*)rs, R, rsh, nbk, rf);
    hipLaunchKernelGGL(k_gather_u64, dim3((unsigned)((nbk + 256) / 256)), dim3(256), 0, st, (const uint64_t*)rq, (const uint64_t*)rf, nbk + 1, pb);
    hipLaunchKernelGGL(k_run_entries, dim3(gr), dim3(256), 0, st, (const uint64_t*)h0, (const uint64_t*)v0, (const uint64_t*)rs,
                       (const uint64_t*)rq, R, M, rsh, (const uint64_t*)rf, dH);
    IXCHK(hipGetLastError());
    std::vector<uint64_t> hrf(nbk + 1), hpb(nbk + 1);
    IXCHK(hipMemcpyAsync(hrf.data(), rf, (nbk + 1) * 8, hipMemcpyDeviceToHost, st));
    IXCHK(hipMemcpyAsync(hpb.data(), pb, (nbk + 1) * 8, hipMemcpyDeviceToHost, st));
    IXCHK(hipStreamSynchronize(st));
    lap("runs -> buckets (device)");
    // ---- 6. the buckets' h and p to the host: every thread sizes its share of the buckets,
    // then copies its slice of H and of P through its own pinned buffer and stream
    int nt = (int)std::min<uint64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
    if (M < (1u << 16)) nt = 1;
    idx.B.assign(nbk, HostBucket());
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() {
            for (uint64_t bk = nbk * t / nt; bk < nbk * (t + 1) / nt; ++bk) {
                HostBucket& B = idx.B[bk];
                B.h.resize(hrf[bk + 1] - hrf[bk]);
                B.p.resize(hpb[bk + 1] - hpb[bk]);
                B.has_h = !B.h.empty();
            }
        });
        for (auto& x : th) x.join();
    }
    lap("host buckets sized");
    constexpr uint64_t PIN_WORDS = 1u << 22;            // 32 MB per thread
    std::vector<std::string> errs(nt);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() {
            auto fail = [&](const char* what, hipError_t e) { errs[t] = std::string(what) + ": " + hipGetErrorString(e); };
            if (hipError_t e = hipSetDevice(device)) { fail("hipSetDevice", e); return; }
            hipStream_t ts;
            if (hipError_t e = hipStreamCreateWithFlags(&ts, hipStreamNonBlocking)) { fail("hipStreamCreate", e); return; }
            uint64_t* pin = nullptr;
            if (hipError_t e = hipHostMalloc((void**)&pin, PIN_WORDS * 8, hipHostMallocDefault)) { fail("hipHostMalloc", e); (void)hipStreamDestroy(ts); return; }
            // words [a, z) of a device array through the pinned buffer; place(first word, host words, count)
            auto pull = [&](const uint64_t* src, uint64_t a, uint64_t z, auto place) -> bool {
                for (uint64_t c = a; c < z; c += PIN_WORDS) {
                    const uint64_t m = std::min<uint64_t>(PIN_WORDS, z - c);
                    hipError_t e = hipMemcpyAsync(pin, src + c, m * 8, hipMemcpyDeviceToHost, ts);
                    if (!e) e = hipStreamSynchronize(ts);
                    if (e) { fail("D2H buckets", e); return false; }
                    place(c, pin, m);
                }
                return true;
            };
            // H: entries (2 words) [e0, e1) of this thread, into the buckets they belong to
            const uint64_t e0 = R * t / nt, e1 = R * (t + 1) / nt;
            bool ok = pull(dH, 2 * e0, 2 * e1, [&](uint64_t c, const uint64_t* hw, uint64_t m) {
                uint64_t e = c / 2;
                const uint64_t ee = (c + m) / 2;
                size_t bk = (size_t)(std::upper_bound(hrf.begin(), hrf.end(), e) - hrf.begin()) - 1;
                while (e < ee) {
                    while (hrf[bk + 1] <= e) ++bk;
                    const uint64_t q = std::min(ee, hrf[bk + 1]) - e;
                    memcpy((void*)(idx.B[bk].h.data() + (e - hrf[bk])), hw + 2 * (e - c / 2), q * 16);
                    e += q;
                }
            });
            const uint64_t p0 = PT * t / nt, p1 = PT * (t + 1) / nt;
            if (ok) ok = pull(dP, p0, p1, [&](uint64_t c, const uint64_t* pw, uint64_t m) {
                uint64_t e = c;
                size_t bk = (size_t)(std::upper_bound(hpb.begin(), hpb.end(), e) - hpb.begin()) - 1;
                while (e < c + m) {
                    while (hpb[bk + 1] <= e) ++bk;
                    const uint64_t q = std::min(c + m, hpb[bk + 1]) - e;
                    memcpy(idx.B[bk].p.data() + (e - hpb[bk]), pw + (e - c), q * 8);
                    e += q;
                }
            });
            (void)hipHostFree(pin);
            (void)hipStreamDestroy(ts);
        });
        for (auto& x : th) x.join();
    }
    for (const std::string& e : errs) if (!e.empty()) { err = e; return false; }
    lap("D2H buckets (pinned, threads)");
    if (s_pack.t.joinable()) s_pack.t.join();
    lap("S (host threads) joined");
    return true;
}

}  // namespace mm2g
