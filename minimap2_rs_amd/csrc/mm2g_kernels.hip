// gfx950 (MI355X, CDNA4) kernels of the sketch -> seed -> chain path.
//
// Every kernel restates one function of the reference crate (file:line in
// /root/reference) bit-exactly; DESIGN.md explains the parallel formulation
// and the roofline of each.  Wave64 throughout: one wavefront owns one read
// (or one contig for index builds) and loops over it; reads are handed out
// by grid-stride or by an atomic work counter.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include <algorithm>
#include <type_traits>
#include "mm2g_internal.h"

using namespace mm2g;

#define DEVI __device__ __forceinline__

// Bounds-checked build (-DMM2G_CHECKED): an out-of-range index is recorded
// (first violation wins) and replaced by 0 instead of faulting the GPU.
#ifdef MM2G_CHECKED
__device__ unsigned long long g_chk[4];
DEVI uint64_t ck_idx(uint64_t i, uint64_t cap, int line) {
    if (i < cap) return i;
    if (atomicCAS(&g_chk[0], 0ULL, (unsigned long long)line) == 0ULL) { g_chk[1] = i; g_chk[2] = cap; }
    return 0;
}
#define CK(i, cap) ck_idx((uint64_t)(i), (uint64_t)(cap), __LINE__)
#define TRACE(tr, slot, v) do { if (tr) __hip_atomic_store(&(tr)[slot], (uint32_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#else
#define TRACE(tr, slot, v) do {} while (0)
#define CK(i, cap) (i)
#endif

// ------------------------------------------------------------------ helpers
DEVI int lane_id() { return (int)(threadIdx.x & 63); }
DEVI uint64_t ballot(bool p) { return __ballot(p); }
DEVI int ctz64(uint64_t x) { return __builtin_ctzll(x); }
DEVI int clz64(uint64_t x) { return __builtin_clzll(x); }
DEVI uint64_t lanemask_lt_of(int l) { return l ? (~0ULL >> (64 - l)) : 0ULL; }
DEVI uint64_t lanemask_lt() { return lanemask_lt_of(lane_id()); }

// LDS visibility inside one wavefront: LDS ops of a wave execute in order;
// the fences stop the compiler from moving LDS accesses across this point.
DEVI void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
DEVI void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

DEVI int32_t rdl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
DEVI uint32_t rdlu(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
DEVI uint64_t rdl64(uint64_t v, int l) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
DEVI int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Shift the wave right by one lane, lane 0 <- `in0` (ds_bpermute based).
DEVI int32_t shr1(int32_t v, int32_t in0) {
    const int32_t t = __shfl_up(v, 1, 64);
    return lane_id() == 0 ? in0 : t;
}

template <typename T, typename F>
DEVI T wave_incl_scan(T v, F op) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (l >= d) v = op(o, v);
    }
    return v;
}
DEVI uint32_t wave_excl_sum(uint32_t v, uint32_t& total) {
    uint32_t inc = wave_incl_scan(v, [](uint32_t a, uint32_t b) { return a + b; });
    total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);   // SGPR: wave-uniform
    return inc - v;
}
DEVI uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, d, 64), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}
DEVI uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// src/nt4.rs:2-10 — `b | 0x20` folds exactly {A,a}->a, {C,c}->c, {G,g}->g, {T,t}->t
DEVI uint32_t nt4d(uint32_t b) {
    uint32_t c = b | 0x20u;
    return c == 'a' ? 0u : c == 'c' ? 1u : c == 'g' ? 2u : c == 't' ? 3u : 4u;
}

// src/sketch.rs:4-13 (wrapping; every step masked to 2k bits).  For k <= 16 the
// 32-bit ring gives the same low 2k bits.
template <typename T>
DEVI T hash64d(T key, T mask) {
    key = ((T)~key + (key << 21)) & mask;
    key ^= key >> 24;
    key = (key + (key << 3) + (key << 8)) & mask;
    key ^= key >> 14;
    key = (key + (key << 2) + (key << 4)) & mask;
    key ^= key >> 28;
    key = (key + (key << 31)) & mask;
    return key;
}

// ------------------------------------------------------------------ control-flow rule
// HIP gives no maximal-reconvergence guarantee: the compiler may restructure a
// lane-divergent LOOP at the end of an outer loop body into a divergent loop
// exit, letting some lanes start the next iteration early (observed on
// gfx950/ROCm 7.2 in a first version of k_chain_dp).  Every kernel that talks
// across lanes (ballot/shuffle/readlane/LDS hand-off) therefore follows one rule:
// every loop has a wave-uniform trip count (fixed, or `while (any(...))`),
// per-read scalars are made provably uniform with readfirstlane, and
// lane-divergence appears only in straight-line code.
DEVI bool any(bool p) { return ballot(p) != 0ULL; }
// wave index inside the workgroup, provably uniform for divergence analysis
DEVI int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
DEVI uint64_t uni64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// ============================================================================
// 1. SKETCH — sketch_sequence (src/sketch.rs:29-100), non-HPC.
//
// One wave per sequence, tiles of TS = 64*CH positions; lane l owns positions
// [t0 + l*CH, +CH).  Parallel restatement (DESIGN.md "Sketch"):
//   * info[i] is valid iff base i is ACGT, the k-mer is not symmetric and
//     l[i] >= k, where l is the segmented count of non-symmetric valid bases
//     since the last ambiguous base (capped at w+k: every comparison the
//     reference makes is against k, w+k-1 or w+k).  l is a wave scan.
//   * after every step the reference's `min` is the NEWEST slot holding the
//     minimum x of the last w slots, so the emissions of step i depend only
//     on info[i-w..i] and l[i]; each lane rebuilds `min` from the w slots
//     before its chunk and replays the reference step logic (A: first-window
//     ties, B: new minimum, C: expiry + rescan + ties) in position order.
//   * emissions are counted, wave-scanned and written in reference order.
// ============================================================================
constexpr int SK_CH = 8;
constexpr int SK_TS = 64 * SK_CH;

// per-wave LDS: X[NB] (x = hash<<8 | span, MAX = no info), LZ[NB] (l | z<<15);
// y = pos<<1 | z is implicit.  Bases stay in registers (8 per lane).
// Lane l works on slots [w + 8l, w + 8l + 8): a stride of 8 slots (16 LDS banks
// for X) would put all 64 lanes on 4 banks.  One pad slot per 8 spreads them.
#define SKP(i) ((i) + ((i) >> 3))
__host__ __device__ inline size_t sketch_wave_slots(int w) {
    const size_t nb = (size_t)SK_TS + (size_t)w;
    return nb + (nb >> 3) + 1;
}
__host__ __device__ inline size_t sketch_wave_lds(int w) {   // + 16 B: the k-mer registers carried from the previous tile
    const size_t pnb = sketch_wave_slots(w);
    return (((pnb * 8 + pnb * 2) + 15) & ~(size_t)15) + 16;
}

// reverse the order of the 32 2-bit groups of x
DEVI uint64_t rev2_64(uint64_t x) {
    x = ((x >> 2) & 0x3333333333333333ULL) | ((x & 0x3333333333333333ULL) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((x & 0x0F0F0F0F0F0F0F0FULL) << 4);
    return __builtin_bswap64(x);
}
// 8 bases (byte u = position p0+u, 'N' outside [0, L)) -> 2-bit codes, latest
// base lowest (code16 = sum c_u << 2(7-u)), and validity (bit u) of nt4 (src/nt4.rs)
DEVI uint64_t load_bases8(const uint8_t* s, int64_t p0, int64_t L) {
    uint64_t v;
    if (p0 >= 0 && p0 + 8 <= L) __builtin_memcpy(&v, s + p0, 8);
    else {
        v = 0;
        for (int u = 0; u < 8; ++u) {
            const int64_t p = p0 + u;
            v |= (uint64_t)((p >= 0 && p < L) ? s[p] : (uint8_t)'N') << (8 * u);
        }
    }
    return v;
}
DEVI void codes8(uint64_t v, uint32_t& code16, uint32_t& valid8) {
    code16 = 0; valid8 = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const uint32_t c = nt4d((uint32_t)(v >> (8 * u)) & 0xffu);
        code16 |= (c & 3u) << (2 * (7 - u));
        valid8 |= (c < 4 ? 1u : 0u) << u;
    }
}
DEVI uint32_t rev8(uint32_t v) { return __builtin_bitreverse32(v) >> 24; }

// Base sources of k_sketch.  raw(p0) loads the 8 bases at p0 (a multiple of 8;
// positions outside [0, L) read as ambiguous), decode() turns that into
// code16/valid8 as above, code(p) is nt4 (src/nt4.rs:2-10) of one base.
//   SeqAscii: ASCII bytes (index-build views into a contig, SketchArgs view_*).
//   SeqNt4:   the device read format (include/mm2g.h "nt4 read batch"): 2-bit
//             codes, base i at bits 2(i%8) of 16-bit word i/8; reads with an
//             ambiguous base also carry a bitmap (bit i%8 of byte i/8).
struct SeqAscii {
    const uint8_t* s; int64_t L;
    DEVI uint64_t raw(int64_t p0) const { return load_bases8(s, p0, L); }
    DEVI void decode(uint64_t v, uint32_t& code16, uint32_t& valid8) const { codes8(v, code16, valid8); }
    DEVI uint32_t code(int64_t p) const { return nt4d(s[p]); }
    DEVI bool amb8(int64_t) const { return false; }
};
DEVI uint32_t rev2_16(uint32_t x) {
    x = ((x >> 2) & 0x3333u) | ((x & 0x3333u) << 2);
    x = ((x >> 4) & 0x0F0Fu) | ((x & 0x0F0Fu) << 4);
    return ((x >> 8) | (x << 8)) & 0xffffu;
}
struct SeqNt4 {
    const uint16_t* s2; const uint8_t* am; int64_t L;
    DEVI uint64_t raw(int64_t p0) const {
        if (p0 < 0 || p0 >= L) return 0;
        const uint64_t nv = L - p0 < 8 ? (uint64_t)(L - p0) : 8u;
        const uint64_t v = s2[p0 >> 3], m = am ? am[p0 >> 3] : 0u;
        return v | (m << 16) | (nv << 24);
    }
    DEVI void decode(uint64_t v, uint32_t& code16, uint32_t& valid8) const {
        const uint32_t nv = (uint32_t)(v >> 24) & 15u;
        code16 = rev2_16((uint32_t)v & 0xffffu);
        valid8 = ~(uint32_t)(v >> 16) & ((1u << nv) - 1u);
    }
    DEVI uint32_t code(int64_t p) const {
        if (am && ((am[p >> 3] >> (p & 7)) & 1u)) return 4u;
        return ((uint32_t)s2[p >> 3] >> (2 * (p & 7))) & 3u;
    }
    // the 8 bases at p8 (a multiple of 8) are all ambiguous (a walk-back steps over N runs 8 at a time)
    DEVI bool amb8(int64_t p8) const { return am && am[p8 >> 3] == 0xffu; }
    // 8 bases at p0 < 0 (a multiple of 8) of a query view: the read's bases before the view
    DEVI uint64_t raw_back(int64_t p0) const {
        const uint64_t v = s2[p0 >> 3], m = am ? am[p0 >> 3] : 0u;
        return v | (m << 16) | (8ULL << 24);
    }
};

// X32 (k <= 15, not HPC): the LDS window holds the 32-bit hash alone (hash < 4^k < 2^30, so
// ~0u stays free for "no info"); every x = hash << 8 | k then, so x and hash order alike
template <bool K32, typename Src, bool HPC = false, bool X32 = false>
// waves per SIMD (override with -D): the query sketch (nt4) at 96 VGPRs 5; the index build
// (ASCII) at 128 4 (also with the 32-bit window: at 80 VGPRs its byte loads and decode spilled
// 57 VGPRs, the build's sketch wrote ~23 GB of scratch); the query's 32-bit window (X32) at 80 VGPRs 6
#ifndef SK_WPE_NT4
#define SK_WPE_NT4 5
#endif
#ifndef SK_WPE_ASCII
#define SK_WPE_ASCII 4
#endif
#ifndef SK_WPE_X32
#define SK_WPE_X32 6
#endif
__global__ __launch_bounds__(256, (!std::is_same<Src, SeqNt4>::value ? SK_WPE_ASCII : (X32 ? SK_WPE_X32 : SK_WPE_NT4))) void k_sketch(SketchArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    static_assert(!X32 || (K32 && !HPC), "X32: k <= 15 query/index sketch without HPC spans");
    using XT = typename std::conditional<X32, uint32_t, uint64_t>::type;
    constexpr XT XMAX = (XT)~(XT)0;
    const int w = a.w, k = a.k;
    auto xout = [&](XT v) -> uint64_t { return X32 ? (v == XMAX ? U64MAX : ((uint64_t)v << 8) | (uint64_t)k) : (uint64_t)v; };
    const int wv = wave_id(), lane = lane_id();
    XT* X = (XT*)(smem + sketch_wave_lds(w) * wv);
    uint16_t* LZ = (uint16_t*)(X + sketch_wave_slots(w));
    const int CAP = w + k;
    const uint64_t mask = (k >= 32) ? U64MAX : ((1ULL << (2 * k)) - 1);
    const uint32_t shift1 = 2u * (uint32_t)(k - 1);
    const int nwaves = (int)(gridDim.x * (blockDim.x >> 6));
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + wv; r < a.n; r += nwaves) {
        uint64_t roff;
        int64_t L, pre = 0, efrom = 0;
        bool flush = true;
        if (a.view_off) {   // index chunk / query view: a view into a contig or read (see SketchArgs)
            L = (int64_t)(uint32_t)uni((int32_t)a.view_len[r]);
            if (L == 0) { if (lane == 0) { a.mz_cnt[r] = 0; if (a.mz_need) a.mz_need[r] = 0; } continue; }   // also unused query views
            roff = uni64(a.view_off[r]);
            pre = (int64_t)(uint32_t)uni((int32_t)a.view_pre[r]); efrom = (int64_t)(uint32_t)uni((int32_t)a.emit_from[r]);
            flush = uni((int32_t)a.view_last[r]) != 0;
        } else {
            roff = uni64(a.rd_off[r]);
            L = (int64_t)(uni64(a.rd_off[r + 1]) - roff);
        }
        Src src;
        if constexpr (std::is_same<Src, SeqNt4>::value) {
            // query view: the read's words from the view start (a multiple of 8 bases); the
            // k-mer walk-back reads the read's earlier words (negative positions, >= -pre)
            const uint32_t rr = a.view_read ? (uint32_t)uni((int32_t)a.view_read[r]) : r;
            const uint64_t v8 = a.view_read ? roff >> 3 : 0;
            const uint64_t ao = uni64(a.amb_off[rr]);
            src = Src{(const uint16_t*)(a.pk_words + uni64(a.pk_off[rr])) + v8, ao == U64MAX ? nullptr : (const uint8_t*)(a.pk_words + ao) + v8, L};
        } else {
            src = Src{a.seq + roff, L};
        }
        const uint64_t obase = uni64(a.out_base[r]), oend = uni64(a.out_end[r]);
        if (L == 0) { if (lane == 0) { a.mz_cnt[r] = 0; if (a.mz_need) a.mz_need[r] = 0; } continue; }
        uint64_t pt[6] = {0, 0, 0, 0, 0, 0}, tz = a.prof ? wall_clock64() : 0;
#define SK_PT(ph) do { if (a.prof) { const uint64_t t_ = wall_clock64(); pt[ph] += t_ - tz; tz = t_; } } while (0)
        // history slots = positions [-w, -1]: MAX
        for (int t0 = 0; t0 < w; t0 += 64) {
            const int t = t0 + lane;
            if (t < w) { X[SKP(t)] = XMAX; LZ[SKP(t)] = 0; }
        }
        uint64_t count = 0;
        uint32_t n_tiles = 0, n_slow = 0;      // MM2G_SKETCH_PROF: tiles, tiles on the exact (2-pass) step path
        int32_t l_carry = 0;
        // k-mer registers at the end of the previous tile, in LDS (held in registers they cost spills)
        uint64_t* CK = (uint64_t*)(smem + sketch_wave_lds(w) * (wv + 1) - 16);
        // bases of this lane's chunk, prefetched one tile ahead; lanes 0-3 also
        // keep the previous tile's last 32 bases (codes | reversed validity << 16)
        uint32_t code16, valid8;
        src.decode(src.raw((int64_t)lane * SK_CH), code16, valid8);
        uint32_t halo = 0;
        if constexpr (std::is_same<Src, SeqNt4>::value) {
            // a query view: the 32 bases before it seed the first tile's k-mer registers (the fast
            // path), instead of every view's lane 0 walking back over HBM base by base
            if (pre >= 32 && lane >= 60) {
                uint32_t c16, v8;
                src.decode(src.raw_back((int64_t)(lane - 64) * SK_CH), c16, v8);
                halo = c16 | (rev8(v8) << 16);
            }
        }
        for (int64_t t0 = 0; t0 < L; t0 += SK_TS) {
            // opaque per tile: keeps lane-derived values from being hoisted and held
            // in registers across the read loop (VGPR pressure)
            int ln = lane;
            asm volatile("" : "+v"(ln));
            const int64_t hbase = t0 - w;            // LDS index = p - hbase
            const int64_t ps = t0 + (int64_t)ln * SK_CH;
            const int64_t pe = ps + SK_CH < L ? ps + SK_CH : L;
            // next tile's bases: loaded now, decoded before this tile's first store
            // (vmcnt also counts stores: decoding later would wait for them)
            const uint64_t nbytes = t0 + SK_TS < L ? src.raw(ps + SK_TS) : 0;
            const uint32_t own = code16 | (rev8(valid8) << 16);
            wave_lds_sync();
            SK_PT(0);
            // ---- phase 1a: k-mers and per-position flags.  Warm-up: the k-mer
            // registers hold the last k-1 ACGT bases before ps (ambiguous bases
            // are skipped, src/sketch.rs:75-76,86-88; from the initial zeros at
            // the read start) -- exactly, since the symmetric-k-mer test that
            // gates l sees them.  Fast path: those k-1 bases are the ACGT bases
            // of the four chunks before ps (ln shuffles); otherwise a walk back
            // over HBM.
            uint64_t kf, kr;
            {
                uint64_t W = 0; uint32_t V = 0;
#pragma unroll
                for (int d = 1; d <= 4; ++d) {
                    const uint32_t o1 = (uint32_t)__shfl((int)own, (ln - d) & 63, 64);
                    const uint32_t o2 = (uint32_t)__shfl((int)halo, (ln - d + 4) & 63, 64);
                    const uint32_t pk = ln >= d ? o1 : o2;
                    W |= (uint64_t)(pk & 0xffffu) << (16 * (d - 1));
                    V |= (pk >> 16) << (8 * (d - 1));
                }
                const uint32_t need_bits = (k - 1 >= 32) ? 0xffffffffu : ((1u << (k - 1)) - 1u);
                const bool slow = ps < pe && (ps + pre < k - 1 || (V & need_bits) != need_bits);
                kf = W & ((k - 1 >= 32) ? U64MAX : ((1ULL << (2 * (k - 1))) - 1));
                kr = (rev2_64(~W) >> (64 - 2 * k)) & ~3ULL;
                if (any(slow) && t0 > 0) {
                    // after the first tile: the registers at the previous tile's end (ckf, ckr, exact)
                    // with the valid bases of the chunks before this lane's shifted in -- an exclusive
                    // wave scan of (last 32 valid codes, count), so no lane walks back over HBM
                    // (an N gap of the index build's contigs had every lane of every tile in it
                    // walk back to its start, base by base)
                    uint64_t pc = 0; uint32_t pn = 0;
#pragma unroll
                    for (int u = 0; u < SK_CH; ++u) {
                        const bool vu = (valid8 >> u) & 1u;
                        pc = vu ? (pc << 2) | ((code16 >> (2 * (7 - u))) & 3u) : pc;
                        pn += vu ? 1u : 0u;
                    }
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t olo = (uint32_t)__shfl_up((int)(uint32_t)pc, d, 64), ohi = (uint32_t)__shfl_up((int)(uint32_t)(pc >> 32), d, 64);
                        const uint32_t on = (uint32_t)__shfl_up((int)pn, d, 64);
                        if (ln >= d && pn < 32) { pc = ((((uint64_t)ohi << 32) | olo) << (2 * pn)) | pc; pn = min(32u, pn + on); }
                    }
                    {   // exclusive
                        const uint32_t olo = (uint32_t)__shfl_up((int)(uint32_t)pc, 1, 64), ohi = (uint32_t)__shfl_up((int)(uint32_t)(pc >> 32), 1, 64);
                        const uint32_t on = (uint32_t)__shfl_up((int)pn, 1, 64);
                        pc = ln ? ((uint64_t)ohi << 32) | olo : 0; pn = ln ? on : 0u;
                    }
                    const uint64_t rc = rev2_64(~pc) >> (64 - 2 * k);   // complements, the newest at the top slot
                    if (pn >= (uint32_t)k) { kf = pc & mask; kr = rc; }
                    else {
                        const uint64_t low = (1ULL << (2 * (k - pn))) - 1;
                        kf = ((CK[0] << (2 * pn)) | pc) & mask;
                        kr = (CK[1] >> (2 * pn)) | (rc & ~low);
                    }
                } else if (any(slow)) {
                    if (slow) { kf = 0; kr = 0; }
                    int64_t wsp = ps;
                    int need = slow ? k - 1 : 0;
                    while (any(need > 0 && wsp > -pre)) {   // back to the contig start (views: before the view)
                        if (need > 0 && wsp > -pre) {
                            if ((wsp & 7) == 0 && wsp - 8 >= -pre && src.amb8(wsp - 8)) wsp -= 8;   // an N run, 8 at a time
                            else { --wsp; if (src.code(wsp) < 4) --need; }
                        }
                    }
                    int64_t pw = slow ? wsp : ps;
                    while (any(pw < ps)) {
                        if (pw < ps) {
                            const uint32_t c = src.code(pw);
                            if (c < 4) { kf = ((kf << 2) | c) & mask; kr = (kr >> 2) | ((uint64_t)(3 ^ c) << shift1); }
                            ++pw;
                        }
                    }
                }
            }
            SK_PT(1);
            // k <= 16: the k-mer registers fit 32 bits (2k <= 32)
            using KT = typename std::conditional<K32, uint32_t, uint64_t>::type;
            KT kf2 = (KT)kf, kr2 = (KT)kr;
            const KT kmask = (KT)mask;
            bool rs = false; int32_t lc = 0;
            uint32_t flz = 0;   // per position t: fl (0 ambiguous, 1 symmetric, 2 info) | z << 2, at bits 3t
            // branch-free per position (a divergent if per position cost exec-mask saves and
            // SGPR spills); every slot of the tile exists in LDS, so a position past the read's
            // end is written too (never read: the next tile's history needs positions < L)
#pragma unroll
            for (int t = 0; t < SK_CH; ++t) {
                const int64_t p = ps + t;
                const bool in = p < pe;
                const int ix = (int)(p - hbase);
                const uint32_t c = (code16 >> (2 * (7 - t))) & 3u;
                const bool v = in && ((valid8 >> t) & 1u);
                const KT nkf = ((kf2 << 2) | (KT)c) & kmask, nkr = (kr2 >> 2) | ((KT)(3 ^ c) << shift1);
                kf2 = v ? nkf : kf2; kr2 = v ? nkr : kr2;
                const bool ns = kf2 != kr2;
                const uint32_t z = kf2 < kr2 ? 0u : 1u;
                const uint64_t km = z ? kr2 : kf2;
                uint64_t h;
                if (K32) h = hash64d<uint32_t>((uint32_t)km, (uint32_t)mask);
                else h = hash64d<uint64_t>(km, mask);
                XT x;
                if constexpr (HPC) {               // TinyQueue span (sketch.rs:51-64, 72)
                    const uint32_t sp = (v && ns) ? a.hpc_span[roff + (uint64_t)p] : 256u;
                    x = sp < 256u ? (h << 8) | (uint64_t)sp : U64MAX;
                } else if constexpr (X32) {
                    x = (v && ns) ? (XT)h : XMAX;  // X32: the hash alone (span == k)
                } else {
                    x = (v && ns) ? (h << 8) | (uint64_t)k : XMAX;   // kmer_span == k whenever info is valid
                }
                const uint32_t fl = v ? (ns ? 2u : 1u) : 0u;
                X[SKP(ix)] = x;
                flz |= (fl | ((v && ns ? z : 0u) << 2)) << (3 * t);
                const bool r0 = in && fl == 0u;
                rs |= r0;
                lc = r0 ? 0 : ((in && fl == 2u) ? (lc + 1 < CAP ? lc + 1 : CAP) : lc);
            }
            if (ln == 63) { CK[0] = (uint64_t)kf2; CK[1] = (uint64_t)kr2; }   // read by the next tile (after its wave_lds_sync)
            // ---- segmented scan of l over lanes: (reset, count)
            int32_t er, ec;
            {
                int32_t ir = rs ? 1 : 0, ic = lc;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int32_t orr = __shfl_up(ir, d, 64), oc = __shfl_up(ic, d, 64);
                    if (ln >= d && !ir) { ic = oc + ic < CAP ? oc + ic : CAP; ir = orr; }
                }
                er = __shfl_up(ir, 1, 64); ec = __shfl_up(ic, 1, 64);
                if (ln == 0) { er = 0; ec = 0; }
            }
            const int32_t lin = er ? ec : (l_carry + ec < CAP ? l_carry + ec : CAP);
            // ---- phase 1b: l per position (the flags from registers); invalidate info where l < k
            int32_t lv = lin;
#pragma unroll
            for (int t = 0; t < SK_CH; ++t) {
                const int64_t p = ps + t;
                const bool in = p < pe;
                const int ix = (int)(p - hbase);
                const uint32_t fl = (flz >> (3 * t)) & 3u, z = (flz >> (3 * t + 2)) & 1u;
                lv = !in ? lv : (fl == 0u ? 0 : (fl == 2u ? (lv + 1 < CAP ? lv + 1 : CAP) : lv));
                LZ[SKP(ix)] = (uint16_t)((z << 15) | (uint32_t)lv);
                if (in && !(fl == 2u && lv >= k)) X[SKP(ix)] = XMAX;
            }
            {
                const int64_t te = t0 + SK_TS < L ? t0 + SK_TS : L;
                const int owner = (int)((te - 1 - t0) / SK_CH);
                l_carry = rdl(lv, owner);
            }
            wave_lds_sync();
            SK_PT(2);
#define SK_Y(q) ((((uint32_t)(hbase + (q))) << 1) | (uint32_t)(LZ[SKP((q))] >> 15))
            uint32_t code16n, valid8n;
            src.decode(nbytes, code16n, valid8n);
            // ---- phase 2: reference step logic, count then write
            uint32_t myoff = 0, tot = 0;
            bool fast_done = false;
#define SK_EMIT(xv, yv) do { if (em_ok) { if (WR && o < oend) { a.mz_x[o] = xout(xv); a.mz_y[o] = (yv); } ++o; ++n_em; } } while (0)
            if (w > SK_CH) {
                // The reference's `min` after step i is the newest minimum of slots
                // [i-w+1, i] (DESIGN.md "Sketch").  Window = [i-w+1, ps-1] u [ps, i]:
                // suffix minima of the history part come from one backward scan
                // (s*[u] for j = ps-w+u), prefix minima of the chunk part are kept
                // while stepping; both carry the multiplicity of the minimum, so
                // tie scans run only where the minimum really occurs twice.
                // s*: (x, LDS slot | multiple<<16) of the newest minimum of [j, ps-1]
                XT sx[SK_CH + 1]; uint32_t sp[SK_CH + 1];
                {
                    XT cx = XMAX; uint32_t cp = 0xffffffffu;
                    const int q0 = (int)(ps - hbase);
                    for (int d = 1; d < w - SK_CH; ++d) {          // slot q0 - d (newest first)
                        const XT x = X[SKP(q0 - d)];
                        if (cp == 0xffffffffu || x < cx) { cx = x; cp = (uint32_t)(q0 - d); } else if (x == cx) cp |= 0x10000u;
                    }
#pragma unroll
                    for (int t = 0; t <= SK_CH; ++t) {
                        const int d = w - SK_CH + t;                 // j = ps - w + (SK_CH - t)
                        const XT x = X[SKP(q0 - d)];
                        if (cp == 0xffffffffu || x < cx) { cx = x; cp = (uint32_t)(q0 - d); } else if (x == cx) cp |= 0x10000u;
                        sx[SK_CH - t] = cx; sp[SK_CH - t] = cp;
                    }
                }
                // B/C emissions only (at most one per position: recorded as a bit and
                // the LDS slot of the emitted minimum); ties (A, or T after C) take
                // the exact path below for the whole wave
                bool need = false;
                uint32_t em = 0, eq[SK_CH / 2] = {};
                {
                    XT px = XMAX; uint32_t pp = 0xffffffffu;   // prefix minimum of [ps, i]
                    XT mxo = sx[0]; int mqo = (int)(sp[0] & 0xffffu);
#pragma unroll
                    for (int t = 0; t < SK_CH; ++t) {
                        const int64_t i = ps + t;
                        const bool act = i < pe;
                        const int ii = (int)(i - hbase);
                        const XT xi = act ? X[SKP(ii)] : XMAX;
                        const int32_t l = act ? (int32_t)(LZ[SKP(ii)] & 0x7fffu) : 0;
                        // A (sketch.rs:90-93): at the first full window, the slots before i that tie
                        // the minimum (other than the minimum's own slot) are emitted.  Ties of random
                        // hashes are rare, so the lane looks for one and only then takes the exact path
                        // (every read start and every N run used to send its tile there: 5 % of tiles)
                        if (act && l == w + k - 1 && mxo != XMAX) {
                            for (int d = 1; d < w; ++d) {
                                const int q = ii - w + d;
                                need |= q != mqo && X[SKP(q)] == mxo;
                            }
                        }
                        const bool doB = act && xi <= mxo;                              // B (94-96)
                        const bool doC = act && !doB && mqo == ii - w;                  // C (97-105)
                        if (((doB && l >= w + k && mxo != XMAX) || (doC && l >= w + k - 1)) && i >= efrom) {
                            em |= 1u << t; eq[t >> 1] |= (uint32_t)mqo << (16 * (t & 1));
                        }
                        if (act) {
                            if (pp == 0xffffffffu || xi < px) { px = xi; pp = (uint32_t)ii; }
                            else if (xi == px) pp = (uint32_t)ii | 0x10000u;
                        }
                        XT mxn; uint32_t mpn;
                        if (px < sx[t + 1]) { mxn = px; mpn = pp; }
                        else if (px > sx[t + 1]) { mxn = sx[t + 1]; mpn = sp[t + 1]; }
                        else { mxn = px; mpn = pp | 0x10000u; }
                        need |= doC && l >= w + k - 1 && mxn != XMAX && (mpn & 0x10000u);   // T
                        mxo = mxn; mqo = (int)(mpn & 0xffffu);
                    }
                }
                if (!any(need)) {
                    myoff = wave_excl_sum((uint32_t)__popc(em), tot);
                    uint64_t o = obase + count + myoff;
#pragma unroll
                    for (int t = 0; t < SK_CH; ++t) {
                        if ((em >> t) & 1u) {
                            const int q = (int)((eq[t >> 1] >> (16 * (t & 1))) & 0xffffu);
                            if (o < oend) { a.mz_x[o] = xout(X[SKP(q)]); a.mz_y[o] = SK_Y(q); }
                            ++o;
                        }
                    }
                    fast_done = true;
                }
            }
            ++n_tiles;
            if (!fast_done) {
              ++n_slow;
              myoff = 0; tot = 0;
              for (int pass = 0; pass < 2; ++pass) {
                const bool WR = pass == 1;
                uint64_t o = obase + count + myoff;
                uint32_t n_em = 0;
                // newest minimum of the w slots before the chunk (same for every ln count)
                XT mx = XMAX; uint32_t my = 0xffffffffu; int64_t mp = ps - w - 1;
                for (int d = 0; d < w; ++d) {
                    const int64_t p = ps - w + d;
                    const int q = (int)(p - hbase);
                    const XT x = X[SKP(q)];
                    if (mx >= x) { mx = x; my = SK_Y(q); mp = p; }
                }
                for (int t = 0; t < SK_CH; ++t) {
                    const int64_t i = ps + t;
                    const bool act = i < pe;
                    const bool em_ok = i >= efrom;   // warm-up steps of an index view emit nothing
                    const int ii = (int)(i - hbase);
                    const XT ix_x = act ? X[SKP(ii)] : XMAX;
                    const uint32_t ix_y = act ? SK_Y(ii) : 0xffffffffu;
                    const int32_t l = act ? (int32_t)(LZ[SKP(ii)] & 0x7fffu) : 0;
                    const bool doA = act && l == w + k - 1 && mx != XMAX;
                    if (any(doA)) {
                        for (int d = 1; d < w; ++d) {
                            const int q = ii - w + d;
                            if (doA && X[SKP(q)] == mx && SK_Y(q) != my) SK_EMIT(X[SKP(q)], SK_Y(q));
                        }
                    }
                    const bool doB = act && ix_x <= mx;
                    const bool doC = act && !doB && mp == i - w;
                    if ((doB && l >= w + k && mx != XMAX) || (doC && l >= w + k - 1)) SK_EMIT(mx, my);
                    if (doB) { mx = ix_x; my = ix_y; mp = i; }
                    if (any(doC)) {
                        XT nx = XMAX; uint32_t ny = 0; int64_t np = mp;
                        for (int d = 1; d <= w; ++d) {
                            const int q = ii - w + d;
                            const XT x = X[SKP(q)];
                            if (nx >= x) { nx = x; ny = SK_Y(q); np = i - w + d; }
                        }
                        if (doC) { mx = nx; my = ny; mp = np; }
                        const bool doT = doC && l >= w + k - 1 && mx != XMAX;
                        if (any(doT)) {
                            for (int d = 1; d <= w; ++d) {
                                const int q = ii - w + d;
                                if (doT && mx == X[SKP(q)] && my != SK_Y(q)) SK_EMIT(X[SKP(q)], SK_Y(q));
                            }
                        }
                    }
                }
                if (!WR) myoff = wave_excl_sum(n_em, tot);
              }
            }
#undef SK_EMIT
            count += tot;
            SK_PT(3);
            // ---- next tile: its halo = this tile's chunks 60-63; prefetched bases
            halo = (uint32_t)__shfl((int)own, (ln + 60) & 63, 64);
            code16 = code16n; valid8 = valid8n;
            // ---- move the last w slots to the history area
            wave_lds_sync();
            if (t0 + SK_TS < L) {
                // source [TS, TS+w) and destination [0, w) never overlap (w < 256 <= TS)
                for (int b0 = 0; b0 < w; b0 += 64) {
                    const int t = b0 + ln;
                    if (t < w) { X[SKP(t)] = X[SKP(SK_TS + t)]; LZ[SKP(t)] = LZ[SKP(SK_TS + t)]; }
                }
            }
            wave_lds_sync();
        }
        // end of sequence (sketch.rs:99): newest minimum of the last window
        {
            const int64_t tl = ((L - 1) / SK_TS) * SK_TS;   // last tile start
            const int64_t hbase = tl - w;
            XT mx = XMAX; uint32_t my = 0;
            for (int d = 0; d < w; ++d) {
                const int q = (int)(L - w + d - hbase);
                const XT x = X[SKP(q)];
                if (mx >= x) { mx = x; my = SK_Y(q); }
            }
            if (mx != XMAX && flush) {
                const uint64_t o = obase + count;
                if (lane == 0 && o < oend) { a.mz_x[o] = xout(mx); a.mz_y[o] = my; }
                ++count;
            }
            if (lane == 0) {
                // a count beyond the slot is clamped (every later kernel stays inside the
                // buffers) and flagged; the true count lets the host size an exact re-run
                const uint64_t capn = oend - obase;
                a.mz_cnt[r] = (uint32_t)(count > capn ? capn : count);
                if (a.mz_need) a.mz_need[r] = (uint32_t)(count > 0xffffffffULL ? 0xffffffffULL : count);
                if (count > capn) atomicOr(a.overflow, 1);
            }
        }
        SK_PT(4);
        if (a.prof && lane == 0) {
            for (int q = 0; q < 5; ++q) a.prof[(uint64_t)r * 8 + q] = pt[q];
            a.prof[(uint64_t)r * 8 + 5] = (uint64_t)L;
            a.prof[(uint64_t)r * 8 + 6] = wall_clock64();
            a.prof[(uint64_t)r * 8 + 7] = ((uint64_t)n_tiles << 32) | n_slow;
        }
#undef SK_PT
#undef SK_Y
        wave_lds_sync();
    }
}

// ============================================================================
// 2. QUERY FILTER — filter_query_minimizers(mv, 10, 0.01) (src/seeds.rs:13-36)
// One wave per read; an open-addressed count table per read in a scratch
// region (size nextpow2(2m) when m > q_occ_max).  keep[i] = 0 for every
// minimizer whose hash occurs cnt > q_occ_max && cnt > (m*frac as f32) as usize.
// ============================================================================
DEVI uint32_t tab_size_for(uint32_t m, int q_occ_max) {
    if ((int64_t)m <= (int64_t)q_occ_max || m == 0) return 0;
    uint32_t t = 2u * m, s = 1;
    while (s < t) s <<= 1;
    return s;
}
DEVI uint32_t fslot(uint64_t h, uint32_t tmask) { return (uint32_t)((h * 0x9E3779B97F4A7C15ULL) >> 32) & tmask; }
constexpr int FT_MAX = 4096;
DEVI bool filter_lds_ok(uint32_t ts, int k) { return ts > 0 && ts <= (uint32_t)FT_MAX && k <= 16; }

// Reads whose count table does not fit k_filter_lds (large m, or k > 16):
// persistent 1024-thread blocks, one read at a time.  Reads with m <= 65535
// (C5's 100 kb reads: m ~ 18.6 k) count in LDS: est[] holds, per slot of
// fslot(h), the number of minimizers hashed there -- at least the count of
// every hash in the slot -- so a minimizer with est <= T = max(q_occ_max,
// cutoff) keeps (the reference drops it iff cnt > q_occ_max && cnt > cutoff);
// only hashes over T get exact counts, in a small LDS table (all occurrences
// of a hash share its slot, so they all enter).  The global open-addressed
// table (the former path, ~1.6 GB of zeroing per C5 step) remains for larger
// reads and for a candidate-table overflow.
constexpr int FB_EST = 32768;          // estimate counters (u32)
constexpr int FB_XT = 1024;            // exact slots for the hashes over T (u64 key + u32 count)
constexpr size_t FB_LDS = (size_t)FB_EST * 4 + (size_t)FB_XT * 12;
__global__ __launch_bounds__(1024) void k_filter(FilterArgs a, int a_k) {
    extern __shared__ __align__(16) unsigned char fsm[];
    uint32_t* est = (uint32_t*)fsm;
    unsigned long long* xk = (unsigned long long*)(fsm + (size_t)FB_EST * 4);
    uint32_t* xc = (uint32_t*)(xk + FB_XT);
    __shared__ uint32_t s_ovf;
    const int tid = threadIdx.x;
    for (uint32_t r = blockIdx.x; r < a.n; r += gridDim.x) {
        const uint64_t mb = a.mz_base[r];
        const uint32_t m = a.mz_cnt[r];
        uint8_t* keep = a.keep + mb;
        const uint32_t ts = tab_size_for(m, a.q_occ_max);
        if (a.q_occ_frac <= 0.0f || a.q_occ_max <= 0 || ts == 0) continue;   // seeds.rs:14-15: k_filter_lds
        if (filter_lds_ok(ts, a_k)) continue;                      // done by k_filter_lds
        const float prod = (float)m * a.q_occ_frac;                // (m as f32 * q_occ_frac) as usize
        const uint64_t cutoff = prod <= 0.0f ? 0ULL : (uint64_t)prod;
        const uint64_t T = cutoff > (uint64_t)a.q_occ_max ? cutoff : (uint64_t)a.q_occ_max;
        if (m <= 65535u) {
            for (int i = tid; i < FB_EST; i += 1024) est[i] = 0;
            for (int i = tid; i < FB_XT; i += 1024) { xk[i] = U64MAX; xc[i] = 0; }
            if (tid == 0) s_ovf = 0;
            __syncthreads();
            for (uint32_t i = tid; i < m; i += 1024) atomicAdd(&est[fslot(a.mz_x[mb + i] >> 8, FB_EST - 1)], 1u);
            __syncthreads();
            for (uint32_t i = tid; i < m; i += 1024) {
                const uint64_t h = a.mz_x[mb + i] >> 8;
                if ((uint64_t)est[fslot(h, FB_EST - 1)] <= T) continue;
                uint32_t sl = fslot(h, FB_XT - 1);
                for (int pr = 0;; ++pr) {
                    if (pr == FB_XT) { s_ovf = 1; break; }
                    const unsigned long long prev = atomicCAS(&xk[sl], (unsigned long long)U64MAX, (unsigned long long)h);
                    if (prev == U64MAX || prev == h) { atomicAdd(&xc[sl], 1u); break; }
                    sl = (sl + 1) & (FB_XT - 1);
                }
            }
            __syncthreads();
            const bool ovf = s_ovf != 0;
            if (!ovf) {
                for (uint32_t i = tid; i < m; i += 1024) {
                    const uint64_t h = a.mz_x[mb + i] >> 8;
                    uint8_t kp = 1;
                    if ((uint64_t)est[fslot(h, FB_EST - 1)] > T) {
                        uint32_t sl = fslot(h, FB_XT - 1), c = 0;
                        for (int pr = 0; pr < FB_XT; ++pr) {
                            const unsigned long long e = xk[sl];
                            if (e == h) { c = xc[sl]; break; }
                            if (e == U64MAX) break;
                            sl = (sl + 1) & (FB_XT - 1);
                        }
                        kp = (uint64_t)c > T ? 0 : 1;
                    }
                    keep[i] = kp;
                }
            }
            __syncthreads();                                   // the LDS tables are reused by the next read
            if (!ovf) continue;
        }
        const uint64_t tb = a.tab_off[r];                          // prefix of the global tables only
        if (tb + ts > a.cap_tab) continue;                         // workspace too small: batch flagged BS_TAB by the scan
        uint64_t* tk = a.tab_key + tb; uint32_t* tc = a.tab_cnt + tb;
        for (uint32_t i = tid; i < ts; i += 1024) { tk[i] = U64MAX; tc[i] = 0; }
        __threadfence_block();
        __syncthreads();
        const uint32_t tmask = ts - 1;
        for (uint32_t b0 = 0; b0 < m; b0 += 1024) {
            const uint32_t i = b0 + tid;
            bool done = i >= m;
            const uint64_t h = done ? 0 : (a.mz_x[mb + i] >> 8);
            uint32_t sl = fslot(h, tmask);
            while (any(!done)) {
                if (!done) {
                    const unsigned long long prev = atomicCAS((unsigned long long*)&tk[sl], (unsigned long long)U64MAX, (unsigned long long)h);
                    if (prev == U64MAX || prev == h) { atomicAdd(&tc[sl], 1u); done = true; }
                    else sl = (sl + 1) & tmask;
                }
            }
        }
        __threadfence_block();
        __syncthreads();
        for (uint32_t b0 = 0; b0 < m; b0 += 1024) {
            const uint32_t i = b0 + tid;
            bool done = i >= m;
            const uint64_t h = done ? 0 : (a.mz_x[mb + i] >> 8);
            uint32_t sl = fslot(h, tmask), c = 0;
            while (any(!done)) {
                if (!done) {
                    const uint64_t kk = __hip_atomic_load(&tk[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (kk == h) { c = __hip_atomic_load(&tc[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); done = true; }
                    else if (kk == U64MAX) done = true;
                    else sl = (sl + 1) & tmask;
                }
            }
            if (i < m) keep[i] = ((int64_t)c > (int64_t)a.q_occ_max && (uint64_t)c > cutoff) ? 0 : 1;
        }
        __syncthreads();                                       // before the next read reuses s_ovf / LDS
    }
}

// LDS variant: one 256-thread block per read, for hashes that fit 32 bits
// (k <= 16) and tables of at most FT_MAX slots; entries pack (count << 32 | hash)
// so one 64-bit LDS CAS claims a slot.  Other reads are left to k_filter.

__global__ __launch_bounds__(256) void k_filter_lds(FilterArgs a, int k) {
    __shared__ unsigned long long T[FT_MAX];
    const uint32_t r = blockIdx.x;
    if (r >= a.n) return;
    const uint64_t mb = a.mz_base[r];
    const uint32_t m = a.mz_cnt[r];
    const uint32_t ts = tab_size_for(m, a.q_occ_max);
    uint8_t* keep = a.keep + mb;
    if (a.q_occ_frac <= 0.0f || a.q_occ_max <= 0 || ts == 0) {      // seeds.rs:14-15 (and m <= q_occ_max)
        for (uint32_t i = threadIdx.x; i < m; i += 256) keep[i] = 1;
        return;
    }
    if (!filter_lds_ok(ts, k)) return;
    const float prod = (float)m * a.q_occ_frac;                       // (m as f32 * q_occ_frac) as usize
    const uint64_t cutoff = prod <= 0.0f ? 0ULL : (uint64_t)prod;
    {
        // Round 5: upper bounds first.  4096 u16 counters (in T's first 8 KB) count the
        // minimizers per fslot of their hash, an upper bound of every hash's count there
        // (m <= 2048 here, so no counter overflows).  A minimizer is dropped only when its
        // count exceeds both q_occ_max and the cutoff; when no counter does, every one is
        // kept and the exact table is not built (nearly every read: a hash must occur over
        // max(10, m / 100) times in one read).
        uint32_t* CM = (uint32_t*)T;
        for (uint32_t i = threadIdx.x; i < 2048; i += 256) CM[i] = 0u;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += 256) {
            const uint32_t sl = fslot(a.mz_x[mb + i] >> 8, 4095u);
            atomicAdd(&CM[sl >> 1], 1u << ((sl & 1u) << 4));
        }
        __syncthreads();
        uint32_t mx = 0;
        for (uint32_t i = threadIdx.x; i < 2048; i += 256) { const uint32_t v = CM[i]; mx = max(mx, max(v & 0xffffu, v >> 16)); }
        const uint64_t thr = (uint64_t)a.q_occ_max > cutoff ? (uint64_t)a.q_occ_max : cutoff;
        if (!__syncthreads_or((uint64_t)mx > thr)) {
            for (uint32_t i = threadIdx.x; i < m; i += 256) keep[i] = 1;
            return;
        }
    }
    const uint32_t tmask = ts - 1;
    for (uint32_t i = threadIdx.x; i < ts; i += 256) T[i] = 0ULL;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += 256) {
        const uint32_t h = (uint32_t)(a.mz_x[mb + i] >> 8);
        uint32_t sl = fslot(h, tmask);
        for (;;) {
            const unsigned long long prev = atomicCAS(&T[sl], 0ULL, (1ULL << 32) | h);
            if (prev == 0ULL) break;
            if ((uint32_t)prev == h) { atomicAdd(&T[sl], 1ULL << 32); break; }
            sl = (sl + 1) & tmask;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += 256) {
        const uint32_t h = (uint32_t)(a.mz_x[mb + i] >> 8);
        uint32_t sl = fslot(h, tmask);
        uint32_t c = 0;
        for (;;) {
            const unsigned long long e = T[sl];
            if (e == 0ULL) break;
            if ((uint32_t)e == h) { c = (uint32_t)(e >> 32); break; }
            sl = (sl + 1) & tmask;
        }
        keep[i] = ((int64_t)c > (int64_t)a.q_occ_max && (uint64_t)c > cutoff) ? 0 : 1;
    }
}

// ============================================================================
// 3. LOOKUP + ANCHORS — Index::get (src/index.rs:143-154), the mid_occ skip of
// build_anchors_filtered (src/seeds.rs:42-57) and push_anchor (seeds.rs:62-79).
// ============================================================================
// One workgroup per read, one wave per part: parts are the same runs of whole 64-minimizer
// chunks k_seed_write takes (round 5; one wave per read left most of the GPU idle on C5's
// 1,000-read units).  The part totals give the read's count and k_seed_write's part starts.
__global__ __launch_bounds__(SEED_PARTS * 64) void k_seed_count(SeedArgs a) {
    static_assert(SEED_PARTS == 16, "a wave per part, 16 per workgroup");
    __shared__ uint32_t s_tot[SEED_PARTS], s_kept[SEED_PARTS];
    const int lane = lane_id();
    const uint32_t cmask = (1u << a.log2cap) - 1;
    for (uint32_t r = blockIdx.x; r < a.n; r += gridDim.x) {
        const uint32_t part = (uint32_t)wave_id();
        const uint64_t mb = uni64(a.mz_base[r]);
        const uint32_t m = (uint32_t)uni((int32_t)a.mz_cnt[r]);
        const uint32_t nch = (m + 63) >> 6;
        const uint32_t cb = (nch * part) / SEED_PARTS, ce = (nch * (part + 1)) / SEED_PARTS;
        const uint32_t iend = ce * 64 < m ? ce * 64 : m;
        uint32_t acc = 0, kept = 0;
        // SC_U chunks of 64 minimizers at a time: their table probes are
        // independent, so SC_U loads per lane are in flight together
        constexpr int SC_U = 4;
        for (uint32_t b0 = cb * 64; b0 < iend; b0 += 64 * SC_U) {
            uint64_t h[SC_U];
            uint32_t sl[SC_U], n[SC_U], off[SC_U];
            bool done[SC_U];
#pragma unroll
            for (int u = 0; u < SC_U; ++u) {
                const uint32_t i = b0 + (uint32_t)u * 64 + lane;
                const bool act = i < iend;
                done[u] = !(act && a.keep[mb + i]);
                kept += done[u] ? 0u : 1u;
                h[u] = act ? (a.mz_x[mb + i] >> 8) : 0;
                sl[u] = ix_slot(h[u], a.log2cap); n[u] = 0; off[u] = 0;
            }
            // linear probing, one slot per step (measured against 64-B groups of
            // four slots per step: twice the load instructions and 2x slower)
            while (any(!(done[0] && done[1] && done[2] && done[3]))) {
                IxEntry e[SC_U];
#pragma unroll
                for (int u = 0; u < SC_U; ++u) if (!done[u]) e[u] = a.tab[sl[u]];
#pragma unroll
                for (int u = 0; u < SC_U; ++u) {
                    if (done[u]) continue;
                    if (e[u].key == h[u]) { off[u] = e[u].off; n[u] = e[u].n; done[u] = true; }
                    else if (e[u].key == U64MAX) done[u] = true;
                    else sl[u] = (sl[u] + 1) & cmask;
                }
            }
#pragma unroll
            for (int u = 0; u < SC_U; ++u) {
                const uint32_t i = b0 + (uint32_t)u * 64 + lane;
                // mz_n: the anchor count, or IX_INLINE | position high word for a Single
                uint32_t nn = n[u];
                if (!(nn & IX_INLINE) && nn > 1 && (int64_t)nn > (int64_t)a.mid_occ) nn = 0;   // Multi with len > mid_occ: skip
                if (i < iend) { a.mz_n[mb + i] = nn; a.mz_poff[mb + i] = off[u]; }
                acc += ix_count(nn);
            }
        }
        acc = wave_sum(acc);
        kept = wave_sum(kept);
        if (lane == 0) { s_tot[part] = acc; s_kept[part] = kept; }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0, kt = 0;
            for (int q = 0; q < SEED_PARTS; ++q) {
                if (q) a.a_part[(uint64_t)r * (SEED_PARTS - 1) + q - 1] = run;
                run += s_tot[q]; kt += s_kept[q];
            }
            a.a_cnt[r] = run; a.out[r].m_kept = (int32_t)kt;
        }
        __syncthreads();                                       // s_tot is reused by the next read
    }
}

// push_anchor (src/seeds.rs:62-79) packed into the sortable 64-bit key.
DEVI uint64_t pack_anchor(uint64_t rr, uint32_t my, int32_t qlen, int span, const KeyLayout& kl) {
    const uint32_t rid = (uint32_t)(rr >> 32);
    const uint32_t rpos32 = (uint32_t)(rr >> 1);       // ((r >> 1) & 0xffffffff)
    const uint32_t rstrand = (uint32_t)(rr & 1);
    const uint32_t qpos = my >> 1, qstrand = my & 1;
    const bool fwd = rstrand == qstrand;
    const uint32_t q = fwd ? qpos : (uint32_t)(qlen - ((int32_t)qpos + 1 - span) - 1);
    uint64_t g; uint32_t p;
    if (rpos32 & 0x80000000u) { g = 2ull * kl.n_seq; p = rpos32 & 0x7fffffffu; }   // Q19 pseudo-group
    else { g = fwd ? (uint64_t)rid : (uint64_t)kl.n_seq + rid; p = rpos32; }
    return (g << (kl.rb + kl.qb)) | ((uint64_t)p << kl.qb) | (uint64_t)q;
}

__global__ __launch_bounds__(256) void k_seed_write(SeedArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    __shared__ uint32_t s_inc[4][64], s_poff[4][64], s_y[4][64], s_hi[4][64];
    const int lane = lane_id(), wv = wave_id();
    const int nwaves = (int)(gridDim.x * (blockDim.x >> 6));
    constexpr int U = 8;   // output batches whose position gathers are in flight together
    // one wave per (read, part): parts are contiguous runs of whole 64-minimizer
    // chunks, starting at the anchor counts seed_count recorded
    for (uint32_t wp = blockIdx.x * (blockDim.x >> 6) + wv; wp < a.n * (uint32_t)SEED_PARTS; wp += nwaves) {
        const uint32_t r = a.order ? (uint32_t)uni((int32_t)a.order[wp / SEED_PARTS]) : wp / SEED_PARTS, part = wp % SEED_PARTS;
        const uint64_t mb = uni64(a.mz_base[r]);
        const uint32_t m = (uint32_t)uni((int32_t)a.mz_cnt[r]);
        const uint32_t nch = (m + 63) >> 6;
        const uint32_t cb = (nch * part) / SEED_PARTS, ce = (nch * (part + 1)) / SEED_PARTS;
        if (cb >= ce) continue;
        const uint64_t obase = uni64(a.a_off[r]);
        if (a.fuse_mmax && m <= a.fuse_mmax) {   // k_sort_read writes this read's keys (its first pass)
            const uint64_t A0 = uni64(a.a_off[r + 1]) - obase;
            if (A0 > a.small_max && A0 <= 65535u) continue;
        }
        if (a.fuse_big && uni64(a.a_off[r + 1]) - obase > 65535u) continue;   // ... k_sort_big's first pass
        const int32_t qlen = (int32_t)(uni64(a.rd_off[r + 1]) - uni64(a.rd_off[r]));
        uint64_t* out = a.keys;
        uint64_t run = part ? (uint64_t)(uint32_t)uni((int32_t)a.a_part[(uint64_t)r * (SEED_PARTS - 1) + part - 1]) : 0;
        const uint32_t cend = ce * 64 < m ? ce * 64 : m;
        for (uint32_t c0 = cb * 64; c0 < cend; c0 += 64) {
            const uint32_t i = c0 + lane;
            const bool vi = i < m;
            const uint32_t nraw = vi ? a.mz_n[CK(mb + i, a.cap_mz)] : 0;
            const uint32_t po = vi ? a.mz_poff[CK(mb + i, a.cap_mz)] : 0;
            const uint32_t yy = vi ? a.mz_y[CK(mb + i, a.cap_mz)] : 0;
            const uint32_t n = ix_count(nraw);
            uint32_t tot;
            const uint32_t ex = wave_excl_sum(n, tot);
            s_inc[wv][lane] = ex + n; s_poff[wv][lane] = po; s_y[wv][lane] = yy;
            s_hi[wv][lane] = nraw;
            wave_lds_sync();
            for (uint32_t tb = 0; tb < tot; tb += 64 * U) {
                uint64_t rr[U];
                uint32_t own[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t t = tb + (uint32_t)u * 64 + (uint32_t)lane;
                    rr[u] = 0; own[u] = 0;
                    if (t < tot) {
                        // owner = number of inclusive offsets <= t (first lane whose offset exceeds t)
                        uint32_t lo = 0;
#pragma unroll
                        for (uint32_t step = 32; step >= 1; step >>= 1)
                            if (s_inc[wv][lo + step - 1] <= t) lo += step;
                        const uint32_t exo = lo ? s_inc[wv][lo - 1] : 0;
                        own[u] = lo;
                        const uint32_t hi = s_hi[wv][lo];
                        if (hi & IX_INLINE) rr[u] = ((uint64_t)(hi & ~IX_INLINE) << 32) | s_poff[wv][lo];   // Single: no gather
                        else rr[u] = a.ix_pos[CK((uint64_t)s_poff[wv][lo] + (t - exo), a.cap_pos)];
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t t = tb + (uint32_t)u * 64 + (uint32_t)lane;
                    if (t < tot) out[CK(obase + run + t, a.cap_keys)] = pack_anchor(rr[u], s_y[wv][own[u]], qlen, a.span, a.kl);
                }
            }
            run += tot;
            wave_lds_sync();
        }
    }
}

// 4. ANCHOR SORT — a.sort_by((x, y)) (src/seeds.rs:58) as a segmented sort of
// the packed keys (a total order; equal keys are identical anchors).
//   small segments (A <= 4096): LDS bitonic sort, one workgroup per read;
//   large segments: LSD radix sort (8-bit digits over the varying bits only),
//   one 1024-thread workgroup per read, stable ranking by wave match.
// ============================================================================
constexpr int SORT_SMALL = 4096;
// Bitonic sort of the 2^LOG keys in s (2^LOG >= 512) by 256 threads with the keys in registers:
// thread t holds keys t*KPT .. t*KPT+KPT-1.  Stages with j < KPT compare inside a thread, stages
// with j < 64 KPT exchange with lane t ^ (j / KPT) of the same wave, and only the stages with
// j >= 64 KPT (three of them) go through LDS with workgroup barriers.  The sorted keys are left in s.
template <int LOG>
DEVI void small_sort_reg(uint64_t* s) {
    constexpr int NP = 1 << LOG, KPT = NP / 256;
    const int t = threadIdx.x;
    uint64_t x[KPT];
#pragma unroll
    for (int r = 0; r < KPT; ++r) x[r] = s[t * KPT + r];
#pragma unroll
    for (int kk = 2; kk <= NP; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j < KPT) {
#pragma unroll
                for (int r = 0; r < KPT; ++r) {
                    if ((r ^ j) > r) {
                        const bool up = ((t * KPT + r) & kk) == 0;
                        const uint64_t p = x[r], q = x[r ^ j];
                        const bool sw = (p > q) == up;
                        x[r] = sw ? q : p; x[r ^ j] = sw ? p : q;
                    }
                }
            } else if (j < 64 * KPT) {
                const int m = j / KPT;
                const bool lowt = (t & m) == 0, up = ((t * KPT) & kk) == 0;
#pragma unroll
                for (int r = 0; r < KPT; ++r) {
                    const uint32_t yl = (uint32_t)__shfl_xor((int)(uint32_t)x[r], m, 64);
                    const uint32_t yh = (uint32_t)__shfl_xor((int)(uint32_t)(x[r] >> 32), m, 64);
                    const uint64_t y = ((uint64_t)yh << 32) | yl;
                    x[r] = (lowt == up) ? (x[r] < y ? x[r] : y) : (x[r] > y ? x[r] : y);
                }
            } else {
                __syncthreads();
#pragma unroll
                for (int r = 0; r < KPT; ++r) s[t * KPT + r] = x[r];
                __syncthreads();
                const int m = j / KPT;
                const bool lowt = (t & m) == 0, up = ((t * KPT) & kk) == 0;
#pragma unroll
                for (int r = 0; r < KPT; ++r) {
                    const uint64_t y = s[(t ^ m) * KPT + r];
                    x[r] = (lowt == up) ? (x[r] < y ? x[r] : y) : (x[r] > y ? x[r] : y);
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KPT; ++r) s[t * KPT + r] = x[r];
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_sort_small(SortArgs a) {
    if (blockIdx.x == 0 && threadIdx.x == 0) { *a.rcount = 0; if (a.rwork) *a.rwork = 0; }   // k_sort_read's list for k_sort_radix / k_sort_big
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    __shared__ uint64_t s[SORT_SMALL];
    const uint32_t r = blockIdx.x;
    if (r >= a.n) return;
    const uint64_t base = a.a_off[r];
    const uint32_t A = (uint32_t)(a.a_off[r + 1] - base);
    if (A > a.small_max) return;
    if (threadIdx.x == 0) { a.cnt2[r] = A; a.smax[r] = 0; }   // no singleton filter for small reads
    if (A == 1 && threadIdx.x == 0) a.tmp[CK(base, a.cap_keys)] = a.keys[CK(base, a.cap_keys)];
    if (A <= 1) return;
    uint32_t np = 1; while (np < A) np <<= 1;
    uint64_t* K = a.keys;
    for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) s[i] = i < A ? K[CK(base + i, a.cap_keys)] : U64MAX;
    __syncthreads();
    if (np >= 512 && a.small_reg) {   // uniform
        if (np == 512) small_sort_reg<9>(s);
        else if (np == 1024) small_sort_reg<10>(s);
        else if (np == 2048) small_sort_reg<11>(s);
        else small_sort_reg<12>(s);
        for (uint32_t i = threadIdx.x; i < A; i += blockDim.x) a.tmp[CK(base + i, a.cap_keys)] = s[i];
        return;
    }
    // Thread t (256 threads) exchanges pairs (i, i ^ j) with i = t + 256 u, i < i ^ j.  For
    // j < 64 both elements stay with the same wave from stage to stage, for j >= 256 with the
    // same thread: only the stages j = 64 and 128 move elements between waves and need the
    // workgroup barrier (7 of the 55 stages of a 1024-key sort; the others a wave-level one).
    for (uint32_t kk = 2; kk <= np; kk <<= 1) {
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            const bool xw = j >= 64 && j < 256;
            if (xw) __syncthreads();
            for (uint32_t i = threadIdx.x; i < np; i += 256) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t x = s[i], y = s[ixj];
                    const bool up = (i & kk) == 0;
                    if ((x > y) == up) { s[i] = y; s[ixj] = x; }
                }
            }
            if (xw) __syncthreads();
            else wave_lds_sync();
        }
    }
    for (uint32_t i = threadIdx.x; i < A; i += blockDim.x) a.tmp[CK(base + i, a.cap_keys)] = s[i];   // sorted keys live in tmp
}

// ---- per-read sort of the large reads (A0 > small_max): cell buckets.
//
// Keys are (group, rpos, q).  The reference coordinate space of every group
// (forward / reverse per contig, plus the Q19 pseudo-group) is cut into 32 kb
// cells (goff: first cell of each group, a guard cell on either side).
//   P1  two LDS bitmaps over all cells: seen, seen twice.
//   KC  kept cells: seen and (seen twice or a neighbouring cell seen).  An
//       anchor in any other cell has no other anchor of its read in the same
//       group within 32 kb >= max_dist_x (both DP passes), so it is a
//       one-anchor segment of chain_dp_all (f = span, pprev = -1) and affects
//       the result only through the "last argmax f" tie-break, which then picks
//       the largest such key (k_chain_fin gets 1 + the largest dropped key).
//       Ranks of the kept cells come from a word prefix of popcounts.
//   P2  per kept cell an anchor count (u16 pairs in LDS), scanned to offsets.
//   P3  scatter of the kept anchors to T, grouped by cell in key order.
//   P4  every cell segment is sorted on its own (cells are ordered, so the
//       concatenation is the full order of src/seeds.rs:58):
//       <= 1024 anchors: one thread per anchor counts its rank inside the
//       segment (its cell rank, written beside T in P3, gives the bounds),
//       over windows of T staged in LDS and cut at segment ends;
//       larger: block-wide rank count over the LDS-staged segment, or the LSD
//       radix below for segments beyond 2048 anchors.
// Reads that do not fit (A0 > 65535, too many kept cells for the LDS budget,
// or no cell table) take the radix path over the whole read.
//
// LSD radix (fallback): 9-bit digits over the varying bits of (group, rpos);
// runs of equal (group, rpos) are then ordered by the full key.
constexpr int RS_ITEMS = 4;
constexpr int RS_CH = 1024 * RS_ITEMS;
constexpr int RS_DB = 9;                 // digit bits
constexpr int RS_ND = 1 << RS_DB;
constexpr int RS_MAXP = 5;               // digit passes: (group, rpos) has at most 7 + 31 bits
// (segments up to SortArgs::read_tiny / big_tiny keys, 16 by default, are ranked by a linear scan)
constexpr uint32_t SEG_RANK = 2048;      // up to this: block-wide rank count; beyond: radix
constexpr int BIG_MAX = 128;             // larger segments listed per read (more: radix over the read)
constexpr int GOFF_LDS = 256;            // group offsets staged in LDS when 2 * n_seq + 2 fits
constexpr int SORT_LDS = 157 * 1024;     // dynamic LDS of k_sort_read (one workgroup per CU; 2.4 KB static)
constexpr int SORT_LDS_HALF = 76 * 1024; // ... two 512-thread workgroups per CU (knob sort_lds_kb <= 76)
#ifndef SORT_U
#define SORT_U 8                          // keys per thread in flight in the block-wide passes over a read
#endif
#ifndef SORT_U1
#define SORT_U1 SORT_U                    // ... in P1 (bitmaps only: few registers per key)
#endif
#ifndef SORT_U2
#define SORT_U2 SORT_U                    // ... in P2
#endif
#ifndef SORT_UG
#define SORT_UG SORT_U                    // ... in the window gathers
#endif
#ifndef SORT_FUSE_U
#define SORT_FUSE_U 16                    // ... in the fused seeding pass (index gathers: more in flight)
#endif

// 8 independent loads per thread, then fn(i, x) for each (i < n): hides HBM
// latency in the block-wide passes of k_sort_read
template <int U = 8, int NT = 1024, typename F>
DEVI void block_pass8(const uint64_t* src, uint32_t n, F fn) {
    for (uint32_t i0 = 0; i0 < n; i0 += NT * U) {
        uint64_t x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { const uint32_t i = i0 + (uint32_t)u * NT + threadIdx.x; x[u] = i < n ? src[i] : 0; }
#pragma unroll
        for (int u = 0; u < U; ++u) { const uint32_t i = i0 + (uint32_t)u * NT + threadIdx.x; if (i < n) fn(i, x[u]); }
    }
}

// bitonic sort of one key per lane across the wave, carrying a payload
DEVI void wave_bitonic64(uint64_t& x, uint32_t& p) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint32_t yl = (uint32_t)__shfl_xor((int)(uint32_t)x, j, 64);
            const uint32_t yh = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), j, 64);
            const uint32_t q = (uint32_t)__shfl_xor((int)p, j, 64);
            const uint64_t y = ((uint64_t)yh << 32) | yl;
            const bool up = (lane & k) == 0, low = (lane & j) == 0;
            if ((low == up) ? (y < x) : (y > x)) { x = y; p = q; }
        }
    }
}

// bitonic sort of one 64-bit key per lane across the wave
DEVI void wave_bitonic64_np(uint64_t& x) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint32_t yl = (uint32_t)__shfl_xor((int)(uint32_t)x, j, 64);
            const uint32_t yh = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), j, 64);
            const uint64_t y = ((uint64_t)yh << 32) | yl;
            const bool up = (lane & k) == 0, low = (lane & j) == 0;
            if ((low == up) ? (y < x) : (y > x)) x = y;
        }
    }
}

// number of keys in the sorted S[lo, hi) of 64-bit keys below x (or <= x when
// incl), comparing only their low dwords S32[2 j] (keys that agree above them)
DEVI uint32_t count_below_lo(const uint32_t* S32, uint32_t lo, uint32_t hi, uint32_t x, bool incl) {
    uint32_t b = lo, n = hi - lo;
    while (n) {
        const uint32_t h = n >> 1;
        const uint32_t y = S32[2 * (b + h)];
        if (y < x || (incl && y == x)) { b += h + 1; n -= h + 1; } else n = h;
    }
    return b - lo;
}

// number of keys in the sorted S[lo, hi) below x (or <= x when incl)
DEVI uint32_t count_below(const uint64_t* S, uint32_t lo, uint32_t hi, uint64_t x, bool incl) {
    uint32_t b = lo, n = hi - lo;
    while (n) {
        const uint32_t h = n >> 1;
        const uint64_t y = S[b + h];
        if (y < x || (incl && y == x)) { b += h + 1; n -= h + 1; } else n = h;
    }
    return b - lo;
}

// as block_pass8 over keys and their u16 tags (loaded together): fn(i, x, m)
template <int U = 8, int NT = 1024, typename F>
DEVI void block_pass_km(const uint64_t* src, const uint16_t* tag, uint32_t n, F fn) {
    for (uint32_t i0 = 0; i0 < n; i0 += NT * U) {
        uint64_t x[U];
        uint16_t m[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + (uint32_t)u * NT + threadIdx.x;
            x[u] = i < n ? src[i] : 0;
            m[u] = i < n ? tag[i] : (uint16_t)0xffffu;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { const uint32_t i = i0 + (uint32_t)u * NT + threadIdx.x; if (i < n) fn(i, x[u], m[u]); }
    }
}

// as block_pass_km, but fn(i, x, m, valid) runs on every lane (block-uniform
// trip count) so that fn may ballot / shuffle
template <int U = 8, int NT = 1024, typename F>
DEVI void block_pass_kmu(const uint64_t* src, const uint16_t* tag, uint32_t n, F fn) {
    for (uint32_t i0 = 0; i0 < n; i0 += NT * U) {
        uint64_t x[U];
        uint16_t m[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + (uint32_t)u * NT + threadIdx.x;
            x[u] = i < n ? src[i] : 0;
            m[u] = i < n ? tag[i] : (uint16_t)0xffffu;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { const uint32_t i = i0 + (uint32_t)u * NT + threadIdx.x; fn(i, x[u], m[u], i < n); }
    }
}

// as block_pass8, but fn(i, x, valid) runs on every lane (block-uniform trip
// count) so that fn may ballot / shuffle
template <int U = 4, typename F>
DEVI void block_pass_u(const uint64_t* src, uint32_t n, F fn) {
    for (uint32_t i0 = 0; i0 < n; i0 += 1024 * U) {
        uint64_t x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { const uint32_t i = i0 + (uint32_t)u * 1024 + threadIdx.x; x[u] = i < n ? src[i] : 0; }
#pragma unroll
        for (int u = 0; u < U; ++u) { const uint32_t i = i0 + (uint32_t)u * 1024 + threadIdx.x; fn(i, x[u], i < n); }
    }
}

// the comput_sc pen LUT (n int16) into LDS in 16-B words, four in flight per
// thread: the rescue pass's LUT (bw_long + 1 = 20,001 entries, 40 KB) was 80
// dependent 2-byte load steps per thread at 256 threads (chain_seg rescue
// 0.137 -> 0.115 ms per 10 k reads, 1 stream).  Both sides hold whole 16-B
// words (LDS: lut_lds; HBM: the LUT buffer is allocated in 8-entry units).
// (No array and no conditional assignment: a conditionally assigned uint4[4]
// was put in scratch memory, and every load then made a serial HBM round trip
// through it, ~10 us at each block start of every chain kernel.)
DEVI void load_lut(int16_t* lut, const int16_t* g, int n) {
    const int nv = (n * 2 + 15) >> 4;
    const uint4* src = (const uint4*)g;
    uint4* dst = (uint4*)lut;
    const int nt = (int)blockDim.x;
    for (int i0 = (int)threadIdx.x; i0 < nv; i0 += 4 * nt) {
        const int i1 = i0 + nt < nv ? i0 + nt : i0, i2 = i0 + 2 * nt < nv ? i0 + 2 * nt : i0, i3 = i0 + 3 * nt < nv ? i0 + 3 * nt : i0;
        const uint4 v0 = src[i0], v1 = src[i1], v2 = src[i2], v3 = src[i3];
        dst[i3] = v3; dst[i2] = v2; dst[i1] = v1; dst[i0] = v0;   // clamped slots rewrite v0's word last with v0
    }
}

// exclusive scan over a block of NW waves (all threads call it: it holds barriers)
template <int NW = 16>
DEVI uint32_t block_excl_sum(uint32_t v, uint32_t& total, uint32_t* sc) {
    const int lane = lane_id(), wv = wave_id();
    uint32_t wt;
    const uint32_t ex = wave_excl_sum(v, wt);
    __syncthreads();
    if (lane == 0) sc[wv] = wt;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int t = 0; t < NW; ++t) { const uint32_t q = sc[t]; pre += t < wv ? q : 0u; tot += q; }
    total = tot;
    return pre + ex;
}

template <int NW = 16>
DEVI uint64_t block_max64(uint64_t v, uint64_t* red) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { const uint64_t o = __shfl_xor(v, d, 64); v = o > v ? o : v; }
    __syncthreads();
    if (lane_id() == 0) red[wave_id()] = v;
    __syncthreads();
    v = 0;
#pragma unroll
    for (int t = 0; t < NW; ++t) v = red[t] > v ? red[t] : v;
    return v;
}

// LSD radix of [src, src+A) by (group, rpos), ties by the full key; the sorted
// keys end in `out` (== src or dst).  dyn: (RS_MAXP + 16) * RS_ND words.
DEVI void radix_range(uint64_t* src, uint64_t* dst, uint64_t* out, uint32_t A, uint32_t qb, uint32_t* dyn, uint64_t* red) {
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    uint32_t (*hist)[RS_ND] = (uint32_t (*)[RS_ND])dyn;                   // RS_MAXP x RS_ND
    uint32_t (*wh)[RS_ND] = (uint32_t (*)[RS_ND])(dyn + RS_MAXP * RS_ND);  // 16 x RS_ND
    __syncthreads();
    for (int t = tid; t < RS_MAXP * RS_ND; t += 1024) (&hist[0][0])[t] = 0;
    // bits of (group, rpos) that vary, and all digit histograms in one pass
    uint64_t vo = 0, va = U64MAX;
    block_pass8(src, A, [&](uint32_t, uint64_t x) { const uint64_t h = x >> qb; vo |= h; va &= h; });
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { vo |= __shfl_xor(vo, d, 64); va &= __shfl_xor(va, d, 64); }
    __syncthreads();
    if (lane == 0) { red[wv] = vo; red[16 + wv] = va; }
    __syncthreads();
    vo = 0; va = U64MAX;
    for (int t = 0; t < 16; ++t) { vo |= red[t]; va &= red[16 + t]; }
    const uint64_t vary = A ? (vo ^ va) : 0;
    const int top = vary ? 64 - clz64(vary) : 0;
    const int npass = (top + RS_DB - 1) / RS_DB;
    const uint64_t dmask = (uint64_t)RS_ND - 1;
    block_pass8(src, A, [&](uint32_t, uint64_t x) {
        const uint64_t h = x >> qb;
        for (int k = 0; k < npass; ++k)
            if ((vary >> (RS_DB * k)) & dmask) atomicAdd(&hist[k][(uint32_t)(h >> (RS_DB * k)) & (uint32_t)dmask], 1u);
    });
    __syncthreads();
    if (tid < npass) {
        uint32_t run = 0;
        for (int d = 0; d < RS_ND; ++d) { const uint32_t c = hist[tid][d]; hist[tid][d] = run; run += c; }
    }
    __syncthreads();
    for (int k = 0; k < npass; ++k) {
        if (((vary >> (RS_DB * k)) & dmask) == 0) continue;       // constant digit: order unchanged
        const int sh = (int)qb + RS_DB * k;
        uint64_t x[RS_ITEMS];
        {   // first chunk
            const uint32_t w0 = (uint32_t)wv * 64 * RS_ITEMS;
#pragma unroll
            for (int it = 0; it < RS_ITEMS; ++it) { const uint32_t i = w0 + (uint32_t)it * 64 + (uint32_t)lane; x[it] = i < A ? src[i] : 0; }
        }
        for (uint32_t c0 = 0; c0 < A; c0 += RS_CH) {
            const uint32_t w0 = c0 + (uint32_t)wv * 64 * RS_ITEMS;
#pragma unroll
            for (int t0 = 0; t0 < RS_ND; t0 += 64) wh[wv][t0 + lane] = 0;
            wave_lds_sync();
#pragma unroll
            for (int it = 0; it < RS_ITEMS; ++it) {
                const uint32_t i = w0 + (uint32_t)it * 64 + (uint32_t)lane;
                if (i < A) atomicAdd(&wh[wv][(uint32_t)(x[it] >> sh) & (uint32_t)dmask], 1u);
            }
            // prefetch the next chunk while the offsets are formed
            uint64_t nx[RS_ITEMS];
            {
                const uint32_t n0 = w0 + RS_CH;
#pragma unroll
                for (int it = 0; it < RS_ITEMS; ++it) { const uint32_t i = n0 + (uint32_t)it * 64 + (uint32_t)lane; nx[it] = i < A ? src[i] : 0; }
            }
            __syncthreads();
            if (tid < RS_ND) {
                uint32_t run = hist[k][tid];
                for (int w = 0; w < 16; ++w) { const uint32_t c = wh[w][tid]; wh[w][tid] = run; run += c; }
                hist[k][tid] = run;
            }
            __syncthreads();
#pragma unroll
            for (int it = 0; it < RS_ITEMS; ++it) {
                const uint32_t i = w0 + (uint32_t)it * 64 + (uint32_t)lane;
                const bool valid = i < A;
                const uint32_t d = (uint32_t)(x[it] >> sh) & (uint32_t)dmask;
                uint64_t peers = ballot(valid);
#pragma unroll
                for (int bb = 0; bb < RS_DB; ++bb) {
                    const bool bit = (d >> bb) & 1u;
                    const uint64_t mb = ballot(bit);
                    peers &= bit ? mb : ~mb;
                }
                const uint64_t lt = peers & lanemask_lt();
                const uint32_t pos = wh[wv][d] + (uint32_t)__popcll(lt);
                if (valid) dst[CK(pos, A)] = x[it];
                wave_lds_sync();
                if (valid && lt == 0) wh[wv][d] += (uint32_t)__popcll(peers);
                wave_lds_sync();
            }
#pragma unroll
            for (int it = 0; it < RS_ITEMS; ++it) x[it] = nx[it];
            __syncthreads();
        }
        uint64_t* t = src; src = dst; dst = t;
        __syncthreads();
    }
    // sorted by (group, rpos) in src; order runs of equal (group, rpos) by the full key
    for (uint32_t i = tid; i < A; i += 1024) {
        const uint64_t h = src[i] >> qb;
        const bool start = (i == 0 || (src[i - 1] >> qb) != h) && (i + 1 < A && (src[i + 1] >> qb) == h);
        if (start) {
            uint32_t e = i + 1;
            while (e < A && (src[e] >> qb) == h) ++e;
            for (uint32_t u = i + 1; u < e; ++u) {      // insertion sort (runs are short)
                const uint64_t v = src[u];
                uint32_t w = u;
                while (w > i && src[w - 1] > v) { src[w] = src[w - 1]; --w; }
                src[w] = v;
            }
        }
    }
    __syncthreads();
    if (src != out) block_pass8(src, A, [&](uint32_t i, uint64_t x) { out[i] = x; });
    __syncthreads();
}

// ---- DPP helpers (wave scans) of the chain kernels
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
DEVI int32_t dpp(int32_t old, int32_t src) { return __builtin_amdgcn_update_dpp(old, src, CTRL, ROW_MASK, BANK_MASK, false); }
// inclusive max-scan over the wave (row_shr 1/2/4/8, row_bcast 15/31)
DEVI int32_t scan_max(int32_t v) {
    v = max(v, dpp<0x111>(INT_MIN, v)); v = max(v, dpp<0x112>(INT_MIN, v));
    v = max(v, dpp<0x114>(INT_MIN, v)); v = max(v, dpp<0x118>(INT_MIN, v));
    v = max(v, dpp<0x142, 0xa>(INT_MIN, v)); v = max(v, dpp<0x143, 0xc>(INT_MIN, v));
    return v;
}
// OR over the wave (row_shr 1/2/4/8 + row_bcast 15/31 leave the total in lane 63)
DEVI uint32_t wave_or32(uint32_t v) {
    int32_t x = (int32_t)v;
    x |= dpp<0x111>(0, x); x |= dpp<0x112>(0, x); x |= dpp<0x114>(0, x); x |= dpp<0x118>(0, x);
    x |= dpp<0x142, 0xa>(0, x); x |= dpp<0x143, 0xc>(0, x);
    return (uint32_t)__builtin_amdgcn_readlane(x, 63);
}
// lane l <- lane l-1, lane 0 <- old0 (wave_shr:1)
DEVI int32_t shr1_dpp(int32_t v, int32_t old0) { return dpp<0x138>(old0, v); }
// composition scan of x -> max(x + a, b) in lane order (earlier applied first)
DEVI void scan_nskip(int32_t& a, int32_t& b) {
    constexpr int32_t NEG = -(1 << 29);
#define NS_STEP(CTRL, RM)                                                   \
    {                                                                       \
        const int32_t oa = dpp<CTRL, RM>(0, a), ob = dpp<CTRL, RM>(NEG, b); \
        b = max(ob + a, b); a = oa + a;                                     \
    }
    NS_STEP(0x111, 0xf) NS_STEP(0x112, 0xf) NS_STEP(0x114, 0xf) NS_STEP(0x118, 0xf)
    NS_STEP(0x142, 0xa) NS_STEP(0x143, 0xc)
#undef NS_STEP
}

// the same composition scan with the additive part clamped at NEG (a chain of
// "no predecessor" steps must not overflow)
DEVI void scan_lb(int32_t& a, int32_t& b) {
    constexpr int32_t NEG = -(1 << 29);
#define LB_STEP(CTRL, RM)                                                   \
    {                                                                       \
        const int32_t oa = dpp<CTRL, RM>(0, a), ob = dpp<CTRL, RM>(NEG, b); \
        b = max(ob + a, b); a = max(oa + a, NEG);                           \
    }
    LB_STEP(0x111, 0xf) LB_STEP(0x112, 0xf) LB_STEP(0x114, 0xf) LB_STEP(0x118, 0xf)
    LB_STEP(0x142, 0xa) LB_STEP(0x143, 0xc)
#undef LB_STEP
}

// GL: the group offsets stay in HBM (2 n_seq + 2 > GOFF_LDS).  A template
// parameter rather than a pointer chosen at run time: a pointer that may be
// LDS or global compiles to flat loads, and every flat load waits for all
// outstanding global loads and stores (vmcnt(0)), which serialised P1/P2 per key.
template <bool GL, int NT>
__global__ __launch_bounds__(NT) void k_sort_read(SortArgs a) {
    constexpr int NW = NT / 64;
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    __shared__ uint64_t red[32];
    __shared__ uint32_t s_sc[16], s_kept, s_nbig;
    __shared__ uint2 s_big[BIG_MAX];
    __shared__ uint32_t s_goff[GOFF_LDS];
    extern __shared__ uint64_t dyn64[];
    uint32_t* dyn = (uint32_t*)dyn64;
    if (blockIdx.x >= a.n) return;
    const uint32_t r = a.order ? a.order[blockIdx.x] : blockIdx.x;   // heaviest reads first
    const uint64_t base = a.a_off[r];
    const uint32_t A0 = (uint32_t)(a.a_off[r + 1] - base);
    if (A0 <= a.small_max) return;    // k_sort_small
#ifdef MM2G_CHECKED
    if (base + A0 > a.cap_keys) { if (threadIdx.x == 0) CK(base + A0, a.cap_keys); return; }
#endif
    const int tid = threadIdx.x, lane = lane_id();
    // MM2G_KNOB_SORT_PROF: per-phase wall-clock sums of thread 0 (after barriers),
    // accumulated in the read's 16 profile words (no registers held across the kernel)
    uint64_t* const pq = a.prof ? a.prof + (uint64_t)r * 24 : nullptr;
    if (pq && tid == 0) pq[10] = pq[12] = wall_clock64();
#define SORT_PH(k) do { if (pq && tid == 0) { const uint64_t t_ = wall_clock64(); pq[k] += t_ - pq[12]; pq[12] = t_; } } while (0)
#define SORT_END(nb, nk) do { if (pq && tid == 0) { pq[8] = A0; pq[9] = ((uint64_t)(nb) << 32) | (nk); pq[11] = wall_clock64(); } } while (0)
    const uint32_t qb = a.qb, gsh = a.qb + a.rb;
    const uint64_t rmask = (1ULL << a.rb) - 1;
    uint64_t* K = a.keys + base;      // unsorted anchors (seed_write); scratch once read for the last time
    uint64_t* O = a.tmp + base;       // sorted output
    const bool filt = a.cells != 0;
    const uint32_t ng = 2u * a.n_seq + 2u;
    if (!GL && filt) {
        for (uint32_t i = tid; i < ng && i < (uint32_t)GOFF_LDS; i += NT) s_goff[i] = a.goff[i];
    }
    if (tid == 0) { s_nbig = 0; s_kept = 0; }
    __syncthreads();
    // cell of a key (every group incl. the Q19 pseudo-group 2 * n_seq has cells)
    auto cell_of = [&](uint64_t x) -> uint32_t {
        const uint32_t g = (uint32_t)(x >> gsh);
        return (GL ? a.goff[g] : s_goff[g]) + 1u + (uint32_t)(((x >> qb) & rmask) >> CELL_SHIFT);
    };
    const uint32_t nw = (a.cells + 31) >> 5;
    const uint32_t LW = a.lds_words;
    uint32_t* B1 = dyn;
    uint32_t* B2 = dyn + nw;
    // reads the cell path does not take are listed for k_sort_radix (whole-read radix)
    auto defer = [&]() { if (tid == 0) { a.rlist[atomicAdd(a.rcount, 1u)] = r; SORT_END(0xffffu, 0u); } };
    if (!filt || A0 > 65535u) { defer(); return; }
    {
        // ---- P1: seen / seen-twice bitmaps
        for (uint32_t i = tid; i < 2 * nw; i += NT) dyn[i] = 0;
        const uint32_t fm = a.fuse_mmax ? a.mz_cnt[r] : 0u;
        if (a.fuse_mmax && fm <= a.fuse_mmax) {
            // fused seeding: k_seed_write skipped this read, so P1 makes its keys (push_anchor,
            // seeds.rs:62-79) in k_seed_write's order (minimizer order, then index position
            // order) from the read's minimizers staged above the bitmaps, writes them to K for
            // P2 and the windows, and sets the bitmaps on the way (no HBM read of K here)
            uint32_t* Mi = dyn + 2 * nw;           // inclusive anchor offsets (searched)
            uint32_t* Mp = Mi + fm;                // index position offsets
            uint32_t* My = Mp + fm;                // query y
            uint32_t* Mh = My + fm;                // raw n (IX_INLINE | position high word for a Single)
            const uint64_t mb = a.mz_base[r];
            if (tid == 0 && a.abort) {             // status words 7 / 14: anchors and minimizers seeded here (bench pricing)
                atomicAdd((unsigned long long*)a.abort + 7, (unsigned long long)A0);
                atomicAdd((unsigned long long*)a.abort + 14, (unsigned long long)fm);
            }
            uint32_t carry = 0;
            constexpr int FS = 2;   // minimizers per thread per step (a 10 kb read's ~1.8 k in one step)
            for (uint32_t i0 = 0; i0 < fm; i0 += NT * FS) {
                uint32_t nraw[FS], po[FS], yy[FS], cs = 0;
#pragma unroll
                for (int j = 0; j < FS; ++j) {
                    const uint32_t i = i0 + (uint32_t)tid * FS + (uint32_t)j;
                    const bool v = i < fm;
                    nraw[j] = v ? a.mz_n[mb + i] : 0u;
                    po[j] = v ? a.mz_poff[mb + i] : 0u; yy[j] = v ? a.mz_y[mb + i] : 0u;
                }
#pragma unroll
                for (int j = 0; j < FS; ++j) cs += ix_count(nraw[j]);
                uint32_t tot;
                uint32_t run = carry + block_excl_sum<NW>(cs, tot, s_sc);
#pragma unroll
                for (int j = 0; j < FS; ++j) {
                    const uint32_t i = i0 + (uint32_t)tid * FS + (uint32_t)j;
                    run += ix_count(nraw[j]);
                    if (i < fm) { Mi[i] = run; Mp[i] = po[j]; My[i] = yy[j]; Mh[i] = nraw[j]; }
                }
                carry += tot;
            }
            __syncthreads();
            // owner of key 16 b (where each key's search starts; its owner lies between that and
            // the owner of key 16 (b + 1), usually the same or the next non-empty minimizer)
            uint16_t* O16 = (uint16_t*)(Mh + fm);
            const uint32_t nb16 = (A0 + 15) >> 4;
            for (uint32_t i = tid; i < fm; i += NT) {
                const uint32_t lo = i ? Mi[i - 1] : 0u, hi = Mi[i];
                for (uint32_t b = (lo + 15) >> 4; (b << 4) < hi; ++b) O16[b] = (uint16_t)i;
            }
            __syncthreads();
            SORT_PH(3);   // MM2G_KNOB_SORT_PROF "fuse_stage": the minimizer staging (the rest of P1 counts as p1)
            const int32_t qlen = (int32_t)(a.rd_off[r + 1] - a.rd_off[r]);
            constexpr int FU = SORT_FUSE_U;
            for (uint32_t i0 = 0; i0 < A0; i0 += NT * FU) {
                uint32_t lo[FU], hi[FU];
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    const uint32_t t = i0 + (uint32_t)u * NT + tid, b = t < A0 ? t >> 4 : 0u;
                    lo[u] = O16[b];
                    hi[u] = t >= A0 ? lo[u] : (b + 1 < nb16 ? (uint32_t)O16[b + 1] : fm - 1);
                }
                // first minimizer from lo with inclusive offset > t (all lanes' searches step together)
                while (true) {
                    bool act = false;
#pragma unroll
                    for (int u = 0; u < FU; ++u) {
                        if (lo[u] < hi[u]) {
                            const uint32_t t = i0 + (uint32_t)u * NT + tid, mid = (lo[u] + hi[u]) >> 1;
                            if (Mi[mid] > t) hi[u] = mid; else lo[u] = mid + 1;
                            act |= lo[u] < hi[u];
                        }
                    }
                    if (!any(act)) break;
                }
                uint64_t x[FU];
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    const uint32_t t = i0 + (uint32_t)u * NT + tid;
                    x[u] = 0;
                    if (t < A0) {
                        const uint32_t ow = lo[u];
                        const uint32_t h = Mh[ow], exo = ow ? Mi[ow - 1] : 0u;
                        x[u] = (h & IX_INLINE) ? ((uint64_t)(h & ~IX_INLINE) << 32) | Mp[ow]   // Single: no gather
                                               : a.ix_pos[CK((uint64_t)Mp[ow] + (t - exo), a.cap_pos)];
                    }
                }
                uint32_t c[FU];
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    const uint32_t t = i0 + (uint32_t)u * NT + tid;
                    x[u] = pack_anchor(x[u], My[lo[u]], qlen, a.span, a.kl);
                    if (t < A0) K[t] = x[u];
                    c[u] = cell_of(x[u]);
                }
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    const uint32_t t = i0 + (uint32_t)u * NT + tid;
                    lo[u] = t < A0 ? atomicOr(&B1[c[u] >> 5], 1u << (c[u] & 31)) : 0u;   // (lo: the old words)
                }
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    const uint32_t t = i0 + (uint32_t)u * NT + tid, bit = 1u << (c[u] & 31);
                    if (t < A0 && (lo[u] & bit)) atomicOr(&B2[c[u] >> 5], bit);
                }
            }
        } else {
        __syncthreads();
        // staged per group of SORT_U1 keys: all cells, then all first atomics
        // (LDS round trips overlap instead of one chain per key)
        for (uint32_t i0 = 0; i0 < A0; i0 += NT * SORT_U1) {
            uint64_t x[SORT_U1];
            uint32_t c[SORT_U1], old[SORT_U1];
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) { const uint32_t i = i0 + (uint32_t)u * NT + tid; x[u] = i < A0 ? K[i] : 0; }
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) c[u] = cell_of(x[u]);
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) {
                const uint32_t i = i0 + (uint32_t)u * NT + tid;
                old[u] = i < A0 ? atomicOr(&B1[c[u] >> 5], 1u << (c[u] & 31)) : 0u;
            }
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) {
                const uint32_t i = i0 + (uint32_t)u * NT + tid, bit = 1u << (c[u] & 31);
                if (i < A0 && (old[u] & bit)) atomicOr(&B2[c[u] >> 5], bit);   // seen before: seen twice
            }
        }
        }
        __syncthreads();
        // ---- KC (in place of B2) and the word prefix of its popcounts (in place of B1)
        const uint32_t per = (nw + NT - 1) / NT;
        const uint32_t wa = min(nw, (uint32_t)tid * per), wb = min(nw, wa + per);
        uint32_t loc = 0;
        for (uint32_t w = wa; w < wb; ++w) {
            const uint32_t b1 = B1[w];
            const uint32_t nb = (b1 << 1) | (w ? B1[w - 1] >> 31 : 0u) | (b1 >> 1) | (w + 1 < nw ? B1[w + 1] << 31 : 0u);
            const uint32_t kc = b1 & (B2[w] | nb);
            B2[w] = kc;
            loc += (uint32_t)__popc(kc);
        }
        uint32_t nkc;
        uint32_t run = block_excl_sum<NW>(loc, nkc, s_sc);      // its barriers end the B1 reads
        for (uint32_t w = wa; w < wb; ++w) { B1[w] = run; run += (uint32_t)__popc(B2[w]); }
        SORT_PH(0);
        if (pq && tid == 0) pq[13] = nkc;
        const uint32_t cw = (nkc + 1) >> 1;                  // u16 counts, two per word
        // C (u16 per kept cell) sits at the top of the LDS.  The bitmaps are dead
        // after P2 (the tags and the window keys carry the ranks), so the windows
        // use everything below C.  Window keys carry their kept-cell rank in the
        // top 16 bits, which the key layout must leave free.
        const uint32_t cofs = LW >= cw + 2 ? (LW - cw) & ~1u : 0u;
        const uint32_t kbits = gsh + (32u - (uint32_t)__builtin_clz(2u * a.n_seq | 1u));
        const uint32_t W = cofs >> 1;                        // keys per window
        if (kbits > 48u || qb + CELL_SHIFT > 32u || cofs < 2 * nw || W < SEG_RANK) { defer(); return; }
        {
            constexpr uint64_t kmask = (1ULL << 48) - 1;
            uint32_t* C = dyn + cofs;
            uint64_t* S = dyn64;
            for (uint32_t i = tid; i < cw; i += NT) C[i] = 0;
            __syncthreads();
            auto c16 = [&](uint32_t rk) -> uint32_t { return (C[rk >> 1] >> ((rk & 1) << 4)) & 0xffffu; };
            // ---- P2: counts per kept cell; the largest dropped key.  Each key's
            // kept-cell rank (0xffff = dropped) goes to the u16 tag array T16 in
            // the DP's f buffer, so the window passes need no cell lookups (and
            // the bitmaps can be overwritten by the first window).
            uint64_t smx = 0;
            uint16_t* T16 = (uint16_t*)(a.meta + base);
            // staged like P1: all cells, all bitmap reads, then counts and tags
            for (uint32_t i0 = 0; i0 < A0; i0 += NT * SORT_U2) {
                uint64_t x[SORT_U2];
                uint32_t c[SORT_U2], kw[SORT_U2], pw[SORT_U2];
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) { const uint32_t i = i0 + (uint32_t)u * NT + tid; x[u] = i < A0 ? K[i] : 0; }
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) c[u] = cell_of(x[u]);
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) { kw[u] = B2[c[u] >> 5]; pw[u] = B1[c[u] >> 5]; }
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) {
                    const uint32_t i = i0 + (uint32_t)u * NT + tid;
                    if (i < A0) {
                        const uint32_t b = c[u] & 31;
                        const bool kept = (kw[u] >> b) & 1u;
                        const uint32_t rk = pw[u] + (uint32_t)__popc(kw[u] & ((1u << b) - 1u));
                        if (kept) atomicAdd(&C[rk >> 1], 1u << ((rk & 1) << 4));
                        else smx = x[u] + 1 > smx ? x[u] + 1 : smx;
                        T16[i] = kept ? (uint16_t)rk : (uint16_t)0xffffu;
                    }
                }
            }
            smx = block_max64<NW>(smx, red);               // (its barriers also end the count atomics)
            // exclusive scan of the u16 counts, in place (offsets < A0 <= 65535)
            const uint32_t per2 = (cw + NT - 1) / NT;
            const uint32_t ca = min(cw, (uint32_t)tid * per2), cb = min(cw, ca + per2);
            uint32_t l2 = 0;
            for (uint32_t i = ca; i < cb; ++i) { const uint32_t v = C[i]; l2 += (v & 0xffffu) + (v >> 16); }
            uint32_t A;
            uint32_t o = block_excl_sum<NW>(l2, A, s_sc);
            for (uint32_t i = ca; i < cb; ++i) {
                const uint32_t v = C[i], lo = v & 0xffffu;
                C[i] = o | ((o + lo) << 16);
                o += lo + (v >> 16);
            }
            if (tid == 0) { a.cnt2[r] = A; a.smax[r] = smx; }
            __syncthreads();
            SORT_PH(1);
            // ---- P3/P4: windows of whole kept cells (<= W keys), each gathered from K
            // into LDS by cell (C turns from start into end offsets as cells are
            // filled), chunk-sorted and ranked per cell segment into O.
            auto offx = [&](uint32_t rk) -> uint32_t { return rk < nkc ? c16(rk) : A; };   // start of an unfilled cell
            uint32_t ra = 0;
            while (ra < nkc) {
                const uint32_t oa = c16(ra);
                uint32_t lo = ra + 1, hi = nkc;                       // last rb with offx(rb) <= oa + W
                while (lo < hi) { const uint32_t mid = (lo + hi + 1) >> 1; if (offx(mid) <= oa + W) lo = mid; else hi = mid - 1; }
                const uint32_t rb = lo;
                const uint32_t ob = offx(rb);
                if (ob > oa + W) {
                    // cell ra alone exceeds the window: gather it into O unsorted (P4b sorts it)
                    __syncthreads();
                    if (tid == 0) s_kept = 0;
                    __syncthreads();
                    block_pass_kmu<8, NT>(K, T16, A0, [&](uint32_t, uint64_t x, uint16_t m, bool valid) {
                        const bool mine = valid && (uint32_t)m == ra;
                        const uint64_t mb = ballot(mine);
                        uint32_t wb0 = 0;
                        if (lane == 0 && mb) wb0 = atomicAdd(&s_kept, (uint32_t)__popcll(mb));
                        wb0 = (uint32_t)__shfl((int)wb0, 0, 64);
                        if (mine) O[CK(oa + wb0 + (uint32_t)__popcll(mb & lanemask_lt()), A0)] = x;
                    });
                    __syncthreads();
                    if (tid == 0) {
                        const uint32_t sh = (ra & 1) << 4;
                        C[ra >> 1] = (C[ra >> 1] & ~(0xffffu << sh)) | (ob << sh);   // now its end offset
                        const uint32_t slot = s_nbig++;
                        if (slot < (uint32_t)BIG_MAX) s_big[slot] = make_uint2(oa, ob);
                    }
                    __syncthreads();
                    SORT_PH(2);
                    ra = ra + 1;
                    continue;
                }
                const uint32_t nwin = ob - oa;
                __syncthreads();
                // window keys carry their rank in the top 16 bits: the rank rises
                // with the key, so the order is unchanged, and a key's segment is
                // one shift away
                block_pass_km<SORT_UG, NT>(K, T16, A0, [&](uint32_t, uint64_t x, uint16_t m) {
                    const uint32_t rk = m;
                    if (m != 0xffffu && rk >= ra && rk < rb) {
                        const uint32_t sh = (rk & 1) << 4;
                        const uint32_t pos = ((atomicAdd(&C[rk >> 1], 1u << sh) >> sh) & 0xffffu) - oa;
                        S[pos] = x | ((uint64_t)rk << 48);
                    }
                });
                __syncthreads();
                SORT_PH(2);
                if (pq && tid == 0) pq[7] += 1;
                // segment [s, e) of a key, window-relative (C holds end offsets for ranks < rb)
                auto seg_of = [&](uint64_t x, uint32_t& s, uint32_t& e) {
                    const uint32_t rk = (uint32_t)(x >> 48);
                    s = (rk ? c16(rk - 1) : 0u) - oa;
                    e = c16(rk) - oa;
                };
                // A: chunks holding a segment longer than SEG_TINY: one wave sorts 64 keys
                const uint32_t nch = (nwin + 63) >> 6;
                for (uint32_t q = (uint32_t)wave_id(); q < nch; q += 2 * NW) {   // two chunks at a time (q, q + NW)
                    const uint32_t ia = q * 64 + (uint32_t)lane, ib = ia + NW * 64;
                    const bool va = ia < nwin, vb = ib < nwin;
                    uint64_t xa = S[va ? ia : 0], xb = S[vb ? ib : 0];
                    uint32_t sa, ea, sb, eb;
                    seg_of(xa, sa, ea);
                    seg_of(xb, sb, eb);
                    xa = va ? xa : U64MAX; xb = vb ? xb : U64MAX;
                    const bool na = any(va && ea - sa > a.read_tiny && ea - sa <= a.seg_small);
                    const bool nb = any(vb && eb - sb > a.read_tiny && eb - sb <= a.seg_small);
                    if (na) { wave_bitonic64_np(xa); if (va) S[ia] = xa; }
                    if (nb) { wave_bitonic64_np(xb); if (vb) S[ib] = xb; }
                }
                __syncthreads();
                SORT_PH(4);
                // B: ranks inside the segments.  Keys of one segment share every bit
                // above the cell-local lb <= 32 (rank, group, cell), so they compare
                // by their low dwords.
                // Each key leaves for its place in O directly (measured against a
                // permutation in LDS with whole-line writes: slower)
                const uint32_t* S32 = (const uint32_t*)S;
                uint32_t pc_tiny = 0, pc_long = 0, pc_srch = 0;     // MM2G_KNOB_SORT_PROF segment classes
                for (uint32_t i = tid; i < nwin; i += NT) {
                    const uint64_t x = S[i];
                    uint32_t s, e;
                    seg_of(x, s, e);
                    const uint32_t L = e - s;
                    if (L > a.seg_small) {             // P4b; copied unsorted
                        O[oa + i] = x & kmask;
                        if (i == s) {
                            const uint32_t slot = atomicAdd(&s_nbig, 1u);
                            if (slot < (uint32_t)BIG_MAX) s_big[slot] = make_uint2(oa + s, oa + e);
                        }
                        continue;
                    }
                    const uint32_t xl = (uint32_t)x;
                    uint32_t rank = 0;
                    if (pq) {
                        if (L <= a.read_tiny) ++pc_tiny;
                        else if (L > 64) { ++pc_long; pc_srch += ((e - 1) >> 6) - (s >> 6); }
                    }
                    if (L <= a.read_tiny) {
                        for (uint32_t j = s; j < e; ++j) { const uint32_t y = S32[2 * j]; rank += (y < xl || (y == xl && j < i)) ? 1u : 0u; }
                    } else {
                        const uint32_t co = i >> 6;
                        rank = i - max(s, co << 6);
                        for (uint32_t c = s >> 6; c <= (e - 1) >> 6; ++c) {
                            if (c == co) continue;
                            rank += count_below_lo(S32, max(s, c << 6), min(e, (c << 6) + 64), xl, c < co);
                        }
                    }
                    O[oa + s + rank] = x & kmask;
                }
                if (pq) {
                    const uint64_t v14 = wave_sum64(((uint64_t)pc_long << 32) | pc_tiny), v15 = wave_sum64(pc_srch);
                    if (lane == 0) { atomicAdd((unsigned long long*)&pq[14], (unsigned long long)v14); atomicAdd((unsigned long long*)&pq[15], (unsigned long long)v15); }
                }
                __syncthreads();
                SORT_PH(5);
                ra = rb;
            }
            // ---- P4b: cells over seg_small, one at a time by the whole block (K is scratch now)
            const uint32_t nbig = s_nbig;
            bool big_radix = nbig > (uint32_t)BIG_MAX;
            for (uint32_t b = 0; b < nbig && !big_radix; ++b) big_radix = s_big[b].y - s_big[b].x > SEG_RANK;
            if (big_radix) { defer(); return; }       // K is still intact: k_sort_radix redoes the read
            {
                for (uint32_t b = 0; b < nbig; ++b) {
                    const uint2 sg = s_big[b];
                    const uint32_t L = sg.y - sg.x;
                    if (L <= SEG_RANK) {
                        __syncthreads();
                        block_pass8<4, NT>(O + sg.x, L, [&](uint32_t i, uint64_t x) { dyn64[i] = x; });
                        __syncthreads();
                        constexpr int KPT = (int)SEG_RANK / NT;   // keys per thread
                        uint64_t xk[KPT];
                        uint32_t rk[KPT];
#pragma unroll
                        for (int u = 0; u < KPT; ++u) { const uint32_t iu = (uint32_t)tid + (uint32_t)u * NT; xk[u] = iu < L ? dyn64[iu] : U64MAX; rk[u] = 0; }
                        const int nu = (int)((L + NT - 1) / NT);
                        for (uint32_t j = 0; j < L; ++j) {
                            const uint64_t y = dyn64[j];
#pragma unroll
                            for (int u = 0; u < KPT; ++u) {
                                const uint32_t iu = (uint32_t)tid + (uint32_t)u * NT;
                                if (u < nu) rk[u] += (y < xk[u] || (y == xk[u] && j < iu)) ? 1u : 0u;
                            }
                        }
                        __syncthreads();
#pragma unroll
                        for (int u = 0; u < KPT; ++u) { const uint32_t iu = (uint32_t)tid + (uint32_t)u * NT; if (iu < L) O[sg.x + rk[u]] = xk[u]; }
                    }
                }
            }
            SORT_PH(6);
            SORT_END(nbig, A);
            return;
        }
    }
#undef SORT_PH
#undef SORT_END
}

// Whole-read LSD radix for the reads k_sort_read listed (A0 > 65535, no cell
// table, a key layout the 32-bit windows cannot hold, too many kept cells for
// the LDS, or cell segments beyond SEG_RANK), with the bitmap singleton filter
// when cells exist.  One workgroup per listed read (grid-stride over the list).
template <bool GL>   // as k_sort_read: group offsets in HBM (true) or LDS, never a flat pointer
__global__ __launch_bounds__(1024) void k_sort_radix(SortArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;
    __shared__ uint64_t red[32];
    __shared__ uint32_t s_kept;
    __shared__ uint32_t s_goff[GOFF_LDS];
    extern __shared__ uint64_t dyn64[];
    uint32_t* dyn = (uint32_t*)dyn64;
    const int tid = threadIdx.x, lane = lane_id();
    const uint32_t nlist = *a.rcount;
    const uint32_t qb = a.qb, gsh = a.qb + a.rb;
    const uint64_t rmask = (1ULL << a.rb) - 1;
    const bool filt = a.cells != 0;
    const uint32_t ng = 2u * a.n_seq + 2u;
    if (!GL && filt) {
        for (uint32_t i = tid; i < ng && i < (uint32_t)GOFF_LDS; i += 1024) s_goff[i] = a.goff[i];
    }
    auto cell_of = [&](uint64_t x) -> uint32_t {
        const uint32_t g = (uint32_t)(x >> gsh);
        return (GL ? a.goff[g] : s_goff[g]) + 1u + (uint32_t)(((x >> qb) & rmask) >> CELL_SHIFT);
    };
    const uint32_t nw = (a.cells + 31) >> 5;
    uint32_t* B1 = dyn;
    uint32_t* B2 = dyn + nw;
    for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
        const uint32_t r = a.rlist[li];
        const uint64_t base = a.a_off[r];
        const uint32_t A0 = (uint32_t)(a.a_off[r + 1] - base);
        uint64_t* K = a.keys + base;
        uint64_t* O = a.tmp + base;
        uint64_t* src = K;
        uint64_t* dst = O;
        uint32_t A = A0;
        uint64_t smx = 0;     // 1 + largest dropped key
        __syncthreads();
        if (filt) {
            if (tid == 0) s_kept = 0;
            for (uint32_t i = tid; i < 2 * nw; i += 1024) dyn[i] = 0;
            __syncthreads();
            block_pass8<4>(K, A0, [&](uint32_t, uint64_t x) {
                const uint32_t c = cell_of(x);
                const uint32_t bit = 1u << (c & 31);
                if (atomicOr(&B1[c >> 5], bit) & bit) atomicOr(&B2[c >> 5], bit);
            });
            __syncthreads();
            // keep non-singletons (compacted into O, order irrelevant: sorted below)
            block_pass_u<4>(K, A0, [&](uint32_t, uint64_t x, bool valid) {
                bool keep = false;
                if (valid) {
                    const uint32_t c = cell_of(x);
                    const bool twice = (B2[c >> 5] >> (c & 31)) & 1u;
                    const bool left = (B1[(c - 1) >> 5] >> ((c - 1) & 31)) & 1u;
                    const bool right = (B1[(c + 1) >> 5] >> ((c + 1) & 31)) & 1u;
                    keep = twice || left || right;
                    if (!keep) smx = x + 1 > smx ? x + 1 : smx;
                }
                const uint64_t km = ballot(keep);
                uint32_t wbase = 0;
                if (lane == 0 && km) wbase = atomicAdd(&s_kept, (uint32_t)__popcll(km));
                wbase = (uint32_t)__shfl((int)wbase, 0, 64);
                if (keep) O[CK(wbase + (uint32_t)__popcll(km & lanemask_lt()), A0)] = x;
            });
            smx = block_max64(smx, red);
            A = s_kept;
            src = O; dst = K;
            __syncthreads();
        }
        if (tid == 0) { a.cnt2[r] = A; a.smax[r] = smx; }
        radix_range(src, dst, O, A, qb, dyn, red);
    }
}

// inclusive max-scan over a 1024-thread block (all threads call it: it holds barriers)
DEVI uint32_t block_incl_max(uint32_t v, uint32_t* sc) {
    const int lane = lane_id(), wv = wave_id();
    uint32_t x = wave_incl_scan(v, [](uint32_t p, uint32_t q) { return p > q ? p : q; });
    __syncthreads();
    if (lane == 63) sc[wv] = x;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int t = 0; t < 16; ++t) { const uint32_t q = sc[t]; pre = (t < wv && q > pre) ? q : pre; }
    return x > pre ? x : pre;
}
// inclusive min-scan over a 1024-thread block
DEVI uint32_t block_incl_min(uint32_t v, uint32_t* sc) {
    const int lane = lane_id(), wv = wave_id();
    uint32_t x = wave_incl_scan(v, [](uint32_t p, uint32_t q) { return p < q ? p : q; });
    __syncthreads();
    if (lane == 63) sc[wv] = x;
    __syncthreads();
    uint32_t pre = 0xffffffffu;
#pragma unroll
    for (int t = 0; t < 16; ++t) { const uint32_t q = sc[t]; pre = (t < wv && q < pre) ? q : pre; }
    return x < pre ? x : pre;
}

// ---- large reads: every read k_sort_read lists while the singleton filter is
// on (A0 > 65535 -- the 100 kb reads of C5 --, key layouts over 48 bits, more
// kept cells or bigger cell segments than its LDS windows hold).  Cell buckets
// through HBM instead of one LDS window pass per window over the whole read:
//   P1/KC  as k_sort_read: seen / seen-twice bitmaps, kept cells, their ranks.
//   P2     counts per bucket of 2^bsh consecutive kept cells (u32, top of the
//          LDS; bsh is the smallest shift that gives <= BIG_NB_MAX buckets) and
//          the largest dropped key; scanned to bucket starts.
//   P3     scatter of the kept keys to O by bucket (LDS atomics hand out the
//          slots).  A bucket is a union of whole cells, so bucket order is key
//          order: O then holds every bucket in place, each one unsorted.
//   P4     windows of whole buckets (<= W keys), read from O into LDS in one
//          coalesced pass: every 64-key chunk is sorted by a wave (a chunk that
//          spans buckets keeps each bucket in its slot range, since all keys of
//          bucket b are below bucket b+1's); a key's rank inside its bucket is
//          its chunk position plus a binary search per other chunk of the
//          bucket (<= 16 keys: a direct count).  Bucket bounds of a slot come
//          from a bucket-start bitmap and its word-level max / min scans.  The
//          window is written back in place.
//   big    buckets over SEG_RANK keys: the LSD radix on their HBM range (K is
//          scratch once P3 has read it).
// Traffic per key: 8 B (P1) + 8 (P2) + 16 (P3) + 16 (P4) = 48 B, against
// ~9 passes of the whole-read radix.  One block per listed read, taken from a
// work counter (the list is roughly heaviest first: k_sort_read defers in its
// heaviest-first order).
constexpr uint32_t BIG_NB_MAX = 16384;
constexpr int BIG_WND = 126;                      // windows appended to by k_sort_big's P3 (more: per-key scatter)
constexpr uint32_t BIG_WREG = 3 * BIG_WND + 4;   // LDS words of their bounds, starts and cursors (below the bucket counts)
// k_sort_big / k_sort_read keep both cell bitmaps (2 x MAX_CELLS bits) plus the
// bucket counts in SORT_LDS; `LW - 2 * nw - 64` below is unsigned
static_assert(SORT_LDS / 4 > 2 * (MAX_CELLS / 32) + 64 + 4096, "MAX_CELLS bitmaps must leave LDS for the bucket counts");
template <bool GL>
__global__ __launch_bounds__(1024) void k_sort_big(SortArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;
    __shared__ uint64_t red[32];
    __shared__ uint32_t s_sc[16], s_read, s_nbig;
    __shared__ uint2 s_big[BIG_MAX];
    __shared__ uint32_t s_goff[GOFF_LDS];
    extern __shared__ uint64_t dyn64[];
    uint32_t* dyn = (uint32_t*)dyn64;
    const int tid = threadIdx.x, lane = lane_id();
    const uint32_t nlist = *a.rcount;
    const uint32_t qb = a.qb, gsh = a.qb + a.rb;
    const uint64_t rmask = (1ULL << a.rb) - 1;
    const uint32_t ng = 2u * a.n_seq + 2u;
    if (!GL) {
        for (uint32_t i = tid; i < ng && i < (uint32_t)GOFF_LDS; i += 1024) s_goff[i] = a.goff[i];
    }
    auto cell_of = [&](uint64_t x) -> uint32_t {
        const uint32_t g = (uint32_t)(x >> gsh);
        return (GL ? a.goff[g] : s_goff[g]) + 1u + (uint32_t)(((x >> qb) & rmask) >> CELL_SHIFT);
    };
    const uint32_t nw = (a.cells + 31) >> 5;
    const uint32_t LW = a.lds_words;
    uint32_t* B1 = dyn;
    uint32_t* B2 = dyn + nw;
    for (;;) {
        __syncthreads();
        if (tid == 0) s_read = atomicAdd(a.rwork, 1u);
        __syncthreads();
        const uint32_t li = (uint32_t)uni((int32_t)s_read);
        if (li >= nlist) break;
        const uint32_t r = a.rlist[li];
        const uint64_t base = a.a_off[r];
        const uint32_t A0 = (uint32_t)(a.a_off[r + 1] - base);
        uint64_t* K = a.keys + base;
        uint64_t* O = a.tmp + base;
        uint64_t* const pq = a.prof ? a.prof + (uint64_t)r * 24 : nullptr;
        if (pq && tid == 0) pq[10] = pq[12] = wall_clock64();
#define BIG_PH(k) do { if (pq && tid == 0) { const uint64_t t_ = wall_clock64(); pq[k] += t_ - pq[12]; pq[12] = t_; } } while (0)
        // ---- P1: seen / seen-twice bitmaps (staged: all cells, then all atomics)
        for (uint32_t i = tid; i < 2 * nw; i += 1024) dyn[i] = 0;
        __syncthreads();
        if (a.fuse_big && A0 > 65535u) {
            // fused seeding: k_seed_write skipped this read, so P1 makes its keys (push_anchor,
            // seeds.rs:62-79) as k_seed_write would: wave w takes part w of the read's 64-minimizer
            // chunks (k_seed_count's part starts), stages each chunk's offsets above the bitmaps,
            // gathers the positions, writes the keys to K for P2 / P3 and sets the bitmaps
            static_assert(SEED_PARTS == 16, "a wave per part, 16 per 1024-thread workgroup");
            const int wv = wave_id();
            uint32_t* Wi = dyn + 2 * nw + (uint32_t)wv * 256;   // inclusive offsets, then poff, y, raw n
            uint32_t* Wp = Wi + 64;
            uint32_t* Wy = Wp + 64;
            uint32_t* Wh = Wy + 64;
            const uint64_t mb = a.mz_base[r];
            const uint32_t m = a.mz_cnt[r];
            const uint32_t nch = (m + 63) >> 6;
            const uint32_t cb = (nch * (uint32_t)wv) / SEED_PARTS, ce = (nch * (uint32_t)(wv + 1)) / SEED_PARTS;
            const uint32_t cend = ce * 64 < m ? ce * 64 : m;
            const int32_t qlen = (int32_t)(a.rd_off[r + 1] - a.rd_off[r]);
            uint32_t run = wv ? a.a_part[(uint64_t)r * (SEED_PARTS - 1) + (uint32_t)wv - 1] : 0u;
            if (tid == 0 && a.abort) {             // status words 15 / 16: anchors and minimizers seeded here (bench pricing)
                atomicAdd((unsigned long long*)a.abort + 15, (unsigned long long)A0);
                atomicAdd((unsigned long long*)a.abort + 16, (unsigned long long)m);
            }
            constexpr int U = 8;
            for (uint32_t c0 = cb * 64; c0 < cend; c0 += 64) {
                const uint32_t i = c0 + (uint32_t)lane;
                const bool vi = i < m;
                const uint32_t nraw = vi ? a.mz_n[mb + i] : 0u;
                const uint32_t n = ix_count(nraw);
                uint32_t tot;
                const uint32_t ex = wave_excl_sum(n, tot);
                Wi[lane] = ex + n; Wp[lane] = vi ? a.mz_poff[mb + i] : 0u; Wy[lane] = vi ? a.mz_y[mb + i] : 0u; Wh[lane] = nraw;
                wave_lds_sync();
                for (uint32_t tb = 0; tb < tot; tb += 64 * U) {
                    uint64_t x[U];
                    uint32_t own[U], c[U], old[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t t = tb + (uint32_t)u * 64 + (uint32_t)lane;
                        x[u] = 0; own[u] = 0;
                        if (t < tot) {
                            uint32_t lo = 0;   // owner: the number of inclusive offsets <= t
#pragma unroll
                            for (uint32_t step = 32; step >= 1; step >>= 1)
                                if (Wi[lo + step - 1] <= t) lo += step;
                            const uint32_t exo = lo ? Wi[lo - 1] : 0u, h = Wh[lo];
                            own[u] = lo;
                            x[u] = (h & IX_INLINE) ? ((uint64_t)(h & ~IX_INLINE) << 32) | Wp[lo]   // Single: no gather
                                                   : a.ix_pos[CK((uint64_t)Wp[lo] + (t - exo), a.cap_pos)];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t t = tb + (uint32_t)u * 64 + (uint32_t)lane;
                        x[u] = pack_anchor(x[u], Wy[own[u]], qlen, a.span, a.kl);
                        if (t < tot) K[CK(run + t, A0)] = x[u];
                        c[u] = cell_of(x[u]);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t t = tb + (uint32_t)u * 64 + (uint32_t)lane;
                        old[u] = t < tot ? atomicOr(&B1[c[u] >> 5], 1u << (c[u] & 31)) : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t t = tb + (uint32_t)u * 64 + (uint32_t)lane, bit = 1u << (c[u] & 31);
                        if (t < tot && (old[u] & bit)) atomicOr(&B2[c[u] >> 5], bit);
                    }
                }
                run += tot;
                wave_lds_sync();
            }
        } else
        for (uint32_t i0 = 0; i0 < A0; i0 += 1024 * SORT_U1) {
            uint64_t x[SORT_U1];
            uint32_t c[SORT_U1], old[SORT_U1];
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) { const uint32_t i = i0 + (uint32_t)u * 1024 + tid; x[u] = i < A0 ? K[i] : 0; }
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) c[u] = cell_of(x[u]);
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) {
                const uint32_t i = i0 + (uint32_t)u * 1024 + tid;
                old[u] = i < A0 ? atomicOr(&B1[c[u] >> 5], 1u << (c[u] & 31)) : 0u;
            }
#pragma unroll
            for (int u = 0; u < SORT_U1; ++u) {
                const uint32_t i = i0 + (uint32_t)u * 1024 + tid, bit = 1u << (c[u] & 31);
                if (i < A0 && (old[u] & bit)) atomicOr(&B2[c[u] >> 5], bit);
            }
        }
        __syncthreads();
        // ---- KC (in place of B2) and the word prefix of its popcounts (in place of B1)
        const uint32_t per = (nw + 1023) >> 10;
        const uint32_t wa = min(nw, (uint32_t)tid * per), wb = min(nw, wa + per);
        uint32_t loc = 0;
        for (uint32_t w = wa; w < wb; ++w) {
            const uint32_t b1 = B1[w];
            const uint32_t nb = (b1 << 1) | (w ? B1[w - 1] >> 31 : 0u) | (b1 >> 1) | (w + 1 < nw ? B1[w + 1] << 31 : 0u);
            const uint32_t kc = b1 & (B2[w] | nb);
            B2[w] = kc;
            loc += (uint32_t)__popc(kc);
        }
        uint32_t nkc;
        uint32_t run = block_excl_sum(loc, nkc, s_sc);
        for (uint32_t w = wa; w < wb; ++w) { B1[w] = run; run += (uint32_t)__popc(B2[w]); }
        BIG_PH(0);
        if (pq && tid == 0) pq[13] = nkc;
        // buckets of 2^bsh kept cells; their counts (then ends) CNT[0..NB] at the top of the LDS
        const uint32_t nbmax = min(BIG_NB_MAX, LW - 2 * nw - 64 - BIG_WREG);
        uint32_t bsh = 0;
        while (((nkc + (1u << bsh) - 1) >> bsh) > nbmax) ++bsh;
        const uint32_t NB = (nkc + (1u << bsh) - 1) >> bsh;
        const uint32_t cofs = (LW - NB - 1) & ~1u;
        uint32_t* CNT = dyn + cofs;
        for (uint32_t i = tid; i <= NB; i += 1024) CNT[i] = 0;
        __syncthreads();
        // ---- P2: counts per bucket, the largest dropped key
        uint64_t smx = 0;
        for (uint32_t i0 = 0; i0 < A0; i0 += 1024 * SORT_U2) {
            uint64_t x[SORT_U2];
            uint32_t c[SORT_U2], kw[SORT_U2], pw[SORT_U2];
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) { const uint32_t i = i0 + (uint32_t)u * 1024 + tid; x[u] = i < A0 ? K[i] : 0; }
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) c[u] = cell_of(x[u]);
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) { kw[u] = B2[c[u] >> 5]; pw[u] = B1[c[u] >> 5]; }
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) {
                const uint32_t i = i0 + (uint32_t)u * 1024 + tid;
                if (i < A0) {
                    const uint32_t b = c[u] & 31;
                    if ((kw[u] >> b) & 1u) atomicAdd(&CNT[(pw[u] + (uint32_t)__popc(kw[u] & ((1u << b) - 1u))) >> bsh], 1u);
                    else smx = x[u] + 1 > smx ? x[u] + 1 : smx;
                }
            }
        }
        smx = block_max64(smx, red);               // (its barriers also end the count atomics)
        // exclusive scan of the counts in place: CNT[b] = start of bucket b
        const uint32_t per2 = (NB + 1023) >> 10;
        const uint32_t ca = min(NB, (uint32_t)tid * per2), cb = min(NB, ca + per2);
        uint32_t l2 = 0;
        for (uint32_t i = ca; i < cb; ++i) l2 += CNT[i];
        uint32_t A;
        uint32_t o = block_excl_sum(l2, A, s_sc);
        for (uint32_t i = ca; i < cb; ++i) { const uint32_t v = CNT[i]; CNT[i] = o; o += v; }
        if (tid == 0) { a.cnt2[r] = A; a.smax[r] = smx; s_nbig = 0; }
        __syncthreads();
        BIG_PH(1);
        // ---- windows of whole buckets (<= W keys; a bucket over W alone is radix-sorted in
        // HBM), fixed before P3 from the bucket starts.  P3 then appends every kept key to its
        // window's range of O (a few append streams per read, so the writes fill whole lines)
        // with its bucket inside the window as a u16 tag, and each window gathers its keys by
        // bucket into LDS.  (Round 4's P3 scattered each key straight to its bucket slot: a
        // partial line per key, 470 us of a C5 read's 1400; measured: P3 473 -> 268 us per
        // read.  Tagging the kept cell instead, with a count pass per window so the segments
        // are single cells, measured slower: 10.7 against 10.0 ms per C5 batch.)  More than
        // BIG_WND windows: that per-key scatter.  WB / WC / WS sit just below CNT.
        uint32_t* WB = dyn + cofs - BIG_WREG;      // window w = buckets [WB[w], WB[w + 1])
        uint32_t* WC = WB + BIG_WND + 1;           // P3 append cursors
        uint32_t* WS = WC + BIG_WND;               // window starts in O (WS[nwnd] = A)
        const uint32_t W = (((cofs - BIG_WREG - 16) * 32u) / 67u) & ~63u;
        auto bstart0 = [&](uint32_t b) -> uint32_t { return b < NB ? CNT[b] : A; };   // bucket starts (before P4)
        if (tid == 0) {
            uint32_t nwnd = 0, ba = 0;
            while (ba < NB && nwnd < min(a.big_wnd, (uint32_t)BIG_WND)) {
                const uint32_t oa = bstart0(ba);
                uint32_t lo = ba + 1, hi = NB;                  // last bb with bstart0(bb) <= oa + W
                while (lo < hi) { const uint32_t mid = (lo + hi + 1) >> 1; if (bstart0(mid) - oa <= W) lo = mid; else hi = mid - 1; }
                WB[nwnd] = ba; WS[nwnd] = oa; WC[nwnd] = oa;
                ++nwnd;
                ba = lo;
            }
            WB[nwnd] = ba; WS[nwnd] = A;
            s_read = ba == NB ? nwnd : 0u;                      // 0: too many windows
        }
        __syncthreads();
        const uint32_t nwnd = s_read;
        uint16_t* T16 = (uint16_t*)(a.meta + base);
        if (nwnd) {
            uint32_t wpw = 1;
            while (wpw * 2 <= nwnd) wpw *= 2;
            for (uint32_t i0 = 0; i0 < A0; i0 += 1024 * SORT_U2) {
                uint64_t x[SORT_U2];
                uint32_t c[SORT_U2], kw[SORT_U2], pw[SORT_U2];
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) { const uint32_t i = i0 + (uint32_t)u * 1024 + tid; x[u] = i < A0 ? K[i] : 0; }
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) c[u] = cell_of(x[u]);
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) { kw[u] = B2[c[u] >> 5]; pw[u] = B1[c[u] >> 5]; }
#pragma unroll
                for (int u = 0; u < SORT_U2; ++u) {
                    const uint32_t i = i0 + (uint32_t)u * 1024 + tid;
                    const uint32_t b = c[u] & 31;
                    const bool kept = i < A0 && ((kw[u] >> b) & 1u);
                    const uint32_t bk = kept ? (pw[u] + (uint32_t)__popc(kw[u] & ((1u << b) - 1u))) >> bsh : 0u;
                    uint32_t wd = 0;                                 // last window with WB[wd] <= bk
                    for (uint32_t st = wpw; st; st >>= 1) if (wd + st < nwnd && WB[wd + st] <= bk) wd += st;
                    // lanes of one window take consecutive slots: one LDS atomic per window per wave
                    uint64_t peers = ballot(kept);
                    for (uint32_t bit = 1; bit < nwnd; bit <<= 1) {
                        const bool on = (wd & bit) != 0;
                        const uint64_t m = ballot(on);
                        peers &= on ? m : ~m;
                    }
                    const uint64_t lt = peers & lanemask_lt();
                    uint32_t slot = 0;
                    if (kept && lt == 0) slot = atomicAdd(&WC[wd], (uint32_t)__popcll(peers));
                    const int leader = kept ? (int)__builtin_ctzll(peers) : lane;
                    slot = (uint32_t)__shfl((int)slot, leader, 64) + (uint32_t)__popcll(lt);
                    if (kept) { O[CK(slot, A0)] = x[u]; T16[CK(slot, A0)] = (uint16_t)(bk - WB[wd]); }
                }
            }
        } else {
        // ---- P3 (more than BIG_WND windows): scatter of the kept keys by bucket; CNT[b] turns into bucket b's end
        for (uint32_t i0 = 0; i0 < A0; i0 += 1024 * SORT_U2) {
            uint64_t x[SORT_U2];
            uint32_t c[SORT_U2], kw[SORT_U2], pw[SORT_U2];
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) { const uint32_t i = i0 + (uint32_t)u * 1024 + tid; x[u] = i < A0 ? K[i] : 0; }
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) c[u] = cell_of(x[u]);
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) { kw[u] = B2[c[u] >> 5]; pw[u] = B1[c[u] >> 5]; }
#pragma unroll
            for (int u = 0; u < SORT_U2; ++u) {
                const uint32_t i = i0 + (uint32_t)u * 1024 + tid;
                const uint32_t b = c[u] & 31;
                if (i < A0 && ((kw[u] >> b) & 1u)) {
                    const uint32_t bk = (pw[u] + (uint32_t)__popc(kw[u] & ((1u << b) - 1u))) >> bsh;
                    O[CK(atomicAdd(&CNT[bk], 1u), A0)] = x[u];
                }
            }
        }
        }
        __syncthreads();
        BIG_PH(2);
        // ---- P4: windows.  LDS below WB: S[W] keys, then the segment-start bitmap SB
        // and its word scans LS / NS (W/32 + 2 words each).
        auto bstart = [&](uint32_t b) -> uint32_t { return b ? CNT[b - 1] : 0u; };   // (fallback: bucket ends)
        uint64_t* S = dyn64;
        uint32_t* SB = dyn + 2 * W;
        uint32_t* LS = SB + (W >> 5) + 2;
        uint32_t* NS = LS + (W >> 5) + 2;
        auto radix_big = [&](uint32_t s0, uint32_t e0) {   // block-wide; keys of O[s0, e0) sorted in place
            __syncthreads();
            radix_range(O + s0, K + s0, O + s0, e0 - s0, qb, dyn, red);
        };
        uint32_t ba = 0, wi = 0;
        while (ba < NB) {
            uint32_t bb, oa, nwin;
            if (nwnd) {
                bb = WB[wi + 1];
                oa = WS[wi];
                const uint32_t oe = WS[wi + 1];
                ++wi;
                if (bb == ba + 1 && oe - oa > W) {             // one bucket beyond a window: radix in HBM
                    radix_big(oa, oe);
                    __syncthreads();
                    if (tid == 0) CNT[ba] = oe;                // its end, for the next window's bstart
                    if (pq && tid == 0) pq[7] += 1;
                    ba = bb;
                    continue;
                }
                nwin = oe - oa;
                __syncthreads();
                // the window's keys by bucket into LDS; CNT[b] (its start) turns into bucket b's end
                block_pass_km<SORT_UG>(O + oa, T16 + oa, nwin, [&](uint32_t, uint64_t x, uint16_t m) {
                    S[atomicAdd(&CNT[ba + (uint32_t)m], 1u) - oa] = x;
                });
                const uint32_t nwd0 = (nwin + 31) >> 5;
                for (uint32_t q = tid; q < nwd0; q += 1024) SB[q] = 0;
                __syncthreads();
                for (uint32_t b = ba + tid; b < bb; b += 1024) { const uint32_t p = bstart(b) - oa; atomicOr(&SB[p >> 5], 1u << (p & 31)); }
                __syncthreads();
            } else {
                oa = bstart(ba);
                if (CNT[ba] - oa > W) {                 // one bucket beyond a window: radix in HBM
                    radix_big(oa, CNT[ba]);
                    if (pq && tid == 0) pq[7] += 1;
                    ba = ba + 1;
                    continue;
                }
                uint32_t lo = ba + 1, hi = NB;          // last bb with bstart(bb) <= oa + W
                while (lo < hi) { const uint32_t mid = (lo + hi + 1) >> 1; if (bstart(mid) - oa <= W) lo = mid; else hi = mid - 1; }
                bb = lo;
                nwin = bstart(bb) - oa;
                __syncthreads();
                block_pass8<SORT_UG>(O + oa, nwin, [&](uint32_t i, uint64_t x) { S[i] = x; });
                const uint32_t nwd0 = (nwin + 31) >> 5;
                for (uint32_t q = tid; q < nwd0; q += 1024) SB[q] = 0;
                __syncthreads();
                for (uint32_t b = ba + tid; b < bb; b += 1024) { const uint32_t p = bstart(b) - oa; atomicOr(&SB[p >> 5], 1u << (p & 31)); }
                __syncthreads();
            }
            const uint32_t nwd = (nwin + 31) >> 5;
            // LS[q]: last bucket start in words <= q; NS[q]: first bucket start in words >= q (NS[nwd] = nwin)
            for (uint32_t q0 = 0; q0 < nwd; q0 += 1024) {
                const uint32_t q = q0 + tid;
                const uint32_t m = q < nwd ? SB[q] : 0u;
                uint32_t v = m ? q * 32 + 31 - (uint32_t)__builtin_clz(m) : 0u;
                v = block_incl_max(v, s_sc);
                const uint32_t carry = q0 ? LS[q0 - 1] : 0u;
                if (q < nwd) LS[q] = v > carry ? v : carry;
                __syncthreads();
            }
            for (uint32_t q0 = 0; q0 < nwd; q0 += 1024) {      // suffix min, from the end
                const uint32_t q = nwd - 1 - (q0 + tid);
                const bool ok = q0 + tid < nwd;
                const uint32_t m = ok ? SB[q] : 0u;
                uint32_t v = m ? q * 32 + (uint32_t)__builtin_ctz(m) : nwin;
                v = block_incl_min(v, s_sc);
                const uint32_t carry = q0 ? NS[nwd - q0] : nwin;
                if (ok) NS[q] = v < carry ? v : carry;
                __syncthreads();
            }
            if (tid == 0) NS[nwd] = nwin;
            __syncthreads();
            auto seg_of = [&](uint32_t i, uint32_t& s0, uint32_t& e0) {
                const uint32_t q = i >> 5, bi = i & 31;
                const uint32_t m = SB[q];
                const uint32_t le = bi == 31 ? 0xffffffffu : ((2u << bi) - 1u);
                const uint32_t lo_m = m & le, hi_m = m & ~le;
                s0 = lo_m ? q * 32 + 31 - (uint32_t)__builtin_clz(lo_m) : LS[q ? q - 1 : 0];
                e0 = hi_m ? q * 32 + (uint32_t)__builtin_ctz(hi_m) : NS[q + 1];
            };
            // A: sort every 64-key chunk holding a bucket of 17..SEG_RANK keys
            const uint32_t nch = (nwin + 63) >> 6;
            for (uint32_t q = (uint32_t)wave_id(); q < nch; q += 16) {
                const uint32_t i = q * 64 + (uint32_t)lane;
                const bool v = i < nwin;
                uint32_t s0 = 0, e0 = 0;
                if (v) seg_of(i, s0, e0);
                if (any(v && e0 - s0 > a.big_tiny && e0 - s0 <= SEG_RANK)) {
                    uint64_t x = v ? S[i] : U64MAX;
                    wave_bitonic64_np(x);
                    if (v) S[i] = x;
                }
            }
            __syncthreads();
            BIG_PH(4);
            // B: ranks inside the buckets, written back in place; buckets over
            // SEG_RANK keys go back unsorted and are radix-sorted below
            for (uint32_t i = tid; i < nwin; i += 1024) {
                const uint64_t x = S[i];
                uint32_t s0, e0;
                seg_of(i, s0, e0);
                const uint32_t L = e0 - s0;
                if (L > SEG_RANK) {
                    O[oa + i] = x;
                    if (i == s0) { const uint32_t slot = atomicAdd(&s_nbig, 1u); if (slot < (uint32_t)BIG_MAX) s_big[slot] = make_uint2(oa + s0, oa + e0); }
                    continue;
                }
                uint32_t rank = 0;
                if (L <= a.big_tiny) {
                    for (uint32_t j = s0; j < e0; ++j) { const uint64_t y = S[j]; rank += (y < x || (y == x && j < i)) ? 1u : 0u; }
                } else {
                    const uint32_t co = i >> 6;
                    rank = i - max(s0, co << 6);
                    for (uint32_t c = s0 >> 6; c <= (e0 - 1) >> 6; ++c) {
                        if (c == co) continue;
                        rank += count_below(S, max(s0, c << 6), min(e0, (c << 6) + 64), x, c < co);
                    }
                }
                O[oa + s0 + rank] = x;
            }
            __syncthreads();
            BIG_PH(5);
            if (pq && tid == 0) pq[7] += 1;
            // a window holds fewer than W / SEG_RANK such buckets (<= BIG_MAX)
            const uint32_t nbig = s_nbig;
            for (uint32_t t = 0; t < nbig; ++t) radix_big(s_big[t].x, s_big[t].y);
            __syncthreads();
            if (tid == 0) s_nbig = 0;
            BIG_PH(6);
            ba = bb;
        }
        if (pq && tid == 0) { pq[8] = A0; pq[9] = (0xfffeULL << 32) | A; pq[11] = wall_clock64(); }
#undef BIG_PH
    }
}

// ============================================================================
// 5. CHAIN DP — chain_dp_all (src/lchain.rs:59-91) + the fallback chain
// (lchain.rs:162-173) + chain_qrange/trange (178-200) + the rescue test of
// rescue_long_join (316-330).
//
// One wave per read; anchors are taken in blocks of 64.
//   isolated  anchor i has no candidate predecessor (st(i) == i) iff i == 0,
//             or i-1 lies in another (rid, strand) group, or
//             rpos_i > rpos_{i-1} + max_dist_x (keys are sorted by group and
//             rpos, so i-1 is the closest candidate).  Then the reference's
//             j-loop is empty: f = span, pprev = -1, no marks.  A ballot
//             finds these per block and resolves them in bulk.
//   others    sequential, in order.  For each i the j-loop runs 64
//             predecessors per step (lane l <-> j = jtop - l, the reference's
//             processing order):
//     valid_j   comput_sc (lchain.rs:17-34) with the integer pen LUT (DESIGN Q6)
//     marks     t[pprev[j]] = i  -> one bit in an LDS ring (targets >= lo only)
//     max_f     strict '>' => exclusive prefix-max (DPP scan) seeded with max_f
//     n_skip    ops x->max(x-1,0) | x->x+1 | id compose as x->max(x+a,b):
//               DPP scan only when some lane is a '+1'; break = first '+1'
//               lane with n_skip > max_skip
// The newest RK anchors (key, f, pprev) live in a per-wave LDS ring; older
// predecessors (deep windows) are read from HBM, where f/pprev are flushed at
// the end of every block.  Keys are prefetched one block ahead.
// ============================================================================
constexpr int DP_NW = 4;          // waves per workgroup
constexpr int RING_WORDS = 256;   // 8192-bit mark ring (max_iter <= 8000)
constexpr int RK = 256;           // anchor ring entries per wave (power of two, >= 256)
static_assert((RK & (RK - 1)) == 0 && RK >= 256, "anchor ring size");

constexpr uint32_t LSEG_DONE = 0x80000000u;   // lseg[].w bit: handled by k_chain_giant (low 31 bits: its wall-clock
                                              // ticks under MM2G_LSEG_PROF; k_chain_long's own ticks otherwise)
constexpr int TINY = CHAIN_TINY;  // segments up to this many anchors: one lane, registers
constexpr int MED = CHAIN_MED;    // up to this many: one lane, state machine over HBM; longer: whole wave

// "last argmax" merge: larger f wins, ties go to the larger index (lchain.rs:162-167)
DEVI void best_merge(int32_t& bf, int32_t& bi, int32_t f, int32_t i) {
    if (f > bf || (f == bf && i > bi)) { bf = f; bi = i; }
}

constexpr int KRING = 512;        // per-wave LDS ring of the newest anchor keys (k_chain_seg)
constexpr int TQ = 128;           // per-wave LDS queue per tiny length class (2 | 3-4 | 5-8 anchors)
constexpr int MEDB = 128;         // per-wave LDS buffer of medium segments before the global append
constexpr int64_t EST_LANE = 2048;   // estimated DP pairs above which a segment goes to a whole wave (debug mode)
// Production (a.est_lane, knobs med_pairs / med_pairs_rescue, both 0): every
// segment over TINY anchors goes to a wave.  One lane walks its segment with a
// dependent HBM round trip per step: k_chain_med took ~0.3 ms per 10 k reads
// (1 stream) in each pass whatever its work (6.9 k rescued anchors as much as
// 0.8 M pass-0 anchors), set by its slowest lane; k_chain_long absorbs the
// same segments for +0.08 ms (pass 0) and +0.00 ms (rescue).

// Scalar chain_dp_all (lchain.rs:73-90) of one segment of <= TINY anchors held
// in registers (keys from the wave's LDS key ring); `act` lanes only.  Local indices; marks t[pprev[j]] = i are a
// per-i bitmask (t is only ever compared with the current i).
template <int N>
DEVI void tiny_segment_dp(bool act, int32_t len, const uint64_t* kring, int32_t s, int32_t* F, int32_t* PP, const int16_t* lut,
                          const ChainKParams& P, uint32_t qb, uint64_t qmask, uint64_t rmask, int32_t& bf, int32_t& bi,
                          uint64_t& pairs) {
    int32_t pp_[N], qq_[N], f_[N], pv_[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
        const uint64_t k = (act && m < len) ? kring[(s + m) & (KRING - 1)] : 0;
        pp_[m] = (int32_t)((k >> qb) & rmask); qq_[m] = (int32_t)(k & qmask);
        f_[m] = P.span; pv_[m] = -1;
    }
    const int32_t maxdx = P.max_dist_x, maxdy = P.max_dist_y, bw = P.bw, span = P.span;
    int32_t st = 0;
    uint32_t npairs = 0;
#pragma unroll
    for (int i = 1; i < N; ++i) {
        const bool ai = act && i < len;
        // st (lchain.rs:75); every anchor of the segment is in i's group
#pragma unroll
        for (int m = 0; m < i; ++m)
            if (st == m && pp_[i] > (int32_t)((uint32_t)pp_[m] + (uint32_t)maxdx)) st = m + 1;
        const int32_t lo = st > i - P.max_iter ? st : i - P.max_iter;
        int32_t max_f = span, max_j = -1, n_skip = 0;
        uint32_t marks = 0;
        bool brk = !ai;
#pragma unroll
        for (int j = i - 1; j >= 0; --j) {
            if (!brk && j >= lo) {
                ++npairs;
                const int32_t dq = qq_[i] - qq_[j], dr = pp_[i] - pp_[j];
                bool ok = dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy;
                const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
                ok = ok && dd <= bw;
                if (ok) {
                    const int32_t dg = dr < dq ? dr : dq;
                    const int32_t sv = (span < dg ? span : dg) - (int32_t)lut[dd] + f_[j];
                    if (sv > max_f) { max_f = sv; max_j = j; if (n_skip > 0) --n_skip; }
                    else if ((marks >> j) & 1u) { ++n_skip; if (n_skip > P.max_skip) brk = true; }
                    if (!brk && pv_[j] >= 0) marks |= 1u << pv_[j];
                }
            }
        }
        if (ai) { f_[i] = max_f; pv_[i] = max_j; }
    }
#pragma unroll
    for (int m = 0; m < N; ++m)
        if (act && m < len) {
            F[s + m] = f_[m];
            PP[s + m] = pv_[m] >= 0 ? s + pv_[m] : -1;
            best_merge(bf, bi, f_[m], s + m);
        }
    pairs += npairs;
}

// packed "last argmax" key: larger f first, then larger index (lchain.rs:162-167)
DEVI unsigned long long best_key(int32_t f, int32_t i) {
    return ((unsigned long long)((uint32_t)f ^ 0x80000000u) << 32) | (uint32_t)i;
}

// ---- work items of the streaming chain kernels: reads in `order` (heaviest
// first) cut into chunks of SEG_CHUNK anchors, so that several waves share a
// heavy read (k_chain_lb, k_chain_seg).  In the rescue pass only rescued reads
// have items.  item_off[t] = first item of order[t]; item_off[n] = total.
// The first kernel of each chain pass also clears the pass's state (no
// separate memset launches): the per-read best keys, its long/medium segment
// queue counters, the k_seg_cands item counter, the LB buffer when asked
// (zero_fmin), and in pass 0 the k_chain_giant hand-out counters.
__global__ __launch_bounds__(1024) void k_seg_items(ChainArgs a) {
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    if (tid == 0) {
        *a.lseg_n = 0; *a.mseg_n = 0; *a.mseg_take = 0;
        if (a.sq_n) *a.sq_n = 0;
        if (a.P.pass == 0 && a.work) { a.work[0] = 0; a.work[1] = 0; a.work[2] = 0; a.work[3] = 0; }
    }
    for (uint32_t t = (uint32_t)tid; t < a.n; t += 1024) {
        a.rbest[t] = 0ULL;
        if (a.zero_fmin) a.fmin[t] = 0;
    }
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    __shared__ uint32_t sc[16];
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < a.n; t0 += 1024) {
        const uint32_t t = t0 + (uint32_t)tid;
        uint32_t c = 0;
        if (t < a.n) {
            const uint32_t r = a.order[t];
            const bool on = a.P.pass == 0 || (a.out[r].flags & RF_RESCUED);
            c = !on ? 0u : (a.cnt2[r] + a.seg_chunk - 1) / a.seg_chunk;   // seg_chunk-anchor chunks
        }
        uint32_t wt;
        const uint32_t ex = wave_excl_sum(c, wt);
        if (lane == 0) sc[wv] = wt;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < 16; ++w) { pre += w < wv ? sc[w] : 0u; tot += sc[w]; }
        if (t < a.n) a.item_off[t] = carry + pre + ex;
        // item -> position in order, so the streaming kernels need no search over item_off
        if (a.item_read && t < a.n) {
            const uint32_t o = carry + pre + ex;
            for (uint32_t j = 0; j < c && o + j < a.item_cap; ++j) a.item_read[o + j] = t;
        }
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) a.item_off[a.n] = carry;
    if (a.bsum) {   // the batch sums of k_batch_sums (minimizers, anchors in the DP)
        __shared__ unsigned long long ws[2][16];
        unsigned long long v[2] = {0, 0};
        for (uint32_t i = (uint32_t)tid; i < a.n; i += 1024) { v[0] += a.mz_cnt[i]; v[1] += a.cnt2[i]; }
#pragma unroll
        for (int q = 0; q < 2; ++q) { v[q] = wave_sum64(v[q]); if (lane == 0) ws[q][wv] = v[q]; }
        __syncthreads();
        if (tid < 2) {
            unsigned long long x = 0;
            for (int t = 0; t < 16; ++t) x += ws[tid][t];
            a.bsum[3 + tid] = x;
        }
    }
}

// item -> (position in order, chunk): last t with item_off[t] <= it
DEVI uint32_t item_owner(const uint32_t* item_off, uint32_t n, uint32_t it) {
    uint32_t lo = 0, hi = n;          // item_off[lo] <= it < item_off[hi]
    while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (item_off[mid] <= it) lo = mid; else hi = mid; }
    return lo;
}

// ---- 5a. per read, one streaming pass over the sorted anchors: isolated
// anchors (st(i) == i: i == 0, another (rid, strand) group than i-1, or
// rpos_i > rpos_{i-1} + max_dist_x) delimit independent segments — the DP of
// a segment never reads outside it (DESIGN.md "Chain DP").  Completed
// segments queue in LDS; per batch of 64, tiny ones run one-per-lane in
// registers (keys from the LDS key ring), the others are routed by their
// estimated pair count to k_chain_med (one lane each) or k_chain_long (one
// wave each).  The read's best (last argmax f) is merged with a packed
// 64-bit atomicMax.
__global__ __launch_bounds__(DP_NW * 64) void k_chain_seg(ChainArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    extern __shared__ __align__(16) unsigned char smem[];
    const ChainKParams P = a.P;
    int16_t* lut = (int16_t*)smem;
    const int lut_bytes = ((P.lut_n * 2) + 15) & ~15;
    uint64_t* krings = (uint64_t*)(smem + lut_bytes);
    int32_t* tqs = (int32_t*)(krings + DP_NW * KRING);          // 3 classes x TQ segment starts
    uint8_t* tls = (uint8_t*)(tqs + DP_NW * 3 * TQ);            // their lengths
    int2* medbs = (int2*)(tls + DP_NW * 3 * TQ);
    if (blockIdx.x * DP_NW >= (a.sq ? min(*a.sq_n, a.sq_cap) : (uint32_t)a.item_off[a.n])) return;   // no work item for this workgroup: skip the LUT load
    load_lut(lut, a.lut, P.lut_n);
    __syncthreads();
    const int lane = lane_id(), wv = wave_id();
    uint64_t* kring = krings + wv * KRING;
    int32_t* tq = tqs + wv * 3 * TQ;
    uint8_t* tl = tls + wv * 3 * TQ;
    int2* medb = medbs + wv * MEDB;
    const uint32_t qb = a.kl.qb, rb = a.kl.rb;
    const uint64_t qmask = (1ULL << qb) - 1, rmask = (1ULL << rb) - 1;
    const uint32_t gsh = rb + qb;
    const int32_t maxdx = P.max_dist_x, span = P.span;
    // Static, wave-uniform assignment of work items: chunks of SEG_CHUNK anchors
    // of the reads in `order` (heaviest first).  A wave starts its chunk at the
    // first isolated anchor at or after c0 and finishes the segment open at c1.
    const uint32_t nwaves = gridDim.x * DP_NW;
    const uint32_t n_items = a.sq ? min((uint32_t)uni((int32_t)*a.sq_n), a.sq_cap) : (uint32_t)uni((int32_t)a.item_off[a.n]);
    for (uint32_t it = blockIdx.x * DP_NW + wv; it < n_items; it += nwaves) {
        uint32_t r, j, t = 0xffffffffu;
        if (a.sq) {   // pass 0 with k_seg_cands: only the reads it left to streaming, (read, chunk) per item
            const uint2 q = a.sq[it];
            r = (uint32_t)uni((int32_t)q.x); j = (uint32_t)uni((int32_t)q.y);
        } else {
            t = (uint32_t)uni((int32_t)((a.item_read && it < a.item_cap) ? a.item_read[it] : item_owner(a.item_off, a.n, it)));
            r = (uint32_t)uni((int32_t)a.order[t]);
            j = it - (uint32_t)uni((int32_t)a.item_off[t]);
        }
        const uint64_t t_start = wall_clock64();
        if (t < (uint32_t)a.n_prio) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(0);
        const uint64_t base = uni64(a.a_off[r]);
        const int32_t c0 = (int32_t)j * (int32_t)a.seg_chunk;
        const int32_t A = (int32_t)uni((int32_t)a.cnt2[r]);      // anchors kept by the singleton filter
        const int32_t c1 = min(A, c0 + (int32_t)a.seg_chunk);
        if (c0 >= A) continue;
#ifdef MM2G_CHECKED
        if (base + (uint64_t)A > a.cap_keys) { if (lane == 0) CK(base + A, a.cap_keys); continue; }
#endif
        const uint64_t* K = a.keys + base;
        int32_t* F = a.f + base; int32_t* PP = a.pp + base;
        uint64_t pairs = 0;
        uint32_t n_big = 0;
        int32_t max_seg = 0;
        const int32_t fm = a.fmin ? uni(a.fmin[r]) : 0;   // segments with len * span < fm are skipped
        if (lane == 0 && a.seg_streamed) atomicAdd(a.seg_streamed, (unsigned long long)(c1 - c0));
        int32_t bf = INT_MIN, bi = -1;      // per-lane best (singletons and tiny segments)
        int32_t pend = -1;                  // start of the open segment
        int32_t th0 = 0, th1 = 0, th2 = 0, tt0 = 0, tt1 = 0, tt2 = 0;   // tiny class queue heads / tails
        int32_t nmb = 0;                    // medium buffer fill (uniform)
        // one batch of a tiny class queue (cls 0: 2 anchors, 1: 3-4, 2: 5-8)
        auto tiny_batch = [&](int cls, int32_t& h, int32_t cnt) {
            const bool vs = lane < cnt;
            const int slot = cls * TQ + ((h + lane) & (TQ - 1));
            const int32_t s0 = vs ? tq[slot] : 0;
            const int32_t len = vs ? (int32_t)tl[slot] : 0;
            if (cls == 0) tiny_segment_dp<2>(vs, len, kring, s0, F, PP, lut, P, qb, qmask, rmask, bf, bi, pairs);
            else if (cls == 1) tiny_segment_dp<4>(vs, len, kring, s0, F, PP, lut, P, qb, qmask, rmask, bf, bi, pairs);
            else tiny_segment_dp<8>(vs, len, kring, s0, F, PP, lut, P, qb, qmask, rmask, bf, bi, pairs);
            h += cnt;
            wave_lds_sync();
        };
        // medium buffer -> global queue for k_chain_med (one atomic per 64)
        auto flush_med = [&](int32_t cnt) {
            uint32_t q0 = 0;
            if (lane == 0) q0 = atomicAdd(a.mseg_n, (uint32_t)cnt);
            q0 = (uint32_t)uni((int32_t)q0);
            if (lane < cnt) {
                const int2 m = medb[lane];
                const uint32_t q = q0 + (uint32_t)lane;
                if (q < a.mseg_cap) a.mseg[q] = make_uint4(r, (uint32_t)m.x, (uint32_t)m.y, 0u);
            }
            wave_lds_sync();
            const int2 rest = (lane + 64 < MEDB) ? medb[lane + 64] : make_int2(0, 0);
            wave_lds_sync();
            if (lane + 64 < MEDB) medb[lane] = rest;
            nmb -= cnt;
            wave_lds_sync();
        };
        // route completed segments [sl, el) of the emitting lanes
        auto route = [&](bool emit, int32_t sl, int32_t el) {
            const int32_t len = el - sl;
            emit = emit && (int64_t)len * span >= (int64_t)fm;   // pruned: cannot hold the read's best f
            if (!any(emit)) return;                               // nothing to route (the usual case when pruning)
            if (emit && len == 1) { F[sl] = span; PP[sl] = -1; best_merge(bf, bi, span, sl); }
            const bool c0 = emit && len == 2, c1 = emit && len >= 3 && len <= 4, c2 = emit && len >= 5 && len <= TINY;
            const uint64_t m0 = ballot(c0), m1 = ballot(c1), m2 = ballot(c2);
            const uint64_t lt = lanemask_lt();
            if (c0) { const int sl0 = 0 * TQ + ((tt0 + __popcll(m0 & lt)) & (TQ - 1)); tq[sl0] = sl; tl[sl0] = (uint8_t)len; }
            if (c1) { const int sl1 = 1 * TQ + ((tt1 + __popcll(m1 & lt)) & (TQ - 1)); tq[sl1] = sl; tl[sl1] = (uint8_t)len; }
            if (c2) { const int sl2 = 2 * TQ + ((tt2 + __popcll(m2 & lt)) & (TQ - 1)); tq[sl2] = sl; tl[sl2] = (uint8_t)len; }
            tt0 += __popcll(m0); tt1 += __popcll(m1); tt2 += __popcll(m2);
            // longer: by estimated pairs (len x expected window) to one lane or one wave
            bool med = false;
            if (emit && len > TINY && len <= MED) {
                const int32_t p0 = (int32_t)((kring[sl & (KRING - 1)] >> qb) & rmask);
                const int32_t p1 = (int32_t)((kring[(el - 1) & (KRING - 1)] >> qb) & rmask);
                const int64_t bp = p1 - p0 > 0 ? (int64_t)(p1 - p0) : 1;
                int64_t win = ((int64_t)len * maxdx + bp - 1) / bp;
                win = win < len ? win : len;
                med = (int64_t)len * win / 2 <= ((P.pass == 0 && a.full_dp) ? EST_LANE : (int64_t)a.est_lane);
            }
            const bool big = emit && len > TINY && !med;
            const uint64_t medM = ballot(med);
            if (med) medb[nmb + __popcll(medM & lt)] = make_int2(sl, el);
            nmb += __popcll(medM);
            const uint64_t bigM = ballot(big);
            if (bigM) {   // long segments: global queue for k_chain_long (rare)
                uint32_t q0 = 0;
                if (lane == 0) q0 = atomicAdd(a.lseg_n, (uint32_t)__popcll(bigM));
                q0 = (uint32_t)uni((int32_t)q0);
                if (big) {
                    const uint32_t q = q0 + (uint32_t)__popcll(bigM & lt);
                    if (q < a.lseg_cap) a.lseg[q] = make_uint4(r, (uint32_t)sl, (uint32_t)el, 0u);
                }
                n_big += (uint32_t)__popcll(bigM);
                const int32_t ml = rdl(scan_max(big ? len : 0), 63);
                max_seg = max_seg > ml ? max_seg : ml;
            }
            wave_lds_sync();
            if (nmb >= 64) flush_med(64);
        };
        // drain tiny queues: full batches, and before the oldest start leaves the key ring
        auto drain = [&](int32_t horizon, bool all) {
            for (;;) {
                const int32_t n0 = tt0 - th0;
                if (n0 <= 0) break;
                if (n0 < 64 && !all && uni(tq[0 * TQ + (th0 & (TQ - 1))]) >= horizon) break;
                tiny_batch(0, th0, n0 < 64 ? n0 : 64);
            }
            for (;;) {
                const int32_t n1 = tt1 - th1;
                if (n1 <= 0) break;
                if (n1 < 64 && !all && uni(tq[1 * TQ + (th1 & (TQ - 1))]) >= horizon) break;
                tiny_batch(1, th1, n1 < 64 ? n1 : 64);
            }
            for (;;) {
                const int32_t n2 = tt2 - th2;
                if (n2 <= 0) break;
                if (n2 < 64 && !all && uni(tq[2 * TQ + (th2 & (TQ - 1))]) >= horizon) break;
                tiny_batch(2, th2, n2 < 64 ? n2 : 64);
            }
        };
        const uint64_t kprev = c0 > 0 ? K[c0 - 1] : 0;
        uint32_t prev_lo = (uint32_t)uni((int32_t)(uint32_t)kprev), prev_hi = (uint32_t)uni((int32_t)(uint32_t)(kprev >> 32));
        uint64_t nk = c0 + lane < A ? K[c0 + lane] : 0;
        bool closed = false;
        for (int32_t i0 = c0; i0 < A; i0 += 64) {
            const bool ext = i0 >= c1;      // past the chunk: only close the open segment
            if (ext && pend < 0) { closed = true; break; }
            const uint64_t ak = nk;
            const int32_t il = i0 + lane;
            const bool valid = il < A;
            nk = (il + 64 < A) ? K[il + 64] : 0;
            kring[il & (KRING - 1)] = ak;
            const uint64_t pk = ((uint64_t)(uint32_t)shr1_dpp((int32_t)(uint32_t)(ak >> 32), (int32_t)prev_hi) << 32) |
                                (uint32_t)shr1_dpp((int32_t)(uint32_t)ak, (int32_t)prev_lo);
            const uint32_t g = (uint32_t)(ak >> gsh), gp = (uint32_t)(pk >> gsh);
            const int32_t p = (int32_t)((ak >> qb) & rmask), pprv = (int32_t)((pk >> qb) & rmask);
            bool iso = valid && (il == 0 || g != gp || p > (int32_t)((uint32_t)pprv + (uint32_t)maxdx));
            uint64_t isoM = ballot(iso);
            if (ext && isoM) {              // the first isolated anchor closes it; nothing opens
                isoM &= (~isoM + 1);
                iso = ((isoM >> lane) & 1ULL) != 0;
            }
            // an isolated anchor closes the segment opened by the previous one
            const uint64_t lower = isoM & lanemask_lt();
            const int32_t sl = lower ? i0 + 63 - clz64(lower) : pend;
            wave_lds_sync();
            route(iso && sl >= 0, sl, il);
            if (isoM) pend = i0 + 63 - clz64(isoM);
            prev_lo = rdlu((uint32_t)ak, 63); prev_hi = rdlu((uint32_t)(ak >> 32), 63);
            // the next block overwrites ring slots of anchors < i0 + 128 - KRING
            drain(i0 + 192 - KRING, false);
            if (ext && isoM) { closed = true; break; }
        }
        if (!closed && pend >= 0) route(lane == 0, pend, A);          // the read's last segment
        drain(0, true);
        if (nmb > 0) flush_med(nmb);
        // the read's best over its singletons and tiny segments
        {
            const int32_t m = rdl(scan_max(bf), 63);
            const int32_t mi = rdl(scan_max(bf == m ? bi : -1), 63);
            const uint64_t wpairs = uni64(wave_sum64(pairs));
            if (lane == 0) {
                if (mi >= 0) atomicMax(a.rbest + r, best_key(m, mi));
                atomicAdd((unsigned long long*)&a.out[r].dp_pairs, (unsigned long long)wpairs);
                ReadOut* O = a.out + r;
                O->t_pass[P.pass] = (uint32_t)(wall_clock64() - t_start);
                const uint32_t st6 = (uint32_t)(max_seg > 65535 ? 65535 : max_seg) | ((n_big > 65535 ? 65535u : n_big) << 16);
                if (P.pass == 0) O->pad2 = st6; else O->n_deep = st6;
            }
        }
    }
}

// ---- 5a'. a lower bound of the read's best f, for segment pruning.
// In chain_dp_all (lchain.rs:73-90) the first predecessor visited for a
// non-isolated anchor i is j = i - 1 (the n_skip break needs > max_skip
// visits first), so f[i] >= max(span, f[i-1] + sc(i, i-1)) whenever comput_sc
// (lchain.rs:17-34) accepts (i, i-1), and f[i] >= span always.  LB[i] =
// max(span, LB[i-1] + sc) is a composition scan of x -> max(x + a, b) over
// the wave.  A segment of len anchors has f <= len * span (every step adds at
// most span), so one with len * span < max LB can hold neither the read's
// largest f nor a tie of it: k_chain_seg skips it (not in debug mode, where
// the full f/pprev arrays are kept).
__global__ __launch_bounds__(256) void k_chain_lb(ChainArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    extern __shared__ __align__(16) unsigned char smem[];
    const ChainKParams P = a.P;
    int16_t* lut = (int16_t*)smem;
    if (blockIdx.x * (blockDim.x >> 6) >= (uint32_t)a.item_off[a.n]) return;   // no work item: skip the LUT load
    load_lut(lut, a.lut, P.lut_n);
    __syncthreads();
    const int lane = lane_id();
    const uint32_t qb = a.kl.qb, rb = a.kl.rb;
    const uint64_t qmask = (1ULL << qb) - 1, rmask = (1ULL << rb) - 1;
    const uint32_t gsh = rb + qb;
    const int32_t maxdx = P.max_dist_x, maxdy = P.max_dist_y, bw = P.bw, span = P.span;
    constexpr int32_t NEG = -(1 << 29);
    constexpr int U = 4;                      // blocks of 64 keys loaded together
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const uint32_t n_items = (uint32_t)uni((int32_t)a.item_off[a.n]);
    for (uint32_t it = blockIdx.x * (blockDim.x >> 6) + wave_id(); it < n_items; it += nwaves) {
        const uint32_t t = (uint32_t)uni((int32_t)((a.item_read && it < a.item_cap) ? a.item_read[it] : item_owner(a.item_off, a.n, it)));
        const uint32_t r = (uint32_t)uni((int32_t)a.order[t]);
        const int32_t c0 = (int32_t)(it - (uint32_t)uni((int32_t)a.item_off[t])) * (int32_t)a.seg_chunk;
        const uint64_t base = uni64(a.a_off[r]);
        const int32_t A = min((int32_t)uni((int32_t)a.cnt2[r]), c0 + (int32_t)a.seg_chunk);
        const uint64_t* K = a.keys + base;
        uint64_t* isw = a.isob ? a.isob + (base >> 6) + r : nullptr;   // this read's segment-start words (ChainArgs::isob)
        int32_t carry = NEG, best = span;      // LB restarts at span at a chunk start: still a lower bound
        uint64_t k0 = c0 > 0 ? K[c0 - 1] : 0;
        uint32_t prev_lo = (uint32_t)uni((int32_t)(uint32_t)k0), prev_hi = (uint32_t)uni((int32_t)(uint32_t)(k0 >> 32));
        for (int32_t i00 = c0; i00 < A; i00 += 64 * U) {
            uint64_t kk[U];
#pragma unroll
            for (int u = 0; u < U; ++u) { const int32_t il = i00 + u * 64 + lane; kk[u] = il < A ? K[il] : 0; }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t ak = kk[u];
                const int32_t il = i00 + u * 64 + lane;
                const bool valid = il < A;
                const uint64_t pk = ((uint64_t)(uint32_t)shr1_dpp((int32_t)(uint32_t)(ak >> 32), (int32_t)prev_hi) << 32) |
                                    (uint32_t)shr1_dpp((int32_t)(uint32_t)ak, (int32_t)prev_lo);
                const uint32_t g = (uint32_t)(ak >> gsh), gp = (uint32_t)(pk >> gsh);
                const int32_t p = (int32_t)((ak >> qb) & rmask), pj = (int32_t)((pk >> qb) & rmask);
                const int32_t q = (int32_t)(ak & qmask), qj = (int32_t)(pk & qmask);
                const bool tiso = il == 0 || g != gp || p > (int32_t)((uint32_t)pj + (uint32_t)maxdx);   // starts a segment
                const bool iso = tiso || il == c0;
                if (isw) {
                    const uint64_t im = ballot(valid && tiso);
                    if (lane == 0 && i00 + u * 64 < A) isw[(i00 + u * 64) >> 6] = im;
                }
                int32_t sa = NEG;
                if (valid && !iso) {
                    const int32_t dq = q - qj, dr = p - pj;
                    const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
                    if (dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy && dd <= bw) {
                        const int32_t dg = dr < dq ? dr : dq;
                        sa = (span < dg ? span : dg) - (int32_t)lut[dd];
                    }
                }
                int32_t sb = valid ? span : NEG;
                scan_lb(sa, sb);
                const int32_t lb = max(carry + sa, sb);
                best = max(best, lb);
                carry = rdl(lb, 63);
                prev_lo = rdlu((uint32_t)ak, 63); prev_hi = rdlu((uint32_t)(ak >> 32), 63);
            }
        }
        const int32_t m = rdl(scan_max(best), 63);
        if (lane == 0) atomicMax(a.fmin + r, m);
    }
}

// ---- 5a''. production, after k_chain_lb (both passes; the rescue pass on its
// rescued reads): per read, the segments that
// can hold its best f.  With fm = k_chain_lb's bound, a segment of len anchors
// has f <= len * span, so only len >= Lmin = ceil(fm / span) can (k_chain_seg's
// pruning rule).  When Lmin > CHAIN_TINY every candidate goes to the
// long-segment queue whole (k_chain_long / k_chain_giant), and the candidates
// come from k_chain_lb's segment-start bits (1 bit per anchor, isob) without
// reading a key.  Reads with a weaker bound (no real chain) are queued for
// k_chain_seg's streaming pass, one (read, chunk) item per seg_chunk anchors.
// One wave per read; its words are walked from the last 64-word chunk to the
// first, carrying the first segment start of the later chunks.
// Candidates go to the queues in per-workgroup batches (one global atomic per
// workgroup and queue: a burst of per-read atomics on one counter serialises).
// A read's segment-start words are split lane-major (lane l takes K = nwd/64
// consecutive words), so all of a read's loads are in flight together; the
// first start after a lane's words is a suffix minimum over the lanes.
constexpr int SC_NW = 16;                 // waves (reads in flight) per workgroup
constexpr int SC_BUF = 128;               // candidate entries buffered per wave
constexpr int SC_KW = 8;                  // words per lane per load group
__global__ __launch_bounds__(SC_NW * 64) void k_seg_cands(ChainArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    __shared__ uint2 s_buf[SC_NW][SC_BUF];            // (start, end) of this wave's read's candidates
    __shared__ uint32_t s_cnt[SC_NW], s_rd[SC_NW], s_nit[SC_NW], s_base[2];
    const int lane = lane_id(), wv = wave_id();
    const int32_t span = a.P.span;
    const uint32_t rounds = (a.n + SC_NW - 1) / SC_NW;
    for (uint32_t g = blockIdx.x; g < rounds; g += gridDim.x) {
        const uint32_t r = g * SC_NW + (uint32_t)wv;
        if (lane == 0) s_cnt[wv] = 0;
        wave_lds_sync();
        uint32_t nit = 0;
        if (r < a.n) {
            const int32_t A = (int32_t)uni((int32_t)a.cnt2[r]);
            const int32_t fm = uni(a.fmin[r]);
            const uint64_t base = uni64(a.a_off[r]);
            const bool on = a.P.pass == 0 || (uni(a.out[r].flags) & RF_RESCUED);   // the rescue pass maps rescued reads only
            const uint64_t t0 = wall_clock64();
            if (((A + 63) >> 6) > (int32_t)a.cands_longw) {
                // a long read (100 kb): the whole workgroup walks it below
            } else if (A > 0 && on && fm <= CHAIN_TINY * span) {
                nit = (uint32_t)((A + (int32_t)a.seg_chunk - 1) / (int32_t)a.seg_chunk);
            } else if (A > 0 && on) {
                const int32_t Lmin = (fm + span - 1) / span;
                const uint64_t* isw = a.isob + (base >> 6) + r;
                const int32_t nwd = (A + 63) >> 6;
                const int32_t K = (nwd + 63) >> 6;
                const int32_t w0 = min(nwd, lane * K), w1 = min(nwd, w0 + K);
                const int32_t ng = (K + SC_KW - 1) / SC_KW;       // load groups per lane (wave-uniform)
                uint64_t wd[SC_KW];
                // pass A: this lane's first segment start (its earliest nonzero word)
                int32_t first = INT_MAX;
                for (int32_t gq = 0; gq < ng; ++gq) {
                    if (ballot(first == INT_MAX) == 0ULL) break;
                    const int32_t gb = w0 + gq * SC_KW;
#pragma unroll
                    for (int u = 0; u < SC_KW; ++u) wd[u] = gb + u < w1 ? isw[gb + u] : 0ULL;
                    if (first == INT_MAX) {
#pragma unroll
                        for (int u = SC_KW - 1; u >= 0; --u) if (wd[u]) first = (gb + u) * 64 + ctz64(wd[u]);
                    }
                }
                int32_t sfx = first;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) { const int32_t o = __shfl_down(sfx, d, 64); if (lane + d < 64) sfx = min(sfx, o); }
                int32_t after = __shfl_down(sfx, 1, 64);
                after = lane == 63 ? A : min(after, A);
                // pass B: each lane walks its words from the last to the first (lane-divergent, no
                // cross-lane work inside); candidates to the wave's LDS buffer
                int32_t mx = 0;
                auto push = [&](int32_t sl, int32_t el) {
                    const uint32_t k = atomicAdd(&s_cnt[wv], 1u);
                    if (k < (uint32_t)SC_BUF) s_buf[wv][k] = make_uint2((uint32_t)sl, (uint32_t)el);
                    else {                                     // rare: more than SC_BUF candidates in one read
                        const uint32_t q = atomicAdd(a.lseg_n, 1u);
                        if (q < a.lseg_cap) a.lseg[q] = make_uint4(r, (uint32_t)sl, (uint32_t)el, 0u);
                    }
                    mx = max(mx, el - sl);
                };
                for (int32_t gq = ng - 1; gq >= 0; --gq) {
                    const int32_t gb = w0 + gq * SC_KW;
                    if (ng > 1) {                               // one group: its words are still in wd
#pragma unroll
                        for (int u = 0; u < SC_KW; ++u) wd[u] = gb + u < w1 ? isw[gb + u] : 0ULL;
                    }
#pragma unroll
                    for (int u = SC_KW - 1; u >= 0; --u) {
                        const uint64_t m = wd[u];
                        if (!m) continue;
                        const int32_t w = gb + u;
                        if (Lmin >= 64) {                         // only a word's last start can begin one
                            const int32_t sl = w * 64 + 63 - clz64(m);
                            if (after - sl >= Lmin) push(sl, after);
                        } else {
                            uint64_t mm = m;
                            int32_t e = after;
                            while (mm) {                          // starts from the highest down
                                const int b = 63 - clz64(mm);
                                mm &= ~(1ULL << b);
                                const int32_t sl = w * 64 + b;
                                if (e - sl >= Lmin) push(sl, e);
                                e = sl;
                            }
                        }
                        after = w * 64 + ctz64(m);
                    }
                }
                const int32_t ml = rdl(scan_max(mx), 63);
                wave_lds_sync();
                if (lane == 0) {
                    ReadOut* O = a.out + r;
                    O->t_pass[a.P.pass] = (uint32_t)(wall_clock64() - t0);
                    const uint32_t ncs = s_cnt[wv];
                    const uint32_t st6 = (uint32_t)(ml > 65535 ? 65535 : ml) | ((ncs > 65535 ? 65535u : ncs) << 16);
                    if (a.P.pass == 0) O->pad2 = st6; else O->n_deep = st6;
                }
            }
        }
        wave_lds_sync();
        if (lane == 0) { s_cnt[wv] = min(s_cnt[wv], (uint32_t)SC_BUF); s_nit[wv] = nit; s_rd[wv] = r; }
        __syncthreads();
        if (threadIdx.x == 0) {                              // one atomic per queue for the workgroup
            uint32_t tc = 0, ti = 0;
            for (int w = 0; w < SC_NW; ++w) { tc += s_cnt[w]; ti += s_nit[w]; }
            s_base[0] = tc ? atomicAdd(a.lseg_n, tc) : 0u;
            s_base[1] = ti ? atomicAdd(a.sq_n, ti) : 0u;
        }
        __syncthreads();
        uint32_t oc = s_base[0], oi = s_base[1];
        for (int w = 0; w < wv; ++w) { oc += s_cnt[w]; oi += s_nit[w]; }
        const uint32_t myc = s_cnt[wv], myi = s_nit[wv], rr = s_rd[wv];
        for (uint32_t k = (uint32_t)lane; k < myc; k += 64) {
            const uint2 e = s_buf[wv][k];
            if (oc + k < a.lseg_cap) a.lseg[oc + k] = make_uint4(rr, e.x, e.y, 0u);
        }
        for (uint32_t k = (uint32_t)lane; k < myi; k += 64)
            if (oi + k < a.sq_cap) a.sq[oi + k] = make_uint2(rr, k);
        __syncthreads();                                     // s_buf / s_cnt are reused by the next round
    }
    // Long reads (over cands_longw words: C5's 100 kb reads, 3 k words), one workgroup each: the
    // read's words split over all 16 waves (K words per lane), the first start after a lane's
    // words is a suffix minimum over the lanes and then the waves; pass B as above, into every
    // wave's buffer with the read's index (one wave per such read used a quarter of the GPU)
    __shared__ int32_t s_wfirst[SC_NW], s_wml[SC_NW];
    for (uint32_t r = blockIdx.x; r < a.n; r += gridDim.x) {
        const int32_t A = (int32_t)uni((int32_t)a.cnt2[r]);
        const int32_t nwd = (A + 63) >> 6;
        if (nwd <= (int32_t)a.cands_longw) continue;         // (workgroup-uniform)
        const bool on = a.P.pass == 0 || (uni(a.out[r].flags) & RF_RESCUED);
        if (!on) continue;
        const int32_t fm = uni(a.fmin[r]);
        const uint64_t base = uni64(a.a_off[r]);
        const uint64_t t0 = wall_clock64();
        if (lane == 0) { s_cnt[wv] = 0; s_nit[wv] = 0; s_rd[wv] = r; }
        __syncthreads();
        int32_t mx = 0;
        if (fm <= CHAIN_TINY * span) {
            if (threadIdx.x == 0) s_nit[0] = (uint32_t)((A + (int32_t)a.seg_chunk - 1) / (int32_t)a.seg_chunk);
        } else {
            const int32_t Lmin = (fm + span - 1) / span;
            const uint64_t* isw = a.isob + (base >> 6) + r;
            const int32_t gl = wv * 64 + lane;                   // lane of the workgroup
            const int32_t K = (nwd + SC_NW * 64 - 1) / (SC_NW * 64);
            const int32_t w0 = min(nwd, gl * K), w1 = min(nwd, w0 + K);
            int32_t first = INT_MAX;
            for (int32_t w = w0; w < w1 && first == INT_MAX; ++w) { const uint64_t m = isw[w]; if (m) first = w * 64 + ctz64(m); }
            int32_t sfx = first;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) { const int32_t o = __shfl_down(sfx, d, 64); if (lane + d < 64) sfx = min(sfx, o); }
            if (lane == 0) s_wfirst[wv] = sfx;
            __syncthreads();
            int32_t later = A;                                   // first start of the later waves
            for (int t = wv + 1; t < SC_NW; ++t) later = min(later, s_wfirst[t]);
            int32_t after = __shfl_down(sfx, 1, 64);
            after = lane == 63 ? later : min(after, later);
            after = min(after, A);
            auto push = [&](int32_t sl, int32_t el) {
                const uint32_t k = atomicAdd(&s_cnt[wv], 1u);
                if (k < (uint32_t)SC_BUF) s_buf[wv][k] = make_uint2((uint32_t)sl, (uint32_t)el);
                else {
                    const uint32_t q = atomicAdd(a.lseg_n, 1u);
                    if (q < a.lseg_cap) a.lseg[q] = make_uint4(r, (uint32_t)sl, (uint32_t)el, 0u);
                }
                mx = max(mx, el - sl);
            };
            for (int32_t w = w1 - 1; w >= w0; --w) {
                const uint64_t m = isw[w];
                if (!m) continue;
                if (Lmin >= 64) {
                    const int32_t sl = w * 64 + 63 - clz64(m);
                    if (after - sl >= Lmin) push(sl, after);
                } else {
                    uint64_t mm = m;
                    int32_t e = after;
                    while (mm) {
                        const int b = 63 - clz64(mm);
                        mm &= ~(1ULL << b);
                        const int32_t sl = w * 64 + b;
                        if (e - sl >= Lmin) push(sl, e);
                        e = sl;
                    }
                }
                after = w * 64 + ctz64(m);
            }
        }
        const int32_t wml = rdl(scan_max(mx), 63);
        if (lane == 0) s_wml[wv] = wml;                      // (not s_wfirst: other waves may still read it)
        __syncthreads();
        if (threadIdx.x == 0 && fm > CHAIN_TINY * span) {
            int32_t ml = 0; uint32_t ncs = 0;
            for (int t = 0; t < SC_NW; ++t) { ml = max(ml, s_wml[t]); ncs += s_cnt[t]; }
            ReadOut* O = a.out + r;
            O->t_pass[a.P.pass] = (uint32_t)(wall_clock64() - t0);
            const uint32_t st6 = (uint32_t)(ml > 65535 ? 65535 : ml) | ((ncs > 65535 ? 65535u : ncs) << 16);
            if (a.P.pass == 0) O->pad2 = st6; else O->n_deep = st6;
        }
        if (lane == 0) s_cnt[wv] = min(s_cnt[wv], (uint32_t)SC_BUF);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tc = 0, ti = 0;
            for (int w = 0; w < SC_NW; ++w) { tc += s_cnt[w]; ti += s_nit[w]; }
            s_base[0] = tc ? atomicAdd(a.lseg_n, tc) : 0u;
            s_base[1] = ti ? atomicAdd(a.sq_n, ti) : 0u;
        }
        __syncthreads();
        uint32_t oc = s_base[0], oi = s_base[1];
        for (int w = 0; w < wv; ++w) { oc += s_cnt[w]; oi += s_nit[w]; }
        const uint32_t myc = s_cnt[wv], myi = s_nit[wv];
        for (uint32_t k = (uint32_t)lane; k < myc; k += 64) {
            const uint2 e = s_buf[wv][k];
            if (oc + k < a.lseg_cap) a.lseg[oc + k] = make_uint4(r, e.x, e.y, 0u);
        }
        for (uint32_t k = (uint32_t)lane; k < myi; k += 64)
            if (oi + k < a.sq_cap) a.sq[oi + k] = make_uint2(r, k);
        __syncthreads();
    }
}

// ---- 5b. medium segments, one lane each, from a global queue: chain_dp_all
// (lchain.rs:73-90) as a flattened per-lane state machine (advance st |
// evaluate up to MJ predecessors | finish i) inside a wave-uniform loop.
// Lane g takes queue entries g, g + stride, ... (interleaved, no atomics).
// The MJ predecessors of one iteration are loaded together; a mark
// t[pprev[j]] = i landing on a later j of the same group is forwarded.  t[]
// is the reference's own mark array (t[j] == i) in HBM scratch, reset to -1
// when anchor j is finished.
constexpr int MJ = 4;
__global__ __launch_bounds__(256) void k_chain_med(ChainArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    extern __shared__ __align__(16) unsigned char smem[];
    const ChainKParams P = a.P;
    int16_t* lut = (int16_t*)smem;
    if (blockIdx.x * blockDim.x >= min(*a.mseg_n, a.mseg_cap)) return;   // no queue entry: skip the LUT load
    load_lut(lut, a.lut, P.lut_n);
    __syncthreads();
    const uint32_t qb = a.kl.qb;
    const uint64_t qmask = (1ULL << qb) - 1, rmask = (1ULL << a.kl.rb) - 1;
    const int32_t maxdx = P.max_dist_x, maxdy = P.max_dist_y, bw = P.bw, span = P.span;
    const uint32_t nm = min((uint32_t)uni((int32_t)*a.mseg_n), a.mseg_cap);
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t kq = blockIdx.x * blockDim.x + threadIdx.x;   // this lane's next queue entry
    const uint64_t* K = nullptr;
    int32_t *F = nullptr, *PP = nullptr, *T = nullptr;
    uint32_t r = 0;
    int32_t me = 0, i = 0, j = 0, lo = 0, sx = 0, max_f = 0, max_j = -1, n_skip = 0, pi = 0, qi = 0, psx = 0;
    int32_t bf = INT_MIN, bi = -1;      // segment best
    int32_t pf = 0, ppf = -1;           // f/pprev of anchor i-1 (forwarded to the first j of i)
    uint32_t pairs = 0;
    int32_t state = 0;                  // 0 idle, 1 advance st, 2 j-loop
    for (;;) {
        const bool idle = state == 0;
        if (any(idle && kq < nm)) {
            if (idle && kq < nm) {
                const uint4 L = a.mseg[kq];
                r = L.x;
                const uint64_t base = a.a_off[r];
                K = a.keys + base; F = a.f + base; PP = a.pp + base; T = a.tmark + base;
                const int32_t ms = (int32_t)L.y;
                me = (int32_t)L.z;
                F[ms] = span; PP[ms] = -1; T[ms] = -1;
                bf = span; bi = ms; pairs = 0;
                const uint64_t k0 = K[ms], k1 = K[ms + 1];
                psx = (int32_t)((k0 >> qb) & rmask);
                pi = (int32_t)((k1 >> qb) & rmask); qi = (int32_t)(k1 & qmask);
                pf = span; ppf = -1;
                sx = ms; i = ms + 1; state = 1;
                kq += stride;
            }
        }
        if (!any(state != 0)) break;
        if (state == 1) {
            if (sx < i && pi > (int32_t)((uint32_t)psx + (uint32_t)maxdx)) {
                ++sx;
                psx = (int32_t)((K[sx] >> qb) & rmask);
            } else {
                lo = sx > i - P.max_iter ? sx : i - P.max_iter;
                j = i - 1; max_f = span; max_j = -1; n_skip = 0; state = 2;
            }
        } else if (state == 2) {
            if (j >= lo) {
                uint64_t kk[MJ];
                int32_t ff[MJ], pv[MJ], tt[MJ];
#pragma unroll
                for (int u = 0; u < MJ; ++u) {
                    const int32_t jj = j - u;
                    kk[u] = 0; ff[u] = 0; pv[u] = -1; tt[u] = -1;
                    if (jj >= lo) {
                        kk[u] = K[jj];
                        if (jj == i - 1) { ff[u] = pf; pv[u] = ppf; }   // just finished: from registers
                        else { ff[u] = F[jj]; pv[u] = PP[jj]; tt[u] = T[jj]; }
                    }
                }
                bool brk = false;
                int32_t done = 0;
#pragma unroll
                for (int u = 0; u < MJ; ++u) {
                    const int32_t jj = j - u;
                    if (!brk && jj >= lo) {
                        ++done; ++pairs;
                        const int32_t pj = (int32_t)((kk[u] >> qb) & rmask), qj = (int32_t)(kk[u] & qmask);
                        const int32_t dq = qi - qj, dr = pi - pj;
                        bool ok = dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy;
                        const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
                        ok = ok && dd <= bw;
                        if (ok) {
                            const int32_t dg = dr < dq ? dr : dq;
                            const int32_t sv = (span < dg ? span : dg) - (int32_t)lut[dd] + ff[u];
                            if (sv > max_f) { max_f = sv; max_j = jj; if (n_skip > 0) --n_skip; }
                            else if (tt[u] == i) { ++n_skip; if (n_skip > P.max_skip) brk = true; }
                            if (!brk && pv[u] >= 0) {
                                T[pv[u]] = i;
#pragma unroll
                                for (int w = u + 1; w < MJ; ++w)
                                    if (pv[u] == j - w) tt[w] = i;
                            }
                        }
                    }
                }
                j = brk ? lo - 1 : j - done;
            } else {
                F[i] = max_f; PP[i] = max_j; T[i] = -1;
                best_merge(bf, bi, max_f, i);
                pf = max_f; ppf = max_j;
                ++i;
                if (i >= me) {
                    atomicMax(a.rbest + r, best_key(bf, bi));
                    atomicAdd((unsigned long long*)&a.out[r].dp_pairs, (unsigned long long)pairs);
                    state = 0;
                } else {
                    const uint64_t ki = K[i];
                    pi = (int32_t)((ki >> qb) & rmask); qi = (int32_t)(ki & qmask);
                    state = 1;
                }
            }
        }
    }
}

// long segments by descending length (largest-first hand-out to k_chain_long);
// also the anchors each chain kernel gets (roofline accounting, mm2g_batch_counters):
// seg_stat[0] long segments below giant_min, [1] from giant_min on, [2] medium segments
__global__ __launch_bounds__(1024) void k_lseg_order(ChainArgs a) {
    __shared__ uint32_t hist[33], offs[33];
    __shared__ unsigned long long ssum[3][16];
    const int tid = threadIdx.x;
    const uint32_t n = min(*a.lseg_n, a.lseg_cap);
    const uint4* lseg = a.lseg;
    uint32_t* order = a.lseg_order;
    if (tid < 33) hist[tid] = 0;
    __syncthreads();
    unsigned long long s_lo = 0, s_hi = 0, s_med = 0;
    for (uint32_t q = tid; q < n; q += 1024) {
        const uint32_t c = lseg[q].z - lseg[q].y;
        atomicAdd(&hist[32 - (32 - __builtin_clz(c | 1))], 1u);
        if (c >= a.giant_min) s_hi += c; else s_lo += c;
    }
    if (a.seg_stat) {
        const uint32_t nm = min(*a.mseg_n, a.mseg_cap);
        for (uint32_t q = tid; q < nm; q += 1024) s_med += a.mseg[q].z - a.mseg[q].y;
        s_lo = wave_sum64(s_lo); s_hi = wave_sum64(s_hi); s_med = wave_sum64(s_med);
        if (lane_id() == 0) { ssum[0][tid >> 6] = s_lo; ssum[1][tid >> 6] = s_hi; ssum[2][tid >> 6] = s_med; }
    }
    __syncthreads();
    if (tid == 0) { uint32_t run = 0; for (int b = 0; b < 33; ++b) { offs[b] = run; run += hist[b]; } }
    if (a.seg_stat && tid < 3) {
        unsigned long long t = 0;
        for (int w = 0; w < 16; ++w) t += ssum[tid][w];
        a.seg_stat[tid] = t;
    }
    __syncthreads();
    for (uint32_t q = tid; q < n; q += 1024) {
        const uint32_t c = lseg[q].z - lseg[q].y;
        order[atomicAdd(&offs[32 - (32 - __builtin_clz(c | 1))], 1u)] = q;
    }
}

// ---- 5b. one long segment per wave, wave-cooperative (heaviest first)
// PROF (MM2G_KNOB_LSEG_PROF): shader-clock cycles of each phase of the
// per-anchor step, summed over the pass's long segments into a.gprof[16..31]:
// [16] anchors, [24] committed by the speculative block pass ([25] its
// rounds); of the per-anchor path's: [17] settled by the simple / chain-shortcut
// step, [19] taken through the exact loop; [18] 64-predecessor window steps;
// cycles of the per-anchor path's [20] st window, [21] simple / shortcut
// attempt, [22] exact loop, [23] register shift + ring store.
// SB: predecessors per step of the speculative rounds (their LDS loads and
// comput_sc issued together; MM2G_KNOB_SPEC_BATCH)
template <bool PROF, int SB>
__global__ __launch_bounds__(DP_NW * 64) void k_chain_long(ChainArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    extern __shared__ __align__(16) unsigned char smem[];
    const ChainKParams P = a.P;
    int16_t* lut = (int16_t*)smem;
    const int lut_bytes = ((P.lut_n * 2) + 15) & ~15;
    uint32_t* rings = (uint32_t*)(smem + lut_bytes);
    uint64_t* rkeys = (uint64_t*)(rings + DP_NW * RING_WORDS);
    int2* rfps = (int2*)(rkeys + DP_NW * RK);
    if (blockIdx.x * DP_NW >= min(*a.lseg_n, a.lseg_cap)) return;   // no long segment: skip the LUT load
    load_lut(lut, a.lut, P.lut_n);
    for (int i = threadIdx.x; i < DP_NW * RING_WORDS; i += blockDim.x) rings[i] = 0;
    __syncthreads();
    const int lane = lane_id(), wv = wave_id();
    uint32_t* ring = rings + wv * RING_WORDS;
    uint64_t* rkey = rkeys + wv * RK;
    int2* rfp = rfps + wv * RK;
    const uint32_t qb = a.kl.qb, rb = a.kl.rb;
    const uint64_t qmask = (1ULL << qb) - 1, rmask = (1ULL << rb) - 1;
    const int32_t maxdx = P.max_dist_x, maxdy = P.max_dist_y, bw = P.bw, span = P.span;
    const uint32_t nl = min((uint32_t)uni((int32_t)*a.lseg_n), a.lseg_cap);
    const uint32_t nwaves = gridDim.x * DP_NW;
    for (uint32_t t = blockIdx.x * DP_NW + wv; t < nl; t += nwaves) {
        const uint32_t q = (uint32_t)uni((int32_t)a.lseg_order[t]);
        const uint4 L = a.lseg[q];
        if ((uint32_t)uni((int32_t)L.w) & LSEG_DONE) continue;   // k_chain_giant did it
        const uint32_t r = (uint32_t)uni((int32_t)L.x);
        const int32_t s = uni((int32_t)L.y), e = uni((int32_t)L.z);
        if (t < 256) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(0);
        const uint64_t base = uni64(a.a_off[r]);
        const int32_t A = (int32_t)(uni64(a.a_off[r + 1]) - base);
        const uint64_t* K = a.keys + base;
        int32_t* F = a.f + base; int32_t* PP = a.pp + base;
        uint64_t cpairs = 0;
        uint32_t n_steps = 0, n_deep = 0;
        int32_t best_f = INT_MIN, best_i = -1;
        (void)A; (void)n_deep;
        const uint64_t seg_t0 = wall_clock64();
        uint64_t pc_spec = 0, pc_seg0 = PROF ? clock64() : 0;   // PROF: the heaviest segment's cycles
        // ---- cooperative DP of segment [s, e): anchor s is isolated, every
        // later anchor has a candidate predecessor.  The 64 newest
        // predecessors (rpos, qpos, f, pprev; lane l <-> j = i-1-l) live in
        // registers and shift one lane per anchor (DPP wave_shr); the newest
        // RK keys and f/pprev also go to the wave's LDS ring for the st
        // window and deep steps; older ones come from HBM (flushed per block).
        int32_t st = s, stb = INT_MIN / 2, skv = INT_MIN / 2;   // st window [stb, stb+63], valid up to skv
        uint64_t sk = 0;
        int32_t wp = 0, wq = 0, wf = 0, wpp = -1;
        bool try_simple = true;
        int32_t next_try = 0, backoff = 16;     // after a failed simple attempt: retry at next_try (backoff 16..128)
        uint64_t pc_st = 0, pc_simple = 0, pc_exact = 0, pc_tail = 0, pn_done = 0, pn_exact = 0, tp = 0, pn_spec = 0, pn_rounds = 0;
#define LP(acc) do { if (PROF) { const uint64_t t_ = clock64(); acc += t_ - tp; tp = t_; } } while (0)
        uint64_t nk = (s + lane < e) ? K[s + lane] : 0;
        for (int32_t i0 = s; i0 < e; i0 += 64) {
            const uint64_t ak = nk;
            const int32_t il = i0 + lane;
            const bool valid = il < e;
            nk = (il + 64 < e) ? K[il + 64] : 0;
            const int32_t ring_lo = i0 + 64 - RK;   // ring holds anchors [max(s, ring_lo), i0+63]
            rkey[il & (RK - 1)] = ak;
            if (il == s) rfp[il & (RK - 1)] = make_int2(span, -1);
            wave_lds_sync();
            bool drained = false;
            const int32_t ib = i0 == s ? s + 1 : i0;
            const int32_t ie = e < i0 + 64 ? e : i0 + 64;
            if (i0 == s) {   // anchor s enters the register window
                const uint64_t k0 = rdl64(ak, 0);
                wp = shr1_dpp(wp, (int32_t)((k0 >> qb) & rmask)); wq = shr1_dpp(wq, (int32_t)(k0 & qmask));
                wf = shr1_dpp(wf, span); wpp = shr1_dpp(wpp, -1);
            }
            // ---- speculative block pass (production): lane l runs the
            // reference loop (lchain.rs:76-89) of anchor k = i0 + l over its 64
            // nearest predecessors, all anchors of the block at once, on guessed
            // f/pprev for the block's earlier anchors.  The first guess follows
            // the chain (pprev[k] = k-1 when comput_sc accepts the pair: a
            // composition scan from the block's final predecessor); each round
            // replaces the guesses with what the lanes computed.  By induction
            // in k, every anchor before the first lane whose result differs from
            // its guess is exact, and so is that lane's result (all its inputs
            // were exact): each round commits at least one anchor.  A lane whose
            // loop would run past its 64 predecessors, and every anchor left after
            // a.spec_rounds rounds, takes the per-anchor path below.
            int32_t i_seq = ib;
            const uint64_t tsp0 = PROF ? clock64() : 0;
            if (a.lazy) {
                const int32_t k = i0 + lane;
                const bool kv = k >= ib && k < ie;
                const int32_t pk = (int32_t)((ak >> qb) & rmask), qk = (int32_t)(ak & qmask);
                // candidates of k (lchain.rs:75-78): j in [max(st_k, k - max_iter), k-1];
                // 65 = more than the 64 predecessors in reach
                int32_t dlim;
                {
                    const int32_t base = max(s, k - 64);
                    const int32_t pb = (int32_t)((rkey[base & (RK - 1)] >> qb) & rmask);
                    int32_t stk = base;
                    if (pk > (int32_t)((uint32_t)pb + (uint32_t)maxdx)) {    // st_k in (base, k]: branch-free search
                        int32_t pos = base;                                 // invariant: pk > p(pos) + maxdx
#pragma unroll
                        for (int stp = 32; stp >= 1; stp >>= 1) {
                            const int32_t m = pos + stp;
                            const int32_t pm = (int32_t)((rkey[(m < k ? m : k) & (RK - 1)] >> qb) & rmask);
                            if (m < k && pk > (int32_t)((uint32_t)pm + (uint32_t)maxdx)) pos = m;
                        }
                        stk = pos + 1;
                    }
                    int32_t nc = (stk == base && base > s) ? 65 : k - stk;
                    nc = nc < P.max_iter ? nc : P.max_iter;
                    dlim = kv ? nc : 0;
                }
                // first guess: the chain through k-1 (composition x -> max(x + a, b) of the lanes)
                {
                    const uint64_t kp = rkey[(k - 1) & (RK - 1)];
                    const int32_t dq = qk - (int32_t)(kp & qmask), dr = pk - (int32_t)((kp >> qb) & rmask);
                    const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
                    const bool okp = kv && dlim >= 1 && dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy && dd <= bw;
                    const int32_t dg = dr < dq ? dr : dq;
                    const int32_t scp = (span < dg ? span : dg) - (int32_t)lut[okp ? dd : 0];
                    constexpr int32_t NEG = -(1 << 29);
                    int32_t ga = kv ? (okp ? scp : NEG) : 0, gb = kv ? (okp ? NEG : span) : NEG;
                    scan_lb(ga, gb);
                    const int32_t f_in = uni(rfp[(ib - 1) & (RK - 1)].x);
                    const int32_t gf = max(f_in + ga, gb);
                    if (kv) rfp[k & (RK - 1)] = make_int2(gf, okp ? k - 1 : -1);
                }
                wave_lds_sync();
                int32_t committed = ib;
                for (int rnd = 0; rnd < (int)a.spec_rounds && committed < ie; ++rnd) {
                    const bool act0 = kv && k >= committed;
                    int32_t mf = span, mj = -1, ns = 0, vis = 0, mfin = 0;   // mfin: the f of mj this round read
                    uint64_t mkm = 0;       // marks t[j] = k by offset d = k - j (bit d-1)
                    bool brk = false;
                    // four predecessors per step: their loads and comput_sc are
                    // independent (issued together), only the running maximum /
                    // n_skip / marks update is sequential
                    for (int d0 = 1; d0 <= 64; d0 += SB) {
                        if (!any(act0 && !brk && d0 <= dlim)) break;
                        int32_t sv4[SB], pp4[SB], fx4[SB];
                        bool ok4[SB];
#pragma unroll
                        for (int u = 0; u < SB; ++u) {
                            const int d = d0 + u;
                            const bool inr = act0 && d <= dlim;
                            const int32_t j = k - d;
                            uint64_t kj = 0;
                            int2 fpj = make_int2(0, -1);
                            if (inr) { kj = rkey[j & (RK - 1)]; fpj = rfp[j & (RK - 1)]; }
                            const int32_t dq = qk - (int32_t)(kj & qmask), dr = pk - (int32_t)((kj >> qb) & rmask);
                            const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
                            ok4[u] = inr && dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy && dd <= bw;
                            const int32_t dg = dr < dq ? dr : dq;
                            sv4[u] = (span < dg ? span : dg) - (int32_t)lut[ok4[u] ? dd : 0] + fpj.x;
                            pp4[u] = fpj.y; fx4[u] = fpj.x;
                        }
#pragma unroll
                        for (int u = 0; u < SB; ++u) {
                            const int d = d0 + u;
                            const bool act = act0 && !brk && d <= dlim;
                            vis += act ? 1 : 0;
                            if (act && ok4[u]) {
                                if (sv4[u] > mf) { mf = sv4[u]; mj = k - d; mfin = fx4[u]; if (ns > 0) --ns; }
                                else if ((mkm >> (d - 1)) & 1ULL) { ++ns; if (ns > P.max_skip) brk = true; }
                                if (!brk && pp4[u] >= 0) { const int32_t t = k - pp4[u]; if (t <= 64) mkm |= 1ULL << ((t - 1) & 63); }
                            }
                        }
                    }
                    const bool deep = act0 && !brk && dlim > 64;
                    const int2 gv = act0 ? rfp[k & (RK - 1)] : make_int2(0, 0);
                    const uint64_t badM = ballot(act0 && (deep || mf != gv.x || mj != gv.y));
                    const int32_t fb = badM ? i0 + ctz64(badM) : ie;
                    const bool fb_deep = badM && ((ballot(deep) >> ((fb - i0) & 63)) & 1ULL);
                    const int32_t cend = fb_deep ? fb : (fb < ie ? fb + 1 : ie);     // committed after this round
                    cpairs += (uint64_t)wave_sum((act0 && k < cend) ? (uint32_t)vis : 0u);
                    ++n_steps;
                    // next guesses of the lanes after fb: by default what they computed (on inputs
                    // that were guesses).  spec_eval: the f those lanes' chosen predecessors give
                    // once evaluated along the choices (policy evaluation, pointer doubling over
                    // the block: f[k] = f[mj] + (mf - the f[mj] this round read), rooted at lane fb,
                    // at committed anchors and at predecessors before fb).  Any guess keeps the
                    // commit rule exact; better ones commit more per round.
                    int32_t gf = mf;
                    if (a.spec_eval && !fb_deep && fb + 1 < ie) {
                        const int l = lane;
                        const bool upd = act0 && k > fb && !deep;
                        bool done = !(upd && mj >= fb);           // roots: lane fb, chains leaving the unsettled part
                        int32_t acc = done ? (upd || k == fb ? mf : gv.x) : mf - mfin;
                        int32_t ptr = done ? l : mj - i0;
#pragma unroll
                        for (int it = 0; it < 6; ++it) {
                            const int32_t pa = __shfl(acc, ptr, 64), pn = __shfl(ptr, ptr, 64);
                            const bool pd = __shfl((int)done, ptr, 64) != 0;
                            if (!done) { acc += pa; ptr = pn; done = pd; }
                        }
                        gf = acc;
                    }
                    wave_lds_sync();
                    if (act0 && k >= fb && !deep) rfp[k & (RK - 1)] = make_int2(k == fb ? mf : gf, mj);   // lane fb exact, later lanes the next guess
                    wave_lds_sync();
                    if (PROF) { pn_spec += (uint64_t)(cend - committed); pn_rounds += 1; }
                    committed = cend;
                    if (fb_deep) break;
                }
                i_seq = committed;
                if (i_seq < ie) {
                    // the per-anchor path from i_seq: its register window (j = i_seq-1-l) from the ring,
                    // and its st from a coarse seek (st only moves forward; the st loop finishes it)
                    const int32_t jw = i_seq - 1 - lane;
                    const uint64_t kw = rkey[jw & (RK - 1)];
                    const int2 fw = rfp[jw & (RK - 1)];
                    wp = (int32_t)((kw >> qb) & rmask); wq = (int32_t)(kw & qmask); wf = fw.x; wpp = fw.y;
                    const int32_t pc = (int32_t)((rdl64(ak, i_seq - i0) >> qb) & rmask);
                    int32_t slo = st, shi = i_seq;   // st_{i_seq} in [slo, shi]; st only ever lags it
                    while (shi - slo > 64) {
                        const int32_t stp = (shi - slo + 63) >> 6;
                        const int32_t j = slo + lane * stp;
                        const bool jin = j < shi;
                        const uint64_t sr = rkey[j & (RK - 1)];
                        const uint64_t sg = (jin && j < ring_lo) ? K[j] : 0;
                        const uint64_t kj = j >= ring_lo ? sr : sg;
                        // "i_seq's st lies beyond j": true on a prefix of the probes
                        const bool past = jin && pc > (int32_t)((uint32_t)(int32_t)((kj >> qb) & rmask) + (uint32_t)maxdx);
                        const int32_t npc = __popcll(ballot(past));
                        if (npc == 0) break;
                        const int32_t jl = slo + (npc - 1) * stp;
                        slo = jl + 1;
                        shi = min(shi, jl + stp);
                    }
                    st = slo > st ? slo : st;
                }
            }
            if (PROF) pc_spec += clock64() - tsp0;
            for (int32_t i = i_seq; i < ie; ++i) {
                if (PROF) tp = clock64();
                const uint64_t ki = rdl64(ak, i - i0);
                const int32_t pi = (int32_t)((ki >> qb) & rmask);
                const int32_t qi = (int32_t)(ki & qmask);
                // st (lchain.rs:75): first j >= st with rpos_i <= rpos_j + max_dist_x
                for (;;) {
                    if (st < stb || st >= stb + 64 || (i > skv && skv < stb + 63)) {
                        stb = st;
                        skv = i0 + 63;
                        const int32_t j = stb + lane;
                        // two loads and a select, not a select of pointers (a flat
                        // load would wait for every outstanding global load)
                        const uint64_t sr = rkey[j & (RK - 1)];
                        const uint64_t sg = (j < e && j < ring_lo) ? K[j] : 0;
                        sk = j < e ? (j >= ring_lo ? sr : sg) : 0;
                    }
                    const int32_t j = stb + lane;
                    const int32_t pj = (int32_t)((sk >> qb) & rmask);
                    const bool cand = j >= st && j <= i;
                    const bool stop = cand && (j == i || !(pi > (int32_t)((uint32_t)pj + (uint32_t)maxdx)));
                    const uint64_t m = ballot(stop);
                    if (m) { st = stb + ctz64(m); break; }
                    st = stb + 64;
                }
                const int32_t lo = st > i - P.max_iter ? st : i - P.max_iter;
                int32_t max_f = span, max_j = -1, n_skip = 0;
                bool marks = false;
                LP(pc_st);
                // Simple path: n_skip only rises on a marked target, and every mark
                // comes from a valid j with pprev[j] >= lo.  With <= max_skip such
                // sources in the whole window no break can happen, so (f[i], pprev[i])
                // is the plain running maximum in visiting order: the largest sv,
                // first visited (largest j) among equal ones.  No prefix scans, no
                // marks.  Tried while it keeps succeeding (and every 16th anchor).
                // Chains (many mark sources): when the first window's maximum is
                // visited within the first max_skip visits (no break can come
                // before it) and more than max_skip marked visits follow it inside
                // that window (none of them is a new maximum, so n_skip only climbs),
                // the reference breaks inside the window after the maximum: the
                // result is that maximum, and deeper j are never visited.
                bool done = false;
                if (a.lazy && (try_simple || i >= next_try)) {
                    int32_t bv = INT_MIN, bj = -1;
                    uint32_t nmk = 0;
                    bool cut = false;
                    for (int32_t jtop = i - 1; jtop >= lo && nmk <= (uint32_t)P.max_skip; jtop -= 64) {
                        const int32_t j = jtop - lane;
                        const bool inr = j >= lo;
                        int32_t pj, qj, fj, ppj;
                        if (jtop == i - 1) { pj = wp; qj = wq; fj = wf; ppj = wpp; }
                        else {
                            const bool deep = inr && j < ring_lo;
                            if (any(deep) && !drained) { vm_drain(); drained = true; }
                            uint64_t kj = 0;
                            int2 fpj = make_int2(0, -1);
                            if (inr) {
                                if (!deep) { kj = rkey[j & (RK - 1)]; fpj = rfp[j & (RK - 1)]; }
                                else { kj = K[CK(j, A)]; fpj = make_int2(F[CK(j, A)], PP[CK(j, A)]); }
                            }
                            pj = (int32_t)((kj >> qb) & rmask); qj = (int32_t)(kj & qmask); fj = fpj.x; ppj = fpj.y;
                        }
                        const int32_t dq = qi - qj, dr = pi - pj;
                        bool ok = inr && dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy;
                        const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
                        ok = ok && dd <= bw;
                        const int32_t dg = dr < dq ? dr : dq;
                        const int32_t sv = (span < dg ? span : dg) - (int32_t)lut[ok ? dd : 0] + fj;
                        const bool mk = ok && ppj >= lo;
                        nmk += (uint32_t)__popcll(ballot(mk));
                        const int32_t v = ok ? sv : INT_MIN;
                        const int32_t m = rdl(scan_max(v), 63);
                        if (m > bv) { bv = m; bj = jtop - ctz64(ballot(v == m)); }
                        cpairs += (uint64_t)__popcll(ballot(inr));
                        ++n_steps;
                        if (jtop == i - 1 && nmk > (uint32_t)P.max_skip && bv > span && i - 1 - bj <= P.max_skip) {
                            // marked lanes of this window (t[pprev[j]] = i from earlier lanes)
                            const int32_t tb = jtop - ppj;
                            const bool mk_in = mk && tb < 64;
                            const uint64_t mkM = ballot(mk_in);
                            uint64_t M = 0;
                            if (ballot(mk_in && tb != lane + 1) == 0) M = mkM << 1;
                            else {
                                const uint64_t tbit = mk_in ? (1ULL << (tb & 63)) : 0ULL;
                                M = ((uint64_t)wave_or32((uint32_t)(tbit >> 32)) << 32) | wave_or32((uint32_t)tbit);
                            }
                            const uint64_t after = ~0ULL << (i - bj);          // lanes after the maximum's
                            cut = (uint32_t)__popcll(ballot(ok) & M & after) > (uint32_t)P.max_skip;
                        }
                    }
                    done = nmk <= (uint32_t)P.max_skip || cut;
                    if (done && bv > span) { max_f = bv; max_j = bj; }
                    try_simple = done;
                    if (done) backoff = 16;
                    else { next_try = i + backoff; backoff = backoff < 128 ? 2 * backoff : 128; }
                }
                LP(pc_simple);
                if (PROF) { pn_done += done ? 1u : 0u; pn_exact += done ? 0u : 1u; }
                if (!done)
                for (int32_t jtop = i - 1; jtop >= lo; jtop -= 64) {
                    const int32_t j = jtop - lane;
                    const bool inr = j >= lo;
                    int32_t pj, qj, fj, ppj;
                    if (jtop == i - 1) { pj = wp; qj = wq; fj = wf; ppj = wpp; }
                    else {
                        const bool deep = inr && j < ring_lo;
                        const bool any_deep = any(deep);
                        n_deep += any_deep ? 1u : 0u;
                        if (any_deep && !drained) { vm_drain(); drained = true; }   // f/pprev flushes
                        uint64_t kj = 0;
                        int2 fpj = make_int2(0, -1);
                        if (inr) {
                            if (!deep) { kj = rkey[j & (RK - 1)]; fpj = rfp[j & (RK - 1)]; }
                            else { kj = K[CK(j, A)]; fpj = make_int2(F[CK(j, A)], PP[CK(j, A)]); }
                        }
                        pj = (int32_t)((kj >> qb) & rmask); qj = (int32_t)(kj & qmask); fj = fpj.x; ppj = fpj.y;
                    }
                    ++n_steps;
                    // comput_sc (lchain.rs:17-34)
                    const int32_t dq = qi - qj, dr = pi - pj;
                    bool ok = inr && dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy;
                    const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
                    ok = ok && dd <= bw;
                    const int32_t dg = dr < dq ? dr : dq;
                    const int32_t sc = (span < dg ? span : dg) - (int32_t)lut[ok ? dd : 0];
                    const int32_t sv = sc + fj;
                    // t[pprev[j]] = i  (lchain.rs:86); targets below lo are never read.
                    // Targets inside this step's window (j' in [jtop-63, jtop]) are a
                    // 64-bit mask built by a DPP OR-reduction; only targets below it
                    // (read by a later, deeper step) and marks of earlier steps use
                    // the LDS ring.
                    const bool mk = ok && ppj >= lo;
                    const int32_t tb = jtop - ppj;                 // target lane
                    const bool mk_in = mk && tb < 64;
                    // along a chain pprev[j] is usually j-1 (target lane l+1): then the
                    // mask is the marking lanes shifted by one, without the OR-reduction
                    const uint64_t mkM = ballot(mk_in);
                    uint64_t M = 0;
                    if (mkM) {
                        if (ballot(mk_in && tb != lane + 1) == 0) M = mkM << 1;
                        else {
                            const uint64_t tbit = mk_in ? (1ULL << (tb & 63)) : 0ULL;
                            M = ((uint64_t)wave_or32((uint32_t)(tbit >> 32)) << 32) | wave_or32((uint32_t)tbit);
                        }
                    }
                    // strict new maximum in processing order
                    const int32_t v = ok ? sv : INT_MIN;
                    const int32_t excl = shr1_dpp(scan_max(v), INT_MIN);
                    const int32_t pb = max_f > excl ? max_f : excl;
                    const bool nm = ok && sv > pb;
                    bool marked = ok && ((M >> lane) & 1ULL);
                    if (marks) marked = marked || (ok && ((ring[(j >> 5) & (RING_WORDS - 1)] >> (j & 31)) & 1u));
                    const bool plus = ok && !nm && marked;
                    const uint64_t nmM = ballot(nm), plusM = ballot(plus), inrM = ballot(inr);
                    uint64_t eff = ~0ULL, brkM = 0;
                    if (plusM) {
                        int32_t sa = nm ? -1 : (plus ? 1 : 0), sb = 0;
                        scan_nskip(sa, sb);
                        const int32_t na = (n_skip + sa) > sb ? (n_skip + sa) : sb;
                        brkM = ballot(plus && na > P.max_skip);
                        if (brkM) eff = lanemask_lt_of(ctz64(brkM));
                        else n_skip = rdl(na, 63);
                    } else {
                        n_skip -= __popcll(nmM);
                        n_skip = n_skip > 0 ? n_skip : 0;
                    }
                    const uint64_t nmm = nmM & eff;
                    if (nmm) { const int L = 63 - clz64(nmm); max_f = rdl(sv, L); max_j = jtop - L; }
                    cpairs += (uint64_t)__popcll(brkM ? (inrM & (eff | (1ULL << ctz64(brkM)))) : inrM);
                    if (brkM) break;
                    // Deeper predecessors can only change (f[i], pprev[i]) if one of them
                    // beats max_f (sv > max_f): marks and n_skip merely end the loop
                    // early.  A cheap scan of the whole deep window (no scans, no
                    // marks) settles most anchors of dense, unchained windows here.
                    if (a.lazy && jtop == i - 1 && jtop - 64 >= lo) {
                        bool cand = false;
                        for (int32_t jd = jtop - 64; jd >= lo && !cand; jd -= 64) {
                            const int32_t j = jd - lane;
                            const bool inr2 = j >= lo;
                            const bool deep = inr2 && j < ring_lo;
                            if (any(deep) && !drained) { vm_drain(); drained = true; }
                            uint64_t kj = 0; int32_t fj2 = 0;
                            if (inr2) {
                                if (!deep) { kj = rkey[j & (RK - 1)]; fj2 = rfp[j & (RK - 1)].x; }
                                else { kj = K[CK(j, A)]; fj2 = F[CK(j, A)]; }
                            }
                            const int32_t dq2 = qi - (int32_t)(kj & qmask), dr2 = pi - (int32_t)((kj >> qb) & rmask);
                            const int32_t dd2 = dr2 - dq2 < 0 ? dq2 - dr2 : dr2 - dq2;
                            const bool ok2 = inr2 && dq2 > 0 && dq2 <= maxdx && dr2 != 0 && dq2 <= maxdy && dd2 <= bw;
                            const int32_t dg2 = dr2 < dq2 ? dr2 : dq2;
                            const int32_t sv2 = (span < dg2 ? span : dg2) - (int32_t)lut[ok2 ? dd2 : 0] + fj2;
                            cand = any(ok2 && sv2 > max_f);
                        }
                        if (!cand) break;
                    }
                    // a deeper step follows: record this step's marks below its window
                    if (jtop - 64 >= lo) {
                        const bool mk_out = mk && !mk_in;
                        if (any(mk_out)) {
                            if (mk_out) atomicOr(&ring[(ppj >> 5) & (RING_WORDS - 1)], 1u << (ppj & 31));
                            marks = true;
                        }
                        wave_lds_sync();
                    }
                }
                LP(pc_exact);
                // clear this i's marks (all targets lie in [lo, i-1])
                if (marks) {
                    const int32_t w0 = lo >> 5, w1 = (i - 1) >> 5;
#pragma clang loop vectorize(disable) unroll(disable)
                    for (int32_t c0 = w0; c0 <= w1; c0 += 64) {
                        const int32_t wd = c0 + lane;
                        if (wd <= w1) ring[wd & (RING_WORDS - 1)] = 0;
                    }
                }
                if (lane == 0) rfp[i & (RK - 1)] = make_int2(max_f, max_j);
                wp = shr1_dpp(wp, pi); wq = shr1_dpp(wq, qi); wf = shr1_dpp(wf, max_f); wpp = shr1_dpp(wpp, max_j);
                LP(pc_tail);
            }
            wave_lds_sync();
            // flush f/pprev of the block; segment best (last index with max f)
            const int2 ev = rfp[il & (RK - 1)];
            if (valid) { F[CK(il, A)] = ev.x; PP[CK(il, A)] = ev.y; }
            const int32_t fv = valid ? ev.x : INT_MIN;
            const int32_t bm = rdl(scan_max(fv), 63);
            best_merge(best_f, best_i, bm, i0 + 63 - clz64(ballot(valid && fv == bm)));
        }
        if (lane == 0) {
            if (a.lseg_prof) a.lseg[q].w = (uint32_t)min<uint64_t>(wall_clock64() - seg_t0, 0x7fffffffull);   // MM2G_LSEG_PROF
            atomicMax(a.rbest + r, best_key(best_f, best_i));
            atomicAdd((unsigned long long*)&a.out[r].dp_pairs, (unsigned long long)cpairs);
            atomicAdd(&a.out[r].n_noniso, (uint32_t)(e - s - 1));
            atomicAdd(&a.out[r].n_steps, n_steps);
            if (PROF && a.gprof) {
                atomicAdd(&a.gprof[16], (unsigned long long)(e - s - 1)); atomicAdd(&a.gprof[17], (unsigned long long)pn_done);
                atomicAdd(&a.gprof[18], (unsigned long long)n_steps); atomicAdd(&a.gprof[19], (unsigned long long)pn_exact);
                atomicAdd(&a.gprof[20], (unsigned long long)pc_st); atomicAdd(&a.gprof[21], (unsigned long long)pc_simple);
                atomicAdd(&a.gprof[22], (unsigned long long)pc_exact); atomicAdd(&a.gprof[23], (unsigned long long)pc_tail);
                atomicAdd(&a.gprof[24], (unsigned long long)pn_spec); atomicAdd(&a.gprof[25], (unsigned long long)pn_rounds);
                if (t == 0) {   // the heaviest segment (lseg_order is longest first)
                    atomicAdd(&a.gprof[26], (unsigned long long)pn_spec); atomicAdd(&a.gprof[27], (unsigned long long)pn_rounds);
                    atomicAdd(&a.gprof[28], (unsigned long long)(pn_done + pn_exact));
                    atomicAdd(&a.gprof[29], (unsigned long long)(pc_st + pc_simple + pc_exact + pc_tail));
                    atomicAdd(&a.gprof[30], (unsigned long long)pc_spec); atomicAdd(&a.gprof[31], (unsigned long long)(clock64() - pc_seg0));
                }
            }
        }
    }
#undef LP
}

// ---- 5b'. giant segments (production only): chain_dp_all (lchain.rs:73-90)
// as a policy-iteration fixed point.  When no window holds more than max_skip
// mark sources (valid j with pprev[j] >= lo), no n_skip break can happen and
// the reference's loop is the plain running maximum in visiting order:
//   f[i] = max(span, max_{j in [lo_i, i-1], valid} f[j] + sc(i, j)),
//   pprev[i] = the first visited (largest) j reaching it (when > span).
// Only j < i appear, so the recurrence has one solution.  Plain value
// iteration needs (longest chain) rounds; policy iteration -- evaluate the
// current predecessor forest by pointer doubling, then re-pick predecessors --
// needs a handful even for chains thousands of anchors deep, each round
// parallel over anchors instead of one dependent 64-lane step per anchor.
// A segment that does not settle in GIANT_IT rounds or violates the mark
// bound is left to k_chain_long.
constexpr int GIANT_MAX = 4096;   // anchors per segment, at most (4 per thread)
constexpr int GIANT_B = 34;       // LDS per anchor: key 8 B, f/val/pprev/ptr/children/next-pprev 6 x 4 B, lo 2 B
// segment capacity left beside the pen LUT in 160 KB of LDS (1 KB for statics)
__host__ __device__ inline int giant_cap(int lut_n) {
    const int c = (160 * 1024 - 1024 - (((lut_n * 2) + 15) & ~15)) / GIANT_B;
    return (c < GIANT_MAX ? c : GIANT_MAX) & ~15;
}
constexpr int GIANT_GB = 42;      // HBM scratch per anchor (global variant): + ping-pong val/ptr 2 x 4 B
constexpr int GIANT_IT = 32;
constexpr int GIANT_PINS = 32;    // exactly evaluated anchors per segment before giving up
constexpr int GIANT_MKW = 160;    // mark bitmap words (window <= max_iter 5000)
// G = false: the segment lives in LDS (len <= giant_cap).  G = true: longer
// segments (the 100 kb rescue's) in a per-workgroup HBM/L2 scratch slice of
// a.giant_gmax anchors; same algorithm, pointer doubling by ping-pong.
template <bool G>
__global__ __launch_bounds__(1024) void k_chain_giant(ChainArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ uint32_t s_flag;
    __shared__ unsigned long long s_best;
    __shared__ uint32_t s_mk[GIANT_MKW];
    __shared__ uint32_t s_red[16];
    const ChainKParams P = a.P;
    int16_t* lut = (int16_t*)smem;
    const int lut_bytes = ((P.lut_n * 2) + 15) & ~15;
    const int gcap = a.giant_lcap ? min(giant_cap(P.lut_n), (int)a.giant_lcap) : giant_cap(P.lut_n);
    const int cap = G ? (int)a.giant_gmax : gcap;
    unsigned char* arr = G ? (unsigned char*)a.giant_scr + (size_t)blockIdx.x * (size_t)cap * GIANT_GB : smem + lut_bytes;
    uint64_t* gk = (uint64_t*)arr;
    int32_t* f0 = (int32_t*)(gk + cap);
    int32_t* f1 = f0 + cap;
    int32_t* gp = f1 + cap;
    int32_t* gptr = gp + cap;
    int32_t* gch = gptr + cap;
    int32_t* gnp = gch + cap;                   // exact mode: the next policy
    uint16_t* glo = (uint16_t*)(gnp + cap);
    int32_t* val2 = (int32_t*)(glo + cap);      // G only
    int32_t* gptr2 = val2 + cap;
    const int tid = threadIdx.x;
    const uint32_t nl = min(*a.lseg_n, a.lseg_cap);
    if constexpr (G) {   // most workgroups have no segment over the LDS capacity: leave before the LUT load
        bool mine = false;
        for (uint32_t q = blockIdx.x; q < nl && !mine; q += gridDim.x) {
            const int32_t len = (int32_t)a.lseg[q].z - (int32_t)a.lseg[q].y;
            mine = len > gcap && len <= cap && len >= (int32_t)a.giant_min;
        }
        if (!mine) return;
    }
    load_lut(lut, a.lut, P.lut_n);
    __syncthreads();
    const uint32_t qb = a.kl.qb, rb = a.kl.rb;
    const uint64_t qmask = (1ULL << qb) - 1, rmask = (1ULL << rb) - 1;
    const int32_t maxdx = P.max_dist_x, maxdy = P.max_dist_y, bw = P.bw, span = P.span;
    // LDS variant: workgroups take segments longest first (k_lseg_order) from a
    // shared counter, so the long ones start early and no workgroup is left with
    // a tail of them (static striding left the slowest workgroup ~2.7x the mean)
    __shared__ uint32_t s_q;
    for (uint32_t qi = blockIdx.x;; qi += gridDim.x) {
        uint32_t q;
        if constexpr (G) {
            if (qi >= nl) break;
            q = qi;
        } else {
            if (tid == 0) s_q = atomicAdd(&a.work[P.pass & 1], 1u);
            __syncthreads();
            const uint32_t t = s_q;
            __syncthreads();
            if (t >= nl) break;
            q = a.lseg_order[t];
        }
        const uint4 L = a.lseg[q];
        const int32_t s = (int32_t)L.y, e = (int32_t)L.z, len = e - s;
        if (len < (int32_t)a.giant_min || (G ? (len <= gcap || len > cap) : len > gcap)) continue;
        const uint32_t r = L.x;
        const uint64_t base = a.a_off[r];
        const uint64_t* K = a.keys + base;
        const uint64_t g_t0 = a.lseg_prof ? wall_clock64() : 0;
        int g_its = 0;
        uint64_t gl = g_t0;   // MM2G_LSEG_PROF phase sums (thread 0, after barriers)
#define GP(k) do { if (a.gprof && tid == 0) { const uint64_t t_ = wall_clock64(); atomicAdd(&a.gprof[k], (unsigned long long)(t_ - gl)); gl = t_; } } while (0)
        for (int t = tid; t < len; t += 1024) { gk[t] = K[s + t]; f0[t] = span; }
        __syncthreads();
        // window start (lchain.rs:75-77): first j with p_i <= p_j + max_dist_x, and max_iter
        for (int t = tid; t < len; t += 1024) {
            const int32_t pi = (int32_t)((gk[t] >> qb) & rmask);
            int32_t lo = 0, hi = t;            // first j in [0, t] with p_j >= p_i - maxdx
            while (lo < hi) { const int32_t mid = (lo + hi) >> 1; if (pi > (int32_t)((uint32_t)((gk[mid] >> qb) & rmask) + (uint32_t)maxdx)) lo = mid + 1; else hi = mid; }
            const int32_t l2 = lo > t - P.max_iter ? lo : t - P.max_iter;
            glo[t] = (uint16_t)min(t - l2, 65535);
        }
        __syncthreads();
        GP(0);
        auto sc_of = [&](uint64_t ki, uint64_t kj, bool& ok) -> int32_t {   // comput_sc (lchain.rs:17-34)
            const int32_t dq = (int32_t)(ki & qmask) - (int32_t)(kj & qmask);
            const int32_t dr = (int32_t)((ki >> qb) & rmask) - (int32_t)((kj >> qb) & rmask);
            const int32_t dd = dr - dq < 0 ? dq - dr : dr - dq;
            ok = dq > 0 && dq <= maxdx && dr != 0 && dq <= maxdy && dd <= bw;
            const int32_t dg = dr < dq ? dr : dq;
            return (span < dg ? span : dg) - (int32_t)lut[ok ? dd : 0];
        };
        // Rounds: Jacobi to convergence, then the mark-bound check.  The first
        // anchor that fails it gets the reference loop exactly (one thread,
        // marks in an LDS bitmap, its predecessors being exact already) and is
        // pinned; the next round re-converges the anchors after it.
        for (int t = tid; t < len; t += 1024) gp[t] = -1;
        int32_t* fo = f0; int32_t* val = f1;
        int dbl = 0;
        while ((1 << dbl) < len) ++dbl;
        // f of the forest gp (pinned anchors keep fo): pointer doubling; returns
        // the array holding the values (fo itself is not written)
        auto eval_forest = [&]() -> const int32_t* {
            for (int t = tid; t < len; t += 1024) {
                const int32_t p = gp[t];
                if ((glo[t] & 0x8000u) || p < 0) { val[t] = (glo[t] & 0x8000u) ? fo[t] : span; gptr[t] = -1; }
                else { bool ok; val[t] = sc_of(gk[t], gk[p], ok); gptr[t] = p; }
            }
            __syncthreads();
            const int32_t* vres = val;
            if constexpr (G) {
                int32_t *v0 = val, *p0 = gptr, *v1 = val2, *p1 = gptr2;
                for (int d = 0; d < dbl; ++d) {
                    bool live = false;
                    for (int t = tid; t < len; t += 1024) {
                        const int32_t p = p0[t];
                        v1[t] = p >= 0 ? v0[t] + v0[p] : v0[t];
                        const int32_t np = p >= 0 ? p0[p] : -1;
                        p1[t] = np;
                        live = live || np >= 0;
                    }
                    const bool more = __syncthreads_or(live);   // every pointer at a root: the forest's depth is reached
                    int32_t* tv = v0; v0 = v1; v1 = tv;
                    int32_t* tp = p0; p0 = p1; p1 = tp;
                    if (!more) break;
                }
                vres = v0;
            } else {
                // rounds stop once every pointer has reached a root (the forest's
                // depth, not its size, sets their number: shallow forests settle
                // in a few)
                for (int d = 0; d < dbl; ++d) {
                    int32_t nv[4], np[4];
                    bool live = false;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int t = tid + k * 1024;
                        if (t < len) {
                            const int32_t p = gptr[t];
                            nv[k] = p >= 0 ? val[t] + val[p] : val[t];
                            np[k] = p >= 0 ? gptr[p] : -1;
                            live = live || np[k] >= 0;
                        }
                    }
                    __syncthreads();
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int t = tid + k * 1024;
                        if (t < len) { val[t] = nv[k]; gptr[t] = np[k]; }
                    }
                    if (!__syncthreads_or(live)) break;
                }
            }
            return vres;
        };
        // Children lists of the forest gp: j is marked for i (t[j] == i) iff a
        // valid c in (j, i) has pprev[c] == j.  gptr = child counts, val = list
        // ends, gch = the lists.  Ends without a barrier.
        auto build_children = [&]() {
            for (int t = tid; t < len; t += 1024) gptr[t] = 0;
            __syncthreads();
            for (int t = tid; t < len; t += 1024) if (gp[t] >= 0) atomicAdd((uint32_t*)&gptr[gp[t]], 1u);
            __syncthreads();
            for (int c0 = 0, carry = 0; c0 < len; c0 += 4096) {   // exclusive scan, 4096 per pass
                uint32_t c4[4], sum = 0, tot;
#pragma unroll
                for (int k = 0; k < 4; ++k) { const int t = c0 + tid * 4 + k; c4[k] = t < len ? (uint32_t)gptr[t] : 0u; sum += c4[k]; }
                uint32_t ex = block_excl_sum(sum, tot, s_red) + (uint32_t)carry;
#pragma unroll
                for (int k = 0; k < 4; ++k) { const int t = c0 + tid * 4 + k; if (t < len) val[t] = (int32_t)ex; ex += c4[k]; }
                carry += (int)tot;
            }
            __syncthreads();
            for (int t = tid; t < len; t += 1024) if (gp[t] >= 0) gch[atomicAdd((uint32_t*)&val[gp[t]], 1u)] = t;
        };
        // marked(j) for anchor t with key ki
        auto marked = [&](int32_t j, int32_t t, uint64_t ki) -> bool {
            const int32_t ce = val[j];
            for (int32_t c = ce - gptr[j]; c < ce; ++c) {
                const int32_t cj = gch[c];
                if (cj < t) { bool okc; (void)sc_of(ki, gk[cj], okc); if (okc) return true; }
            }
            return false;
        };
        bool ok_seg = false;
        if (a.giant_exact) {
            // Pass 0 (real chains, marks everywhere): policy iteration on the
            // reference loop itself (lchain.rs:78-87, n_skip and break, marks from
            // the current forest's children).  Each anchor depends only on
            // earlier ones, so a forest that the loop reproduces everywhere, with
            // its evaluated values, is the reference's solution.
            bool conv = false;
            for (int it = 0; it < GIANT_IT && !conv; ++it) {
                build_children();
                if (tid == 0) s_flag = 0;
                __syncthreads();
                uint32_t ch = 0;
                for (int t = tid; t < len; t += 1024) {
                    const uint64_t ki = gk[t];
                    const int32_t lo = t - (int32_t)glo[t];
                    int32_t mf = span, mj = -1, n_skip = 0;
                    for (int32_t j = t - 1; j >= lo; --j) {
                        bool ok;
                        const int32_t sv = sc_of(ki, gk[j], ok) + fo[j];
                        if (!ok) continue;
                        if (sv > mf) { mf = sv; mj = j; if (n_skip > 0) --n_skip; continue; }
                        if (marked(j, t, ki) && ++n_skip > P.max_skip) break;
                    }
                    gnp[t] = mj;
                    ch |= (mf != fo[t] || mj != gp[t]) ? 1u : 0u;
                }
                if (ch) atomicOr(&s_flag, 1u);
                __syncthreads();
                conv = s_flag == 0;
                ++g_its;
                if (!conv) {
                    for (int t = tid; t < len; t += 1024) gp[t] = gnp[t];
                    __syncthreads();
                    const int32_t* vres = eval_forest();
                    for (int t = tid; t < len; t += 1024) fo[t] = vres[t];
                }
                __syncthreads();
            }
            ok_seg = conv;
        } else
        for (int round = 0; round < GIANT_PINS; ++round) {
            // Policy iteration: evaluate the current predecessor forest exactly
            // (pointer doubling, ceil(log2 len) rounds), then let every anchor
            // re-pick its best predecessor (reference order, strict >) under
            // those values.  Values never decrease; when no anchor's value
            // changes they are the DP's fixed point and gp is its argmax.
            bool conv = false;
            for (int it = 0; it < GIANT_IT && !conv; ++it) {
                const int32_t* vres = eval_forest();
                GP(1);
                if (tid == 0) s_flag = 0;
                // Values that moved in this evaluation, as a prefix count (gch is free
                // until the children lists).  An anchor none of whose predecessors
                // moved keeps its argmax, and its own value already equals that
                // maximum: the improvement skips it (after the first iteration).
                // The moved anchors themselves are listed in gptr (free until the
                // children lists) in index order.
                for (int c0 = 0, carry = 0; c0 < len; c0 += 4096) {
                    uint32_t c4[4], sum = 0, tot;
#pragma unroll
                    for (int k = 0; k < 4; ++k) { const int t = c0 + tid * 4 + k; c4[k] = (t < len && vres[t] != fo[t]) ? 1u : 0u; sum += c4[k]; }
                    uint32_t ex = block_excl_sum(sum, tot, s_red) + (uint32_t)carry;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int t = c0 + tid * 4 + k;
                        if (t < len) { gch[t] = (int32_t)ex; if (c4[k]) gptr[ex] = t; fo[t] = vres[t]; }
                        ex += c4[k];
                    }
                    carry += (int)tot;
                }
                __syncthreads();
                GP(2);
                uint32_t ch = 0;
                for (int t = tid; t < len; t += 1024) {
                    const uint32_t lw = glo[t];
                    if (lw & 0x8000u) continue;          // pinned: exact already
                    const uint64_t ki = gk[t];
                    const int32_t lo = t - (int32_t)lw;
                    int32_t mf = span, mj = -1;
                    if (it == 0) {
                        for (int32_t j = t - 1; j >= lo; --j) {
                            bool ok;
                            const int32_t sv = sc_of(ki, gk[j], ok) + fo[j];
                            if (ok && sv > mf) { mf = sv; mj = j; }
                        }
                    } else {
                        // Incremental: within a round values only rise (each policy is
                        // greedy on its predecessor's values), so the previous argmax
                        // J, now worth fo[t] = sc(t, J) + fo[J], still dominates every
                        // window anchor whose value did not move; only the moved ones
                        // can overtake it.  Same (value, visiting-order) maximum as the
                        // full scan: strict > in decreasing j, the root (-1) first.
                        const int32_t c1 = gch[t], cl = gch[lo];
                        if (c1 == cl) continue;
                        mf = fo[t]; mj = gp[t];
                        for (int32_t c = c1 - 1; c >= cl; --c) {
                            const int32_t j = gptr[c];
                            bool ok;
                            const int32_t sv = sc_of(ki, gk[j], ok) + fo[j];
                            if (ok && (sv > mf || (sv == mf && mj >= 0 && j > mj))) { mf = sv; mj = j; }
                        }
                        ch |= mf != fo[t] ? 1u : 0u;
                        gp[t] = mj;
                        continue;
                    }
                    gp[t] = mj;
                    ch |= mf != fo[t] ? 1u : 0u;
                }
                if (ch) atomicOr(&s_flag, 1u);
                __syncthreads();
                conv = s_flag == 0;
                ++g_its;
                __syncthreads();
                GP(3);
            }
            if (!conv) break;                    // k_chain_long runs it
            // Children lists of the converged forest: j is marked for i (t[j]
            // == i) iff a valid c in (j, i) has pprev[c] == j.  gptr = child
            // counts, val = list ends, gch = the lists.
            build_children();
            __syncthreads();
            GP(4);
            // No break is possible where a window holds <= max_skip mark
            // sources.  Elsewhere run the reference loop on the converged
            // values: the first anchor where it disagrees is pinned below.
            if (tid == 0) s_flag = 0x7fffffffu;
            __syncthreads();
            for (int t = tid; t < len; t += 1024) {
                const uint32_t lw = glo[t];
                if (lw & 0x8000u) continue;
                const uint64_t ki = gk[t];
                const int32_t lo = t - (int32_t)lw;
                int32_t nmk = 0;
                for (int32_t j = t - 1; j >= lo && nmk <= P.max_skip; --j) {
                    bool ok;
                    (void)sc_of(ki, gk[j], ok);
                    nmk += (ok && gp[j] >= lo) ? 1 : 0;
                }
                if (nmk <= P.max_skip) continue;
                int32_t mf = span, mj = -1, n_skip = 0;
                for (int32_t j = t - 1; j >= lo; --j) {
                    bool ok;
                    const int32_t sv = sc_of(ki, gk[j], ok) + fo[j];
                    if (!ok) continue;
                    if (sv > mf) { mf = sv; mj = j; if (n_skip > 0) --n_skip; continue; }
                    if (marked(j, t, ki) && ++n_skip > P.max_skip) break;
                }
                if (mf != fo[t] || mj != gp[t]) atomicMin(&s_flag, (uint32_t)t);
            }
            __syncthreads();
            GP(5);
            const uint32_t tf = s_flag;
            if (tf == 0x7fffffffu) {
                ok_seg = true;
                break;
            }
            if (tid == 0) {   // the reference loop (lchain.rs:78-87) for anchor tf
                const int32_t t = (int32_t)tf, lo = t - (int32_t)glo[t];
                const int32_t nw = (t - lo + 31) >> 5;
                for (int32_t w = 0; w < nw; ++w) s_mk[w] = 0;   // marks t[j] == i, j in [lo, t)
                const uint64_t ki = gk[t];
                int32_t mf = span, mj = -1, n_skip = 0;
                for (int32_t j = t - 1; j >= lo; --j) {
                    bool ok;
                    const int32_t sv = sc_of(ki, gk[j], ok) + fo[j];
                    if (!ok) continue;
                    if (sv > mf) { mf = sv; mj = j; if (n_skip > 0) --n_skip; }
                    else if ((s_mk[(j - lo) >> 5] >> ((j - lo) & 31)) & 1u) { if (++n_skip > P.max_skip) break; }
                    const int32_t pj = gp[j];
                    if (pj >= lo) s_mk[(pj - lo) >> 5] |= 1u << ((pj - lo) & 31);
                }
                fo[t] = mf; gp[t] = mj; glo[t] = (uint16_t)(glo[t] | 0x8000u);
            }
            __syncthreads();
            GP(6);
            if (a.gprof && tid == 0) atomicAdd(&a.gprof[11], 1ull);
        }
        if (a.gprof && tid == 0) {
            atomicAdd(&a.gprof[8], 1ull); atomicAdd(&a.gprof[9], (unsigned long long)len); atomicAdd(&a.gprof[10], (unsigned long long)g_its);
            atomicAdd(&a.gprof[12], (unsigned long long)(wall_clock64() - g_t0)); if (!ok_seg) atomicAdd(&a.gprof[13], 1ull);
        }
        if (!ok_seg) continue;
        if (tid == 0) s_best = 0;
        __syncthreads();
        uint64_t pairs = 0;
        for (int t = tid; t < len; t += 1024) { glo[t] &= 0x7fffu; pairs += glo[t]; }
        int32_t* F = a.f + base; int32_t* PP = a.pp + base;
        int32_t bf = INT_MIN, bi = -1;
        for (int t = tid; t < len; t += 1024) {
            F[s + t] = fo[t];
            PP[s + t] = gp[t] >= 0 ? s + gp[t] : -1;
            best_merge(bf, bi, fo[t], s + t);
        }
        // one LDS / global atomic per wave, not per thread (same-address atomics serialize)
        uint64_t bk = bi >= 0 ? best_key(bf, bi) : 0ull;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) { const uint64_t o = __shfl_xor(bk, d, 64); bk = o > bk ? o : bk; }
        pairs = wave_sum64(pairs);
        if (lane_id() == 0) {
            if (bk) atomicMax(&s_best, bk);
            if (pairs) atomicAdd((unsigned long long*)&a.out[r].dp_pairs, (unsigned long long)pairs);
        }
        __syncthreads();
        if (tid == 0) {
            atomicMax(a.rbest + r, s_best);
            a.lseg[q].w = LSEG_DONE | (a.lseg_prof ? (uint32_t)min<uint64_t>(wall_clock64() - g_t0, 0x7fffffffull) : 0u);
        }
        // LDS-only barrier: the next segment may reuse the LDS arrays, but the
        // global stores above need not have landed (a full __syncthreads would
        // wait for them)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        GP(7);
#undef GP
    }
}

// ---- 5c. per read: fallback chain walk (lchain.rs:162-171), chain_qrange /
// chain_trange (178-200) and the rescue test of rescue_long_join (316-330).
constexpr int FIN_CH = 2048;   // pprev entries staged per wave (LDS) for the chain walk
__global__ __launch_bounds__(256) void k_chain_fin(ChainArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    // one wave per read; the pprev walk reads chunks of FIN_CH entries staged in
    // LDS (coalesced) instead of one dependent HBM load per chain anchor
    __shared__ int32_t s_pp[4][FIN_CH];
    const int lane = lane_id(), wv = wave_id();
    const uint32_t r = blockIdx.x * 4 + (uint32_t)wv;
    if (r >= a.n) return;
    int32_t* spp = s_pp[wv];
    const ChainKParams P = a.P;
    ReadOut* O = a.out + r;
    const int32_t flags0 = uni(O->flags);
    if (P.pass == 1 && !(flags0 & RF_RESCUED)) return;
    const uint64_t base = uni64(a.a_off[r]);
    const int32_t A = (int32_t)(uni64(a.a_off[r + 1]) - base);
    const int32_t qlen = (int32_t)(uni64(a.rd_off[r + 1]) - uni64(a.rd_off[r]));
    if (A == 0) {
        if (lane == 0) {
            O->flags = flags0 & RF_EMPTY; O->n_anchors = 0; O->score = 0; O->cm = 0;
            O->qs = O->qe = O->ts = O->te = 0; O->group = 0; O->best_i = -1; O->qlen = qlen;
        }
        return;
    }
    const uint32_t qb = a.kl.qb, rb = a.kl.rb;
    const uint64_t qmask = (1ULL << qb) - 1, rmask = (1ULL << rb) - 1;
    const uint32_t gsh = rb + qb;
    const int32_t span = P.span;
    const int32_t A2 = (int32_t)uni((int32_t)a.cnt2[r]);     // anchors in the DP (singleton filter)
    const uint64_t sm = uni64(a.smax[r]);                   // 1 + largest dropped key, 0 = none
    uint64_t* K = (uint64_t*)a.keys + base;       // writable: slot A2 receives a dropped best
    const int32_t* PP = a.pp + base;
    uint32_t* CB = a.chain + base;
    int32_t best_f = span, best_i = -1;
    if (A2 > 0) {
        const unsigned long long bk = uni64(a.rbest[r]);
        best_f = (int32_t)((uint32_t)(bk >> 32) ^ 0x80000000u); best_i = (int32_t)(uint32_t)bk;
    }
    // "last argmax f" over all anchors: a dropped singleton (f = span) wins when
    // every kept anchor also has f == span and its key is the largest
    const bool single = sm != 0 && (A2 == 0 || (best_f == span && sm - 1 > uni64(K[CK(A2 - 1, A)])));
    int32_t root, cm = 0;
    if (single) {
        if (lane == 0) { K[CK(A2, A)] = sm - 1; CB[0] = (uint32_t)A2; }   // slot A2 is free (A2 < A); k_dv reads it via CB
        cm = 1; root = A2; best_i = A2; best_f = span;
    } else {
        // fallback chain walk (lchain.rs:162-171), wave-uniform
        int32_t idx = best_i;
        root = best_i;
        while (idx >= 0 && cm < A2) {
            const int32_t lo_c = idx - FIN_CH + 1 > 0 ? idx - FIN_CH + 1 : 0;
            for (int32_t t = lo_c + lane; t <= idx; t += 64) spp[t - lo_c] = PP[CK(t, A)];
            wave_lds_sync();
            // up to 64 links per step: lane l looks at anchor idx - l; while the links are
            // consecutive (pprev[t] == t - 1, the usual case along a chain) the walk passes
            // them all at once, and the first other link continues it
            while (idx >= lo_c && cm < A2) {
                const int32_t t = idx - lane;
                const bool in = t >= lo_c;
                const int32_t pt = in ? spp[t - lo_c] : -1;
                const uint64_t nl = ballot(!(in && pt == t - 1));
                int32_t cnt, nxt;
                if (nl == 0ULL) { cnt = 64; nxt = idx - 64; }
                else {
                    const int32_t m = (int32_t)ctz64(nl);
                    const bool min_ = idx - m >= lo_c;             // lane m's anchor is staged: it is on the chain
                    cnt = min_ ? m + 1 : m;
                    nxt = min_ ? __shfl(pt, m, 64) : idx - m;       // (idx - m = lo_c - 1: restaged below)
                }
                cnt = min(cnt, A2 - cm);
                if (lane < cnt) CB[cm + lane] = (uint32_t)(idx - lane);
                cm += cnt; root = idx - (cnt - 1);
                idx = uni(nxt);
            }
            wave_lds_sync();
        }
    }
    if (lane != 0) return;
    const uint64_t kb = K[CK(best_i, A)], kr = K[CK(root, A)];
    const uint32_t g = (uint32_t)(kb >> gsh);
    const int32_t qe = (int32_t)(kb & qmask) + 1;
    int32_t qs = (int32_t)(kr & qmask) - (span - 1); if (qs < 0) qs = 0;
    int32_t ts, te;
    if (g == 2u * a.kl.n_seq) {
        // Q19: rpos = (x as i32) = p - 2^31 < 0 (paf.rs:133-145, wrapping i32).
        // te starts at -1 and only rpos + 1 > -1 raises it.  rpos - (span-1)
        // wraps to a large positive value exactly when p < span-1; p rises
        // along the chain, so the minimum is negative (ts clamps to 0) unless
        // every anchor wraps, and then it is the root's.
        const uint32_t pb = (uint32_t)((kb >> qb) & rmask), pr = (uint32_t)((kr >> qb) & rmask);
        te = max(-1, (int32_t)(pb | 0x80000000u) + 1);
        ts = pb >= (uint32_t)(span - 1) ? 0 : (int32_t)(0x80000000u + pr - (uint32_t)(span - 1));
    }
    else {
        te = (int32_t)((kb >> qb) & rmask) + 1;
        ts = (int32_t)((kr >> qb) & rmask) - (span - 1); if (ts < 0) ts = 0;
    }
    int32_t fl = RF_MAPPED | (flags0 & RF_RESCUED);
    if (g == 2u * a.kl.n_seq) fl |= RF_PANIC;
    if (P.pass == 0) {
        // rescue_long_join tests chains[0] (lchain.rs:321-326): the fallback chain, or under P.multi the
        // best one-anchor backtrack chain, whose coverage is the span
        int32_t cov = P.multi ? span : qe - qs; if (cov < 0) cov = 0;
        int32_t unc = qlen - cov; if (unc < 0) unc = 0;
        if (unc > P.rescue_size || (float)cov < (float)qlen * P.rescue_ratio_f) fl |= RF_RESCUED;
    }
    O->flags = fl; O->n_anchors = A; O->qlen = qlen;
    O->score = best_f; O->cm = cm; O->qs = qs; O->qe = qe; O->ts = ts; O->te = te;
    O->group = (int32_t)g; O->best_i = best_i;
}

// order[t] = reads heaviest first (a counting sort on buckets of 512 anchors,
// descending): the hand-out order of the per-read sort and of the chain work
// items (longest-processing-time first, so the heaviest reads do not form the
// kernels' tails; exact LPT is not needed).  Block-wide.
DEVI void read_order_block(uint32_t n, const uint32_t* a_cnt, uint32_t* order, uint32_t* hist, uint32_t* s_sc) {
    constexpr int NB = 1024;
    const int tid = threadIdx.x;
    hist[tid] = 0;
    __syncthreads();
    auto bucket = [](uint32_t c) -> int { const uint32_t b = c >> 9; return NB - 1 - (int)(b < (uint32_t)NB - 1 ? b : (uint32_t)NB - 1); };
    for (uint32_t r = tid; r < n; r += 1024) atomicAdd(&hist[bucket(a_cnt[r])], 1u);
    __syncthreads();
    uint32_t tot;
    const uint32_t ex = block_excl_sum(hist[tid], tot, s_sc);
    __syncthreads();
    hist[tid] = ex;
    __syncthreads();
    for (uint32_t r = tid; r < n; r += 1024) order[atomicAdd(&hist[bucket(a_cnt[r])], 1u)] = r;
}

__global__ __launch_bounds__(1024) void k_read_order(uint32_t n, const uint32_t* a_cnt, uint32_t* order) {
    __shared__ uint32_t hist[1024], s_sc[16];
    read_order_block(n, a_cnt, order, hist, s_sc);
}

// 6. dv inputs — paf_from_chain_with_primary (src/paf.rs:156-199): binary
// search (Rust >= 1.82 slice::binary_search) of the first chain position among
// the minimizer positions of the (idx.w, idx.k) sketch, then the greedy match.
// ============================================================================

constexpr int DV_LDS = 4096;   // minimizer positions staged per read (longer reads read HBM)
__global__ __launch_bounds__(64) void k_dv(DvArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;   // anchor workspace too small: the host re-runs the batch
    __shared__ int32_t Ps[DV_LDS];
    const uint32_t r = blockIdx.x;
    if (r >= a.n) return;
    const int lane = lane_id();
    const int32_t flags = uni(a.out[r].flags), cm = uni(a.out[r].cm);
    const uint32_t m = (uint32_t)uni((int32_t)a.mz_cnt[r]);
    const bool go = (flags & RF_MAPPED) && !(flags & RF_PANIC) && m > 0 && cm > 0;
    if (!go) {
        if (lane == 0) { a.out[r].m_dv = (int32_t)m; a.out[r].flags = flags & ~RF_DV_FOUND; }
        return;
    }
    const uint64_t mzb = uni64(a.mz_base[r]), ab = uni64(a.a_off[r]);
    const uint64_t An = uni64(a.a_off[r + 1]) - ab;
    (void)An;
    const uint32_t* Y = a.mz_y + mzb;
    const uint32_t* CB = a.chain + ab;
    const uint64_t* K = a.keys + ab;
    const uint64_t qmask = (1ULL << a.kl.qb) - 1;
    const bool rev = (uint32_t)uni(a.out[r].group) >= a.kl.n_seq;
    const int32_t qlen = uni(a.out[r].qlen), span = a.span;
    const bool in_lds = m <= (uint32_t)DV_LDS;
    if (in_lds) {
        for (uint32_t j0 = 0; j0 < m; j0 += 64) { const uint32_t j = j0 + lane; if (j < m) Ps[j] = (int32_t)(Y[j] >> 1); }
        __syncthreads();
    }
    if (a.strict && !in_lds && m <= a.long_m) return;   // k_dv_long (a workgroup per read)
    auto mpos = [&](uint32_t j) -> int32_t { return in_lds ? Ps[j] : (int32_t)(Y[CK(j, m)] >> 1); };
    // t-th chain anchor in forward-query order (paf.rs:165-176)
    auto fwdq = [&](int32_t t) -> int32_t {
        if (!rev) return (int32_t)(K[CK(CB[cm - 1 - t], An)] & qmask);
        const int32_t q = (int32_t)(K[CK(CB[t], An)] & qmask);
        return qlen - 1 - (q + 1 - span);
    };
    const int32_t first = uni(fwdq(0));
    // Rust >= 1.82 slice::binary_search (base/size halving, no early exit) (paf.rs:178)
    uint32_t size = m, b = 0;
    while (size > 1) { const uint32_t half = size / 2, mid = b + half; if (!(uni(mpos(mid)) > first)) b = mid; size -= half; }
    if (uni(mpos(b)) != first) {
        if (lane == 0) { a.out[r].m_dv = (int32_t)m; a.out[r].flags = flags & ~RF_DV_FOUND; }
        return;
    }
    uint32_t st = b;
    while (st > 0 && uni(mpos(st - 1)) == first) --st;
    uint32_t j = st, en = st;
    int32_t n_match = 1;
    if (a.strict) {
        // Strictly increasing P (odd index k) and chain positions (dq > 0 along a
        // chain): the greedy walk (paf.rs:179-186) matches C[kk] exactly where P holds it, and
        // stops matching at the first C[kk] that P lacks.  So each lane finds its C[kk] by a
        // lower-bound search (64 chain anchors at a time, the same halving steps for every lane),
        // and the first lane that misses ends the matches.
        for (int32_t kb = 1; kb < cm; kb += 64) {
            const int32_t t = kb + lane;
            const bool tv = t < cm;
            const int32_t v = tv ? fwdq(t) : INT_MAX;
            uint32_t b0 = 0, sz = m;
            while (sz > 1) { const uint32_t half = sz / 2; if (mpos(b0 + half) < v) b0 += half; sz -= half; }
            const uint32_t ix = b0 + (mpos(b0) < v ? 1u : 0u);
            const bool hit = tv && ix < m && mpos(ix < m ? ix : 0) == v;
            const uint64_t miss = ballot(tv && !hit);
            const int32_t nv = min(64, cm - kb);
            const int32_t lim = miss ? ctz64(miss) : nv;
            if (lim > 0) { n_match += lim; en = (uint32_t)rdl((int32_t)ix, lim - 1); }
            if (miss) break;
        }
    } else {
    // greedy match (paf.rs:179-186): the next j with P[j] == C[kk].  A window of
    // 64 positions after j sits in registers; successive targets are matched in
    // it by ballot (each after the previous match) until one is not there, and
    // then the window moves past its end.
    int32_t kk = 1, kb = 1;
    int32_t cv = (kb + lane < cm) ? fwdq(kb + lane) : 0;
    while (kk < cm && j + 1 < m) {
        const uint32_t c0 = j + 1;
        const uint32_t jl = c0 + (uint32_t)lane;
        const int32_t pv = jl < m ? mpos(jl) : 0;
        uint64_t avail = ballot(jl < m);
        while (kk < cm) {
            if (kk - kb >= 64) { kb = kk; cv = (kb + lane < cm) ? fwdq(kb + lane) : 0; }
            const int32_t target = rdl(cv, kk - kb);
            const uint64_t hit = ballot(pv == target) & avail;
            if (!hit) break;
            const int L = ctz64(hit);
            j = c0 + (uint32_t)L; ++n_match; en = j; ++kk;
            avail &= L == 63 ? 0ULL : ~((2ULL << L) - 1ULL);
        }
        if (kk < cm) j = (c0 + 63 < m - 1) ? c0 + 63 : m - 1;   // C[kk] is not in this window
    }
    }
    if (lane == 0) {
        ReadOut* O = a.out + r;
        O->m_dv = (int32_t)m;
        O->flags = flags | RF_DV_FOUND; O->n_match = n_match; O->dv_st = (int32_t)st; O->dv_en = (int32_t)en;
    }
}

// Round 5: k_dv's strict match (odd k) for reads with more minimizers than one wave stages
// (C5's 100 kb reads: ~18 k): a workgroup per read, the positions in LDS, and every chain
// anchor's lower-bound search in parallel over 1024 lanes; the first anchor P lacks ends the
// matches (its index is a workgroup minimum).  Same results as k_dv (paf.rs:156-199).
constexpr uint32_t DV_LONG = 32768;   // positions staged (128 KB of LDS)
__global__ __launch_bounds__(1024) void k_dv_long(DvArgs a) {
    if (a.abort && (*a.abort & BS_ANCHORS)) return;
    extern __shared__ int32_t Pl[];
    __shared__ uint32_t s_miss, s_st, s_ok;
    __shared__ int32_t s_en;
    const int tid = threadIdx.x;
    for (uint32_t r = blockIdx.x; r < a.n; r += gridDim.x) {
        const uint32_t m = a.mz_cnt[r];
        if (m <= (uint32_t)DV_LDS || m > a.long_m) continue;          // (k_dv's reads)
        const int32_t flags = a.out[r].flags, cm = a.out[r].cm;
        if (!((flags & RF_MAPPED) && !(flags & RF_PANIC) && cm > 0)) continue;   // k_dv wrote these
        const uint64_t mzb = a.mz_base[r], ab = a.a_off[r];
        [[maybe_unused]] const uint64_t An = a.a_off[r + 1] - ab;   // (CK's bound in checked builds)
        const uint32_t* Y = a.mz_y + mzb;
        const uint32_t* CB = a.chain + ab;
        const uint64_t* K = a.keys + ab;
        const uint64_t qmask = (1ULL << a.kl.qb) - 1;
        const bool rev = (uint32_t)a.out[r].group >= a.kl.n_seq;
        const int32_t qlen = a.out[r].qlen, span = a.span;
        auto fwdq = [&](int32_t t) -> int32_t {
            if (!rev) return (int32_t)(K[CK(CB[cm - 1 - t], An)] & qmask);
            const int32_t q = (int32_t)(K[CK(CB[t], An)] & qmask);
            return qlen - 1 - (q + 1 - span);
        };
        for (uint32_t j = tid; j < m; j += 1024) Pl[j] = (int32_t)(Y[CK(j, m)] >> 1);
        if (tid == 0) s_miss = (uint32_t)cm;
        __syncthreads();
        if (tid == 0) {   // Rust >= 1.82 slice::binary_search of the first chain position (paf.rs:178)
            const int32_t first = fwdq(0);
            uint32_t size = m, b = 0;
            while (size > 1) { const uint32_t half = size / 2, mid = b + half; if (!(Pl[mid] > first)) b = mid; size -= half; }
            s_ok = Pl[b] == first ? 1u : 0u;
            uint32_t st = b;
            while (st > 0 && Pl[st - 1] == first) --st;
            s_st = st;
            s_en = (int32_t)st;
        }
        __syncthreads();
        if (s_ok) {
            // chain anchor t >= 1: its lower bound in P; the first miss ends the matches
            for (int32_t t = 1 + tid; t < cm; t += 1024) {
                const int32_t v = fwdq(t);
                uint32_t b0 = 0, sz = m;
                while (sz > 1) { const uint32_t half = sz / 2; if (Pl[b0 + half] < v) b0 += half; sz -= half; }
                const uint32_t ix = b0 + (Pl[b0] < v ? 1u : 0u);
                if (!(ix < m && Pl[ix < m ? ix : 0] == v)) atomicMin(&s_miss, (uint32_t)t);
            }
            __syncthreads();
            const uint32_t tm = s_miss;                                   // matches: anchors 0 .. tm-1
            if (tm > 1 && (int32_t)(tm - 1) % 1024 == tid) {             // en = the last match's position
                const int32_t v = fwdq((int32_t)tm - 1);
                uint32_t b0 = 0, sz = m;
                while (sz > 1) { const uint32_t half = sz / 2; if (Pl[b0 + half] < v) b0 += half; sz -= half; }
                s_en = (int32_t)(b0 + (Pl[b0] < v ? 1u : 0u));
            }
            __syncthreads();
            if (tid == 0) {
                ReadOut* O = a.out + r;
                O->m_dv = (int32_t)m;
                O->flags = flags | RF_DV_FOUND; O->n_match = (int32_t)tm; O->dv_st = (int32_t)s_st; O->dv_en = s_en;
            }
        } else if (tid == 0) {
            a.out[r].m_dv = (int32_t)m; a.out[r].flags = flags & ~RF_DV_FOUND;
        }
        __syncthreads();
    }
}

// ============================================================================
// misc: scans and per-read setup
// ============================================================================
// out[i] = sum_{t<i} f(in[t]) for i in [0, n]; mode 0: identity, mode 1: filter
// table size.  Single workgroup, 1024 threads, chunked with carry.
__global__ __launch_bounds__(1024) void k_excl_scan(const uint32_t* in, uint32_t n, uint64_t* out, int mode, int q_occ_max, int k,
                                                    uint64_t cap, uint32_t* status, uint32_t bit, int slot, uint32_t* order) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry_s;
    __shared__ uint32_t hist[1024], s_sc[16];
    const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < n; c0 += 1024) {
        const uint32_t i = c0 + tid;
        uint64_t v = 0;
        if (i < n) {
            const uint32_t x = in[i];
            if (mode == 1) { const uint32_t ts = tab_size_for(x, q_occ_max); v = filter_lds_ok(ts, k) ? 0 : ts; }
            else v = x;
        }
        uint64_t inc = wave_incl_scan(v, [](uint64_t x, uint64_t y) { return x + y; });
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint64_t woff = 0;
        for (int t = 0; t < wv; ++t) woff += wsum[t];
        const uint64_t carry = carry_s;
        if (i < n) out[i] = carry + woff + inc - v;
        __syncthreads();
        if (tid == 1023) carry_s = carry + woff + inc;
        __syncthreads();
    }
    if (tid == 0) {
        const uint64_t tot = carry_s;
        out[n] = tot;
        if (status) {
            ((unsigned long long*)status)[slot] = tot;
            if (cap && tot > cap) atomicOr(status, bit);
        }
    }
    if (order) read_order_block(n, in, order, hist, s_sc);   // the anchor scan also orders the reads (one launch less)
}

// per-batch sums for mm2g_batch_counters (st[3] = minimizers, st[4] = anchors in the DP)
__global__ __launch_bounds__(1024) void k_batch_sums(uint32_t n, const uint32_t* mz_cnt, const uint32_t* cnt2, unsigned long long* st) {
    // st[3] minimizers, st[4] anchors in the DP
    __shared__ unsigned long long ws[2][16];
    unsigned long long v[2] = {0, 0};
    for (uint32_t i = threadIdx.x; i < n; i += 1024) { v[0] += mz_cnt[i]; v[1] += cnt2 ? cnt2[i] : 0u; }
#pragma unroll
    for (int k = 0; k < 2; ++k) { v[k] = wave_sum64(v[k]); if (lane_id() == 0) ws[k][threadIdx.x >> 6] = v[k]; }
    __syncthreads();
    if (threadIdx.x < 2) {
        unsigned long long x = 0;
        for (int t = 0; t < 16; ++t) x += ws[threadIdx.x][t];
        st[3 + threadIdx.x] = x;
    }
}

// Also clears the batch's per-read outputs and status block (when given): the
// first kernel of a map, in place of two memset launches.
__global__ void k_mz_base(uint32_t n, const uint64_t* rd_off, uint64_t* base, uint64_t* end, uint32_t slot, ReadOut* zout,
                          unsigned long long* zst, int zst_words) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (zout && r <= n) { uint4* o = (uint4*)(zout + r); for (int q = 0; q < (int)(sizeof(ReadOut) / 16); ++q) o[q] = make_uint4(0u, 0u, 0u, 0u); }
    if (zst && r < (uint32_t)zst_words) zst[r] = 0ULL;
    if (r >= n) return;
    if (slot) { base[r] = (uint64_t)slot * r; end[r] = (uint64_t)slot * (r + 1); return; }   // tests: fixed slots
    base[r] = rd_off[r] + 16ull * r;
    end[r] = rd_off[r + 1] + 16ull * (r + 1);
}

// ---- Query sketch views (DESIGN.md "Query sketch views"): a read longer than
// V bases is sketched as views of V emitting bases, each after a warm-up of
// >= W0 bases (W0 = 2(w+k)+64 rounded up to 8: enough for odd k, DESIGN.md
// §10), one wave per view, so a 10 kb read is not 20 sequential tiles of one
// wave.  View outputs go to their own slots and are concatenated per read.
constexpr int VIEW_PLAN_LDS = 4096;
// The view plan in one single-workgroup launch (C2's 500-read units; round 4 used four
// launches: a memset, a count, a scan and a fill), which also does k_mz_base's slots and clears when
// `base` is given: per-read view counts, their exclusive scan vo, the view table, and
// v_len = 0 for the views past the real count up to nvmax.  View v = vo[r] + j of read r
// emits [jV, min(L, (j+1)V)), starting W0 (or more, to a multiple of 8) bases earlier; its
// output slot is [rd_off[r] + jV + 16v, + emitting bases + 16), disjoint across all views.
__global__ __launch_bounds__(1024) void k_view_plan(uint32_t n, const uint64_t* rd_off, uint32_t V, uint32_t W0, uint64_t nvmax, uint64_t* vo,
                                                    uint32_t* v_read, uint64_t* v_off, uint32_t* v_len, uint32_t* v_pre, uint32_t* v_from,
                                                    uint8_t* v_last, uint64_t* v_base, uint64_t* v_end, uint64_t* base, uint64_t* end,
                                                    ReadOut* zout, unsigned long long* zst, int zst_words) {
    __shared__ uint32_t s_sc[16];
    __shared__ uint32_t s_vo[VIEW_PLAN_LDS];   // the view offsets of batches of up to VIEW_PLAN_LDS reads
    const uint32_t tid = threadIdx.x;
    if (base) {
        for (uint32_t r = tid; r <= n; r += 1024) {
            if (zout) { uint4* o = (uint4*)(zout + r); for (int q = 0; q < (int)(sizeof(ReadOut) / 16); ++q) o[q] = make_uint4(0u, 0u, 0u, 0u); }
            if (r < n) { base[r] = rd_off[r] + 16ull * r; end[r] = rd_off[r + 1] + 16ull * (r + 1); }
        }
        if (zst) for (uint32_t q = tid; q < (uint32_t)zst_words; q += 1024) zst[q] = 0ULL;
    }
    auto nview = [&](uint32_t r) -> uint32_t { const uint64_t L = rd_off[r + 1] - rd_off[r]; return L <= V ? 1u : (uint32_t)((L + V - 1) / V); };
    const bool lds = n <= (uint32_t)VIEW_PLAN_LDS;
    uint64_t carry = 0;
    for (uint32_t r0 = 0; r0 < n; r0 += 1024) {
        const uint32_t r = r0 + tid;
        const uint32_t c = r < n ? nview(r) : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_sum(c, tot, s_sc);
        if (r < n) { vo[r] = carry + ex; if (lds) s_vo[r] = (uint32_t)(carry + ex); }
        carry += tot;
    }
    if (tid == 0) vo[n] = carry;
    __syncthreads();
    auto fill = [&](uint32_t r, uint32_t j, uint64_t v) {
        const uint64_t L = rd_off[r + 1] - rd_off[r];
        const uint64_t c0 = (uint64_t)j * V, ve = c0 + V < L ? c0 + V : L;
        const uint64_t vs = j ? (c0 > W0 ? (c0 - W0) & ~7ULL : 0) : 0;
        v_read[v] = r; v_off[v] = vs; v_len[v] = (uint32_t)(ve - vs); v_pre[v] = (uint32_t)vs;
        v_from[v] = (uint32_t)(c0 - vs); v_last[v] = ve == L ? 1 : 0;
        v_base[v] = rd_off[r] + c0 + 16 * v; v_end[v] = v_base[v] + (ve - c0) + 16;
    };
    if (lds && carry <= 0xffffffffULL) {
        // a thread per view (the table's stores coalesce): its read is the last r with
        // vo[r] <= v (every read has a view, so vo rises strictly)
        for (uint64_t v = tid; v < carry; v += 1024) {
            uint32_t lo = 0, hi = n - 1;
            while (lo < hi) { const uint32_t mid = (lo + hi + 1) >> 1; if (s_vo[mid] <= (uint32_t)v) lo = mid; else hi = mid - 1; }
            fill(lo, (uint32_t)v - s_vo[lo], v);
        }
    } else {
        for (uint32_t r = tid; r < n; r += 1024) {
            const uint32_t nv = nview(r);
            for (uint32_t j = 0; j < nv; ++j) fill(r, j, vo[r] + j);
        }
    }
    for (uint64_t v = carry + tid; v < nvmax; v += 1024) v_len[v] = 0;   // views past the real count: empty
}

// a workgroup per read: its views' minimizers, in view order, into the read's slot
// (y + view start << 1: positions are view-relative), clamped and flagged like k_sketch.
// Wave w copies views w, w + 4, ... at their offsets (a wave scan of the view counts,
// 64 views at a time), 4 entries per lane in flight: round 4's one wave per read copied
// a 100 kb read's ~18 k minimizers one dependent 64-entry step at a time.
__global__ __launch_bounds__(256) void k_view_compact(uint32_t n, const uint64_t* __restrict__ vo, const uint64_t* __restrict__ v_off,
                                                      const uint64_t* __restrict__ v_base, const uint32_t* __restrict__ v_cnt,
                                                      const uint32_t* __restrict__ v_need, const uint64_t* __restrict__ vx,
                                                      const uint32_t* __restrict__ vy, const uint64_t* __restrict__ base,
                                                      const uint64_t* __restrict__ end, uint64_t* __restrict__ x, uint32_t* __restrict__ y,
                                                      uint32_t* cnt, uint32_t* need, int32_t* overflow) {
    constexpr int CU = 4;
    const uint32_t r = blockIdx.x;
    if (r >= n) return;
    const int lane = lane_id(), wv = wave_id();
    const uint64_t b = base[r], capn = end[r] - b;
    const uint64_t v0 = vo[r], v1 = vo[r + 1];
    uint64_t o = 0, tn = 0;   // the views before this chunk: entries (unclamped), true counts
    for (uint64_t c0 = v0; c0 < v1; c0 += 64) {
        const uint64_t v = c0 + lane;
        const uint32_t c = v < v1 ? v_cnt[v] : 0u;
        uint32_t tot;
        const uint32_t ex = wave_excl_sum(c, tot);
        const int nc = (int)(v1 - c0 < 64 ? v1 - c0 : 64);
        for (int j = wv; j < nc; j += 4) {
            const uint32_t cj = rdlu(c, j);
            const uint64_t oj = o + rdlu(ex, j), vb = v_base[c0 + j];
            const uint32_t add = (uint32_t)(v_off[c0 + j] << 1);
            for (uint32_t i0 = 0; i0 < cj; i0 += 64 * CU) {
                uint64_t xv[CU];
                uint32_t yv[CU];
#pragma unroll
                for (int u = 0; u < CU; ++u) {
                    const uint32_t i = i0 + u * 64 + lane;
                    if (i < cj) { xv[u] = vx[vb + i]; yv[u] = vy[vb + i]; }
                }
#pragma unroll
                for (int u = 0; u < CU; ++u) {
                    const uint32_t i = i0 + u * 64 + lane;
                    if (i < cj && oj + i < capn) { x[b + oj + i] = xv[u]; y[b + oj + i] = yv[u] + add; }
                }
            }
        }
        o += tot;
        tn += wave_sum64(v < v1 ? (uint64_t)v_need[v] : 0ULL);
    }
    if (threadIdx.x == 0) {   // a view that overflowed its own slot flagged it already; the re-run has views off
        cnt[r] = (uint32_t)(o > capn ? capn : o);
        need[r] = (uint32_t)(tn > 0xffffffffULL ? 0xffffffffULL : tn);
        if (o > capn) atomicOr(overflow, 1);
    }
}

// Build the device index table from (key, off, n) triples (insert with CAS).
__global__ void k_ix_build(const uint64_t* keys, const uint32_t* offs, const uint32_t* ns, uint64_t nk, IxEntry* tab, uint32_t log2cap) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nk) return;
    const uint64_t h = keys[t];
    const uint32_t cmask = (1u << log2cap) - 1;
    uint32_t sl = ix_slot(h, log2cap);
    for (;;) {
        unsigned long long prev = atomicCAS((unsigned long long*)&tab[sl].key, (unsigned long long)U64MAX, (unsigned long long)h);
        if (prev == U64MAX) { tab[sl].off = offs[t]; tab[sl].n = ns[t]; return; }
        sl = (sl + 1) & cmask;
    }
}

// calc_mid_occ (src/index.rs:124-141) on the device table: a histogram of the
// per-key occurrence counts (1 for a Single) below `nbins`, plus the counts at
// or above it (`ovf`, gathered only when the quantile falls there).  Singletons
// dominate, so count == 1 is tallied per wave by ballot.
__global__ __launch_bounds__(256) void k_mid_hist(const IxEntry* tab, uint64_t cap, uint32_t nbins, unsigned long long* hist,
                                                  uint32_t* ovf, uint32_t ovf_cap, uint32_t* ovf_n) {
    extern __shared__ uint32_t sh[];
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x) sh[i] = 0;
    __syncthreads();
    uint32_t ones = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < cap; b0 += stride) {   // block-uniform trips
        const uint64_t t = b0 + threadIdx.x;
        bool one = false;
        if (t < cap && tab[t].key != U64MAX) {
            const uint32_t n = ix_count(tab[t].n);
            one = n == 1;
            if (n < nbins) { if (!one) atomicAdd(&sh[n], 1u); }
            else if (ovf) { const uint32_t q = atomicAdd(ovf_n, 1u); if (q < ovf_cap) ovf[q] = n; }
            else atomicAdd(ovf_n, 1u);
        }
        const uint64_t m = ballot(one);
        if (lane_id() == 0) ones += (uint32_t)__popcll(m);
    }
    if (lane_id() == 0 && ones && nbins > 1) atomicAdd(&sh[1], ones);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x)
        if (sh[i]) atomicAdd(hist + i, (unsigned long long)sh[i]);
}

// ---------------------------------------------------------------- launchers
#define LAUNCH_CHECK() do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)

int launch_sketch(const SketchArgs& a, int n_blocks, hipStream_t st) {
    const size_t lds = sketch_wave_lds(a.w) * 4;
    const bool x32 = a.k <= 15 && !a.x64;   // 32-bit LDS window (k_sketch X32)
    if (a.pk_words) {
        if (x32) hipLaunchKernelGGL((k_sketch<true, SeqNt4, false, true>), dim3(n_blocks), dim3(256), lds, st, a);
        else if (a.k <= 16) hipLaunchKernelGGL((k_sketch<true, SeqNt4>), dim3(n_blocks), dim3(256), lds, st, a);
        else hipLaunchKernelGGL((k_sketch<false, SeqNt4>), dim3(n_blocks), dim3(256), lds, st, a);
    } else {
        if (a.hpc_span) {
            if (a.k <= 16) hipLaunchKernelGGL((k_sketch<true, SeqAscii, true>), dim3(n_blocks), dim3(256), lds, st, a);
            else hipLaunchKernelGGL((k_sketch<false, SeqAscii, true>), dim3(n_blocks), dim3(256), lds, st, a);
        } else if (x32) hipLaunchKernelGGL((k_sketch<true, SeqAscii, false, true>), dim3(n_blocks), dim3(256), lds, st, a);
        else if (a.k <= 16) hipLaunchKernelGGL((k_sketch<true, SeqAscii>), dim3(n_blocks), dim3(256), lds, st, a);
        else hipLaunchKernelGGL((k_sketch<false, SeqAscii>), dim3(n_blocks), dim3(256), lds, st, a);
    }
    LAUNCH_CHECK();
    return 0;
}
int launch_filter(const FilterArgs& a, int k, int n_blocks, hipStream_t st) {
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(k_filter_lds, dim3(a.n), dim3(256), 0, st, a, k);
    LAUNCH_CHECK();
    (void)n_blocks;
    // persistent: one workgroup per CU (its LDS), reads taken by grid stride; most reads of
    // 10 kb batches are k_filter_lds's and are skipped after one load of their count
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    hipLaunchKernelGGL(k_filter, dim3(std::min<uint32_t>(a.n, (uint32_t)std::max(ncu, 1))), dim3(1024), FB_LDS, st, a, k);
    LAUNCH_CHECK();
    return 0;
}
int launch_seed_count(const SeedArgs& a, int n_blocks, hipStream_t st) {
    (void)n_blocks;
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(k_seed_count, dim3(std::min<uint32_t>(a.n, 16384)), dim3(SEED_PARTS * 64), 0, st, a);
    LAUNCH_CHECK();
    return 0;
}
int launch_seed_write(const SeedArgs& a, int n_blocks, hipStream_t st) {
    (void)n_blocks;
    const uint64_t parts = (uint64_t)a.n * SEED_PARTS;
    const int blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>((parts + 3) / 4, 16384));
    hipLaunchKernelGGL(k_seed_write, dim3(blocks), dim3(256), 0, st, a);
    LAUNCH_CHECK();
    return 0;
}
uint32_t sort_read_lds_words(const SortArgs& a) {
    // the requested LDS (default SORT_LDS: one workgroup per CU), at least the two bitmaps
    const size_t bmb = (size_t)2 * ((a.cells + 31) / 32) * 4;
    size_t lds = std::max<size_t>(a.lds_words ? (size_t)a.lds_words * 4 : (size_t)SORT_LDS, bmb);
    return (uint32_t)(std::min<size_t>(lds, (size_t)SORT_LDS) / 4);
}
int launch_sort_read(int stage, const SortArgs& a, hipStream_t st) {
    if (a.n == 0) return 0;
    if (stage == 0) hipLaunchKernelGGL(k_sort_small, dim3(a.n), dim3(256), 0, st, a);
    else if (stage == 1) {
        const size_t lds = (size_t)sort_read_lds_words(a) * 4;
        SortArgs b = a;
        b.lds_words = (uint32_t)(lds / 4);
        // up to SORT_LDS_HALF: 512-thread workgroups, two per CU (one read's
        // barrier and latency phases overlap the other's)
        const bool gl = 2u * b.n_seq + 2u > (uint32_t)GOFF_LDS;
#define SR_LAUNCH(G, T) hipLaunchKernelGGL((k_sort_read<G, T>), dim3(a.n), dim3(T), lds, st, b)
        if (lds <= (size_t)SORT_LDS_HALF) {
            if (gl) SR_LAUNCH(true, 512);
            else SR_LAUNCH(false, 512);
        } else if (gl) SR_LAUNCH(true, 1024);
        else SR_LAUNCH(false, 1024);
#undef SR_LAUNCH
    } else if (a.cells) {       // the singleton filter is on: every listed read takes the bucket path
        SortArgs b = a;
        b.lds_words = (uint32_t)(SORT_LDS / 4);
        // persistent workgroups on a work counter: one per CU (the LDS allows no
        // more); most batches list no read, and every extra workgroup would wait
        // for a CU the other streams' kernels hold
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        const unsigned grid = std::min<uint32_t>(a.n, (uint32_t)std::max(ncu, 1));
        if (2u * b.n_seq + 2u > (uint32_t)GOFF_LDS) hipLaunchKernelGGL(k_sort_big<true>, dim3(grid), dim3(1024), (size_t)SORT_LDS, st, b);
        else hipLaunchKernelGGL(k_sort_big<false>, dim3(grid), dim3(1024), (size_t)SORT_LDS, st, b);
    } else {
        const size_t bmb = (size_t)2 * ((a.cells + 31) / 32) * 4;
        const size_t hb = (size_t)(RS_MAXP + 16) * RS_ND * 4;
        const size_t lds = std::min<size_t>(std::max<size_t>(bmb, hb), (size_t)SORT_LDS);
        if (2u * a.n_seq + 2u > (uint32_t)GOFF_LDS) hipLaunchKernelGGL(k_sort_radix<true>, dim3(std::min<uint32_t>(a.n, 512)), dim3(1024), lds, st, a);
        else hipLaunchKernelGGL(k_sort_radix<false>, dim3(std::min<uint32_t>(a.n, 512)), dim3(1024), lds, st, a);
    }
    LAUNCH_CHECK();
    return 0;
}
static size_t chain_lds(int lut_n) {
    return (size_t)(((lut_n * 2) + 15) & ~15) + (size_t)DP_NW * (RING_WORDS * 4 + RK * 8 + RK * 8);
}
static size_t lut_lds(int lut_n) { return (size_t)(((lut_n * 2) + 15) & ~15); }
// LDS of the LDS variant: the pen LUT plus its segment capacity (giant_lcap, when set, lowers it:
// smaller workgroups fit twice on a CU, the longer segments going to the HBM variant)
static size_t giant_lds(int lut_n, uint32_t lcap) {
    const int cap = lcap ? std::min<int>(giant_cap(lut_n), (int)lcap) : giant_cap(lut_n);
    return lut_lds(lut_n) + (size_t)cap * GIANT_B;
}
static size_t seg_lds(int lut_n) { return lut_lds(lut_n) + (size_t)DP_NW * (KRING * 8 + 3 * TQ * 5 + MEDB * 8); }
int chain_max_blocks(int lut_n, int which) {
    int dev = 0, ncu = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    hipError_t e = which == 0   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_chain_seg, DP_NW * 64, seg_lds(lut_n))
                   : which == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_chain_long<false, 4>, DP_NW * 64, chain_lds(lut_n))
                                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_chain_med, 256, lut_lds(lut_n));
    if (e != hipSuccess) return 0;
    return ncu * (per > 0 ? per : 1);
}
int launch_read_order(uint32_t n, const uint32_t* a_cnt, uint32_t* order, hipStream_t st) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_read_order, dim3(1), dim3(1024), 0, st, n, a_cnt, order);
    LAUNCH_CHECK();
    return 0;
}
int launch_chain_stage(int stage, const ChainArgs& a, int blocks, hipStream_t st) {
    if (a.n == 0) return 0;
    switch (stage) {
    case 0: hipLaunchKernelGGL(k_chain_seg, dim3(blocks), dim3(DP_NW * 64), seg_lds(a.P.lut_n), st, a); break;
    case 1: hipLaunchKernelGGL(k_chain_med, dim3(blocks), dim3(256), lut_lds(a.P.lut_n), st, a); break;
    case 2: hipLaunchKernelGGL(k_lseg_order, dim3(1), dim3(1024), 0, st, a); break;
    case 3:
        if (a.lseg_prof) {
            if (a.spec_batch == 8) hipLaunchKernelGGL((k_chain_long<true, 8>), dim3(blocks), dim3(DP_NW * 64), chain_lds(a.P.lut_n), st, a);
            else hipLaunchKernelGGL((k_chain_long<true, 4>), dim3(blocks), dim3(DP_NW * 64), chain_lds(a.P.lut_n), st, a);
        } else if (a.spec_batch == 8) hipLaunchKernelGGL((k_chain_long<false, 8>), dim3(blocks), dim3(DP_NW * 64), chain_lds(a.P.lut_n), st, a);
        else hipLaunchKernelGGL((k_chain_long<false, 4>), dim3(blocks), dim3(DP_NW * 64), chain_lds(a.P.lut_n), st, a);
        break;
    case 5: hipLaunchKernelGGL(k_chain_lb, dim3(blocks), dim3(256), lut_lds(a.P.lut_n), st, a); break;
    case 6: hipLaunchKernelGGL(k_seg_items, dim3(1), dim3(1024), 0, st, a); break;
    case 10: hipLaunchKernelGGL(k_seg_cands, dim3(blocks), dim3(SC_NW * 64), 0, st, a); break;
    case 7: {
        const size_t lds = giant_lds(a.P.lut_n, a.giant_lcap);
        if (blocks <= 0) {   // as many workgroups as fit on the CUs at once (they take segments from a counter)
            int dev = 0, ncu = 256;
            if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
            blocks = std::max(1, ncu) * (int)std::max<size_t>(1, std::min<size_t>(2, (size_t)(158 * 1024) / std::max<size_t>(lds, 1)));
        }
        hipLaunchKernelGGL(k_chain_giant<false>, dim3(blocks), dim3(1024), lds, st, a);
        break;
    }
    case 8: hipLaunchKernelGGL(k_chain_giant<true>, dim3(blocks), dim3(1024), lut_lds(a.P.lut_n), st, a); break;
    default: hipLaunchKernelGGL(k_chain_fin, dim3((a.n + 3) / 4), dim3(256), 0, st, a); break;
    }
    LAUNCH_CHECK();
    return 0;
}
int launch_dv(const DvArgs& a, hipStream_t st) {
    if (a.n == 0) return 0;
    DvArgs b = a;
    b.long_m = a.strict ? std::min<uint32_t>(a.long_m, DV_LONG) : 0u;   // both kernels see the same split
    hipLaunchKernelGGL(k_dv, dim3(a.n), dim3(64), 0, st, b);
    LAUNCH_CHECK();
    if (b.long_m) {   // reads over DV_LDS minimizers (the host sets long_m only when some may be)
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        hipLaunchKernelGGL(k_dv_long, dim3(std::min<uint32_t>(a.n, (uint32_t)std::max(ncu, 1))), dim3(1024), (size_t)b.long_m * 4, st, b);
        LAUNCH_CHECK();
    }
    return 0;
}
int launch_excl_scan(const uint32_t* in, uint32_t n, uint64_t* out, int mode, int q_occ_max, int k, uint64_t cap, uint32_t* status,
                     uint32_t bit, int slot, hipStream_t st, uint32_t* order) {
    hipLaunchKernelGGL(k_excl_scan, dim3(1), dim3(1024), 0, st, in, n, out, mode, q_occ_max, k, cap, status, bit, slot, order);
    LAUNCH_CHECK();
    return 0;
}
int launch_batch_sums(uint32_t n, const uint32_t* mz_cnt, const uint32_t* cnt2, unsigned long long* status64, hipStream_t st) {
    hipLaunchKernelGGL(k_batch_sums, dim3(1), dim3(1024), 0, st, n, mz_cnt, cnt2, status64);
    LAUNCH_CHECK();
    return 0;
}
int launch_view_plan(uint32_t n, const uint64_t* rd_off, uint32_t V, uint32_t W0, uint64_t nvmax, uint64_t* vo, uint32_t* v_read,
                     uint64_t* v_off, uint32_t* v_len, uint32_t* v_pre, uint32_t* v_from, uint8_t* v_last, uint64_t* v_base, uint64_t* v_end,
                     uint64_t* base, uint64_t* end, mm2g::ReadOut* zout, unsigned long long* zst, int zst_words, hipStream_t st) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_view_plan, dim3(1), dim3(1024), 0, st, n, rd_off, V, W0, nvmax, vo, v_read, v_off, v_len, v_pre, v_from, v_last,
                       v_base, v_end, base, end, zout, zst, zst_words);
    LAUNCH_CHECK();
    return 0;
}
int launch_view_compact(uint32_t n, const uint64_t* vo, const uint64_t* v_off, const uint64_t* v_base, const uint32_t* v_cnt,
                        const uint32_t* v_need, const uint64_t* vx, const uint32_t* vy, const uint64_t* base, const uint64_t* end, uint64_t* x,
                        uint32_t* y, uint32_t* cnt, uint32_t* need, int32_t* overflow, hipStream_t st) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_view_compact, dim3(n), dim3(256), 0, st, n, vo, v_off, v_base, v_cnt, v_need, vx, vy, base, end, x, y,
                       cnt, need, overflow);
    LAUNCH_CHECK();
    return 0;
}
int launch_mz_base(uint32_t n, const uint64_t* rd_off, uint64_t* base, uint64_t* end, uint32_t slot, hipStream_t st,
                   mm2g::ReadOut* zout, unsigned long long* zst, int zst_words) {
    if (n == 0) return 0;
    const uint32_t nt = std::max<uint32_t>(n + 1, zst ? (uint32_t)zst_words : 0u);
    hipLaunchKernelGGL(k_mz_base, dim3((nt + 255) / 256), dim3(256), 0, st, n, rd_off, base, end, slot, zout, zst, zst_words);
    LAUNCH_CHECK();
    return 0;
}
int launch_mid_hist(const IxEntry* tab, uint64_t cap, uint32_t nbins, unsigned long long* hist, uint32_t* ovf, uint32_t ovf_cap,
                    uint32_t* ovf_n, hipStream_t st) {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
    const uint64_t want = (cap + 255) / 256;
    const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)ncu * 8));
    hipLaunchKernelGGL(k_mid_hist, dim3(blocks), dim3(256), nbins * 4, st, tab, cap, nbins, hist, ovf, ovf_cap, ovf_n);
    LAUNCH_CHECK();
    return 0;
}
int launch_ix_build(const uint64_t* keys, const uint32_t* offs, const uint32_t* ns, uint64_t nk, IxEntry* tab, uint32_t log2cap, hipStream_t st) {
    if (nk == 0) return 0;
    hipLaunchKernelGGL(k_ix_build, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, st, keys, offs, ns, nk, tab, log2cap);
    LAUNCH_CHECK();
    return 0;
}

int mm2g_checked_read(unsigned long long out[4], hipStream_t st) {
#ifdef MM2G_CHECKED
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chk), sizeof(unsigned long long) * 4, 0, hipMemcpyDeviceToHost);
    return (int)e;
#else
    (void)st; out[0] = out[1] = out[2] = out[3] = 0;
    return 0;
#endif
}
