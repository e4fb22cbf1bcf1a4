// Host epilogue for several output chains per read (mm2g_multi.h).
#include "mm2g_multi.h"

#include <algorithm>
#include <cmath>
#include <utility>

namespace mm2g {
namespace {

// i32 arithmetic of the reference (release build: wrapping)
inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
inline int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

// Anchor fields (src/lchain.rs:3-12, src/paf.rs:26-33)
struct Anc {
    const uint64_t* xy;
    int32_t qpos(size_t i) const { return (int32_t)(uint32_t)xy[2 * i + 1]; }
    int32_t qspan(size_t i) const { return (int32_t)((xy[2 * i + 1] >> 32) & 0xff); }
    int32_t rpos(size_t i) const { return (int32_t)(uint32_t)xy[2 * i]; }
    bool rev(size_t i) const { return (xy[2 * i] >> 63) != 0; }
    int32_t rid(size_t i) const { return (int32_t)((xy[2 * i] >> 32) & 0x7fffffff); }
};

// ---- Rust slice::sort_unstable_by_key, rustc 1.81+ (core/src/slice/sort/unstable):
// insertion sort up to 20, else find_existing_run + quicksort with a
// 2*log2(len) imbalance limit (heapsort beyond), pseudo-median pivots,
// Lomuto branchless cyclic partitions and, up to 32 elements, the general
// small sort (stable for a 16-byte Copy type).
using Pair = std::pair<int32_t, uint32_t>;
struct Ipn {
    static bool lt(const Pair& a, const Pair& b) { return a.first < b.first; }
    static bool le(const Pair& a, const Pair& b) { return !(b.first < a.first); }

    static void insertion(Pair* v, size_t n) {
        for (size_t i = 1; i < n; ++i) {
            if (!lt(v[i], v[i - 1])) continue;
            const Pair t = v[i];
            size_t j = i;
            for (; j > 0 && lt(t, v[j - 1]); --j) v[j] = v[j - 1];
            v[j] = t;
        }
    }
    static void heap(Pair* v, size_t n) {
        auto sift = [&](size_t len, size_t node) {
            for (size_t ch; (ch = 2 * node + 1) < len; node = ch) {
                if (ch + 1 < len && lt(v[ch], v[ch + 1])) ++ch;
                if (!lt(v[node], v[ch])) return;
                std::swap(v[node], v[ch]);
            }
        };
        for (size_t i = n + n / 2; i-- > 0;) {
            if (i >= n) sift(n, i - n);
            else { std::swap(v[0], v[i]); sift(i, 0); }
        }
    }
    static size_t med3(const Pair* v, size_t a, size_t b, size_t c) {
        const bool x = lt(v[a], v[b]), y = lt(v[a], v[c]);
        if (x != y) return a;
        return (lt(v[b], v[c]) != x) ? c : b;
    }
    static size_t med3r(const Pair* v, size_t a, size_t b, size_t c, size_t n) {
        if (n >= 8) {   // n * 8 >= 64
            const size_t m = n / 8;
            a = med3r(v, a, a + 4 * m, a + 7 * m, m);
            b = med3r(v, b, b + 4 * m, b + 7 * m, m);
            c = med3r(v, c, c + 4 * m, c + 7 * m, m);
        }
        return med3(v, a, b, c);
    }
    template <bool LE>
    static size_t partition(Pair* v, size_t n, size_t piv) {
        std::swap(v[0], v[piv]);
        const Pair p = v[0];
        Pair* w = v + 1;
        const size_t m = n - 1;
        size_t cnt = 0;
        if (m) {
            const Pair saved = w[0];
            size_t gap = 0;
            for (size_t r = 1; r <= m; ++r) {
                const Pair e = r < m ? w[r] : saved;
                const bool take = LE ? le(e, p) : lt(e, p);
                w[gap] = w[cnt];
                w[cnt] = e;
                gap = r;
                cnt += take;
            }
        }
        std::swap(v[0], v[cnt]);
        return cnt;
    }
    static void quick(Pair* v, size_t n, bool has_anc, Pair anc, uint32_t limit) {
        for (;;) {
            if (n <= 32) { std::stable_sort(v, v + n, lt); return; }
            if (limit == 0) { heap(v, n); return; }
            --limit;
            const size_t d = n / 8;
            const size_t piv = n < 64 ? med3(v, 0, 4 * d, 7 * d) : med3r(v, 0, 4 * d, 7 * d, d);
            if (has_anc && !lt(anc, v[piv])) {
                const size_t k = partition<true>(v, n, piv);
                v += k + 1; n -= k + 1;
                has_anc = false;
                continue;
            }
            const size_t k = partition<false>(v, n, piv);
            quick(v, k, has_anc, anc, limit);
            anc = v[k]; has_anc = true;
            v += k + 1; n -= k + 1;
        }
    }
    static void sort(Pair* v, size_t n) {
        if (n < 2) return;
        if (n <= 20) { insertion(v, n); return; }
        const bool desc = lt(v[1], v[0]);
        size_t run = 2;
        while (run < n && (desc ? lt(v[run], v[run - 1]) : !lt(v[run], v[run - 1]))) ++run;
        if (run == n) { if (desc) std::reverse(v, v + n); return; }
        uint32_t lg = 0;
        for (size_t x = n | 1; x >>= 1;) ++lg;
        quick(v, n, false, Pair{}, 2 * lg);
    }
};

// the first index of the greatest element of `v` equal to `x`, or -1 (Rust >= 1.82 binary_search + walk back, paf.rs:178-180)
int64_t find_first(const int32_t* v, int64_t n, int32_t x) {
    if (n == 0) return -1;
    int64_t base = 0, size = n;
    while (size > 1) {
        const int64_t half = size / 2, mid = base + half;
        if (!(v[mid] > x)) base = mid;
        size -= half;
    }
    if (v[base] != x) return -1;
    while (base > 0 && v[base - 1] == x) --base;
    return base;
}

}  // namespace

void rust_sort_unstable_pairs(std::vector<std::pair<int32_t, uint32_t>>& v) { Ipn::sort(v.data(), v.size()); }

namespace {

// Ranges of a chain (lchain.rs:178-200) folded anchor by anchor: min / max are associative and
// the clamp at 0 commutes with min, so the range of a concatenation is the fold of its parts'.
struct Rng {
    int32_t qs = INT32_MAX, qe = -1, ts = INT32_MAX, te = -1;   // qs, ts before the clamp
    void add(const Anc& a, uint32_t i) {
        qs = std::min(qs, wsub(a.qpos(i), a.qspan(i) - 1)); qe = std::max(qe, wadd(a.qpos(i), 1));
        ts = std::min(ts, wsub(a.rpos(i), a.qspan(i) - 1)); te = std::max(te, wadd(a.rpos(i), 1));
    }
    void add(const Rng& r) { qs = std::min(qs, r.qs); qe = std::max(qe, r.qe); ts = std::min(ts, r.ts); te = std::max(te, r.te); }
    int32_t q0() const { return std::max(qs, 0); }
    int32_t t0() const { return std::max(ts, 0); }
};

// Chains live in one flat anchor buffer; a merged chain is a linked list of its parts in merge order.
struct Part { uint32_t off, len, next; };
struct Merged { uint32_t head, tail, n; Rng r; };

// per-thread scratch: the epilogue runs once per read on the host_threads pool
struct Scratch {
    std::vector<Pair> z, items;
    std::vector<int32_t> t, scores, sq, st, mscore;
    std::vector<uint32_t> flat, ix;
    std::vector<uint32_t> sd, tmp;
    std::vector<Part> parts;
    std::vector<Rng> rng;
    std::vector<Merged> merged, msorted;
    std::vector<int32_t> keys, tpqe, tplen;   // select: distinct qs (past 2^20), max-pqe and max-plen trees
    std::vector<uint8_t> is_pri;
    std::vector<uint64_t> seen;
    std::vector<int32_t> first_qe;
    std::vector<uint32_t> ch;
    std::vector<int32_t> cq;
};

// stable order of sort_chains_stable (lchain.rs:202-218): score desc, qs asc, ts asc, ties in input
// order.  LSD radix on 8-bit digits (ts, then qs, then the inverted score) is stable, so it gives the
// stable sort's order; the 12 digit histograms come from one pass and constant digits are skipped.
void stable_order(std::vector<uint32_t>& sd, std::vector<uint32_t>& tmp, std::vector<uint32_t>& ix, size_t m,
                  const int32_t* sc, const int32_t* q, const int32_t* t) {
    sd.resize(m); tmp.resize(m); ix.resize(m);
    if (m == 0) return;
    for (size_t i = 0; i < m; ++i) { sd[i] = ~((uint32_t)sc[i] ^ 0x80000000u); ix[i] = (uint32_t)i; }
    const uint32_t* key[3] = {(const uint32_t*)t, (const uint32_t*)q, sd.data()};   // q, t >= 0 (clamped)
    uint32_t cnt[12][256] = {};
    for (size_t i = 0; i < m; ++i)
        for (int f = 0; f < 3; ++f) {
            const uint32_t v = key[f][i];
            ++cnt[4 * f][v & 255]; ++cnt[4 * f + 1][(v >> 8) & 255]; ++cnt[4 * f + 2][(v >> 16) & 255]; ++cnt[4 * f + 3][v >> 24];
        }
    for (int d = 0; d < 12; ++d) {
        uint32_t* c = cnt[d];
        const uint32_t* k = key[d / 4];
        const int sh = 8 * (d % 4);
        if (c[(k[0] >> sh) & 255] == m) continue;     // one value: the pass keeps the order
        uint32_t sum = 0;
        for (int v = 0; v < 256; ++v) { const uint32_t x = c[v]; c[v] = sum; sum += x; }
        for (size_t i = 0; i < m; ++i) { const uint32_t j = ix[i]; tmp[c[(k[j] >> sh) & 255]++] = j; }
        ix.swap(tmp);
    }
}

// The least o in [0, omax] with (f32)o / (f32)len >= mask (select_primary_secondary's test,
// lchain.rs:228-230), or -1.  Both conversions and the division round monotonically, so the test
// is monotone in o: start from the real-valued boundary and step to the f32 one.
int32_t min_overlap(int32_t omax, int32_t len, float mask) {
    auto ok = [&](int32_t o) { return (float)o / (float)len >= mask; };
    if (!ok(omax)) return -1;
    if (ok(0)) return 0;
    int32_t o = (int32_t)std::min<double>((double)omax, std::max(0.0, std::ceil((double)mask * (double)len)));
    if (ok(o)) { while (o > 0 && ok(o - 1)) --o; }
    else { while (!ok(o)) ++o; }                      // ok(omax) holds: terminates
    return o;
}

}  // namespace

void multi_chain_read(const uint64_t* xy, const int32_t* f, const int32_t* pprev, int64_t n, int32_t qlen,
                      const int32_t* mini_pos, int64_t n_mini, float avg_k, int32_t idx_k, const uint32_t* tlen, uint32_t n_seq,
                      const MultiParams& P, MultiRead& out) {
    out = MultiRead{};
    if (n <= 0) return;                               // no anchors: chain_dp is empty, no line (main.rs:210-212)
    const Anc a{xy};
    thread_local Scratch S;
    // ---- backtrack (lchain.rs:92-160): chains in extraction order, anchors appended to `flat`
    std::vector<Pair>& z = S.z;
    z.clear();
    for (int64_t i = 0; i < n; ++i) if (f[i] > 0) z.push_back({f[i], (uint32_t)i});
    std::vector<uint32_t>& flat = S.flat;
    std::vector<Part>& parts = S.parts;
    std::vector<int32_t>& scores = S.scores;
    flat.clear(); parts.clear(); scores.clear();
    if (!z.empty()) {
        Ipn::sort(z.data(), z.size());
        std::vector<int32_t>& t = S.t;
        t.assign((size_t)n, 0);
        for (size_t k = z.size(); k-- > 0;) {
            const int64_t i0 = z[k].second;
            if (t[i0] != 0) continue;
            int64_t i = i0, end_i = -1, max_i = i;
            int32_t max_s = 0;
            if (t[i] == 0) {                          // mg_chain_bk_end
                for (;;) {
                    t[i] = 2;
                    end_i = pprev[i];
                    const int32_t s = end_i < 0 ? z[k].first : wsub(z[k].first, f[end_i]);
                    if (s > max_s) { max_s = s; max_i = end_i; }
                    else if (wsub(max_s, s) > P.max_drop) break;
                    if (!(i >= 0 && t[i] == 0 && end_i >= 0)) break;
                    i = end_i;
                }
                for (int64_t ii = i0; ii >= 0 && ii != end_i; ii = pprev[ii]) t[ii] = 0;
            }
            const size_t off = flat.size();
            int64_t j = i0;
            for (; j >= 0 && j != max_i; j = pprev[j]) { flat.push_back((uint32_t)j); t[j] = 1; }
            const int32_t sc = j < 0 ? z[k].first : wsub(z[k].first, f[j]);
            if (sc >= P.min_chain_score && (int64_t)(flat.size() - off) >= (int64_t)P.min_cnt) {
                std::reverse(flat.begin() + off, flat.end());
                scores.push_back(sc);
                parts.push_back({(uint32_t)off, (uint32_t)(flat.size() - off), UINT32_MAX});
            } else {
                flat.resize(off);
            }
        }
    }
    // fallback (lchain.rs:162-173): last argmax f, score v[best].  Unreachable under
    // multi_chain_opts (-m <= k, min_cnt <= 1): anchor 0 has pprev -1 and f = span >= -m, so it
    // always yields a one-anchor chain above; kept for callers with other f / pprev.
    if (parts.empty()) {
        std::vector<int32_t> vv((size_t)n);
        int64_t best = 0;
        for (int64_t i = 0; i < n; ++i) {
            vv[i] = (pprev[i] >= 0 && vv[pprev[i]] > f[i]) ? vv[pprev[i]] : f[i];
            if (f[i] >= f[best]) best = i;
        }
        for (int64_t i = best; i >= 0; i = pprev[i]) flat.push_back((uint32_t)i);
        std::reverse(flat.begin(), flat.end());
        parts.push_back({0, (uint32_t)flat.size(), UINT32_MAX});
        scores.push_back(vv[best]);
    }
    const size_t m = parts.size();
    std::vector<Rng>& rng = S.rng;
    rng.assign(m, Rng{});
    for (size_t c = 0; c < m; ++c)
        for (uint32_t u = 0; u < parts[c].len; ++u) rng[c].add(a, flat[parts[c].off + u]);
    // ---- sort_chains_stable (lchain.rs:202-218)
    std::vector<int32_t>& sq = S.sq;
    std::vector<int32_t>& st = S.st;
    sq.resize(m); st.resize(m);
    for (size_t c = 0; c < m; ++c) { sq[c] = rng[c].q0(); st[c] = rng[c].t0(); }
    std::vector<uint32_t>& ix = S.ix;
    stable_order(S.sd, S.tmp, ix, m, scores.data(), sq.data(), st.data());
    // ---- merge_adjacent_chains_with_gap (lchain.rs:288-314): unwraps last()/first() past the first chain
    if (m >= 2)
        for (const Part& p : parts) if (p.len == 0) { out.panic = true; return; }
    std::vector<Pair>& items = S.items;
    items.resize(m);
    for (size_t i = 0; i < m; ++i) items[i] = {sq[ix[i]], (uint32_t)i};   // i: position in the sorted list
    Ipn::sort(items.data(), items.size());
    std::vector<Merged>& merged = S.merged;
    merged.clear();
    for (const Pair& it : items) {
        const uint32_t c = ix[it.second];
        const Part& pc = parts[c];
        if (merged.empty() || pc.len == 0) { merged.push_back({c, c, pc.len, rng[c]}); continue; }
        Merged& last = merged.back();
        const uint32_t al = flat[parts[last.tail].off + parts[last.tail].len - 1], af = flat[pc.off];
        const bool same = a.rid(al) == a.rid(af) && a.rev(al) == a.rev(af);
        const int32_t qg = wsub(rng[c].q0(), last.r.qe), tg = wsub(rng[c].t0(), last.r.te);
        if (same && qg >= 0 && tg >= 0 && qg <= P.max_gap && tg <= P.max_gap) {
            parts[last.tail].next = c; last.tail = c; last.n += pc.len; last.r.add(rng[c]);
        } else {
            merged.push_back({c, c, pc.len, rng[c]});
        }
    }
    // ---- select_and_filter_chains (lchain.rs:237-260) with the rescued scores: merged chain i takes
    // the i-th score of the sorted pre-merge list
    const size_t mm = merged.size();
    std::vector<int32_t>& ms = S.mscore;
    ms.resize(mm);
    for (size_t i = 0; i < mm; ++i) { ms[i] = scores[ix[i]]; sq[i] = merged[i].r.q0(); st[i] = merged[i].r.t0(); }
    stable_order(S.sd, S.tmp, ix, mm, ms.data(), sq.data(), st.data());
    std::vector<Merged>& ord = S.msorted;
    ord.resize(mm);
    scores.resize(mm);
    for (size_t i = 0; i < mm; ++i) { ord[i] = merged[ix[i]]; scores[i] = ms[ix[i]]; }
    ms.swap(scores);
    // select_primary_secondary (lchain.rs:220-235).  Chain (qs, qe) is secondary iff some primary p
    // overlaps it by o >= o*, o* = min_overlap(...).  A primary with pqs <= qs overlaps by
    // min(qe, pqe) - qs, one with pqs > qs by min(qe - pqs, plen); so the test is a prefix max of pqe
    // and a range max of plen over primaries keyed by pqs: two max segment trees over the query
    // coordinate (or, past 2^20, the sorted distinct qs of all merged chains), O(log) per chain
    // instead of a scan of every primary.
    int32_t qmax_all = 0;
    for (size_t i = 0; i < mm; ++i) qmax_all = std::max(qmax_all, ord[i].r.q0());
    const bool direct = qmax_all < (1 << 20);
    std::vector<int32_t>& keys = S.keys;
    size_t K;
    if (direct) K = (size_t)qmax_all + 1;
    else {
        keys.resize(mm);
        for (size_t i = 0; i < mm; ++i) keys[i] = ord[i].r.q0();
        std::sort(keys.begin(), keys.end());
        keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
        K = keys.size();
    }
    auto rank = [&](int32_t x) -> size_t {           // number of keys <= x
        if (direct) return x < 0 ? 0 : std::min((size_t)x + 1, K);
        return (size_t)(std::upper_bound(keys.begin(), keys.end(), x) - keys.begin());
    };
    size_t T = 1;
    while (T < K) T <<= 1;
    std::vector<int32_t>& tpqe = S.tpqe;
    std::vector<int32_t>& tl = S.tplen;
    tpqe.assign(2 * T, INT32_MIN); tl.assign(2 * T, INT32_MIN);
    auto upd = [&](std::vector<int32_t>& tr, size_t pos, int32_t v) {
        for (size_t x = pos + T; x >= 1; x >>= 1) { if (tr[x] >= v) break; tr[x] = v; }
    };
    auto qmax = [&](const std::vector<int32_t>& tr, size_t lo, size_t hi) {   // [lo, hi)
        int32_t r = INT32_MIN;
        for (size_t l = lo + T, h = hi + T; l < h; l >>= 1, h >>= 1) {
            if (l & 1) r = std::max(r, tr[l++]);
            if (h & 1) r = std::max(r, tr[--h]);
        }
        return r;
    };
    std::vector<uint8_t>& is_pri = S.is_pri;
    is_pri.assign(mm, 1);
    size_t n_prim = 0;
    int32_t p0s = 0, p0e = 0;
    // A chain with the (qs, qe) of an earlier chain is secondary whenever a full overlap passes the
    // test: either that chain became a primary (overlap qe - qs with it) or a primary overlapped it
    // by o >= o*, and the primaries only grow.  Most chains repeat one (one query minimizer hitting
    // many loci), so a hash of the ranges seen settles them before the trees.
    // Direct coordinates: the qe of the first chain at each qs (a chain's qe is set by its qs
    // when it is one anchor, the usual repeat); a miss only means the trees decide.
    std::vector<uint64_t>& seen = S.seen;
    std::vector<int32_t>& first_qe = S.first_qe;
    size_t hcap = 16;
    if (direct) first_qe.assign(K, -1);
    else {
        while (hcap < 2 * mm) hcap <<= 1;
        seen.assign(hcap, ~0ULL);
    }
    auto seen_insert = [&](int32_t qs, int32_t qe) -> bool {   // true if (qs, qe) was seen before
        if (direct) {
            int32_t& f = first_qe[(size_t)qs];
            if (f == qe) return true;
            if (f < 0) f = qe;
            return false;
        }
        const uint64_t key = ((uint64_t)(uint32_t)qs << 32) | (uint32_t)qe;   // never ~0: qs >= 0 fits 31 bits
        size_t h = (size_t)((key * 0x9E3779B97F4A7C15ULL) >> 32) & (hcap - 1);
        for (;; h = (h + 1) & (hcap - 1)) {
            if (seen[h] == key) return true;
            if (seen[h] == ~0ULL) { seen[h] = key; return false; }
        }
    };
    for (size_t ci = 0; ci < mm; ++ci) {
        const int32_t qs = ord[ci].r.q0(), qe = ord[ci].r.qe;
        const int32_t len = std::max(wsub(qe, qs), 1);
        bool ov = false;
        if (seen_insert(qs, qe) && (float)std::max(wsub(qe, qs), 0) / (float)len >= P.mask_level) { is_pri[ci] = 0; continue; }
        const size_t kq = rank(qs);                   // keys <= qs: [0, kq)
        if (n_prim) {
            // the first primary (the best chain) covers most chains: its test alone settles them
            const int32_t o0 = std::max(wsub(std::min(qe, p0e), std::max(qs, p0s)), 0);
            if ((float)o0 / (float)len >= P.mask_level) { is_pri[ci] = 0; continue; }
            const int32_t os = min_overlap(std::max(wsub(qe, qs), 0), len, P.mask_level);
            if (os == 0) ov = true;                   // o = max(., 0) >= 0 against any primary
            else if (os > 0) {
                const int32_t pe = qmax(tpqe, 0, kq);
                if (pe != INT32_MIN && wsub(std::min(qe, pe), qs) >= os) ov = true;
                else {
                    const size_t kh = rank(wsub(qe, os));
                    if (kh > kq && qmax(tl, kq, kh) >= os) ov = true;
                }
            }
        }
        if (ov) { is_pri[ci] = 0; continue; }
        if (!n_prim) { p0s = qs; p0e = qe; }
        upd(tpqe, kq - 1, qe);                        // qs is a key: its slot is kq - 1
        upd(tl, kq - 1, wsub(qe, qs));
        ++n_prim;
    }
    std::vector<uint32_t> sel;
    out.s1 = ms[0];
    int32_t sec = 0;
    for (size_t i = 0; i < mm; ++i) {
        if (i == 0) { sel.push_back(0); continue; }
        if (!is_pri[i]) continue;
        if ((float)ms[i] >= P.pri_ratio * (float)out.s1 && sec < P.best_n) { sel.push_back((uint32_t)i); ++sec; }
        if (out.s2 == 0) out.s2 = ms[i];
    }
    // ---- PAF records (paf.rs:130-222, 238-248)
    std::vector<uint32_t>& ch = S.ch;
    std::vector<int32_t>& cq = S.cq;
    for (size_t si = 0; si < sel.size(); ++si) {
        const Merged& M = ord[sel[si]];
        ch.clear();
        for (uint32_t c = M.head; c != UINT32_MAX; c = parts[c].next) {
            ch.insert(ch.end(), flat.begin() + parts[c].off, flat.begin() + parts[c].off + parts[c].len);
            if (c == M.tail) break;
        }
        if (ch.empty()) continue;                     // paf_from_chain_with_primary -> None
        MultiLine L{};
        L.rev = a.rev(ch[0]) ? 1 : 0;
        const int32_t qs = M.r.q0(), qe = M.r.qe, ts = M.r.t0(), te = M.r.te;
        L.rid = (int32_t)((xy[2 * (size_t)ch[0]] >> 32) & 0x7fffffff);
        if ((uint32_t)L.rid >= n_seq) { out.panic = true; out.lines.clear(); return; }   // idx.seq[rid0]: Q19
        L.qs = qs; L.qe = qe; L.ts = ts; L.te = te; L.cm = (int32_t)ch.size(); L.primary = si == 0;
        // dv (paf.rs:155-199)
        L.dv = 0.0f;
        if (n_mini > 0) {
            cq.clear();
            auto fwd = [&](uint32_t i) { return a.rev(i) ? wsub(wsub(qlen, 1), wsub(wadd(a.qpos(i), 1), a.qspan(i))) : a.qpos(i); };
            if (L.rev) for (size_t t = ch.size(); t-- > 0;) cq.push_back(fwd(ch[t]));
            else for (uint32_t i : ch) cq.push_back(fwd(i));
            const int64_t st0 = find_first(mini_pos, n_mini, cq[0]);
            if (st0 >= 0) {
                int64_t j = st0, en = st0;
                size_t k = 1;
                int32_t n_match = 1;
                while (j + 1 < n_mini && k < cq.size()) {
                    ++j;
                    if (mini_pos[j] == cq[k]) { ++n_match; en = j; ++k; }
                }
                int32_t n_tot = (int32_t)(en - st0 + 1);
                const int32_t rqs = L.rev ? qlen - qe : qs, rqe = L.rev ? qlen - qs : qe;
                const int32_t ak = (int32_t)avg_k;
                if (rqs > ak && ts > ak) ++n_tot;
                if (qlen - rqe > ak && (int32_t)tlen[L.rid] - te > ak) ++n_tot;
                const float frac = (float)n_match / (float)n_tot;
                L.dv = frac >= 1.0f ? 0.0f : 1.0f - powf(frac, 1.0f / std::max(avg_k, 1.0f));
                L.dv_found = true; L.n_match = n_match; L.dv_st = (int32_t)st0; L.dv_en = (int32_t)en;
            }
        }
        (void)idx_k;
        out.lines.push_back(L);
    }
}

}  // namespace mm2g
