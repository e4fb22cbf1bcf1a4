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

using Chain = std::vector<uint32_t>;

void qrange(const Anc& a, const Chain& ch, int32_t& qs, int32_t& qe) {   // lchain.rs:178-188
    qs = INT32_MAX; qe = -1;
    for (uint32_t i : ch) {
        const int32_t s = wsub(a.qpos(i), a.qspan(i) - 1), e = wadd(a.qpos(i), 1);
        qs = std::min(qs, s); qe = std::max(qe, e);
    }
    qs = std::max(qs, 0);
}
void trange(const Anc& a, const Chain& ch, int32_t& ts, int32_t& te) {   // lchain.rs:190-200
    ts = INT32_MAX; te = -1;
    for (uint32_t i : ch) {
        const int32_t s = wsub(a.rpos(i), a.qspan(i) - 1), e = wadd(a.rpos(i), 1);
        ts = std::min(ts, s); te = std::max(te, e);
    }
    ts = std::max(ts, 0);
}

// sort_chains_stable (lchain.rs:202-218) over the first chains.size() scores
void sort_stable(const Anc& a, std::vector<Chain>& chains, std::vector<int32_t>& scores) {
    const size_t m = chains.size();
    std::vector<int32_t> q(m), t(m);
    for (size_t i = 0; i < m; ++i) { int32_t e; qrange(a, chains[i], q[i], e); trange(a, chains[i], t[i], e); }
    std::vector<uint32_t> ix(m);
    for (size_t i = 0; i < m; ++i) ix[i] = (uint32_t)i;
    std::stable_sort(ix.begin(), ix.end(), [&](uint32_t i, uint32_t j) {
        if (scores[i] != scores[j]) return scores[i] > scores[j];
        if (q[i] != q[j]) return q[i] < q[j];
        return t[i] < t[j];
    });
    std::vector<Chain> c2(m);
    std::vector<int32_t> s2(m);
    for (size_t i = 0; i < m; ++i) { c2[i] = std::move(chains[ix[i]]); s2[i] = scores[ix[i]]; }
    chains.swap(c2); scores.swap(s2);
}

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

void multi_chain_read(const uint64_t* xy, const int32_t* f, const int32_t* pprev, int64_t n, int32_t qlen,
                      const int32_t* mini_pos, int64_t n_mini, float avg_k, int32_t idx_k, const uint32_t* tlen, uint32_t n_seq,
                      const MultiParams& P, MultiRead& out) {
    out = MultiRead{};
    if (n <= 0) return;                               // no anchors: chain_dp is empty, no line (main.rs:210-212)
    const Anc a{xy};
    // ---- backtrack (lchain.rs:92-160); the first pass only counts, the second extracts
    std::vector<Pair> z;
    z.reserve((size_t)n);
    for (int64_t i = 0; i < n; ++i) if (f[i] > 0) z.push_back({f[i], (uint32_t)i});
    std::vector<Chain> chains;
    std::vector<int32_t> scores;
    if (!z.empty()) {
        Ipn::sort(z.data(), z.size());
        std::vector<int32_t> t((size_t)n, 0);
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
            Chain v;
            int64_t j = i0;
            for (; j >= 0 && j != max_i; j = pprev[j]) { v.push_back((uint32_t)j); t[j] = 1; }
            const int32_t sc = j < 0 ? z[k].first : wsub(z[k].first, f[j]);
            if (sc >= P.min_chain_score && (int64_t)v.size() >= (int64_t)P.min_cnt) {
                std::reverse(v.begin(), v.end());
                scores.push_back(sc);
                chains.push_back(std::move(v));
            }
        }
    }
    // fallback (lchain.rs:162-173): last argmax f, score v[best].  Unreachable under
    // multi_chain_opts (-m <= k, min_cnt <= 1): anchor 0 has pprev -1 and f = span >= -m, so it
    // always yields a one-anchor chain above; kept for callers with other f / pprev.
    if (chains.empty()) {
        std::vector<int32_t> vv((size_t)n);
        int64_t best = 0;
        for (int64_t i = 0; i < n; ++i) {
            vv[i] = (pprev[i] >= 0 && vv[pprev[i]] > f[i]) ? vv[pprev[i]] : f[i];
            if (f[i] >= f[best]) best = i;
        }
        Chain v;
        for (int64_t i = best; i >= 0; i = pprev[i]) v.push_back((uint32_t)i);
        std::reverse(v.begin(), v.end());
        chains.push_back(std::move(v));
        scores.push_back(vv[best]);
    }
    sort_stable(a, chains, scores);
    // ---- merge_adjacent_chains_with_gap (lchain.rs:288-314): unwraps last()/first() past the first chain
    if (chains.size() >= 2)
        for (const Chain& c : chains) if (c.empty()) { out.panic = true; return; }
    std::vector<Pair> items(chains.size());
    for (size_t i = 0; i < chains.size(); ++i) { int32_t qs, qe; qrange(a, chains[i], qs, qe); items[i] = {qs, (uint32_t)i}; }
    Ipn::sort(items.data(), items.size());
    std::vector<Chain> merged;
    for (const Pair& it : items) {
        const Chain& ch = chains[it.second];
        if (merged.empty()) { merged.push_back(ch); continue; }
        Chain& last = merged.back();
        const uint32_t al = last.back(), af = ch.front();
        const bool same = a.rid(al) == a.rid(af) && a.rev(al) == a.rev(af);
        int32_t lqs, lqe, cqs, cqe, lts, lte, cts, cte;
        qrange(a, last, lqs, lqe); qrange(a, ch, cqs, cqe);
        trange(a, last, lts, lte); trange(a, ch, cts, cte);
        const int32_t qg = wsub(cqs, lqe), tg = wsub(cts, lte);
        if (same && qg >= 0 && tg >= 0 && qg <= P.max_gap && tg <= P.max_gap) last.insert(last.end(), ch.begin(), ch.end());
        else merged.push_back(ch);
    }
    // ---- select_and_filter_chains (lchain.rs:237-260) with the rescued scores (one per pre-merge chain)
    scores.resize(merged.size());
    sort_stable(a, merged, scores);
    std::vector<std::pair<int32_t, int32_t>> prim;    // select_primary_secondary (lchain.rs:220-235)
    std::vector<bool> is_pri(merged.size(), true);
    for (size_t ci = 0; ci < merged.size(); ++ci) {
        int32_t qs, qe; qrange(a, merged[ci], qs, qe);
        bool ov = false;
        for (const auto& p : prim) {
            const float o = (float)std::max(wsub(std::min(qe, p.second), std::max(qs, p.first)), 0);
            const float len = (float)std::max(wsub(qe, qs), 1);
            if (o / len >= P.mask_level) { ov = true; break; }
        }
        if (ov) is_pri[ci] = false; else prim.push_back({qs, qe});
    }
    std::vector<const Chain*> sel;
    out.s1 = scores[0];
    int32_t sec = 0;
    for (size_t i = 0; i < merged.size(); ++i) {
        if (i == 0) { sel.push_back(&merged[0]); continue; }
        if (!is_pri[i]) continue;
        if ((float)scores[i] >= P.pri_ratio * (float)out.s1 && sec < P.best_n) { sel.push_back(&merged[i]); ++sec; }
        if (out.s2 == 0) out.s2 = scores[i];
    }
    // ---- PAF records (paf.rs:130-222, 238-248)
    for (size_t ci = 0; ci < sel.size(); ++ci) {
        const Chain& ch = *sel[ci];
        if (ch.empty()) continue;                     // paf_from_chain_with_primary -> None
        MultiLine L{};
        L.rev = a.rev(ch[0]) ? 1 : 0;
        int32_t qs = INT32_MAX, qe = -1, ts = INT32_MAX, te = -1;
        for (uint32_t i : ch) {
            qs = std::min(qs, wsub(a.qpos(i), a.qspan(i) - 1)); qe = std::max(qe, wadd(a.qpos(i), 1));
            ts = std::min(ts, wsub(a.rpos(i), a.qspan(i) - 1)); te = std::max(te, wadd(a.rpos(i), 1));
        }
        qs = std::max(qs, 0); ts = std::max(ts, 0);
        L.rid = (int32_t)((xy[2 * (size_t)ch[0]] >> 32) & 0x7fffffff);
        if ((uint32_t)L.rid >= n_seq) { out.panic = true; out.lines.clear(); return; }   // idx.seq[rid0]: Q19
        L.qs = qs; L.qe = qe; L.ts = ts; L.te = te; L.cm = (int32_t)ch.size(); L.primary = ci == 0;
        // dv (paf.rs:155-199)
        L.dv = 0.0f;
        if (n_mini > 0) {
            std::vector<int32_t> cq;
            cq.reserve(ch.size());
            auto fwd = [&](uint32_t i) { return a.rev(i) ? wsub(wsub(qlen, 1), wsub(wadd(a.qpos(i), 1), a.qspan(i))) : a.qpos(i); };
            if (L.rev) for (size_t t = ch.size(); t-- > 0;) cq.push_back(fwd(ch[t]));
            else for (uint32_t i : ch) cq.push_back(fwd(i));
            const int64_t st = find_first(mini_pos, n_mini, cq[0]);
            if (st >= 0) {
                int64_t j = st, en = st;
                size_t k = 1;
                int32_t n_match = 1;
                while (j + 1 < n_mini && k < cq.size()) {
                    ++j;
                    if (mini_pos[j] == cq[k]) { ++n_match; en = j; ++k; }
                }
                int32_t n_tot = (int32_t)(en - st + 1);
                const int32_t rqs = L.rev ? qlen - qe : qs, rqe = L.rev ? qlen - qs : qe;
                const int32_t ak = (int32_t)avg_k;
                if (rqs > ak && ts > ak) ++n_tot;
                if (qlen - rqe > ak && (int32_t)tlen[L.rid] - te > ak) ++n_tot;
                const float frac = (float)n_match / (float)n_tot;
                L.dv = frac >= 1.0f ? 0.0f : 1.0f - powf(frac, 1.0f / std::max(avg_k, 1.0f));
                L.dv_found = true; L.n_match = n_match; L.dv_st = (int32_t)st; L.dv_en = (int32_t)en;
            }
        }
        (void)idx_k;
        out.lines.push_back(L);
    }
}

}  // namespace mm2g
