// ============================================================================
// mm2rs CPU ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A line-by-line C++17 restatement of the reference Rust crate `mm2rs`
// (xuzhougeng/minimap2_rs @ 2025-08-24, /root/reference/src/*.rs).  It is the
// parity checker for the MI355X path and the CPU baseline ("kind": "port") in
// bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load it.  The product (minimap2_rs_amd/, libmm2g.so, the mm2rs CLI)
// never links or calls it.
//
// PARITY UNPINNED: the reference has no tests, no golden vectors and no
// fixtures; its only final-code known answer
// (README.md:24-26) needs hg38 chr8+chr12 and a read that are not in this
// container, and the Rust toolchain needed to run the reference is absent.
// This restatement is therefore checked only against itself (committed
// fixtures in tests/golden/ generated from it) and against an independent
// pure-Python restatement of the same Rust on small inputs (tests/).
//
// Arithmetic conventions:
//  * Rust release profile => wrapping u64 arithmetic in hash64 (Q18).
//  * f32 math evaluated op-by-op, compiled with -ffp-contract=off (Rust never
//    contracts).  logf/powf come from glibc, as Rust's f32::ln/powf lower to
//    libm calls on x86-64 Linux.
//  * Rust `as i32` from f32 saturates (NaN -> 0): sat_f32_to_i32().
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>
#include <atomic>
#include <chrono>

namespace orc {

typedef uint64_t u64;
typedef uint32_t u32;

// ---------------------------------------------------------------- nt4.rs:2-10
static inline uint8_t nt4(uint8_t b) {
    switch (b) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 4;
    }
}

// ------------------------------------------------------------- sketch.rs:4-13
static inline u64 hash64(u64 key, u64 mask) {
    key = ((~key) + (key << 21)) & mask;       // wrapping_add
    key ^= key >> 24;
    key = (key + (key << 3) + (key << 8)) & mask;
    key ^= key >> 14;
    key = (key + (key << 2) + (key << 4)) & mask;
    key ^= key >> 28;
    key = (key + (key << 31)) & mask;
    return key;
}

// sketch.rs:15-19
struct Minimizer { u64 key_span; u64 rid_pos_strand; };

// sketch.rs:21-27
struct TinyQueue {
    size_t front = 0, count = 0; int32_t a[32];
    void clear() { front = 0; count = 0; }
    void push(int32_t x) { size_t idx = (count + front) & 0x1f; a[idx] = x; count += 1; }
    int32_t shift() { if (count == 0) return -1; int32_t x = a[front]; front = (front + 1) & 0x1f; count -= 1; return x; }
};

// sketch.rs:29-100 (panics on bad args -> here: returns false)
static bool sketch_sequence(const uint8_t* seq, size_t len, size_t w, size_t k, u32 rid,
                            bool is_hpc, std::vector<Minimizer>& out) {
    if (len == 0) return false;                    // assert!(!seq.is_empty())
    if (!(w > 0 && w < 256)) return false;         // assert!(w > 0 && w < 256)
    if (!(k > 0 && k <= 28)) return false;         // assert!(k > 0 && k <= 28)
    const u64 shift1 = 2 * ((u64)k - 1);
    const u64 mask = (1ULL << (2 * k)) - 1;
    u64 kmer[2] = {0, 0};
    int32_t l = 0;
    size_t buf_pos = 0, min_pos = 0;
    int32_t kmer_span = 0;
    const u64 MAX = ~0ULL;
    std::vector<std::pair<u64, u64>> buf(w, {MAX, MAX});
    std::pair<u64, u64> mn = {MAX, MAX};
    TinyQueue tq;
    const int32_t wi = (int32_t)w, ki = (int32_t)k;
    auto emit = [&](const std::pair<u64, u64>& m) { out.push_back(Minimizer{m.first, m.second}); };
    for (size_t i = 0; i < len; ++i) {
        int32_t c = nt4(seq[i]);
        std::pair<u64, u64> info = {MAX, MAX};
        if (c < 4) {
            if (is_hpc) {
                size_t skip_len = 1;
                if (i + 1 < len && (int32_t)nt4(seq[i + 1]) == c) {
                    size_t t = i + 2;
                    while (t < len && (int32_t)nt4(seq[t]) == c) t += 1;
                    skip_len = t - i;
                }
                tq.push((int32_t)skip_len);
                kmer_span += (int32_t)skip_len;
                if ((int32_t)tq.count > ki) kmer_span -= tq.shift();
            } else {
                kmer_span = (l + 1 < ki) ? l + 1 : ki;
            }
            kmer[0] = ((kmer[0] << 2) | (u64)c) & mask;
            kmer[1] = (kmer[1] >> 2) | (((u64)(3 ^ c)) << shift1);
            if (kmer[0] != kmer[1]) {
                int z = kmer[0] < kmer[1] ? 0 : 1;
                l += 1;
                if (l >= ki && kmer_span < 256) {
                    u64 key_span = (hash64(kmer[z], mask) << 8) | (u64)kmer_span;
                    u64 rps = ((u64)rid << 32) | ((u64)i << 1) | (u64)z;
                    info = {key_span, rps};
                }
            }
        } else {
            l = 0; tq.clear(); kmer_span = 0;
        }
        buf[buf_pos] = info;
        if (l == wi + ki - 1 && mn.first != MAX) {
            for (size_t j = buf_pos + 1; j < w; ++j) if (mn.first == buf[j].first && buf[j].second != mn.second) emit(buf[j]);
            for (size_t j = 0; j < buf_pos; ++j) if (mn.first == buf[j].first && buf[j].second != mn.second) emit(buf[j]);
        }
        if (info.first <= mn.first) {
            if (l >= wi + ki && mn.first != MAX) emit(mn);
            mn = info; min_pos = buf_pos;
        } else if (buf_pos == min_pos) {
            if (l >= wi + ki - 1 && mn.first != MAX) emit(mn);
            mn.first = MAX;
            for (size_t j = buf_pos + 1; j < w; ++j) if (mn.first >= buf[j].first) { mn = buf[j]; min_pos = j; }
            for (size_t j = 0; j <= buf_pos; ++j) if (mn.first >= buf[j].first) { mn = buf[j]; min_pos = j; }
            if (l >= wi + ki - 1 && mn.first != MAX) {
                for (size_t j = buf_pos + 1; j < w; ++j) if (mn.first == buf[j].first && mn.second != buf[j].second) emit(buf[j]);
                for (size_t j = 0; j <= buf_pos; ++j) if (mn.first == buf[j].first && mn.second != buf[j].second) emit(buf[j]);
            }
        }
        buf_pos += 1; if (buf_pos == w) buf_pos = 0;
    }
    if (mn.first != MAX) emit(mn);
    return true;
}

// ------------------------------------------------------------- index.rs:1-475
static inline size_t kroundup64(size_t x) { x -= 1; x |= x >> 1; x |= x >> 2; x |= x >> 4; x |= x >> 8; x |= x >> 16; x |= x >> 32; return x + 1; }

static inline void mm_seq4_set(std::vector<u32>& S, u64 o, uint8_t c) {   // index.rs:14-19
    size_t i = (size_t)(o >> 3);
    unsigned shift = (unsigned)((o & 7) << 2);
    u32 v = S[i];
    S[i] = (v & ~(0xFu << shift)) | ((((u32)c) & 0xF) << shift);
}

struct IndexSeq { bool has_name; std::string name; u64 offset; u32 len; bool is_alt; };
struct Bucket { std::vector<Minimizer> a; std::vector<u64> p; bool has_h = false; std::unordered_map<u64, u64> h; };

struct Index {   // index.rs:33-42
    int32_t w, k, b, flag;
    u32 n_seq = 0;
    std::vector<IndexSeq> seq;
    std::vector<u32> S;
    std::vector<Bucket> B;
    Index(int32_t w_, int32_t k_, int32_t b_, int32_t flag_) : w(w_), k(k_), b(b_), flag(flag_) { B.resize((size_t)1 << b_); }

    void add_minimizers(const std::vector<Minimizer>& v) {   // index.rs:69-72
        u64 mask = (1ULL << b) - 1;
        for (const auto& m : v) B[(size_t)((m.key_span >> 8) & mask)].a.push_back(m);
    }

    void post_process_bucket(Bucket& bk) {   // index.rs:77-108 (one bucket)
        if (bk.a.empty()) return;
        std::stable_sort(bk.a.begin(), bk.a.end(), [](const Minimizer& x, const Minimizer& y) { return (x.key_span >> 8) < (y.key_span >> 8); });
        int32_t n = 1; size_t total_p = 0;
        for (size_t j = 1; j <= bk.a.size(); ++j) {
            if (j == bk.a.size() || (bk.a[j].key_span >> 8) != (bk.a[j - 1].key_span >> 8)) { if (n > 1) total_p += (size_t)n; n = 1; } else n += 1;
        }
        bk.p.assign(total_p, 0);
        std::unordered_map<u64, u64> h;
        n = 1; size_t start_a = 0, start_p = 0;
        for (size_t j = 1; j <= bk.a.size(); ++j) {
            if (j == bk.a.size() || (bk.a[j].key_span >> 8) != (bk.a[j - 1].key_span >> 8)) {
                const Minimizer& p = bk.a[j - 1];
                u64 key_top = ((p.key_span >> 8) >> b) << 1;
                if (n == 1) {
                    h[key_top | 1] = p.rid_pos_strand;
                } else {
                    for (int32_t kk = 0; kk < n; ++kk) bk.p[start_p + kk] = bk.a[start_a + kk].rid_pos_strand;
                    std::sort(bk.p.begin() + start_p, bk.p.begin() + start_p + n);
                    h[key_top] = ((u64)start_p << 32) | (u64)n;
                    start_p += (size_t)n;
                }
                start_a = j; n = 1;
            } else n += 1;
        }
        bk.h = std::move(h); bk.has_h = true;
        bk.a.clear(); bk.a.shrink_to_fit();
    }

    void post_process(int nthreads) {   // index.rs:74-109 (rayon par_iter over buckets)
        size_t nb = B.size();
        if (nthreads <= 1) { for (auto& bk : B) post_process_bucket(bk); return; }
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t)
            th.emplace_back([&, t]() { for (size_t i = t; i < nb; i += nthreads) post_process_bucket(B[i]); });
        for (auto& x : th) x.join();
    }

    void stats(u64& n_keys, double& avg_occ, double& avg_spacing, u64& total_len) const {   // index.rs:111-122
        n_keys = 0; u64 sum_occ = 0;
        for (const auto& bk : B) if (bk.has_h) for (const auto& kv : bk.h) {
            if ((kv.first & 1) == 1) { n_keys += 1; sum_occ += 1; } else { n_keys += 1; sum_occ += (kv.second & 0xffffffffULL); }
        }
        total_len = 0; for (const auto& s : seq) total_len += s.len;
        avg_occ = n_keys > 0 ? (double)sum_occ / (double)n_keys : 0.0;
        avg_spacing = sum_occ > 0 ? (double)total_len / (double)sum_occ : 0.0;
    }

    int32_t calc_mid_occ(float frac) const {   // index.rs:124-141
        std::vector<u32> counts;
        for (const auto& bk : B) if (bk.has_h) for (const auto& kv : bk.h)
            counts.push_back((kv.first & 1) == 1 ? 1u : (u32)(kv.second & 0xffffffffULL));
        if (counts.empty()) return INT32_MAX;
        std::sort(counts.begin(), counts.end());
        size_t n = counts.size();
        double fidx = (1.0 - (double)frac) * (double)n;
        size_t idx = fidx <= 0.0 ? 0 : (size_t)fidx;     // Rust f64 `as usize` saturates
        if (idx > n - 1) idx = n - 1;
        return (int32_t)counts[idx] + 1;
    }

    // index.rs:143-154.  kind: 0 none, 1 single (val), 2 multi (ptr,n)
    int get(u64 minier, u64& single, const u64*& slice, size_t& n) const {
        u64 mask = (1ULL << b) - 1;
        const Bucket& bk = B[(size_t)(minier & mask)];
        if (!bk.has_h) return 0;
        u64 key = (minier >> b) << 1;
        auto it = bk.h.find(key | 1);
        if (it != bk.h.end()) { single = it->second; return 1; }
        it = bk.h.find(key);
        if (it != bk.h.end()) {
            size_t off = (size_t)(it->second >> 32); n = (size_t)(it->second & 0xffffffffULL);
            slice = bk.p.data() + off; return 2;
        }
        return 0;
    }
};

// ---- FASTA reading (noodles-fasta stand-in: name = header up to first
// whitespace; sequence lines concatenated, '\r' stripped).  Parity unpinned
// at this boundary.
struct FastaRec { std::string name; std::string seq; };
static bool read_fasta(const char* path, std::vector<FastaRec>& recs, bool first_only) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return false;
    std::string data;
    {
        std::vector<char> buf(1 << 22);
        size_t nr;
        while ((nr = fread(buf.data(), 1, buf.size(), fp)) > 0) data.append(buf.data(), nr);
    }
    fclose(fp);
    size_t pos = 0, n = data.size();
    bool have = false;
    while (pos < n) {
        size_t e = data.find('\n', pos);
        if (e == std::string::npos) e = n;
        size_t le = e;
        if (le > pos && data[le - 1] == '\r') --le;
        if (le > pos && data[pos] == '>') {
            if (have && first_only) break;
            size_t ne = pos + 1;
            while (ne < le && data[ne] != ' ' && data[ne] != '\t') ++ne;
            recs.push_back(FastaRec{data.substr(pos + 1, ne - pos - 1), std::string()});
            have = true;
        } else if (have) {
            recs.back().seq.append(data, pos, le - pos);
        }
        pos = e + 1;
    }
    return true;
}

// index.rs:427-475
static Index* build_index_from_recs(const std::vector<FastaRec>& records, int32_t w, int32_t k, int32_t b, int32_t flag, int nthreads) {
    Index* idx = new Index(w, k, b, flag);
    idx->n_seq = (u32)records.size();
    bool is_hpc = (flag & 1) != 0;
    std::vector<std::vector<Minimizer>> minis(records.size());
    {
        std::vector<std::thread> th;
        int nt = std::max(1, nthreads);
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t]() {
                for (size_t rid = t; rid < records.size(); rid += nt)
                    if (!records[rid].seq.empty())
                        sketch_sequence((const uint8_t*)records[rid].seq.data(), records[rid].seq.size(), (size_t)w, (size_t)k, (u32)rid, is_hpc, minis[rid]);
            });
        for (auto& x : th) x.join();
    }
    u64 total_len = 0; for (const auto& r : records) total_len += r.seq.size();
    size_t words = kroundup64((size_t)((total_len + 7) / 8));
    idx->S.assign(words, 0);
    u64 sum_len = 0;
    for (size_t rid = 0; rid < records.size(); ++rid) {
        const std::string& s = records[rid].seq;
        for (size_t j = 0; j < s.size(); ++j) mm_seq4_set(idx->S, sum_len + j, nt4((uint8_t)s[j]));
        idx->seq.push_back(IndexSeq{true, records[rid].name, sum_len, (u32)s.size(), false});
        idx->add_minimizers(minis[rid]);
        std::vector<Minimizer>().swap(minis[rid]);
        sum_len += s.size();
    }
    idx->post_process(nthreads);
    return idx;
}

// index.rs:233-307 — hash entries written in ascending key order (Rust: HashMap order, Q11)
static bool save_to_mmi(const Index& idx, const char* path) {
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    fwrite("MMI\x02", 1, 4, f);
    u32 hdr[5] = {(u32)idx.w, (u32)idx.k, (u32)idx.b, (u32)idx.seq.size(), (u32)idx.flag};
    fwrite(hdr, 4, 5, f);
    u64 sum_len = 0;
    for (const auto& s : idx.seq) {
        if (s.has_name) { uint8_t l = (uint8_t)std::min<size_t>(s.name.size(), 255); fwrite(&l, 1, 1, f); fwrite(s.name.data(), 1, l, f); }
        else { uint8_t z = 0; fwrite(&z, 1, 1, f); }
        fwrite(&s.len, 4, 1, f);
        sum_len += s.len;
    }
    size_t nb = (size_t)1 << idx.b;
    std::vector<std::pair<u64, u64>> kv;
    for (size_t i = 0; i < nb; ++i) {
        const Bucket& bk = idx.B[i];
        u32 n = (u32)bk.p.size(); fwrite(&n, 4, 1, f);
        if (n) fwrite(bk.p.data(), 8, n, f);
        u32 size = bk.has_h ? (u32)bk.h.size() : 0; fwrite(&size, 4, 1, f);
        if (bk.has_h) {
            kv.assign(bk.h.begin(), bk.h.end());
            std::sort(kv.begin(), kv.end());
            for (auto& e : kv) { fwrite(&e.first, 8, 1, f); fwrite(&e.second, 8, 1, f); }
        }
    }
    size_t words = (size_t)((sum_len + 7) / 8);
    if (words) fwrite(idx.S.data(), 4, words, f);
    fclose(f);
    return true;
}

// index.rs:361-424
static Index* load_from_mmi(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return nullptr;
    auto rd = [&](void* p, size_t n) -> bool { return fread(p, 1, n, f) == n; };
    char magic[4];
    if (!rd(magic, 4) || memcmp(magic, "MMI\x02", 4) != 0) { fclose(f); return nullptr; }
    u32 hdr[5]; if (!rd(hdr, 20)) { fclose(f); return nullptr; }
    Index* idx = new Index((int32_t)hdr[0], (int32_t)hdr[1], (int32_t)hdr[2], (int32_t)hdr[4]);
    idx->n_seq = hdr[3];
    u64 sum_len = 0;
    for (u32 i = 0; i < hdr[3]; ++i) {
        uint8_t nl; if (!rd(&nl, 1)) { delete idx; fclose(f); return nullptr; }
        IndexSeq s; s.has_name = nl > 0; s.name.assign(nl, '\0');
        if (nl && !rd(&s.name[0], nl)) { delete idx; fclose(f); return nullptr; }
        u32 len; if (!rd(&len, 4)) { delete idx; fclose(f); return nullptr; }
        s.offset = sum_len; s.len = len; s.is_alt = false; sum_len += len;
        idx->seq.push_back(s);
    }
    size_t nb = (size_t)1 << idx->b;
    for (size_t i = 0; i < nb; ++i) {
        u32 n; if (!rd(&n, 4)) { delete idx; fclose(f); return nullptr; }
        Bucket& bk = idx->B[i];
        bk.p.resize(n); if (n && !rd(bk.p.data(), 8 * (size_t)n)) { delete idx; fclose(f); return nullptr; }
        u32 size; if (!rd(&size, 4)) { delete idx; fclose(f); return nullptr; }
        if (size > 0) {
            bk.has_h = true; bk.h.reserve(size);
            for (u32 j = 0; j < size; ++j) { u64 kk, vv; if (!rd(&kk, 8) || !rd(&vv, 8)) { delete idx; fclose(f); return nullptr; } bk.h[kk] = vv; }
        }
    }
    size_t words = (size_t)((sum_len + 7) / 8);
    idx->S.assign(words, 0);
    if (words && !rd(idx->S.data(), 4 * words)) { delete idx; fclose(f); return nullptr; }
    fclose(f);
    return idx;
}

// ------------------------------------------------------------- seeds.rs:1-79
struct Anchor { u64 x, y; };

static std::vector<Minimizer> collect_query_minimizers(const uint8_t* seq, size_t len, size_t w, size_t k) {   // seeds.rs:7-11
    std::vector<Minimizer> v;
    if (!sketch_sequence(seq, len, w, k, 0, false, v)) { fprintf(stderr, "oracle: sketch_sequence assertion failed (empty seq or bad w/k)\n"); abort(); }
    return v;
}

static void filter_query_minimizers(std::vector<Minimizer>& mv, int32_t q_occ_max, float q_occ_frac) {   // seeds.rs:13-36
    if (mv.empty() || q_occ_frac <= 0.0f || q_occ_max <= 0) return;
    if ((int32_t)mv.size() <= q_occ_max) return;
    std::vector<std::pair<u64, size_t>> keys; keys.reserve(mv.size());
    for (size_t i = 0; i < mv.size(); ++i) keys.push_back({mv[i].key_span >> 8, i});
    std::sort(keys.begin(), keys.end(), [](const std::pair<u64, size_t>& a, const std::pair<u64, size_t>& b) { return a.first < b.first; });
    std::vector<bool> keep(mv.size(), true);
    size_t st = 0, n = keys.size();
    float prod = (float)mv.size() * q_occ_frac;
    size_t cutoff = prod <= 0.0f ? 0 : (size_t)prod;                 // f32 `as usize` (saturating)
    for (size_t i = 1; i <= n; ++i) {
        if (i == n || keys[i].first != keys[st].first) {
            size_t cnt = i - st;
            if ((int32_t)cnt > q_occ_max && cnt > cutoff) for (size_t j = st; j < i; ++j) keep[keys[j].second] = false;
            st = i;
        }
    }
    size_t j = 0;
    for (size_t i = 0; i < mv.size(); ++i) if (keep[i]) mv[j++] = mv[i];
    mv.resize(j);
}

static inline void push_anchor(std::vector<Anchor>& out, u64 r, const Minimizer& m, int32_t qlen) {   // seeds.rs:62-79
    u64 rid = (r >> 32) & 0xffffffffULL;
    int32_t rpos = (int32_t)((r >> 1) & 0xffffffffULL);
    int32_t rstrand = (int32_t)(r & 1);
    int32_t qpos = (int32_t)((m.rid_pos_strand >> 1) & 0xffffffffULL);
    int32_t qstrand = (int32_t)(m.rid_pos_strand & 1);
    int32_t qspan = (int32_t)(m.key_span & 0xff);
    bool forward = rstrand == qstrand;
    // `rpos as u64` sign-extends an i32: for odd rid the rid's low bit sits in
    // bit 31 of rpos (the `(r >> 1) & 0xffffffff` above), so x's top 32 bits
    // become all ones — rev=1, rid=0x7fffffff for BOTH strands.
    u64 x = forward ? ((rid << 32) | (u64)(int64_t)rpos) : ((1ULL << 63) | (rid << 32) | (u64)(int64_t)rpos);
    u64 y;
    if (forward) y = ((u64)(uint32_t)qspan << 32) | (u64)(int64_t)qpos;
    else {
        // (qlen - (qpos + 1 - qspan) - 1) as u64 : i32 -> u64 sign-extends
        int32_t qp = (int32_t)((uint32_t)qlen - ((uint32_t)qpos + 1u - (uint32_t)qspan) - 1u);
        y = ((u64)(uint32_t)qspan << 32) | (u64)(int64_t)qp;
    }
    out.push_back(Anchor{x, y});
}

static std::vector<Anchor> build_anchors_filtered(const Index& idx, const std::vector<Minimizer>& mv, int32_t qlen, int32_t mid_occ) {   // seeds.rs:42-60
    std::vector<Anchor> a;
    for (const auto& m : mv) {
        u64 minier = m.key_span >> 8;
        u64 single; const u64* slice; size_t n;
        int kind = idx.get(minier, single, slice, n);
        if (kind == 1) push_anchor(a, single, m, qlen);
        else if (kind == 2) {
            if ((int32_t)n > mid_occ) continue;
            for (size_t t = 0; t < n; ++t) push_anchor(a, slice[t], m, qlen);
        }
    }
    std::stable_sort(a.begin(), a.end(), [](const Anchor& p, const Anchor& q) { return p.x == q.x ? p.y < q.y : p.x < q.x; });
    return a;
}

// ------------------------------------------------------------ lchain.rs:1-330
static inline int32_t qpos(const Anchor& a) { return (int32_t)(a.y & 0xffffffffULL); }
static inline int32_t qspan(const Anchor& a) { return (int32_t)((a.y >> 32) & 0xff); }
static inline int32_t rpos(const Anchor& a) { return (int32_t)(a.x & 0xffffffffULL); }
static inline bool rev(const Anchor& a) { return (a.x >> 63) != 0; }
static inline int32_t rid(const Anchor& a) { return (int32_t)((a.x >> 32) & 0x7fffffff); }
static inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

static inline int32_t sat_f32_to_i32(float v) {   // Rust `f32 as i32`
    if (std::isnan(v)) return 0;
    if (v >= 2147483647.0f) return INT32_MAX;
    if (v <= -2147483648.0f) return INT32_MIN;
    return (int32_t)v;
}

static inline float mg_log2(int32_t x) {   // lchain.rs:15
    if (x <= 1) return 0.0f;
    return logf((float)x) / 0.693147180559945309417232121458176568f;
}

struct ChainParams {   // lchain.rs:36-52
    int32_t max_dist_x, max_dist_y, bw, max_chain_iter, min_chain_score, min_cnt;
    float chn_pen_gap, chn_pen_skip;
    int32_t max_chain_skip, max_drop, bw_long, rmq_rescue_size;
    float rmq_rescue_ratio;
};

// lchain.rs:17-34
static inline bool comput_sc(const Anchor& ai, const Anchor& aj, int32_t max_dist_x, int32_t max_dist_y, int32_t bw,
                             float chn_pen_gap, float chn_pen_skip, int32_t& out) {
    int32_t dq = wsub(qpos(ai), qpos(aj));
    if (dq <= 0 || dq > max_dist_x) return false;
    int32_t dr = wsub(rpos(ai), rpos(aj));
    if (dr == 0 || dq > max_dist_y) return false;
    int32_t dd = std::abs(wsub(dr, dq));
    if (dd > bw) return false;
    int32_t dg = std::min(dr, dq);
    int32_t q_span = qspan(aj);
    int32_t sc = std::min(q_span, dg);
    if (dd != 0 || dg > q_span) {
        float lin_pen = chn_pen_gap * (float)dd + chn_pen_skip * (float)dg;
        float log_pen = dd >= 1 ? mg_log2(dd + 1) : 0.0f;
        sc = wsub(sc, sat_f32_to_i32(lin_pen + 0.5f * log_pen));
    }
    out = sc;
    return true;
}

struct ChainStats { u64 inner_iters = 0; };

struct DpResult { std::vector<std::vector<size_t>> chains; std::vector<int32_t> scores; std::vector<int32_t> f; std::vector<int64_t> pprev; };

static void sort_chains_stable(const std::vector<Anchor>& anchors, std::vector<std::vector<size_t>>& chains, std::vector<int32_t>& scores);

// ----------------------------------------------------------- Rust sort_unstable
// `slice::sort_unstable_by_key` (lchain.rs:97 z by f, :267 / :292 merge items by
// qs) leaves the order of equal keys to the std algorithm, which changed in
// rustc 1.81.  Both are restated here from rust-lang/rust library/core (no Rust
// toolchain in this image: unpinned, DESIGN.md §2 "-n <= 1"); the element type
// is the reference's `(i32, usize)` (16 B, Copy) with is_less = key a < key b.
//   ipnsort   (1.81+): core/src/slice/sort/unstable/{mod,quicksort,heapsort}.rs,
//                      shared/pivot.rs, shared/smallsort.rs
//   pdqsort (<= 1.80): core/src/slice/sort.rs (quicksort / recurse)
namespace rsort {
template <typename E, typename L>
static void insert_tail(E* v, size_t i, L& lt) {   // v[..i] sorted; insert v[i] (stable)
    if (!lt(v[i], v[i - 1])) return;
    E tmp = v[i];
    size_t j = i;
    do { v[j] = v[j - 1]; --j; } while (j > 0 && lt(tmp, v[j - 1]));
    v[j] = tmp;
}
template <typename E, typename L>
static void insertion_sort_shift_left(E* v, size_t len, size_t offset, L& lt) {
    for (size_t i = offset; i < len; ++i) insert_tail(v, i, lt);
}
template <typename E, typename L>
static void insert_head(E* v, size_t len, L& lt) {   // v[1..] sorted; insert v[0] (insertion_sort_shift_right, offset 1)
    if (len < 2 || !lt(v[1], v[0])) return;
    E tmp = v[0];
    size_t i = 1;
    v[0] = v[1];
    while (i + 1 < len && lt(v[i + 1], tmp)) { v[i] = v[i + 1]; ++i; }
    v[i] = tmp;
}
// heapsort: 1.81's single loop and the older build-then-pop loops perform the
// same sift-downs in the same order
template <typename E, typename L>
static void sift_down(E* v, size_t len, size_t node, L& lt) {
    for (;;) {
        size_t child = 2 * node + 1;
        if (child >= len) break;
        if (child + 1 < len) child += lt(v[child], v[child + 1]) ? 1 : 0;
        if (!lt(v[node], v[child])) break;
        std::swap(v[node], v[child]);
        node = child;
    }
}
template <typename E, typename L>
static void heapsort(E* v, size_t len, L& lt) {
    for (size_t i = len + len / 2; i-- > 0;) {
        size_t sift_idx;
        if (i >= len) sift_idx = i - len;
        else { std::swap(v[0], v[i]); sift_idx = 0; }
        sift_down(v, std::min(i, len), sift_idx, lt);
    }
}

// ---- ipnsort (1.81+)
// small_sort_general (smallsort.rs): sort8_stable / sort4_stable presorting, insert_tail and
// bidirectional_merge are all stable, so for a strict weak order it is a stable sort of the slice.
template <typename E, typename L>
static void small_sort_general(E* v, size_t len, L& lt) {
    std::stable_sort(v, v + len, [&](const E& a, const E& b) { return lt(a, b); });
}
template <typename E, typename L>
static size_t median3(const E* v, size_t a, size_t b, size_t c, L& lt) {   // pivot.rs median3
    const bool x = lt(v[a], v[b]), y = lt(v[a], v[c]);
    if (x == y) { const bool z = lt(v[b], v[c]); return (z ^ x) ? c : b; }
    return a;
}
template <typename E, typename L>
static size_t median3_rec(const E* v, size_t a, size_t b, size_t c, size_t n, L& lt) {
    if (n * 8 >= 64) {
        const size_t n8 = n / 8;
        a = median3_rec(v, a, a + n8 * 4, a + n8 * 7, n8, lt);
        b = median3_rec(v, b, b + n8 * 4, b + n8 * 7, n8, lt);
        c = median3_rec(v, c, c + n8 * 4, c + n8 * 7, n8, lt);
    }
    return median3(v, a, b, c, lt);
}
template <typename E, typename L>
static size_t choose_pivot_ipn(const E* v, size_t len, L& lt) {   // pivot.rs choose_pivot (len >= 8)
    const size_t d8 = len / 8, a = 0, b = d8 * 4, c = d8 * 7;
    return len < 64 ? median3(v, a, b, c, lt) : median3_rec(v, a, b, c, d8, lt);
}
// partition_lomuto_branchless_cyclic (quicksort.rs; sizeof(T) <= 96), on w = v[1..]
template <typename E, typename P>
static size_t lomuto_cyclic(E* w, size_t n, const E& pivot, P& lt) {
    if (n == 0) return 0;
    E tmp = w[0];
    size_t gap = 0, num_lt = 0;
    for (size_t right = 1; right <= n; ++right) {
        const E rv = right < n ? w[right] : tmp;   // the last step takes the saved first element
        const bool is_lt = lt(rv, pivot);
        w[gap] = w[num_lt];
        w[num_lt] = rv;
        gap = right;                               // (after the last step the gap is the temporary)
        num_lt += is_lt ? 1 : 0;
    }
    return num_lt;
}
template <typename E, typename P>
static size_t partition_ipn(E* v, size_t len, size_t pivot, P& lt) {
    std::swap(v[0], v[pivot]);
    const E pv = v[0];
    const size_t num_lt = lomuto_cyclic(v + 1, len - 1, pv, lt);
    std::swap(v[0], v[num_lt]);
    return num_lt;
}
template <typename E, typename L>
static void quicksort_ipn(E* v, size_t len, const E* ancestor, uint32_t limit, L& lt) {
    E anc_val{};
    bool has_anc = ancestor != nullptr;
    if (has_anc) anc_val = *ancestor;
    for (;;) {
        if (len <= 32) { small_sort_general(v, len, lt); return; }   // SMALL_SORT_GENERAL_THRESHOLD (16-B Copy type)
        if (limit == 0) { heapsort(v, len, lt); return; }
        limit -= 1;
        const size_t pp = choose_pivot_ipn(v, len, lt);
        if (has_anc && !lt(anc_val, v[pp])) {
            auto le = [&](const E& a, const E& b) { return !lt(b, a); };
            const size_t num_le = partition_ipn(v, len, pp, le);
            v += num_le + 1; len -= num_le + 1;
            has_anc = false;
            continue;
        }
        const size_t num_lt = partition_ipn(v, len, pp, lt);
        quicksort_ipn(v, num_lt, has_anc ? &anc_val : nullptr, limit, lt);
        anc_val = v[num_lt]; has_anc = true;
        v += num_lt + 1; len -= num_lt + 1;
    }
}
template <typename E, typename L>
static void ipnsort(E* v, size_t len, L lt) {   // unstable/mod.rs sort + ipnsort
    if (len < 2) return;
    if (len <= 20) { insertion_sort_shift_left(v, len, 1, lt); return; }
    size_t run = 2;                                 // find_existing_run
    const bool desc = lt(v[1], v[0]);
    if (desc) while (run < len && lt(v[run], v[run - 1])) ++run;
    else while (run < len && !lt(v[run], v[run - 1])) ++run;
    if (run == len) { if (desc) std::reverse(v, v + len); return; }
    uint32_t lg = 0;
    for (size_t x = len | 1; x > 1; x >>= 1) ++lg;
    quicksort_ipn(v, len, (const E*)nullptr, 2 * lg, lt);
}

// ---- pdqsort (<= 1.80)
template <typename E>
static void break_patterns(E* v, size_t len) {
    if (len < 8) return;
    uint64_t seed = (uint64_t)len;
    auto gen = [&]() { uint64_t r = seed; r ^= r << 13; r ^= r >> 7; r ^= r << 17; seed = r; return r; };
    size_t modulus = 1;
    while (modulus < len) modulus <<= 1;           // next_power_of_two
    const size_t pos = len / 4 * 2;
    for (size_t i = 0; i < 3; ++i) {
        size_t other = (size_t)(gen() & (modulus - 1));
        if (other >= len) other -= len;
        std::swap(v[pos - 1 + i], v[other]);
    }
}
template <typename E, typename L>
static size_t choose_pivot_pdq(E* v, size_t len, L& lt, bool& likely_sorted) {
    size_t a = len / 4 * 1, b = len / 4 * 2, c = len / 4 * 3;
    size_t swaps = 0;
    if (len >= 8) {
        auto sort2 = [&](size_t& x, size_t& y) { if (lt(v[y], v[x])) { std::swap(x, y); ++swaps; } };
        auto sort3 = [&](size_t& x, size_t& y, size_t& z) { sort2(x, y); sort2(y, z); sort2(x, y); };
        if (len >= 50) {
            auto adj = [&](size_t& x) { size_t lo = x - 1, hi = x + 1; sort3(lo, x, hi); };
            adj(a); adj(b); adj(c);
        }
        sort3(a, b, c);
    }
    if (swaps < 12) { likely_sorted = swaps == 0; return b; }
    std::reverse(v, v + len);
    likely_sorted = true;
    return len - 1 - b;
}
template <typename E, typename L>
static bool partial_insertion_sort(E* v, size_t len, L& lt) {
    size_t i = 1;
    for (int step = 0; step < 5; ++step) {
        while (i < len && !lt(v[i], v[i - 1])) ++i;
        if (i == len) return true;
        if (len < 50) return false;
        std::swap(v[i - 1], v[i]);
        if (i >= 2) {
            insertion_sort_shift_left(v, i, i - 1, lt);   // the smaller element to the left
            insert_head(v + i, len - i, lt);             // the greater element to the right
        }
    }
    return false;
}
template <typename E, typename L>
static size_t partition_in_blocks(E* v, size_t n, const E& pivot, L& lt) {
    constexpr size_t BLOCK = 128;
    size_t l = 0, r = n;                           // element indices into v
    size_t block_l = BLOCK, block_r = BLOCK;
    uint8_t offs_l[BLOCK], offs_r[BLOCK];
    size_t sl = 0, el = 0, sr = 0, er = 0;         // start/end into offs_*
    for (;;) {
        const bool is_done = r - l <= 2 * BLOCK;
        if (is_done) {
            size_t rem = r - l;
            if (sl < el || sr < er) rem -= BLOCK;
            if (sl < el) block_r = rem;
            else if (sr < er) block_l = rem;
            else { block_l = rem / 2; block_r = rem - block_l; }
        }
        if (sl == el) {
            sl = el = 0;
            for (size_t i = 0; i < block_l; ++i) { offs_l[el] = (uint8_t)i; el += !lt(v[l + i], pivot) ? 1 : 0; }
        }
        if (sr == er) {
            sr = er = 0;
            for (size_t i = 0; i < block_r; ++i) { offs_r[er] = (uint8_t)i; er += lt(v[r - 1 - i], pivot) ? 1 : 0; }
        }
        const size_t count = std::min(el - sl, er - sr);
        if (count > 0) {                           // cyclic permutation
            auto L_ = [&]() -> E& { return v[l + offs_l[sl]]; };
            auto R_ = [&]() -> E& { return v[r - 1 - offs_r[sr]]; };
            E tmp = L_();
            L_() = R_();
            for (size_t c = 1; c < count; ++c) {
                ++sl; R_() = L_();
                ++sr; L_() = R_();
            }
            R_() = tmp;
            ++sl; ++sr;
        }
        if (sl == el) l += block_l;
        if (sr == er) r -= block_r;
        if (is_done) break;
    }
    if (sl < el) {
        while (sl < el) { --el; std::swap(v[l + offs_l[el]], v[r - 1]); --r; }
        return r;
    } else if (sr < er) {
        while (sr < er) { --er; std::swap(v[l], v[r - 1 - offs_r[er]]); ++l; }
        return l;
    }
    return l;
}
template <typename E, typename L>
static size_t partition_pdq(E* v, size_t len, size_t pivot, L& lt, bool& was_partitioned) {
    std::swap(v[0], v[pivot]);
    const E pv = v[0];
    E* w = v + 1;
    const size_t n = len - 1;
    size_t l = 0, r = n;
    while (l < r && lt(w[l], pv)) ++l;
    while (l < r && !lt(w[r - 1], pv)) --r;
    was_partitioned = l >= r;
    const size_t mid = l + partition_in_blocks(w + l, r - l, pv, lt);
    std::swap(v[0], v[mid]);
    return mid;
}
template <typename E, typename L>
static size_t partition_equal(E* v, size_t len, size_t pivot, L& lt) {
    std::swap(v[0], v[pivot]);
    const E pv = v[0];
    E* w = v + 1;
    const size_t n = len - 1;
    if (n == 0) return 0;
    size_t l = 0, r = n;
    for (;;) {
        while (l < r && !lt(pv, w[l])) ++l;
        while (l < r && lt(pv, w[r - 1])) --r;
        if (l >= r) break;
        --r;
        std::swap(w[l], w[r]);
        ++l;
    }
    return l + 1;
}
template <typename E, typename L>
static void pdq_recurse(E* v, size_t len, L& lt, const E* pred, uint32_t limit) {
    E pred_val{};
    bool has_pred = pred != nullptr;
    if (has_pred) pred_val = *pred;
    bool was_balanced = true, was_partitioned = true;
    for (;;) {
        if (len <= 20) { if (len >= 2) insertion_sort_shift_left(v, len, 1, lt); return; }
        if (limit == 0) { heapsort(v, len, lt); return; }
        if (!was_balanced) { break_patterns(v, len); limit -= 1; }
        bool likely_sorted = false;
        const size_t pivot = choose_pivot_pdq(v, len, lt, likely_sorted);
        if (was_balanced && was_partitioned && likely_sorted)
            if (partial_insertion_sort(v, len, lt)) return;
        if (has_pred && !lt(pred_val, v[pivot])) {
            const size_t mid = partition_equal(v, len, pivot, lt);
            v += mid; len -= mid;
            continue;
        }
        bool was_p = false;
        const size_t mid = partition_pdq(v, len, pivot, lt, was_p);
        was_balanced = std::min(mid, len - mid) >= len / 8;
        was_partitioned = was_p;
        const size_t nl = mid, nr = len - mid - 1;
        if (nl < nr) {
            pdq_recurse(v, nl, lt, has_pred ? &pred_val : nullptr, limit);
            pred_val = v[mid]; has_pred = true;
            v += mid + 1; len = nr;
        } else {
            const E pv = v[mid];
            pdq_recurse(v + mid + 1, nr, lt, &pv, limit);
            len = nl;
        }
    }
}
template <typename E, typename L>
static void pdqsort(E* v, size_t len, L lt) {
    uint32_t limit = 0;
    for (size_t x = len; x; x >>= 1) ++limit;      // usize::BITS - leading_zeros
    pdq_recurse(v, len, lt, (const E*)nullptr, limit);
}
}  // namespace rsort

// Tie order of sort_unstable_by_key (orc_set_tie_order): 3 = ipnsort (rustc
// 1.81+, the default, matching the rustc >= 1.82 assumed for binary_search),
// 4 = pdqsort (rustc 1.78-1.80; Cargo.lock v4 needs >= 1.78); 0 = std::sort,
// 1 / 2 = stable with equal keys in ascending / descending input order (the
// two extremes, for measuring which outputs depend on the order).
static int g_tie_order = 3;
template <typename T>
static void sort_unstable_by_first(std::vector<std::pair<int32_t, T>>& v) {
    auto lt = [](const std::pair<int32_t, T>& a, const std::pair<int32_t, T>& b) { return a.first < b.first; };
    if (g_tie_order == 3) { rsort::ipnsort(v.data(), v.size(), lt); return; }
    if (g_tie_order == 4) { rsort::pdqsort(v.data(), v.size(), lt); return; }
    if (g_tie_order == 0) { std::sort(v.begin(), v.end(), lt); return; }
    if (g_tie_order == 2) std::reverse(v.begin(), v.end());
    std::stable_sort(v.begin(), v.end(), lt);
}

// lchain.rs:59-176
static DpResult chain_dp_all(const std::vector<Anchor>& anchors, const ChainParams& p, ChainStats* stats) {
    DpResult R;
    size_t n = anchors.size();
    if (n == 0) return R;
    int32_t max_dist_x = p.max_dist_x, max_dist_y = p.max_dist_y;
    if (max_dist_x < p.bw) max_dist_x = p.bw;
    if (max_dist_y < p.bw) max_dist_y = p.bw;
    std::vector<int32_t> f(n, 0), v(n, 0), t(n, 0);
    std::vector<int64_t> pprev(n, -1);
    size_t st = 0;
    for (size_t i = 0; i < n; ++i) {
        while (st < i && (rid(anchors[st]) != rid(anchors[i]) || rev(anchors[st]) != rev(anchors[i]) || rpos(anchors[i]) > wadd(rpos(anchors[st]), max_dist_x))) st += 1;
        int64_t max_j = -1;
        int32_t max_f = qspan(anchors[i]);
        size_t start_j = ((int32_t)i - p.max_chain_iter > (int32_t)st) ? (size_t)((int32_t)i - p.max_chain_iter) : st;
        int32_t n_skip = 0;
        for (size_t jj = i; jj > start_j; --jj) {
            size_t j = jj - 1;
            if (stats) stats->inner_iters++;
            if (rid(anchors[j]) != rid(anchors[i]) || rev(anchors[j]) != rev(anchors[i])) continue;
            int32_t sc0;
            if (comput_sc(anchors[i], anchors[j], max_dist_x, max_dist_y, p.bw, p.chn_pen_gap, p.chn_pen_skip, sc0)) {
                int32_t sc = wadd(sc0, f[j]);
                if (sc > max_f) { max_f = sc; max_j = (int64_t)j; if (n_skip > 0) n_skip -= 1; }
                else if (t[j] == (int32_t)i) { n_skip += 1; if (n_skip > p.max_chain_skip) break; }
                if (pprev[j] >= 0) t[(size_t)pprev[j]] = (int32_t)i;
            }
        }
        f[i] = max_f; pprev[i] = max_j;
        v[i] = (max_j >= 0 && v[(size_t)max_j] > max_f) ? v[(size_t)max_j] : max_f;
    }
    R.f = f; R.pprev = pprev;
    // backtrack like minimap2 (lchain.rs:92-160)
    std::vector<std::pair<int32_t, size_t>> z;
    for (size_t i = 0; i < n; ++i) if (f[i] > 0) z.push_back({f[i], i});
    if (z.empty()) return R;
    // sort_unstable_by_key: tie order unspecified (g_tie_order); observable only when a backtrack chain passes
    // min_chain_score, i.e. min_cnt <= 1 and min_chain_score <= span (DESIGN.md "-n <= 1")
    sort_unstable_by_first(z);
    std::fill(t.begin(), t.end(), 0);
    size_t n_v = 0, n_u = 0;
    for (size_t kk = z.size(); kk-- > 0;) {   // first pass
        size_t i0 = z[kk].second;
        if (t[i0] != 0) continue;
        int64_t i = (int64_t)i0, end_i = -1;
        int32_t max_s = 0; int64_t max_i = i;
        if (i >= 0 && t[(size_t)i] == 0) {
            for (;;) {
                t[(size_t)i] = 2;
                end_i = pprev[(size_t)i];
                int32_t s = end_i < 0 ? z[kk].first : wsub(z[kk].first, f[(size_t)end_i]);
                if (s > max_s) { max_s = s; max_i = end_i; } else if (wsub(max_s, s) > p.max_drop) break;
                if (!(i >= 0 && t[(size_t)i] == 0 && end_i >= 0)) break;
                i = end_i;
            }
            int64_t ii = (int64_t)i0;
            while (ii >= 0 && ii != end_i) { t[(size_t)ii] = 0; ii = pprev[(size_t)ii]; }
        }
        size_t len0 = n_v;
        int64_t i2 = (int64_t)i0; int64_t end2 = max_i;
        while (i2 >= 0 && i2 != end2) { n_v += 1; t[(size_t)i2] = 1; i2 = pprev[(size_t)i2]; }
        int32_t sc = i2 < 0 ? z[kk].first : wsub(z[kk].first, f[(size_t)i2]);
        if (sc >= p.min_chain_score && n_v > len0 && (int32_t)(n_v - len0) >= p.min_cnt) n_u += 1; else n_v = len0;
    }
    (void)n_u;
    std::fill(t.begin(), t.end(), 0);
    for (size_t kk = z.size(); kk-- > 0;) {   // second pass
        size_t i0 = z[kk].second;
        if (t[i0] != 0) continue;
        int64_t i = (int64_t)i0, end_i = -1;
        int32_t max_s = 0; int64_t max_i = i;
        if (i >= 0 && t[(size_t)i] == 0) {
            for (;;) {
                t[(size_t)i] = 2;
                end_i = pprev[(size_t)i];
                int32_t s = end_i < 0 ? z[kk].first : wsub(z[kk].first, f[(size_t)end_i]);
                if (s > max_s) { max_s = s; max_i = end_i; } else if (wsub(max_s, s) > p.max_drop) break;
                if (!(i >= 0 && t[(size_t)i] == 0 && end_i >= 0)) break;
                i = end_i;
            }
            int64_t ii = (int64_t)i0;
            while (ii >= 0 && ii != end_i) { t[(size_t)ii] = 0; ii = pprev[(size_t)ii]; }
        }
        std::vector<size_t> v_idxs;
        int64_t i2 = (int64_t)i0; int64_t end2 = max_i;
        while (i2 >= 0 && i2 != end2) { v_idxs.push_back((size_t)i2); t[(size_t)i2] = 1; i2 = pprev[(size_t)i2]; }
        int32_t sc = i2 < 0 ? z[kk].first : wsub(z[kk].first, f[(size_t)i2]);
        if (sc >= p.min_chain_score && (int32_t)v_idxs.size() >= p.min_cnt) {
            std::reverse(v_idxs.begin(), v_idxs.end());
            R.scores.push_back(sc); R.chains.push_back(std::move(v_idxs));
        }
    }
    // Fallback (lchain.rs:162-173): best_i = LAST index with maximal f (Iterator::max_by_key)
    if (R.chains.empty()) {
        size_t best_i = 0; int32_t best = f[0];
        for (size_t i = 1; i < n; ++i) if (f[i] >= best) { best = f[i]; best_i = i; }
        std::vector<size_t> v_idxs;
        int64_t i = (int64_t)best_i;
        while (i >= 0) { v_idxs.push_back((size_t)i); i = pprev[(size_t)i]; }
        std::reverse(v_idxs.begin(), v_idxs.end());
        if (!v_idxs.empty()) { R.chains.push_back(std::move(v_idxs)); R.scores.push_back(v[best_i]); }
    }
    sort_chains_stable(anchors, R.chains, R.scores);
    return R;
}

static inline void chain_qrange(const std::vector<Anchor>& anchors, const std::vector<size_t>& chain, int32_t& qs, int32_t& qe) {   // lchain.rs:178-188
    qs = INT32_MAX; qe = -1;
    for (size_t i : chain) {
        const Anchor& a = anchors[i];
        int32_t s = wsub(qpos(a), qspan(a) - 1), e = wadd(qpos(a), 1);
        if (s < qs) qs = s;
        if (e > qe) qe = e;
    }
    qs = std::max(qs, 0);
}
static inline void chain_trange(const std::vector<Anchor>& anchors, const std::vector<size_t>& chain, int32_t& ts, int32_t& te) {   // lchain.rs:190-200
    ts = INT32_MAX; te = -1;
    for (size_t i : chain) {
        const Anchor& a = anchors[i];
        int32_t s = wsub(rpos(a), qspan(a) - 1), e = wadd(rpos(a), 1);
        if (s < ts) ts = s;
        if (e > te) te = e;
    }
    ts = std::max(ts, 0);
}

static void sort_chains_stable(const std::vector<Anchor>& anchors, std::vector<std::vector<size_t>>& chains, std::vector<int32_t>& scores) {   // lchain.rs:202-218
    std::vector<size_t> idxs(chains.size());
    for (size_t i = 0; i < idxs.size(); ++i) idxs[i] = i;
    std::stable_sort(idxs.begin(), idxs.end(), [&](size_t i, size_t j) {
        int32_t si = scores[i], sj = scores[j];
        if (si != sj) return si > sj;
        int32_t qi, qj, dummy;
        chain_qrange(anchors, chains[i], qi, dummy); chain_qrange(anchors, chains[j], qj, dummy);
        if (qi != qj) return qi < qj;
        int32_t ti, tj;
        chain_trange(anchors, chains[i], ti, dummy); chain_trange(anchors, chains[j], tj, dummy);
        return ti < tj;
    });
    std::vector<std::vector<size_t>> c2; std::vector<int32_t> s2;
    for (size_t i : idxs) { c2.push_back(chains[i]); s2.push_back(scores[i]); }
    chains.swap(c2); scores.swap(s2);
}

static std::vector<bool> select_primary_secondary(const std::vector<Anchor>& anchors, const std::vector<std::vector<size_t>>& chains, const std::vector<int32_t>& scores, float mask_level) {   // lchain.rs:220-235
    std::vector<std::pair<int32_t, std::pair<int32_t, int32_t>>> primaries;
    std::vector<bool> is_primary(chains.size(), true);
    for (size_t ci = 0; ci < chains.size(); ++ci) {
        int32_t qs, qe; chain_qrange(anchors, chains[ci], qs, qe);
        bool overlapped = false;
        for (auto& pr : primaries) {
            int32_t pqs = pr.second.first, pqe = pr.second.second;
            float ov = (float)std::max(wsub(std::min(qe, pqe), std::max(qs, pqs)), 0);
            float len = (float)std::max(wsub(qe, qs), 1);
            if (ov / len >= mask_level) { overlapped = true; break; }
        }
        if (overlapped) is_primary[ci] = false; else primaries.push_back({scores[ci], {qs, qe}});
    }
    return is_primary;
}

static void select_and_filter_chains(const std::vector<Anchor>& anchors, const std::vector<std::vector<size_t>>& chains_in, const std::vector<int32_t>& scores_in,
                                     float mask_level, float pri_ratio, size_t best_n,
                                     std::vector<std::vector<size_t>>& out_chains, int32_t& s1, int32_t& s2) {   // lchain.rs:237-260
    out_chains.clear(); s1 = 0; s2 = 0;
    if (chains_in.empty()) return;
    std::vector<std::vector<size_t>> chains = chains_in; std::vector<int32_t> scores = scores_in;
    sort_chains_stable(anchors, chains, scores);
    std::vector<bool> is_primary = select_primary_secondary(anchors, chains, scores, mask_level);
    s1 = scores[0];
    size_t sec_kept = 0;
    for (size_t i = 0; i < chains.size(); ++i) {
        if (i == 0) { out_chains.push_back(chains[i]); }
        else {
            if (!is_primary[i]) continue;
            if ((float)scores[i] >= pri_ratio * (float)s1) { if (sec_kept < best_n) { out_chains.push_back(chains[i]); sec_kept += 1; } }
            if (s2 == 0) s2 = scores[i];
        }
    }
}

static std::vector<std::vector<size_t>> merge_adjacent_chains_with_gap(const std::vector<Anchor>& anchors, const std::vector<std::vector<size_t>>& chains, int32_t max_gap_q, int32_t max_gap_t) {   // lchain.rs:288-314
    std::vector<std::pair<int32_t, size_t>> items;
    for (size_t i = 0; i < chains.size(); ++i) { int32_t qs, qe; chain_qrange(anchors, chains[i], qs, qe); items.push_back({qs, i}); }
    sort_unstable_by_first(items);   // ties: see g_tie_order
    std::vector<std::vector<size_t>> merged;
    for (auto& it : items) {
        const auto& ch = chains[it.second];
        if (merged.empty()) { merged.push_back(ch); continue; }
        auto& last = merged.back();
        const Anchor& a_last = anchors[last.back()];
        const Anchor& a_first = anchors[ch.front()];
        bool same = rid(a_last) == rid(a_first) && rev(a_last) == rev(a_first);
        int32_t lqs, lqe, cqs, cqe, lts, lte, cts, cte;
        chain_qrange(anchors, last, lqs, lqe); chain_qrange(anchors, ch, cqs, cqe);
        chain_trange(anchors, last, lts, lte); chain_trange(anchors, ch, cts, cte);
        int32_t q_gap = wsub(cqs, lqe), t_gap = wsub(cts, lte);
        if (same && q_gap >= 0 && t_gap >= 0 && q_gap <= max_gap_q && t_gap <= max_gap_t) last.insert(last.end(), ch.begin(), ch.end());
        else merged.push_back(ch);
    }
    return merged;
}

static int32_t chain_query_coverage(const std::vector<Anchor>& anchors, const std::vector<size_t>& chain) {   // lchain.rs:316-319
    int32_t qs, qe; chain_qrange(anchors, chain, qs, qe);
    return std::max(wsub(qe, qs), 0);
}

// lchain.rs:321-330.  rescued flag reported for byte accounting.
static DpResult rescue_long_join(const std::vector<Anchor>& anchors, const DpResult& in, const ChainParams& p, int32_t qlen, bool* rescued, ChainStats* stats) {
    if (rescued) *rescued = false;
    if (in.chains.empty()) return in;
    int32_t best_cov = chain_query_coverage(anchors, in.chains[0]);
    int32_t uncovered = std::max(wsub(qlen, best_cov), 0);
    bool rescue = uncovered > p.rmq_rescue_size || (float)best_cov < (float)qlen * (1.0f - p.rmq_rescue_ratio);
    if (!rescue) return in;
    if (rescued) *rescued = true;
    ChainParams p2 = p; p2.bw = p.bw_long;
    return chain_dp_all(anchors, p2, stats);
}

// --------------------------------------------------------------- paf.rs
struct PafRecord {
    std::string qname; u32 qlen, qstart, qend; char strand; std::string tname; u32 tlen, tstart, tend, nm, blen; uint8_t mapq;
    char tp; u32 cm, s1, s2; float dv; u32 rl;
    bool panic = false;   // the reference would panic here (idx.seq[rid0] out of bounds)
};

// paf.rs:178 `mini_pos.binary_search(&first)`.  Cargo.lock version 4 bounds
// the reference's rustc only from below (>= 1.78), and std changed the
// algorithm in 1.82.  mini_pos is strictly increasing for odd k (no symmetric
// k-mers: every position is emitted once, in order), where both versions give
// the same answer; with even k a symmetric k-mer keeps l at w+k-1 for several
// steps, the first-window tie emission (sketch.rs:79-82) repeats, and mini_pos
// can hold duplicates and go backwards.  There the two versions
// can disagree; the device (k_dv) follows >= 1.82, the oracle either one.
static int g_binsearch_pre182 = 0;   // orc_set_binary_search(1): the 1.52-1.81 algorithm

// Rust >= 1.82 slice::binary_search_by (base/size halving, no early exit)
static bool rust_binary_search_182(const std::vector<int32_t>& v, int32_t target, size_t& idx) {
    size_t size = v.size();
    if (size == 0) { idx = 0; return false; }
    size_t base = 0;
    while (size > 1) {
        size_t half = size / 2, mid = base + half;
        if (!(v[mid] > target)) base = mid;   // cmp == Greater ? base : mid
        size -= half;
    }
    if (v[base] == target) { idx = base; return true; }
    idx = base + (v[base] < target ? 1 : 0);
    return false;
}

// Rust 1.52-1.81 slice::binary_search_by: midpoint of [left, right), early
// return on Equal
static bool rust_binary_search_pre182(const std::vector<int32_t>& v, int32_t target, size_t& idx) {
    size_t size = v.size(), left = 0, right = size;
    while (left < right) {
        const size_t mid = left + size / 2;
        const int32_t y = v[mid];
        if (y < target) left = mid + 1;        // cmp == Less
        else if (y > target) right = mid;      // cmp == Greater
        else { idx = mid; return true; }
        size = right - left;
    }
    idx = left;
    return false;
}

static bool rust_binary_search(const std::vector<int32_t>& v, int32_t target, size_t& idx) {
    return g_binsearch_pre182 ? rust_binary_search_pre182(v, target, idx) : rust_binary_search_182(v, target, idx);
}

// paf.rs:130-222
static bool paf_from_chain_with_primary(const Index& idx, const std::vector<Anchor>& anchors, const std::vector<size_t>& chain,
                                        const std::string& qname, const uint8_t* qseq, size_t qlen_sz, bool is_primary, PafRecord& rec) {
    if (chain.empty()) return false;
    char strand = rev(anchors[chain[0]]) ? '-' : '+';
    int32_t qs = INT32_MAX, qe = -1, ts = INT32_MAX, te = -1;
    u32 cm = 0;
    for (size_t i : chain) {
        const Anchor& a = anchors[i];
        cm += 1;
        int32_t s = wsub(qpos(a), qspan(a) - 1), e = wadd(qpos(a), 1);
        if (s < qs) qs = s;
        if (e > qe) qe = e;
        int32_t rs = wsub(rpos(a), qspan(a) - 1), re = wadd(rpos(a), 1);
        if (rs < ts) ts = rs;
        if (re > te) te = re;
    }
    if (qs < 0) qs = 0;
    if (ts < 0) ts = 0;
    size_t rid0 = (size_t)((anchors[chain[0]].x >> 32) & 0x7fffffff);
    if (rid0 >= idx.seq.size()) {   // Rust: index out of bounds -> panic (Q19)
        // the fields computed before the panic, for per-read comparisons (orc_align_records)
        rec.panic = true; rec.qlen = (u32)qlen_sz; rec.qstart = (u32)qs; rec.qend = (u32)qe; rec.strand = strand;
        rec.tstart = (u32)ts; rec.tend = (u32)te; rec.cm = cm;
        return false;
    }
    const IndexSeq& sq = idx.seq[rid0];
    std::string tname = sq.has_name ? sq.name : std::string("*");
    u32 tlen = sq.len;
    int32_t qs2 = qs, qe2 = qe, ts2 = ts, te2 = te;
    u32 mlen = (u32)std::max(wsub(qe2, qs2), 0);
    u32 blen = (u32)std::max(wsub(te2, ts2), 0);
    std::vector<Minimizer> mv = collect_query_minimizers(qseq, qlen_sz, (size_t)idx.w, (size_t)idx.k);
    std::vector<int32_t> mini_pos; mini_pos.reserve(mv.size());
    u64 sum_k = 0;
    for (const auto& m : mv) { mini_pos.push_back((int32_t)((m.rid_pos_strand >> 1) & 0xffffffffULL)); sum_k += (m.key_span & 0xff); }
    float avg_k = !mv.empty() ? (float)sum_k / (float)mv.size() : (float)idx.k;
    int32_t qlen = (int32_t)qlen_sz;
    auto qpos_fwd = [&](const Anchor& a) -> int32_t {
        int32_t qp = qpos(a), qsp = qspan(a);
        return rev(a) ? wsub(wsub(qlen, 1), wsub(wadd(qp, 1), qsp)) : qp;
    };
    std::vector<int32_t> chain_qs_fwd; chain_qs_fwd.reserve(chain.size());
    if (strand == '-') { for (size_t t = chain.size(); t-- > 0;) chain_qs_fwd.push_back(qpos_fwd(anchors[chain[t]])); }
    else { for (size_t i : chain) chain_qs_fwd.push_back(qpos_fwd(anchors[i])); }
    float dv = 0.0f;
    if (!mini_pos.empty() && !chain_qs_fwd.empty()) {
        int32_t first = chain_qs_fwd[0];
        size_t st;
        if (rust_binary_search(mini_pos, first, st)) {
            while (st > 0 && mini_pos[st - 1] == first) st -= 1;
            size_t j = st, k = 1, en = st;
            int32_t n_match = 1;
            while (j + 1 < mini_pos.size() && k < chain_qs_fwd.size()) {
                j += 1;
                if (mini_pos[j] == chain_qs_fwd[k]) { n_match += 1; en = j; k += 1; }
            }
            int32_t n_tot = (int32_t)((en - st) + 1);
            int32_t r_qs_final = strand == '-' ? wsub(qlen, qe2) : qs2;
            int32_t r_qe_final = strand == '-' ? wsub(qlen, qs2) : qe2;
            int32_t r_rs = ts2, r_re = te2;
            int32_t ak = sat_f32_to_i32(avg_k);
            if (r_qs_final > ak && r_rs > ak) n_tot += 1;
            if (wsub(qlen, r_qe_final) > ak && wsub((int32_t)tlen, r_re) > ak) n_tot += 1;
            float frac = (float)n_match / (float)n_tot;
            if (frac >= 1.0f) dv = 0.0f;
            else dv = 1.0f - powf(frac, 1.0f / fmaxf(avg_k, 1.0f));
        }
    }
    rec.qname = qname; rec.qlen = (u32)qlen_sz; rec.qstart = (u32)qs2; rec.qend = (u32)qe2; rec.strand = strand;
    rec.tname = tname; rec.tlen = tlen; rec.tstart = (u32)ts2; rec.tend = (u32)te2; rec.nm = mlen; rec.blen = blen;
    rec.mapq = 60; rec.tp = is_primary ? 'P' : 'S'; rec.cm = cm; rec.s1 = 0; rec.s2 = 0; rec.dv = dv; rec.rl = 0;
    return true;
}

static std::string write_paf(const PafRecord& r) {   // paf.rs:224-236
    u32 qs = r.qstart, qe = r.qend;
    if (r.strand == '-') { qs = r.qlen - r.qend; qe = r.qlen - r.qstart; }
    char buf[512];
    snprintf(buf, sizeof buf, "\t%u\t%u\t%u\t%c\t", r.qlen, qs, qe, r.strand);
    std::string s = r.qname + buf + r.tname;
    snprintf(buf, sizeof buf, "\t%u\t%u\t%u\t%u\t%u\t%u\ttp:A:%c\tcm:i:%u\ts1:i:%u\ts2:i:%u\tdv:f:%.4f\trl:i:%u",
             r.tlen, r.tstart, r.tend, r.nm, r.blen, (unsigned)r.mapq, r.tp, r.cm, r.s1, r.s2, (double)r.dv, r.rl);
    return s + buf;
}

// main.rs:105-123
static ChainParams default_chain_params(int32_t k) {
    float chain_gap_scale = 0.8f;
    float chn_pen_gap = 0.01f * chain_gap_scale * (float)k;
    return ChainParams{5000, 5000, 500, 5000, 40, 3, chn_pen_gap, 0.0f, 25, 500, 20000, 1000, 0.1f};
}

// Per-read accounting the bench uses for algorithmic bytes
static bool g_quiet = false;   // orc_set_quiet: silence per-read panic notes (bench)
struct ReadCounts { u64 m_all = 0, m_kept = 0, anchors = 0, rescued = 0, inner_iters = 0, lines = 0, panics = 0; };
// One read's outcome for per-read comparisons (orc_align_records), also for
// reads on which the reference panics (Q19): the first chain's PAF columns as
// paf_from_chain_with_primary computes them before the out-of-bounds index.
struct ReadRec {
    int32_t flags = 0;       // 1 a chain (a PAF line or a panic), 2 rescued, 8 panic
    int32_t n_anchors = 0, score = 0, cm = 0, qs = 0, qe = 0, ts = 0, te = 0, rid = 0, rev = 0;
    float dv = 0.0f;
    int32_t m_kept = 0;
};

struct AlignOpts {
    int32_t w = 10, k = 15; float frac = 2e-4f; int32_t max_gap = 5000; int32_t bw = -1, bw_long = -1;
    int32_t min_cnt = 3, min_chain_score = 40; float mask_level = 0.5f, pri_ratio = 0.8f; size_t best_n = 5;
};

// main.rs:189-230 Align flow for ONE read (the reference maps only the first
// record; we apply it to every record and concatenate — SURVEY §0.3)
static void align_one(const Index& idx, int32_t mid_occ, const AlignOpts& o, const std::string& qname, const uint8_t* q, size_t qlen,
                      std::vector<std::string>& lines, ReadCounts* rc, ReadRec* rr = nullptr) {
    std::vector<Minimizer> mv = collect_query_minimizers(q, qlen, (size_t)o.w, (size_t)o.k);
    if (rc) rc->m_all += mv.size();
    filter_query_minimizers(mv, 10, 0.01f);
    if (rc) rc->m_kept += mv.size();
    std::vector<Anchor> anchors = build_anchors_filtered(idx, mv, (int32_t)qlen, mid_occ);
    if (rc) rc->anchors += anchors.size();
    if (rr) { rr->n_anchors = (int32_t)anchors.size(); rr->m_kept = (int32_t)mv.size(); }
    ChainParams p = default_chain_params(o.k);
    p.max_dist_x = o.max_gap; p.max_dist_y = o.max_gap;
    p.min_cnt = o.min_cnt; p.min_chain_score = o.min_chain_score;
    if (o.bw >= 0) p.bw = o.bw;
    if (o.bw_long >= 0) p.bw_long = o.bw_long;
    ChainStats cs;
    DpResult all = chain_dp_all(anchors, p, rc ? &cs : nullptr);
    if (all.chains.empty()) {
        // chain_dp -> empty for zero anchors -> paf_from_chain None -> no line
        if (rc) rc->inner_iters += cs.inner_iters;
        return;
    }
    bool rescued = false;
    DpResult resc = rescue_long_join(anchors, all, p, (int32_t)qlen, &rescued, rc ? &cs : nullptr);
    if (rr && rescued) rr->flags |= 2;
    if (rc) { rc->rescued += rescued ? anchors.size() : 0; rc->inner_iters += cs.inner_iters; }
    // merge_adjacent_chains_with_gap unwraps last()/first() of the chains it meets after the first
    // (lchain.rs:297-298): an empty chain (only min_cnt <= 0 lets one through) among two or more panics
    if (resc.chains.size() >= 2) {
        for (const auto& ch : resc.chains)
            if (ch.empty()) {
                if (!g_quiet) fprintf(stderr, "oracle: read %s: reference panics (unwrap on an empty chain)\n", qname.c_str());
                if (rc) rc->panics += 1;
                if (rr) rr->flags |= 8;
                return;
            }
    }
    std::vector<std::vector<size_t>> merged = merge_adjacent_chains_with_gap(anchors, resc.chains, p.max_dist_y, p.max_dist_y);
    std::vector<std::vector<size_t>> chains; int32_t s1, s2;
    const size_t lines0 = lines.size();
    select_and_filter_chains(anchors, merged, resc.scores, o.mask_level, o.pri_ratio, o.best_n, chains, s1, s2);
    for (size_t ci = 0; ci < chains.size(); ++ci) {   // paf.rs:238-248
        PafRecord rec;
        const bool ok = paf_from_chain_with_primary(idx, anchors, chains[ci], qname, q, qlen, ci == 0, rec);
        if (rr && ci == 0 && (ok || rec.panic)) {
            rr->flags |= 1 | (rec.panic ? 8 : 0);
            rr->score = s1; rr->cm = (int32_t)rec.cm; rr->qs = (int32_t)rec.qstart; rr->qe = (int32_t)rec.qend;
            rr->ts = (int32_t)rec.tstart; rr->te = (int32_t)rec.tend;
            rr->rid = (int32_t)((anchors[chains[ci][0]].x >> 32) & 0x7fffffff); rr->rev = rec.strand == '-';
            rr->dv = ok ? rec.dv : 0.0f;
        }
        if (ok) {
            rec.s1 = (u32)std::max(s1, 0); rec.s2 = (u32)std::max(s2, 0);
            lines.push_back(write_paf(rec));
            if (rc) rc->lines += 1;
        } else if (rec.panic) {
            // The reference aborts the whole process here, before it prints any
            // of the read's lines (main.rs:218-226); per-read concatenation
            // semantics: this read yields no line (and is counted).
            if (!g_quiet) fprintf(stderr, "oracle: read %s: reference panics (index out of bounds: rid 2147483647)\n", qname.c_str());
            if (rc) { rc->panics += 1; rc->lines -= (u64)(lines.size() - lines0); }
            if (rr) rr->flags |= 8;
            lines.resize(lines0);
            break;
        }
    }
}

}  // namespace orc

// ============================================================================
// C ABI for tests/bench (ctypes).  All functions prefixed orc_.
// ============================================================================
using namespace orc;
extern "C" {

// Sketch one sequence. Returns number of minimizers (or -1 on assertion failure);
// writes min(n, cap) pairs (key_span, rid_pos_strand) into out[2*i], out[2*i+1].
long long orc_sketch(const uint8_t* seq, long long len, int w, int k, unsigned rid, int is_hpc, uint64_t* out, long long cap) {
    std::vector<Minimizer> v;
    if (!sketch_sequence(seq, (size_t)len, (size_t)w, (size_t)k, rid, is_hpc != 0, v)) return -1;
    for (size_t i = 0; i < v.size() && (long long)i < cap; ++i) { out[2 * i] = v[i].key_span; out[2 * i + 1] = v[i].rid_pos_strand; }
    return (long long)v.size();
}

// Filter (seeds.rs:13-36) in place on an array of n minimizer pairs; returns new n.
long long orc_filter(uint64_t* mv, long long n, int q_occ_max, float q_occ_frac) {
    std::vector<Minimizer> v((size_t)n);
    for (long long i = 0; i < n; ++i) v[(size_t)i] = Minimizer{mv[2 * i], mv[2 * i + 1]};
    filter_query_minimizers(v, q_occ_max, q_occ_frac);
    for (size_t i = 0; i < v.size(); ++i) { mv[2 * i] = v[i].key_span; mv[2 * i + 1] = v[i].rid_pos_strand; }
    return (long long)v.size();
}

void* orc_index_build(const char* fasta, int w, int k, int b, int flag, int nthreads) {
    std::vector<FastaRec> recs;
    if (!read_fasta(fasta, recs, false)) return nullptr;
    return build_index_from_recs(recs, w, k, b, flag, nthreads);
}
void* orc_index_load_mmi(const char* path) { return load_from_mmi(path); }
int orc_index_save_mmi(void* idx, const char* path) { return save_to_mmi(*(Index*)idx, path) ? 0 : -1; }
void orc_index_free(void* idx) { delete (Index*)idx; }
int orc_index_calc_mid_occ(void* idx, float frac) { return ((Index*)idx)->calc_mid_occ(frac); }
void orc_index_params(void* idx, int* out5) { Index* I = (Index*)idx; out5[0] = I->w; out5[1] = I->k; out5[2] = I->b; out5[3] = I->flag; out5[4] = (int)I->n_seq; }
void orc_index_stats(void* idx, uint64_t* n_keys, double* avg_occ, double* avg_spacing, uint64_t* total_len) { ((Index*)idx)->stats(*n_keys, *avg_occ, *avg_spacing, *total_len); }
// Index::get: returns kind (0 none, 1 single, 2 multi) and copies up to cap positions.
long long orc_index_get(void* idx, uint64_t minier, int* kind, uint64_t* out, long long cap) {
    u64 single; const u64* slice = nullptr; size_t n = 0;
    int kd = ((Index*)idx)->get(minier, single, slice, n);
    *kind = kd;
    if (kd == 1) { if (cap > 0) out[0] = single; return 1; }
    if (kd == 2) { for (size_t i = 0; i < n && (long long)i < cap; ++i) out[i] = slice[i]; return (long long)n; }
    return 0;
}
// Dump all (minier, positions) key entries of the index: for each distinct key
// emits minier and count, positions in a flat array. Returns #keys. Call with
// null outputs first to size (returns #keys and sets *n_pos).
long long orc_index_dump(void* idx, uint64_t* keys, uint32_t* counts, uint64_t* pos, long long* n_pos) {
    Index* I = (Index*)idx;
    long long nk = 0, np = 0;
    std::vector<std::pair<u64, std::pair<u64, int>>> all;
    for (size_t bi = 0; bi < I->B.size(); ++bi) {
        const Bucket& bk = I->B[bi];
        if (!bk.has_h) continue;
        for (const auto& kv : bk.h) {
            u64 minier = ((kv.first >> 1) << I->b) | (u64)bi;
            all.push_back({minier, {kv.second, (int)(kv.first & 1)}});
        }
    }
    std::sort(all.begin(), all.end(), [](const std::pair<u64, std::pair<u64, int>>& a, const std::pair<u64, std::pair<u64, int>>& b) { return a.first < b.first; });
    for (auto& e : all) {
        u64 minier = e.first;
        const Bucket& bk = I->B[(size_t)(minier & ((1ULL << I->b) - 1))];
        if (e.second.second == 1) {
            if (keys) { keys[nk] = minier; counts[nk] = 1; pos[np] = e.second.first; }
            np += 1;
        } else {
            size_t off = (size_t)(e.second.first >> 32), n = (size_t)(e.second.first & 0xffffffffULL);
            if (keys) { keys[nk] = minier; counts[nk] = (uint32_t)n; for (size_t t = 0; t < n; ++t) pos[np + t] = bk.p[off + t]; }
            np += (long long)n;
        }
        nk += 1;
    }
    if (n_pos) *n_pos = np;
    return nk;
}

// Query path up to anchors: sketch(w,k) -> filter(10,0.01) -> build_anchors_filtered.
// Returns #anchors (writes up to cap pairs x,y); n_mini_out[0]=m, [1]=m'.
long long orc_anchors(void* idx, const uint8_t* q, long long qlen, int w, int k, int mid_occ, uint64_t* out, long long cap, long long* n_mini_out) {
    std::vector<Minimizer> mv = collect_query_minimizers(q, (size_t)qlen, (size_t)w, (size_t)k);
    if (n_mini_out) n_mini_out[0] = (long long)mv.size();
    filter_query_minimizers(mv, 10, 0.01f);
    if (n_mini_out) n_mini_out[1] = (long long)mv.size();
    std::vector<Anchor> a = build_anchors_filtered(*(Index*)idx, mv, (int32_t)qlen, mid_occ);
    for (size_t i = 0; i < a.size() && (long long)i < cap; ++i) { out[2 * i] = a[i].x; out[2 * i + 1] = a[i].y; }
    return (long long)a.size();
}

// chain_dp_all DP arrays for a given anchor list (lchain.rs:59-91) plus the
// chosen chain. params: [max_dist_x, max_dist_y, bw, max_chain_iter, min_chain_score,
// min_cnt, max_chain_skip, max_drop, bw_long, rmq_rescue_size]; fparams: [gap, skip, ratio].
// Outputs f[n], pprev[n]; chain indices into chain_out (cap), returns chain length,
// score in *score (or -1 length for no chain).
long long orc_chain_dp(const uint64_t* anchors_xy, long long n, const int* params, const float* fparams,
                       int* f_out, long long* pprev_out, long long* chain_out, long long cap, int* score, unsigned long long* inner_iters) {
    std::vector<Anchor> a((size_t)n);
    for (long long i = 0; i < n; ++i) a[(size_t)i] = Anchor{anchors_xy[2 * i], anchors_xy[2 * i + 1]};
    ChainParams p{params[0], params[1], params[2], params[3], params[4], params[5], fparams[0], fparams[1], params[6], params[7], params[8], params[9], fparams[2]};
    ChainStats cs;
    DpResult R = chain_dp_all(a, p, &cs);
    if (inner_iters) *inner_iters = cs.inner_iters;
    for (size_t i = 0; i < R.f.size(); ++i) { if (f_out) f_out[i] = R.f[i]; if (pprev_out) pprev_out[i] = R.pprev[i]; }
    if (R.chains.empty()) return -1;
    if (score) *score = R.scores[0];
    for (size_t i = 0; i < R.chains[0].size() && (long long)i < cap; ++i) chain_out[i] = (long long)R.chains[0][i];
    return (long long)R.chains[0].size();
}

// Full align of a FASTA (all records, or first only) -> PAF text file.
// Returns #lines or -1. counts (if non-null, 7 u64): m_all, m_kept, anchors, rescued-anchors, inner_iters, lines, panics.
// opts_i: [w, k, max_gap, bw, bw_long, min_cnt, min_chain_score, best_n, first_only, max_reads]; opts_f: [frac, mask_level, pri_ratio]
// mid_occ < 0 -> computed as the reference does (calc_mid_occ(frac), >= 10).
// time_s (if non-null) receives wall seconds of the mapping loop only (index excluded).
long long orc_align_fasta(void* idx, const char* reads_fa, const char* out_path, const int* oi, const float* of, int mid_occ,
                          uint64_t* counts, double* time_s) {
    Index* I = (Index*)idx;
    AlignOpts o;
    o.w = oi[0]; o.k = oi[1]; o.max_gap = oi[2]; o.bw = oi[3]; o.bw_long = oi[4]; o.min_cnt = oi[5]; o.min_chain_score = oi[6]; o.best_n = (size_t)oi[7];
    bool first_only = oi[8] != 0; long long max_reads = oi[9];
    o.frac = of[0]; o.mask_level = of[1]; o.pri_ratio = of[2];
    std::vector<FastaRec> recs;
    if (!read_fasta(reads_fa, recs, first_only)) return -1;
    if (mid_occ < 0) { mid_occ = I->calc_mid_occ(o.frac); if (mid_occ < 10) mid_occ = 10; }
    ReadCounts rc;
    std::vector<std::string> lines;
    auto t0 = std::chrono::steady_clock::now();
    long long nr = 0;
    for (const auto& r : recs) {
        if (max_reads > 0 && nr >= max_reads) break;
        nr++;
        if (r.seq.empty()) continue;   // reference asserts (sketch.rs:30); skipped here
        align_one(*I, mid_occ, o, r.name, (const uint8_t*)r.seq.data(), r.seq.size(), lines, counts ? &rc : nullptr);
    }
    auto t1 = std::chrono::steady_clock::now();
    if (time_s) *time_s = std::chrono::duration<double>(t1 - t0).count();
    if (out_path) {
        FILE* f = (strcmp(out_path, "-") == 0) ? stdout : fopen(out_path, "w");
        if (!f) return -1;
        for (auto& l : lines) { fputs(l.c_str(), f); fputc('\n', f); }
        if (f != stdout) fclose(f);
    }
    if (counts) { counts[0] = rc.m_all; counts[1] = rc.m_kept; counts[2] = rc.anchors; counts[3] = rc.rescued; counts[4] = rc.inner_iters; counts[5] = rc.lines; counts[6] = rc.panics; }
    return (long long)lines.size();
}

void orc_set_quiet(int q) { g_quiet = q != 0; }
// paf.rs:178's binary_search as rustc 1.52-1.81 (1) or >= 1.82 (0, default) compiles it
void orc_set_binary_search(int pre182) { g_binsearch_pre182 = pre182 != 0; }
void orc_set_tie_order(int mode) { g_tie_order = mode; }
// Rust's sort_unstable_by_key on (keys[i], i) pairs under tie order `mode`; the indices in output order.
void orc_rust_sort(const int32_t* keys, uint64_t n, int mode, uint64_t* perm) {
    std::vector<std::pair<int32_t, size_t>> v(n);
    for (uint64_t i = 0; i < n; ++i) v[i] = {keys[i], (size_t)i};
    const int keep = g_tie_order;
    g_tie_order = mode;
    sort_unstable_by_first(v);
    g_tie_order = keep;
    for (uint64_t i = 0; i < n; ++i) perm[i] = v[i].second;
}
// the two algorithms on a caller array (tests): returns found, *idx = Ok / Err index
int orc_binary_search(const int32_t* v, uint64_t n, int32_t target, int pre182, uint64_t* idx) {
    std::vector<int32_t> a(v, v + n);
    size_t i = 0;
    const bool f = pre182 ? rust_binary_search_pre182(a, target, i) : rust_binary_search_182(a, target, i);
    *idx = i;
    return f ? 1 : 0;
}

// build_index_from_fasta (src/index.rs:427-475) on in-memory records
// (bench.py: avoids a multi-GB FASTA round trip for the hg38-shaped genome).
void* orc_index_build_seqs(int n, const char* const* names, const uint8_t* const* seqs, const uint64_t* lens, int w, int k, int b,
                           int flag, int nthreads) {
    std::vector<FastaRec> recs((size_t)n);
    for (int i = 0; i < n; ++i) {
        recs[i].name = names && names[i] ? names[i] : "";
        recs[i].seq.assign((const char*)seqs[i], (size_t)lens[i]);
    }
    return build_index_from_recs(recs, w, k, b, flag, nthreads);
}

// The Align flow (src/main.rs:189-230) over in-memory reads; the mapping loop
// alone is timed (index and mid_occ excluded).  nthreads > 1
// hands reads out dynamically (the reference align is single-threaded; this
// is the all-cores variant of the CPU baseline).  Lines go to out_path when
// given (in read order).
long long orc_align_seqs(void* idx, int n, const char* const* names, const uint8_t* const* seqs, const uint64_t* lens,
                         const char* out_path, const int* oi, const float* of, int mid_occ, int nthreads, uint64_t* counts,
                         double* time_s) {
    Index* I = (Index*)idx;
    AlignOpts o;
    o.w = oi[0]; o.k = oi[1]; o.max_gap = oi[2]; o.bw = oi[3]; o.bw_long = oi[4]; o.min_cnt = oi[5]; o.min_chain_score = oi[6]; o.best_n = (size_t)oi[7];
    o.frac = of[0]; o.mask_level = of[1]; o.pri_ratio = of[2];
    if (mid_occ < 0) { mid_occ = I->calc_mid_occ(o.frac); if (mid_occ < 10) mid_occ = 10; }
    if (nthreads < 1) nthreads = 1;
    std::vector<std::vector<std::string>> per(n > 0 ? (size_t)n : 0);
    std::vector<ReadCounts> rcs((size_t)nthreads);
    std::atomic<int> next{0};
    auto worker = [&](int t) {
        for (;;) {
            const int r = next.fetch_add(1);
            if (r >= n) break;
            if (lens[r] == 0) continue;   // reference asserts (sketch.rs:30)
            align_one(*I, mid_occ, o, names ? std::string(names[r]) : std::string("*"), seqs[r], (size_t)lens[r], per[r], &rcs[t]);
        }
    };
    auto t0 = std::chrono::steady_clock::now();
    if (nthreads == 1) worker(0);
    else {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
        for (auto& x : th) x.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    if (time_s) *time_s = std::chrono::duration<double>(t1 - t0).count();
    ReadCounts rc;
    long long nl = 0;
    for (auto& c : rcs) {
        rc.m_all += c.m_all; rc.m_kept += c.m_kept; rc.anchors += c.anchors; rc.rescued += c.rescued;
        rc.inner_iters += c.inner_iters; rc.lines += c.lines; rc.panics += c.panics;
    }
    FILE* f = nullptr;
    if (out_path) { f = (strcmp(out_path, "-") == 0) ? stdout : fopen(out_path, "w"); if (!f) return -1; }
    for (auto& v : per)
        for (auto& l : v) { ++nl; if (f) { fputs(l.c_str(), f); fputc('\n', f); } }
    if (f && f != stdout) fclose(f);
    if (counts) { counts[0] = rc.m_all; counts[1] = rc.m_kept; counts[2] = rc.anchors; counts[3] = rc.rescued; counts[4] = rc.inner_iters; counts[5] = rc.lines; counts[6] = rc.panics; }
    return nl;
}

// Per-read outcomes (ReadRec, 12 int32 each: flags, n_anchors, score, cm, qs,
// qe, ts, te, rid, rev, dv bits, m_kept) of the Align flow over in-memory reads.
long long orc_align_records(void* idx, int n, const uint8_t* const* seqs, const uint64_t* lens, const int* oi, const float* of,
                            int mid_occ, int nthreads, int32_t* rec) {
    Index* I = (Index*)idx;
    AlignOpts o;
    o.w = oi[0]; o.k = oi[1]; o.max_gap = oi[2]; o.bw = oi[3]; o.bw_long = oi[4]; o.min_cnt = oi[5]; o.min_chain_score = oi[6]; o.best_n = (size_t)oi[7];
    o.frac = of[0]; o.mask_level = of[1]; o.pri_ratio = of[2];
    if (mid_occ < 0) { mid_occ = I->calc_mid_occ(o.frac); if (mid_occ < 10) mid_occ = 10; }
    if (nthreads < 1) nthreads = 1;
    std::atomic<int> next{0};
    auto worker = [&]() {
        std::vector<std::string> lines;
        for (;;) {
            const int r = next.fetch_add(1);
            if (r >= n) break;
            ReadRec R;
            if (lens[r]) { lines.clear(); align_one(*I, mid_occ, o, std::string("q"), seqs[r], (size_t)lens[r], lines, nullptr, &R); }
            int32_t* d = rec + 12 * (size_t)r;
            d[0] = R.flags; d[1] = R.n_anchors; d[2] = R.score; d[3] = R.cm; d[4] = R.qs; d[5] = R.qe; d[6] = R.ts; d[7] = R.te;
            d[8] = R.rid; d[9] = R.rev; memcpy(&d[10], &R.dv, 4); d[11] = R.m_kept;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(worker);
    worker();
    for (auto& x : th) x.join();
    return n;
}

// Pen LUT value as the reference computes it inline (comput_sc), for LUT parity tests.
int orc_pen(int dd, int dg, int q_span, float chn_pen_gap) {
    float lin_pen = chn_pen_gap * (float)dd + 0.0f * (float)dg;
    float log_pen = dd >= 1 ? mg_log2(dd + 1) : 0.0f;
    (void)q_span;
    return sat_f32_to_i32(lin_pen + 0.5f * log_pen);
}
float orc_default_gap(int k) { return default_chain_params(k).chn_pen_gap; }

}  // extern "C"

// ============================================================================
// CLI: mm2rs-cpu index|align (main.rs:147-233), oracle build only.
// ============================================================================
#ifdef ORC_MAIN
static void usage() {
    fprintf(stderr, "usage: mm2rs-cpu index <ref.fa> [-w 10] [-k 15] [-b 14] [-H] [-d out.mmi] [-t threads]\n"
                    "       mm2rs-cpu align <ref.mmi|ref.fa> <reads.fa> [-w] [-k] [-H] [-f] [-g] [-r bw[,bw_long]] [-n] [-m] [-M] [-p] [-N] [-x preset] [-a] [-o out] [--first-only] [-t threads]\n");
}
int main(int argc, char** argv) {
    if (argc < 3) { usage(); return 2; }
    std::string cmd = argv[1];
    std::vector<std::string> pos;
    int w = 10, k = 15, b = 14, threads = 1; bool hpc = false; std::string dump, out, preset, r;
    AlignOpts o; bool first_only = false;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto nxt = [&]() -> std::string { if (i + 1 >= argc) { usage(); exit(2); } return argv[++i]; };
        if (a == "-w") w = atoi(nxt().c_str());
        else if (a == "-k") k = atoi(nxt().c_str());
        else if (a == "-b") b = atoi(nxt().c_str());
        else if (a == "-H" || a == "--hpc") hpc = true;
        else if (a == "-d" || a == "--dump") dump = nxt();
        else if (a == "-t") threads = atoi(nxt().c_str());
        else if (a == "-f") o.frac = (float)atof(nxt().c_str());
        else if (a == "-g") o.max_gap = atoi(nxt().c_str());
        else if (a == "-r") r = nxt();
        else if (a == "-n") o.min_cnt = atoi(nxt().c_str());
        else if (a == "-m") o.min_chain_score = atoi(nxt().c_str());
        else if (a == "-M" || a == "--mask-level") o.mask_level = (float)atof(nxt().c_str());
        else if (a == "-p" || a == "--pri-ratio") o.pri_ratio = (float)atof(nxt().c_str());
        else if (a == "-N" || a == "--best-n") o.best_n = (size_t)atol(nxt().c_str());
        else if (a == "-x") preset = nxt();
        else if (a == "-a") {}
        else if (a == "-o") out = nxt();
        else if (a == "--first-only") first_only = true;
        else pos.push_back(a);
    }
    if (cmd == "index") {
        if (pos.size() != 1) { usage(); return 2; }
        int flag = hpc ? 1 : 0;
        std::vector<FastaRec> recs;
        if (!read_fasta(pos[0].c_str(), recs, false)) { fprintf(stderr, "Error: cannot read %s\n", pos[0].c_str()); return 1; }
        Index* idx = build_index_from_recs(recs, w, k, b, flag, threads);
        u64 nk, tl; double ao, as;
        idx->stats(nk, ao, as, tl);
        printf("kmer size: %d; skip: %d; is_hpc: %d; #seq: %u\n", k, w, hpc ? 1 : 0, idx->n_seq);
        printf("distinct minimizers: %llu (avg occ %.2f) avg spacing %.3f total length %llu\n", (unsigned long long)nk, ao, as, (unsigned long long)tl);
        if (!dump.empty()) {
            if (dump.size() >= 4 && dump.compare(dump.size() - 4, 4, ".mmi") == 0) { if (!save_to_mmi(*idx, dump.c_str())) { fprintf(stderr, "Error: write failed\n"); return 1; } }
            else { fprintf(stderr, "Error: only .mmi dumps are supported by the oracle\n"); return 1; }
        }
        delete idx;
        return 0;
    }
    if (cmd == "align") {
        if (pos.size() != 2) { usage(); return 2; }
        if (preset == "map-ont") { k = 15; w = 10; } else if (preset == "map-hifi" || preset == "lr:hq") { k = 19; w = 10; } else if (preset == "sr") { k = 21; w = 11; }
        o.w = w; o.k = k;
        if (!r.empty()) {
            size_t c = r.find(',');
            std::string a0 = r.substr(0, c);
            char* e; long v = strtol(a0.c_str(), &e, 10); if (!a0.empty() && *e == 0) o.bw = (int32_t)v;
            if (c != std::string::npos) { std::string a1 = r.substr(c + 1); v = strtol(a1.c_str(), &e, 10); if (!a1.empty() && *e == 0) o.bw_long = (int32_t)v; }
        }
        Index* idx;
        const std::string& ref = pos[0];
        if (ref.size() >= 4 && ref.compare(ref.size() - 4, 4, ".mmi") == 0) idx = load_from_mmi(ref.c_str());
        else { std::vector<FastaRec> recs; if (!read_fasta(ref.c_str(), recs, false)) idx = nullptr; else idx = build_index_from_recs(recs, w, k, 14, hpc ? 1 : 0, threads); }
        if (!idx) { fprintf(stderr, "Error: cannot load index %s\n", ref.c_str()); return 1; }
        int oi[10] = {o.w, o.k, o.max_gap, o.bw, o.bw_long, o.min_cnt, o.min_chain_score, (int)o.best_n, first_only ? 1 : 0, 0};
        float of[3] = {o.frac, o.mask_level, o.pri_ratio};
        long long n = orc_align_fasta(idx, pos[1].c_str(), out.empty() ? "-" : out.c_str(), oi, of, -1, nullptr, nullptr);
        delete idx;
        return n < 0 ? 1 : 0;
    }
    usage();
    return 2;
}
#endif
