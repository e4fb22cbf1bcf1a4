// Host-side index for the MI355X path: FASTA input, reference sketching,
// bucket post-processing, Index::get/stats/calc_mid_occ and the minimap2 MMI
// v2 format (src/index.rs).  The device layout built from it lives in
// mm2g_host.hip.
#include "mm2g_index.h"

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <thread>
#include <atomic>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace mm2g {

// ------------------------------------------------------------------ FASTA
bool read_fasta(const char* path, std::vector<FastaRecord>& out, bool first_only, std::string& err) {
    FILE* fp = fopen(path, "rb");
    if (!fp) { err = std::string("cannot open ") + path; return false; }
    std::string data;
    {
        std::vector<char> buf(1 << 22);
        size_t n;
        while ((n = fread(buf.data(), 1, buf.size(), fp)) > 0) data.append(buf.data(), n);
    }
    fclose(fp);
    const size_t N = data.size();
    size_t pos = 0;
    bool in_rec = false;
    while (pos < N) {
        const char* nl = (const char*)memchr(data.data() + pos, '\n', N - pos);
        size_t e = nl ? (size_t)(nl - data.data()) : N;
        size_t le = e;
        if (le > pos && data[le - 1] == '\r') --le;
        if (le > pos && data[pos] == '>') {
            if (in_rec && first_only) break;
            size_t ne = pos + 1;
            while (ne < le && data[ne] != ' ' && data[ne] != '\t') ++ne;
            out.push_back(FastaRecord{data.substr(pos + 1, ne - pos - 1), std::string()});
            in_rec = true;
        } else if (in_rec && le > pos) {
            out.back().seq.append(data, pos, le - pos);
        }
        pos = e + 1;
    }
    return true;
}

SeqStream::~SeqStream() {
    if (fp_) fclose(fp_);
    free(buf_);
}
bool SeqStream::open(const char* path, std::string& err) {
    fp_ = fopen(path, "rb");
    if (!fp_) { err = std::string("cannot open ") + path; return false; }
    return true;
}
bool SeqStream::getline_(std::string& s) {
    if (has_pending_) { s.swap(pending_); has_pending_ = false; return true; }
    const ssize_t n = ::getline(&buf_, &cap_, fp_);
    if (n < 0) return false;
    size_t le = (size_t)n;
    if (le && buf_[le - 1] == '\n') --le;
    if (le && buf_[le - 1] == '\r') --le;
    s.assign(buf_, le);
    return true;
}
bool SeqStream::next(FastaRecord& rec) {
    std::string ln;
    for (;;) {   // header: text before the first record is ignored (read_fasta)
        if (!getline_(ln)) return false;
        if (!ln.empty() && (ln[0] == '>' || ln[0] == '@')) break;
    }
    const bool fastq = ln[0] == '@';
    size_t ne = 1;
    while (ne < ln.size() && ln[ne] != ' ' && ln[ne] != '\t') ++ne;
    rec.name = ln.substr(1, ne - 1);
    rec.seq.clear();
    while (getline_(ln)) {
        if (!ln.empty() && (fastq ? ln[0] == '+' : ln[0] == '>')) {
            if (!fastq) { pending_.swap(ln); has_pending_ = true; }
            break;
        }
        rec.seq += ln;
    }
    if (fastq) {   // quality: as many characters as the sequence
        size_t q = 0;
        while (q < rec.seq.size() && getline_(ln)) q += ln.size();
    }
    return true;
}

// ------------------------------------------------------------------ sketch
static inline uint32_t nt4h(uint8_t c) {
    static const uint8_t T[256] = {
        4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,
        4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,
        4,0,4,1,4,4,4,2,4,4,4,4,4,4,4,4, 4,4,4,4,3,4,4,4,4,4,4,4,4,4,4,4,
        4,0,4,1,4,4,4,2,4,4,4,4,4,4,4,4, 4,4,4,4,3,4,4,4,4,4,4,4,4,4,4,4,
        4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,
        4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,
        4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,
        4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4, 4,4,4,4,4,4,4,4,4,4,4,4,4,4,4,4};
    return T[c];
}

static inline uint64_t mix64(uint64_t key, uint64_t mask) {   // src/sketch.rs:4-13
    key = ((~key) + (key << 21)) & mask;
    key ^= key >> 24;
    key = (key + (key << 3) + (key << 8)) & mask;
    key ^= key >> 14;
    key = (key + (key << 2) + (key << 4)) & mask;
    key ^= key >> 28;
    key = (key + (key << 31)) & mask;
    return key;
}

// src/sketch.rs:29-100, with the ring buffer held as parallel arrays.
bool host_sketch(const uint8_t* seq, size_t len, int w, int k, uint32_t rid, bool hpc, std::vector<HostMinimizer>& out) {
    if (len == 0 || w <= 0 || w >= 256 || k <= 0 || k > 28) return false;
    const uint64_t NONE = ~0ULL;
    const uint64_t mask = (1ULL << (2 * k)) - 1, shift1 = 2ULL * (uint64_t)(k - 1);
    uint64_t fw = 0, rv = 0;
    int32_t l = 0, span = 0;
    uint64_t bx[256], by[256];
    for (int j = 0; j < w; ++j) { bx[j] = NONE; by[j] = NONE; }
    int bp = 0, mp = 0;
    uint64_t mx = NONE, my = NONE;
    int32_t hq[32]; int hq_front = 0, hq_count = 0;   // TinyQueue (sketch.rs:21-27)
    const int32_t W = w, K = k;
    auto push = [&](uint64_t x, uint64_t y) { out.push_back(HostMinimizer{x, y}); };
    for (size_t i = 0; i < len; ++i) {
        const uint32_t c = nt4h(seq[i]);
        uint64_t ix = NONE, iy = NONE;
        if (c < 4) {
            if (hpc) {
                size_t run = 1;
                if (i + 1 < len && nt4h(seq[i + 1]) == c) {
                    size_t t = i + 2;
                    while (t < len && nt4h(seq[t]) == c) ++t;
                    run = t - i;
                }
                hq[(hq_count + hq_front) & 31] = (int32_t)run; ++hq_count;
                span += (int32_t)run;
                if (hq_count > K) {
                    int32_t x = hq_count ? hq[hq_front] : -1;
                    if (hq_count) { hq_front = (hq_front + 1) & 31; --hq_count; }
                    span -= x;
                }
            } else {
                span = (l + 1 < K) ? l + 1 : K;
            }
            fw = ((fw << 2) | c) & mask;
            rv = (rv >> 2) | ((uint64_t)(3 ^ c) << shift1);
            if (fw != rv) {
                const int z = fw < rv ? 0 : 1;
                ++l;
                if (l >= K && span < 256) {
                    ix = (mix64(z ? rv : fw, mask) << 8) | (uint64_t)span;
                    iy = ((uint64_t)rid << 32) | ((uint64_t)i << 1) | (uint64_t)z;
                }
            }
        } else {
            l = 0; hq_front = 0; hq_count = 0; span = 0;
        }
        bx[bp] = ix; by[bp] = iy;
        if (l == W + K - 1 && mx != NONE) {
            for (int j = bp + 1; j < W; ++j) if (bx[j] == mx && by[j] != my) push(bx[j], by[j]);
            for (int j = 0; j < bp; ++j) if (bx[j] == mx && by[j] != my) push(bx[j], by[j]);
        }
        if (ix <= mx) {
            if (l >= W + K && mx != NONE) push(mx, my);
            mx = ix; my = iy; mp = bp;
        } else if (bp == mp) {
            if (l >= W + K - 1 && mx != NONE) push(mx, my);
            mx = NONE;
            for (int j = bp + 1; j < W; ++j) if (mx >= bx[j]) { mx = bx[j]; my = by[j]; mp = j; }
            for (int j = 0; j <= bp; ++j) if (mx >= bx[j]) { mx = bx[j]; my = by[j]; mp = j; }
            if (l >= W + K - 1 && mx != NONE) {
                for (int j = bp + 1; j < W; ++j) if (bx[j] == mx && by[j] != my) push(bx[j], by[j]);
                for (int j = 0; j <= bp; ++j) if (bx[j] == mx && by[j] != my) push(bx[j], by[j]);
            }
        }
        if (++bp == W) bp = 0;
    }
    if (mx != NONE) push(mx, my);
    return true;
}

// ------------------------------------------------------------------ index
static inline size_t kroundup64(size_t x) { --x; x |= x >> 1; x |= x >> 2; x |= x >> 4; x |= x >> 8; x |= x >> 16; x |= x >> 32; return x + 1; }

template <typename F>
static void parallel_for(size_t n, int n_threads, F fn) {
    if (n_threads <= 1 || n <= 1) { for (size_t i = 0; i < n; ++i) fn(i); return; }
    std::atomic<size_t> next(0);
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t)
        th.emplace_back([&]() { for (size_t i; (i = next.fetch_add(1)) < n;) fn(i); });
    for (auto& x : th) x.join();
}

// post_process of one bucket (src/index.rs:77-108): stable sort by hash; a
// run of one becomes h[(hash>>b)<<1|1] = pos, a longer run a sorted slice of
// p and h[(hash>>b)<<1] = start<<32|n.
static void finish_bucket(std::vector<HostMinimizer>& a, int b, HostBucket& bk) {
    if (a.empty()) return;
    std::stable_sort(a.begin(), a.end(), [](const HostMinimizer& x, const HostMinimizer& y) { return (x.key_span >> 8) < (y.key_span >> 8); });
    size_t n_multi = 0;
    for (size_t s = 0; s < a.size();) {
        size_t e = s + 1;
        while (e < a.size() && (a[e].key_span >> 8) == (a[s].key_span >> 8)) ++e;
        if (e - s > 1) n_multi += e - s;
        s = e;
    }
    bk.p.resize(n_multi);
    bk.h.clear();
    size_t sp = 0;
    for (size_t s = 0; s < a.size();) {
        size_t e = s + 1;
        while (e < a.size() && (a[e].key_span >> 8) == (a[s].key_span >> 8)) ++e;
        const uint64_t key_top = ((a[s].key_span >> 8) >> b) << 1;
        if (e - s == 1) {
            bk.h.push_back({key_top | 1, a[s].rid_pos_strand});
        } else {
            for (size_t t = s; t < e; ++t) bk.p[sp + (t - s)] = a[t].rid_pos_strand;
            std::sort(bk.p.begin() + sp, bk.p.begin() + sp + (e - s));
            bk.h.push_back({key_top, ((uint64_t)sp << 32) | (uint64_t)(e - s)});
            sp += e - s;
        }
        s = e;
    }
    std::sort(bk.h.begin(), bk.h.end());
    bk.has_h = true;
    std::vector<HostMinimizer>().swap(a);
}

bool build_index(const std::vector<const uint8_t*>& seqs, const std::vector<uint64_t>& lens, const std::vector<std::string>* names,
                 int w, int k, int b, int flag, int n_threads, HostIndex& idx, std::string& err) {
    if (w <= 0 || w >= 256 || k <= 0 || k > 28) { err = "invalid w/k (0 < w < 256, 0 < k <= 28)"; return false; }
    if (b < 1 || b > 30) { err = "invalid bucket bits"; return false; }
    const size_t n = seqs.size();
    for (size_t i = 0; i < n; ++i)
        if (lens[i] >= (1ULL << 31)) { err = "sequences must be shorter than 2^31"; return false; }
    idx = HostIndex();
    idx.w = w; idx.k = k; idx.b = b; idx.flag = flag; idx.n_seq = (uint32_t)n;
    const bool hpc = (flag & 1) != 0;
    std::vector<std::vector<HostMinimizer>> minis(n);
    parallel_for(n, n_threads, [&](size_t rid) {
        if (lens[rid]) host_sketch(seqs[rid], lens[rid], w, k, (uint32_t)rid, hpc, minis[rid]);
    });
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) total += lens[i];
    idx.S.assign(kroundup64((size_t)((total + 7) / 8)), 0u);
    uint64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        HostSeq s;
        s.has_name = names != nullptr;
        if (names) s.name = (*names)[i];
        s.offset = off; s.len = (uint32_t)lens[i];
        idx.seq.push_back(s);
        idx.max_len = std::max(idx.max_len, s.len);
        off += lens[i];
    }
    // 4-bit pack (index.rs:14-19, 454-465): contigs are independent word ranges
    // except at shared boundary words, so pack serially per word boundary.
    {
        const uint32_t* dummy = nullptr; (void)dummy;
        for (size_t i = 0; i < n; ++i) {
            const uint8_t* s = seqs[i];
            uint64_t o = idx.seq[i].offset;
            for (uint64_t j = 0; j < lens[i]; ++j, ++o) {
                const size_t wd = (size_t)(o >> 3); const unsigned sh = (unsigned)((o & 7) << 2);
                idx.S[wd] = (idx.S[wd] & ~(0xFu << sh)) | ((nt4h(s[j]) & 0xFu) << sh);
            }
        }
    }
    // buckets in rid-major, sketch order (index.rs:69-72, 469)
    const size_t nb = (size_t)1 << b;
    const uint64_t bmask = nb - 1;
    std::vector<std::vector<HostMinimizer>> bk(nb);
    {
        std::vector<uint32_t> cnt(nb, 0);
        for (size_t i = 0; i < n; ++i) for (const auto& m : minis[i]) cnt[(m.key_span >> 8) & bmask]++;
        for (size_t t = 0; t < nb; ++t) bk[t].reserve(cnt[t]);
        for (size_t i = 0; i < n; ++i) {
            for (const auto& m : minis[i]) bk[(m.key_span >> 8) & bmask].push_back(m);
            std::vector<HostMinimizer>().swap(minis[i]);
        }
    }
    idx.B.assign(nb, HostBucket());
    parallel_for(nb, n_threads, [&](size_t t) { finish_bucket(bk[t], b, idx.B[t]); });
    return true;
}

bool HostIndex::get(uint64_t minier, int& kind, const uint64_t*& pos, size_t& n, uint64_t& single) const {
    kind = 0; n = 0; pos = nullptr;
    const HostBucket& bk = B[(size_t)(minier & ((1ULL << b) - 1))];
    if (!bk.has_h) return false;
    const uint64_t key = (minier >> b) << 1;
    auto find = [&](uint64_t kk) -> const std::pair<uint64_t, uint64_t>* {
        auto it = std::lower_bound(bk.h.begin(), bk.h.end(), std::make_pair(kk, (uint64_t)0));
        return (it != bk.h.end() && it->first == kk) ? &*it : nullptr;
    };
    if (auto e = find(key | 1)) { kind = 1; single = e->second; n = 1; pos = &e->second; return true; }
    if (auto e = find(key)) {
        kind = 2; n = (size_t)(e->second & 0xffffffffULL);
        pos = bk.p.data() + (size_t)(e->second >> 32);
        return true;
    }
    return false;
}

void HostIndex::stats(uint64_t& n_keys, double& avg_occ, double& avg_spacing, uint64_t& total_len) const {
    n_keys = 0; uint64_t sum_occ = 0;
    for (const auto& bk : B) for (const auto& e : bk.h) { ++n_keys; sum_occ += (e.first & 1) ? 1 : (e.second & 0xffffffffULL); }
    total_len = 0; for (const auto& s : seq) total_len += s.len;
    avg_occ = n_keys ? (double)sum_occ / (double)n_keys : 0.0;
    avg_spacing = sum_occ ? (double)total_len / (double)sum_occ : 0.0;
}

int32_t HostIndex::calc_mid_occ(float frac) const {
    std::vector<uint32_t> c;
    for (const auto& bk : B) for (const auto& e : bk.h) c.push_back((e.first & 1) ? 1u : (uint32_t)(e.second & 0xffffffffULL));
    if (c.empty()) return INT32_MAX;
    const size_t n = c.size();
    const double f = (1.0 - (double)frac) * (double)n;
    size_t i = f <= 0.0 ? 0 : (size_t)f;
    if (i > n - 1) i = n - 1;
    std::nth_element(c.begin(), c.begin() + i, c.end());
    return (int32_t)c[i] + 1;
}

// Process-wide switches of the index build / .mmi load (mm2g_set_index_knob).
std::atomic<int64_t> g_index_knob[8] = {};

static int load_threads() {
    if (const int64_t t = g_index_knob[3].load()) return (int)std::max<int64_t>(1, t);   // MM2G_IKNOB_LOAD_THREADS
    return (int)std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
}

// The device table's input: per key (minier, first position, count) and the
// positions, buckets in order.  Per-bucket prefix sums, then threads fill
// disjoint slices.
void HostIndex::flatten(std::vector<uint64_t>& keys, std::vector<uint32_t>& offs, std::vector<uint32_t>& ns, std::vector<uint64_t>& pos) const {
    const size_t nb = B.size();
    std::vector<size_t> ko(nb + 1, 0), po(nb + 1, 0);
    for (size_t t = 0; t < nb; ++t) {
        size_t np = 0;
        for (const auto& e : B[t].h) np += (e.first & 1) ? 1 : (size_t)(e.second & 0xffffffffULL);
        ko[t + 1] = ko[t] + B[t].h.size();
        po[t + 1] = po[t] + np;
    }
    keys.resize(ko[nb]); offs.resize(ko[nb]); ns.resize(ko[nb]); pos.resize(po[nb]);
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t t; (t = next.fetch_add(1)) < nb;) {
            const HostBucket& bk = B[t];
            size_t kq = ko[t], pq = po[t];
            for (const auto& e : bk.h) {
                keys[kq] = ((e.first >> 1) << b) | (uint64_t)t;
                offs[kq] = (uint32_t)pq;
                if (e.first & 1) { ns[kq] = 1; pos[pq++] = e.second; }
                else {
                    const size_t o = (size_t)(e.second >> 32), c = (size_t)(e.second & 0xffffffffULL);
                    ns[kq] = (uint32_t)c;
                    memcpy(pos.data() + pq, bk.p.data() + o, c * 8);
                    pq += c;
                }
                ++kq;
            }
        }
    };
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)load_threads(), nb));
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
}

// ------------------------------------------------------------------ MMI v2
bool save_mmi(const HostIndex& idx, const char* path, std::string& err) {
    FILE* f = fopen(path, "wb");
    if (!f) { err = std::string("cannot create ") + path; return false; }
    std::vector<char> iobuf(1 << 22);
    setvbuf(f, iobuf.data(), _IOFBF, iobuf.size());
    bool ok = fwrite("MMI\x02", 1, 4, f) == 4;
    const uint32_t hdr[5] = {(uint32_t)idx.w, (uint32_t)idx.k, (uint32_t)idx.b, (uint32_t)idx.seq.size(), (uint32_t)idx.flag};
    ok = ok && fwrite(hdr, 4, 5, f) == 5;
    uint64_t sum = 0;
    for (const auto& s : idx.seq) {
        uint8_t l = s.has_name ? (uint8_t)std::min<size_t>(s.name.size(), 255) : 0;
        ok = ok && fwrite(&l, 1, 1, f) == 1;
        if (l) ok = ok && fwrite(s.name.data(), 1, l, f) == l;
        ok = ok && fwrite(&s.len, 4, 1, f) == 1;
        sum += s.len;
    }
    for (const auto& bk : idx.B) {
        const uint32_t n = (uint32_t)bk.p.size();
        ok = ok && fwrite(&n, 4, 1, f) == 1;
        if (n) ok = ok && fwrite(bk.p.data(), 8, n, f) == n;
        const uint32_t sz = bk.has_h ? (uint32_t)bk.h.size() : 0;
        ok = ok && fwrite(&sz, 4, 1, f) == 1;
        for (const auto& e : bk.h) { ok = ok && fwrite(&e.first, 8, 1, f) == 1 && fwrite(&e.second, 8, 1, f) == 1; }
    }
    const size_t words = (size_t)((sum + 7) / 8);
    if (words) ok = ok && fwrite(idx.S.data(), 4, words, f) == words;
    ok = (fclose(f) == 0) && ok;
    if (!ok) err = std::string("write failed: ") + path;
    return ok;
}

// load_from_mmi (src/index.rs:361-424).  The reference reads word by word;
// here the file is mapped, a sequential walk records where each bucket starts
// (two words per bucket), and threads then copy, sort and de-duplicate the
// buckets' tables independently.
bool load_mmi(const char* path, HostIndex& idx, std::string& err) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { err = std::string("cannot open ") + path; return false; }
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); err = std::string("cannot stat ") + path; return false; }
    const size_t fsz = (size_t)st.st_size;
    const uint8_t* m = nullptr;
    if (fsz) {
        void* mp = mmap(nullptr, fsz, PROT_READ, MAP_PRIVATE, fd, 0);
        if (mp == MAP_FAILED) { close(fd); err = std::string("cannot map ") + path; return false; }
        m = (const uint8_t*)mp;
        madvise(mp, fsz, MADV_WILLNEED);
    }
    close(fd);
    struct Unmap { const uint8_t* m; size_t n; ~Unmap() { if (m) munmap((void*)m, n); } } um{m, fsz};
    size_t cur = 0;
    auto rd = [&](void* p, size_t n) { if (fsz - cur < n) return false; memcpy(p, m + cur, n); cur += n; return true; };
    auto fail = [&](const char* msg) { err = msg; return false; };
    char magic[4];
    if (!rd(magic, 4) || memcmp(magic, "MMI\x02", 4) != 0) return fail("invalid MMI magic");
    uint32_t hdr[5];
    if (!rd(hdr, 20)) return fail("truncated MMI header");
    if (hdr[2] < 1 || hdr[2] > 30) return fail("invalid MMI bucket bits");
    idx = HostIndex();
    idx.w = (int32_t)hdr[0]; idx.k = (int32_t)hdr[1]; idx.b = (int32_t)hdr[2]; idx.n_seq = hdr[3]; idx.flag = (int32_t)hdr[4];
    uint64_t sum = 0;
    for (uint32_t i = 0; i < hdr[3]; ++i) {
        uint8_t nl;
        if (!rd(&nl, 1)) return fail("truncated MMI sequence table");
        HostSeq s; s.has_name = nl > 0; s.name.assign(nl, '\0');
        if (nl && !rd(&s.name[0], nl)) return fail("truncated MMI sequence name");
        if (!rd(&s.len, 4)) return fail("truncated MMI sequence length");
        s.offset = sum; sum += s.len;
        idx.max_len = std::max(idx.max_len, s.len);
        idx.seq.push_back(std::move(s));
    }
    const size_t nb = (size_t)1 << idx.b;
    std::vector<size_t> at(nb);                    // file offset of bucket i's `n`
    for (size_t i = 0; i < nb; ++i) {
        at[i] = cur;
        uint32_t n, sz;
        if (!rd(&n, 4)) return fail("truncated MMI bucket");
        if (fsz - cur < 8 * (size_t)n) return fail("truncated MMI positions");
        cur += 8 * (size_t)n;
        if (!rd(&sz, 4)) return fail("truncated MMI bucket size");
        if ((fsz - cur) / 16 < (size_t)sz) return fail("truncated MMI hash table");
        cur += 16 * (size_t)sz;
    }
    const size_t words = (size_t)((sum + 7) / 8);
    if ((fsz - cur) / 4 < words) return fail("truncated MMI packed sequence");
    idx.S.resize(words);
    if (words) memcpy(idx.S.data(), m + cur, 4 * words);
    idx.B.assign(nb, HostBucket());
    std::atomic<size_t> next{0};
    std::atomic<bool> bad{false};
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < nb && !bad.load(std::memory_order_relaxed);) {
            HostBucket& bk = idx.B[i];
            const uint8_t* q = m + at[i];
            uint32_t n, sz;
            memcpy(&n, q, 4); q += 4;
            bk.p.resize(n);
            if (n) memcpy(bk.p.data(), q, 8 * (size_t)n);
            q += 8 * (size_t)n;
            memcpy(&sz, q, 4); q += 4;
            if (!sz) continue;
            bk.has_h = true;
            bk.h.resize(sz);
            memcpy((void*)bk.h.data(), q, 16 * (size_t)sz);
            std::stable_sort(bk.h.begin(), bk.h.end(), [](const std::pair<uint64_t, uint64_t>& x, const std::pair<uint64_t, uint64_t>& y) { return x.first < y.first; });
            // HashMap::insert semantics: a later duplicate key overwrites an earlier one
            size_t o = 0;
            for (size_t j = 0; j < bk.h.size(); ++j) {
                if (o && bk.h[o - 1].first == bk.h[j].first) bk.h[o - 1] = bk.h[j];
                else bk.h[o++] = bk.h[j];
            }
            bk.h.resize(o);
            for (const auto& e : bk.h)
                if (!(e.first & 1) && (e.second >> 32) + (e.second & 0xffffffffULL) > bk.p.size()) bad = true;
        }
    };
    const int nt = (int)std::min<size_t>((size_t)load_threads(), nb);
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (bad) return fail("MMI multi entry out of range");
    return true;
}

}  // namespace mm2g
