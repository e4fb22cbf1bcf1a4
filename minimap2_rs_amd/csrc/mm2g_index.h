// Host-side index (src/index.rs) and FASTA input for the MI355X path.
#pragma once
#include <atomic>
#include <stdint.h>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace mm2g {

struct FastaRecord { std::string name; std::string seq; };
// noodles-fasta stand-in: name = header up to the first
// space/tab; sequence lines concatenated with '\r' stripped.
bool read_fasta(const char* path, std::vector<FastaRecord>& out, bool first_only, std::string& err);

// Streaming reader of FASTA ('>', the read_fasta rules) and FASTQ ('@' header,
// sequence lines up to '+', quality skipped by length) records, one at a time
// (the CLI's double-buffered align pipeline).
class SeqStream {
  public:
    ~SeqStream();
    bool open(const char* path, std::string& err);
    bool next(FastaRecord& rec);          // false at end of input
  private:
    bool getline_(std::string& s);        // without '\n' / trailing '\r'
    FILE* fp_ = nullptr;
    char* buf_ = nullptr;
    size_t cap_ = 0;
    std::string pending_;
    bool has_pending_ = false;
};

struct HostMinimizer { uint64_t key_span, rid_pos_strand; };
// sketch_sequence (src/sketch.rs:29-100) on the host, incl. the HPC branch
// (index build with -H).  Returns false on the reference's assert conditions.
bool host_sketch(const uint8_t* seq, size_t len, int w, int k, uint32_t rid, bool hpc, std::vector<HostMinimizer>& out);

struct HostSeq { bool has_name; std::string name; uint64_t offset; uint32_t len; };

// An allocator whose resize leaves new elements uninitialised (no zero fill of the
// ~2 GB S of hg38 on one thread); every writer of S fills all of it.
template <typename T>
struct DefaultInitAlloc : std::allocator<T> {
    template <typename U> struct rebind { using other = DefaultInitAlloc<U>; };
    DefaultInitAlloc() = default;
    template <typename U> DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <typename U> void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <typename U, typename... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
using SVec = std::vector<uint32_t, DefaultInitAlloc<uint32_t>>;

// Bucket b of the reference Index (src/index.rs:31): `p` plus the hash table
// `h`, kept here as (key, value) pairs sorted by key.
struct HostBucket {
    std::vector<uint64_t> p;
    std::vector<std::pair<uint64_t, uint64_t>> h;
    bool has_h = false;
};

struct HostIndex {
    int32_t w = 0, k = 0, b = 0, flag = 0;
    uint32_t n_seq = 0;
    std::vector<HostSeq> seq;
    SVec S;                                // 4-bit packed reference (index.rs:14-19)
    std::vector<HostBucket> B;
    uint32_t max_len = 0;

    bool get(uint64_t minier, int& kind, const uint64_t*& pos, size_t& n, uint64_t& single) const;
    void stats(uint64_t& n_keys, double& avg_occ, double& avg_spacing, uint64_t& total_len) const;
    int32_t calc_mid_occ(float frac) const;
    // Flat (minier, off, n) + positions export for the device table.
    void flatten(std::vector<uint64_t>& keys, std::vector<uint32_t>& offs, std::vector<uint32_t>& ns, std::vector<uint64_t>& pos) const;
};

bool build_index(const std::vector<const uint8_t*>& seqs, const std::vector<uint64_t>& lens, const std::vector<std::string>* names,
                 int w, int k, int b, int flag, int n_threads, HostIndex& idx, std::string& err);
// The same index built on `device` (mm2g_ixbuild.hip).  unsupported = the GPU
// path does not apply (HPC, even k, slot overflow): use build_index.
bool build_index_gpu(int device, const std::vector<const uint8_t*>& seqs, const std::vector<uint64_t>& lens,
                     const std::vector<std::string>* names, int w, int k, int b, int flag, HostIndex& idx, std::string& err,
                     bool& unsupported);
bool load_mmi(const char* path, HostIndex& idx, std::string& err);
// mm2g_set_index_knob values (index = MM2G_IKNOB_*; 0 = default)
extern std::atomic<int64_t> g_index_knob[8];
bool save_mmi(const HostIndex& idx, const char* path, std::string& err);

}  // namespace mm2g
