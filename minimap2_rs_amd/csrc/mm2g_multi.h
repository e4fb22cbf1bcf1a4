// Host epilogue of the Align flow when several chains reach the output:
// `-n <= 1` with `-m <= k` (DESIGN.md §2 "-n <= 1").  The device maps the batch
// with full anchor and DP arrays (no singleton filter) and decides the rescue;
// this code takes one read's sorted anchors and the final pass's f / pprev and
// runs what follows the DP in the reference:
//   backtrack            src/lchain.rs:92-160  (z sorted with sort_unstable_by_key)
//   sort_chains_stable   src/lchain.rs:202-218
//   merge (with gap)     src/lchain.rs:288-314 (sort_unstable_by_key on qs)
//   select + filter      src/lchain.rs:220-260
//   PAF records          src/paf.rs:130-248    (dv with binary_search, rustc >= 1.82)
// Rust's sort_unstable is the rustc 1.81+ algorithm (ipnsort); the order of
// equal keys matters here, so it is restated, not replaced by std::sort.
#pragma once
#include <cstdint>
#include <vector>

namespace mm2g {

struct MultiParams {
    int32_t min_cnt, min_chain_score, max_drop, max_gap;   // -n, -m, max_drop (500), -g (max_dist_y)
    float mask_level, pri_ratio;                           // -M, -p
    int32_t best_n;                                        // -N
};

struct MultiLine {              // one PAF line (paf_from_chain_with_primary)
    int32_t qs, qe, ts, te;     // chain ranges (forward-of-anchor coordinates, as the device's results)
    int32_t rid, rev, cm;
    float dv;
    bool primary;
    int32_t n_match, dv_st, dv_en;
    bool dv_found;
};

struct MultiRead {
    bool panic = false;         // the reference panics on this read (Q19 rid, or an empty chain in the merge)
    int32_t s1 = 0, s2 = 0;
    std::vector<MultiLine> lines;
};

// xy: n anchors {x, y} sorted by (x, y); f, pprev: the final chain_dp_all pass;
// mini_pos: positions of the query minimizers of the dv sketch (idx.w, idx.k),
// avg_k their mean span (f32); tlen[rid] for the n_seq targets.
void multi_chain_read(const uint64_t* xy, const int32_t* f, const int32_t* pprev, int64_t n, int32_t qlen,
                      const int32_t* mini_pos, int64_t n_mini, float avg_k, int32_t idx_k, const uint32_t* tlen, uint32_t n_seq,
                      const MultiParams& P, MultiRead& out);

// Rust's slice::sort_unstable_by_key on (key, payload) pairs (rustc 1.81+), exposed for tests.
void rust_sort_unstable_pairs(std::vector<std::pair<int32_t, uint32_t>>& v);

}  // namespace mm2g
