"""Independent pure-Python restatement of the reference Rust (small inputs only).

TEST INFRASTRUCTURE: a second, separately written reading of
/root/reference/src/*.rs used to cross-check the C++ oracle
(oracle/mm2rs_oracle.cpp).  Integers are masked to the Rust widths where
the Rust wraps; f32 arithmetic is emulated with numpy.float32 op by op.
"""
from __future__ import annotations

import math

import numpy as np

U64 = (1 << 64) - 1
MAXU = U64
f32 = np.float32


def nt4(b: int) -> int:  # nt4.rs:2-10
    return {ord("A"): 0, ord("a"): 0, ord("C"): 1, ord("c"): 1, ord("G"): 2, ord("g"): 2, ord("T"): 3, ord("t"): 3}.get(b, 4)


def hash64(key: int, mask: int) -> int:  # sketch.rs:4-13
    key = ((~key & U64) + (key << 21)) & U64 & mask
    key ^= key >> 24
    key = (key + (key << 3) + (key << 8)) & U64 & mask
    key ^= key >> 14
    key = (key + (key << 2) + (key << 4)) & U64 & mask
    key ^= key >> 28
    key = (key + (key << 31)) & U64 & mask
    return key


def sketch_sequence(seq: bytes, w: int, k: int, rid: int, is_hpc: bool):  # sketch.rs:29-100
    assert len(seq) > 0 and 0 < w < 256 and 0 < k <= 28
    out = []
    shift1 = 2 * (k - 1)
    mask = (1 << (2 * k)) - 1
    kmer = [0, 0]
    l = 0
    buf_pos = 0
    min_pos = 0
    kmer_span = 0
    buf = [(MAXU, MAXU)] * w
    mn = (MAXU, MAXU)
    tq = []
    for i in range(len(seq)):
        c = nt4(seq[i])
        info = (MAXU, MAXU)
        if c < 4:
            if is_hpc:
                skip_len = 1
                if i + 1 < len(seq) and nt4(seq[i + 1]) == c:
                    t = i + 2
                    while t < len(seq) and nt4(seq[t]) == c:
                        t += 1
                    skip_len = t - i
                tq.append(skip_len)
                kmer_span += skip_len
                if len(tq) > k:
                    kmer_span -= tq.pop(0)
            else:
                kmer_span = l + 1 if l + 1 < k else k
            kmer[0] = ((kmer[0] << 2) | c) & mask
            kmer[1] = (kmer[1] >> 2) | ((3 ^ c) << shift1)
            if kmer[0] != kmer[1]:
                z = 0 if kmer[0] < kmer[1] else 1
                l += 1
                if l >= k and kmer_span < 256:
                    info = ((hash64(kmer[z], mask) << 8) | kmer_span, (rid << 32) | (i << 1) | z)
        else:
            l = 0
            tq = []
            kmer_span = 0
        buf[buf_pos] = info
        if l == w + k - 1 and mn[0] != MAXU:
            for j in list(range(buf_pos + 1, w)) + list(range(0, buf_pos)):
                if mn[0] == buf[j][0] and buf[j][1] != mn[1]:
                    out.append(buf[j])
        if info[0] <= mn[0]:
            if l >= w + k and mn[0] != MAXU:
                out.append(mn)
            mn = info
            min_pos = buf_pos
        elif buf_pos == min_pos:
            if l >= w + k - 1 and mn[0] != MAXU:
                out.append(mn)
            mn = (MAXU, mn[1])
            for j in list(range(buf_pos + 1, w)) + list(range(0, buf_pos + 1)):
                if mn[0] >= buf[j][0]:
                    mn = buf[j]
                    min_pos = j
            if l >= w + k - 1 and mn[0] != MAXU:
                for j in list(range(buf_pos + 1, w)) + list(range(0, buf_pos + 1)):
                    if mn[0] == buf[j][0] and mn[1] != buf[j][1]:
                        out.append(buf[j])
        buf_pos += 1
        if buf_pos == w:
            buf_pos = 0
    if mn[0] != MAXU:
        out.append(mn)
    return out


def filter_query_minimizers(mv, q_occ_max=10, q_occ_frac=0.01):  # seeds.rs:13-36
    if len(mv) == 0 or q_occ_frac <= 0 or q_occ_max <= 0:
        return list(mv)
    if len(mv) <= q_occ_max:
        return list(mv)
    counts = {}
    for m in mv:
        counts[m[0] >> 8] = counts.get(m[0] >> 8, 0) + 1
    cutoff = int(f32(len(mv)) * f32(q_occ_frac))
    return [m for m in mv if not (counts[m[0] >> 8] > q_occ_max and counts[m[0] >> 8] > cutoff)]


class Index:  # index.rs:28-154 (buckets with a dict as the HashMap)
    def __init__(self, w, k, b, flag):
        self.w, self.k, self.b, self.flag = w, k, b, flag
        self.seq = []
        self.B = [{"a": [], "p": [], "h": None} for _ in range(1 << b)]

    @classmethod
    def build(cls, records, w, k, b, flag):  # index.rs:427-475
        idx = cls(w, k, b, flag)
        mask = (1 << b) - 1
        for rid, (name, s) in enumerate(records):
            mv = sketch_sequence(s, w, k, rid, (flag & 1) != 0) if len(s) else []
            idx.seq.append((name, len(s)))
            for m in mv:
                idx.B[(m[0] >> 8) & mask]["a"].append(m)
        for bk in idx.B:
            a = bk["a"]
            if not a:
                continue
            a.sort(key=lambda m: m[0] >> 8)  # stable
            h = {}
            j = 0
            while j < len(a):
                e = j + 1
                while e < len(a) and (a[e][0] >> 8) == (a[j][0] >> 8):
                    e += 1
                key_top = ((a[j][0] >> 8) >> b) << 1
                if e - j == 1:
                    h[key_top | 1] = a[j][1]
                else:
                    start = len(bk["p"])
                    bk["p"].extend(sorted(m[1] for m in a[j:e]))
                    h[key_top] = (start << 32) | (e - j)
                j = e
            bk["h"] = h
            bk["a"] = []
        return idx

    def get(self, minier):
        bk = self.B[minier & ((1 << self.b) - 1)]
        if bk["h"] is None:
            return None
        key = (minier >> self.b) << 1
        if key | 1 in bk["h"]:
            return ("Single", bk["h"][key | 1])
        if key in bk["h"]:
            v = bk["h"][key]
            off, n = v >> 32, v & 0xFFFFFFFF
            return ("Multi", bk["p"][off:off + n])
        return None

    def calc_mid_occ(self, frac):
        counts = []
        for bk in self.B:
            if bk["h"] is not None:
                for kk, v in bk["h"].items():
                    counts.append(1 if kk & 1 else v & 0xFFFFFFFF)
        if not counts:
            return 2 ** 31 - 1
        counts.sort()
        n = len(counts)
        idx = min(int((1.0 - float(f32(frac))) * n), n - 1)
        return counts[idx] + 1


def i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def as_u64_from_i32(x):
    return x & U64


def push_anchor(r, m, qlen):  # seeds.rs:62-79
    rid = (r >> 32) & 0xFFFFFFFF
    rpos = i32((r >> 1) & 0xFFFFFFFF)
    rstrand = r & 1
    qpos = i32((m[1] >> 1) & 0xFFFFFFFF)
    qstrand = m[1] & 1
    qspan = m[0] & 0xFF
    forward = rstrand == qstrand
    x = ((rid << 32) | as_u64_from_i32(rpos)) if forward else ((1 << 63) | (rid << 32) | as_u64_from_i32(rpos))
    if forward:
        y = (qspan << 32) | as_u64_from_i32(qpos)
    else:
        y = (qspan << 32) | as_u64_from_i32(i32(qlen - (qpos + 1 - qspan) - 1))
    return (x & U64, y & U64)


def build_anchors_filtered(idx, mv, qlen, mid_occ):  # seeds.rs:42-60
    a = []
    for m in mv:
        occ = idx.get(m[0] >> 8)
        if occ is None:
            continue
        if occ[0] == "Single":
            a.append(push_anchor(occ[1], m, qlen))
        else:
            if len(occ[1]) > mid_occ:
                continue
            for r in occ[1]:
                a.append(push_anchor(r, m, qlen))
    a.sort()
    return a


def qpos(a):
    return i32(a[1] & 0xFFFFFFFF)


def qspan(a):
    return (a[1] >> 32) & 0xFF


def rpos(a):
    return i32(a[0] & 0xFFFFFFFF)


def rev(a):
    return (a[0] >> 63) != 0


def rid(a):
    return (a[0] >> 32) & 0x7FFFFFFF


def mg_log2(x):
    if x <= 1:
        return f32(0.0)
    return f32(np.log(f32(x))) / f32(math.log(2.0))


def comput_sc(ai, aj, max_dist_x, max_dist_y, bw, gap, skip):  # lchain.rs:17-34
    dq = i32(qpos(ai) - qpos(aj))
    if dq <= 0 or dq > max_dist_x:
        return None
    dr = i32(rpos(ai) - rpos(aj))
    if dr == 0 or dq > max_dist_y:
        return None
    dd = abs(dr - dq)
    if dd > bw:
        return None
    dg = min(dr, dq)
    q_span = qspan(aj)
    sc = min(q_span, dg)
    if dd != 0 or dg > q_span:
        lin_pen = f32(gap) * f32(dd) + f32(skip) * f32(dg)
        log_pen = mg_log2(dd + 1) if dd >= 1 else f32(0.0)
        sc -= int(f32(lin_pen + f32(0.5) * log_pen))
    return sc


def chain_dp_all_dp(anchors, max_dist_x=5000, max_dist_y=5000, bw=500, max_iter=5000, gap=None, k=15, max_skip=25):
    """The DP fill of chain_dp_all (lchain.rs:59-91): returns f, pprev, v."""
    if gap is None:
        gap = f32(f32(0.01) * f32(0.8)) * f32(k)
    n = len(anchors)
    max_dist_x = max(max_dist_x, bw)
    max_dist_y = max(max_dist_y, bw)
    f = [0] * n
    v = [0] * n
    t = [0] * n
    pprev = [-1] * n
    st = 0
    for i in range(n):
        while st < i and (rid(anchors[st]) != rid(anchors[i]) or rev(anchors[st]) != rev(anchors[i])
                          or rpos(anchors[i]) > rpos(anchors[st]) + max_dist_x):
            st += 1
        max_j = -1
        max_f = qspan(anchors[i])
        start_j = i - max_iter if i - max_iter > st else st
        n_skip = 0
        for j in range(i - 1, start_j - 1, -1):
            if rid(anchors[j]) != rid(anchors[i]) or rev(anchors[j]) != rev(anchors[i]):
                continue
            sc0 = comput_sc(anchors[i], anchors[j], max_dist_x, max_dist_y, bw, gap, 0.0)
            if sc0 is not None:
                sc = sc0 + f[j]
                if sc > max_f:
                    max_f = sc
                    max_j = j
                    if n_skip > 0:
                        n_skip -= 1
                elif t[j] == i:
                    n_skip += 1
                    if n_skip > max_skip:
                        break
                if pprev[j] >= 0:
                    t[pprev[j]] = i
        f[i] = max_f
        pprev[i] = max_j
        v[i] = v[max_j] if (max_j >= 0 and v[max_j] > max_f) else max_f
    return f, pprev, v


def fallback_chain(f, pprev, v):
    """lchain.rs:162-173 (the only chain under min_cnt >= 2): last argmax."""
    best_i = max(range(len(f)), key=lambda i: (f[i], i))
    ch = []
    i = best_i
    while i >= 0:
        ch.append(i)
        i = pprev[i]
    return ch[::-1], v[best_i]


# ---------------------------------------------------------------- align flow
I32MAX = 2 ** 31 - 1


def chain_qrange(anchors, chain):  # lchain.rs:178-188
    qs, qe = I32MAX, -1
    for i in chain:
        s = qpos(anchors[i]) - (qspan(anchors[i]) - 1)
        e = qpos(anchors[i]) + 1
        qs = min(qs, s)
        qe = max(qe, e)
    return max(qs, 0), qe


def rust_binary_search(xs, target):
    """slice::binary_search as implemented in Rust >= 1.82 (base/size halving);
    returns the index found or None (paf.rs:178)."""
    size = len(xs)
    if size == 0:
        return None
    base = 0
    while size > 1:
        half = size // 2
        mid = base + half
        base = base if xs[mid] > target else mid
        size -= half
    return base if xs[base] == target else None


def paf_line(index, anchors, chain, qname, q, s1):  # paf.rs:130-236
    a0 = anchors[chain[0]]
    strand = "-" if rev(a0) else "+"
    qs, qe, ts, te = I32MAX, -1, I32MAX, -1
    for i in chain:
        a = anchors[i]
        qs = min(qs, qpos(a) - (qspan(a) - 1)); qe = max(qe, qpos(a) + 1)
        ts = min(ts, rpos(a) - (qspan(a) - 1)); te = max(te, rpos(a) + 1)
    qs, ts = max(qs, 0), max(ts, 0)
    rid0 = (a0[0] >> 32) & 0x7FFFFFFF
    if rid0 >= len(index.seq):
        return None, True                     # idx.seq[rid] out of bounds: the reference panics
    tname, tlen = index.seq[rid0]
    mv = sketch_sequence(q, index.w, index.k, 0, False)
    mini_pos = [i32((m[1] >> 1) & 0xFFFFFFFF) for m in mv]
    sum_k = sum(m[0] & 0xFF for m in mv)
    avg_k = f32(f32(sum_k) / f32(len(mv))) if mv else f32(index.k)
    qlen = len(q)

    def qfwd(a):
        return (qlen - 1 - (qpos(a) + 1 - qspan(a))) if rev(a) else qpos(a)

    cq = [qfwd(anchors[i]) for i in (reversed(chain) if strand == "-" else chain)]
    dv = f32(0.0)
    if mini_pos and cq:
        st = rust_binary_search(mini_pos, cq[0])
        if st is not None:
            while st > 0 and mini_pos[st - 1] == cq[0]:
                st -= 1
            j, k, en, n_match = st, 1, st, 1
            while j + 1 < len(mini_pos) and k < len(cq):
                j += 1
                if mini_pos[j] == cq[k]:
                    n_match += 1; en = j; k += 1
            n_tot = en - st + 1
            rqs = qlen - qe if strand == "-" else qs
            rqe = qlen - qs if strand == "-" else qe
            ak = int(avg_k)                   # `avg_k as i32` (truncation)
            if rqs > ak and ts > ak:
                n_tot += 1
            if qlen - rqe > ak and tlen - te > ak:
                n_tot += 1
            frac = f32(f32(n_match) / f32(n_tot))
            dv = f32(0.0) if frac >= f32(1.0) else f32(f32(1.0) - np.power(frac, f32(f32(1.0) / max(avg_k, f32(1.0)))))
    pqs, pqe = (qlen - qe, qlen - qs) if strand == "-" else (qs, qe)
    line = (f"{qname}\t{qlen}\t{pqs}\t{pqe}\t{strand}\t{tname or '*'}\t{tlen}\t{ts}\t{te}\t{max(qe - qs, 0)}\t{max(te - ts, 0)}"
            f"\t60\ttp:A:P\tcm:i:{len(chain)}\ts1:i:{max(s1, 0)}\ts2:i:0\tdv:f:{float(dv):.4f}\trl:i:0")
    return line, False


def align_one(index, qname, q, mid_occ, w=10, k=15):
    """The Align flow of src/main.rs:189-230 for one read with default chain
    parameters (main.rs:105-123): -> (PAF line or None, panics?, rescued?)."""
    if len(q) == 0:
        return None, False, False
    mv = filter_query_minimizers(sketch_sequence(q, w, k, 0, False))
    anchors = build_anchors_filtered(index, mv, len(q), mid_occ)
    if not anchors:
        return None, False, False
    gap = f32(f32(0.01) * f32(0.8)) * f32(k)
    f, pprev, v = chain_dp_all_dp(anchors, 5000, 5000, 500, 5000, gap, k, 25)
    chain, score = fallback_chain(f, pprev, v)
    qs, qe = chain_qrange(anchors, chain)
    cov = max(qe - qs, 0)
    rescued = max(len(q) - cov, 0) > 1000 or f32(cov) < f32(len(q)) * (f32(1.0) - f32(0.1))
    if rescued:   # rescue_long_join: bw = bw_long -> max_dist_x = max_dist_y = 20000 (lchain.rs:63-66)
        f, pprev, v = chain_dp_all_dp(anchors, 5000, 5000, 20000, 5000, gap, k, 25)
        chain, score = fallback_chain(f, pprev, v)
    line, panic = paf_line(index, anchors, chain, qname, q, score)
    return line, panic, rescued


# ---------------------------------------------------------------- Rust sort_unstable
# Second restatement (the oracle's is C++, rsort:: in oracle/mm2rs_oracle.cpp) of
# `slice::sort_unstable_by_key` as rustc compiles lchain.rs:97 / :267 / :292, on a
# list of (key, payload) with is_less = key(a) < key(b).  Written against
# rust-lang/rust library/core: ipnsort (1.81+) sort/unstable/{mod,quicksort,
# heapsort}.rs + sort/shared/{pivot,smallsort}.rs; pdqsort (<= 1.80) slice/sort.rs.

def _lt(a, b):
    return a[0] < b[0]


def _insertion_left(v, lo, hi, offset, lt):  # insertion_sort_shift_left(v[lo:hi], offset)
    for i in range(lo + offset, hi):
        tmp = v[i]
        if lt(tmp, v[i - 1]):
            j = i
            while True:
                v[j] = v[j - 1]
                j -= 1
                if j == lo or not lt(tmp, v[j - 1]):
                    break
            v[j] = tmp


def _heapsort(v, lo, hi, lt):  # unstable/heapsort.rs (same sift order as the <= 1.80 heapsort)
    n = hi - lo

    def sift(end, node):
        while True:
            child = 2 * node + 1
            if child >= end:
                return
            if child + 1 < end and lt(v[lo + child], v[lo + child + 1]):
                child += 1
            if not lt(v[lo + node], v[lo + child]):
                return
            v[lo + node], v[lo + child] = v[lo + child], v[lo + node]
            node = child

    for i in range(n + n // 2 - 1, -1, -1):
        if i >= n:
            sift(n, i - n)
        else:
            v[lo], v[lo + i] = v[lo + i], v[lo]
            sift(i, 0)


def _small_sort_general(v, lo, hi, lt):
    # sort8_stable/sort4_stable + insert_tail + bidirectional_merge: a stable sort
    v[lo:hi] = sorted(v[lo:hi], key=lambda e: e[0])


def _median3(v, a, b, c, lt):
    x = lt(v[a], v[b])
    y = lt(v[a], v[c])
    if x == y:
        z = lt(v[b], v[c])
        return c if (z != x) else b
    return a


def _median3_rec(v, a, b, c, n, lt):
    if n * 8 >= 64:
        n8 = n // 8
        a = _median3_rec(v, a, a + n8 * 4, a + n8 * 7, n8, lt)
        b = _median3_rec(v, b, b + n8 * 4, b + n8 * 7, n8, lt)
        c = _median3_rec(v, c, c + n8 * 4, c + n8 * 7, n8, lt)
    return _median3(v, a, b, c, lt)


def _partition_lomuto(v, lo, hi, piv, lt):
    """partition(): pivot to the front, partition_lomuto_branchless_cyclic on the rest, pivot to num_lt."""
    v[lo], v[piv] = v[piv], v[lo]
    p = v[lo]
    base, n = lo + 1, hi - lo - 1
    num_lt = 0
    if n:
        gap_val = v[base]
        gap = base
        srcs = list(range(base + 1, base + n)) + [None]
        for s in srcs:
            rv = gap_val if s is None else v[s]
            is_lt = lt(rv, p)
            v[gap] = v[base + num_lt]
            v[base + num_lt] = rv
            gap = s
            num_lt += 1 if is_lt else 0
    v[lo], v[lo + num_lt] = v[lo + num_lt], v[lo]
    return num_lt


def _quicksort_ipn(v, lo, hi, anc, limit, lt):
    while True:
        n = hi - lo
        if n <= 32:
            _small_sort_general(v, lo, hi, lt)
            return
        if limit == 0:
            _heapsort(v, lo, hi, lt)
            return
        limit -= 1
        d8 = n // 8
        if n < 64:
            pp = _median3(v, lo, lo + d8 * 4, lo + d8 * 7, lt)
        else:
            pp = _median3_rec(v, lo, lo + d8 * 4, lo + d8 * 7, d8, lt)
        if anc is not None and not lt(anc, v[pp]):
            num = _partition_lomuto(v, lo, hi, pp, lambda a, b: not lt(b, a))
            lo += num + 1
            anc = None
            continue
        num = _partition_lomuto(v, lo, hi, pp, lt)
        _quicksort_ipn(v, lo, lo + num, anc, limit, lt)
        anc = v[lo + num]
        lo += num + 1


def rust_sort_unstable_ipn(v, lt=_lt):
    """rustc 1.81+ sort_unstable_by (in place)."""
    n = len(v)
    if n < 2:
        return v
    if n <= 20:
        _insertion_left(v, 0, n, 1, lt)
        return v
    run = 2
    desc = lt(v[1], v[0])
    if desc:
        while run < n and lt(v[run], v[run - 1]):
            run += 1
    else:
        while run < n and not lt(v[run], v[run - 1]):
            run += 1
    if run == n:
        if desc:
            v.reverse()
        return v
    limit = 2 * ((n | 1).bit_length() - 1)
    _quicksort_ipn(v, 0, n, None, limit, lt)
    return v


def _pdq_partition_in_blocks(v, lo, hi, p, lt):
    BLOCK = 128
    l, r = lo, hi
    bl, br = BLOCK, BLOCK
    offl, offr = [], []          # pending offsets (consumed from the front)
    il = ir = 0
    while True:
        done = r - l <= 2 * BLOCK
        if done:
            rem = r - l
            if il < len(offl) or ir < len(offr):
                rem -= BLOCK
            if il < len(offl):
                br = rem
            elif ir < len(offr):
                bl = rem
            else:
                bl = rem // 2
                br = rem - bl
        if il == len(offl):
            offl = [i for i in range(bl) if not lt(v[l + i], p)]
            il = 0
        if ir == len(offr):
            offr = [i for i in range(br) if lt(v[r - 1 - i], p)]
            ir = 0
        cnt = min(len(offl) - il, len(offr) - ir)
        if cnt:
            L = lambda: l + offl[il]
            R = lambda: r - 1 - offr[ir]
            tmp = v[L()]
            v[L()] = v[R()]
            for _ in range(1, cnt):
                il += 1
                v[R()] = v[L()]
                ir += 1
                v[L()] = v[R()]
            v[R()] = tmp
            il += 1
            ir += 1
        if il == len(offl):
            l += bl
        if ir == len(offr):
            r -= br
        if done:
            break
    if il < len(offl):
        end = len(offl)
        while il < end:
            end -= 1
            a, b = l + offl[end], r - 1
            v[a], v[b] = v[b], v[a]
            r -= 1
        return r - lo
    if ir < len(offr):
        end = len(offr)
        while ir < end:
            end -= 1
            a, b = l, r - 1 - offr[end]
            v[a], v[b] = v[b], v[a]
            l += 1
        return l - lo
    return l - lo


def _pdq_choose_pivot(v, lo, hi, lt):
    n = hi - lo
    idx = [n // 4, n // 4 * 2, n // 4 * 3]
    swaps = [0]

    def s2(i, j):
        if lt(v[lo + idx[j]], v[lo + idx[i]]):
            idx[i], idx[j] = idx[j], idx[i]
            swaps[0] += 1

    if n >= 8:
        if n >= 50:
            for t in range(3):
                m = idx[t]
                trip = [m - 1, m, m + 1]
                for (i, j) in ((0, 1), (1, 2), (0, 1)):
                    if lt(v[lo + trip[j]], v[lo + trip[i]]):
                        trip[i], trip[j] = trip[j], trip[i]
                        swaps[0] += 1
                idx[t] = trip[1]
        s2(0, 1)
        s2(1, 2)
        s2(0, 1)
    if swaps[0] < 12:
        return idx[1], swaps[0] == 0
    v[lo:hi] = v[lo:hi][::-1]
    return n - 1 - idx[1], True


def _pdq_partial_insertion(v, lo, hi, lt):
    n = hi - lo
    i = 1
    for _ in range(5):
        while i < n and not lt(v[lo + i], v[lo + i - 1]):
            i += 1
        if i == n:
            return True
        if n < 50:
            return False
        v[lo + i - 1], v[lo + i] = v[lo + i], v[lo + i - 1]
        if i >= 2:
            _insertion_left(v, lo, lo + i, i - 1, lt)
            # shift_head of v[i..]: v[i] moves right past smaller successors
            j = lo + i
            if j + 1 < hi and lt(v[j + 1], v[j]):
                tmp = v[j]
                while j + 1 < hi and lt(v[j + 1], tmp):
                    v[j] = v[j + 1]
                    j += 1
                v[j] = tmp
    return False


def _pdq_recurse(v, lo, hi, pred, limit, lt):
    balanced = partitioned = True
    while True:
        n = hi - lo
        if n <= 20:
            if n >= 2:
                _insertion_left(v, lo, hi, 1, lt)
            return
        if limit == 0:
            _heapsort(v, lo, hi, lt)
            return
        if not balanced:
            if n >= 8:      # break_patterns: xorshift64 seeded with len
                seed = n
                mod = 1 << (n - 1).bit_length()
                pos = n // 4 * 2
                for i in range(3):
                    r = seed
                    r ^= (r << 13) & 0xFFFFFFFFFFFFFFFF
                    r ^= r >> 7
                    r ^= (r << 17) & 0xFFFFFFFFFFFFFFFF
                    seed = r
                    other = r & (mod - 1)
                    if other >= n:
                        other -= n
                    a, b = lo + pos - 1 + i, lo + other
                    v[a], v[b] = v[b], v[a]
            limit -= 1
        piv, likely = _pdq_choose_pivot(v, lo, hi, lt)
        if balanced and partitioned and likely:
            if _pdq_partial_insertion(v, lo, hi, lt):
                return
        pv = lo + piv
        if pred is not None and not lt(pred, v[pv]):
            v[lo], v[pv] = v[pv], v[lo]
            p = v[lo]
            l, r = lo + 1, hi
            while True:
                while l < r and not lt(p, v[l]):
                    l += 1
                while l < r and lt(p, v[r - 1]):
                    r -= 1
                if l >= r:
                    break
                r -= 1
                v[l], v[r] = v[r], v[l]
                l += 1
            lo = l           # (l - (lo + 1)) + 1 elements equal to the pivot
            continue
        v[lo], v[pv] = v[pv], v[lo]
        p = v[lo]
        l, r = lo + 1, hi
        while l < r and lt(v[l], p):
            l += 1
        while l < r and not lt(v[r - 1], p):
            r -= 1
        mid = (l - (lo + 1)) + _pdq_partition_in_blocks(v, l, r, p, lt)
        was_p = l >= r
        v[lo], v[lo + mid] = v[lo + mid], v[lo]
        balanced = min(mid, n - mid) >= n // 8
        partitioned = was_p
        if mid < n - mid - 1:
            _pdq_recurse(v, lo, lo + mid, pred, limit, lt)
            pred = v[lo + mid]
            lo = lo + mid + 1
        else:
            _pdq_recurse(v, lo + mid + 1, hi, v[lo + mid], limit, lt)
            hi = lo + mid


def rust_sort_unstable_pdq(v, lt=_lt):
    """rustc <= 1.80 sort_unstable_by (pdqsort, in place)."""
    _pdq_recurse(v, 0, len(v), None, len(v).bit_length(), lt)
    return v
