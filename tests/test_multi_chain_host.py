"""CPU: the product's host multi-chain epilogue (mm2g_multi_chain_lines, the
code mm2g_batch_results runs per read under -n <= 1 -m <= k) against the
oracle's Align flow, read by read, with the oracle's own anchors and DP arrays
as input -- so the backtrack, the restated rustc 1.81+ sort_unstable, the
merge, the selection and the PAF records are checked without a GPU
(DESIGN.md §2 "-n <= 1").  The rescue decision follows the device's rule for
this mode: chains[0] is one anchor, its coverage is the span (lchain.rs:321-326)."""
import numpy as np
import pytest

import minimap2_rs_amd as M
from oracle import oracle as O
from tools import simdata


@pytest.fixture(scope="module")
def world(tmp_path_factory):
    td = tmp_path_factory.mktemp("multihost")
    ref = str(td / "ref.fa")
    reads = str(td / "reads.fa")
    simdata.write_genome("small", 1.0, 11, ref)
    simdata.write_reads(ref, 60, 4000, 12, reads)
    return ref, reads, td


def _paf_line(name, qlen, ln, tnames, tlens):
    qs, qe = (qlen - ln.qe, qlen - ln.qs) if ln.rev else (ln.qs, ln.qe)
    dv = float(np.float32(ln.dv))
    return (f"{name}\t{qlen}\t{qs}\t{qe}\t{'-' if ln.rev else '+'}\t{tnames[ln.rid]}\t{tlens[ln.rid]}\t{ln.ts}\t{ln.te}\t"
            f"{max(ln.qe - ln.qs, 0)}\t{max(ln.te - ln.ts, 0)}\t60\ttp:A:{'P' if ln.primary else 'S'}\tcm:i:{ln.cm}\t"
            f"s1:i:{max(ln.s1, 0)}\ts2:i:{max(ln.s2, 0)}\tdv:f:{dv:.4f}\trl:i:0")


@pytest.mark.parametrize("mc,m,best_n,mask,pri", [(1, 15, 5, 0.5, 0.8), (0, 0, 5, 0.5, 0.8), (-1, 8, 2, 0.5, 0.8), (1, 1, 5, 0.5, 0.8),
                                                  (1, 15, 50, 0.1, 0.5), (1, 15, 50, 0.9, 0.0), (1, 15, 5, 1.0, 0.8), (1, 15, 20, 0.0, 0.3)])
def test_multi_chain_host_vs_oracle(world, mc, m, best_n, mask, pri):
    """-M (mask_level) and -p (pri_ratio) across their range exercise the primary test's
    overlap threshold, its range memo and both segment trees (mm2g_multi.cpp)."""
    ref, reads, td = world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    mid = max(oi.mid_occ(2e-4), 10)
    recs = O.read_fasta(reads)
    targets = O.read_fasta(ref)
    tnames = [t[0] for t in targets]
    tlens = np.array([len(t[1]) for t in targets], dtype=np.uint32)
    want_path = str(td / f"want_{mc}_{m}_{best_n}_{mask}_{pri}.paf")
    oi.align_fasta(reads, want_path, min_cnt=mc, min_chain_score=m, best_n=best_n, mid_occ=mid, mask_level=mask, pri_ratio=pri)
    want = {}
    for ln in open(want_path).read().splitlines():
        want.setdefault(ln.split("\t")[0], []).append(ln)
    opts = M.map_opts(min_cnt=mc, min_chain_score=m, best_n=best_n, mask_level=mask, pri_ratio=pri)
    n_lines = n_panic = 0
    for name, q in recs:
        xy, _ = oi.anchors(q, 10, 15, mid)
        got = []
        if len(xy):
            qlen = len(q)
            cov = 15                                   # one-anchor chains[0]
            rescue = max(qlen - cov, 0) > 1000 or np.float32(cov) < np.float32(qlen) * (np.float32(1.0) - np.float32(0.1))
            f, pp, _, _, _ = O.chain_dp(xy, k=15, bw=20000 if rescue else 500)
            mv = O.sketch(q, 10, 15)
            pos = ((mv[:, 1] >> np.uint64(1)) & np.uint64(0xffffffff)).astype(np.uint32).view(np.int32) if len(mv) else np.zeros(0, np.int32)
            avg_k = np.float32(np.float32(int((mv[:, 0] & np.uint64(0xff)).sum())) / np.float32(len(mv))) if len(mv) else np.float32(15)
            lines, panic = M.multi_chain_lines(xy, f, pp, qlen, pos, float(avg_k), tlens, opts)
            n_panic += panic
            got = [_paf_line(name, qlen, ln, tnames, tlens) for ln in lines]
        assert got == want.get(name, []), name
        n_lines += len(got)
    assert n_lines > len(want) > 5 or n_panic


@pytest.fixture(scope="module")
def repeat_world(tmp_path_factory):
    """The first contig of a 1 %-scale hg38-shaped genome (repeat families, no odd rid, so
    no Q19 panic): hundreds of one-anchor chains per 10 kb read at -n 1 -m 15."""
    td = tmp_path_factory.mktemp("multirep")
    names, lens, buf = simdata.genome("hg38", 0.01, 38, threads=4)
    n0 = int(lens[0])
    ref = str(td / "ref.fa")
    simdata.write_fasta(ref, names[:1], [buf[:n0].tobytes()])
    reads = str(td / "reads.fa")
    simdata.write_reads(ref, 16, 10000, 7, reads)
    return ref, reads, td


@pytest.mark.parametrize("mask,pri,best_n", [(0.5, 0.8, 5), (0.2, 0.0, 100)])
def test_multi_chain_host_repeats(repeat_world, mask, pri, best_n):
    """Dense repeats: the range memo and both trees of the primary test decide most
    chains; the lines must equal the oracle Align flow's."""
    ref, reads, td = repeat_world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    mid = max(oi.mid_occ(2e-4), 10)
    want_path = str(td / f"want_{mask}_{pri}_{best_n}.paf")
    oi.align_fasta(reads, want_path, min_cnt=1, min_chain_score=15, best_n=best_n, mid_occ=mid, mask_level=mask, pri_ratio=pri)
    want = {}
    for ln in open(want_path).read().splitlines():
        want.setdefault(ln.split("\t")[0], []).append(ln)
    targets = O.read_fasta(ref)
    tnames = [t[0] for t in targets]
    tlens = np.array([len(t[1]) for t in targets], dtype=np.uint32)
    opts = M.map_opts(min_cnt=1, min_chain_score=15, best_n=best_n, mask_level=mask, pri_ratio=pri)
    n_chains = 0
    for name, q in O.read_fasta(reads):
        xy, _ = oi.anchors(q, 10, 15, mid)
        got = []
        if len(xy):
            qlen = len(q)
            cov = 15
            rescue = max(qlen - cov, 0) > 1000 or np.float32(cov) < np.float32(qlen) * (np.float32(1.0) - np.float32(0.1))
            f, pp, _, _, _ = O.chain_dp(xy, k=15, bw=20000 if rescue else 500)
            mv = O.sketch(q, 10, 15)
            pos = ((mv[:, 1] >> np.uint64(1)) & np.uint64(0xffffffff)).astype(np.uint32).view(np.int32)
            avg_k = np.float32(np.float32(int((mv[:, 0] & np.uint64(0xff)).sum())) / np.float32(len(mv)))
            lines, panic = M.multi_chain_lines(xy, f, pp, qlen, pos, float(avg_k), tlens, opts)
            got = [_paf_line(name, qlen, ln, tnames, tlens) for ln in lines]
            n_chains += len(xy)
        assert got == want.get(name, []), name
    assert n_chains > 16 * 500 and sum(len(v) for v in want.values()) > 16
