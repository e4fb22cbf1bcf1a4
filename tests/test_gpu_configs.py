"""GPU: every BASELINE.json configuration at its real shape (SURVEY.md §8d
inputs) against the CPU oracle.

  C1  `mm2rs index -d x.mmi` + `mm2rs align x.mmi q.fa` on a 145 + 133 Mb
      chr8/chr12-shaped pair and one 600 bp read, vs the oracle CLI
  C2  E. coli-shaped 4.64 Mb + 1,000 x 10 kb: every read vs the oracle
  C3  the full 3.09 Gb hg38-shaped index + 300 x 10 kb reads vs the oracle
  C5  the same index + 24 x 100 kb reads (+ 8 chimeras): reads above 65,535 anchors (the
      whole-read radix sort) and rescue segments beyond LDS (the HBM variant
      of k_chain_giant) vs the oracle's PAF, per-read outcome and DP arrays
C4 is C3's workload sharded over 8 GPUs; its per-GPU path is C3's.
Every comparison covers reads on which the reference panics (Q19) through
the per-read outcome (O.align_records)."""
import os
import subprocess

import numpy as np
import pytest

import minimap2_rs_amd as M
from oracle import oracle as O
from tools import simdata
from tests.gpu_common import _singleton_keep, assert_records, knobs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MM2RS = os.path.join(ROOT, "minimap2_rs_amd", "build", "mm2rs")
MM2RS_CPU = os.path.join(ROOT, "oracle", "build", "mm2rs-cpu")
THREADS = 16


def _reads(gbuf, lens, n, L, seed):
    rb, offs, _ = simdata.reads(gbuf, lens, n, L, seed)
    return [rb[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(n)], [f"r{i}" for i in range(n)]


def _map_vs_oracle(dev, idx, oi, mid, names, seqs, tmp_path, tag):
    dev.set_debug(False)
    dev.set_reads(seqs)
    res = dev.map(M.map_opts())
    rec = O.align_records(oi, seqs, mid_occ=mid, threads=THREADS)
    assert_records(res, seqs, rec, tag)
    fa = str(tmp_path / f"{tag}.fa")
    simdata.write_fasta(fa, names, seqs)
    want = str(tmp_path / f"{tag}.paf")
    oi.align_fasta(fa, want, mid_occ=mid)
    assert dev.paf(names, res) == open(want).read()
    return res, rec


def test_c1_cli_mmi_600bp(tmp_path):
    """C1: `mm2rs index -d` then `mm2rs align <.mmi> <read>` (README.md:24-26 flow)
    on the synthetic chr8 + chr12 pair; the .mmi equals the oracle's and the
    PAF line equals the oracle CLI's, from either .mmi."""
    names, lens, gbuf = simdata.genome("chr8chr12", 1.0, 8, threads=THREADS)
    ref = str(tmp_path / "chr8chr12.fa")
    offs = np.concatenate([[0], np.cumsum(lens)])
    simdata.write_fasta(ref, names, [gbuf[offs[i]:offs[i + 1]].tobytes() for i in range(len(names))])
    rng = np.random.default_rng(9)
    chr8 = gbuf[:lens[0]]
    while True:   # an N-free 600 bp window of chr8, forward strand
        st = int(rng.integers(0, lens[0] - 600))
        q = chr8[st:st + 600].tobytes()
        if b"N" not in q.upper():
            break
    qfa = str(tmp_path / "q.fa")
    simdata.write_fasta(qfa, ["q600"], [q])
    gmmi, cmmi = str(tmp_path / "g.mmi"), str(tmp_path / "c.mmi")
    subprocess.run([MM2RS, "index", ref, "-d", gmmi], check=True, capture_output=True)
    subprocess.run([MM2RS_CPU, "index", ref, "-d", cmmi, "-t", str(THREADS)], check=True, capture_output=True)
    assert open(gmmi, "rb").read() == open(cmmi, "rb").read()
    got = subprocess.run([MM2RS, "align", gmmi, qfa], check=True, capture_output=True, text=True).stdout
    want = subprocess.run([MM2RS_CPU, "align", cmmi, qfa], check=True, capture_output=True, text=True).stdout
    assert got == want and got.count("\n") == 1
    f = got.split("\t")
    assert f[0] == "q600" and f[4] == "+" and f[5] == "chr8" and st <= int(f[7]) < int(f[8]) <= st + 600


def test_c2_ecoli_1k_x_10kb(tmp_path):
    """C2: E. coli-shaped 4.64 Mb (ref seed 1) + 1,000 x 10 kb ONT-shaped reads
    (seed 2): every read's PAF line and outcome equal the oracle's."""
    names, lens, gbuf = simdata.genome("ecoli", 1.0, 1, threads=THREADS)
    oi = O.OIndex.build_from_buffer(names, gbuf, lens, threads=THREADS)
    idx = M.Index.build_from_buffer(names, gbuf, lens, threads=THREADS, device=0)
    mid = max(idx.calc_mid_occ(2e-4), 10)
    assert mid == max(oi.mid_occ(2e-4), 10)
    seqs, rn = _reads(gbuf, lens, 1000, 10000, 2)
    dev = M.Device(0)
    dev.upload_index(idx, mid)
    res, rec = _map_vs_oracle(dev, idx, oi, mid, rn, seqs, tmp_path, "c2")
    assert (rec[:, 0] & 1).sum() > 900
    dev.close()


@pytest.fixture(scope="module")
def hg38():
    """The full hg38-shaped reference (ref seed 38), its oracle index and the
    device index built on the GPU."""
    names, lens, gbuf = simdata.genome("hg38", 1.0, 38, threads=THREADS)
    oi = O.OIndex.build_from_buffer(names, gbuf, lens, threads=THREADS)
    idx = M.Index.build_from_buffer(names, gbuf, lens, threads=THREADS, device=0)
    mid = max(oi.mid_occ(2e-4), 10)
    dev = M.Device(0)
    dev.upload_index(idx, 10)
    assert dev.index_mid_occ(2e-4) == oi.mid_occ(2e-4)
    dev.set_mid_occ(mid)
    yield names, lens, gbuf, oi, idx, mid, dev
    dev.close()
    oi.close()
    idx.close()


def test_c3_hg38_300_x_10kb(hg38, tmp_path):
    """C3: 300 x 10 kb reads (seed 3) against the full hg38-shaped index:
    PAF and per-read outcome (incl. Q19 panic reads) equal the oracle's, and
    the first 60 reads' anchors (mm2g_seed_batch) equal build_anchors_filtered."""
    names, lens, gbuf, oi, idx, mid, dev = hg38
    seqs, rn = _reads(gbuf, lens, 300, 10000, 3)
    res, rec = _map_vs_oracle(dev, idx, oi, mid, rn, seqs, tmp_path, "c3")
    assert (rec[:, 0] & 8).sum() > 20 and (rec[:, 0] & 2).sum() >= 1     # panics and rescues are covered
    dev.set_reads(seqs[:60])
    got = dev.seed_batch(M.map_opts())
    for r in range(60):
        want, _ = oi.anchors(seqs[r], 10, 15, mid)
        assert np.array_equal(got[r], want), r


def test_c5_hg38_100kb(hg38, tmp_path):
    """C5: 24 x 100 kb reads (seed 5) plus 8 chimeras of two 50 kb halves
    (rescued: their chains cover half the read): reads with > 65,535 anchors
    (whole-read radix sort) and rescue segments of thousands of anchors
    (k_chain_giant).  PAF and per-read outcome equal the oracle's, by default
    and with every rescue segment over 64 anchors sent to the HBM-scratch
    variant (k_chain_giant<true>); for rescued reads the production DP arrays
    of the rescue pass equal the oracle's chain_dp_all at bw_long on the same
    anchors."""
    names, lens, gbuf, oi, idx, mid, dev = hg38
    seqs, rn = _reads(gbuf, lens, 24, 100000, 5)
    for i in range(8):
        a, b = seqs[i], seqs[8 + i]
        seqs.append(a[:50000] + b[50000:])
        rn.append(f"chim{i}")
    # the rescue pass's full DP arrays (its segment pruning off) against chain_dp_all at bw_long
    with knobs(dev, prune_rescue=0):
        res, rec = _map_vs_oracle(dev, idx, oi, mid, rn, seqs, tmp_path, "c5")
        assert rec[:, 1].max() > 65535
        rescued = [r for r in range(len(seqs)) if res[r].flags & 2]
        assert len(rescued) >= 4
        for r in rescued:
            want, _ = oi.anchors(seqs[r], 10, 15, mid)
            want = want[_singleton_keep(want)]
            got = dev.debug_anchors(r)
            assert np.array_equal(got, want), r
            f, pp, _, _, _ = O.chain_dp(want, 15, bw=20000)
            gf, gpp = dev.debug_dp(r)
            n = len(want)
            assert np.array_equal(gf[:n], f) and np.array_equal(gpp[:n].astype(np.int64), pp), r
        with knobs(dev, giant_lcap=64):
            _map_vs_oracle(dev, idx, oi, mid, rn, seqs, tmp_path, "c5hbm")
            for r in rescued:
                want, _ = oi.anchors(seqs[r], 10, 15, mid)
                want = want[_singleton_keep(want)]
                f, pp, _, _, _ = O.chain_dp(want, 15, bw=20000)
                gf, gpp = dev.debug_dp(r)
                n = len(want)
                assert np.array_equal(gf[:n], f) and np.array_equal(gpp[:n].astype(np.int64), pp), r
    # production defaults (the rescue pass pruned by pass 0's bound): PAF and per-read outcome
    _map_vs_oracle(dev, idx, oi, mid, rn, seqs, tmp_path, "c5prune")
    # the reads over 65535 anchors were seeded by k_sort_big's first pass (counters 21-22) ...
    c = dev.counters()
    assert 0 < c["fused_big_anchors"] <= c["sort_whole_anchors"], c
    # ... and the same with k_seed_write writing their keys
    with knobs(dev, seed_fuse_big=0):
        _map_vs_oracle(dev, idx, oi, mid, rn, seqs, tmp_path, "c5nofuse")
        assert dev.counters()["fused_big_anchors"] == 0
    # pass 0's 100 kb chains with more speculative rounds per block, 8 predecessors per step,
    # and the long reads' candidate segments found by one wave each (cands_longw=0)
    with knobs(dev, spec_rounds=8, spec_batch=8, cands_longw=0):
        _map_vs_oracle(dev, idx, oi, mid, rn, seqs, tmp_path, "c5sr8")


@pytest.mark.parametrize("mc,m", [(1, 15), (0, 0)])
def test_hg38_multi_chain(hg38, tmp_path, mc, m):
    """`-n <= 1 -m <= k` (several chains per read: tp:A:P/S lines, real s2)
    at the C3 and C5 shapes, mm2g_batch_paf's text against the oracle's PAF:
    120 x 10 kb and 12 x 100 kb reads (+ 4 chimeras).  On the full
    hg38-shaped index nearly every read has some chain on an odd rid (the Q19
    pseudo-group), so the reference panics on it and both sides print
    nothing; the same reads against an index of the first contig alone
    (rid 0: no Q19) give the primary and secondary lines."""
    names, lens, gbuf, oi, idx, mid, dev = hg38
    n0 = int(lens[0])
    oi1 = O.OIndex.build_from_buffer(names[:1], gbuf[:n0], lens[:1], threads=THREADS)
    idx1 = M.Index.build_from_buffer(names[:1], gbuf[:n0], lens[:1], threads=THREADS, device=0)
    mid1 = max(idx1.calc_mid_occ(2e-4), 10)
    dev1 = M.Device(0)
    dev1.upload_index(idx1, mid1)
    try:
        for tag, n, L, seed in (("c3", 120, 10000, 3), ("c5", 12, 100000, 5)):
            for one, (d, o, mo, g, ln) in enumerate(((dev, oi, mid, gbuf, lens), (dev1, oi1, mid1, gbuf[:n0], lens[:1]))):
                seqs, rn = _reads(g, ln, n, L, seed)
                if L == 100000:
                    for i in range(4):
                        seqs.append(seqs[i][:50000] + seqs[4 + i][50000:])
                        rn.append(f"chim{i}")
                d.set_debug(False)
                d.set_reads(seqs)
                d.map(M.map_opts(min_cnt=mc, min_chain_score=m))
                got = d.batch_paf(rn)
                fa = str(tmp_path / f"{tag}_{one}_multi.fa")
                simdata.write_fasta(fa, rn, seqs)
                want = str(tmp_path / f"{tag}_{one}_multi_{mc}_{m}.paf")
                o.align_fasta(fa, want, mid_occ=mo, min_cnt=mc, min_chain_score=m)
                want = open(want).read()
                assert got == want, (tag, one, mc, m)
                if one and not (mc <= 0 and L == 100000):   # -n 0 on 100 kb reads: an empty chain always reaches the merge (a panic)
                    assert "tp:A:S" in want and len({ln.split("\t")[0] for ln in want.splitlines()}) > n // 2, (tag, mc, m)
    finally:
        dev1.close()
        oi1.close()
        idx1.close()
