"""GPU: the stage entry points of the C ABI (include/mm2g.h) against the CPU
oracle -- nt4 read input, mm2g_seed_batch (build_anchors_filtered),
mm2g_chain_batch (chain_dp_all / rescue_long_join on caller anchors) -- plus
the workspace re-map and the wide-gap envelope of the sort's singleton filter.
All calls go through libmm2g.so; the oracle is only the checker."""
import os
import random

import numpy as np
import pytest

import minimap2_rs_amd as M
from minimap2_rs_amd._lib import Mm2gError
from oracle import oracle as O
from tests.gpu_common import (_production_vs_oracle, _rand_seq, assert_records, dense_world, knobs,  # noqa: F401
                              small_world)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = M.Device(0)
    yield d
    d.close()


def test_nt4_input_paths_agree(dev, small_world, tmp_path):
    """Reads staged as ASCII (packed by the library) and as caller-packed nt4
    words (mm2g_batch_set_reads_nt4) map to the oracle's PAF, incl. reads with
    N runs, IUPAC codes, lowercase and lengths around the 32/64-base word edges."""
    ref, reads, rnames, rseqs = small_world
    rng = random.Random(17)
    extra = [_rand_seq(rng, n, p_n=pn) for n, pn in ((31, 0.0), (33, 0.1), (64, 0.0), (65, 0.3), (4097, 0.01), (7000, 0.2))]
    extra += [rseqs[3][:2000] + b"NNNNRYKM" + rseqs[3][2000:], rseqs[5].lower()]
    names = list(rnames) + [f"e{i}" for i in range(len(extra))]
    seqs = list(rseqs) + extra
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    mid = max(idx.calc_mid_occ(2e-4), 10)
    dev.upload_index(idx, mid)
    dev.set_debug(False)
    dev.set_reads(seqs)
    res_a = dev.map(M.map_opts())
    paf_a = dev.paf(names, res_a)
    cat = np.frombuffer(b"".join(seqs), np.uint8)
    offs = np.zeros(len(seqs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(s) for s in seqs])
    pk, amb, words = M.nt4_pack(cat, offs, threads=4)
    dev.set_reads_nt4(offs[1:] - offs[:-1], pk, amb, words)
    res_b = dev.map(M.map_opts())
    assert dev.paf(names, res_b) == paf_a
    rec = O.align_records(oi, seqs, mid_occ=mid)
    assert_records(res_a, seqs, rec, "ascii")
    assert_records(res_b, seqs, rec, "nt4")
    fa = str(tmp_path / "r.fa")
    from tools import simdata
    simdata.write_fasta(fa, names, seqs)
    want = str(tmp_path / "want.paf")
    oi.align_fasta(fa, want, mid_occ=mid)
    assert paf_a == open(want).read()
    dev.set_debug(True)


def test_workspace_remap(dev, small_world, dense_world):
    """Minimizer slots, filter tables and anchor workspaces far too small for
    the batch (MM2G_KNOB_WS_MIN): the device flags them, mm2g_batch_results
    grows them and maps again, and every result still equals the oracle's."""
    for ws in (1, 700):
        with knobs(dev, ws_min=ws):
            _production_vs_oracle(dev, small_world, dense_world, tag=f"ws_min {ws}")


def test_workspace_exact_fallback(small_world, dense_world):
    """The up-front anchor reservation fails as if HBM were full
    (MM2G_KNOB_WS_FAIL: keys grabbed at the estimate, then the failure): the
    context frees all five anchor buffers, clears the hipMalloc error, takes
    the batch's exact anchor count and stays in exact-size mode; later batches
    (larger ones grow by the re-map) still equal the oracle."""
    d = M.Device(0)
    try:
        with knobs(d, ws_fail=2):
            _production_vs_oracle(d, small_world, dense_world, tag="ws_fail")
        _production_vs_oracle(d, small_world, dense_world, tag="exact-size mode")
    finally:
        d.close()


@pytest.mark.parametrize("kn", [dict(prune_rescue=0), dict(sketch_view=0), dict(sort_small=1), dict(seg_sparse=0),
                                dict(spec_rounds=1), dict(spec_batch=8), dict(dv_par=0), dict(seed_fuse=0, sketch_x32=0),
                                dict(sort_small=1, spec_rounds=16, sketch_view=300, seg_chunk=128)])
def test_round4_paths_vs_oracle(dev, small_world, dense_world, kn):
    """Production paths, on and off, against the oracle (PAF and per-read
    outcome, small and dense worlds at mid_occ 20 and 5000): the rescue pass's
    pruning by pass 0's bound, query sketch views, every read through
    k_sort_read (sort_small=1), k_chain_seg's sparse items off (seg_sparse=0) and
    over 128-anchor items (their segment-start words cut mid-segment),
    k_chain_long's speculative rounds and step widths, and k_dv's sequential
    walk (dv_par=0) beside its parallel match."""
    with knobs(dev, **kn):
        _production_vs_oracle(dev, small_world, dense_world, tag=str(kn))


def test_sparse_items_taken(dev, small_world, dense_world):
    """Production pass 0 finds most candidate segments from k_chain_lb's
    segment-start bits (k_chain_seg's sparse items read no keys): fewer
    anchors are streamed than enter the DP, and the results equal the oracle's."""
    _production_vs_oracle(dev, small_world, dense_world, tag="sparse")
    c = dev.counters()
    assert c["dp_anchors"] > 0 and c["seg_stream_anchors"] < c["dp_anchors"], c
    # the batch sums (written by the last chain pass's k_seg_items since round 5)
    assert c["minimizers"] >= c["kept_minimizers"] > 0 and c["anchors"] >= c["dp_anchors"], c
    # sort classes (counters 18-20): the filter is on, so the cell path takes the reads above the small class
    assert c["sort_cell_anchors"] > 0 and c["sort_small_anchors"] + c["sort_cell_anchors"] + c["sort_whole_anchors"] <= c["anchors"], c
    with knobs(dev, seg_sparse=0):
        _production_vs_oracle(dev, small_world, dense_world, tag="streamed")
        c = dev.counters()
        assert c["seg_stream_anchors"] == c["dp_anchors"], c


@pytest.mark.parametrize("max_gap,bw_long", [(5000, 40000), (40000, 20000)])
def test_wide_gaps_vs_oracle(dev, small_world, dense_world, max_gap, bw_long):
    """max_dist_x beyond the sort's 32 kb cells (-g 40000, -r 500,40000): the
    singleton filter must step aside (it is exact only for max_dist_x <= 2^15);
    PAF and per-read fields equal the oracle's, also for reads with thousands
    of anchors (dense world at mid_occ 5000)."""
    with knobs(dev, sort_small=1):
        _production_vs_oracle(dev, small_world, dense_world, opts=M.map_opts(max_gap=max_gap, bw_long=bw_long),
                              tag=f"-g {max_gap} -r 500,{bw_long}")
        c = dev.counters()
        # no singleton filter: k_sort_read lists every read above the small class for k_sort_radix
        assert c["sort_cell_anchors"] == 0 and c["sort_whole_anchors"] > 0, c


@pytest.mark.parametrize("max_gap,bw,bw_long", [(5000, 500, 200), (300, 500, 400), (300, 2000, 20000)])
def test_narrow_rescue_vs_oracle(dev, small_world, dense_world, max_gap, bw, bw_long):
    """A rescue pass narrower than pass 0 in some comput_sc limit (-r 500,200:
    bw_long < bw, main.rs:205-206 accepts it; -g below bw: max_dist_x of the
    rescue is max(max_gap, bw_long) < pass 0's max(max_gap, bw)).  Pass 0's best-f
    bound no longer bounds the rescue's DP there, so the rescue pass must not be
    pruned by it; the last case keeps every limit wider and prunes."""
    with knobs(dev, prune_rescue=1):
        _production_vs_oracle(dev, small_world, dense_world, opts=M.map_opts(max_gap=max_gap, bw=bw, bw_long=bw_long),
                              tag=f"-g {max_gap} -r {bw},{bw_long}")


def test_seed_batch_vs_oracle(dev, small_world, dense_world):
    """mm2g_seed_batch = build_anchors_filtered (seeds.rs:42-60) after the
    Align flow's sketch + filter, for every read, at several mid_occ."""
    for world, mids in ((small_world, (None,)), (dense_world, (10, 20, 5000))):
        ref, reads, rnames, rseqs = world
        oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
        idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
        for mid in mids:
            mid = mid if mid is not None else max(idx.calc_mid_occ(2e-4), 10)
            dev.upload_index(idx, mid)
            dev.set_reads(rseqs)
            got = dev.seed_batch(M.map_opts())
            for r, q in enumerate(rseqs):
                want, _ = oi.anchors(q, 10, 15, mid)
                assert np.array_equal(got[r], want), (mid, r, len(got[r]), len(want))
    # the query filter's drop path (seeds.rs:13-36): tandem repeats whose minimizers recur
    # more than max(10, m/100) times in a read, beside reads where none does (k_filter_lds
    # keeps every minimizer without its exact table only when no count can exceed that)
    rng = random.Random(11)
    ref, _, _, rseqs = dense_world
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    dev.upload_index(idx, 5000)
    unit = _rand_seq(rng, 37, p_low=0.0)
    qs = [rseqs[1][:3000] + unit * reps + rseqs[2][:3000] for reps in (5, 12, 30, 60)]
    qs += [unit * 250, _rand_seq(rng, 9000, p_low=0.0) + (b"AC" * 40) * 20]
    dev.set_reads(qs)
    got = dev.seed_batch(M.map_opts())
    dropped = 0
    for r, q in enumerate(qs):
        want, _ = oi.anchors(q, 10, 15, 5000)
        assert np.array_equal(got[r], want), ("repeat", r, len(got[r]), len(want))
        mv = O.sketch(q, 10, 15)
        dropped += int(len(mv) - len(O.filter_minimizers(mv))) if mv is not None and len(mv) else 0
    assert dropped > 0   # the drop path was exercised
    # (w, k) of the opts, not the index's (Q3)
    ref = small_world[0]
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    dev.upload_index(idx, 10)
    dev.set_reads(small_world[3][:20])
    got = dev.seed_batch(M.map_opts(w=7, k=15))
    for r, q in enumerate(small_world[3][:20]):
        want, _ = oi.anchors(q, 7, 15, 10)
        assert np.array_equal(got[r], want)


def test_chain_batch_vs_oracle(dev, small_world, dense_world):
    """mm2g_chain_batch on caller anchors (the oracle's build_anchors_filtered
    output): f, pprev, chains[0] and its score equal chain_dp_all's (lchain.rs:
    59-176) at bw 500 and 20000; with rescue, the per-read chain equals the
    Align flow's after rescue_long_join (lchain.rs:321-330)."""
    for world, mid in ((small_world, None), (dense_world, 5000), (dense_world, 20)):
        ref, reads, rnames, rseqs = world
        oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
        mid = mid if mid is not None else max(oi.mid_occ(2e-4), 10)
        anchors = [oi.anchors(q, 10, 15, mid)[0] for q in rseqs]
        qlens = [len(q) for q in rseqs]
        for bw in (500, 20000):
            p = M.chain_params(15, bw=bw)
            res, chains, fs, pps = dev.chain_batch(anchors, qlens, p, rescue=False, want_dp=True)
            for r, a in enumerate(anchors):
                f, pp, chain, score, _ = O.chain_dp(a, 15, bw=bw)
                assert np.array_equal(fs[r], f) and np.array_equal(pps[r].astype(np.int64), pp), (mid, bw, r)
                if len(a) == 0:
                    assert not (res[r].flags & 1)
                    continue
                assert res[r].flags & 1 and res[r].score == score and np.array_equal(chains[r], chain), (mid, bw, r)
        # Align-flow chain (pass 0 + rescue) vs the oracle's per-read outcome
        res, chains = dev.chain_batch(anchors, qlens, M.chain_params(15), rescue=True)
        rec = O.align_records(oi, rseqs, mid_occ=mid)
        for r in range(len(rseqs)):
            o = rec[r]
            got = (res[r].flags & 11, res[r].n_anchors, res[r].score, res[r].cm, res[r].qs, res[r].qe, res[r].ts, res[r].te,
                   res[r].rid, res[r].rev)
            assert got == tuple(int(v) for v in o[:10]), (mid, r, got, o[:10])


def test_chain_batch_rejects(dev):
    """Outside the envelope the chain entry point refuses instead of guessing."""
    a = np.array([[5 << 32 | 100, 15 << 32 | 10], [5 << 32 | 50, 15 << 32 | 20]], np.uint64)   # unsorted
    with pytest.raises(Mm2gError):
        dev.chain_batch([a], [1000])
    b = np.array([[5 << 32 | 100, 15 << 32 | 10], [5 << 32 | 150, 17 << 32 | 20]], np.uint64)  # two spans
    with pytest.raises(Mm2gError):
        dev.chain_batch([b], [1000])
    with pytest.raises(Mm2gError):
        dev.chain_batch([a[::-1].copy()], [1000], M.chain_params(15, chn_pen_skip=0.5))
    with pytest.raises(Mm2gError):   # -n <= 1 with -m <= span: Rust sort_unstable tie order (DESIGN.md "-n <= 1")
        dev.chain_batch([a[::-1].copy()], [1000], M.chain_params(15, min_cnt=1, min_chain_score=15))
    # -n <= 1 with -m above the span: no backtrack chain can pass, the result is -n 3's
    for mc in (1, 0):
        r1 = dev.chain_batch([a[::-1].copy()], [1000], M.chain_params(15, min_cnt=mc))
        r3 = dev.chain_batch([a[::-1].copy()], [1000], M.chain_params(15))
        assert np.array_equal(r1[1][0], r3[1][0]) and bytes(r1[0][0]) == bytes(r3[0][0])


def test_dv_binary_search_even_k(dev):
    """Even-k reads whose dv depends on the reference's rustc (tests/golden/
    binsearch_even_k.json): the device follows paf.rs:178's binary_search as
    rustc >= 1.82 compiles it."""
    import json
    doc = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "binsearch_even_k.json")))
    for c in doc["cases"]:
        idx = M.Index.build_from_seqs([doc["ref_name"]], [c["ref"].encode()], w=doc["w"], k=doc["k"], b=14, flag=0, threads=2)
        dev.set_debug(False)
        dev.upload_index(idx, 10000)
        dev.set_reads([c["read"].encode()])
        res = dev.map(M.map_opts(w=doc["w"], k=doc["k"]))
        assert dev.paf([doc["read_name"]], res).rstrip("\n") == c["paf_rust_ge_1_82"]
    dev.set_debug(True)
