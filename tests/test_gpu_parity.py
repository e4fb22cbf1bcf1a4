"""GPU parity: every stage of the MI355X path against the CPU oracle, bit-exact.

All calls go through libmm2g.so's C ABI (minimap2_rs_amd wraps it with
ctypes); the oracle is only the checker."""
import contextlib
import os
import random

import numpy as np
import pytest

import minimap2_rs_amd as M
from oracle import oracle as O
from tools import simdata
from tests.gpu_common import (_mutate, _production_vs_oracle, _rand_seq, _singleton_keep, assert_records, dense_world, knobs,  # noqa: F401
                              small_world)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = M.Device(0)
    yield d
    d.close()


def _edge_seqs(rng):
    seqs = [b"A", b"ACGT", b"N" * 50, b"ACGTACGTACGTACGTACGTACGTACGT", b"A" * 300, b"AC" * 200, b"ACGTTGCA" * 80]
    for n in [5, 14, 15, 16, 24, 25, 26, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 2049, 5000]:
        seqs.append(_rand_seq(rng, n, p_n=0.0))
    for n in [200, 3000, 9000]:
        seqs.append(_rand_seq(rng, n, p_n=0.01))
        seqs.append(_rand_seq(rng, n, p_n=0.2))
    s = bytearray(_rand_seq(rng, 6000))
    s[1000:1020] = b"N" * 20
    s[3000:3600] = b"N" * 600
    seqs.append(bytes(s))
    # low complexity / periodic (ties, C-case rescans)
    seqs.append((b"ACGTTA" * 900)[:5000])
    seqs.append(b"".join(rng.choice([b"AAAAAAA", b"CCCC", b"GT", b"TTTTTTTTTT"]) for _ in range(800)))
    return seqs


@pytest.mark.parametrize("w,k", [(10, 15), (10, 19), (11, 21), (5, 16), (3, 4), (1, 1), (1, 2), (50, 7), (255, 28), (7, 28), (2, 10), (64, 12), (65, 13)])
def test_sketch_parity(dev, w, k):
    rng = random.Random(1000 * w + k)
    seqs = _edge_seqs(rng)
    got = dev.sketch_sequences(seqs, w, k, rid=0)
    for i, s in enumerate(seqs):
        want = O.sketch(s, w, k, 0, False)
        g = got[i]
        assert g.shape == want.shape, (i, len(s), g.shape, want.shape)
        assert np.array_equal(g, want), (i, len(s))


@pytest.mark.parametrize("view", [64, 512, 2560])
def test_sketch_views_parity(dev, view):
    """Query sketch views (odd k: reads longer than `view` bases are sketched as
    views of `view` emitting bases after a warm-up, one wave each, then
    concatenated; DESIGN.md "Query sketch views") equal the oracle's
    sketch_sequence, also across N runs, lowercase and periodic stretches at
    view edges; even k keeps the whole-read path."""
    rng = random.Random(77 + view)
    seqs = []
    for i in range(24):
        n = rng.choice([60, 700, 3000, 10000, 31000])
        s = bytearray(_rand_seq(rng, n, p_n=0.002 if i % 3 else 0.0))
        if i % 4 == 1:   # a periodic stretch (ties) and an N run around a view edge
            st = min(len(s) - 1, view - 40) if len(s) > view else 0
            unit = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(1, 6)))
            for j in range(st, min(len(s), st + 300)):
                s[j] = unit[(j - st) % len(unit)]
            for j in range(min(len(s), st + 310), min(len(s), st + 330)):
                s[j] = ord("N")
        seqs.append(bytes(s))
    with knobs(dev, sketch_view=view):
        for w, k in ((10, 15), (5, 11), (19, 19), (1, 3), (255, 21), (3, 16)):
            got = dev.sketch_sequences(seqs, w, k, rid=0)
            for i, s in enumerate(seqs):
                want = O.sketch(s, w, k, 0, False)
                assert np.array_equal(got[i], want), (view, w, k, i, len(s))


@pytest.mark.parametrize("n_reads", [300, 4200])
def test_sketch_views_plan_sizes(dev, n_reads):
    """k_view_plan's two fills: a thread per view from the view offsets in LDS
    (up to 4,096 reads) and a thread per read beyond that; both must give the
    oracle's minimizers for every read (view_reads raised so both batches take views)."""
    rng = random.Random(91 + n_reads)
    seqs = [_rand_seq(rng, rng.choice([40, 64, 65, 200, 513]), p_n=0.003) for _ in range(n_reads)]
    with knobs(dev, sketch_view=64, view_reads=8192):
        got = dev.sketch_sequences(seqs, 10, 15, rid=0)
    for i, s in enumerate(seqs):
        assert np.array_equal(got[i], O.sketch(s, 10, 15, 0, False)), (n_reads, i, len(s))


def test_sketch_rid(dev):
    rng = random.Random(5)
    seqs = [_rand_seq(rng, 3000, p_n=0.01) for _ in range(3)]
    got = dev.sketch_sequences(seqs, 10, 15, rid=7)
    for i, s in enumerate(seqs):
        assert np.array_equal(got[i], O.sketch(s, 10, 15, 7, False))


def _map_nodebug(dev, rnames, rseqs):
    """Map with debug off: the production path, incl. the singleton filter of the sort."""
    dev.set_debug(False)
    dev.set_reads(rseqs)
    res = dev.map(M.map_opts())
    return dev.paf(rnames, res), res


_RES_FIELDS = ("flags", "n_anchors", "score", "cm", "qs", "qe", "ts", "te", "rid", "rev", "n_match", "dv_st", "dv_en",
               "m_dv", "sum_k", "qlen", "dv")


def _dp_diff(gf, gpp, f, pp, want_a):
    bad = np.nonzero((gf != f) | (gpp.astype(np.int64) != pp))[0]
    if len(bad) == 0:
        return ""
    i = int(bad[0])
    lo, hi = max(0, i - 3), min(len(f), i + 3)
    return (f"A={len(f)} first diff at i={i} ({len(bad)} diffs): got f={gf[lo:hi].tolist()} pp={gpp[lo:hi].tolist()} "
            f"want f={f[lo:hi].tolist()} pp={pp[lo:hi].tolist()} key_i={[hex(int(x)) for x in want_a[i]]}")


def test_pipeline_parity(dev, small_world, tmp_path):
    ref, reads, rnames, rseqs = small_world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    mid = max(idx.calc_mid_occ(2e-4), 10)
    assert mid == max(oi.mid_occ(2e-4), 10)
    dev.upload_index(idx, mid)
    dev.set_debug(True)
    dev.set_reads(rseqs)
    res = dev.map(M.map_opts())
    n_checked = 0
    for r, q in enumerate(rseqs):
        want_a, _ = oi.anchors(q, 10, 15, mid)
        got_a = dev.debug_anchors(r)
        assert np.array_equal(got_a, want_a), f"anchors differ for read {r}"
        if len(want_a) == 0:
            assert not (res[r].flags & 1)
            continue
        rescued = bool(res[r].flags & 2)
        f, pp, chain, score, _ = O.chain_dp(want_a, 15, bw=(20000 if rescued else 500))
        gf, gpp = dev.debug_dp(r)
        assert np.array_equal(gf, f) and np.array_equal(gpp.astype(np.int64), pp), \
            f"DP differs for read {r}: " + _dp_diff(gf, gpp, f, pp, want_a)
        n_checked += 1
    assert n_checked > 100
    want_paf = str(tmp_path / "want.paf")
    oi.align_fasta(reads, want_paf)
    got = dev.paf(rnames, res)
    assert got == open(want_paf).read()
    assert _map_nodebug(dev, rnames, rseqs)[0] == got          # production path (singleton filter on)


@pytest.mark.parametrize("mid_occ,sr,sb,se", [(None, 3, 4, 1), (20, 3, 4, 1), (5000, 3, 4, 1), (None, 1, 8, 1), (20, 8, 8, 1),
                                            (5000, 16, 8, 1), (None, 3, 4, 0), (5000, 3, 4, 0)])
def test_lazy_dp_exact(dev, small_world, dense_world, mid_occ, sr, sb, se):
    """The production DP shortcuts keep every f/pprev exact: k_chain_long's
    simple paths (no mark source can break the loop; a chain's maximum visited
    early with a break proven inside the first window) and lazy windows, and
    the giant-segment kernels, here run with the full DP arrays kept (debug
    mode, lazy=2), equal the oracle's chain_dp_all for every read."""
    world = small_world if mid_occ is None else dense_world
    ref, reads, rnames, rseqs = world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    mid = max(idx.calc_mid_occ(2e-4), 10) if mid_occ is None else mid_occ
    dev.upload_index(idx, mid)
    # sr / sb: speculative rounds of k_chain_long per 64-anchor block and predecessors per step;
    # se: next-round guesses evaluated along the round's predecessor choices (1) or taken as computed
    with knobs(dev, lazy=2, giant_min=64, spec_rounds=sr, spec_batch=sb, spec_eval=se):
        dev.set_debug(True)
        dev.set_reads(rseqs)
        res = dev.map(M.map_opts())
        n = 0
        for r, q in enumerate(rseqs):
            want_a, _ = oi.anchors(q, 10, 15, mid)
            if len(want_a) == 0:
                continue
            rescued = bool(res[r].flags & 2)
            f, pp, chain, score, _ = O.chain_dp(want_a, 15, bw=(20000 if rescued else 500))
            gf, gpp = dev.debug_dp(r)
            assert np.array_equal(gf, f) and np.array_equal(gpp.astype(np.int64), pp), \
                f"DP differs for read {r} (rescued={rescued}): " + _dp_diff(gf, gpp, f, pp, want_a)
            n += 1
        assert n >= len(rseqs) // 2
    dev.set_debug(False)


def test_pipeline_determinism(dev, small_world):
    ref, reads, rnames, rseqs = small_world
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    p1 = M.align(idx, rnames, rseqs, dev=dev)
    p2 = M.align(idx, rnames, rseqs, dev=dev)
    assert p1 == p2 and p1.count("\n") > 50


@pytest.mark.parametrize("mid_occ", [20, 5000])
def test_pipeline_parity_dense(dev, dense_world, tmp_path, mid_occ):
    ref, reads, rnames, rseqs = dense_world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    dev.upload_index(idx, mid_occ)
    dev.set_debug(True)
    dev.set_reads(rseqs)
    res = dev.map(M.map_opts())
    dbg_pairs = dev.counters()["dp_pairs"]      # debug mode: full DP, no segment pruning
    deep = 0
    for r, q in enumerate(rseqs):
        want_a, _ = oi.anchors(q, 10, 15, mid_occ)
        got_a = dev.debug_anchors(r)
        assert np.array_equal(got_a, want_a), f"anchors differ for read {r}"
        if len(want_a) == 0:
            continue
        rescued = bool(res[r].flags & 2)
        f, pp, chain, score, _ = O.chain_dp(want_a, 15, bw=(20000 if rescued else 500))
        gf, gpp = dev.debug_dp(r)
        assert np.array_equal(gf, f) and np.array_equal(gpp.astype(np.int64), pp), \
            f"DP differs for read {r} (rescued={rescued}): " + _dp_diff(gf, gpp, f, pp, want_a)
        deep += int(len(want_a) > 2000)
    if mid_occ == 5000:
        assert deep >= 4
    want_paf = str(tmp_path / "want.paf")
    _, counts, _ = oi.align_fasta(reads, want_paf, mid_occ=mid_occ)
    assert dev.paf(rnames, res) == open(want_paf).read()
    assert _map_nodebug(dev, rnames, rseqs)[0] == open(want_paf).read()
    dev.set_debug(True)
    # the DP pair counter equals the reference's inner-loop iterations when every segment is run
    assert dbg_pairs == counts["inner_iters"]


@pytest.mark.parametrize("small_reg", [1, 0])
def test_anchor_sort_many_shapes(dev, dense_world, small_reg):
    """Sorted anchors equal the oracle's for reads whose buckets take every
    path of the per-read sort (single keys, <= 8, <= 64, <= 512, block radix),
    with k_sort_small's register bitonic (reads of 257..4096 anchors, 512..4096
    padded) or its LDS-only network."""
    ref, reads, rnames, rseqs = dense_world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
    rng = random.Random(9)
    qs = list(rseqs) + [rseqs[0] * 3, rseqs[8] + rseqs[16], _rand_seq(rng, 20000)]
    qs += [rseqs[i][: 300 * (i + 1)] for i in range(12)]          # prefixes: anchor counts across the padded sizes
    with knobs(dev, small_reg=small_reg):
        for mid_occ in (10, 100000):
            dev.upload_index(idx, mid_occ)
            dev.set_debug(True)
            dev.set_reads(qs)
            dev.map(M.map_opts())
            sizes = set()
            for r, q in enumerate(qs):
                want_a, _ = oi.anchors(q, 10, 15, mid_occ)
                sizes.add(len(want_a))
                assert np.array_equal(dev.debug_anchors(r), want_a), (mid_occ, r, len(want_a))
            assert any(256 < n <= 4096 for n in sizes), sorted(sizes)


def test_golden_world_gpu(dev, tmp_path):
    """The committed fixtures (pure-Python restatement, tests/golden) on the GPU:
    anchors, DP arrays and PAF lines."""
    import json
    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "world.json")))
    ref = str(tmp_path / "ref.fa")
    simdata.write_fasta(ref, [c[0] for c in gold["contigs"]], [c[1].encode() for c in gold["contigs"]])
    idx = M.Index.build_index_from_fasta(ref, gold["w"], gold["k"], gold["b"], 0, 2)
    dev.upload_index(idx, gold["mid_occ"])
    dev.set_debug(True)
    seqs = [r["seq"].encode() for r in gold["reads"]]
    dev.set_reads(seqs)
    res = dev.map(M.map_opts())
    for i, r in enumerate(gold["reads"]):
        assert dev.debug_anchors(i).reshape(-1).tolist() == [v for xy in r["anchors"] for v in xy], r["name"]
        if r["anchors"] and not r["rescued"]:
            f, pp = dev.debug_dp(i)
            assert f.tolist() == r["f"] and pp.tolist() == r["pprev"], r["name"]
        assert bool(res[i].flags & 8) == r["panic"], r["name"]
        assert bool(res[i].flags & 2) == r["rescued"], r["name"]
    got = dev.paf([r["name"] for r in gold["reads"]], res).splitlines()
    assert got == [r["paf"] for r in gold["reads"] if r["paf"]]
    assert _map_nodebug(dev, [r["name"] for r in gold["reads"]], seqs)[0].splitlines() == got
    dev.set_debug(True)


def test_singleton_filter_vs_oracle(dev, small_world, dense_world):
    """Production path with every read through k_sort_read (the filtering
    sort): PAF and every per-read field equal the oracle's (dropped anchors
    only ever form one-anchor segments; the largest dropped key settles
    f == span ties)."""
    with knobs(dev, sort_small=1):
        _production_vs_oracle(dev, small_world, dense_world)


def test_cli_align_gpu(small_world, tmp_path):
    """`mm2rs align` (GPU) prints the oracle CLI's lines for every read."""
    import subprocess
    ref, reads, rnames, rseqs = small_world
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mm2rs = os.path.join(root, "minimap2_rs_amd", "build", "mm2rs")
    cpu = os.path.join(root, "oracle", "build", "mm2rs-cpu")
    mmi = str(tmp_path / "ref.mmi")
    subprocess.run([mm2rs, "index", ref, "-d", mmi], check=True, capture_output=True)
    g = subprocess.run([mm2rs, "align", mmi, reads], check=True, capture_output=True, text=True).stdout
    c = subprocess.run([cpu, "align", ref, reads], check=True, capture_output=True, text=True).stdout
    assert g == c and g.count("\n") > 50


def test_cli_align_min_cnt(small_world, dense_world, tmp_path):
    """`mm2rs align -n 1` / `-n 0` / `-n -1` with -m above k (the default 40,
    and 16): byte-identical to the oracle CLI with the same flags -- the
    backtrack yields one-anchor chains scored <= k, so none passes and the
    fallback path runs (DESIGN.md "-n <= 1").  -m <= k: test_multi_chain_*."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mm2rs = os.path.join(root, "minimap2_rs_amd", "build", "mm2rs")
    cpu = os.path.join(root, "oracle", "build", "mm2rs-cpu")
    for wi, world in enumerate((small_world, dense_world)):
        ref, reads, rnames, rseqs = world
        mmi = str(tmp_path / f"ref{wi}.mmi")
        subprocess.run([mm2rs, "index", ref, "-d", mmi], check=True, capture_output=True)
        for flags in (["-n", "1"], ["-n", "0"], ["-n", "-1", "-m", "16"]):
            g = subprocess.run([mm2rs, "align", mmi, reads] + flags, check=True, capture_output=True, text=True).stdout
            c = subprocess.run([cpu, "align", ref, reads] + flags, check=True, capture_output=True, text=True).stdout
            c3 = subprocess.run([cpu, "align", ref, reads], check=True, capture_output=True, text=True).stdout
            assert g == c == c3 and g.count("\n") > 10, flags


def test_cli_multi_chain(small_world, dense_world, tmp_path):
    """`mm2rs align -n 1 -m 15` (and -n 0 -m 0, -n -1 -m 8): several chains per
    read reach the output (tp:A:P / tp:A:S, s2) through the backtrack, merge
    and selection of lchain.rs:92-160,237-314 -- byte-identical to the oracle
    CLI under the restated rustc 1.81+ sort_unstable (DESIGN.md "-n <= 1")."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mm2rs = os.path.join(root, "minimap2_rs_amd", "build", "mm2rs")
    cpu = os.path.join(root, "oracle", "build", "mm2rs-cpu")
    for wi, world in enumerate((small_world, dense_world)):
        ref, reads, rnames, rseqs = world
        mmi = str(tmp_path / f"ref{wi}.mmi")
        subprocess.run([mm2rs, "index", ref, "-d", mmi], check=True, capture_output=True)
        for flags in (["-n", "1", "-m", "15"], ["-n", "0", "-m", "0"], ["-n", "-1", "-m", "8", "-N", "2"]):
            g = subprocess.run([mm2rs, "align", mmi, reads] + flags, check=True, capture_output=True, text=True).stdout
            c = subprocess.run([cpu, "align", ref, reads] + flags, check=True, capture_output=True, text=True).stdout
            assert g == c, (wi, flags)
            assert "tp:A:S" in g, (wi, flags)


@pytest.mark.parametrize("mc,m", [(1, 15), (0, 0), (-1, 8), (1, 1)])
def test_multi_chain_vs_oracle(dev, small_world, dense_world, mc, m):
    """-n <= 1 with -m <= k through the library (api.align -> mm2g_batch_paf):
    the PAF text, several lines per read, equals the oracle's on the small and
    dense worlds (mid_occ 20 and 5000)."""
    for world, mid in ((small_world, None), (dense_world, 5000), (dense_world, 20)):
        ref, reads, rnames, rseqs = world
        oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
        idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
        mid = mid if mid is not None else max(idx.calc_mid_occ(2e-4), 10)
        dev.upload_index(idx, mid)
        dev.set_debug(False)
        dev.set_reads(rseqs)
        dev.map(M.map_opts(min_cnt=mc, min_chain_score=m))
        got = dev.batch_paf(rnames)
        want_paf = os.path.join(os.path.dirname(reads), f"want_multi_{mid}_{mc}_{m}.paf")
        oi.align_fasta(reads, want_paf, mid_occ=mid, min_cnt=mc, min_chain_score=m)
        want = open(want_paf).read()
        assert got == want, (mid, mc, m)
        assert want.count("\n") > len({ln.split("\t")[0] for ln in want.splitlines()})
    dev.set_debug(True)


@pytest.mark.parametrize("seg_small,lds_kb,big_wnd", [(1024, 0, 126), (64, 0, 126), (8, 0, 126), (1, 0, 126), (1024, 76, 126),
                                                     (8, 76, 126), (1024, 0, 0), (1024, 0, 2)])
def test_filtered_sort_parity(dev, small_world, dense_world, seg_small, lds_kb, big_wnd):
    """Production sort (cell buckets + per-segment ranking, singleton filter
    on): the anchors the DP runs on equal the oracle's sorted anchors minus
    the singletons, for every path -- thread-ranked small segments, block-
    ranked and radix-sorted big ones, the whole-read radix when too many big
    segments (seg_small 1) or too many anchors (> 65535) appear.  lds_kb 76:
    the 512-thread, two-per-CU k_sort_read (smaller windows, more of them).
    big_wnd: k_sort_big's bucket pass appends to at most that many windows
    (0: the per-key scatter; 2: reads with more windows fall back to it)."""
    with knobs(dev, sort_small=1, seg_small=seg_small, sort_lds_kb=lds_kb, big_wnd=big_wnd):
        rng = random.Random(5)
        for world, mids in ((small_world, (None,)), (dense_world, (20, 5000, 100000))):
            ref, reads, rnames, rseqs = world
            qs = list(rseqs)
            if world is dense_world:
                qs += [rseqs[0] * 3, rseqs[8] + rseqs[16], _rand_seq(rng, 20000)]
            oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
            idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
            for mid in mids:
                mid = mid if mid is not None else max(idx.calc_mid_occ(2e-4), 10)
                dev.upload_index(idx, mid)
                dev.set_debug(False)
                dev.set_reads(qs)
                dev.map(M.map_opts())
                for r, q in enumerate(qs):
                    want, _ = oi.anchors(q, 10, 15, mid)
                    if len(want) > 1:
                        want = want[_singleton_keep(want)]
                    got = dev.debug_anchors(r)
                    assert np.array_equal(got, want), (seg_small, mid, r, len(got), len(want))
    dev.set_debug(True)


@pytest.mark.parametrize("chunk", [64, 192])
def test_chunked_chain_items(dev, small_world, dense_world, tmp_path, chunk):
    """Reads cut into many small work items (a wave per chunk, each finishing
    the segment open at its end; the lower bound restarting per chunk): DP
    arrays (debug) and PAF (production, pruning on) still equal the oracle's."""
    with knobs(dev, seg_chunk=chunk):
        for world, mid in ((small_world, None), (dense_world, 5000), (dense_world, 20)):
            ref, reads, rnames, rseqs = world
            oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
            idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
            mid = mid if mid is not None else max(idx.calc_mid_occ(2e-4), 10)
            dev.upload_index(idx, mid)
            dev.set_debug(True)
            dev.set_reads(rseqs)
            res = dev.map(M.map_opts())
            for r, q in enumerate(rseqs):
                want_a, _ = oi.anchors(q, 10, 15, mid)
                if len(want_a) == 0:
                    continue
                rescued = bool(res[r].flags & 2)
                f, pp, _, _, _ = O.chain_dp(want_a, 15, bw=(20000 if rescued else 500))
                gf, gpp = dev.debug_dp(r)
                assert np.array_equal(gf, f) and np.array_equal(gpp.astype(np.int64), pp), \
                    f"chunk {chunk}: DP differs for read {r}: " + _dp_diff(gf, gpp, f, pp, want_a)
            want_paf = str(tmp_path / "want.paf")
            oi.align_fasta(reads, want_paf, mid_occ=mid)
            want = open(want_paf).read()
            assert dev.paf(rnames, res) == want
            assert _map_nodebug(dev, rnames, rseqs)[0] == want
    dev.set_debug(True)


def _mmi_bytes(idx, path):
    idx.save_to_mmi(path)
    return open(path, "rb").read()


@pytest.mark.parametrize("chunk,sortv", [(None, 0), (4096, 1), (300, 0)])
def test_gpu_index_build(tmp_path, chunk, sortv):
    """GPU index build (sketch views, pair sort, bucket distribution, packed S)
    equals the oracle's build_index_from_fasta + save_to_mmi (index.rs:74-109,
    233-307) byte for byte (.mmi), with stats and calc_mid_occ (index.rs:
    111-141), on an hg38-shaped and an E. coli-shaped genome plus edge contigs:
    N runs across view boundaries, lowercase, contigs shorter than k, empty
    contigs; even k (symmetric k-mers) with palindromic runs ((AT)n, (ACGT)n,
    (TA)n in lowercase) that span view boundaries, so the per-view warm-up has
    to grow past its default; HPC (flag 1: TinyQueue spans, sketch.rs:51-64)
    with homopolymer runs up to 400 bases (spans >= 256 give no info).  The build must run on the device
    (MM2G_IKNOB_GPU_STRICT: no host fallback).  The product's host build must
    agree as well.  The device pair sort is the hand-written radix; sortv=1 forces its
    stable value pass too (otherwise only taken when the pairs arrive out of value
    order), and w/k with over a quarter minimizer per base ((3, 2), (2, 3)) outgrow
    the first per-view slots, so the sketch re-runs with exact slots."""
    rng = random.Random(11)
    names, lens, gbuf = simdata.genome("hg38", 0.0006, 5)
    seqs = [gbuf[int(o):int(o + l)].tobytes() for o, l in zip(np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)]
    e_names, e_lens, e_buf = simdata.genome("ecoli", 0.2, 1)
    seqs.append(e_buf.tobytes()); names.append("ecoli")
    s = bytearray(_rand_seq(rng, 20000))
    for st_ in (4096 - 40, 8192 - 3, 12000):
        s[st_:st_ + 60] = b"N" * 60
    seqs += [bytes(s), _rand_seq(rng, 9000, p_low=0.3), b"ACGTACGT", b"", _rand_seq(rng, 15, p_n=0.0), b"N" * 500 + _rand_seq(rng, 3000)]
    names += ["nruns", "lower", "short", "empty", "k15", "leadingN"]
    pal = bytearray(_rand_seq(rng, 1000))
    for unit, n in ((b"AT", 700), (b"ACGT", 350), (b"ta", 2200), (b"GC", 90)):
        pal += unit * n + _rand_seq(rng, rng.randrange(200, 900))
    pal += b"AT" * 5000                      # ends inside a palindromic run
    seqs.append(bytes(pal)); names.append("palindromes")
    # HPC spans: homopolymer runs of 2-400 bases (>= 256: no info), across view
    # boundaries, broken by N, in lowercase, and at the contig end
    hp = bytearray(_rand_seq(rng, 500))
    for _ in range(60):
        c = rng.choice(b"ACGTacgt")
        hp += bytes([c]) * rng.choice((2, 3, 5, 9, 17, 40, 120, 255, 256, 257, 400))
        if rng.random() < 0.2:
            hp += b"N" * rng.randrange(1, 4) + bytes([c]) * rng.randrange(1, 30)
        hp += _rand_seq(rng, rng.randrange(5, 300))
    hp += b"G" * 300
    seqs.append(bytes(hp)); names.append("homopolymers")
    M.set_index_knob("ixchunk", chunk or 0)
    M.set_index_knob("gpu_strict", 1)
    M.set_index_knob("ixsortv", sortv)
    try:
        buf = np.frombuffer(b"".join(seqs), dtype=np.uint8)
        lv = np.array([len(x) for x in seqs], dtype=np.uint64)
        for w, k, fl in ((10, 15, 0), (5, 11, 0), (19, 19, 0), (10, 27, 0), (10, 16, 0), (7, 8, 0), (12, 28, 0), (3, 2, 0),
                         (10, 15, 1), (5, 12, 1), (19, 19, 1), (12, 28, 1), (2, 3, 1)):
            oi = O.OIndex.build_from_buffer(names, buf, lv, w=w, k=k, b=14, flag=fl, threads=4)
            ig = M.Index.build_from_buffer(names, buf, lv, w=w, k=k, b=14, flag=fl, threads=4, device=0)
            ih = M.Index.build_from_seqs(names, seqs, w=w, k=k, b=14, flag=fl, threads=4)
            assert ig.stats() == oi.stats() == ih.stats(), (w, k, fl)
            assert ig.origin == ("gpu build", None) and ih.origin == ("host build", None)
            for fr in (2e-4, 0.01, 0.5):
                assert ig.calc_mid_occ(fr) == oi.mid_occ(fr) == ih.calc_mid_occ(fr)
            oi.save_mmi(str(tmp_path / "o.mmi"))
            want = open(str(tmp_path / "o.mmi"), "rb").read()
            assert _mmi_bytes(ig, str(tmp_path / "g.mmi")) == want, (w, k, fl)
            assert _mmi_bytes(ih, str(tmp_path / "h.mmi")) == want, (w, k, fl)
    finally:
        M.set_index_knob("ixchunk", 0)
        M.set_index_knob("gpu_strict", 0)
        M.set_index_knob("ixsortv", 0)


def test_cli_align_devices(small_world, tmp_path):
    """`mm2rs align --devices 0,0[,0]`: one index copy per listed device
    (uploaded in parallel), reads pulled from one queue by every device's
    contexts, PAF written in input order -- byte-identical to the oracle CLI
    (the multi-GPU drop-in; one GPU here, so the device repeats)."""
    import subprocess
    ref, reads, rnames, rseqs = small_world
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mm2rs = os.path.join(root, "minimap2_rs_amd", "build", "mm2rs")
    cpu = os.path.join(root, "oracle", "build", "mm2rs-cpu")
    mmi = str(tmp_path / "ref.mmi")
    subprocess.run([mm2rs, "index", ref, "-d", mmi], check=True, capture_output=True)
    want = subprocess.run([cpu, "align", ref, reads], check=True, capture_output=True, text=True).stdout
    for devs, streams in (("0,0", "2"), ("0,0,0", "1")):
        got = subprocess.run([mm2rs, "align", mmi, reads, "--devices", devs, "--streams", streams, "--batch-bases", "15000"],
                             check=True, capture_output=True, text=True).stdout
        assert got == want and want.count("\n") > 50, devs
    bad = subprocess.run([mm2rs, "align", mmi, reads, "--devices", "0,99"], capture_output=True, text=True)
    assert bad.returncode != 0 and "out of range" in bad.stderr


def test_cli_streaming_fastq(small_world, tmp_path):
    """`mm2rs align` streams: many small batches over 3 contexts (out-of-order
    completion, in-order output) and FASTQ input give the oracle CLI's lines."""
    import subprocess
    ref, reads, rnames, rseqs = small_world
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mm2rs = os.path.join(root, "minimap2_rs_amd", "build", "mm2rs")
    cpu = os.path.join(root, "oracle", "build", "mm2rs-cpu")
    want = subprocess.run([cpu, "align", ref, reads], check=True, capture_output=True, text=True).stdout
    got = subprocess.run([mm2rs, "align", ref, reads, "--streams", "3", "--batch-bases", "20000"], check=True,
                         capture_output=True, text=True).stdout
    assert got == want and want.count("\n") > 50
    fq = str(tmp_path / "reads.fq")
    with open(fq, "w") as fh:
        for n, s in zip(rnames, rseqs):
            fh.write(f"@{n} extra\n{s.decode()}\n+\n{'I' * len(s)}\n")
    got = subprocess.run([mm2rs, "align", ref, fq, "--batch-bases", "50000"], check=True, capture_output=True, text=True).stdout
    assert got == want


def test_cli_anchors_chain(small_world, tmp_path):
    """`mm2rs anchors` / `mm2rs chain` (main.rs:160-186) on the first read, against
    the oracle's build_anchors_filtered and chain_dp (bw from -r, no rescue)."""
    import subprocess
    ref, reads, rnames, rseqs = small_world
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mm2rs = os.path.join(root, "minimap2_rs_amd", "build", "mm2rs")
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    mid = max(oi.mid_occ(2e-4), 10)
    a, _ = oi.anchors(rseqs[0], 10, 15, mid)
    want = f"anchors: {len(a)}\n" + "".join(f"x=0x{int(x):016x} y=0x{int(y):016x}\n" for x, y in a[:10])
    got = subprocess.run([mm2rs, "anchors", ref, reads], check=True, capture_output=True, text=True).stdout
    assert got == want
    for bw in (5000, 500):
        _, _, chain, _, _ = O.chain_dp(a, 15, max_gap=5000, bw=bw)
        want = f"best_chain_len: {len(chain)}\n"
        if len(chain):
            s, e = a[chain[0]], a[chain[-1]]
            want += f"start: x=0x{int(s[0]):016x} y=0x{int(s[1]):016x}\nend:   x=0x{int(e[0]):016x} y=0x{int(e[1]):016x}\n"
        args = [mm2rs, "chain", ref, reads] + ([] if bw == 5000 else ["-r", str(bw)])
        got = subprocess.run(args, check=True, capture_output=True, text=True).stdout
        assert got == want, bw


@pytest.mark.parametrize("giant_min,giant_min0,lcap", [(16, 0, 0), (200, 0, 0), (16, 0, 64), (16, 16, 0), (16, 16, 64)])
def test_giant_segments(dev, small_world, dense_world, giant_min, giant_min0, lcap):
    """Long segments through k_chain_giant (policy iteration to the fixed point
    of the no-break DP, the reference loop verified wherever a window holds
    more than max_skip mark sources, k_chain_long when it does not settle),
    in the rescue pass and (giant_min0) pass 0's exact mode: PAF and every
    per-read field equal the oracle's.  lcap 64 sends every segment over 64
    anchors to the HBM-scratch variant (k_chain_giant<true>)."""
    with knobs(dev, giant_min=giant_min, giant_min0=giant_min0, giant_lcap=lcap):
        _production_vs_oracle(dev, small_world, dense_world, tag=f"giant {giant_min}/{giant_min0}/{lcap}")


@pytest.mark.parametrize("bins", [4096, 2, 3, 64])
def test_device_mid_occ(dev, small_world, dense_world, bins):
    """calc_mid_occ (index.rs:124-141) from the device table's count histogram
    equals the oracle's sort of all counts, at quantiles inside the histogram
    and in its overflow (few bins force the gathered-overflow path)."""
    with knobs(dev, midhist_bins=bins):
        for ref in (small_world[0], dense_world[0]):
            oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
            idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
            dev.upload_index(idx, 10)
            for fr in (0.0, 2e-4, 1e-3, 0.01, 0.1, 0.5, 0.9, 1.0, 1.5, -0.25):
                assert dev.index_mid_occ(fr) == oi.mid_occ(fr), (ref, fr)
    dev.set_mid_occ(10)
