"""CPU: the C++ oracle (and the product's host-side index) against the golden
fixtures written by tests/golden/make_golden.py from the independent
pure-Python restatement tests/pyref.py.

The reference has no tests of its own and cannot be built here (SURVEY.md
§8c), so these fixtures are the pin: two separately written readings of the
Rust sources must agree bit for bit before the oracle is trusted as the GPU
checker.  PAF lines of reads whose chain lies on an odd rid are absent: the
reference panics there."""
import json
import os
import tempfile

import numpy as np
import pytest

import minimap2_rs_amd as M
from oracle import oracle as O

import pyref as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def sf():
    with open(os.path.join(GOLD, "sketch_filter.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def world(tmp_path_factory):
    with open(os.path.join(GOLD, "world.json")) as fh:
        w = json.load(fh)
    td = tmp_path_factory.mktemp("gold")
    ref = str(td / "ref.fa")
    with open(ref, "w") as fh:
        for n, s in w["contigs"]:
            fh.write(f">{n}\n{s}\n")
    reads = str(td / "reads.fa")
    with open(reads, "w") as fh:
        for r in w["reads"]:
            fh.write(f">{r['name']}\n{r['seq']}\n")
    w["ref_path"], w["reads_path"] = ref, reads
    return w


def test_oracle_sketch(sf):
    for c in sf["sketch"]:
        got = O.sketch(c["seq"].encode(), c["w"], c["k"], c["rid"], c["hpc"])
        want = np.array(c["out"], dtype=np.uint64).reshape(-1, 2)
        assert np.array_equal(got.reshape(-1, 2), want), (c["w"], c["k"], c["hpc"], len(c["seq"]))


def test_oracle_filter(sf):
    for c in sf["filter"]:
        got = O.filter_minimizers(np.array(c["mv"], dtype=np.uint64).reshape(-1, 2))
        assert np.array_equal(got.reshape(-1, 2), np.array(c["out"], dtype=np.uint64).reshape(-1, 2))


def test_pyref_reproduces_fixtures(sf):
    """Guards the generator against drift (a subset: pure Python is slow)."""
    for c in sf["sketch"][::7]:
        assert [list(x) for x in R.sketch_sequence(c["seq"].encode(), c["w"], c["k"], c["rid"], c["hpc"])] == c["out"]


def test_oracle_index(world):
    oi = O.OIndex.build(world["ref_path"], world["w"], world["k"], world["b"], 0, 2)
    for fr, want in world["calc_mid_occ"].items():
        assert oi.mid_occ(float(fr)) == want, fr
    assert oi.stats()[0] == world["n_keys"]
    for g in world["gets"]:
        got = oi.get(g["key"])
        if g["kind"] == 0:
            assert got is None
        elif g["kind"] == 1:
            assert got == ("Single", g["pos"][0])
        else:
            assert got == ("Multi", g["pos"])


def test_oracle_anchors_dp_paf(world, tmp_path):
    oi = O.OIndex.build(world["ref_path"], world["w"], world["k"], world["b"], 0, 2)
    mid = world["mid_occ"]
    for r in world["reads"]:
        a, _ = oi.anchors(r["seq"].encode(), world["w"], world["k"], mid)
        assert np.array_equal(a.reshape(-1, 2), np.array(r["anchors"], dtype=np.uint64).reshape(-1, 2)), r["name"]
        if not r["anchors"]:
            continue
        f, pp, chain, score, _ = O.chain_dp(a, world["k"])
        assert f.tolist() == r["f"] and pp.tolist() == r["pprev"], r["name"]
        assert chain.tolist() == r["chain"] and score == r["score"], r["name"]
    out = str(tmp_path / "o.paf")
    _, counts, _ = oi.align_fasta(world["reads_path"], out, mid_occ=mid)
    want = [r["paf"] for r in world["reads"] if r["paf"]]
    assert open(out).read().splitlines() == want
    assert counts["panics"] == sum(r["panic"] for r in world["reads"])
    assert counts["rescued_anchors"] == sum(len(r["anchors"]) for r in world["reads"] if r["rescued"])


def test_host_index_matches_oracle(world, tmp_path):
    """The product's host index (libmm2g.so host code; no GPU needed) against
    the oracle: stats, calc_mid_occ, Index::get and byte-identical .mmi."""
    idx = M.Index.build_index_from_fasta(world["ref_path"], world["w"], world["k"], world["b"], 0, 2)
    oi = O.OIndex.build(world["ref_path"], world["w"], world["k"], world["b"], 0, 2)
    assert idx.stats()[0] == world["n_keys"]
    assert tuple(idx.stats()) == tuple(oi.stats())
    for fr, want in world["calc_mid_occ"].items():
        assert idx.calc_mid_occ(float(fr)) == want
    for g in world["gets"]:
        got = idx.get(g["key"])
        exp = None if g["kind"] == 0 else (("Single", g["pos"][0]) if g["kind"] == 1 else ("Multi", g["pos"]))
        assert got == exp
    p1, p2 = str(tmp_path / "p.mmi"), str(tmp_path / "o.mmi")
    idx.save_to_mmi(p1)
    oi.save_mmi(p2)
    assert open(p1, "rb").read() == open(p2, "rb").read()
    back = M.Index.load_from_mmi(p1)
    assert tuple(back.stats()) == tuple(idx.stats())
    assert back.params == idx.params
    for g in world["gets"][:50]:
        assert back.get(g["key"]) == idx.get(g["key"])


@pytest.mark.parametrize("w,k,flag", [(10, 15, 0), (5, 11, 1), (19, 19, 0)])
def test_host_index_params(world, tmp_path, w, k, flag):
    """HPC and other (w, k): product host index == oracle, byte for byte."""
    idx = M.Index.build_index_from_fasta(world["ref_path"], w, k, 12, flag, 3)
    oi = O.OIndex.build(world["ref_path"], w, k, 12, flag, 3)
    p1, p2 = str(tmp_path / "p.mmi"), str(tmp_path / "o.mmi")
    idx.save_to_mmi(p1)
    oi.save_mmi(p2)
    assert open(p1, "rb").read() == open(p2, "rb").read()
    assert idx.calc_mid_occ(2e-4) == oi.mid_occ(2e-4)


def _mmi_rewrite(src: bytes, fn) -> bytes:
    """Re-emit an .mmi (index.rs:233-307 layout) with each bucket's hash
    table passed through fn(list of (key, val)) -> list."""
    import struct
    o = 4
    w, k, b, n_seq, flag = struct.unpack_from("<5I", src, o); o += 20
    for _ in range(n_seq):
        nl = src[o]; o += 1 + nl + 4
    out = bytearray(src[:o])
    for _ in range(1 << b):
        (n,) = struct.unpack_from("<I", src, o)
        out += src[o:o + 4 + 8 * n]; o += 4 + 8 * n
        (sz,) = struct.unpack_from("<I", src, o); o += 4
        ents = [struct.unpack_from("<QQ", src, o + 16 * j) for j in range(sz)]
        o += 16 * sz
        ents = fn(ents)
        out += struct.pack("<I", len(ents))
        for e in ents:
            out += struct.pack("<QQ", *e)
    out += src[o:]
    return bytes(out)


def test_mmi_load_mapped_parallel(world, tmp_path, monkeypatch):
    """load_from_mmi (index.rs:361-424) via the mapped, bucket-parallel loader:
    HashMap iteration order in the file does not matter, a later duplicate key
    overwrites an earlier one (HashMap::insert), any thread count gives the
    same index, and every truncation is an MM2G_E_IO error."""
    idx = M.Index.build_index_from_fasta(world["ref_path"], world["w"], world["k"], world["b"], 0, 2)
    p = str(tmp_path / "a.mmi")
    idx.save_to_mmi(p)
    raw = open(p, "rb").read()
    rev = tmp_path / "rev.mmi"
    rev.write_bytes(_mmi_rewrite(raw, lambda e: e[::-1]))
    # duplicate: the first entry of each table again, with a bogus value first
    dup = tmp_path / "dup.mmi"
    dup.write_bytes(_mmi_rewrite(raw, lambda e: ([(e[0][0], 1 | 0)] + e) if e and (e[0][0] & 1) else e))
    want = [idx.get(g["key"]) for g in world["gets"]]
    for path in (p, str(rev), str(dup)):
        for thr in (1, 5):
            M.set_index_knob("load_threads", thr)
            back = M.Index.load_from_mmi(path)
            assert tuple(back.stats()) == tuple(idx.stats())
            assert [back.get(g["key"]) for g in world["gets"]] == want
            for fr, mo in world["calc_mid_occ"].items():
                assert back.calc_mid_occ(float(fr)) == mo
            q = str(tmp_path / "re.mmi")
            back.save_to_mmi(q)
            assert open(q, "rb").read() == raw
    M.set_index_knob("load_threads", 0)
    cut = tmp_path / "cut.mmi"
    for n in (3, 20, 30, len(raw) // 3, len(raw) // 2, len(raw) - 1):
        cut.write_bytes(raw[:n])
        with pytest.raises(RuntimeError):
            M.Index.load_from_mmi(str(cut))


def test_rust_binary_search_versions():
    """paf.rs:178's `binary_search` as rustc 1.52-1.81 and >= 1.82 compile it:
    identical on sorted arrays once the reference walks back to the first equal
    element; on unsorted arrays they disagree (hand-traced: [5,1,3,2,4,0] for 3
    is Err(4) with base/size halving, Err(6) with the early-exit midpoint)."""
    assert O.binary_search([5, 1, 3, 2, 4, 0], 3) == ("Err", 4)
    assert O.binary_search([5, 1, 3, 2, 4, 0], 3, pre182=True) == ("Err", 6)
    assert O.binary_search([1, 3, 3, 3, 3], 3) == ("Ok", 4)
    assert O.binary_search([1, 3, 3, 3, 3], 3, pre182=True) == ("Ok", 2)
    rng = np.random.default_rng(4)
    for _ in range(300):
        v = np.sort(rng.integers(0, 50, size=int(rng.integers(0, 40))))
        t = int(rng.integers(-2, 52))
        a, b = O.binary_search(v, t), O.binary_search(v, t, pre182=True)
        assert a[0] == b[0]
        if a[0] == "Ok":
            first = lambda i: int(np.searchsorted(v, v[i]))   # paf.rs:180 walks back to the first equal
            assert first(a[1]) == first(b[1])
        else:
            assert a[1] == b[1] == int(np.searchsorted(v, t))


def test_binary_search_exposure_even_k():
    """Reads whose dv depends on the reference's rustc (tests/golden/
    make_binsearch.py): with k = 16 their dv sketch's positions are not
    increasing, and the oracle reproduces both recorded PAF lines under the
    matching setting.  With odd k (every preset) positions are strictly
    increasing and the setting changes nothing (bench.py counts it)."""
    doc = json.load(open(os.path.join(GOLD, "binsearch_even_k.json")))
    assert doc["cases"]
    for c in doc["cases"]:
        mv = O.sketch(c["read"].encode(), doc["w"], doc["k"])
        pos = ((mv[:, 1] >> np.uint64(1)) & np.uint64(0xffffffff)).astype(np.int64)
        assert np.any(np.diff(pos) <= 0)
        ref = c["ref"].encode()
        oi = O.OIndex.build_from_buffer([doc["ref_name"]], np.frombuffer(ref, np.uint8), np.array([len(ref)], np.uint64),
                                        w=doc["w"], k=doc["k"], b=14, flag=0, threads=2)
        q = c["read"].encode()
        offs = np.array([0, len(q)], np.uint64)
        try:
            for pre, want in ((False, c["paf_rust_ge_1_82"]), (True, c["paf_rust_1_52_to_1_81"])):
                O.set_binary_search(pre)
                with tempfile.TemporaryDirectory() as td:
                    p = os.path.join(td, "o.paf")
                    oi.align_buffer([doc["read_name"]], np.frombuffer(q, np.uint8), offs, p, w=doc["w"], k=doc["k"], mid_occ=10000, threads=1)
                    assert open(p).read().rstrip("\n") == want
        finally:
            O.set_binary_search(False)
        assert c["paf_rust_ge_1_82"] != c["paf_rust_1_52_to_1_81"]
