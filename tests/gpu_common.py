"""Shared fixtures and checks of the GPU parity tests (test_gpu_*.py): seeded
synthetic worlds, context knobs, and per-read comparison with the oracle."""
import contextlib
import os
import random

import numpy as np
import pytest

import minimap2_rs_amd as M
from oracle import oracle as O
from tools import simdata


@contextlib.contextmanager
def knobs(dev, **kv):
    """Set context knobs (include/mm2g.h MM2G_KNOB_*) for the block, then restore them."""
    old = {k: dev.get_knob(k) for k in kv}
    for k, v in kv.items():
        dev.set_knob(k, v)
    try:
        yield
    finally:
        for k, v in old.items():
            dev.set_knob(k, v)


def assert_records(res, seqs, rec, what=""):
    """Per-read result fields of the device path equal the oracle's per-read
    outcome (O.align_records): chain flags, anchors, score, cm, q/t ranges,
    rid/strand and dv -- for reads on which the reference panics (Q19) too."""
    bad = []
    for i in range(len(seqs)):
        r, o = res[i], rec[i]
        dv = np.array([r.dv], np.float32).view(np.int32)[0]
        got = (r.flags & 11, r.n_anchors, r.score, r.cm, r.qs, r.qe, r.ts, r.te, r.rid, r.rev, int(dv))
        want = tuple(int(v) for v in (o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8], o[9], o[10]))
        if len(seqs[i]) == 0:
            got = (0,) + got[1:]
        if got != want:
            bad.append((i, got, want))
    assert not bad, f"{what}: {len(bad)} reads differ, first: {bad[:3]}"


def _rand_seq(rng, n, p_n=0.0, p_low=0.1, alphabet=b"ACGT"):
    s = bytearray(rng.choice(alphabet) for _ in range(n))
    for i in range(n):
        r = rng.random()
        if r < p_n:
            s[i] = ord(rng.choice("NnRYKM-*"))
        elif r < p_n + p_low:
            s[i] = s[i] | 0x20 if chr(s[i]).isalpha() else s[i]
    return bytes(s)


@pytest.fixture(scope="module")
def small_world(tmp_path_factory):
    td = tmp_path_factory.mktemp("world")
    ref = str(td / "ref.fa")
    simdata.write_genome("hg38", 0.0008, 21, ref)        # 24 contigs, ~2.5 Mb, hg38-shaped repeats
    names, seqs = simdata.read_fasta_seqs(ref)
    lens = np.array([len(s) for s in seqs], dtype=np.int64)
    g = np.frombuffer(b"".join(seqs), dtype=np.uint8)
    rb, offs, _ = simdata.reads(g, lens, 150, 6000, 22)
    rnames = [f"r{i}" for i in range(150)]
    rseqs = [rb[offs[i]:offs[i + 1]].tobytes() for i in range(150)]
    rng = random.Random(3)
    extra = [(b"ACGT" * 3), _rand_seq(rng, 5000), _rand_seq(rng, 30), b"N" * 100,
             seqs[0][20000:21000], seqs[1][30000:30500].lower(), seqs[2][40000:52000]]
    for i, s in enumerate(extra):
        rnames.append(f"x{i}")
        rseqs.append(s)
    reads = str(td / "reads.fa")
    simdata.write_fasta(reads, rnames, rseqs)
    return ref, reads, rnames, rseqs


def _mutate(rng, s: bytes, p: float) -> bytes:
    b = bytearray(s)
    for i in range(len(b)):
        if rng.random() < p:
            b[i] = ord(rng.choice("ACGT"))
    return bytes(b)


@pytest.fixture(scope="module")
def dense_world(tmp_path_factory):
    """Satellite arrays + segmental duplications: windows of thousands of
    anchors once mid_occ is lifted (deep j-steps beyond the LDS ring, n_skip
    breaks, max_iter clipping, rescue)."""
    td = tmp_path_factory.mktemp("dense")
    rng = random.Random(77)
    mono = _rand_seq(rng, 171, p_low=0.0)
    sat = b"".join(_mutate(rng, mono, 0.03) for _ in range(120))                 # ~20 kb alpha-like array
    unit = _rand_seq(rng, 2000, p_low=0.0)
    sd = b"".join(_mutate(rng, unit, 0.01) for _ in range(12))                   # 24 kb tandem segmental dup
    c0 = _rand_seq(rng, 30000, p_low=0.0) + sat + _rand_seq(rng, 30000, p_low=0.0)
    c1 = _rand_seq(rng, 10000, p_low=0.0) + sd + _rand_seq(rng, 10000, p_low=0.0)
    sd2 = b"".join(_mutate(rng, unit[:1500], 0.02) for _ in range(10))          # 15 kb on an even rid
    c2 = _rand_seq(rng, 40000, p_low=0.0) + sd2 + _rand_seq(rng, 8000, p_low=0.0)
    ref = str(td / "dense.fa")
    simdata.write_fasta(ref, ["c0", "c1", "c2"], [c0, c1, c2])
    rnames, rseqs = [], []
    for t in range(8):                       # inside the satellite
        st = 30000 + rng.randrange(0, len(sat) - 4000)
        rseqs.append(_mutate(rng, c0[st:st + 3500], 0.04))
    for t in range(8):                       # inside / across the segmental dup
        st = 10000 + rng.randrange(-3000, len(sd) - 3000)
        rseqs.append(_mutate(rng, c1[st:st + 6000], 0.03))
    for t in range(6):                       # unique sequence, one crossing into the array
        st = rng.randrange(0, len(c2) - 5000)
        rseqs.append(_mutate(rng, c2[st:st + 5000], 0.05))
    rseqs.append(c0[27000:27000 + 6000])
    for t in range(4):                       # chimeras: half unique, half elsewhere -> rescue DP
        a0 = rng.randrange(0, 20000)
        b0 = rng.randrange(0, 30000)
        rseqs.append(_mutate(rng, c2[a0:a0 + 4000] + c0[b0:b0 + 4000], 0.03))
    for t in range(4):                       # inside the even-rid duplication
        st = 40000 + rng.randrange(0, len(sd2) - 5000)
        rseqs.append(_mutate(rng, c2[st:st + 5000], 0.03))
    rnames = [f"d{i}" for i in range(len(rseqs))]
    reads = str(td / "dense_reads.fa")
    simdata.write_fasta(reads, rnames, rseqs)
    return ref, reads, rnames, rseqs


def _production_vs_oracle(dev, small_world, dense_world, opts=None, tag=""):
    o = opts if opts is not None else M.map_opts()
    for world, mid in ((small_world, None), (dense_world, 5000), (dense_world, 20)):
        ref, reads, rnames, rseqs = world
        oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
        idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 4)
        mid = mid if mid is not None else max(idx.calc_mid_occ(2e-4), 10)
        dev.upload_index(idx, mid)
        dev.set_debug(False)
        dev.set_reads(rseqs)
        res = dev.map(o)
        rec = O.align_records(oi, rseqs, mid_occ=mid, max_gap=o.max_gap, bw=o.bw, bw_long=o.bw_long)
        assert_records(res, rseqs, rec, f"{tag} mid {mid}")
        assert (rec[:, 0] & 8).any() or world is dense_world      # Q19 panic reads are compared too
        want_paf = os.path.join(os.path.dirname(reads), f"want_{mid}.paf")
        oi.align_fasta(reads, want_paf, mid_occ=mid, max_gap=o.max_gap, bw=o.bw, bw_long=o.bw_long)
        assert dev.paf(rnames, res) == open(want_paf).read()
    dev.set_debug(True)




def _singleton_keep(a: np.ndarray) -> np.ndarray:
    """The sort's singleton filter restated on (x, y) anchors: keep an anchor
    iff its 32 kb cell of its (rid, strand) group -- or of the Q19
    pseudo-group -- holds another anchor, or a neighbouring cell does."""
    x = a[:, 0]
    hi = x >> np.uint64(32)
    gid = np.where(hi == np.uint64(0xffffffff), np.uint64(1 << 33), hi)
    cell = (gid << np.uint64(20)) | ((x & np.uint64(0x7fffffff)) >> np.uint64(15))
    u, inv, cnt = np.unique(cell, return_inverse=True, return_counts=True)
    occ = set(u.tolist())
    left = np.array([(c - 1) in occ for c in cell.tolist()], dtype=bool)
    right = np.array([(c + 1) in occ for c in cell.tolist()], dtype=bool)
    return (cnt[inv] >= 2) | left | right
