"""CPU: randomized cross-check of the C++ oracle against the independent
pure-Python restatement (tests/pyref.py) beyond the committed fixtures:
sketch for random (w, k) incl. even k (symmetric k-mers) and HPC spans,
the query filter, and chain_dp_all + fallback on synthetic anchor sets with
clustered, repetitive and multi-group layouts."""
import random

import numpy as np
import pytest

from oracle import oracle as O

import pyref as R


def _seq(rng, n):
    kind = rng.random()
    if kind < 0.3:
        unit = "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 7)))
        s = (unit * (n // len(unit) + 1))[:n]
        s = "".join(c if rng.random() > 0.05 else rng.choice("ACGTN") for c in s)
    else:
        s = "".join(rng.choice("ACGTacgtN" if rng.random() < 0.05 else "ACGT") for _ in range(n))
    return s.encode()


@pytest.mark.parametrize("seed", range(6))
def test_sketch_random(seed):
    rng = random.Random(100 + seed)
    for _ in range(25):
        w = rng.choice([1, 2, 3, 5, 10, 16, 31, 64, 100, 255])
        k = rng.choice([1, 2, 4, 8, 11, 14, 15, 16, 17, 20, 21, 28])
        hpc = rng.random() < 0.25
        s = _seq(rng, rng.randint(1, 1500))
        got = O.sketch(s, w, k, rng.randint(0, 5), hpc)
        want = np.array(R.sketch_sequence(s, w, k, int(got[0][1] >> 32) if len(got) else 0, hpc), dtype=np.uint64)
        assert np.array_equal(got.reshape(-1, 2), want.reshape(-1, 2)), (w, k, hpc, len(s))


def test_filter_random():
    rng = random.Random(7)
    for _ in range(40):
        n = rng.randint(0, 400)
        pool = [rng.getrandbits(20) for _ in range(rng.randint(1, 50))]
        mv = [((rng.choice(pool) << 8) | 15, rng.getrandbits(20)) for _ in range(n)]
        got = O.filter_minimizers(np.array(mv, dtype=np.uint64).reshape(-1, 2))
        want = np.array(R.filter_query_minimizers(mv), dtype=np.uint64).reshape(-1, 2)
        assert np.array_equal(got.reshape(-1, 2), want)


def _anchors(rng, n):
    """Sorted (x, y) anchors: several groups, clustered diagonals and junk."""
    out = []
    for _ in range(n):
        rid = rng.choice([0, 0, 0, 2, 4])
        rev = rng.random() < 0.3
        if rng.random() < 0.6:   # a diagonal with noise
            q = rng.randint(0, 9000)
            p = 100000 + q + rng.randint(-300, 300)
        else:
            q = rng.randint(0, 9000)
            p = rng.randint(0, 400000)
        x = ((1 << 63) if rev else 0) | (rid << 32) | p
        y = (15 << 32) | q
        out.append((x, y))
    out.sort()
    return out


@pytest.mark.parametrize("seed", range(8))
def test_chain_dp_random(seed):
    rng = random.Random(500 + seed)
    n = rng.choice([1, 2, 5, 40, 300, 900])
    a = _anchors(rng, n)
    bw = rng.choice([500, 500, 20000])
    gap = R.f32(R.f32(0.01) * R.f32(0.8)) * R.f32(15)
    f, pp, v = R.chain_dp_all_dp(a, 5000, 5000, bw, 5000, gap, 15, 25)
    chain, score = R.fallback_chain(f, pp, v)
    of, opp, och, osc, _ = O.chain_dp(np.array(a, dtype=np.uint64), 15, bw=bw)
    assert of.tolist() == f and opp.tolist() == pp
    assert och.tolist() == chain and osc == int(score)


def test_pen_lut_matches_reference_float_path():
    """comput_sc's penalty (lchain.rs:28-31) as the oracle computes it inline
    equals pyref's op-by-op f32 restatement for every dd the LUT covers."""
    gap = float(R.f32(R.f32(0.01) * R.f32(0.8)) * R.f32(15))
    for dd in list(range(0, 2000)) + list(range(2000, 20001, 37)):
        want = int(R.f32(R.f32(gap) * R.f32(dd) + R.f32(0.5) * (R.mg_log2(dd + 1) if dd >= 1 else R.f32(0.0))))
        assert O.lib().orc_pen(dd, 0, 15, gap) == want, dd
