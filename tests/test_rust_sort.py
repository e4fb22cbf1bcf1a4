"""CPU: the two restatements of Rust's `sort_unstable_by_key` (the oracle's C++
rsort:: and tests/pyref.py) give the same permutation -- including the order of
equal keys, which is what lchain.rs:97 / :292 expose under `-n <= 1 -m <= k`
(DESIGN.md §2 "-n <= 1").  Both algorithms: ipnsort (rustc 1.81+) and pdqsort
(rustc 1.78-1.80).  No Rust toolchain here: unpinned against rustc itself."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import pyref as P


def _inputs():
    rng = np.random.default_rng(7)
    out = []
    for n in list(range(0, 40)) + [47, 48, 49, 50, 63, 64, 65, 100, 129, 257, 300, 513, 1000, 2049, 5000]:
        for hi in (2, 5, 40, 1 << 20):
            out.append(rng.integers(0, hi, n))
    for n in (30, 100, 1000, 4000):
        out.append(np.arange(n))                              # sorted
        out.append(np.arange(n)[::-1].copy())                 # strictly descending
        out.append(np.arange(n) // 7)                         # non-descending with ties
        out.append((np.arange(n) // 7)[::-1].copy())          # descending with ties
        out.append(np.arange(n) % 13)                         # sawtooth
        a = np.arange(n)
        sw = rng.integers(0, n, 6)
        a[sw] = a[sw[::-1]]
        out.append(a)                                         # nearly sorted
        out.append(np.full(n, 3))                             # all equal
        b = rng.integers(15, 60, n)
        b[rng.random(n) < 0.7] = 15                           # chain f values: mostly the span
        out.append(b)
    return out


@pytest.mark.parametrize("mode", [O.TIE_IPNSORT, O.TIE_PDQSORT])
def test_rust_sort_restatements_agree(mode):
    fn = P.rust_sort_unstable_ipn if mode == O.TIE_IPNSORT else P.rust_sort_unstable_pdq
    n_tie_diff = 0
    for keys in _inputs():
        keys = [int(x) for x in keys]
        got = [int(x) for x in O.rust_sort_perm(keys, mode)]
        want = [e[1] for e in fn([(k, i) for i, k in enumerate(keys)])]
        assert got == want, (mode, len(keys), keys[:40])
        assert all(keys[got[i]] <= keys[got[i + 1]] for i in range(len(got) - 1))
        assert sorted(got) == list(range(len(keys)))
        stable = sorted(range(len(keys)), key=lambda i: keys[i])
        n_tie_diff += got != stable
    assert n_tie_diff > 0          # the tie order is really unstable on some inputs


def test_ipnsort_and_pdqsort_differ_on_ties():
    keys = [int(x) for x in np.random.default_rng(3).integers(0, 4, 500)]
    a = list(O.rust_sort_perm(keys, O.TIE_IPNSORT))
    b = list(O.rust_sort_perm(keys, O.TIE_PDQSORT))
    assert a != b
