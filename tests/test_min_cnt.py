"""CPU: `-n <= 1` (min_cnt) in the Align flow, on the oracle (DESIGN.md "-n <= 1").

The backtrack of chain_dp_all (/root/reference/src/lchain.rs:92-160) sets
t[i] = 2 and then tests t[i] == 0 in the same iteration of mg_chain_bk_end's
loop (lchain.rs:110,114 and 140,144), so the loop always stops after one step: every chain
it extracts is the single anchor i0, with score f[i0] - f[pprev[i0]] (or f[i0]
= span when pprev is -1), never above the span.  Hence:
  * -m above the span (the default 40 > k <= 28): no backtrack chain passes
    min_chain_score, chain_dp_all falls back exactly as under -n >= 2, and the
    PAF is -n 3's whatever Rust's sort_unstable tie order (checked under both
    extreme tie orders);
  * -m at or below the span: one-anchor chains pass, and merge_adjacent_chains
    _with_gap's sort_unstable_by_key on qs (lchain.rs:292) meets large tie
    classes (every hit of one minimizer has the same qs), so the PAF depends
    on the tie order, which Rust leaves unspecified and which changed with the
    rustc sort implementation (both restated in the oracle: ipnsort, the
    default, and pdqsort); these tests measure the exposure, and the device
    path's multi-chain output is compared in test_gpu_parity.py.
"""
import os

import pytest

from oracle import oracle as O
from tools import simdata


@pytest.fixture(scope="module")
def world(tmp_path_factory):
    td = tmp_path_factory.mktemp("mincnt")
    ref = str(td / "ref.fa")
    reads = str(td / "reads.fa")
    simdata.write_genome("small", 1.0, 11, ref)
    simdata.write_reads(ref, 60, 4000, 12, reads)
    return ref, reads, td


def _paf(oi, reads, out, **kw):
    oi.align_fasta(reads, out, **kw)
    return open(out).read()


def test_min_cnt_le1_equals_default_when_m_above_span(world):
    ref, reads, td = world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    try:
        base = _paf(oi, reads, str(td / "n3.paf"))
        assert base.count("\n") > 20
        for mode in (1, 2):
            O.set_tie_order(mode)
            for mc in (1, 0, -1):
                for m in (40, 16):
                    got = _paf(oi, reads, str(td / f"n{mc}_{m}_{mode}.paf"), min_cnt=mc, min_chain_score=m)
                    assert got == base, (mc, m, mode)
    finally:
        O.set_tie_order(O.TIE_IPNSORT)


def test_min_cnt_le1_low_m_depends_on_tie_order(world):
    """-n 1 -m <= k: the two extreme tie orders give different PAF for many
    reads (why Rust's sort_unstable is restated, not replaced)."""
    ref, reads, td = world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    try:
        outs = []
        for mode in (1, 2):
            O.set_tie_order(mode)
            outs.append(_paf(oi, reads, str(td / f"low_m_{mode}.paf"), min_cnt=1, min_chain_score=15))
    finally:
        O.set_tie_order(O.TIE_IPNSORT)
    by = [{} for _ in outs]
    for d, txt in zip(by, outs):
        for ln in txt.splitlines():
            d.setdefault(ln.split("\t")[0], []).append(ln)
    names = set(by[0]) | set(by[1])
    differ = sum(1 for q in names if by[0].get(q) != by[1].get(q))
    print(f"-n 1 -m 15: {differ} of {len(names)} reads' PAF depend on the sort_unstable tie order")
    assert differ > 0


def _by_read(txt):
    d = {}
    for ln in txt.splitlines():
        d.setdefault(ln.split("\t")[0], []).append(ln)
    return d


@pytest.mark.parametrize("m", [15, 0])
def test_min_cnt_le1_ipnsort_vs_pdqsort(world, m):
    """-n 1 -m <= k under the two restated rustc sorts (ipnsort, rustc 1.81+,
    the default; pdqsort, rustc 1.78-1.80): how many reads' PAF depend on the
    rustc version (reported; DESIGN.md §2 "-n <= 1")."""
    ref, reads, td = world
    oi = O.OIndex.build(ref, 10, 15, 14, 0, 4)
    outs = []
    try:
        for mode in (O.TIE_IPNSORT, O.TIE_PDQSORT):
            O.set_tie_order(mode)
            outs.append(_paf(oi, reads, str(td / f"rs_{m}_{mode}.paf"), min_cnt=1, min_chain_score=m))
    finally:
        O.set_tie_order(O.TIE_IPNSORT)
    a, b = _by_read(outs[0]), _by_read(outs[1])
    names = set(a) | set(b)
    differ = sum(1 for q in names if a.get(q) != b.get(q))
    lines = outs[0].count("\n")
    print(f"-n 1 -m {m}: {differ} of {len(names)} reads' PAF differ between ipnsort and pdqsort ({lines} lines)")
    assert lines > len(names)      # several chains per read: the multi-chain output is exercised
