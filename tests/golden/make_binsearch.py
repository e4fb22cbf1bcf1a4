"""Generate tests/golden/binsearch_even_k.json: reads whose PAF dv depends on
the rustc version the reference is built with.

paf.rs:178 calls `mini_pos.binary_search(&first)`; std changed the algorithm
in rustc 1.82 (1.52-1.81: midpoint of [left, right) with an early return on
Equal; >= 1.82: base/size halving).  For odd k, mini_pos is strictly
increasing and the two agree.  For even k a symmetric k-mer keeps `l` at
w+k-1 for several steps, the first-window tie emission (sketch.rs:79-82)
repeats, and mini_pos holds duplicates and runs backwards: the two searches
can then return different Ok indices or Ok vs Err.  This script searches a
seeded palindrome-rich reference with (w, k) = (10, 16) for reads whose PAF
differs between the two oracle settings, cuts a small reference window around
each, and records both lines (regenerated on the cut reference).

    python tests/golden/make_binsearch.py   # rewrites tests/golden/binsearch_even_k.json
"""
import json
import os
import random
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

W, K = 10, 16


def paf_both(ref: bytes, reads, names):
    oi = O.OIndex.build_from_buffer(["c0"], np.frombuffer(ref, np.uint8), np.array([len(ref)], np.uint64), w=W, k=K, b=14,
                                    flag=0, threads=4)
    cat = np.frombuffer(b"".join(reads), np.uint8)
    offs = np.zeros(len(reads) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in reads])
    out = []
    for pre in (False, True):
        O.set_binary_search(pre)
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "o.paf")
            oi.align_buffer(names, cat, offs, p, w=W, k=K, mid_occ=10000, threads=4)
            out.append({ln.split(b"\t")[0].decode(): ln.decode() for ln in open(p, "rb").read().splitlines()})
    O.set_binary_search(False)
    oi.close()
    return out


def main():
    rng = random.Random(3)

    def rs(n):
        return "".join(rng.choice("ACGT") for _ in range(n))

    def pal_region():
        s = ""
        for _ in range(rng.randint(3, 12)):
            u = rng.choice(["AT", "TA", "GC", "CG", "ACGT", "AATT", "CCGG", "TGCA", "AGCT"])
            s += u * rng.randint(3, 20) + rs(rng.randint(1, 12))
        return s
    ref = "".join(rs(rng.randint(50, 400)) + pal_region() for _ in range(200)).encode()
    reads, starts = [], []
    for _ in range(3000):
        L = rng.randint(150, 1500)
        st = rng.randint(0, len(ref) - L)
        q = bytearray(ref[st:st + L])
        for j in range(len(q)):
            if rng.random() < 0.02:
                q[j] = ord(rng.choice("ACGT"))
        reads.append(bytes(q))
        starts.append(st)
    names = [f"r{i}" for i in range(len(reads))]
    new, old = paf_both(ref, reads, names)
    cases = []
    for n in names:
        if new[n] == old.get(n) or len(cases) >= 4:
            continue
        i = int(n[1:])
        lo = max(0, starts[i] - 3000)
        cut = ref[lo:starts[i] + len(reads[i]) + 3000]
        a, b = paf_both(cut, [reads[i]], ["q"])
        if a.get("q") and a["q"] != b.get("q"):
            cases.append({"read": reads[i].decode(), "ref": cut.decode(), "paf_rust_ge_1_82": a["q"], "paf_rust_1_52_to_1_81": b["q"]})
    doc = {"w": W, "k": K, "ref_name": "c0", "read_name": "q",
           "note": "PAF of `mm2rs align -w 10 -k 16 ref.fa q.fa` with paf.rs:178's binary_search as rustc >= 1.82 and "
                   "as rustc 1.52-1.81 compile it; both lines from oracle/mm2rs_oracle.cpp (this script)",
           "cases": cases}
    with open(os.path.join(ROOT, "tests", "golden", "binsearch_even_k.json"), "w") as fh:
        json.dump(doc, fh, indent=1)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
