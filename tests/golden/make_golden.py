"""Generate the golden fixtures under tests/golden/ with the independent
pure-Python restatement (tests/pyref.py) of the reference crate.

The reference ships no tests or known-answer vectors for this path and
cannot be built here (no Rust toolchain), so parity is
"unpinned" against the reference itself.  These fixtures pin the C++ oracle
(oracle/mm2rs_oracle.cpp) — and through it the GPU path — against a second,
separately written reading of the Rust sources.  Inputs are stored in the
fixtures, so tests do not depend on this script or on tools/simgen.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.json
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import pyref as R  # noqa: E402

COMP = str.maketrans("ACGTacgtN", "TGCAtgcaN")


def rand_seq(rng, n, p_low=0.0, p_n=0.0):
    s = [rng.choice("ACGT") for _ in range(n)]
    for i in range(n):
        x = rng.random()
        if x < p_n:
            s[i] = rng.choice("NnRYKM")
        elif x < p_n + p_low:
            s[i] = s[i].lower()
    return "".join(s)


def mutate(rng, s, p_sub, p_ins=0.0, p_del=0.0):
    out = []
    for c in s:
        x = rng.random()
        if x < p_del:
            continue
        if x < p_del + p_sub:
            out.append(rng.choice("ACGT"))
        else:
            out.append(c)
        if rng.random() < p_ins:
            out.append(rng.choice("ACGT"))
    return "".join(out)


def revcomp(s):
    return s.translate(COMP)[::-1]


def sketch_cases(rng):
    seqs = ["A", "ACGT", "N" * 40, "ACGTACGTACGTACGTACGTACGTACGT", "A" * 200, "AC" * 120,
            "ACGTTGCA" * 40, rand_seq(rng, 15), rand_seq(rng, 16), rand_seq(rng, 64), rand_seq(rng, 300, p_low=0.2),
            rand_seq(rng, 1200, p_n=0.01), rand_seq(rng, 800, p_n=0.2), ("ACGTTA" * 200)[:1100],
            "".join(rng.choice(["AAAAAAA", "CCCC", "GT", "TTTTTTTTTT"]) for _ in range(150))]
    s = list(rand_seq(rng, 1500))
    s[300:320] = "N" * 20
    seqs.append("".join(s))
    params = [(10, 15, False), (10, 19, False), (5, 16, False), (3, 4, False), (1, 1, False), (2, 10, False),
              (50, 7, False), (25, 28, False), (10, 15, True), (4, 8, True)]
    cases = []
    for w, k, hpc in params:
        for sq in seqs:
            out = R.sketch_sequence(sq.encode(), w, k, 3, hpc)
            cases.append({"seq": sq, "w": w, "k": k, "rid": 3, "hpc": hpc, "out": [[a, b] for a, b in out]})
    return cases


def filter_cases(rng):
    cases = []
    for sq in [("ACGTTA" * 300), rand_seq(rng, 3000), ("AC" * 500) + rand_seq(rng, 500), "A" * 50, rand_seq(rng, 40)]:
        mv = R.sketch_sequence(sq.encode(), 10, 15, 0, False)
        # duplicate a few entries so that counts cross the (10, 0.01) thresholds
        mv = mv + mv[: len(mv) // 3] * 12 if len(mv) > 20 else mv
        cases.append({"mv": [[a, b] for a, b in mv], "out": [[a, b] for a, b in R.filter_query_minimizers(mv)]})
    return cases


def world(rng):
    unit = rand_seq(rng, 1500)
    mono = rand_seq(rng, 171)
    sat = "".join(mutate(rng, mono, 0.03) for _ in range(40))
    c0 = rand_seq(rng, 9000) + mutate(rng, unit, 0.02) + rand_seq(rng, 6000, p_low=0.05) + sat + rand_seq(rng, 5000)
    c1 = rand_seq(rng, 7000) + mutate(rng, unit, 0.01) + rand_seq(rng, 8000)
    c2 = rand_seq(rng, 6000, p_n=0.001) + mutate(rng, unit, 0.03) + rand_seq(rng, 9000)
    contigs = [("chrA", c0), ("chrB", c1), ("chrC", c2), ("chrD", rand_seq(rng, 30))]
    reads = []

    def take(c, st, n):
        return contigs[c][1][st:st + n]

    reads.append(("fwd_exact", take(0, 1000, 2500)))
    reads.append(("fwd_err", mutate(rng, take(0, 12000, 3000), 0.04, 0.02, 0.02)))
    reads.append(("rev_err", revcomp(mutate(rng, take(2, 2000, 3000), 0.04, 0.02, 0.02))))
    reads.append(("odd_rid", mutate(rng, take(1, 1000, 2500), 0.03)))              # chrB (rid 1): Q19
    reads.append(("repeat", mutate(rng, unit, 0.02)))
    reads.append(("satellite", take(0, len(c0) - 5000 - len(sat) + 500, 3000)))
    reads.append(("chimera", take(0, 500, 1800) + take(2, 9000, 1800)))           # rescue DP
    reads.append(("gappy", take(2, 100, 1200) + rand_seq(rng, 1500) + take(2, 4000, 1200)))
    reads.append(("n_run", take(0, 3000, 1200) + "N" * 20 + take(0, 4220, 1200)))
    reads.append(("lower", take(2, 6500, 2000).lower()))
    reads.append(("random", rand_seq(rng, 2000)))
    reads.append(("short", take(0, 5000, 30)))
    reads.append(("tiny", "ACGTAC"))
    return contigs, reads


def world_fixture(rng):
    contigs, reads = world(rng)
    w, k, b = 10, 15, 14
    idx = R.Index.build([(n, s.encode()) for n, s in contigs], w, k, b, 0)
    mid_occs = {str(fr): idx.calc_mid_occ(fr) for fr in (2e-4, 0.01, 0.1, 0.5)}
    mid = max(idx.calc_mid_occ(2e-4), 10)
    # Index::get for minimizers of some reads + random (mostly absent) keys
    probes = []
    for q in [s for _, s in reads[:3]]:
        for m in R.sketch_sequence(q.encode(), w, k, 0, False)[:40]:
            probes.append(m[0] >> 8)
    probes += [rng.getrandbits(30) for _ in range(20)]
    gets = []
    for h in probes:
        g = idx.get(h)
        gets.append({"key": h, "kind": 0 if g is None else (1 if g[0] == "Single" else 2),
                     "pos": [] if g is None else ([g[1]] if g[0] == "Single" else list(g[1]))})
    out_reads = []
    for name, q in reads:
        qb = q.encode()
        mv = R.filter_query_minimizers(R.sketch_sequence(qb, w, k, 0, False))
        anchors = R.build_anchors_filtered(idx, mv, len(qb), mid)
        rec = {"name": name, "seq": q, "anchors": [[x, y] for x, y in anchors]}
        if anchors:
            gap = R.f32(R.f32(0.01) * R.f32(0.8)) * R.f32(k)
            f, pp, v = R.chain_dp_all_dp(anchors, 5000, 5000, 500, 5000, gap, k, 25)
            chain, score = R.fallback_chain(f, pp, v)
            rec.update({"f": f, "pprev": pp, "chain": chain, "score": int(score)})
        line, panic, rescued = R.align_one(idx, name, qb, mid, w, k)
        rec.update({"paf": line, "panic": bool(panic), "rescued": bool(rescued)})
        out_reads.append(rec)
    n_keys = sum(len(bk["h"]) for bk in idx.B if bk["h"])
    return {"contigs": [[n, s] for n, s in contigs], "w": w, "k": k, "b": b, "mid_occ": mid, "calc_mid_occ": mid_occs,
            "n_keys": n_keys, "gets": gets, "reads": out_reads}


def main():
    rng = random.Random(20251015)
    fx = {"sketch": sketch_cases(rng), "filter": filter_cases(rng)}
    with open(os.path.join(HERE, "sketch_filter.json"), "w") as fh:
        json.dump(fx, fh, separators=(",", ":"))
    wf = world_fixture(rng)
    with open(os.path.join(HERE, "world.json"), "w") as fh:
        json.dump(wf, fh, separators=(",", ":"))
    n_lines = sum(1 for r in wf["reads"] if r["paf"])
    print(f"sketch cases {len(fx['sketch'])}, filter cases {len(fx['filter'])}, world reads {len(wf['reads'])} "
          f"({n_lines} PAF lines, {sum(r['panic'] for r in wf['reads'])} panics, {sum(r['rescued'] for r in wf['reads'])} rescued)")


if __name__ == "__main__":
    main()
