"""nt4 read packing (include/mm2g.h "nt4 read batch"; src/nt4.rs:2-10), host side:
mm2g_nt4_pack against a direct restatement, on CPU (no device calls)."""
import random

import numpy as np
import pytest

import minimap2_rs_amd as M


def _nt4(b: int) -> int:
    """src/nt4.rs:2-10"""
    return {ord("A"): 0, ord("a"): 0, ord("C"): 1, ord("c"): 1, ord("G"): 2, ord("g"): 2, ord("T"): 3, ord("t"): 3}.get(b, 4)


def _expect(seqs):
    pk, amb, words = [], [], []
    w = 0
    for s in seqs:
        pk.append(w)
        w += (len(s) + 31) // 32
    codes = np.zeros(w, np.uint64)
    ambw = []
    for r, s in enumerate(seqs):
        has = False
        for i, b in enumerate(s):
            c = _nt4(b)
            if c < 4:
                codes[pk[r] + i // 32] |= np.uint64(c << (2 * (i % 32)))
            else:
                has = True
        if has:
            amb.append(w)
            bm = np.zeros((len(s) + 63) // 64, np.uint64)
            for i, b in enumerate(s):
                if _nt4(b) == 4:
                    bm[i // 64] |= np.uint64(1 << (i % 64))
            ambw.append(bm)
            w += len(bm)
        else:
            amb.append(2**64 - 1)
    allw = np.concatenate([codes] + ambw) if ambw else codes
    return np.array(pk, np.uint64), np.array(amb, np.uint64), allw


@pytest.mark.parametrize("threads", [1, 3])
def test_nt4_pack_matches_restatement(threads):
    rng = random.Random(7)
    seqs = [b"", b"A", b"N", b"acgtn" * 13]
    for n in [1, 31, 32, 33, 63, 64, 65, 95, 96, 97, 200, 1000, 4099]:
        alpha = rng.choice([b"ACGT", b"ACGTacgt", b"ACGTNnRY-*", b"ACGT" * 50 + b"N"])
        seqs.append(bytes(rng.choice(alpha) for _ in range(n)))
    seqs += [bytes(rng.randrange(256) for _ in range(300)) for _ in range(3)]   # every byte value
    cat = np.frombuffer(b"".join(seqs) or b"\0", np.uint8)
    offs = np.zeros(len(seqs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(s) for s in seqs])
    pk, amb, words = M.nt4_pack(cat, offs, threads=threads)
    epk, eamb, ewords = _expect(seqs)
    assert np.array_equal(pk, epk)
    assert np.array_equal(amb, eamb)
    assert np.array_equal(words, ewords)


def test_nt4_pack_many_reads_threads():
    rng = np.random.default_rng(3)
    n = 3000
    lens = rng.integers(0, 4000, n)
    cat = rng.choice(np.frombuffer(b"ACGTacgtN", np.uint8), int(lens.sum()), p=[.12] * 8 + [.04])
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    a = M.nt4_pack(cat, offs, threads=1)
    b = M.nt4_pack(cat, offs, threads=8)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
