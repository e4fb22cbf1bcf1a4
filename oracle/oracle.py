"""ctypes binding of the CPU oracle (oracle/mm2rs_oracle.cpp) — TEST
INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / baseline, never as the
product path.  PARITY UNPINNED: see the header of mm2rs_oracle.cpp.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liborc.so")
CLI = os.path.join(HERE, "build", "mm2rs-cpu")
_lib = None
_P64 = C.POINTER(C.c_uint64)


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.orc_sketch.restype = C.c_longlong
        L.orc_sketch.argtypes = [C.c_char_p, C.c_longlong, C.c_int, C.c_int, C.c_uint, C.c_int, _P64, C.c_longlong]
        L.orc_filter.restype = C.c_longlong
        L.orc_filter.argtypes = [_P64, C.c_longlong, C.c_int, C.c_float]
        L.orc_index_build.restype = C.c_void_p
        L.orc_index_build.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_index_load_mmi.restype = C.c_void_p
        L.orc_index_load_mmi.argtypes = [C.c_char_p]
        L.orc_index_save_mmi.restype = C.c_int
        L.orc_index_save_mmi.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_index_free.argtypes = [C.c_void_p]
        L.orc_index_calc_mid_occ.restype = C.c_int
        L.orc_index_calc_mid_occ.argtypes = [C.c_void_p, C.c_float]
        L.orc_index_params.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        L.orc_index_stats.argtypes = [C.c_void_p, _P64, C.POINTER(C.c_double), C.POINTER(C.c_double), _P64]
        L.orc_index_get.restype = C.c_longlong
        L.orc_index_get.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_int), _P64, C.c_longlong]
        L.orc_index_dump.restype = C.c_longlong
        L.orc_index_dump.argtypes = [C.c_void_p, _P64, C.POINTER(C.c_uint32), _P64, C.POINTER(C.c_longlong)]
        L.orc_anchors.restype = C.c_longlong
        L.orc_anchors.argtypes = [C.c_void_p, C.c_char_p, C.c_longlong, C.c_int, C.c_int, C.c_int, _P64, C.c_longlong,
                                  C.POINTER(C.c_longlong)]
        L.orc_chain_dp.restype = C.c_longlong
        L.orc_chain_dp.argtypes = [_P64, C.c_longlong, C.POINTER(C.c_int), C.POINTER(C.c_float), C.POINTER(C.c_int),
                                   C.POINTER(C.c_longlong), C.POINTER(C.c_longlong), C.c_longlong, C.POINTER(C.c_int),
                                   C.POINTER(C.c_ulonglong)]
        L.orc_align_fasta.restype = C.c_longlong
        L.orc_align_fasta.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_float), C.c_int,
                                      _P64, C.POINTER(C.c_double)]
        L.orc_index_build_seqs.restype = C.c_void_p
        L.orc_index_build_seqs.argtypes = [C.c_int, C.c_void_p, C.c_void_p, _P64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_align_seqs.restype = C.c_longlong
        L.orc_align_seqs.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, _P64, C.c_char_p, C.POINTER(C.c_int),
                                     C.POINTER(C.c_float), C.c_int, C.c_int, _P64, C.POINTER(C.c_double)]
        L.orc_set_quiet.argtypes = [C.c_int]
        L.orc_set_binary_search.argtypes = [C.c_int]
        L.orc_set_tie_order.argtypes = [C.c_int]
        L.orc_rust_sort.argtypes = [C.POINTER(C.c_int32), C.c_uint64, C.c_int, _P64]
        L.orc_binary_search.restype = C.c_int
        L.orc_binary_search.argtypes = [C.POINTER(C.c_int32), C.c_uint64, C.c_int32, C.c_int, _P64]
        L.orc_align_records.restype = C.c_longlong
        L.orc_align_records.argtypes = [C.c_void_p, C.c_int, C.c_void_p, _P64, C.POINTER(C.c_int), C.POINTER(C.c_float), C.c_int,
                                        C.c_int, C.POINTER(C.c_int32)]
        L.orc_pen.restype = C.c_int
        L.orc_pen.argtypes = [C.c_int, C.c_int, C.c_int, C.c_float]
        L.orc_default_gap.restype = C.c_float
        L.orc_default_gap.argtypes = [C.c_int]
        _lib = L
    return _lib


def sketch(seq: bytes, w: int, k: int, rid: int = 0, hpc: bool = False) -> Optional[np.ndarray]:
    """sketch_sequence -> (m, 2) uint64 [key_span, rid_pos_strand]; None on assertion failure."""
    L = lib()
    cap = 2 * len(seq) + 16
    out = np.zeros(2 * cap, dtype=np.uint64)
    n = L.orc_sketch(seq, len(seq), w, k, rid, 1 if hpc else 0, out.ctypes.data_as(_P64), cap)
    if n < 0:
        return None
    assert n <= cap
    return out[: 2 * n].reshape(n, 2)


def filter_minimizers(mv: np.ndarray, q_occ_max: int = 10, q_occ_frac: float = 0.01) -> np.ndarray:
    a = np.ascontiguousarray(mv, dtype=np.uint64).copy()
    n = lib().orc_filter(a.ctypes.data_as(_P64), len(a), q_occ_max, q_occ_frac)
    return a[:n]


class OIndex:
    def __init__(self, h: int):
        self.h = C.c_void_p(h)

    @classmethod
    def build(cls, fasta: str, w: int = 10, k: int = 15, b: int = 14, flag: int = 0, threads: int = 8) -> "OIndex":
        h = lib().orc_index_build(fasta.encode(), w, k, b, flag, threads)
        if not h:
            raise RuntimeError("oracle index build failed")
        return cls(h)

    @classmethod
    def build_from_buffer(cls, names, buf: np.ndarray, lens: np.ndarray, w: int = 10, k: int = 15, b: int = 14, flag: int = 0,
                          threads: int = 8) -> "OIndex":
        """Index from sequences concatenated in one uint8 buffer (no copies on the Python side)."""
        ptrs, lv, nm, _keep = _seq_views(names, buf, lens)
        h = lib().orc_index_build_seqs(len(lv), nm, ptrs, lv.ctypes.data_as(_P64), w, k, b, flag, threads)
        if not h:
            raise RuntimeError("oracle index build failed")
        return cls(h)

    @classmethod
    def load_mmi(cls, path: str) -> "OIndex":
        h = lib().orc_index_load_mmi(path.encode())
        if not h:
            raise RuntimeError("oracle mmi load failed")
        return cls(h)

    def save_mmi(self, path: str) -> None:
        assert lib().orc_index_save_mmi(self.h, path.encode()) == 0

    def close(self):
        if self.h:
            lib().orc_index_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def mid_occ(self, frac: float = 2e-4) -> int:
        return lib().orc_index_calc_mid_occ(self.h, frac)

    def params(self) -> Tuple[int, int, int, int, int]:
        out = (C.c_int * 5)()
        lib().orc_index_params(self.h, out)
        return tuple(out)

    def stats(self):
        a, d = C.c_uint64(), C.c_uint64()
        b, c = C.c_double(), C.c_double()
        lib().orc_index_stats(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
        return a.value, b.value, c.value, d.value

    def get(self, minier: int):
        kind = C.c_int()
        buf = (C.c_uint64 * 1)()
        n = lib().orc_index_get(self.h, minier, C.byref(kind), buf, 0)
        if kind.value == 0:
            return None
        buf = (C.c_uint64 * max(n, 1))()
        lib().orc_index_get(self.h, minier, C.byref(kind), buf, n)
        return ("Single", buf[0]) if kind.value == 1 else ("Multi", list(buf[:n]))

    def dump(self):
        """All keys: (keys, counts, positions) sorted by minimizer hash."""
        npos = C.c_longlong()
        nk = lib().orc_index_dump(self.h, None, None, None, C.byref(npos))
        keys = np.zeros(max(nk, 1), np.uint64)
        cnt = np.zeros(max(nk, 1), np.uint32)
        pos = np.zeros(max(npos.value, 1), np.uint64)
        lib().orc_index_dump(self.h, keys.ctypes.data_as(_P64), cnt.ctypes.data_as(C.POINTER(C.c_uint32)),
                             pos.ctypes.data_as(_P64), C.byref(npos))
        return keys[:nk], cnt[:nk], pos[: npos.value]

    def anchors(self, q: bytes, w: int, k: int, mid_occ: int):
        L = lib()
        nm = (C.c_longlong * 2)()
        n = L.orc_anchors(self.h, q, len(q), w, k, mid_occ, None, 0, nm)
        out = np.zeros(2 * max(n, 1), np.uint64)
        L.orc_anchors(self.h, q, len(q), w, k, mid_occ, out.ctypes.data_as(_P64), n, nm)
        return out[: 2 * n].reshape(n, 2), (nm[0], nm[1])

    def align_fasta(self, reads_fa: str, out_path: str, w: int = 10, k: int = 15, max_gap: int = 5000, bw: int = -1,
                    bw_long: int = -1, min_cnt: int = 3, min_chain_score: int = 40, best_n: int = 5, first_only: bool = False,
                    max_reads: int = 0, frac: float = 2e-4, mask_level: float = 0.5, pri_ratio: float = 0.8,
                    mid_occ: int = -1):
        """Align flow over a FASTA -> (#lines, counts dict, seconds of mapping)."""
        oi = (C.c_int * 10)(w, k, max_gap, bw, bw_long, min_cnt, min_chain_score, best_n, 1 if first_only else 0, max_reads)
        of = (C.c_float * 3)(frac, mask_level, pri_ratio)
        cnt = (C.c_uint64 * 7)()
        t = C.c_double()
        n = lib().orc_align_fasta(self.h, reads_fa.encode(), out_path.encode() if out_path else None, oi, of, mid_occ, cnt,
                                  C.byref(t))
        keys = ["m_all", "m_kept", "anchors", "rescued_anchors", "inner_iters", "lines", "panics"]
        return n, dict(zip(keys, list(cnt))), t.value


    def align_buffer(self, names, buf: np.ndarray, offs: np.ndarray, out_path: Optional[str] = None, w: int = 10, k: int = 15,
                     mid_occ: int = -1, threads: int = 1, max_gap: int = 5000, bw: int = -1, bw_long: int = -1, min_cnt: int = 3,
                     min_chain_score: int = 40, best_n: int = 5, frac: float = 2e-4, mask_level: float = 0.5, pri_ratio: float = 0.8):
        """Align flow over reads concatenated in buf (offsets offs[n+1]) -> (#lines, counts, seconds of mapping)."""
        offs = np.asarray(offs, dtype=np.uint64)
        lens = (offs[1:] - offs[:-1]).astype(np.uint64)
        ptrs, lv, nm, _keep = _seq_views(names, buf, lens, offs[:-1])
        oi = (C.c_int * 10)(w, k, max_gap, bw, bw_long, min_cnt, min_chain_score, best_n, 0, 0)
        of = (C.c_float * 3)(frac, mask_level, pri_ratio)
        cnt = (C.c_uint64 * 7)()
        t = C.c_double()
        n = lib().orc_align_seqs(self.h, len(lv), nm, ptrs, lv.ctypes.data_as(_P64), out_path.encode() if out_path else None,
                                 oi, of, mid_occ, threads, cnt, C.byref(t))
        keys = ["m_all", "m_kept", "anchors", "rescued_anchors", "inner_iters", "lines", "panics"]
        return n, dict(zip(keys, list(cnt))), t.value


REC_FIELDS = ("flags", "n_anchors", "score", "cm", "qs", "qe", "ts", "te", "rid", "rev", "dv", "m_kept")


def align_records(oi: "OIndex", seqs, mid_occ: int = -1, threads: int = 4, w: int = 10, k: int = 15, max_gap: int = 5000,
                  bw: int = -1, bw_long: int = -1, min_cnt: int = 3):
    """Per-read outcome of the Align flow (incl. reads on which the reference
    panics, Q19): an (n, 12) int32 array with columns REC_FIELDS (dv as f32 bits)."""
    n = len(seqs)
    bufs = [C.create_string_buffer(bytes(s), max(len(s), 1)) for s in seqs]
    ptrs = (C.c_void_p * max(n, 1))(*[C.cast(b, C.c_void_p).value for b in bufs])
    lens = np.array([len(s) for s in seqs], dtype=np.uint64)
    oi_ = (C.c_int * 10)(w, k, max_gap, bw, bw_long, min_cnt, 40, 5, 0, 0)
    of = (C.c_float * 3)(2e-4, 0.5, 0.8)
    rec = np.zeros((max(n, 1), 12), dtype=np.int32)
    set_quiet(True)
    lib().orc_align_records(oi.h, n, ptrs, lens.ctypes.data_as(_P64), oi_, of, mid_occ, threads,
                            rec.ctypes.data_as(C.POINTER(C.c_int32)))
    return rec[:n]


def set_quiet(q: bool = True) -> None:
    lib().orc_set_quiet(1 if q else 0)


def set_binary_search(pre182: bool) -> None:
    """paf.rs:178's `binary_search` as rustc 1.52-1.81 (True) or >= 1.82 (False, the default) compiles it."""
    lib().orc_set_binary_search(1 if pre182 else 0)


TIE_IPNSORT, TIE_PDQSORT = 3, 4


def set_tie_order(mode: int) -> None:
    """Tie order of the reference's two sort_unstable_by_key calls (lchain.rs:97, :292): 3 rustc 1.81+
    ipnsort (the default), 4 rustc 1.78-1.80 pdqsort, 0 std::sort, 1 / 2 stable with equal keys in
    ascending / descending input order (the extremes, for exposure counts)."""
    lib().orc_set_tie_order(int(mode))


def rust_sort_perm(keys, mode: int = TIE_IPNSORT):
    """Order of indices after Rust's sort_unstable_by_key on (keys[i], i) (tie order `mode`)."""
    k = np.ascontiguousarray(np.asarray(keys, dtype=np.int32))
    out = np.zeros(len(k), dtype=np.uint64)
    lib().orc_rust_sort(k.ctypes.data_as(C.POINTER(C.c_int32)), len(k), int(mode), out.ctypes.data_as(_P64))
    return out


def binary_search(v, target: int, pre182: bool = False):
    """Rust slice::binary_search of `target` in the i32 array v: ("Ok", i) or ("Err", i)."""
    a = np.ascontiguousarray(v, dtype=np.int32)
    out = np.zeros(1, np.uint64)
    f = lib().orc_binary_search(a.ctypes.data_as(C.POINTER(C.c_int32)), len(a), int(target), 1 if pre182 else 0,
                                out.ctypes.data_as(_P64))
    return ("Ok" if f else "Err", int(out[0]))


def _seq_views(names, buf: np.ndarray, lens, starts=None):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    lv = np.ascontiguousarray(lens, dtype=np.uint64)
    if starts is None:
        starts = np.concatenate([[0], np.cumsum(lv)[:-1]]).astype(np.uint64) if len(lv) else np.zeros(0, np.uint64)
    base = buf.ctypes.data
    ptrs = (C.c_void_p * max(len(lv), 1))(*[base + int(s) for s in starts])
    nm = None
    if names is not None:
        nm = (C.c_char_p * max(len(lv), 1))(*[x.encode() for x in names])
    return ptrs, lv, nm, (buf,)


def chain_dp(anchors_xy: np.ndarray, k: int = 15, max_gap: int = 5000, bw: int = 500, max_iter: int = 5000,
             min_chain_score: int = 40, min_cnt: int = 3, max_skip: int = 25, max_drop: int = 500, bw_long: int = 20000):
    """chain_dp_all on an anchor array -> (f, pprev, chain, score, inner_iters)."""
    L = lib()
    a = np.ascontiguousarray(anchors_xy, dtype=np.uint64).reshape(-1)
    n = len(a) // 2
    params = (C.c_int * 10)(max_gap, max_gap, bw, max_iter, min_chain_score, min_cnt, max_skip, max_drop, bw_long, 1000)
    fparams = (C.c_float * 3)(L.orc_default_gap(k), 0.0, 0.1)
    f = np.zeros(max(n, 1), np.int32)
    pp = np.zeros(max(n, 1), np.int64)
    ch = np.zeros(max(n, 1), np.int64)
    score = C.c_int()
    it = C.c_ulonglong()
    m = L.orc_chain_dp(a.ctypes.data_as(_P64), n, params, fparams, f.ctypes.data_as(C.POINTER(C.c_int)),
                       pp.ctypes.data_as(C.POINTER(C.c_longlong)), ch.ctypes.data_as(C.POINTER(C.c_longlong)), n,
                       C.byref(score), C.byref(it))
    chain = ch[:m] if m >= 0 else ch[:0]
    return f[:n], pp[:n], chain, (score.value if m >= 0 else None), it.value


def read_fasta(path: str) -> List[Tuple[str, bytes]]:
    out = []
    name, parts = None, []
    with open(path, "rb") as fh:
        for line in fh:
            line = line.rstrip(b"\n").rstrip(b"\r")
            if line.startswith(b">"):
                if name is not None:
                    out.append((name, b"".join(parts)))
                name = line[1:].split(b" ")[0].split(b"\t")[0].decode()
                parts = []
            elif name is not None:
                parts.append(line)
    if name is not None:
        out.append((name, b"".join(parts)))
    return out
