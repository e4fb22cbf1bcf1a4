"""Python mirror of the reference crate's public interface for the hot path.

Names follow the Rust crate (src/lib.rs:1-6):

=========================================  ==========================================
reference (file:line)                      here
=========================================  ==========================================
``sketch_sequence`` (sketch.rs:29)         :meth:`Device.sketch_sequences`
``Index::{load_from_mmi,save_to_mmi}``     :meth:`Index.load_from_mmi`, :meth:`Index.save_to_mmi`
``build_index_from_fasta`` (index.rs:427)  :meth:`Index.build_index_from_fasta`
``Index::get`` (index.rs:143)              :meth:`Index.get`
``Index::calc_mid_occ`` (index.rs:124)     :meth:`Index.calc_mid_occ`
``Index::stats`` (index.rs:111)            :meth:`Index.stats`
``nt4`` (nt4.rs:2-10) on a read batch      :func:`nt4_pack`, :meth:`Device.set_reads_nt4`
``build_anchors_filtered`` (seeds.rs:42)   :meth:`Device.seed_batch`
``chain_dp_all`` (lchain.rs:59)            :meth:`Device.chain_batch`
``rescue_long_join`` (lchain.rs:321)       :meth:`Device.chain_batch` (``rescue=True``)
``default_chain_params`` (main.rs:105)     :func:`chain_params`
``write_paf`` (paf.rs:224)                 :meth:`Device.paf`
Align flow (main.rs:189-230)               :func:`align`
=========================================  ==========================================

All compute runs on the MI355X through libmm2g.so; errors are raised, never
papered over with a CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from ._lib import ChainLine, ChainParams, ChainResult, MapOpts, Nt4Batch, ReadResult, check, load


@dataclass
class Minimizer:
    key_span: int           # hash << 8 | span
    rid_pos_strand: int     # rid << 32 | pos << 1 | strand


def map_opts(**kw) -> MapOpts:
    """``mm2rs align`` defaults (main.rs:105-123) with keyword overrides."""
    o = MapOpts()
    load().mm2g_map_opts_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def chain_params(k: int = 15, **kw) -> ChainParams:
    """``default_chain_params(k)`` (main.rs:105-123) with keyword overrides."""
    p = ChainParams()
    load().mm2g_chain_params_default(C.byref(p), k)
    for name, v in kw.items():
        setattr(p, name, v)
    return p


def set_index_knob(name: str, value: int) -> None:
    """Process-wide switch of the index build / .mmi load (``mm2g_set_index_knob``)."""
    check(load().mm2g_set_index_knob(L.INDEX_KNOBS[name], int(value)), "set_index_knob")


def nt4_pack(seq: np.ndarray, offs: np.ndarray, threads: int = 4):
    """ASCII reads -> the device nt4 format (include/mm2g.h): (pk_off, amb_off, words)."""
    seq = np.ascontiguousarray(seq, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    n = len(offs) - 1
    cap = int(load().mm2g_nt4_words_bound(offs.ctypes.data_as(L._P64), n))
    pk = np.zeros(max(n, 1), np.uint64)
    amb = np.zeros(max(n, 1), np.uint64)
    words = np.zeros(max(cap, 1), np.uint64)
    nw = check(load().mm2g_nt4_pack(seq.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(L._P64), n, pk.ctypes.data_as(L._P64),
                                    amb.ctypes.data_as(L._P64), words.ctypes.data_as(L._P64), cap, threads), "nt4_pack")
    return pk[:n], amb[:n], words[:nw]


class Index:
    """Host index (``Index``, src/index.rs:33-42)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @classmethod
    def build_index_from_fasta(cls, path: str, w: int = 10, k: int = 15, b: int = 14, flag: int = 0, threads: int = 8) -> "Index":
        h = C.c_void_p()
        check(load().mm2g_index_build_fasta(path.encode(), w, k, b, flag, threads, C.byref(h)), "build_index_from_fasta")
        return cls(h.value)

    @classmethod
    def build_from_seqs(cls, names: Optional[Sequence[str]], seqs: Sequence[bytes], w: int = 10, k: int = 15, b: int = 14,
                        flag: int = 0, threads: int = 8) -> "Index":
        n = len(seqs)
        bufs = [C.create_string_buffer(bytes(s), len(s)) for s in seqs]
        ptrs = (C.c_void_p * max(n, 1))(*[C.cast(x, C.c_void_p).value for x in bufs])
        lens = (C.c_uint64 * max(n, 1))(*[len(s) for s in seqs])
        nm = None
        if names is not None:
            nm = (C.c_char_p * max(n, 1))(*[x.encode() for x in names])
        h = C.c_void_p()
        check(load().mm2g_index_build_seqs(n, nm, ptrs, lens, w, k, b, flag, threads, C.byref(h)), "build_from_seqs")
        return cls(h.value)

    @classmethod
    def build_index_from_fasta_gpu(cls, path: str, w: int = 10, k: int = 15, b: int = 14, flag: int = 0, device: int = 0,
                                   threads: int = 8) -> "Index":
        """The same index built on a GPU (mm2g_index_build_fasta_gpu; HPC / even k build on the host)."""
        h = C.c_void_p()
        check(load().mm2g_index_build_fasta_gpu(path.encode(), w, k, b, flag, device, threads, C.byref(h)),
              "build_index_from_fasta_gpu")
        return cls(h.value)

    @classmethod
    def build_from_buffer(cls, names: Optional[Sequence[str]], buf: np.ndarray, lens: np.ndarray, w: int = 10, k: int = 15,
                          b: int = 14, flag: int = 0, threads: int = 8, device: Optional[int] = None) -> "Index":
        """Index from sequences concatenated in one uint8 buffer (pointers into it; no copies).
        device = a GPU index build (mm2g_index_build_seqs_gpu) instead of the host build."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        lv = np.ascontiguousarray(lens, dtype=np.uint64)
        n = len(lv)
        starts = np.concatenate([[0], np.cumsum(lv)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
        base = buf.ctypes.data
        ptrs = (C.c_void_p * max(n, 1))(*[base + int(x) for x in starts])
        nm = (C.c_char_p * max(n, 1))(*[x.encode() for x in names]) if names is not None else None
        h = C.c_void_p()
        if device is None:
            check(load().mm2g_index_build_seqs(n, nm, ptrs, lv.ctypes.data_as(L._P64), w, k, b, flag, threads, C.byref(h)),
                  "build_from_buffer")
        else:
            check(load().mm2g_index_build_seqs_gpu(n, nm, ptrs, lv.ctypes.data_as(L._P64), w, k, b, flag, device, threads,
                                                   C.byref(h)), "build_from_buffer_gpu")
        return cls(h.value)

    @classmethod
    def load_from_mmi(cls, path: str) -> "Index":
        h = C.c_void_p()
        check(load().mm2g_index_load_mmi(path.encode(), C.byref(h)), "load_from_mmi")
        return cls(h.value)

    def save_to_mmi(self, path: str) -> None:
        check(load().mm2g_index_save_mmi(self._h, path.encode()), "save_to_mmi")

    def close(self) -> None:
        if self._h:
            load().mm2g_index_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def origin(self) -> Tuple[str, Optional[str]]:
        """How the index was made (``mm2g_index_origin``): ("gpu build" | "host build" |
        "gpu build fell back to the host build" | ".mmi load", reason of a fallback or None)."""
        note = C.c_char_p()
        o = check(load().mm2g_index_origin(self._h, C.byref(note)), "index_origin")
        return L.INDEX_ORIGINS.get(o, f"unknown ({o})"), (note.value.decode() if note.value else None)

    def release_tables(self) -> None:
        """Free the host hash tables once the device copies exist (``mm2g_index_release_tables``)."""
        check(load().mm2g_index_release_tables(self._h), "release_tables")

    def stats(self) -> Tuple[int, float, float, int]:
        a, d = C.c_uint64(), C.c_uint64()
        b, c = C.c_double(), C.c_double()
        check(load().mm2g_index_stats(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)), "stats")
        return a.value, b.value, c.value, d.value

    def calc_mid_occ(self, frac: float) -> int:
        out = C.c_int32()
        check(load().mm2g_index_calc_mid_occ(self._h, frac, C.byref(out)), "calc_mid_occ")
        return out.value

    @property
    def params(self) -> Tuple[int, int, int, int, int]:
        w, k, b, f = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        n = C.c_uint32()
        check(load().mm2g_index_params(self._h, C.byref(w), C.byref(k), C.byref(b), C.byref(f), C.byref(n)), "params")
        return w.value, k.value, b.value, f.value, n.value

    def seq(self, rid: int) -> Tuple[Optional[str], int]:
        nm, ln = C.c_char_p(), C.c_uint32()
        check(load().mm2g_index_seq(self._h, rid, C.byref(nm), C.byref(ln)), "seq")
        return (nm.value.decode() if nm.value is not None else None), ln.value

    def get(self, minier: int):
        """``Index::get``: None, ('Single', pos) or ('Multi', [pos, ...])."""
        kind = C.c_int()
        n = load().mm2g_index_get(self._h, minier, C.byref(kind), None, 0)
        if kind.value == 0:
            return None
        buf = (C.c_uint64 * max(n, 1))()
        load().mm2g_index_get(self._h, minier, C.byref(kind), buf, n)
        if kind.value == 1:
            return ("Single", buf[0])
        return ("Multi", list(buf[:n]))


class Device:
    """One MI355X context (stream + device index + batch workspaces)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(load().mm2g_ctx_create(device, C.byref(h)), "ctx_create")
        self._h = h
        self.index: Optional[Index] = None
        self.n_reads = 0

    def close(self) -> None:
        if self._h:
            load().mm2g_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload_index(self, index: Index, mid_occ: int) -> None:
        check(load().mm2g_ctx_upload_index(self._h, index._h, mid_occ), "upload_index")
        self.index = index

    @staticmethod
    def upload_index_many(devs: Sequence["Device"], index: Index, mid_occ: int) -> None:
        """One index copy per context (normally one per GPU), made in parallel host threads."""
        arr = (C.c_void_p * max(len(devs), 1))(*[d._h.value for d in devs])
        check(load().mm2g_ctx_upload_index_many(arr, len(devs), index._h, mid_occ), "upload_index_many")
        for d in devs:
            d.index = index

    def share_index(self, other: "Device", mid_occ: int) -> None:
        """Map against `other`'s device index (same GPU) without another copy."""
        check(load().mm2g_ctx_share_index(self._h, other._h, mid_occ), "share_index")
        self.index = other.index

    def index_mid_occ(self, frac: float) -> int:
        """``Index::calc_mid_occ`` (index.rs:124-141) on the uploaded device
        table (count histogram); equals :meth:`Index.calc_mid_occ`."""
        out = C.c_int32()
        check(load().mm2g_ctx_index_mid_occ(self._h, frac, C.byref(out)), "index_mid_occ")
        return out.value

    def set_mid_occ(self, mid_occ: int) -> None:
        check(load().mm2g_ctx_set_mid_occ(self._h, mid_occ), "set_mid_occ")

    def set_reads(self, seqs: Sequence[bytes]) -> None:
        offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
        if seqs:
            offs[1:] = np.cumsum([len(s) for s in seqs], dtype=np.uint64)
        cat = b"".join(bytes(s) for s in seqs)
        self.set_reads_packed(np.frombuffer(cat, dtype=np.uint8) if cat else np.zeros(1, np.uint8), offs)

    def set_reads_packed(self, seq: np.ndarray, offs: np.ndarray) -> None:
        seq = np.ascontiguousarray(seq, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        n = len(offs) - 1
        check(load().mm2g_batch_set_reads(self._h, seq.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(L._P64), n), "set_reads")
        self.n_reads = n

    def set_reads_nt4(self, lens: np.ndarray, pk_off: np.ndarray, amb_off: np.ndarray, words: np.ndarray) -> None:
        """Stage reads the caller packed (:func:`nt4_pack`)."""
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        pk_off = np.ascontiguousarray(pk_off, dtype=np.uint64)
        amb_off = np.ascontiguousarray(amb_off, dtype=np.uint64)
        words = np.ascontiguousarray(words, dtype=np.uint64)
        b = Nt4Batch(len(lens), lens.ctypes.data_as(L._P64), pk_off.ctypes.data_as(L._P64), amb_off.ctypes.data_as(L._P64),
                     words.ctypes.data_as(L._P64), len(words))
        check(load().mm2g_batch_set_reads_nt4(self._h, C.byref(b)), "set_reads_nt4")
        self.n_reads = len(lens)

    def set_knob(self, name: str, value: int) -> None:
        check(load().mm2g_ctx_set_knob(self._h, L.KNOBS[name], int(value)), "set_knob")

    def get_knob(self, name: str) -> int:
        return check(load().mm2g_ctx_get_knob(self._h, L.KNOBS[name]), "get_knob")

    def seed_batch(self, opts: Optional[MapOpts] = None) -> List[np.ndarray]:
        """``build_anchors_filtered`` for every resident read: list of (A, 2) uint64 (x, y) arrays."""
        o = opts if opts is not None else map_opts()
        n = self.n_reads
        off = np.zeros(n + 1, dtype=np.uint64)
        A = check(load().mm2g_seed_batch(self._h, C.byref(o), off.ctypes.data_as(L._P64), None, 0), "seed_batch")
        xy = np.zeros(2 * max(A, 1), dtype=np.uint64)
        check(load().mm2g_seed_batch(self._h, C.byref(o), off.ctypes.data_as(L._P64), xy.ctypes.data_as(L._P64), A), "seed_batch")
        xy = xy[: 2 * A].reshape(A, 2)
        return [xy[int(off[r]):int(off[r + 1])] for r in range(n)]

    def chain_batch(self, anchors: Sequence[np.ndarray], qlens: Sequence[int], params: Optional[ChainParams] = None,
                    rescue: bool = True, want_dp: bool = False):
        """``chain_dp_all`` (+ ``rescue_long_join``) on caller anchors, one (A, 2) (x, y) array per read.
        Returns (results, chains[, f, pprev]) with per-read numpy arrays."""
        p = params if params is not None else chain_params()
        n = len(anchors)
        cnt = np.array([len(a) for a in anchors], dtype=np.uint64)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum(cnt)
        A = int(off[-1])
        xy = np.ascontiguousarray(np.concatenate([np.asarray(a, np.uint64).reshape(-1, 2) for a in anchors]) if A else
                                  np.zeros((1, 2), np.uint64), dtype=np.uint64)
        ql = np.ascontiguousarray(qlens, dtype=np.int32)
        res = (ChainResult * max(n, 1))()
        ch = np.zeros(max(A, 1), np.uint32)
        f = np.zeros(max(A, 1), np.int32) if want_dp else None
        pp = np.zeros(max(A, 1), np.int32) if want_dp else None
        check(load().mm2g_chain_batch(self._h, C.byref(p), n, off.ctypes.data_as(L._P64), xy.ctypes.data_as(L._P64),
                                      ql.ctypes.data_as(L._PI32), 1 if rescue else 0, res,
                                      f.ctypes.data_as(L._PI32) if want_dp else None, pp.ctypes.data_as(L._PI32) if want_dp else None,
                                      ch.ctypes.data_as(C.POINTER(C.c_uint32))), "chain_batch")
        chains = [ch[int(off[r]):int(off[r]) + res[r].cm].astype(np.int64) for r in range(n)]
        out = [res[r] for r in range(n)]
        if want_dp:
            return out, chains, [f[int(off[r]):int(off[r + 1])] for r in range(n)], [pp[int(off[r]):int(off[r + 1])] for r in range(n)]
        return out, chains

    def sketch_sequences(self, seqs: Sequence[bytes], w: int, k: int, rid: int = 0) -> List[np.ndarray]:
        """``sketch_sequence`` for each sequence; returns (m, 2) uint64 arrays of (key_span, rid_pos_strand)."""
        self.set_reads(seqs)
        n = len(seqs)
        off = np.zeros(n + 1, dtype=np.uint64)
        check(load().mm2g_batch_sketch(self._h, w, k, rid, off.ctypes.data_as(L._P64), None, None, 0), "sketch")
        tot = int(off[-1])
        ks = np.zeros(max(tot, 1), dtype=np.uint64)
        rps = np.zeros(max(tot, 1), dtype=np.uint64)
        check(load().mm2g_batch_sketch(self._h, w, k, rid, off.ctypes.data_as(L._P64), ks.ctypes.data_as(L._P64),
                                       rps.ctypes.data_as(L._P64), tot), "sketch")
        return [np.stack([ks[off[i]:off[i + 1]], rps[off[i]:off[i + 1]]], axis=1) for i in range(n)]

    def map(self, opts: Optional[MapOpts] = None) -> "C.Array[ReadResult]":
        """Run the whole device pipeline on the resident batch and fetch per-read results."""
        o = opts if opts is not None else map_opts()
        check(load().mm2g_batch_map(self._h, C.byref(o)), "batch_map")
        res = (ReadResult * max(self.n_reads, 1))()
        check(load().mm2g_batch_results(self._h, res, self.n_reads), "batch_results")
        return res

    def map_async(self, opts: MapOpts) -> None:
        check(load().mm2g_batch_map(self._h, C.byref(opts)), "batch_map")

    def results(self, n: Optional[int] = None):
        n = self.n_reads if n is None else n
        res = (ReadResult * max(n, 1))()
        check(load().mm2g_batch_results(self._h, res, n), "batch_results")
        return res

    def paf(self, names: Sequence[str], res) -> str:
        n = len(names)
        arr = (C.c_char_p * max(n, 1))(*[x.encode() for x in names])
        need = check(load().mm2g_format_paf(self.index._h, res, arr, n, None, 0), "format_paf")
        buf = C.create_string_buffer(need + 1)
        got = check(load().mm2g_format_paf(self.index._h, res, arr, n, buf, need + 1), "format_paf")
        return buf.raw[:got].decode()

    def batch_paf(self, names: Sequence[str]) -> str:
        """PAF of the batch collected last (mm2g_batch_paf): also the several lines per read of -n <= 1 -m <= k."""
        n = len(names)
        arr = (C.c_char_p * max(n, 1))(*[x.encode() for x in names])
        need = check(load().mm2g_batch_paf(self._h, arr, n, None, 0), "batch_paf")
        buf = C.create_string_buffer(need + 1)
        got = check(load().mm2g_batch_paf(self._h, arr, n, buf, need + 1), "batch_paf")
        return buf.raw[:got].decode()

    def set_debug(self, on: bool) -> None:
        check(load().mm2g_ctx_set_debug(self._h, 1 if on else 0), "set_debug")

    def debug_anchors(self, r: int) -> np.ndarray:
        n = check(load().mm2g_debug_anchors(self._h, r, None, 0), "debug_anchors")
        out = np.zeros(2 * max(n, 1), dtype=np.uint64)
        load().mm2g_debug_anchors(self._h, r, out.ctypes.data_as(L._P64), n)
        return out[: 2 * n].reshape(n, 2)

    def debug_dp(self, r: int) -> Tuple[np.ndarray, np.ndarray]:
        n = check(load().mm2g_debug_dp(self._h, r, None, None, 0), "debug_dp")
        f = np.zeros(max(n, 1), dtype=np.int32)
        p = np.zeros(max(n, 1), dtype=np.int32)
        load().mm2g_debug_dp(self._h, r, f.ctypes.data_as(L._PI32), p.ctypes.data_as(L._PI32), n)
        return f[:n], p[:n]

    def debug_keep(self, r: int) -> np.ndarray:
        n = check(load().mm2g_debug_keep(self._h, r, None, 0), "debug_keep")
        out = np.zeros(max(n, 1), dtype=np.uint8)
        load().mm2g_debug_keep(self._h, r, out.ctypes.data_as(C.POINTER(C.c_uint8)), n)
        return out[:n]

    def prof_enable(self, on: bool = True) -> None:
        check(load().mm2g_prof_enable(self._h, 1 if on else 0), "prof_enable")

    def prof_reset(self) -> None:
        check(load().mm2g_prof_reset(self._h), "prof_reset")

    def prof(self) -> dict:
        out = {}
        i = 0
        while True:
            nm, ms, calls = C.c_char_p(), C.c_double(), C.c_int64()
            if load().mm2g_prof_get(self._h, i, C.byref(nm), C.byref(ms), C.byref(calls)) != 0:
                break
            out[nm.value.decode()] = (ms.value, calls.value)
            i += 1
        return out

    def chain_stats(self) -> np.ndarray:
        """(n, 6) uint32: pass-0/1 ticks (10 ns), anchors in long segments, j-steps, HBM j-steps,
        longest segment | #long segments << 16, per read."""
        n = self.n_reads
        out = np.zeros(6 * max(n, 1), dtype=np.uint32)
        check(load().mm2g_debug_chain_stats(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), n), "chain_stats")
        return out[: 6 * n].reshape(n, 6)

    def counters(self) -> dict:
        keys = ["bases", "minimizers", "kept_minimizers", "anchors", "rescued_anchors", "dp_pairs", "dp_anchors",
                "long_anchors", "giant_anchors", "med_anchors", "long_anchors_rescue", "giant_anchors_rescue", "med_anchors_rescue",
                "seg_stream_anchors", "lb_stream_anchors", "seg_stream_rescue", "fused_anchors", "fused_minimizers",
                "sort_small_anchors", "sort_cell_anchors", "sort_whole_anchors",
                "fused_big_anchors", "fused_big_minimizers"]
        buf = (C.c_uint64 * len(keys))()
        check(load().mm2g_batch_counters(self._h, buf, len(keys)), "counters")
        return dict(zip(keys, list(buf)))


def align(index: Index, names: Sequence[str], seqs: Sequence[bytes], frac: float = 2e-4, device: int = 0,
          opts: Optional[MapOpts] = None, dev: Optional[Device] = None) -> str:
    """The Align flow (main.rs:189-230) applied to every read; returns PAF text."""
    mid = max(index.calc_mid_occ(frac), 10)
    d = dev or Device(device)
    if d.index is not index:
        d.upload_index(index, mid)
    d.set_reads(seqs)
    res = d.map(opts)
    return d.batch_paf(list(names))


def multi_chain_lines(xy: np.ndarray, f: np.ndarray, pprev: np.ndarray, qlen: int, mini_pos: np.ndarray, avg_k: float,
                      tlen: np.ndarray, opts: Optional[MapOpts] = None):
    """mm2g_multi_chain_lines (host only): the -n <= 1 -m <= k epilogue of one read -> (lines, panic)."""
    o = opts if opts is not None else map_opts(min_cnt=1, min_chain_score=15)
    a = np.ascontiguousarray(xy, dtype=np.uint64).reshape(-1)
    n = len(a) // 2
    f32 = np.ascontiguousarray(f, dtype=np.int32)
    p32 = np.ascontiguousarray(pprev, dtype=np.int32)
    mp = np.ascontiguousarray(mini_pos, dtype=np.int32)
    tl = np.ascontiguousarray(tlen, dtype=np.uint32)
    cap = max(n, 1) + 8
    out = (ChainLine * cap)()
    pan = C.c_int32(0)
    I32 = C.POINTER(C.c_int32)
    m = load().mm2g_multi_chain_lines(a.ctypes.data_as(L._P64), f32.ctypes.data_as(I32), p32.ctypes.data_as(I32), n, int(qlen),
                                      mp.ctypes.data_as(I32), len(mp), float(avg_k), tl.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      len(tl), C.byref(o), out, cap, C.byref(pan))
    if pan.value:
        return [], True
    check(m, "multi_chain_lines")
    return [out[i] for i in range(min(m, cap))], False

