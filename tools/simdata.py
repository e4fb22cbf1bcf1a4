"""Python binding of tools/simgen.c (seeded synthetic references and
ONT-shaped reads).  Used by tests, smoke() and bench.py."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libsimgen.so")
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = C.CDLL(LIB)
        L.sim_genome_layout.restype = C.c_int
        L.sim_genome_layout.argtypes = [C.c_char_p, C.c_double, C.POINTER(C.c_int64), C.c_char_p, C.c_int]
        L.sim_genome_fill.restype = C.c_int
        L.sim_genome_fill.argtypes = [C.c_char_p, C.c_double, C.c_uint64, C.c_void_p, C.c_int]
        L.sim_reads.restype = C.c_int64
        L.sim_reads.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_int, C.c_int64, C.c_int64, C.c_uint64,
                                C.c_void_p, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        _lib = L
    return _lib


def genome(preset: str, scale: float, seed: int, threads: int = 8) -> Tuple[List[str], np.ndarray, np.ndarray]:
    """-> (names, lens[int64], concatenated sequence bytes as uint8 array)."""
    L = lib()
    lens = (C.c_int64 * 64)()
    names = C.create_string_buffer(64 * 16)
    n = L.sim_genome_layout(preset.encode(), scale, lens, names, 64)
    if n < 0:
        raise ValueError(f"unknown preset {preset}")
    lv = np.array(lens[:n], dtype=np.int64)
    buf = np.empty(int(lv.sum()), dtype=np.uint8)
    assert L.sim_genome_fill(preset.encode(), scale, seed, buf.ctypes.data_as(C.c_void_p), threads) == 0
    nm = [names.raw[16 * i:16 * i + 16].split(b"\0")[0].decode() for i in range(n)]
    return nm, lv, buf


def reads(genome_buf: np.ndarray, lens: np.ndarray, n_reads: int, read_len: int, seed: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """-> (concatenated read bases uint8, offsets uint64[n+1], origin int64[n,4])."""
    L = lib()
    cap = int(n_reads * read_len * 1.2) + 4096
    out = np.empty(cap, dtype=np.uint8)
    offs = np.zeros(n_reads + 1, dtype=np.int64)
    origin = np.zeros(4 * n_reads, dtype=np.int64)
    lv = (C.c_int64 * len(lens))(*[int(x) for x in lens])
    tot = L.sim_reads(genome_buf.ctypes.data_as(C.c_void_p), lv, len(lens), n_reads, read_len, seed,
                      out.ctypes.data_as(C.c_void_p), cap, offs.ctypes.data_as(C.POINTER(C.c_int64)),
                      origin.ctypes.data_as(C.POINTER(C.c_int64)))
    if tot < 0:
        raise RuntimeError("read simulation failed")
    return out[:tot], offs.astype(np.uint64), origin.reshape(n_reads, 4)


def write_fasta(path: str, names, seqs) -> None:
    with open(path, "wb") as fh:
        for nm, s in zip(names, seqs):
            fh.write(b">" + nm.encode() + b"\n")
            s = bytes(s)
            for i in range(0, len(s), 80):
                fh.write(s[i:i + 80] + b"\n")


def write_genome(preset: str, scale: float, seed: int, path: str) -> None:
    names, lens, buf = genome(preset, scale, seed)
    offs = np.concatenate([[0], np.cumsum(lens)])
    write_fasta(path, names, [buf[offs[i]:offs[i + 1]].tobytes() for i in range(len(names))])


def read_fasta_seqs(path: str):
    names, seqs, cur = [], [], None
    with open(path, "rb") as fh:
        for line in fh:
            line = line.rstrip(b"\r\n")
            if line.startswith(b">"):
                if cur is not None:
                    seqs.append(b"".join(cur))
                names.append(line[1:].split()[0].decode() if len(line) > 1 else "")
                cur = []
            elif cur is not None:
                cur.append(line)
    if cur is not None:
        seqs.append(b"".join(cur))
    return names, seqs


def write_reads(ref_fa: str, n: int, length: int, seed: int, path: str) -> None:
    names, seqs = read_fasta_seqs(ref_fa)
    lens = np.array([len(s) for s in seqs], dtype=np.int64)
    g = np.frombuffer(b"".join(seqs), dtype=np.uint8)
    rb, offs, _ = reads(g, lens, n, length, seed)
    write_fasta(path, [f"r{i}" for i in range(n)], [rb[offs[i]:offs[i + 1]].tobytes() for i in range(n)])
