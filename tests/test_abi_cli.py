"""CPU: the C-ABI boundary and the host-only parts of the product.

* libmm2g.so loads without a GPU and exports every function include/mm2g.h
  declares (the drop-in boundary);
* mm2g_format_paf (write_paf, src/paf.rs:224-236) formats results exactly;
* `mm2rs index` (src/main.rs:147-158) prints the reference's stats lines and
  writes the same .mmi bytes as the oracle CLI."""
import ctypes as C
import json
import os
import re
import subprocess

import pytest

import minimap2_rs_amd as M
from minimap2_rs_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mm2g.h")
GOLD = os.path.join(ROOT, "tests", "golden", "world.json")


def _declared():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mm2g_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    names = _declared()
    assert len(names) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mm2g_[a-z0-9_]+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    lib = C.CDLL(L.LIB_PATH)
    for n in names:
        getattr(lib, n)


def test_python_binding_covers_header():
    assert set(_declared()) <= set(L.SIGNATURES), sorted(set(_declared()) - set(L.SIGNATURES))


def test_library_loads_without_gpu():
    lib = M.load()
    assert lib.mm2g_version() >= 1
    assert lib.mm2g_device_count() >= 0
    assert isinstance(lib.mm2g_last_error(), bytes)


def test_errors_are_status_codes():
    lib = M.load()
    assert lib.mm2g_index_load_mmi(b"/nonexistent.mmi", C.byref(C.c_void_p())) == -2   # MM2G_E_IO
    assert b"" != lib.mm2g_last_error()


@pytest.fixture(scope="module")
def gold_ref(tmp_path_factory):
    w = json.load(open(GOLD))
    td = tmp_path_factory.mktemp("abi")
    ref = str(td / "ref.fa")
    with open(ref, "w") as fh:
        for n, s in w["contigs"]:
            fh.write(f">{n}\n{s}\n")
    return ref, w


def _result(**kw):
    r = L.ReadResult()
    for k, v in kw.items():
        setattr(r, k, v)
    return r


def test_format_paf(gold_ref):
    ref, w = gold_ref
    idx = M.Index.build_index_from_fasta(ref, 10, 15, 14, 0, 2)
    res = (L.ReadResult * 4)()
    res[0] = _result(flags=1, score=123, cm=40, qs=10, qe=2010, ts=100, te=2105, rid=0, rev=0, qlen=2500, dv=0.0123)
    res[1] = _result(flags=1, score=-5, cm=3, qs=0, qe=500, ts=0, te=510, rid=2, rev=1, qlen=600, dv=0.00004999)
    res[2] = _result(flags=0, qlen=100)                                   # no chain: no line
    res[3] = _result(flags=1 | 8, score=50, cm=5, qs=1, qe=2, rid=0x7fffffff, rev=1, qlen=30)   # reference panics
    names = (C.c_char_p * 4)(b"r0", b"r1", b"r2", b"r3")
    lib = M.load()
    n = lib.mm2g_format_paf(idx._h, res, names, 4, None, 0)
    buf = C.create_string_buffer(n + 1)
    assert lib.mm2g_format_paf(idx._h, res, names, 4, buf, n + 1) == n
    lines = buf.raw[:n].decode().splitlines()
    lc = {c[0]: len(c[1]) for c in w["contigs"]}
    assert lines == [
        f"r0\t2500\t10\t2010\t+\tchrA\t{lc['chrA']}\t100\t2105\t2000\t2005\t60\ttp:A:P\tcm:i:40\ts1:i:123\ts2:i:0\tdv:f:0.0123\trl:i:0",
        f"r1\t600\t100\t600\t-\tchrC\t{lc['chrC']}\t0\t510\t500\t510\t60\ttp:A:P\tcm:i:3\ts1:i:0\ts2:i:0\tdv:f:0.0000\trl:i:0",
    ]
    assert lib.mm2g_format_paf(idx._h, res, names, 4, buf, 10) == -4       # buffer too small: MM2G_E_NOMEM


def test_cli_index_matches_oracle(gold_ref, tmp_path):
    ref, _ = gold_ref
    mm2rs = os.path.join(ROOT, "minimap2_rs_amd", "build", "mm2rs")
    cpu = os.path.join(ROOT, "oracle", "build", "mm2rs-cpu")
    a, b = str(tmp_path / "gpu.mmi"), str(tmp_path / "cpu.mmi")
    o1 = subprocess.run([mm2rs, "index", ref, "-d", a, "-t", "2"], capture_output=True, text=True, check=True)
    o2 = subprocess.run([cpu, "index", ref, "-d", b, "-t", "2"], capture_output=True, text=True, check=True)
    assert o1.stdout == o2.stdout and o1.stdout.strip()
    assert open(a, "rb").read() == open(b, "rb").read()
    o3 = subprocess.run([mm2rs, "index", ref, "-d", a, "-H", "-w", "7", "-k", "13"], capture_output=True, text=True, check=True)
    o4 = subprocess.run([cpu, "index", ref, "-d", b, "-H", "-w", "7", "-k", "13"], capture_output=True, text=True, check=True)
    assert o3.stdout == o4.stdout
    assert open(a, "rb").read() == open(b, "rb").read()


def test_cli_usage_errors():
    mm2rs = os.path.join(ROOT, "minimap2_rs_amd", "build", "mm2rs")
    assert subprocess.run([mm2rs], capture_output=True).returncode != 0
    assert subprocess.run([mm2rs, "index", "/nonexistent.fa"], capture_output=True).returncode != 0


def test_index_origin_and_forced_fallback(tmp_path):
    """mm2g_index_origin tells how an index was made; a GPU build the device
    cannot do falls back to the host build and says so (forced here by
    MM2G_IKNOB_FORCE_FALLBACK, which returns before any device call, so this
    runs without a GPU).  The fallback index equals the host build byte for
    byte; released tables refuse later use but keep the stats."""
    import numpy as np
    import minimap2_rs_amd as M
    from tools import simdata
    names, lens, g = simdata.genome("small", 1.0, 11)
    ih = M.Index.build_from_buffer(names, g, lens, threads=2)
    assert ih.origin == ("host build", None)
    M.set_index_knob("force_fallback", 1)
    try:
        ig = M.Index.build_from_buffer(names, g, lens, threads=2, device=0)
    finally:
        M.set_index_knob("force_fallback", 0)
    kind, why = ig.origin
    assert kind == "gpu build fell back to the host build" and "forced" in why
    ig.save_to_mmi(str(tmp_path / "g.mmi"))
    ih.save_to_mmi(str(tmp_path / "h.mmi"))
    assert open(tmp_path / "g.mmi", "rb").read() == open(tmp_path / "h.mmi", "rb").read()
    im = M.Index.load_from_mmi(str(tmp_path / "g.mmi"))
    assert im.origin == (".mmi load", None)
    st = im.stats()
    im.release_tables()
    assert im.stats() == st
    with pytest.raises(M.Mm2gError if hasattr(M, "Mm2gError") else Exception):
        im.calc_mid_occ(2e-4)
    with pytest.raises(Exception):
        im.save_to_mmi(str(tmp_path / "x.mmi"))
    assert im.seq(0)[1] == int(lens[0])
