"""ctypes binding of libmm2g.so (include/mm2g.h).

The shared library is built in-tree by ``__graft_entry__.build()`` into
``minimap2_rs_amd/build/``.  There is no fallback: if the library is missing
or a device call fails, the error is raised — the product path never routes
through the CPU oracle.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(HERE, "build")
LIB_PATH = os.environ.get("MM2G_LIB") or os.path.join(BUILD_DIR, "libmm2g.so")
CLI_PATH = os.path.join(BUILD_DIR, "mm2rs")

MM2G_R_MAPPED = 1
MM2G_R_RESCUED = 2
MM2G_R_DV_FOUND = 4
MM2G_R_PANIC = 8
MM2G_R_EMPTY = 16


class MapOpts(C.Structure):
    _fields_ = [("w", C.c_int32), ("k", C.c_int32), ("max_gap", C.c_int32), ("bw", C.c_int32), ("bw_long", C.c_int32),
                ("min_cnt", C.c_int32), ("min_chain_score", C.c_int32), ("mask_level", C.c_float),
                ("pri_ratio", C.c_float), ("best_n", C.c_int32)]


class ReadResult(C.Structure):
    _fields_ = [("flags", C.c_int32), ("n_anchors", C.c_int32), ("score", C.c_int32), ("cm", C.c_int32),
                ("qs", C.c_int32), ("qe", C.c_int32), ("ts", C.c_int32), ("te", C.c_int32),
                ("rid", C.c_int32), ("rev", C.c_int32), ("n_match", C.c_int32), ("dv_st", C.c_int32),
                ("dv_en", C.c_int32), ("m_dv", C.c_int32), ("sum_k", C.c_int64), ("qlen", C.c_int32), ("dv", C.c_float)]


assert C.sizeof(ReadResult) == 72


class Nt4Batch(C.Structure):
    _fields_ = [("n_reads", C.c_uint32), ("lens", C.POINTER(C.c_uint64)), ("pk_off", C.POINTER(C.c_uint64)),
                ("amb_off", C.POINTER(C.c_uint64)), ("words", C.POINTER(C.c_uint64)), ("n_words", C.c_uint64)]


class ChainParams(C.Structure):
    _fields_ = [("max_dist_x", C.c_int32), ("max_dist_y", C.c_int32), ("bw", C.c_int32), ("max_chain_iter", C.c_int32),
                ("min_chain_score", C.c_int32), ("min_cnt", C.c_int32), ("chn_pen_gap", C.c_float), ("chn_pen_skip", C.c_float),
                ("max_chain_skip", C.c_int32), ("max_drop", C.c_int32), ("bw_long", C.c_int32), ("rmq_rescue_size", C.c_int32),
                ("rmq_rescue_ratio", C.c_float)]


class ChainResult(C.Structure):
    _fields_ = [("flags", C.c_int32), ("n_anchors", C.c_int32), ("score", C.c_int32), ("cm", C.c_int32), ("qs", C.c_int32),
                ("qe", C.c_int32), ("ts", C.c_int32), ("te", C.c_int32), ("rid", C.c_int32), ("rev", C.c_int32)]


class ChainLine(C.Structure):
    _fields_ = [("qs", C.c_int32), ("qe", C.c_int32), ("ts", C.c_int32), ("te", C.c_int32), ("rid", C.c_int32),
                ("rev", C.c_int32), ("cm", C.c_int32), ("primary", C.c_int32), ("dv", C.c_float), ("s1", C.c_int32),
                ("s2", C.c_int32)]


# knobs (include/mm2g.h)
KNOBS = {"sort_small": 1, "seg_small": 2, "seg_chunk": 3, "giant_min": 4, "giant_min0": 5, "giant_lcap": 6, "giant_gmax": 7,
         "giant_gblocks": 8, "filter": 9, "lazy": 10, "prune": 11, "giant": 12, "sketch_prof": 13, "sort_prof": 14,
         "lseg_prof": 15, "midhist_bins": 16, "sync_each": 17, "host_threads": 18, "ws_min": 19,
         "sort_lds_kb": 20, "stop_at": 21, "spec_rounds": 22, "med_pairs": 23, "med_pairs_rescue": 24, "ws_fail": 25, "sketch_view": 27, "prune_rescue": 29, "view_reads": 30, "seg_sparse": 31, "spec_batch": 32, "dv_par": 33, "seed_fuse": 36, "sketch_x32": 37, "big_wnd": 38, "cands_longw": 39, "seed_fuse_big": 40, "read_tiny": 41, "big_tiny": 42, "spec_eval": 43, "small_reg": 44}
INDEX_KNOBS = {"ixchunk": 1, "ixprof": 2, "load_threads": 3, "gpu_strict": 4, "force_fallback": 5, "ixsortv": 6}
# mm2g_index_origin values
INDEX_ORIGINS = {1: "host build", 2: "gpu build", 3: "gpu build fell back to the host build", 4: ".mmi load"}

_VP = C.c_void_p
_P64 = C.POINTER(C.c_uint64)
_PI32 = C.POINTER(C.c_int32)

# name -> (restype, argtypes); every entry point declared in include/mm2g.h
SIGNATURES = {
    "mm2g_version": (C.c_int, []),
    "mm2g_last_error": (C.c_char_p, []),
    "mm2g_device_count": (C.c_int, []),
    "mm2g_index_build_fasta": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]),
    "mm2g_index_build_seqs": (C.c_int, [C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p), _P64,
                                        C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]),
    "mm2g_index_build_fasta_gpu": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]),
    "mm2g_index_build_seqs_gpu": (C.c_int, [C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p), _P64,
                                            C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]),
    "mm2g_index_load_mmi": (C.c_int, [C.c_char_p, C.POINTER(_VP)]),
    "mm2g_index_save_mmi": (C.c_int, [_VP, C.c_char_p]),
    "mm2g_index_free": (None, [_VP]),
    "mm2g_index_stats": (C.c_int, [_VP, _P64, C.POINTER(C.c_double), C.POINTER(C.c_double), _P64]),
    "mm2g_index_calc_mid_occ": (C.c_int, [_VP, C.c_float, _PI32]),
    "mm2g_index_params": (C.c_int, [_VP, _PI32, _PI32, _PI32, _PI32, C.POINTER(C.c_uint32)]),
    "mm2g_index_seq": (C.c_int, [_VP, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_uint32)]),
    "mm2g_index_get": (C.c_int64, [_VP, C.c_uint64, C.POINTER(C.c_int), _P64, C.c_int64]),
    "mm2g_ctx_create": (C.c_int, [C.c_int, C.POINTER(_VP)]),
    "mm2g_ctx_destroy": (None, [_VP]),
    "mm2g_ctx_upload_index": (C.c_int, [_VP, _VP, C.c_int32]),
    "mm2g_ctx_upload_index_many": (C.c_int, [C.POINTER(_VP), C.c_int, _VP, C.c_int32]),
    "mm2g_index_origin": (C.c_int, [_VP, C.POINTER(C.c_char_p)]),
    "mm2g_index_release_tables": (C.c_int, [_VP]),
    "mm2g_map_opts_default": (None, [C.POINTER(MapOpts)]),
    "mm2g_batch_set_reads": (C.c_int, [_VP, C.c_void_p, _P64, C.c_uint32]),
    "mm2g_batch_map": (C.c_int, [_VP, C.POINTER(MapOpts)]),
    "mm2g_batch_results": (C.c_int, [_VP, C.POINTER(ReadResult), C.c_uint32]),
    "mm2g_format_paf": (C.c_int64, [_VP, C.POINTER(ReadResult), C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.c_int64]),
    "mm2g_batch_paf": (C.c_int64, [_VP, C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p, C.c_int64]),
    "mm2g_multi_chain_lines": (C.c_int64, [_P64, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int64, C.c_int32,
                                           C.POINTER(C.c_int32), C.c_int64, C.c_float, C.POINTER(C.c_uint32), C.c_uint32,
                                           C.POINTER(MapOpts), C.POINTER(ChainLine), C.c_int64, C.POINTER(C.c_int32)]),
    "mm2g_batch_sketch": (C.c_int, [_VP, C.c_int, C.c_int, C.c_uint32, _P64, _P64, _P64, C.c_uint64]),
    "mm2g_ctx_set_debug": (C.c_int, [_VP, C.c_int]),
    "mm2g_debug_anchors": (C.c_int64, [_VP, C.c_uint32, _P64, C.c_int64]),
    "mm2g_debug_dp": (C.c_int64, [_VP, C.c_uint32, _PI32, _PI32, C.c_int64]),
    "mm2g_debug_keep": (C.c_int64, [_VP, C.c_uint32, C.POINTER(C.c_uint8), C.c_int64]),
    "mm2g_prof_enable": (C.c_int, [_VP, C.c_int]),
    "mm2g_prof_get": (C.c_int, [_VP, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "mm2g_prof_reset": (C.c_int, [_VP]),
    "mm2g_debug_chain_stats": (C.c_int64, [_VP, C.POINTER(C.c_uint32), C.c_uint32]),
    "mm2g_ctx_share_index": (C.c_int, [_VP, _VP, C.c_int32]),
    "mm2g_ctx_index_mid_occ": (C.c_int, [_VP, C.c_float, _PI32]),
    "mm2g_ctx_set_mid_occ": (C.c_int, [_VP, C.c_int32]),
    "mm2g_batch_counters": (C.c_int, [_VP, _P64, C.c_int]),
    "mm2g_nt4_words_bound": (C.c_uint64, [_P64, C.c_uint32]),
    "mm2g_nt4_pack": (C.c_int64, [C.c_void_p, _P64, C.c_uint32, _P64, _P64, _P64, C.c_uint64, C.c_int]),
    "mm2g_batch_set_reads_nt4": (C.c_int, [_VP, C.POINTER(Nt4Batch)]),
    "mm2g_seed_batch": (C.c_int64, [_VP, C.POINTER(MapOpts), _P64, _P64, C.c_uint64]),
    "mm2g_chain_params_default": (None, [C.POINTER(ChainParams), C.c_int]),
    "mm2g_chain_batch": (C.c_int, [_VP, C.POINTER(ChainParams), C.c_uint32, _P64, _P64, _PI32, C.c_int, C.POINTER(ChainResult),
                                   _PI32, _PI32, C.POINTER(C.c_uint32)]),
    "mm2g_ctx_set_knob": (C.c_int, [_VP, C.c_int, C.c_int64]),
    "mm2g_ctx_get_knob": (C.c_int64, [_VP, C.c_int]),
    "mm2g_set_index_knob": (C.c_int, [C.c_int, C.c_int64]),
}

_lib = None


class Mm2gError(RuntimeError):
    pass


def load() -> C.CDLL:
    """Load libmm2g.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise Mm2gError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str = "") -> int:
    if status < 0:
        msg = load().mm2g_last_error().decode(errors="replace")
        raise Mm2gError(f"{what}: status {status}: {msg}")
    return status
