"""minimap2_rs_amd — MI355X-native sketch -> seed -> chain path of mm2rs.

The compute lives in libmm2g.so (hand-written HIP kernels for gfx950 plus a
C++ host, C ABI in include/mm2g.h); this package is the thin Python binding
used by tests and bench.py.
"""
from ._lib import Mm2gError, load  # noqa: F401
from .api import Device, Index, Minimizer, align, chain_params, map_opts, multi_chain_lines, nt4_pack, set_index_knob  # noqa: F401

__all__ = ["Device", "Index", "Minimizer", "align", "chain_params", "map_opts", "multi_chain_lines", "nt4_pack", "set_index_knob", "load", "Mm2gError"]
