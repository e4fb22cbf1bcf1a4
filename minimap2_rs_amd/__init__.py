"""minimap2_rs_amd — MI355X-native sketch -> seed -> chain path of mm2rs.

The compute lives in libmm2g.so (hand-written HIP kernels for gfx950 plus a
C++ host, C ABI in include/mm2g.h); this package is the thin Python binding
used by tests and bench.py.
"""
from ._lib import Mm2gError, load  # noqa: F401
from .api import Device, Index, Minimizer, align, map_opts  # noqa: F401

__all__ = ["Device", "Index", "Minimizer", "align", "map_opts", "load", "Mm2gError"]
