"""MI355X-native Multi-BRWT row-query engine (drop-in for the BRWT get_row
path of ratschlab/genome_graph_annotation).

The product is libmbrwt.so (HIP kernels for gfx950 behind the C ABI in
include/mbrwt.h, plus the BinRel-WT engine of include/mbrwt_wt.h).  Python modules here are thin bindings used by the tests
and bench.py; there is no CPU fallback anywhere in the package.
"""
from ._lib import MBRWTError, lib  # noqa: F401
from .binrel_wt import BinRelWTDevice  # noqa: F401
from .brwt import BRWTDevice, BRWTMulti  # noqa: F401

__all__ = ["BRWTDevice", "BRWTMulti", "BinRelWTDevice", "MBRWTError", "lib"]
