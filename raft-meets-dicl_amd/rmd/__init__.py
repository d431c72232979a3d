"""rmd — MI355X-native (gfx950) cost-volume backend for qzed/raft-meets-dicl.

Drop-in host mirror of the reference's hot-path modules; every compute call goes through the C ABI
of librmd.so (include/rmd.h) on the current HIP stream.  No CPU fallback.

  rmd.raft.CorrBlock      <- src/models/impls/raft.py:15-95
"""

from . import blocks, corr, dicl, ops, raft  # noqa: F401
from .ops import set_default_precision, get_default_precision  # noqa: F401

__version__ = "0.1"
