"""rmd — MI355X-native (gfx950) cost-volume backend for qzed/raft-meets-dicl.

Drop-in host mirror of the reference's hot-path modules; every compute call on GPU tensors goes
through the C ABI of librmd.so (include/rmd.h) on the current HIP stream and raises if the library
is missing.  CPU tensors dispatch to the operators' CPU kernels (rmd/cpu.py: the reference's ATen
algorithm), so the modules also run on device='cpu' as the reference's do.

  rmd.raft.CorrBlock                    <- src/models/impls/raft.py:15-95
  rmd.raft_fs.CorrBlock                 <- src/models/impls/raft_fs.py:13-87
  rmd.corr.make_cmod / CorrelationModule <- src/models/common/corr/{dicl,dicl_1x1,dicl_emb,dot}.py
  rmd.raft_dicl_ml.CorrelationModule    <- src/models/impls/raft_dicl_ml.py:235-343
  rmd.blocks.dicl                       <- src/models/common/blocks/dicl.py:93-150
  rmd.dicl.compute_cost                 <- src/models/impls/dicl.py:171-241 (+ fused warp)
  rmd.warp.warp_backwards               <- src/models/common/warp.py:5-33
  rmd.raft.Up8Network / SoftArgMax*     <- src/models/impls/raft.py:98-190,299-331 (rmd.heads)
  rmd.input.InputSpec / ModuloPadding   <- src/models/input.py:32-313 (frame pair + flow target format)
"""

from . import blocks, config, corr, cpu, dicl, heads, input, ops, raft, raft_dicl_ml, raft_fs, warp  # noqa: F401
from .ops import set_default_precision, get_default_precision  # noqa: F401

__version__ = "0.1"
