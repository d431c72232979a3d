"""Drop-in for raft.CorrBlock — qzed/raft-meets-dicl src/models/impls/raft.py:15-95.

Same constructor and call signature; the all-pairs volume and its pooled pyramid are built by one
MFMA GEMM launch with a pooling epilogue (rmd_corr_pyramid) and each lookup is one bandwidth-bound
gather launch (rmd_corr_lookup).  Output: contiguous float32 (B, L*(2r+1)^2, H, W), as raft.py:95.

Training: when the feature maps require gradients (and grad mode is on) the block is an autograd
node — the lookups' backward passes accumulate one dense pyramid gradient (rmd_corr_lookup_backward)
and the pyramid's backward turns it into d fmap1 / d fmap2 (ops._CorrPyramidFn), matching the
reference's autograd through grid_sample / avg_pool2d / matmul.  Coordinates get no gradient
(the reference detaches them, raft.py:402).
"""

import torch

from . import ops


class CorrBlock:
    """Correlation volume for matching costs (drop-in for raft.CorrBlock)."""

    scale = None            # 1/sqrt(C) (raft.py:33); raft_fs.CorrBlock overrides with 1.0

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, precision=None):
        self.num_levels = num_levels
        self.radius = radius
        self.precision = precision or ops.get_default_precision()
        self._state = self._token = None
        if torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad):
            self.pyramid, self._state, self._token = ops.corr_block_autograd(fmap1, fmap2, num_levels,
                                                                             self.precision, self.scale)
        else:
            self.pyramid = ops.corr_pyramid(fmap1, fmap2, num_levels, self.precision, scale=self.scale)

    @property
    def corr_pyramid(self):
        """Levels in the reference layout (B, H, W, 1, H_i, W_i) — unpacked copies, for inspection."""
        return [self.pyramid.unpack(i) for i in range(self.num_levels)]

    def __call__(self, coords, mask_costs=[]):
        if self._token is not None and torch.is_grad_enabled():
            return ops.corr_lookup_autograd(self._token, self._state, coords, self.radius, mask_costs)
        return ops.corr_lookup(self.pyramid, coords, self.radius, mask_costs)


# per-iteration heads of raft.py (Up8Network :299-331, soft-argmax regressions :98-190)
from .heads import (Up8Network, SoftArgMaxFlowRegression, SoftArgMaxFlowRegressionWithDap,  # noqa: E402,F401
                    make_flow_regression)
