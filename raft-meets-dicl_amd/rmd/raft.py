"""Drop-in for raft.CorrBlock — qzed/raft-meets-dicl src/models/impls/raft.py:15-95.

Same constructor and call signature; the all-pairs volume and its pooled pyramid are built by one
MFMA GEMM launch with a pooling epilogue (rmd_corr_pyramid) and each lookup is one bandwidth-bound
gather launch (rmd_corr_lookup).  Output: contiguous float32 (B, L*(2r+1)^2, H, W), as raft.py:95.
"""

from . import ops


class CorrBlock:
    """Correlation volume for matching costs (drop-in for raft.CorrBlock)."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, precision=None):
        self.num_levels = num_levels
        self.radius = radius
        self.precision = precision or ops.get_default_precision()
        self.pyramid = ops.corr_pyramid(fmap1, fmap2, num_levels, self.precision)

    @property
    def corr_pyramid(self):
        """Levels in the reference layout (B, H, W, 1, H_i, W_i) — unpacked copies, for inspection."""
        return [self.pyramid.unpack(i) for i in range(self.num_levels)]

    def __call__(self, coords, mask_costs=[]):
        return ops.corr_lookup(self.pyramid, coords, self.radius, mask_costs)
