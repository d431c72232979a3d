"""Drop-in for corr.dot.CorrelationModule — src/models/common/corr/dot.py:8-66.

Single-level windowed dot-product cost: for displacement (a, b) the reference grid-samples fmap2
at coords + (a-r, b-r) (normalised with fmap1's size, :39-41), dots it with fmap1 and divides by
sqrt(C) (:55-57), then applies the displacement-aware projection (:63-64).  That is one level of
the RAFT pyramid lookup, so it runs as rmd_corr_pyramid (levels = 1, scale 1/sqrt(C)) + one
rmd_corr_lookup, and `dap` stays the reference's module (state_dict key `dap.conv1.weight`, forward
hooks intact).  fmap2 must have fmap1's spatial size — the reference's own callers always pass
equal sizes (a different size would make its normalisation sample a rescaled grid).
"""

import torch
import torch.nn as nn

from .. import raft
from ..blocks.dicl import DisplacementAwareProjection


def _delta(radius):
    r = torch.linspace(-radius, radius, 2 * radius + 1)
    return torch.stack(torch.meshgrid(r, r, indexing="ij"), dim=-1)     # (2r+1, 2r+1, 2)


class CorrelationModule(nn.Module):
    def __init__(self, radius, dap_init="identity", precision=None):
        super().__init__()
        self.radius = radius
        self.precision = precision
        self.dap = DisplacementAwareProjection((radius, radius), init=dap_init)
        self.register_buffer("delta", _delta(radius), persistent=False)
        self.output_dim = (2 * self.radius + 1) ** 2

    def forward(self, f1, f2, coords, dap=True):
        batch, _, h, w = f1.shape
        if tuple(f2.shape) != tuple(f1.shape):
            raise ValueError(f"corr.dot: fmap2 {tuple(f2.shape)} must match fmap1 {tuple(f1.shape)}")
        r = self.radius
        corr = raft.CorrBlock(f1, f2, num_levels=1, radius=r, precision=self.precision)(coords)
        corr = corr.view(batch, 2 * r + 1, 2 * r + 1, h, w)
        if dap:
            corr = self.dap(corr)
        return corr.reshape(batch, -1, h, w)


# single-level soft-argmax regressions of this module (reference classes of the same names)
from ..heads import CorrSoftArgMaxFlowRegression as SoftArgMaxFlowRegression  # noqa: E402,F401
from ..heads import CorrSoftArgMaxFlowRegressionWithDap as SoftArgMaxFlowRegressionWithDap  # noqa: E402,F401
