"""Drop-in for corr.dicl.CorrelationModule — src/models/common/corr/dicl.py:8-61.

The grid_sample / expand / cat that build the (B, 2r+1, 2r+1, 2C, h, w) MatchingNet input
(:36-54) run as one rmd_dicl_stack pass; `mnet` and `dap` stay the reference's modules (names,
parameters and forward hooks unchanged).
"""

import torch
import torch.nn as nn

from .. import ops
from ..blocks.dicl import DisplacementAwareProjection, MatchingNet


def _delta(radius):
    r = torch.linspace(-radius, radius, 2 * radius + 1)
    return torch.stack(torch.meshgrid(r, r, indexing="ij"), dim=-1)     # (2r+1, 2r+1, 2)


class CorrelationModule(nn.Module):
    def __init__(self, feature_dim, radius, dap_init="identity", norm_type="batch", relu_inplace=True,
                 mnet_scale=1):
        super().__init__()
        self.radius = radius
        self.mnet = MatchingNet(2 * feature_dim, norm_type=norm_type, relu_inplace=relu_inplace, scale=mnet_scale)
        self.dap = DisplacementAwareProjection((radius, radius), init=dap_init)
        self.register_buffer("delta", _delta(radius), persistent=False)
        self.output_dim = (2 * self.radius + 1) ** 2

    def forward(self, f1, f2, coords, dap=True):
        batch, _, h, w = f1.shape
        stack = ops.dicl_stack(f1, f2, coords, self.radius)          # (B, 2r+1, 2r+1, 2C, h, w)
        cost = self.mnet(stack)
        if dap:
            cost = self.dap(cost)
        return cost.reshape(batch, -1, h, w)


# single-level soft-argmax regressions of this module (reference classes of the same names)
from ..heads import CorrSoftArgMaxFlowRegression as SoftArgMaxFlowRegression  # noqa: E402,F401
from ..heads import CorrSoftArgMaxFlowRegressionWithDap as SoftArgMaxFlowRegressionWithDap  # noqa: E402,F401
