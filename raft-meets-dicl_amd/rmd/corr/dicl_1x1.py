"""Drop-in for corr.dicl_1x1.CorrelationModule — src/models/common/corr/dicl_1x1.py:33-86."""

import torch.nn as nn

from .. import ops
from ..blocks.dicl import DisplacementAwareProjection, MatchingNet1x1
from .dicl import _delta


class CorrelationModule(nn.Module):
    def __init__(self, feature_dim, radius, dap_init="identity", norm_type="batch", relu_inplace=True,
                 mnet_scale=1):
        super().__init__()
        self.radius = radius
        self.mnet = MatchingNet1x1(2 * feature_dim, norm_type=norm_type, relu_inplace=relu_inplace, scale=mnet_scale)
        self.dap = DisplacementAwareProjection((radius, radius), init=dap_init)
        self.register_buffer("delta", _delta(radius), persistent=False)
        self.output_dim = (2 * self.radius + 1) ** 2

    def forward(self, f1, f2, coords, dap=True):
        batch, _, h, w = f1.shape
        cost = self.mnet(ops.dicl_stack(f1, f2, coords, self.radius))
        if dap:
            cost = self.dap(cost)
        return cost.reshape(batch, -1, h, w)


# single-level soft-argmax regressions of this module (reference classes of the same names)
from ..heads import CorrSoftArgMaxFlowRegression as SoftArgMaxFlowRegression  # noqa: E402,F401
from ..heads import CorrSoftArgMaxFlowRegressionWithDap as SoftArgMaxFlowRegressionWithDap  # noqa: E402,F401
