"""Drop-in for corr.dicl_emb.CorrelationModule — src/models/common/corr/dicl_emb.py:32-104.

The stack carries the two displacement channels (dx, dy) after the feature pair (:81-85), written
by the same rmd_dicl_stack pass (extra_delta).
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..blocks.dicl import DisplacementAwareProjection, MatchingNet
from .dicl import _delta


class PairEmbedding(nn.Sequential):
    def __init__(self, input_dim, output_dim, relu_inplace=True):
        super().__init__(
            nn.Conv2d(input_dim, 48, kernel_size=1), nn.ReLU(inplace=relu_inplace),
            nn.Conv2d(48, 64, kernel_size=1), nn.ReLU(inplace=relu_inplace),
            nn.Conv2d(64, output_dim, kernel_size=1),
        )
        self.output_dim = output_dim

    def forward(self, fstack):
        batch, du, dv, c, h, w = fstack.shape
        emb = super().forward(fstack.view(batch * du * dv, c, h, w))
        return emb.view(batch, du, dv, self.output_dim, h, w)


class CorrelationModule(nn.Module):
    def __init__(self, feature_dim, radius, embedding_dim=32, dap_init="identity", norm_type="batch",
                 relu_inplace=True):
        super().__init__()
        self.radius = radius
        self.mnet = MatchingNet(2 * feature_dim + 2, norm_type=norm_type, relu_inplace=relu_inplace)
        self.emb = PairEmbedding(2 * feature_dim + 2, embedding_dim, relu_inplace=relu_inplace)
        self.dap = DisplacementAwareProjection((radius, radius), init=dap_init)
        self.register_buffer("delta", _delta(radius), persistent=False)
        self.output_dim = (2 * self.radius + 1) ** 2 + embedding_dim

    def forward(self, f1, f2, coords, dap=True):
        batch, _, h, w = f1.shape
        r = self.radius
        stack = ops.dicl_stack(f1, f2, coords, r, extra_delta=True)   # (B, d, d, 2C+2, h, w)
        cost = self.mnet(stack)
        emb = self.emb(stack)
        score = self.dap(cost) if dap else cost
        score = F.softmax(score.view(batch, (2 * r + 1) ** 2, h, w), dim=1).view(batch, 2 * r + 1, 2 * r + 1, 1, h, w)
        emb = (score * emb).sum(dim=(1, 2))
        return torch.cat((cost.view(batch, -1, h, w), emb), dim=1)


# single-level soft-argmax regressions of this module (reference classes of the same names)
from ..heads import CorrSoftArgMaxFlowRegression as SoftArgMaxFlowRegression  # noqa: E402,F401
from ..heads import CorrSoftArgMaxFlowRegressionWithDap as SoftArgMaxFlowRegressionWithDap  # noqa: E402,F401
