"""DICL building blocks — drop-in for src/models/common/blocks/dicl.py (qzed/raft-meets-dicl v2).

MatchingNet stays a plain nn.Sequential of MIOpen convolutions (out of scope for custom kernels)
with the reference's module names, so checkpoints load unchanged (`mnet.0.0.weight`, ...) and
forward hooks on `*.mnet` keep working.  DisplacementAwareProjection keeps its `conv1` parameter
((D, D, 1, 1), identity init) but runs the projection through rmd_dap.
"""

import numpy as np
import torch
import torch.nn as nn

from .. import ops


def make_norm2d(ty, num_channels, num_groups):
    """src/models/common/norm.py:4-15."""
    if ty == "group":
        return nn.GroupNorm(num_groups=num_groups, num_channels=num_channels)
    if ty == "batch":
        return nn.BatchNorm2d(num_channels)
    if ty == "instance":
        return nn.InstanceNorm2d(num_channels)
    if ty == "none":
        return nn.Sequential()
    raise ValueError(f"unknown norm type '{ty}'")


class ConvBlock(nn.Sequential):
    """conv (no bias) -> norm -> ReLU (blocks/dicl.py:15-23)."""

    def __init__(self, c_in, c_out, norm_type="batch", relu_inplace=True, num_groups=8, **kwargs):
        super().__init__(nn.Conv2d(c_in, c_out, bias=False, **kwargs),
                         make_norm2d(norm_type, c_out, num_groups),
                         nn.ReLU(inplace=relu_inplace))


class ConvBlockTransposed(nn.Sequential):
    """transposed conv (no bias) -> norm -> ReLU (blocks/dicl.py:26-34)."""

    def __init__(self, c_in, c_out, norm_type="batch", relu_inplace=True, num_groups=8, **kwargs):
        super().__init__(nn.ConvTranspose2d(c_in, c_out, bias=False, **kwargs),
                         make_norm2d(norm_type, c_out, num_groups),
                         nn.ReLU(inplace=relu_inplace))


class MatchingNet(nn.Sequential):
    """Stacked feature pairs (B, du, dv, 2C, h, w) -> cost (B, du, dv, h, w) (blocks/dicl.py:93-118)."""

    def __init__(self, input_channels, norm_type="batch", relu_inplace=True, scale=1):
        c1, c2, c3, c4 = int(scale * 96), int(scale * 128), int(scale * 64), int(scale * 32)
        kw = dict(norm_type=norm_type, relu_inplace=relu_inplace)
        super().__init__(
            ConvBlock(input_channels, c1, kernel_size=3, padding=1, **kw),
            ConvBlock(c1, c2, kernel_size=3, padding=1, stride=2, **kw),
            ConvBlock(c2, c2, kernel_size=3, padding=1, **kw),
            ConvBlock(c2, c3, kernel_size=3, padding=1, **kw),
            ConvBlockTransposed(c3, c4, kernel_size=4, padding=1, stride=2, num_groups=4, **kw),
            nn.Conv2d(c4, 1, kernel_size=3, padding=1),
        )

    def forward(self, mvol):
        b, du, dv, c2, h, w = mvol.shape
        cost = super().forward(mvol.view(b * du * dv, c2, h, w))
        return cost.view(b, du, dv, h, w)


class MatchingNet1x1(nn.Sequential):
    """1x1-conv matching network (src/models/common/corr/dicl_1x1.py:8-30)."""

    def __init__(self, input_channels, norm_type="batch", relu_inplace=True, scale=1):
        c1, c2, c3 = int(scale * 96), int(scale * 128), int(scale * 64)
        kw = dict(norm_type=norm_type, relu_inplace=relu_inplace)
        super().__init__(
            ConvBlock(input_channels, c1, kernel_size=1, **kw),
            ConvBlock(c1, c2, kernel_size=1, **kw),
            ConvBlock(c2, c3, kernel_size=1, **kw),
            nn.Conv2d(c3, 1, kernel_size=1),
        )

    def forward(self, mvol):
        b, du, dv, c2, h, w = mvol.shape
        cost = super().forward(mvol.view(b * du * dv, c2, h, w))
        return cost.view(b, du, dv, h, w)


class DisplacementAwareProjection(nn.Module):
    """1x1 conv over the (2u+1)(2v+1) displacement channels, no bias (blocks/dicl.py:121-150)."""

    def __init__(self, disp_range, init="identity"):
        super().__init__()
        if init not in ("identity", "standard"):
            raise ValueError(f"unknown init value '{init}'")
        disp_range = np.asarray(disp_range)
        assert disp_range.shape == (2,)
        n = int(np.prod(2 * disp_range + 1))
        self.conv1 = nn.Conv2d(n, n, bias=False, kernel_size=1)
        if init == "identity":
            nn.init.eye_(self.conv1.weight[:, :, 0, 0])

    def forward(self, x):
        return ops.dap(x, self.conv1.weight)
