"""Per-iteration flow heads — drop-ins for the reference's soft-argmax regressions and Up8Network.

  Up8Network                              <- src/models/impls/raft.py:299-331
  SoftArgMaxFlowRegression(+WithDap)      <- raft.py:98-181 (num_levels levels, level l scaled by 2^l)
  CorrSoftArgMaxFlowRegression(+WithDap)  <- the single-level classes of corr/dicl.py:64-110,
                                             corr/dot.py:69-120, corr/dicl_1x1.py:89-134,
                                             corr/dicl_emb.py:107-161 (re-exported there under the
                                             reference's names)

The convolutions of Up8Network stay MIOpen (`conv1`, `relu1`, `conv2`: state_dict keys and forward
hooks unchanged); the softmax + 3x3 convex combination runs as rmd_up8.  Soft-argmax runs as one
rmd_softargmax launch over all levels; the DAP variants call their `dap` modules (rmd_dap) first.
Both are autograd functions with HIP backward kernels.
"""

import torch
import torch.nn as nn

from . import ops
from .blocks.dicl import DisplacementAwareProjection


def _delta(radius):
    r = torch.linspace(-radius, radius, 2 * radius + 1)
    return torch.stack(torch.meshgrid(r, r, indexing="ij"), dim=-1)     # (2r+1, 2r+1, 2), raft.py:106-109


class Up8Network(nn.Module):
    """RAFT 8x flow upsampling module for the finest level (raft.py:299-331)."""

    def __init__(self, hidden_dim=128, mixed_precision=False, relu_inplace=True, temperature=4.0):
        super().__init__()
        self.mixed_precision = mixed_precision
        self.conv1 = nn.Conv2d(hidden_dim, 256, 3, padding=1)
        self.relu1 = nn.ReLU(inplace=relu_inplace)
        self.conv2 = nn.Conv2d(256, 8 * 8 * 9, 1, padding=0)
        self.temperature = temperature

    def forward(self, hidden, flow):
        with torch.autocast("cuda", enabled=self.mixed_precision):
            mask = self.conv2(self.relu1(self.conv1(hidden)))
        # the reference applies the softmax inside the autocast region too; rmd_up8 computes it in fp32
        return ops.up8(mask, flow, self.temperature)


class SoftArgMaxFlowRegression(nn.Module):
    """raft.SoftArgMaxFlowRegression: (B, L*(2r+1)^2, h, w) -> L flows (B, 2, h, w)."""

    def __init__(self, num_levels, radius, temperature=1.0):
        super().__init__()
        self.num_levels = num_levels
        self.radius = radius
        self.temperature = temperature
        self.register_buffer("delta", _delta(radius), persistent=False)

    def forward(self, corr):
        return ops.softargmax(corr, self.num_levels, self.radius, self.temperature)


class SoftArgMaxFlowRegressionWithDap(nn.Module):
    """raft.SoftArgMaxFlowRegressionWithDap: per-level DAP (identity init), then soft-argmax."""

    def __init__(self, num_levels, radius, temperature=1.0):
        super().__init__()
        self.num_levels = num_levels
        self.radius = radius
        self.temperature = temperature
        self.dap = nn.ModuleList([DisplacementAwareProjection((radius, radius), init="identity")
                                  for _ in range(num_levels)])
        self.register_buffer("delta", _delta(radius), persistent=False)

    def forward(self, corr):
        batch, _, h, w = corr.shape
        d = 2 * self.radius + 1
        levels = torch.split(corr, d * d, dim=1)
        score = torch.cat([self.dap[i](levels[i].reshape(batch, d, d, h, w)).view(batch, d * d, h, w)
                           for i in range(self.num_levels)], dim=1)
        return ops.softargmax(score, self.num_levels, self.radius, self.temperature)


class CorrSoftArgMaxFlowRegression(nn.Module):
    """Single-level soft-argmax of the correlation modules (corr/dot.py:69-90): no level scaling.

    Regresses on the first (2r+1)^2 channels, so it also serves dicl_emb's embedding input
    (corr/dicl_emb.py:120-125, whose reference body calls .view on the tuple torch.split returns
    and therefore raises; this mirror implements the evident intent)."""

    def __init__(self, radius, temperature=1.0):
        super().__init__()
        self.radius = radius
        self.temperature = temperature
        self.register_buffer("delta", _delta(radius), persistent=False)

    def forward(self, cost):
        return ops.softargmax(cost, 1, self.radius, self.temperature)[0]


class CorrSoftArgMaxFlowRegressionWithDap(nn.Module):
    """corr/dot.py:93-120: DAP (identity init) over the (2r+1)^2 costs, then soft-argmax."""

    def __init__(self, radius, temperature=1.0):
        super().__init__()
        self.radius = radius
        self.temperature = temperature
        self.dap = DisplacementAwareProjection((radius, radius))
        self.register_buffer("delta", _delta(radius), persistent=False)

    def forward(self, cost):
        batch, _, h, w = cost.shape
        d = 2 * self.radius + 1
        score = self.dap(cost[:, :d * d].reshape(batch, d, d, h, w)).view(batch, d * d, h, w)
        return ops.softargmax(score, 1, self.radius, self.temperature)[0]


def make_flow_regression(type, num_levels, radius, **kwargs):
    """raft.make_flow_regression (raft.py:184-190)."""
    if type == "softargmax":
        return SoftArgMaxFlowRegression(num_levels, radius, **kwargs)
    if type == "softargmax+dap":
        return SoftArgMaxFlowRegressionWithDap(num_levels, radius, **kwargs)
    raise ValueError(f"unknown correlation module type '{type}'")


def make_corr_flow_regression(cmod_type, type, radius, **kwargs):
    """corr.make_flow_regression (corr/__init__.py:23-49): same classes for every module type."""
    if cmod_type in ("dicl", "dicl-1x1", "dicl-emb", "dot"):
        if type == "softargmax":
            return CorrSoftArgMaxFlowRegression(radius, **kwargs)
        if type == "softargmax+dap":
            return CorrSoftArgMaxFlowRegressionWithDap(radius, **kwargs)
    raise ValueError(f"unknown correlation module type '{type}' for correlation module '{cmod_type}'")
