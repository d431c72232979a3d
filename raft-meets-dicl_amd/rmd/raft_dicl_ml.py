"""Drop-in for raft_dicl_ml.CorrelationModule — src/models/impls/raft_dicl_ml.py:235-343.

Per level i the reference grid-samples fmap2[i] at coords / 2^i + delta — normalising with
fmap1[i]'s (full-resolution) size, :295-305 — then expands fmap1[i] and concatenates the two into
the (B, 2r+1, 2r+1, 2C, h, w) MatchingNet input (:308-316).  Here that gather is one
rmd_dicl_stack pass per level (level = i, norm = fmap1[i]'s size, reproducing the quirk), the
MatchingNets stay the reference's modules, `mask_costs` zeroes a level's cost (:325-326) and the
displacement-aware projection runs through rmd_dap — per level ('separate', :328-332) or as the
(L*(2r+1)^2)^2 1x1 conv over all costs ('full', :268-273, :339-341).  State-dict keys are the
reference's (`mnet.{i}.*` / `mnet.*` when shared, `dap.{i}.conv1.weight`, or `dap.weight`).
"""

import torch
import torch.nn as nn

from . import ops
from .blocks.dicl import DisplacementAwareProjection, MatchingNet


class FullDap(nn.Conv2d):
    """The 'full' DAP: a bias-free 1x1 nn.Conv2d over all levels' costs, applied with rmd_dap."""

    def __init__(self, n_channels, init="identity"):
        super().__init__(n_channels, n_channels, bias=False, kernel_size=1)
        if init == "identity":
            nn.init.eye_(self.weight[:, :, 0, 0])

    def forward(self, x):
        return ops.dap(x, self.weight)


class CorrelationModule(nn.Module):
    def __init__(self, feature_dim, levels, radius, dap_init="identity", dap_type="separate",
                 norm_type="batch", share=False, relu_inplace=True):
        super().__init__()
        if dap_type not in ("full", "separate"):
            raise ValueError(f"DAP type '{dap_type}' not supported")
        self.radius = radius
        self.dap_type = dap_type
        self.share = share

        def mk_mnet():
            return MatchingNet(2 * feature_dim, norm_type=norm_type, relu_inplace=relu_inplace)

        def mk_dap():
            return DisplacementAwareProjection((radius, radius), init=dap_init)

        if share:
            self.mnet = mk_mnet()
            if dap_type == "separate":
                self.dap = mk_dap()
        else:
            self.mnet = nn.ModuleList([mk_mnet() for _ in range(levels)])
            if dap_type == "separate":
                self.dap = nn.ModuleList([mk_dap() for _ in range(levels)])
        if dap_type == "full":
            self.dap = FullDap(levels * (2 * radius + 1) ** 2, init=dap_init)
        r = torch.linspace(-radius, radius, 2 * radius + 1)
        self.register_buffer("delta", torch.stack(torch.meshgrid(r, r, indexing="ij"), dim=-1), persistent=False)

    def forward(self, fmap1, fmap2, coords, dap=True, mask_costs=[]):
        batch, _, h, w = coords.shape
        out = []
        for i, (f1, f2) in enumerate(zip(fmap1, fmap2)):
            _, _, h1, w1 = f1.shape
            stack = ops.dicl_stack(f1, f2, coords, self.radius, level=i, norm_hw=(h1, w1))
            cost = (self.mnet if self.share else self.mnet[i])(stack)
            if i + 3 in mask_costs:
                cost = torch.zeros_like(cost)
            if dap and self.dap_type == "separate":
                cost = (self.dap if self.share else self.dap[i])(cost)
            out.append(cost.reshape(batch, -1, h, w))
        out = torch.cat(out, dim=-3)
        if dap and self.dap_type == "full":
            out = self.dap(out)
        return out
