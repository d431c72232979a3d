"""RAFT+DICL coarse-to-fine (3 levels) network for the hybrid-model parity tests — test
infrastructure, not product code.

A from-scratch restatement of src/models/impls/raft_dicl_ctf_l3.py:19-260 (RaftPlusDiclModule at
its defaults: share_dicl False, share_rnn True, upsample_hidden 'none', corr-type 'dicl',
corr-reg-type 'softargmax') with the p35 RAFT encoder (src/models/common/encoders/raft/p35.py,
common.py), written with the SAME module names and registration order so that
tests/golden/detinit.det_init_fanin (name-keyed) fills it with the weights the reference held when
tests/golden/gen_ctf_l3.py produced the fixtures.  The correlation modules come from a `make_cmod`
factory: rmd.corr.make_cmod (the HIP path: rmd_dicl_stack + MatchingNet + rmd_dap) on the GPU box,
the reference's own factory when the generator checks this restatement bitwise on the CPU.

The multi-level sequence loss (src/models/common/loss/mlseq.py:34-67) is restated as
`mlseq_loss` for the training-step test (cfg/model/raft+dicl-ctf3l.yaml: ord 1, gamma 0.85,
alpha (0.38, 0.6, 1.0)).
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from .raft_net import BasicUpdateBlock, ResidualBlock, Up8Network, _norm


class EncoderOutputNet(nn.Module):
    """encoders/raft/common.py:6-22: conv3x3 - norm - relu - conv1x1 (- dropout 0)."""

    def __init__(self, input_dim, output_dim, hidden_dim, norm):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, kernel_size=3, padding=1)
        self.norm1 = _norm(norm, hidden_dim)
        self.relu1 = nn.ReLU()
        self.conv2 = nn.Conv2d(hidden_dim, output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=0.0)

    def forward(self, x):
        return self.dropout(self.conv2(self.relu1(self.norm1(self.conv1(x)))))


class FeatureEncoderP35(nn.Module):
    """encoders/raft/p35.py:9-78: 1/8, 1/16 and 1/32 outputs (x3, x4, x5)."""

    def __init__(self, output_dim, norm):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3)
        self.norm1 = _norm(norm, 64)
        self.relu1 = nn.ReLU()
        self.layer1 = nn.Sequential(ResidualBlock(64, 64, norm), ResidualBlock(64, 64, norm))
        self.layer2 = nn.Sequential(ResidualBlock(64, 96, norm, 2), ResidualBlock(96, 96, norm))
        self.layer3 = nn.Sequential(ResidualBlock(96, 128, norm, 2), ResidualBlock(128, 128, norm))
        self.layer4 = nn.Sequential(ResidualBlock(128, 160, norm, 2), ResidualBlock(160, 160, norm))
        self.layer5 = nn.Sequential(ResidualBlock(160, 192, norm, 2), ResidualBlock(192, 192, norm))
        self.out3 = EncoderOutputNet(128, output_dim, 160, norm)
        self.out4 = EncoderOutputNet(160, output_dim, 192, norm)
        self.out5 = EncoderOutputNet(192, output_dim, 224, norm)

    def forward(self, x):
        x = self.relu1(self.norm1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        x3 = self.out3(x)
        x = self.layer4(x)
        x4 = self.out4(x)
        x = self.layer5(x)
        return x3, x4, self.out5(x)


def coordinate_grid(b, h, w, device):
    """common/grid.py:4-12: (B, 2, h, w), channel 0 = x, channel 1 = y."""
    ys, xs = torch.meshgrid(torch.arange(h, device=device), torch.arange(w, device=device), indexing="ij")
    return torch.stack([xs, ys]).float()[None].expand(b, -1, -1, -1)


class HUpNone(nn.Module):
    """common/hsup.py:8-13: keep the level's own initial hidden state."""

    def forward(self, h_prev, h_init):
        return h_init


class CtfL3Net(nn.Module):
    """RaftPlusDiclModule (raft_dicl_ctf_l3.py:19-260) at its defaults."""

    def __init__(self, make_cmod, make_flow_regression=None, upnet_cls=None, corr_radius=4, corr_channels=32,
                 context_channels=128, recurrent_channels=128):
        super().__init__()
        self.hidden_dim, self.context_dim = recurrent_channels, context_channels
        self.corr_radius = corr_radius
        self.fnet = FeatureEncoderP35(corr_channels, "instance")
        self.cnet = FeatureEncoderP35(recurrent_channels + context_channels, "batch")
        kw = dict(radius=corr_radius, dap_init="identity", norm_type="batch", relu_inplace=True)
        self.corr_3 = make_cmod("dicl", corr_channels, **kw)
        self.corr_4 = make_cmod("dicl", corr_channels, **kw)
        self.corr_5 = make_cmod("dicl", corr_channels, **kw)
        if make_flow_regression is not None:        # parameter-free for 'softargmax'; used only with corr_flow
            self.flow_reg_3 = make_flow_regression("dicl", "softargmax", radius=corr_radius)
            self.flow_reg_4 = make_flow_regression("dicl", "softargmax", radius=corr_radius)
            self.flow_reg_5 = make_flow_regression("dicl", "softargmax", radius=corr_radius)
        self.update_block = BasicUpdateBlock(self.corr_3.output_dim, input_dim=context_channels,
                                             hidden_dim=recurrent_channels)
        self.upnet_h = HUpNone()
        self.upnet = (upnet_cls or Up8Network)(recurrent_channels)

    def _level(self, corr, f1, f2, h, ctx, coords0, flow, iterations, dap, out, upnet):
        coords1 = coords0 + flow         # not re-derived as coords1 - coords0: the reference keeps `flow`
        for _ in range(iterations):
            coords1 = coords1.detach()
            c = corr(f1, f2, coords1, dap=dap)
            h, d = self.update_block(h, ctx, c, flow.detach())
            coords1 = coords1 + d
            flow = coords1 - coords0
            out.append(self.upnet(h, flow) if upnet else flow)
        return h, flow

    def forward(self, img1, img2, iterations=(4, 3, 3), dap=True, upnet=True):
        hdim, cdim = self.hidden_dim, self.context_dim
        b, _, h, w = img1.shape
        f1_3, f1_4, f1_5 = self.fnet(img1)
        f2_3, f2_4, f2_5 = self.fnet(img2)
        ctx_3, ctx_4, ctx_5 = self.cnet(img1)
        hs, ctxs = [], []
        for c in (ctx_3, ctx_4, ctx_5):
            hh, cc = torch.split(c, (hdim, cdim), dim=1)
            hs.append(torch.tanh(hh))
            ctxs.append(torch.relu(cc))
        h_3, h_4, h_5 = hs
        ctx_3, ctx_4, ctx_5 = ctxs

        # coarse level (1/32), zero initial flow (raft_dicl_ctf_l3.py:133-165)
        coords0 = coordinate_grid(b, h // 32, w // 32, img1.device)
        out_5 = []
        h_5, flow = self._level(self.corr_5, f1_5, f2_5, h_5, ctx_5, coords0, coords0 - coords0, iterations[0],
                                dap, out_5, False)
        # middle level (1/16) (:167-202)
        flow = 2 * F.interpolate(flow, (h // 16, w // 16), mode="bilinear", align_corners=True)
        coords0 = coordinate_grid(b, h // 16, w // 16, img1.device)
        h_4 = self.upnet_h(h_5, h_4)
        out_4 = []
        h_4, flow = self._level(self.corr_4, f1_4, f2_4, h_4, ctx_4, coords0, flow, iterations[1], dap,
                                out_4, False)
        # fine level (1/8) with convex upsampling of every estimate (:204-245)
        flow = 2 * F.interpolate(flow, (h // 8, w // 8), mode="bilinear", align_corners=True)
        coords0 = coordinate_grid(b, h // 8, w // 8, img1.device)
        h_3 = self.upnet_h(h_4, h_3)
        out_3 = []
        self._level(self.corr_3, f1_3, f2_3, h_3, ctx_3, coords0, flow, iterations[2], dap, out_3, upnet)
        return out_5, out_4, out_3


def freeze_batchnorm(module):
    """common/norm.py:17-24 (the ctf-l3 stage default on-stage freeze_batchnorm: True)."""
    for m in module.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.eval()
    return module


def _upsample(flow, shape):
    """loss/mlseq.py:59-67: bilinear, align_corners=True, each component scaled by its size ratio."""
    _, _, fh, fw = flow.shape
    _, _, th, tw = shape
    flow = F.interpolate(flow, (th, tw), mode="bilinear", align_corners=True)
    scale = torch.tensor([tw / fw, th / fh], dtype=flow.dtype, device=flow.device).view(1, 2, 1, 1)
    return flow * scale


def mlseq_loss(result, target, valid, ord=1, gamma=0.85, alpha=(0.38, 0.6, 1.0), scale=1.0):
    """MultiLevelSequenceLoss.compute (loss/mlseq.py:34-57)."""
    loss = 0.0
    for i_level, level in enumerate(result):
        n = len(level)
        for i_seq, flow in enumerate(level):
            weight = alpha[i_level] * gamma ** (n - i_seq - 1)
            if flow.shape != target.shape:
                flow = _upsample(flow, target.shape)
            dist = torch.linalg.vector_norm(flow - target, ord=ord, dim=-3)
            loss = loss + weight * dist[valid].mean()
    return loss * scale
