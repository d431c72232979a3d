"""RAFT baseline network for the end-to-end EPE parity test — test infrastructure, not product code.

The north star's end-to-end gate is "RAFT 12-iteration inference matches reference EPE within 1e-3
px".  The encoders / GRU / upsampler are outside the hot path but are needed to run
the model on the GPU box, where the reference cannot travel.  This is a from-scratch restatement of
the architecture of src/models/impls/raft.py:193-433 (RaftModule) and
src/models/common/encoders/raft/s3.py + common/blocks/raft.py (FeatureEncoder, ResidualBlock),
written with the SAME module names and registration order, so that tests/golden/detinit.det_init
(name-keyed) fills it with the weights the reference held when tests/golden/gen_e2e.py produced the
fixture.  The correlation volume and its lookups go through rmd.raft.CorrBlock (the HIP path).
"""

import torch
import torch.nn as nn
import torch.nn.functional as F


def _norm(kind, ch):
    if kind == "instance":
        return nn.InstanceNorm2d(ch)
    if kind == "batch":
        return nn.BatchNorm2d(ch)
    if kind == "group":
        return nn.GroupNorm(ch // 8, ch)
    return nn.Sequential()


class ResidualBlock(nn.Module):
    """common/blocks/raft.py:13-46: conv-norm-relu x2 (+ strided 1x1 projection), relu(x + y)."""

    def __init__(self, cin, cout, norm, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.relu1, self.relu2, self.relu3 = nn.ReLU(), nn.ReLU(), nn.ReLU()
        self.norm1 = _norm(norm, cout)
        self.norm2 = _norm(norm, cout)
        if stride > 1:
            self.norm3 = _norm(norm, cout)
        self.downsample = None
        if stride > 1:      # shares norm3 (two state_dict keys, one module — as the reference)
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride), self.norm3)

    def forward(self, x):
        y = self.relu1(self.norm1(self.conv1(x)))
        y = self.relu2(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu3(x + y)


class FeatureEncoder(nn.Module):
    """encoders/raft/s3.py:8-72: 1/8-resolution feature / context encoder."""

    def __init__(self, output_dim, norm):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3)
        self.norm1 = _norm(norm, 64)
        self.relu1 = nn.ReLU()
        self.layer1 = nn.Sequential(ResidualBlock(64, 64, norm), ResidualBlock(64, 64, norm))
        self.layer2 = nn.Sequential(ResidualBlock(64, 96, norm, 2), ResidualBlock(96, 96, norm))
        self.layer3 = nn.Sequential(ResidualBlock(96, 128, norm, 2), ResidualBlock(128, 128, norm))
        self.conv2 = nn.Conv2d(128, output_dim, 1)
        self.dropout = nn.Dropout2d(p=0.0)

    def forward(self, x):
        x = self.relu1(self.norm1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        return self.dropout(self.conv2(x))


class BasicMotionEncoder(nn.Module):
    """raft.py:193-225."""

    def __init__(self, corr_planes):
        super().__init__()
        self.convc1 = nn.Conv2d(corr_planes, 256, 1)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(192 + 64, 126, 3, padding=1)

    def forward(self, flow, corr):
        c = F.relu(self.convc2(F.relu(self.convc1(corr))))
        f = F.relu(self.convf2(F.relu(self.convf1(flow))))
        return torch.cat([F.relu(self.conv(torch.cat([c, f], 1))), flow], 1)


class SepConvGru(nn.Module):
    """raft.py:228-259: horizontal (1x5) then vertical (5x1) convolutional GRU."""

    def __init__(self, hidden_dim, input_dim):
        super().__init__()
        cin = hidden_dim + input_dim
        self.convz1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))

    @staticmethod
    def _step(h, x, cz, cr, cq):
        hx = torch.cat([h, x], 1)
        z, r = torch.sigmoid(cz(hx)), torch.sigmoid(cr(hx))
        q = torch.tanh(cq(torch.cat([r * h, x], 1)))
        return (1.0 - z) * h + z * q

    def forward(self, h, x):
        h = self._step(h, x, self.convz1, self.convr1, self.convq1)
        return self._step(h, x, self.convz2, self.convr2, self.convq2)


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU()

    def forward(self, x):
        return self.conv2(self.relu(self.conv1(x)))


class BasicUpdateBlock(nn.Module):
    def __init__(self, corr_planes, input_dim=128, hidden_dim=128):
        super().__init__()
        self.enc = BasicMotionEncoder(corr_planes)
        self.gru = SepConvGru(hidden_dim, input_dim + 128)
        self.flow = FlowHead(hidden_dim, 256)

    def forward(self, h, x, corr, flow):
        h = self.gru(h, torch.cat([x, self.enc(flow, corr)], 1))
        return h, self.flow(h)


class Up8Network(nn.Module):
    """raft.py:299-331: convex 8x upsampling with a softmax over the 3x3 neighbourhood."""

    def __init__(self, hidden_dim=128, temperature=4.0):
        super().__init__()
        self.conv1 = nn.Conv2d(hidden_dim, 256, 3, padding=1)
        self.relu1 = nn.ReLU()
        self.conv2 = nn.Conv2d(256, 8 * 8 * 9, 1)
        self.temperature = temperature

    def forward(self, hidden, flow):
        b, c, h, w = flow.shape
        mask = self.conv2(self.relu1(self.conv1(hidden))).view(b, 1, 9, 8, 8, h, w)
        mask = torch.softmax(mask / self.temperature, dim=2)
        up = F.unfold(8 * flow, (3, 3), padding=1).view(b, c, 9, 1, 1, h, w)
        up = torch.sum(mask * up, dim=2).permute(0, 1, 4, 2, 5, 3)
        return up.reshape(b, 2, h * 8, w * 8)


class RaftNet(nn.Module):
    """RaftModule (raft.py:334-433) at its defaults; `corr_block` is rmd.raft.CorrBlock, `upnet_cls`
    optionally rmd.raft.Up8Network (default: the eager restatement above)."""

    def __init__(self, corr_block, corr_levels=4, corr_radius=4, precision="fp32", upnet_cls=None):
        super().__init__()
        self.corr_block = corr_block
        self.precision = precision
        self.corr_levels, self.corr_radius = corr_levels, corr_radius
        self.fnet = FeatureEncoder(256, "instance")
        self.cnet = FeatureEncoder(256, "batch")
        self.update_block = BasicUpdateBlock(corr_levels * (2 * corr_radius + 1) ** 2)
        self.upnet = (upnet_cls or Up8Network)(128)     # rmd.raft.Up8Network: the HIP convex upsampling

    def forward(self, img1, img2, iterations=12):
        fmap1, fmap2 = self.fnet(img1).float(), self.fnet(img2).float()
        corr_vol = self.corr_block(fmap1, fmap2, num_levels=self.corr_levels, radius=self.corr_radius,
                                   precision=self.precision)
        h, x = torch.split(self.cnet(img1), (128, 128), dim=1)
        h, x = torch.tanh(h), torch.relu(x)
        b, _, ih, iw = img1.shape
        ys, xs = torch.meshgrid(torch.arange(ih // 8, device=img1.device), torch.arange(iw // 8, device=img1.device),
                                indexing="ij")
        coords0 = torch.stack([xs, ys]).float()[None].expand(b, -1, -1, -1)
        coords1 = coords0.clone()
        flow = coords1 - coords0
        out = []
        for _ in range(iterations):
            coords1 = coords1.detach()
            corr = corr_vol(coords1)
            h, d = self.update_block(h, x, corr, flow.detach())
            coords1 = coords1 + d
            flow = coords1 - coords0
            out.append(self.upnet(h, flow))
        return out
