"""The reference's eager-torch correlation, restated for runs where the reference cannot travel —
test infrastructure, not product code.

EagerCorrBlock follows raft.CorrBlock (src/models/impls/raft.py:15-95) op for op: matmul of the
flattened maps / sqrt(C) (:26-33), avg_pool2d pyramid over the target dims (:35-47), and per lookup
a grid_sample (bilinear, zeros, align_corners=True) of the (2r+1)^2 integer-offset window around
coords/2^i normalised by (W_i-1, H_i-1) (:49-95).  Device-agnostic: tools/bench_e2e.py runs it on
the GPU as the "reference GPU path"; bench.py's cpu_baseline leg runs the whole RAFT network on it
on the host's cores (BASELINE configs[0]).
"""

import torch
import torch.nn.functional as F


class EagerCorrBlock:
    """raft.CorrBlock (raft.py:15-95) in eager torch — the reference GPU path."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, precision=None):
        self.num_levels, self.radius = num_levels, radius
        b, c, h, w = fmap1.shape
        corr = torch.matmul(fmap1.view(b, c, h * w).transpose(1, 2), fmap2.view(b, c, h * w))
        corr = (corr / torch.tensor(c).float().sqrt()).view(b * h * w, 1, h, w)
        self.pyr = [corr]
        for _ in range(1, num_levels):
            corr = F.avg_pool2d(corr, kernel_size=2, stride=2)
            self.pyr.append(corr)

    def __call__(self, coords, mask_costs=()):
        r = self.radius
        b, _, h, w = coords.shape
        d = torch.linspace(-r, r, 2 * r + 1, device=coords.device)
        delta = torch.stack(torch.meshgrid(d, d, indexing="ij"), dim=-1).view(1, 2 * r + 1, 2 * r + 1, 2)
        co = coords.permute(0, 2, 3, 1).reshape(b * h * w, 1, 1, 2)
        out = []
        for i, corr in enumerate(self.pyr):
            _, _, hh, ww = corr.shape
            c = co / 2 ** i + delta
            xg, yg = c.split(1, dim=-1)
            grid = torch.cat((2 * xg / (ww - 1) - 1, 2 * yg / (hh - 1) - 1), dim=-1)
            s = F.grid_sample(corr, grid, align_corners=True)
            out.append(s.view(b, h, w, -1))
        return torch.cat(out, dim=-1).permute(0, 3, 1, 2).contiguous().float()
