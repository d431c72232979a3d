"""Drop-in for raft.CorrBlock — qzed/raft-meets-dicl src/models/impls/raft.py:15-95.

Same constructor and call signature; the all-pairs volume and its pooled pyramid are built by one
MFMA GEMM launch with a pooling epilogue (rmd_corr_pyramid) and each lookup is one bandwidth-bound
gather launch (rmd_corr_lookup).  Output: contiguous float32 (B, L*(2r+1)^2, H, W), as raft.py:95.

Training: when the feature maps require gradients (and grad mode is on) the block is an autograd
node — the lookups' backward passes accumulate one dense pyramid gradient (rmd_corr_lookup_backward)
and the pyramid's backward turns it into d fmap1 / d fmap2 (ops._CorrPyramidFn), matching the
reference's autograd through grid_sample / avg_pool2d / matmul.  Coordinates get no gradient
(the reference detaches them, raft.py:402).
"""

import torch

from . import config, ops


class CorrBlock:
    """Correlation volume for matching costs (drop-in for raft.CorrBlock).

    ``precision`` / ``method`` / ``memory_budget`` are the drop-in's op selection (rmd.config; None =
    the process values, set from a cfg/model ``parameters`` section by rmd.config.configure): method
    'volume' builds the all-pairs pyramid, 'otf' samples pooled features on the fly each lookup (no
    O(N^2) memory; raft_fs semantics with this block's scale), 'auto' takes the volume while it fits
    the memory budget.  Both are differentiable.
    """

    scale = None            # 1/sqrt(C) (raft.py:33); raft_fs.CorrBlock overrides with 1.0

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, precision=None, method=None, memory_budget=None):
        opts = config.corr_options(None, precision=precision, method=method, memory_budget=memory_budget)
        self.num_levels = num_levels
        self.radius = radius
        self.precision = opts.precision
        self._state = self._token = None
        training = torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad)
        # GPU training runs the token-linked autograd functions of rmd.ops; on the CPU the operators'
        # ATen kernels (rmd/cpu.py) carry the gradient themselves
        tokens = training and fmap1.is_cuda
        b, c, h, w = fmap1.shape
        # the C <= 256 limit of the on-the-fly backward is the HIP kernel's (rmd_corr_otf_backward):
        # the CPU kernels train any channel count, so only a GPU training block is steered by it; the
        # volume's bytes are those of the storage this (device, C) resolves to
        self.method = config.choose_method(opts.method, b, h, w, num_levels, self.precision, training,
                                           opts.memory_budget, channels=c, gpu=fmap1.is_cuda)
        scale = float(c) ** -0.5 if self.scale is None else float(self.scale)
        if self.method == "otf":
            self.pyramid = None
            if tokens:
                self._otf, self._state, self._token = ops.otf_block_autograd(fmap1, fmap2, num_levels, self.precision,
                                                                             scale)
            else:
                self._otf = ops.otf_prepare(fmap1, fmap2, num_levels, self.precision, scale=scale)
        elif tokens:
            self.pyramid, self._state, self._token = ops.corr_block_autograd(fmap1, fmap2, num_levels,
                                                                             self.precision, self.scale)
        else:
            self.pyramid = ops.corr_pyramid(fmap1, fmap2, num_levels, self.precision, scale=self.scale)

    @property
    def corr_pyramid(self):
        """Levels in the reference layout (B, H, W, 1, H_i, W_i) — unpacked copies, for inspection."""
        if self.pyramid is None:
            raise AttributeError("corr_pyramid: this block runs on the fly (method='otf') and holds no volume")
        return [self.pyramid.unpack(i) for i in range(self.num_levels)]

    def __call__(self, coords, mask_costs=[]):
        if self.method == "otf":
            if self._token is not None and torch.is_grad_enabled():
                return ops.otf_lookup_autograd(self._token, self._state, coords, self.radius, mask_costs)
            return ops.otf_lookup(self._otf, coords, self.radius, mask_costs)
        if self._token is not None and torch.is_grad_enabled():
            return ops.corr_lookup_autograd(self._token, self._state, coords, self.radius, mask_costs)
        return ops.corr_lookup(self.pyramid, coords, self.radius, mask_costs)


# per-iteration heads of raft.py (Up8Network :299-331, soft-argmax regressions :98-190)
from .heads import (Up8Network, SoftArgMaxFlowRegression, SoftArgMaxFlowRegressionWithDap,  # noqa: E402,F401
                    make_flow_regression)
