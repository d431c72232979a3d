"""Drop-in for raft_fs.CorrBlock — qzed/raft-meets-dicl src/models/impls/raft_fs.py:13-87.

The reference samples the (2r+1)^2 window of each avg-pooled fmap2 level with grid_sample and dots
it with fmap1, without the 1/sqrt(C) of raft.CorrBlock.  Two implementations behind the reference's
constructor / call / output ((B, L*(2r+1)^2, H, W) contiguous float32):

* method="volume" (default): pooling fmap2 commutes with the product and bilinear sampling of
  features then a dot equals sampling of the dots, so this is the all-pairs pyramid + lookup of
  rmd.raft.CorrBlock with scale 1 (the reference's two blocks agree to 1.9e-6).
  Differentiable (training).  On MI355X the fp16 volume of a B=8, 1/8-of-440x1024 batch is 1 GB,
  so building it once beats re-gathering features every GRU iteration at these sizes.
* method="otf": rmd_corr_otf_* — no volume in HBM (O(B*C*N) memory), each lookup computes the
  windowed products on the fly with MFMA over the union box of a query block's windows
  (inference only).
"""

import torch

from . import ops, raft


class CorrBlock(raft.CorrBlock):
    """Correlation volume for matching costs, raft/fs semantics (no 1/sqrt(C))."""

    scale = 1.0

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, precision=None, method="volume"):
        if method not in ("volume", "otf"):
            raise ValueError(f"unknown method '{method}'")
        self.method = method
        if method == "volume":
            super().__init__(fmap1, fmap2, num_levels, radius, precision)
            return
        if torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad):
            raise RuntimeError("raft_fs.CorrBlock(method='otf') is inference-only; use method='volume' to train")
        self.num_levels, self.radius = num_levels, radius
        self.precision = precision or ops.get_default_precision()
        self._state = self._token = None
        self._otf = ops.otf_prepare(fmap1, fmap2, num_levels, self.precision, scale=1.0)

    def __call__(self, coords, mask_costs=[]):
        if self.method == "otf":
            return ops.otf_lookup(self._otf, coords, self.radius, mask_costs)
        return super().__call__(coords, mask_costs)
