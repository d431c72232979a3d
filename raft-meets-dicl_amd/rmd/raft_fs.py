"""Drop-in for raft_fs.CorrBlock — qzed/raft-meets-dicl src/models/impls/raft_fs.py:13-87.

The reference samples the (2r+1)^2 window of each avg-pooled fmap2 level with grid_sample and dots
it with fmap1, without the 1/sqrt(C) of raft.CorrBlock.  Two implementations behind the reference's
constructor / call / output ((B, L*(2r+1)^2, H, W) contiguous float32):

* method="volume": pooling fmap2 commutes with the product and bilinear sampling of
  features then a dot equals sampling of the dots, so this is the all-pairs pyramid + lookup of
  rmd.raft.CorrBlock with scale 1 (the reference's two blocks agree to 1.9e-6).
  Differentiable (training).  On MI355X the fp16 volume of a B=8, 1/8-of-440x1024 batch is 1 GB,
  so building it once beats re-gathering features every GRU iteration at these sizes.
* method="otf": rmd_corr_otf_* — no volume in HBM (O(B*C*N) memory), each lookup computes the
  windowed products on the fly with MFMA over the union box of a query block's windows
  (SURVEY.md §8(f) rank 1); its backward records each lookup's patch weights and turns them into
  d fmap1 / d fmap2 in one pass (rmd_corr_otf_backward).
* method="auto" (default, rmd.config): the volume while it fits the memory budget, else otf.
"""

from . import raft


class CorrBlock(raft.CorrBlock):
    """Correlation volume for matching costs, raft/fs semantics (no 1/sqrt(C)).  Same op selection as
    rmd.raft.CorrBlock (precision / method / memory_budget, rmd.config)."""

    scale = 1.0
