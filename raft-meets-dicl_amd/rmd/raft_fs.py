"""Drop-in for raft_fs.CorrBlock — qzed/raft-meets-dicl src/models/impls/raft_fs.py:13-87.

The reference samples the (2r+1)^2 window of each avg-pooled fmap2 level with grid_sample and dots
it with fmap1, without the 1/sqrt(C) of raft.CorrBlock.  Pooling fmap2 commutes with the product
(level l of fmap1 . fmap2 pooled over 2^l x 2^l targets == fmap1 . pooled fmap2), and bilinear
sampling of features followed by a dot equals bilinear sampling of the dots, so this block is the
all-pairs pyramid + windowed lookup of rmd.raft.CorrBlock with scale 1 instead of 1/sqrt(C)
(the two agree to 1.9e-6 in the reference itself).  On MI355X the volume of
a (B=8, 1/8 of 440x1024) pair batch is 1 GB in fp16, so building it beats re-gathering
B*C*81*H*W features per GRU iteration (raft_fs.py:68-71); a memory-lean on-the-fly kernel for
volumes beyond HBM is SURVEY.md §8(f) rank 1.  Same constructor / call / output as the reference
((B, L*(2r+1)^2, H, W) contiguous float32); autograd to fmap1 and fmap2 as rmd.raft.CorrBlock.
"""

from . import raft


class CorrBlock(raft.CorrBlock):
    """Correlation volume for matching costs, raft/fs semantics (no 1/sqrt(C))."""

    scale = 1.0
