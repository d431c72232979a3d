"""DICL baseline cost volume — drop-in for FlowLevel.compute_cost (src/models/impls/dicl.py:212-241).

`compute_cost(mnet, feat1, feat2, maxdisp)` builds the masked integer-displacement volume with one
rmd_dicl_stack_int pass and runs the (unchanged) MatchingNet on it.  `FlowLevelCostMixin` gives a
reference FlowLevel the same method:  class FlowLevel(FlowLevelCostMixin, reference.FlowLevel).
"""

from . import ops


def cost_volume(feat1, feat2, maxdisp):
    """(B,C,h,w) x2 -> (B, 2ru+1, 2rv+1, 2C, h, w) masked matching volume (dicl.py:212-238)."""
    ru, rv = (int(m) for m in maxdisp)
    return ops.dicl_stack_int(feat1, feat2, ru, rv)


def compute_cost(mnet, feat1, feat2, maxdisp):
    return mnet(cost_volume(feat1, feat2, maxdisp))


class FlowLevelCostMixin:
    def compute_cost(self, feat1, feat2):
        return compute_cost(self.mnet, feat1, feat2, self.maxdisp)
