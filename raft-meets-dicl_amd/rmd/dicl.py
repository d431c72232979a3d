"""DICL baseline cost volume — drop-in for FlowLevel.compute_cost (src/models/impls/dicl.py:212-241)
and the feature warp in front of it (FlowLevel.forward, :171-184).

`compute_cost(mnet, feat1, feat2, maxdisp)` builds the masked integer-displacement volume with one
rmd_dicl_stack_int pass and runs the (unchanged) MatchingNet on it.  With `flow` given, feat2 is first
warped back by it (common/warp.py) inside the same kernel pair (rmd_dicl_stack_int_warped), so the
warped map never makes the reference's extra grid_sample/mask round trip.

`FlowLevelCostMixin` gives a reference FlowLevel the same methods:
    class FlowLevel(FlowLevelCostMixin, reference.FlowLevel)
Its forward reproduces FlowLevel.forward (coarse flow upsampled x2, detached) and hands the flow to
compute_cost instead of warping feat2 separately.
"""

import torch.nn.functional as F

from . import ops


def cost_volume(feat1, feat2, maxdisp, flow=None):
    """(B,C,h,w) x2 [+ flow (B,2,h,w)] -> (B, 2ru+1, 2rv+1, 2C, h, w) masked matching volume."""
    ru, rv = (int(m) for m in maxdisp)
    if flow is not None:
        return ops.dicl_stack_int_warped(feat1, feat2, flow, ru, rv)
    return ops.dicl_stack_int(feat1, feat2, ru, rv)


def compute_cost(mnet, feat1, feat2, maxdisp, flow=None):
    return mnet(cost_volume(feat1, feat2, maxdisp, flow))


class FlowLevelCostMixin:
    _warp_flow = None

    def forward(self, img1, feat1, feat2, flow_coarse, raw=False, dap=True, ctx=True, scale=1.0):
        _, _, h, w = feat1.shape
        flow_up = None
        if flow_coarse is not None:
            flow_up = (2.0 * F.interpolate(flow_coarse, (h, w), mode="bilinear", align_corners=True)).detach()
        self._warp_flow = flow_up                  # consumed by compute_cost (fused warp)
        try:
            return self.compute_flow(img1, feat1, feat2, flow_up, raw, dap, ctx, scale)
        finally:
            self._warp_flow = None

    def compute_cost(self, feat1, feat2):
        return compute_cost(self.mnet, feat1, feat2, self.maxdisp, self._warp_flow)
