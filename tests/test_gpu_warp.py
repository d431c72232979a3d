"""GPU parity of backward warping (rmd_warp_backwards) and the warped DICL integer volume
(rmd_dicl_stack_int_warped) against reference golden vectors and the float64 oracle.

Tolerances (max-normalised): warped values and volumes 1e-5 (bilinear in fp32 pixel coordinates vs the
reference's [-1, 1] grid round trip); validity masks and the zero pattern of the occlusion-masked
volume exact.  Edge cases from the fixture: zero flow at a corner, a sample landing exactly on the far
corner, half a pixel outside, far outside, 1e-7 past the border (mask tolerance eps), zeroed feature
vectors (occlusion holes after warping).
"""

import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden, rel_max_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a, grad=False):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV).requires_grad_(grad)


def test_warp_backwards_matches_reference_golden():
    import rmd
    g = load_golden("warp_b2_c8_10x12")
    img = _t(g["img2"], True)
    est, mask = rmd.warp.warp_backwards(img, _t(g["flow"]))
    assert est.shape == img.shape and mask.dtype == torch.bool and tuple(mask.shape) == g["mask"].shape
    assert np.array_equal(mask.cpu().numpy(), g["mask"])
    assert rel_max_err(est.detach().cpu().numpy(), g["est"]) < 1e-5
    (gi,) = torch.autograd.grad(est, img, _t(g["grad_out"]))
    assert rel_max_err(gi.cpu().numpy(), g["grad_img2"]) < 1e-5


@pytest.mark.parametrize("b,c,h,w,sigma", [(2, 32, 48, 64, 4.0), (1, 3, 37, 53, 10.0), (3, 1, 1, 8, 2.0)])
def test_warp_backwards_vs_oracle(b, c, h, w, sigma):
    import rmd
    rng = np.random.default_rng(c * 7 + h)
    img = rng.standard_normal((b, c, h, w)).astype(np.float32)
    flow = (sigma * rng.standard_normal((b, 2, h, w))).astype(np.float32)
    ti = _t(img, True)
    est, mask = rmd.warp.warp_backwards(ti, _t(flow))
    rest, rmask = oracle.warp_backwards(img.astype(np.float64), flow.astype(np.float64))
    assert np.array_equal(mask[:, 0].cpu().numpy(), rmask)
    assert rel_max_err(est.detach().cpu().numpy(), rest) < 1e-5
    go = rng.standard_normal(img.shape).astype(np.float32)
    (gi,) = torch.autograd.grad(est, ti, _t(go))
    assert rel_max_err(gi.cpu().numpy(), oracle.warp_backwards_backward(flow.astype(np.float64),
                                                                       go.astype(np.float64))) < 1e-5


def test_warped_dicl_volume_matches_reference_golden():
    import rmd
    g = load_golden("warp_dicl_cost_b2_c16_10x12")
    ru, rv = g["maxdisp"].tolist()
    f1, f2 = _t(g["fmap1"], True), _t(g["fmap2"], True)
    mvol = rmd.ops.dicl_stack_int_warped(f1, f2, _t(g["flow_up"]), ru, rv)
    got = mvol.detach().cpu().numpy()
    assert got.shape == g["mvol"].shape
    assert np.array_equal(got == 0, g["mvol"] == 0)           # occlusion / out-of-bounds zeros exact
    assert rel_max_err(got, g["mvol"]) < 1e-5
    d1, d2 = torch.autograd.grad(mvol, (f1, f2), _t(g["grad_mvol"]))
    assert rel_max_err(d1.cpu().numpy(), g["grad_fmap1"]) < 1e-5
    assert rel_max_err(d2.cpu().numpy(), g["grad_fmap2"]) < 1e-5


def test_flow_level_mixin_fuses_the_warp():
    """A FlowLevel using the mixin sees the reference's MatchingNet input (coarse flow upsampled x2)."""
    import rmd
    g = load_golden("warp_dicl_cost_b2_c16_10x12")
    seen = {}

    class _Level:                                   # the parts of impls/dicl.FlowLevel the mixin relies on
        maxdisp = tuple(g["maxdisp"].tolist())

        def mnet(self, mvol):
            seen["mvol"] = mvol
            return mvol

        def compute_flow(self, img1, feat1, feat2, flow_coarse, raw, dap, ctx, scale):
            seen["flow_up"] = flow_coarse
            return self.compute_cost(feat1, feat2)

    class Level(rmd.dicl.FlowLevelCostMixin, _Level):
        pass

    Level().forward(None, _t(g["fmap1"]), _t(g["fmap2"]), _t(g["flow_coarse"]), ctx=False)
    assert rel_max_err(seen["flow_up"].cpu().numpy(), g["flow_up"]) < 1e-6
    assert rel_max_err(seen["mvol"].cpu().numpy(), g["mvol"]) < 1e-5


def test_warped_volume_cfg3_shape_vs_oracle():
    """cfg3 level-3 shape (48x64, C=32, ru=rv=3, B=2) against the oracle's warp + volume."""
    import rmd
    rng = np.random.default_rng(11)
    b, c, h, w = 2, 32, 48, 64
    f1 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    f2 = rng.standard_normal((b, c, h, w)).astype(np.float32)
    flow = (3.0 * rng.standard_normal((b, 2, h, w))).astype(np.float32)
    got = rmd.ops.dicl_stack_int_warped(_t(f1), _t(f2), _t(flow), 3, 3).cpu().numpy()
    warped, _ = oracle.warp_backwards(f2.astype(np.float64), flow.astype(np.float64))
    ref = oracle.dicl_stack_int(f1.astype(np.float64), warped, 3, 3)
    assert np.array_equal(got == 0, ref == 0)
    assert rel_max_err(got, ref) < 1e-5
