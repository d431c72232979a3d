"""torch.library registration of the rmd operators (SURVEY.md §8(b) op schemas).

CPU: every operator is registered with a schema, its fake (meta) kernel propagates shapes and dtypes
without a GPU (FakeTensor tracing for torch.compile / export), and real CPU tensors raise (no CPU
fallback).  GPU (marked): torch.library.opcheck — schema, fake-vs-real outputs, autograd
registration — on small shapes of every operator family.
"""

import pytest
import torch

EXPECTED = ["corr_lookup", "corr_otf_lookup", "corr_otf_prepare", "corr_pyramid", "dap", "dap_transpose",
            "dap_weight_grad",
            "dicl_stack", "dicl_stack_backward", "dicl_stack_int", "dicl_stack_int_backward", "dicl_stack_int_warped",
            "dicl_stack_int_warped_backward", "softargmax", "softargmax_backward", "up8", "up8_backward",
            "warp_backwards", "warp_backwards_backward"]


def test_every_operator_registered():
    from rmd import library
    assert library.operators() == EXPECTED
    for name in EXPECTED:
        assert hasattr(torch.ops.rmd, name)


def test_fake_kernels_propagate_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    from rmd import _lib
    with FakeTensorMode():
        f1 = torch.empty(2, 256, 55, 128, device="cuda")
        pyr = torch.ops.rmd.corr_pyramid(f1, f1, 4, _lib.RMD_BF16, _lib.RMD_F16, 0.0625)
        d = _lib.describe(2, 55, 128, 4, _lib.RMD_F16, _lib.RMD_LAYOUT_TILES)     # the w8 GEMM's layout
        assert pyr.dtype == torch.float16 and pyr.numel() == d.total_elements
        assert pyr.shape == (d.total_elements // 8, 8)                              # tiles: (n, 8)
        co = torch.empty(2, 2, 55, 128, device="cuda")
        assert torch.ops.rmd.corr_lookup(pyr, co, 4, 4, 0).shape == (2, 324, 55, 128)
        rows = torch.ops.rmd.corr_pyramid(f1, f1, 4, _lib.RMD_BF16X3, _lib.RMD_F32, 0.0625)
        assert rows.dim() == 1                                                       # row layout: 1-D
        assert torch.ops.rmd.corr_lookup(rows, co, 4, 4, 0).shape == (2, 324, 55, 128)
        s24 = torch.ops.rmd.corr_pyramid(f1, f1, 4, _lib.RMD_BF16X3, _lib.RMD_S24, 0.0625)
        assert s24.dtype == torch.uint8 and s24.shape == (rows.numel(), 3)          # S24: (n, 3) bytes
        assert torch.ops.rmd.corr_lookup(s24, co, 4, 4, 0).shape == (2, 324, 55, 128)
        f320 = torch.empty(2, 320, 55, 128, device="cuda")                           # C > 256: no x3 -> F32
        assert torch.ops.rmd.corr_pyramid(f320, f320, 4, _lib.RMD_BF16X3, _lib.RMD_S24, 0.0625).dtype == torch.float32
        with pytest.raises(ValueError, match="tiles layout"):
            torch.ops.rmd.corr_lookup(pyr.view(-1, 16), co, 4, 4, 0)
        f = torch.empty(2, 32, 12, 16, device="cuda")
        c2 = torch.empty(2, 2, 12, 16, device="cuda")
        assert torch.ops.rmd.dicl_stack(f, f, c2, 4, 0, 12, 16, False).shape == (2, 9, 9, 64, 12, 16)
        assert torch.ops.rmd.dicl_stack(f, f, c2, 4, 0, 12, 16, True).shape == (2, 9, 9, 66, 12, 16)
        assert torch.ops.rmd.dicl_stack_int(f, f, 3, 3).shape == (2, 7, 7, 64, 12, 16)
        assert torch.ops.rmd.dap(torch.empty(2, 81, 12, 16, device="cuda"), torch.empty(81, 81, 1, 1, device="cuda")).shape == (2, 81, 12, 16)
        assert torch.ops.rmd.up8(torch.empty(2, 576, 12, 16, device="cuda"), c2, 4.0).shape == (2, 2, 96, 128)
        assert torch.ops.rmd.softargmax(torch.empty(2, 324, 12, 16, device="cuda"), 4, 4, 1.0).shape == (4, 2, 2, 12, 16)
        out, mask = torch.ops.rmd.warp_backwards(f, c2, 1e-5)
        assert out.shape == f.shape and mask.shape == (2, 1, 12, 16) and mask.dtype == torch.bool


def test_cpu_tensors_dispatch_to_the_cpu_kernels():
    """CPU tensors reach rmd/cpu.py (the reference's ATen algorithm; tests/test_cpu_dispatch.py checks
    it against the golden vectors); mixed devices are rejected before any kernel runs."""
    import torch.nn.functional as F
    x, w = torch.randn(2, 81, 4, 5), torch.randn(81, 81)
    assert torch.allclose(torch.ops.rmd.dap(x, w), F.conv2d(x, w[:, :, None, None]), atol=1e-5)
    assert torch.ops.rmd.dicl_stack_int(torch.ones(1, 8, 4, 4), torch.ones(1, 8, 4, 4), 1, 1).shape == (1, 3, 3, 16, 4, 4)
    from rmd import ops
    with pytest.raises(ValueError, match="different devices"):
        ops.dap(x, w.to("meta"))


@pytest.mark.gpu
def test_opcheck_operator_families():
    from rmd import _lib
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    ys, xs = torch.meshgrid(torch.arange(10.0), torch.arange(12.0), indexing="ij")
    co = (torch.stack([xs, ys])[None].expand(2, -1, -1, -1) + torch.randn(2, 2, 10, 12, generator=g) * 2).to(dev)
    f1, f2 = r(2, 16, 10, 12), r(2, 16, 10, 12)
    cases = [
        (torch.ops.rmd.corr_pyramid, (f1, f2, 3, _lib.RMD_BF16X3, _lib.RMD_F32, 0.25)),
        (torch.ops.rmd.dicl_stack, (f1.requires_grad_(), f2.requires_grad_(), co, 2, 0, 10, 12, False)),
        (torch.ops.rmd.dicl_stack_int, (f1, f2, 2, 2)),
        (torch.ops.rmd.dap, (r(2, 25, 10, 12).requires_grad_(), r(25, 25, 1, 1).requires_grad_())),
        (torch.ops.rmd.dap_weight_grad, (r(2, 25, 10, 12), r(2, 25, 10, 12), 25)),
        (torch.ops.rmd.up8, (r(2, 576, 10, 12).requires_grad_(), r(2, 2, 10, 12).requires_grad_(), 4.0)),
        (torch.ops.rmd.softargmax, (r(2, 81, 10, 12).requires_grad_(), 1, 4, 1.0)),
    ]
    for op, args in cases:
        torch.library.opcheck(op, args, test_utils=("test_schema", "test_autograd_registration", "test_faketensor"))
    for compute, storage in ((_lib.RMD_BF16X3, _lib.RMD_F32), (_lib.RMD_BF16, _lib.RMD_F16)):     # rows, tiles
        pyr = torch.ops.rmd.corr_pyramid(f1.detach(), f2.detach(), 3, compute, storage, 0.25)
        torch.library.opcheck(torch.ops.rmd.corr_lookup, (pyr, co, 3, 2, 0),
                              test_utils=("test_schema", "test_autograd_registration", "test_faketensor"))


@pytest.mark.parametrize("kind,fixture", [("dicl", "dicl_b1_c16_8x12"), ("dicl-1x1", "dicl1x1_b2_c16_8x12"),
                                          ("dicl-emb", "diclemb_b2_c16_8x12")])
def test_correlation_module_state_dict_keys_match_reference(kind, fixture):
    """The drop-in modules keep the reference's state-dict keys (checkpoints load unchanged): compared
    with the keys the reference module had when the fixture was generated (CPU, no kernels run)."""
    import rmd
    from conftest import load_golden
    g = load_golden(fixture)
    mod = rmd.corr.make_cmod(kind, 16, int(g["radius"]), dap_init="standard")
    assert sorted(mod.state_dict().keys()) == sorted(g["sd.keys"].tolist())
