"""Host logic of rmd.config (op selection from cfg/model ``parameters``; SURVEY.md §5 "Config / flags")."""

import pytest

from rmd import config


def test_defaults_reproduce_the_reference():
    o = config.corr_options({})
    assert o.precision == config.current().precision
    assert o.method == config.current().method


def test_parameters_and_overrides():
    o = config.corr_options({"corr-precision": "bf16", "corr-method": "volume", "corr-memory-budget": "2GiB"})
    assert o == ("bf16", "volume", 2 << 30)
    o = config.corr_options({"corr-precision": "bf16"}, precision="fp32-exact", memory_budget=4096)
    assert o.precision == "fp32-exact" and o.memory_budget == 4096
    assert config.corr_options(None, **o.kwargs()) == o
    assert config.corr_options(o.parameters()) == o


@pytest.mark.parametrize("kw", [{"memory_budget": 0}, {"memory_budget": -5}, {"precision": ""}, {"method": ""},
                                {"precision": "fp64"}, {"method": "fast"}])
def test_explicit_invalid_overrides_raise(kw):
    # falsy explicit values reach the validation instead of silently falling back
    with pytest.raises(ValueError):
        config.corr_options({}, **kw)


def test_budget_strings():
    assert config._bytes("64KiB") == 64 << 10
    assert config._bytes("1.5 GiB") == 3 << 29
    with pytest.raises(ValueError):
        config._bytes("lots")


def test_auto_method_by_budget():
    small = config.choose_method("auto", 1, 8, 8, 4, "bf16", False, 1 << 30)
    big = config.choose_method("auto", 8, 270, 480, 4, "bf16", False, 1 << 30)
    assert (small, big) == ("volume", "otf")
    assert config.choose_method("volume", 8, 270, 480, 4, "bf16", False, 1) == "volume"


def test_otf_training_channel_limit():
    # the on-the-fly backward takes C <= 256: auto keeps the volume for wider training blocks and an
    # explicit 'otf' fails at construction, not in backward
    assert config.choose_method("auto", 8, 270, 480, 4, "bf16", True, 1 << 30, channels=256) == "otf"
    assert config.choose_method("auto", 8, 270, 480, 4, "bf16", True, 1 << 30, channels=320) == "volume"
    assert config.choose_method("auto", 8, 270, 480, 4, "bf16", False, 1 << 30, channels=320) == "otf"
    with pytest.raises(ValueError, match="C <= 256"):
        config.choose_method("otf", 8, 270, 480, 4, "bf16", True, 1 << 30, channels=512)
    assert config.choose_method("otf", 8, 270, 480, 4, "bf16", False, 1 << 30, channels=512) == "otf"


def test_cpu_otf_block_trains_above_256_channels():
    # the C <= 256 limit is the HIP backward's: a CPU block with C = 320 and method='otf' trains
    # through the ATen kernels
    import torch

    import rmd
    g = torch.Generator().manual_seed(0)
    f1 = torch.randn(1, 320, 6, 8, generator=g, requires_grad=True)
    f2 = torch.randn(1, 320, 6, 8, generator=g, requires_grad=True)
    cb = rmd.raft.CorrBlock(f1, f2, 2, 2, precision="fp32", method="otf")
    assert cb.method == "otf"
    ys, xs = torch.meshgrid(torch.arange(6.0), torch.arange(8.0), indexing="ij")
    coords = torch.stack([xs, ys])[None] + 0.3
    cb(coords).square().sum().backward()
    assert f1.grad is not None and f2.grad is not None
    assert torch.isfinite(f1.grad).all() and float(f2.grad.abs().sum()) > 0


def test_configure_restore():
    prev = config.configure({"corr-precision": "bf16"})
    try:
        assert config.current().precision == "bf16"
    finally:
        config.restore(prev)
    assert config.current() == prev


def test_volume_bytes_resolve_the_pyramid_storage():
    """'fp32' stores S24 (3 bytes) only where the x3 GEMM runs; C > 256, a level slab of
    >= 2 GiB (large maps) and CPU blocks store F32, and the budget must charge those 4 bytes."""
    from rmd import _lib
    tot = _lib.describe(8, 55, 128, 4, _lib.RMD_F32).total_elements
    assert config.pyramid_bytes(8, 55, 128, 4, "fp32", channels=256) == 3 * tot
    assert config.pyramid_bytes(8, 55, 128, 4, "fp32", channels=320) == 4 * tot       # tiled f32 GEMM
    assert config.pyramid_bytes(8, 55, 128, 4, "fp32", channels=256, gpu=False) == 4 * tot
    assert config.pyramid_bytes(8, 55, 128, 4, "fp32") == 4 * tot                     # C unknown: larger
    assert config.pyramid_bytes(8, 55, 128, 4, "fp32-f32", channels=256) == 4 * tot
    # bf16: the w8 GEMM's tiles layout (odd H pads level-0/1 chunk rows)
    tiles = _lib.describe_for(8, 55, 128, 4, _lib.RMD_F16, 256, _lib.RMD_BF16)
    assert config.pyramid_bytes(8, 55, 128, 4, "bf16", channels=256) == 2 * tiles.total_elements > 2 * tot
    big = _lib.describe(1, 270, 480, 4, _lib.RMD_F32).total_elements                 # 4K 1/8 map
    assert config.pyramid_bytes(1, 270, 480, 4, "fp32", channels=256) == 4 * big
    # a budget between the S24 and the F32 size: auto keeps the volume only where S24 applies
    budget = int(3.5 * tot)
    assert config.choose_method("auto", 8, 55, 128, 4, "fp32", False, budget, channels=256) == "volume"
    assert config.choose_method("auto", 8, 55, 128, 4, "fp32", False, budget, channels=320) == "otf"
    assert config.choose_method("auto", 8, 55, 128, 4, "fp32", False, budget, channels=256, gpu=False) == "otf"
