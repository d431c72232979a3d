"""GPU parity of the input format kernels (rmd_input_images / rmd_input_flow through rmd.input)
against golden vectors from the reference's ModuloPadding + Input + TorchAdapter (input.py:32-313)
and the numpy oracle.  Tolerance: bit-exact (clip, one multiply and one add in float32, copies)."""

import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden

pytestmark = pytest.mark.gpu

CASES = ["zeros_lt", "zeros_cc64", "ones_rb", "edge_cc", "reflect_lt", "symmetric_rb", "wrap_cc", "trep_lt",
         "trefl_cc", "tcirc_rb"]


def _spec(g):
    from rmd.input import InputSpec, ModuloPadding
    pad = ModuloPadding(str(g["mode"]), g["size"].tolist(), align_hz=str(g["align_hz"]), align_vt=str(g["align_vt"]))
    return InputSpec(tuple(g["clip"].tolist()), tuple(g["range"].tolist()), pad)


@pytest.mark.parametrize("case", CASES)
def test_input_format_matches_reference_golden(case):
    g = load_golden(f"input_{case}")
    o1, o2, fo, vo, ext = _spec(g).prepare(g["img1"], g["img2"], g["flow"], g["valid"])
    assert np.array_equal(o1.cpu().numpy(), g["out1"])
    assert np.array_equal(o2.cpu().numpy(), g["out2"])
    assert np.array_equal(fo.cpu().numpy(), g["out_flow"])
    assert np.array_equal(vo.cpu().numpy(), g["out_valid"])
    assert [list(e) for e in ext] == g["extents"].tolist()


@pytest.mark.parametrize("mode", ["zeros", "reflect", "wrap"])
def test_input_sintel_shape_vs_oracle(mode):
    """cfg2 frames: 436x1024 -> 440x1024 (raft-baseline.yaml modulo 8), B=2, from GPU-resident frames;
    plus a 376x1242 KITTI frame padded to 384x1280 (ctf-l3 modulo 64), centred."""
    from rmd.input import InputSpec, ModuloPadding
    rng = np.random.default_rng(11)
    for (h, w, size, al) in ((436, 1024, [8, 8], "left"), (376, 1242, [64, 64], "center")):
        img = rng.uniform(-0.1, 1.1, (2, h, w, 3)).astype(np.float32)
        spec = InputSpec(padding=ModuloPadding(mode, size, align_hz=al, align_vt="top" if al == "left" else "center"))
        o1, o2, _, _, _ = spec.prepare(torch.from_numpy(img).cuda(), img)
        ref = oracle.input_images(img, mode=mode, size=size, align_hz=al, align_vt="top" if al == "left" else "center")
        assert o1.shape == (2, 3) + ref.shape[2:] and np.array_equal(o1.cpu().numpy(), ref)
        assert np.array_equal(o2.cpu().numpy(), ref)


def test_input_errors_match_reference():
    from rmd.input import InputSpec, ModuloPadding
    with pytest.raises(ValueError, match="invalid padding mode"):
        ModuloPadding("nearest", [8, 8])
    with pytest.raises(ValueError, match="invalid horizontal alignment"):
        ModuloPadding("zeros", [8, 8], align_hz="middle")
    with pytest.raises(ValueError, match="expected list/tuple of 2 integers"):
        ModuloPadding.from_config({"type": "modulo", "mode": "zeros", "size": [8]})
    spec = InputSpec(padding=ModuloPadding("median", [8, 8]))
    with pytest.raises(NotImplementedError):
        spec.prepare(np.zeros((1, 4, 4, 3), np.float32), np.zeros((1, 4, 4, 3), np.float32))
    with pytest.raises(RuntimeError, match="runs on 'cuda'"):
        InputSpec().prepare(np.zeros((1, 4, 4, 3), np.float32), np.zeros((1, 4, 4, 3), np.float32), device="meta")


def test_input_gpu_and_host_paths_agree():
    """The same frames through prepare(device='cuda') (HIP kernels) and prepare(device='cpu') (the
    reference's host numpy path): bitwise equal, the GPU result on the GPU, the host one on the CPU."""
    from rmd.input import InputSpec, ModuloPadding
    rng = np.random.default_rng(12)
    img1, img2 = (rng.uniform(-0.2, 1.2, (2, 37, 53, 3)).astype(np.float32) for _ in range(2))
    flow = rng.normal(0, 5, (2, 37, 53, 2)).astype(np.float32)
    flow[0, 0, 0, 0] = np.nan
    valid = rng.uniform(size=(2, 37, 53)) > 0.3
    spec = InputSpec(padding=ModuloPadding("reflect", [16, 8], align_hz="center", align_vt="bottom"))
    g = spec.prepare(img1, img2, flow, valid)
    h = spec.prepare(img1, img2, flow, valid, device="cpu")
    assert g[0].is_cuda and not h[0].is_cuda
    for a, b in zip(g[:4], h[:4]):
        assert np.array_equal(a.cpu().numpy(), b.numpy())
    assert g[4] == h[4]
