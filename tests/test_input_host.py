"""rmd.input.InputSpec.prepare(device='cpu'): the host path of the input format (the reference's own
numpy clip / range map / np.pad and NCHW permute, input.py:32-313) against the golden vectors the
reference produced (tests/golden/gen_golden_input.py).  Bit-exact.  CPU only: no HIP library call."""

import numpy as np
import pytest

from conftest import load_golden

CASES = ["zeros_lt", "zeros_cc64", "ones_rb", "edge_cc", "reflect_lt", "symmetric_rb", "wrap_cc", "trep_lt",
         "trefl_cc", "tcirc_rb"]


@pytest.mark.parametrize("case", CASES)
def test_host_input_format_matches_reference_golden(case):
    from rmd.input import InputSpec, ModuloPadding
    g = load_golden(f"input_{case}")
    pad = ModuloPadding(str(g["mode"]), g["size"].tolist(), align_hz=str(g["align_hz"]), align_vt=str(g["align_vt"]))
    spec = InputSpec(tuple(g["clip"].tolist()), tuple(g["range"].tolist()), pad)
    o1, o2, fo, vo, ext = spec.prepare(g["img1"], g["img2"], g["flow"], g["valid"], device="cpu")
    assert not o1.is_cuda and o1.is_contiguous() and vo.dtype.is_floating_point is False
    assert np.array_equal(o1.numpy(), g["out1"])
    assert np.array_equal(o2.numpy(), g["out2"])
    assert np.array_equal(fo.numpy(), g["out_flow"])
    assert np.array_equal(vo.numpy(), g["out_valid"])
    assert [list(e) for e in ext] == g["extents"].tolist()


def test_host_statistic_pad_mode_follows_np_pad():
    """The statistic modes (no GPU kernel) pad as the reference's np.pad does (input.py:79-118)."""
    from rmd.input import InputSpec, ModuloPadding
    rng = np.random.default_rng(3)
    img = rng.uniform(0, 1, (1, 5, 7, 3)).astype(np.float32)
    spec = InputSpec(clip=(0.0, 1.0), range=(0.0, 1.0), padding=ModuloPadding("median", [8, 8]))
    o1, _, fo, vo, ext = spec.prepare(img, img, device="cpu")
    ref = np.pad(img, ((0, 0), (0, 3), (0, 1), (0, 0)), mode="median").transpose(0, 3, 1, 2)
    assert fo is None and vo is None and ext == ((0, 8), (0, 8))
    assert np.array_equal(o1.numpy(), ref)


def test_host_input_shape_errors():
    from rmd.input import InputSpec
    with pytest.raises(ValueError, match="equal"):
        InputSpec().prepare(np.zeros((1, 4, 4, 3), np.float32), np.zeros((1, 4, 5, 3), np.float32), device="cpu")
    with pytest.raises(ValueError, match="flow/valid"):
        InputSpec().prepare(np.zeros((1, 4, 4, 3), np.float32), np.zeros((1, 4, 4, 3), np.float32),
                            np.zeros((1, 4, 4, 3), np.float32), np.zeros((1, 4, 4), bool), device="cpu")
