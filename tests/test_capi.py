"""CPU-side checks of the C ABI: the library loads, exports every symbol include/rmd.h declares,
and the host-only geometry call behaves (no compute calls without a GPU)."""

import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rmd.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(rmd_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from rmd import _lib
    lib = _lib.lib()
    names = _declared()
    assert "rmd_corr_pyramid" in names and "rmd_corr_lookup" in names
    for n in names:
        assert hasattr(lib, n), f"librmd.so does not export {n}"
    assert set(_lib.symbols()) == set(names), "ctypes signatures out of sync with include/rmd.h"


def test_version():
    from rmd import _lib
    assert _lib.lib().rmd_version().startswith(b"rmd ")


def test_describe_cfg2_geometry():
    from rmd import _lib
    d = _lib.describe(8, 55, 128, 4, _lib.RMD_F16)
    assert [d.level_h[i] for i in range(4)] == [55, 27, 13, 6]
    assert [d.level_w[i] for i in range(4)] == [128, 64, 32, 16]
    assert [d.tile_h[i] for i in range(4)] == [1, 1, 1, 1]
    assert [d.tile_w[i] for i in range(4)] == [8, 8, 4, 2]
    assert [d.tiles_y[i] for i in range(4)] == [55, 27, 13, 6]
    assert [d.tiles_x[i] for i in range(4)] == [16, 8, 8, 8]
    n = 55 * 128
    sizes = [55 * 128, 27 * 64, 13 * 32, 6 * 16]
    assert d.total_elements == 8 * n * sum(sizes)
    assert [d.level_offset[i] for i in range(4)] == [0] + [8 * n * sum(sizes[:i]) for i in range(1, 4)]


@pytest.mark.parametrize("args", [(0, 4, 4, 1, 0), (1, 4, 4, 5, 0), (1, 4, 4, 1, 7), (1, 7, 9, 4, 0)])
def test_describe_rejects_bad_shapes(args):
    from rmd import _lib
    with pytest.raises(_lib.RmdError):
        _lib.describe(*args)


def test_no_cpu_fallback():
    import torch
    import rmd
    f = torch.zeros(1, 8, 8, 8)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        rmd.raft.CorrBlock(f, f)
