"""CPU-side checks of the C ABI: the library loads, exports every symbol include/rmd.h declares,
and the host-only geometry call behaves (no compute calls without a GPU)."""

import os
import re

import numpy as np
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


def test_abi_version_matches_header_and_binding():
    """the rmd_corr_grad_gemm signature change is ABI 2; the header, the library and the
    ctypes binding agree on it, and the binding refuses a library of another ABI."""
    from rmd import _lib
    m = re.search(r"#define RMD_ABI_VERSION (\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == _lib.ABI_VERSION == _lib.lib().rmd_abi_version() == 2
    assert _lib.lib().rmd_version().endswith(b"abi 2")


def test_library_was_built_from_these_sources():
    """VERDICT r05 hygiene: the prebuilt library travels with the tree, so it must be the one these
    sources build.  The Makefile bakes a fingerprint of csrc/ + include/rmd.h into it; the file's,
    the loaded library's and the tree's fingerprints agree (build() rebuilds on a mismatch)."""
    from rmd import _lib
    info = _lib.build_info()
    assert info["tree_hash"] is not None and len(info["tree_hash"]) == 16
    assert info["source_hash"] == info["tree_hash"], (
        f"librmd.so was built from other sources ({info['source_hash']} vs tree {info['tree_hash']}): "
        f"run __graft_entry__.build()")
    assert _lib.lib().rmd_source_hash().decode() == info["tree_hash"]


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


def test_describe_for_w8_tiles_layout_geometry():
    """The w8 GEMM (bf16 compute, fp16 storage, C = 256) writes the tiles layout (include/rmd.h):
    2x4, 2x4, 1x4, 1x2 chunks and 2 x 16 query tiles; cfg2's odd H = 55 puts its last row in raster
    slots, so query_slots == H*W."""
    from rmd import _lib
    d = _lib.describe_for(8, 55, 128, 4, _lib.RMD_F16, 256, _lib.RMD_BF16)
    assert d.layout == _lib.RMD_LAYOUT_TILES and d.query_slots == 27 * 8 * 32 + 128 == 55 * 128
    assert [d.tile_h[i] for i in range(4)] == [2, 2, 1, 1]
    assert [d.tile_w[i] for i in range(4)] == [4, 4, 4, 2]
    assert [d.tiles_y[i] for i in range(4)] == [28, 14, 13, 6]
    assert [d.tiles_x[i] for i in range(4)] == [32, 16, 8, 8]
    sizes = [28 * 2 * 128, 14 * 2 * 64, 13 * 32, 6 * 16]
    assert d.total_elements == 8 * d.query_slots * sum(sizes)
    # every other GEMM keeps the row layout
    for storage, compute, c in ((_lib.RMD_F32, _lib.RMD_BF16X3, 256), (_lib.RMD_F16, _lib.RMD_BF16, 128),
                                (_lib.RMD_F32, _lib.RMD_F32, 256)):
        assert _lib.describe_for(8, 55, 128, 4, storage, c, compute).layout == _lib.RMD_LAYOUT_ROWS
    with pytest.raises(_lib.RmdError):
        _lib.describe(1, 8, 8, 2, _lib.RMD_F32, _lib.RMD_LAYOUT_TILES)     # tiles are fp16 only


def test_describe_for_x3_s24_geometry():
    """The x3 GEMM (split-bf16 compute) writes S24 pyramids in the row layout with 1 x 4 level-3 chunks;
    an S24 request another GEMM serves (C > 256, exact f32) resolves to F32 rows."""
    from rmd import _lib
    d = _lib.describe_for(8, 55, 128, 4, _lib.RMD_S24, 256, _lib.RMD_BF16X3)
    assert d.storage == _lib.RMD_S24 and d.layout == _lib.RMD_LAYOUT_ROWS
    assert [d.tile_w[i] for i in range(4)] == [8, 8, 4, 4]
    for c, compute in ((320, _lib.RMD_BF16X3), (256, _lib.RMD_F32)):
        r = _lib.describe_for(8, 55, 128, 4, _lib.RMD_S24, c, compute)
        assert r.storage == _lib.RMD_F32 and r.layout == _lib.RMD_LAYOUT_ROWS


@pytest.mark.parametrize("h,w", [(55, 128), (46, 62), (9, 17), (1, 40), (48, 160)])
def test_tiles_slots_are_a_padded_bijection(h, w):
    """rmd.ops.tiles_slots (the unpack map) is injective, stays below query_slots, and every 8-slot
    group is a 2 x 4 query patch (or 8 consecutive pixels of an odd last row)."""
    from rmd import _lib, ops
    s = ops.tiles_slots(h, w).numpy()
    d = _lib.describe(1, h, w, 1, _lib.RMD_F16, _lib.RMD_LAYOUT_TILES)
    assert len(set(s.tolist())) == h * w and s.max() < d.query_slots and d.query_slots % 32 == 0
    y1, x1 = np.divmod(np.arange(h * w), w)
    for g in np.unique(s // 8):
        m = s // 8 == g
        dy, dx = np.ptp(y1[m]), np.ptp(x1[m])
        assert (dy <= 1 and dx <= 3) or (dy == 0 and dx <= 7 and (h % 2 == 1) and y1[m][0] == h - 1)


@pytest.mark.parametrize("args", [(0, 4, 4, 1, 0), (1, 4, 4, 5, 0), (1, 4, 4, 1, 7), (1, 7, 9, 4, 0)])
def test_describe_rejects_bad_shapes(args):
    from rmd import _lib
    with pytest.raises(_lib.RmdError):
        _lib.describe(*args)


def test_gpu_path_fails_loudly_without_the_library(monkeypatch):
    """No fallback: with librmd.so missing, the HIP path raises instead of computing anything else."""
    from rmd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/librmd.so")
    with pytest.raises(_lib.RmdError, match="HIP library not found"):
        _lib.lib()


def test_cpu_dispatch_launches_no_hip_kernel(monkeypatch):
    """CPU tensors run the ATen kernels of rmd/cpu.py: the only C-ABI calls they make are the host-only
    geometry helpers (no kernel launcher is ever reached), so the CPU path is a dispatch by device, not
    a stand-in for the HIP path."""
    import torch
    import rmd
    from rmd import _lib
    real = _lib.lib()
    allowed = {"rmd_pyramid_describe_layout", "rmd_pyramid_describe_for", "rmd_last_error"}

    class HostOnly:
        def __getattr__(self, name):
            if name not in allowed:
                raise AssertionError(f"CPU path reached {name}")
            return getattr(real, name)

    monkeypatch.setattr(_lib, "_lib", HostOnly())
    f = torch.randn(1, 8, 8, 12)
    co = torch.rand(1, 2, 8, 12) * 8
    assert rmd.raft.CorrBlock(f, f, 2, 2, method="volume")(co).shape == (1, 50, 8, 12)
    assert rmd.raft_fs.CorrBlock(f, f, 2, 2, method="otf")(co).shape == (1, 50, 8, 12)
    assert rmd.ops.dicl_stack(f, f, co, 2).shape == (1, 5, 5, 16, 8, 12)
    assert rmd.ops.dicl_stack_int(f, f, 1, 1).shape == (1, 3, 3, 16, 8, 12)
