import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raft-meets-dicl_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C-ABI")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture
def golden():
    return load_golden


def rel_max_err(got, ref):
    """max|got - ref| / max|ref| over finite reference entries (the tolerance metric used throughout)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    fin = np.isfinite(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    if not fin.any():
        return 0.0
    scale = np.abs(ref[fin]).max()
    return float(np.abs(got[fin] - ref[fin]).max() / max(scale, 1e-30))


def assert_close_elementwise(got, ref, rtol, atol):
    """Elementwise |got - ref| <= atol + rtol * |ref| (NaN patterns must match); reports the worst entry."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    fin = np.isfinite(ref)
    err = np.abs(got[fin] - ref[fin])
    lim = atol + rtol * np.abs(ref[fin])
    if err.size and not (err <= lim).all():
        k = int(np.argmax(err - lim))
        raise AssertionError(f"elementwise tolerance exceeded at flat {k}: got {got[fin][k]!r} ref {ref[fin][k]!r} "
                             f"err {err[k]:.3e} > {lim[k]:.3e} ({int((err > lim).sum())} of {err.size} entries)")


def assert_fp32_gate(got, ref):
    """north_star's fp32 cost-volume gate applied per element: |got - ref| <= 1e-4 |ref| + 1e-5 max|ref|
    (max over the finite reference entries; NaN patterns must match)."""
    ref = np.asarray(ref, dtype=np.float64)
    fin = np.isfinite(ref)
    scale = float(np.abs(ref[fin]).max()) if fin.any() else 0.0
    assert_close_elementwise(got, ref, rtol=1e-4, atol=1e-5 * scale)
