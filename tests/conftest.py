"""Shared test setup: import paths, the ``gpu`` marker, and small helpers.

CPU tests (``-m "not gpu"``) cover the oracle against the reference and the golden fixtures, the
host logic (synthetic mesh, partition, halo lists, gloo multi-rank) and that the C-ABI library
loads and exports every symbol include/fesom2-accelerate.h declares.  GPU tests (``-m gpu``) are the
parity tests proper: they drive the HIP engine through the C-ABI and compare with the oracle.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "fesom2-accelerate_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


# The tuning build's knob tests (tests/test_gpu_tuning.py) run only when FESOM2_LIB_NAME selects that
# library; otherwise they are not collected at all, so product runs report no skips for them.
collect_ignore = [] if os.environ.get("FESOM2_LIB_NAME") == "libfesom2-accelerate-tuning.so" else \
    ["test_gpu_tuning.py"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running (full-size meshes)")


def wet_mask(nlev, L):
    """(ncols, L) mask of the levels z < nlev-1 a column owns."""
    return np.arange(L)[None, :] < (np.asarray(nlev)[:, None] - 1)


def assert_cols_equal(got, want, nlev, L, ncols, what, atol=0.0):
    """Compare the wet part of the first ``ncols`` columns of two (L, cols) fields."""
    g = np.asarray(got)[: ncols * L].reshape(ncols, L)
    w = np.asarray(want)[: ncols * L].reshape(ncols, L)
    mask = wet_mask(nlev[:ncols], L)
    if atol == 0.0:
        bad = np.argwhere(mask & ~(g == w))
        assert bad.size == 0, f"{what}: {len(bad)} cells differ, first {bad[:5].tolist()}: " \
                              f"got {g[tuple(bad[0])]!r} want {w[tuple(bad[0])]!r}"
    else:
        err = np.max(np.abs(np.where(mask, g - w, 0.0))) if mask.any() else 0.0
        assert err <= atol, f"{what}: max abs err {err} > {atol}"
