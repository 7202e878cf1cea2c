"""GPU parity on unstructured meshes: Delaunay triangulations of random points.

The structured synthetic mesh has degree 6 everywhere; a FESOM mesh does not.  Here node degrees run
3..13, so clusters and edge lists overflow the 8 entries a NodeRec holds inline (the kernels' CSR
fallback), the numbering is scattered (the plan picks the Cuthill-McKee patch order), boundaries
exist (edges with one element), and element levels vary.  Every kernel path must still equal the
oracle cell for cell; the oracle itself is pinned to reference.cpp on these meshes in
test_oracle.py.
"""
import pytest

from fesom2_amd import abi, engine, synth
from test_gpu_batched import check_tracer
from test_gpu_parity import check_pass, run_pass, run_split

import oracle as O

pytestmark = pytest.mark.gpu

_CACHE = {}


def mesh(npts, nl, full, numbering="scipy"):
    key = (npts, nl, full, numbering)
    if key not in _CACHE:
        m = synth.delaunay_mesh(npts, nl, full_depth=full, numbering=numbering)
        _CACHE[key] = (m, synth.make_fields(m))
    return _CACHE[key]


@pytest.fixture(scope="module", autouse=True)
def device():
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    abi.set_path("fused")
    yield
    abi.set_path("fused")


MESHES = [(3000, 21, False), (20000, 48, False), (20000, 81, True), (500, 4, False)]


@pytest.mark.parametrize("npts,nl,full,numbering", [k + ("scipy",) for k in MESHES] +
                         [(30000, 48, False, "hilbert"), (20000, 81, True, "hilbert")])
@pytest.mark.parametrize("mode", ["split", "split_internal", "fused", "sequence", "stepwise"])
def test_unstructured_paths_match_oracle(npts, nl, full, numbering, mode, monkeypatch):
    """numbering "hilbert": the plan takes the sorted-patch order (locality detected), "scipy": the
    Cuthill-McKee patches."""
    m, f = mesh(npts, nl, full, numbering)
    assert m.dim > 8  # some clusters overflow the inline NodeRec entries
    monkeypatch.setenv("FESOM2_P1V_B3H", "1" if mode == "split_internal" else "0")
    if mode.startswith("split"):
        got = run_split(m, f)
    else:
        st, got = run_pass(m, f, fused=mode == "fused", path="stepwise" if mode == "stepwise" else "fused")
        assert st == 9
    check_pass(m, got, O.full_pass(m, f))


@pytest.mark.parametrize("npts,nl,full", MESHES)
def test_unstructured_packed_b3h(npts, nl, full, monkeypatch):
    """b3h packed by depth (FESOM2_B3H_PACK=1) on variable-depth unstructured meshes."""
    monkeypatch.setenv("FESOM2_B3H_PACK", "1")
    m, f = mesh(npts, nl, full)
    check_pass(m, run_split(m, f), O.full_pass(m, f))


@pytest.mark.parametrize("npts,nl,full", MESHES[:2])
def test_unstructured_batched_split(npts, nl, full):
    m, _ = mesh(npts, nl, full)
    tracers = synth.make_tracer_fields(m, 3)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        for k in range(3):
            check_tracer(m, e, k, O.full_pass(m, tracers[k]))
    finally:
        e.free()
        dm.free()
