"""GPU, tuning build only: every A/B knob of the tuning build is exact too.

The product library (lib/libfesom2-accelerate.so) compiles every FESOM2_* A/B knob to its measured
default.  The tuning build (``make -C fesom2-accelerate_amd tuning``, built on demand, not by
``build()``) reads them from the environment for tools/sweep_env.sh; this file runs only against it::

    FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so python -m pytest tests/test_gpu_tuning.py -m gpu

and is not collected otherwise (tests/conftest.py), so product runs show no skips for it.  The
variants that lost their A/B by 5 % or more (persistent p1v, tracer loop, LDS-DMA gathers, early
loads, b3h folded into phase 2, persistent phase 2, node-centric b3h, edge/staged phase 1, chunked
phase 2) were deleted in round 4; DESIGN.md §3 keeps their measurements.
"""
import os

import pytest

from fesom2_amd import abi
from test_gpu_parity import check_pass, mesh, run_pass, run_split

import oracle as O

TUNING_LIB = "libfesom2-accelerate-tuning.so"
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("FESOM2_LIB_NAME") != TUNING_LIB,
                                 reason="the knobs exist in the tuning build only (FESOM2_LIB_NAME)")]


@pytest.fixture(scope="module", autouse=True)
def device():
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    abi.set_path("fused")
    yield


KNOBS = [{"FESOM2_B3H_U": "1", "FESOM2_B3H_NT": "0"}, {"FESOM2_B3H_U": "4", "FESOM2_B3H_NT": "0"},
         {"FESOM2_B3H_U": "1", "FESOM2_B3H_NT": "1"}, {"FESOM2_B3H_CPT": "4"}, {"FESOM2_NT": "3"},
         {"FESOM2_P1_BATCH": "44", "FESOM2_P2_BATCH": "8"}, {"FESOM2_PATCH": "0"}, {"FESOM2_PATCH": "7"},
         {"FESOM2_NT": "0"}, {"FESOM2_P2_CPT": "1"}, {"FESOM2_P2_CPT": "1", "FESOM2_NT": "0"},
         {"FESOM2_GROUP_SHIFT": "-1"}, {"FESOM2_XCD": "0"}]


@pytest.mark.parametrize("knobs", KNOBS, ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()))
@pytest.mark.parametrize("name", ["8k x 20", "127k x 47"])
def test_kernel_variants_match_oracle(knobs, name, monkeypatch):
    """Every tuning variant the launchers can select (env knobs read at launch) is exact too."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    m, f = mesh(name)
    st, got = run_pass(m, f)
    assert st == 9
    check_pass(m, got, O.full_pass(m, f))


SPLIT_KNOBS = [{"FESOM2_ODD_PAIR": "0"}, {"FESOM2_NL_PAIR": "0"}, {"FESOM2_NL_PAIR": "0", "FESOM2_NT": "0"},
               {"FESOM2_PATCH_ORDER": "1"}, {"FESOM2_PATCH_ORDER": "1", "FESOM2_PATCH": "100"},
               {"FESOM2_PATCH_ORDER": "0", "FESOM2_PATCH": "64"}, {"FESOM2_B3H_PACK": "0"},
               {"FESOM2_B3H_PACK": "1", "FESOM2_B3H_NT": "0"},
               {"FESOM2_B3HP_H": "1"}, {"FESOM2_B3HP_H": "4"}, {"FESOM2_B3HP_CAP": "100"},
               {"FESOM2_P1V_B3H": "0"}, {"FESOM2_P1V_B3H": "1", "FESOM2_NL_PAIR": "0"},
               {"FESOM2_P1V_B3H": "1", "FESOM2_CPT": "1"}, {"FESOM2_P1V_B3H": "1", "FESOM2_B3H_PACK": "0"},
               {"FESOM2_NT": "2"}, {"FESOM2_NT": "2", "FESOM2_P1V_B3H": "1"}, {"FESOM2_NT": "6", "FESOM2_P1V_B3H": "0"},
               {"FESOM2_P1V_B3H": "1", "FESOM2_P1V_INT_DMA": "0"}, {"FESOM2_P1V_B3H": "1", "FESOM2_B3HP_REG": "0"},
               # round 3
               {"FESOM2_P1V_BATCH": "23"}, {"FESOM2_P1V_BATCH": "32"}, {"FESOM2_P1V_BATCH": "33", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_P1V_BATCH": "62"}, {"FESOM2_P1V_BATCH": "26", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_TILE_REV": "7"},
               {"FESOM2_TILE_REV": "6", "FESOM2_P1V_B3H": "1"}, {"FESOM2_P1V_WAVES": "8"},
               {"FESOM2_P2H_BATCH": "6"}, {"FESOM2_P2H_BATCH": "8"},
               {"FESOM2_B3H_STPLAIN": "1"}, {"FESOM2_B3H_STPLAIN": "1", "FESOM2_P1V_B3H": "1", "FESOM2_TILE_REV": "5"},
               {"FESOM2_ROWPAIR": "1"}, {"FESOM2_ROWPAIR": "1", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_ROWPAIR": "1", "FESOM2_P1V_B3H": "1", "FESOM2_PATCH": "100"},
               {"FESOM2_P1V_STASH": "1", "FESOM2_P1V_B3H": "1"}, {"FESOM2_P1V_STASH": "2", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_P1V_STASH": "1", "FESOM2_P1V_B3H": "1", "FESOM2_ROWPAIR": "1"},
               {"FESOM2_P1V_STASH": "1", "FESOM2_P1V_B3H": "1", "FESOM2_PATCH": "100"},
               {"FESOM2_ROWPAIR": "3", "FESOM2_P1V_STASH": "1", "FESOM2_P1V_B3H": "1"}]


@pytest.mark.parametrize("knobs", SPLIT_KNOBS, ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()))
@pytest.mark.parametrize("name,perm", [("8k x 20", False), ("8k x 20", True), ("127k x 47", False)])
def test_split_variants_match_oracle(knobs, name, perm, monkeypatch):
    """The direction-split kernels' switches (odd-L pairs, 16-byte stride-nl loads, processing
    orders, b3h forms, gather batches, wave counts, tile orders) are all exact."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    m, f = mesh(name, False, perm)
    check_pass(m, run_split(m, f), O.full_pass(m, f))


@pytest.mark.parametrize("knobs", [{"FESOM2_C_BATCH": "2"}, {"FESOM2_P2_BATCH": "2"}],
                         ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()))
@pytest.mark.parametrize("name", ["8k x 20", "127k x 47"])
def test_reference_sequence_variants_match_oracle(knobs, name, monkeypatch):
    """Round-3 node-kernel batches: the reference sequence's c-step (k_c) and the fused phase 2."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    m, f = mesh(name)
    for fused in (True, False):
        st, got = run_pass(m, f, fused=fused)
        assert st == 9
        check_pass(m, got, O.full_pass(m, f))


@pytest.mark.parametrize("strip", ["6", "12", "18", "24"])
@pytest.mark.parametrize("large", [True, False])
@pytest.mark.parametrize("name,nl", [("structured", 21), ("structured", 48), ("permuted", 21)])
def test_batched_strip_orders_match_oracle(strip, large, name, nl, monkeypatch):
    """Round 5: strips inside the batched plan's patches (FESOM2_BATCH_STRIP, strip_order), with the
    large-partition rules (row pairs, stash, internal edges; FESOM2_LARGE_CELLS=0) and without; a
    scattered numbering (no rows: strip_order leaves the patch alone).  3 tracers, split pass."""
    from fesom2_amd import engine, synth
    monkeypatch.setenv("FESOM2_BATCH_STRIP", strip)
    if large:
        monkeypatch.setenv("FESOM2_LARGE_CELLS", "0")
    g = synth.make_mesh(96, 40, nl, full_depth=nl == 48)
    m = synth.permute_mesh(g) if name == "permuted" else g
    tracers = synth.make_tracer_fields(m, 3)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k).reshape(3, -1) for k in ("del_v", "del_h", "adf_v", "adf_h")}
        for k in range(3):
            want = O.full_pass(m, tracers[k])
            for name_, n in (("adf_v", m.N * m.nl), ("del_v", m.N * m.L), ("del_h", m.N * m.L), ("adf_h", m.E * m.L)):
                assert (got[name_][k][:n] == want[name_][:n]).all(), (name_, k)
    finally:
        e.free()
        dm.free()


@pytest.mark.parametrize("mode,cap", [("1", ""), ("2", ""), ("2", "1"), ("2", "12")])
@pytest.mark.parametrize("ntr", [1, 3])
@pytest.mark.parametrize("large", [True, False])
@pytest.mark.parametrize("name,nl", [("structured", 21), ("structured", 48), ("permuted", 21),
                                     ("delaunay", 21), ("delaunay", 48)])
def test_cluster_union_staging_matches_oracle(mode, cap, ntr, large, name, nl, monkeypatch):
    """Round 6: p1v with each block's cluster union staged into LDS by DMA
    (FESOM2_P1V_UNION, MeshPlanDev::cu_ptr) -- the cluster bound read from the union's slots -- with
    and without the large-partition rules (row pairs, stash, internal edges), odd and even L, variable
    depth, a scattered numbering and Delaunay meshes (degrees 3..13: ring slices past the inline 8),
    1 and 3 tracers; mode 2 puts the union's images in tvert's LDS region; a cap on the union's size
    (FESOM2_P1V_UNION_MAX; 1: the block's own columns only) leaves the rest to memory gathers; every
    output exact."""
    from fesom2_amd import engine, synth
    monkeypatch.setenv("FESOM2_P1V_UNION", mode)
    if cap:
        monkeypatch.setenv("FESOM2_P1V_UNION_MAX", cap)
    if large:
        monkeypatch.setenv("FESOM2_LARGE_CELLS", "0")
    if name == "delaunay":
        m = synth.delaunay_mesh(3000, nl, full_depth=nl == 48)
    else:
        g = synth.make_mesh(96, 40, nl, full_depth=nl == 48)
        m = synth.permute_mesh(g) if name == "permuted" else g
    tracers = synth.make_tracer_fields(m, ntr)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers) if ntr > 1 else engine.FctAle(dm, tracers[0])
    try:
        dm.prepare()
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        keys = ("plus", "minus", "del_v", "del_h", "adf_v", "adf_h")
        got = {k: e.download(k).reshape(ntr, -1) for k in keys}
        for k in range(ntr):
            check_pass(m, {n: got[n][k] for n in keys}, O.full_pass(m, tracers[k]))
    finally:
        e.free()
        dm.free()


@pytest.mark.parametrize("group", ["2", "3"])
@pytest.mark.parametrize("large", [True, False])
@pytest.mark.parametrize("nl", [21, 48])
def test_tracer_group_tile_order_matches_oracle(group, large, nl, monkeypatch):
    """Round 6: batched tiles in groups of g tracers (FESOM2_TRACER_GROUP: every
    column group of tracers 0..g-1, then the next g) for the tracer-fastest kernels; 6 tracers, with
    and without the large-partition rules, split pass, every output exact."""
    from fesom2_amd import engine, synth
    monkeypatch.setenv("FESOM2_TRACER_GROUP", group)
    if large:
        monkeypatch.setenv("FESOM2_LARGE_CELLS", "0")
    m = synth.make_mesh(96, 40, nl, full_depth=nl == 48)
    tracers = synth.make_tracer_fields(m, 6)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        keys = ("plus", "minus", "del_v", "del_h", "adf_v", "adf_h")
        got = {k: e.download(k).reshape(6, -1) for k in keys}
        for k in range(6):
            check_pass(m, {n: got[n][k] for n in keys}, O.full_pass(m, tracers[k]))
    finally:
        e.free()
        dm.free()
