"""GPU, tuning build only: every measured-and-rejected kernel variant is exact too.

The product library (lib/libfesom2-accelerate.so) compiles every FESOM2_* A/B knob to its measured
default and ships none of the variants (DESIGN.md §3 records why each lost).  They live in the
tuning build (``make -C fesom2-accelerate_amd tuning``), which tools/sweep_env.sh measures; this file
runs only against it::

    FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so python -m pytest tests/test_gpu_tuning.py -m gpu

and is skipped otherwise.
"""
import os

import pytest

from fesom2_amd import abi, engine, synth
from test_gpu_parity import check_pass, mesh, run_pass, run_split

import oracle as O

TUNING_LIB = "libfesom2-accelerate-tuning.so"
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("FESOM2_LIB_NAME") != TUNING_LIB,
                                 reason="the variants exist in the tuning build only (FESOM2_LIB_NAME)")]


@pytest.fixture(scope="module", autouse=True)
def device():
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    abi.set_path("fused")
    yield


KNOBS = [{"FESOM2_B3H_U": "1", "FESOM2_B3H_NT": "0"}, {"FESOM2_B3H_U": "4", "FESOM2_B3H_NT": "0"},
         {"FESOM2_B3H_U": "1", "FESOM2_B3H_NT": "1"}, {"FESOM2_B3H_CPT": "4"}, {"FESOM2_NT": "3"},
         {"FESOM2_P1_BATCH": "44", "FESOM2_P2_BATCH": "8"}, {"FESOM2_PATCH": "0"}, {"FESOM2_PATCH": "7"}, {"FESOM2_FUSE_B3H": "1"},
         {"FESOM2_FUSE_B3H": "1", "FESOM2_P2F_BATCH": "1"}, {"FESOM2_FUSE_B3H": "1", "FESOM2_P2F_BATCH": "4"},
         {"FESOM2_P1_STAGE": "1", "FESOM2_P1_EDGE": "0"},
         {"FESOM2_P1_STAGE": "1", "FESOM2_P1_EDGE": "0", "FESOM2_P1S_EB": "4"}, {"FESOM2_P1_EDGE": "0"},
         {"FESOM2_P1E_EB": "1"}, {"FESOM2_P1E_EB": "4"}, {"FESOM2_NT": "0"}, {"FESOM2_P2_CPT": "1"},
         {"FESOM2_P2_CPT": "1", "FESOM2_NT": "0"}, {"FESOM2_P2_CHUNK": "1000"},
         {"FESOM2_P2_CHUNK": "37", "FESOM2_B3H_NT": "0"}, {"FESOM2_P2_WF": "1"},
         {"FESOM2_P2_CHUNK": "1000", "FESOM2_P2_MERGE": "1"}, {"FESOM2_P2_CHUNK": "333", "FESOM2_P2_MERGE": "1"}]


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


SPLIT_KNOBS = [{"FESOM2_P1V_EARLY": "1"}, {"FESOM2_P1V_EARLY": "2"}, {"FESOM2_P1V_EARLY": "8"},
               {"FESOM2_ODD_PAIR": "0"}, {"FESOM2_NL_PAIR": "0"}, {"FESOM2_NL_PAIR": "0", "FESOM2_NT": "0"},
               {"FESOM2_PATCH_ORDER": "1"}, {"FESOM2_PATCH_ORDER": "1", "FESOM2_PATCH": "100"},
               {"FESOM2_PATCH_ORDER": "0", "FESOM2_PATCH": "64"}, {"FESOM2_B3H_NODE": "1"},
               {"FESOM2_B3H_NODE": "1", "FESOM2_B3HN_EB": "1"}, {"FESOM2_B3H_NODE": "1", "FESOM2_B3HN_EB": "3"},
               {"FESOM2_B3H_NODE": "1", "FESOM2_ODD_PAIR": "0"}, {"FESOM2_B3H_PACK": "0"},
               {"FESOM2_B3H_PACK": "1", "FESOM2_B3H_NT": "0"},
               {"FESOM2_B3HP_H": "1"}, {"FESOM2_B3HP_H": "4"}, {"FESOM2_B3HP_CAP": "100"},
               {"FESOM2_P2H_FUSE": "1"}, {"FESOM2_P2H_FUSE": "1", "FESOM2_P2HF_KB": "1"},
               {"FESOM2_P2H_FUSE": "1", "FESOM2_P2HF_KB": "4"}, {"FESOM2_P2H_FUSE": "1", "FESOM2_NT": "0"},
               {"FESOM2_P2H_FUSE": "1", "FESOM2_ODD_PAIR": "0"}, {"FESOM2_P1V_B3H": "0"},
               {"FESOM2_P1V_B3H": "1", "FESOM2_SUBPATCH": "8"}, {"FESOM2_P1V_B3H": "1", "FESOM2_NL_PAIR": "0"},
               {"FESOM2_P1V_B3H": "1", "FESOM2_CPT": "1"}, {"FESOM2_P1V_B3H": "1", "FESOM2_B3H_PACK": "0"},
               {"FESOM2_NT": "2"}, {"FESOM2_NT": "2", "FESOM2_P1V_B3H": "1"}, {"FESOM2_NT": "6", "FESOM2_P1V_B3H": "0"},
               {"FESOM2_BLOB": "1"}, {"FESOM2_BLOB": "1", "FESOM2_PATCH_ORDER": "1"}, {"FESOM2_BLOB": "0"},
               {"FESOM2_P1V_B3H": "1", "FESOM2_P1V_INT_DMA": "0"}, {"FESOM2_P1V_B3H": "1", "FESOM2_B3HP_REG": "0"},
               # round 3
               {"FESOM2_P1V_BATCH": "23"}, {"FESOM2_P1V_BATCH": "32"}, {"FESOM2_P1V_BATCH": "33", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_P1V_BATCH": "62"}, {"FESOM2_P1V_BATCH": "26", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_P1V_PERSIST": "1"}, {"FESOM2_P1V_PERSIST": "1", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_P1V_PERSIST": "2", "FESOM2_P1V_B3H": "1"}, {"FESOM2_TILE_REV": "7"},
               {"FESOM2_TILE_REV": "6", "FESOM2_P1V_B3H": "1"}, {"FESOM2_P1V_WAVES": "8"},
               {"FESOM2_P1V_DMA": "1"}, {"FESOM2_P1V_DMA": "2", "FESOM2_P1V_B3H": "1"},
               {"FESOM2_P2H_BATCH": "6"}, {"FESOM2_P2H_BATCH": "8"}]


@pytest.mark.parametrize("knobs", SPLIT_KNOBS, ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()))
@pytest.mark.parametrize("name,perm", [("8k x 20", False), ("8k x 20", True), ("127k x 47", False)])
def test_split_variants_match_oracle(knobs, name, perm, monkeypatch):
    """The direction-split kernels' switches (p1v load placement, LDS-DMA tail, odd-L pairs,
    16-byte stride-nl loads, processing orders, b3h forms, b3h folded into p2h) are all exact."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    m, f = mesh(name, False, perm)
    check_pass(m, run_split(m, f), O.full_pass(m, f))


@pytest.mark.parametrize("nl", [3, 4, 5, 48, 81, 129])
@pytest.mark.parametrize("full", [False, True])
def test_p2h_fuse_level_counts_and_repeats(nl, full, monkeypatch):
    """FESOM2_P2H_FUSE=1 (b3h folded into c-horizontal with per-edge arrival counters, zeroed at every
    pass): three passes on the same plan, inputs re-uploaded before each, every one exact."""
    monkeypatch.setenv("FESOM2_P2H_FUSE", "1")
    m = synth.make_mesh(40, 14, nl, full_depth=full)
    f = synth.make_fields(m)
    want = O.full_pass(m, f)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        for _ in range(3):
            for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
                e.upload(k)
            assert e.pre_comm_v() == 7, abi.last_error()
            assert e.post_comm_h() == 9, abi.last_error()
            e.sync()
            check_pass(m, {k: e.download(k) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")}, want)
    finally:
        e.free()
        dm.free()


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


@pytest.mark.parametrize("chunk", ["1", "3", "256"])
@pytest.mark.parametrize("name", ["8k x 20", "127k x 47"])
def test_tracer_chunks_match_oracle(chunk, name, monkeypatch):
    """FESOM2_TRACER_CHUNK: batched p1v in XCD-chunked tracer tiles (padding tiles past the last group
    exit before any barrier); every tracer equals its own oracle pass."""
    monkeypatch.setenv("FESOM2_TRACER_CHUNK", chunk)
    m, _ = mesh(name)
    tracers = synth.make_tracer_fields(m, 3)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        assert e.split_pass() == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k).reshape(3, -1) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")}
    finally:
        e.free()
        dm.free()
    for t in range(3):
        check_pass(m, {k: v[t] for k, v in got.items()}, O.full_pass(m, tracers[t]))
