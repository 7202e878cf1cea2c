"""GPU: the multi-tracer batched entry points (fct_ale_pre_comm_batched_acc_,
fct_ale_post_comm_c_batched_acc_, the batched exchanges) against the oracle, one single-tracer
oracle pass per tracer slice (SURVEY.md 8(b) "multi-tracer batched variant", BASELINE config 3).
"""
import ctypes as C

import numpy as np
import pytest

from conftest import assert_cols_equal
from fesom2_amd import abi, engine, partition, synth
from fesom2_amd.abi import arr, dll, ip

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def device():
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    abi.set_path("fused")
    yield


def check_tracer(m, e, k, want):
    L = m.L
    NT = m.N + m.H
    assert_cols_equal(e.tracer("plus", k)[: m.N * L], want["plus"][: m.N * L], m.nlev_nod, L, m.N, f"plus[{k}]")
    assert_cols_equal(e.tracer("minus", k)[: m.N * L], want["minus"][: m.N * L], m.nlev_nod, L, m.N, f"minus[{k}]")
    for name, n in (("adf_v", m.N * m.nl), ("del_v", m.N * L), ("del_h", m.N * L), ("adf_h", m.E * L)):
        got, w = e.tracer(name, k)[:n], want[name][:n]
        bad = np.flatnonzero(got != w)
        assert bad.size == 0, f"{name}[{k}]: {bad.size} differ, first at {bad[:5]}"
    assert NT * L * e.ntr == e.host["plus"].size


@pytest.mark.parametrize("name,ntr", [("tiny", 2), ("8k x 20", 1), ("8k x 20", 3), ("8k x 20", 6),
                                      ("127k x 47", 6)])
@pytest.mark.parametrize("resident", [True, False])
def test_batched_pass_matches_per_tracer_oracle(name, ntr, resident):
    m = synth.config_mesh(name)
    tracers = synth.make_tracer_fields(m, ntr)
    abi.set_resident(resident)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        assert e.full_pass() == 9, abi.last_error()
        e.sync()
        for k in range(ntr):
            check_tracer(m, e, k, O.full_pass(m, tracers[k]))
    finally:
        abi.set_resident(True)
        e.free()
        dm.free()


def test_batched_tracers_differ_and_match_single_entry():
    """Tracer k of a batch equals the single-tracer entry points on tracer k's fields."""
    m = synth.config_mesh("8k x 20")
    tracers = synth.make_tracer_fields(m, 3)
    dm = engine.DeviceMesh(m)
    eb = engine.FctAleBatch(dm, tracers)
    singles = [engine.FctAle(dm, t) for t in tracers]
    try:
        assert eb.full_pass() == 9
        for s in singles:
            assert s.full_pass() == 9
        eb.sync()
        for k, s in enumerate(singles):
            s.sync()
            for name in ("del_v", "del_h", "adf_v", "adf_h"):
                assert np.array_equal(eb.tracer(name, k), s.download(name)), (name, k)
        assert not np.array_equal(eb.tracer("del_h", 0), eb.tracer("del_h", 1))
    finally:
        eb.free()
        for s in singles:
            s.free()
        dm.free()


def test_batched_rejects_short_buffers():
    m = synth.config_mesh("tiny")
    tracers = synth.make_tracer_fields(m, 2)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        e.ntr = 3  # buffers hold 2 tracers
        assert e.pre_comm() == 0
        assert "holds" in abi.last_error() or "bytes" in abi.last_error()
        assert e.post_comm_c() != 9
    finally:
        e.free()
        dm.free()


@pytest.fixture(scope="module")
def comm():
    uid = engine.Halo.unique_id()
    h = abi.Handle("comm")
    st = C.c_int(0)
    dll().fesom2_comm_init_(h.ref, uid, ip(0), ip(1), C.byref(st))
    abi.check(st, "fesom2_comm_init_")
    yield h
    dll().fesom2_comm_free_(h.ref)


def make_plan(send, recv, nl):
    h = abi.Handle("plan")
    st = C.c_int(0)
    dll().fesom2_halo_plan_(h.ref, ip(1), arr(np.zeros(1, np.int32)), arr(np.array([send.size], np.int32)),
                            arr(np.ascontiguousarray(send, np.int32)), arr(np.array([recv.size], np.int32)),
                            arr(np.ascontiguousarray(recv, np.int32)), ip(nl), C.byref(st))
    abi.check(st, "fesom2_halo_plan_")
    return h


@pytest.mark.parametrize("overlap", [False, True])
def test_batched_partitioned_exchange(comm, overlap):
    """Two partitions, 3 tracers: after phase 1 each partition's halo columns get the neighbour's
    values, stored deranged (c_j holds the value of c_{j+1}) for every tracer; a one-rank plan
    sending c_j into c_{j+1} restores them -- through fct_ale_exchange_batched_acc_ then the batched
    phase 2, or the overlapped batched entry.  Owned results equal the global oracle per tracer."""
    nx, ny, nl, ntr = 64, 48, 21, 3
    g = synth.make_mesh(nx, ny, nl)
    gtr = synth.make_tracer_fields(g, ntr)
    wants = [O.full_pass(g, t) for t in gtr]
    part = partition.strip_parts(nx, ny, 2)
    locs = [partition.local_mesh(g, part, r) for r in range(2)]
    runs, plans, outs, pm = [], [], [], []
    L = g.L
    try:
        for m, _ in locs:
            dm = engine.DeviceMesh(m)
            runs.append((dm, engine.FctAleBatch(dm, synth.make_tracer_fields(m, ntr))))
        for _, e in runs:
            assert e.pre_comm() == 6
            e.sync()
            pm.append([e.download("plus").reshape(ntr, -1, L), e.download("minus").reshape(ntr, -1, L)])
        for r, (m, h) in enumerate(locs):
            for q in h.neighbors:
                src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
                for a in range(2):
                    pm[r][a][:, dst] = pm[q][a][:, src]
            cols = np.arange(m.N, m.N + m.H)
            nxt = np.roll(cols, -1)
            for a, name in enumerate(("plus", "minus")):
                stored = pm[r][a].copy()
                stored[:, cols] = pm[r][a][:, nxt]
                runs[r][1].upload(name, stored.reshape(-1))
            plans.append(make_plan(cols + 1, nxt + 1, nl))
        for (_, e), plan in zip(runs, plans):
            if overlap:
                assert e.exchange_post_comm_c(comm, plan) == 9, abi.last_error()
            else:
                e.exchange(comm, plan)
                assert e.post_comm_c() == 9, abi.last_error()
        for _, e in runs:
            e.sync()
            outs.append({k: e.download(k) for k in ("del_v", "del_h", "adf_v")})
    finally:
        for plan in plans:
            dll().fesom2_halo_plan_free_(plan.ref)
        for dm, e in runs:
            e.free()
            dm.free()
    ms = [m for m, _ in locs]
    for k in range(ntr):
        for name, w in (("del_v", L), ("del_h", L), ("adf_v", nl)):
            got = partition.gather_owned(ms, lambda r: outs[r][name].reshape(ntr, -1)[k], w, g.N)
            assert np.array_equal(got, wants[k][name]), (name, k)


@pytest.mark.parametrize("internal", ["0", "1"])
def test_batched_split_by_direction(internal, monkeypatch):
    monkeypatch.setenv("FESOM2_P1V_B3H", internal)  # block-internal edges in p1v (per tracer) or not
    m = synth.config_mesh("8k x 20")
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


@pytest.mark.parametrize("nl", [21, 48])
@pytest.mark.parametrize("internal", ["0", "1"])
def test_split_by_direction_partitioned_overlap(comm, internal, nl, monkeypatch):
    """Two partitions, 2 tracers, the split entries with the exchange inside fct_ale_post_comm_h_acc_
    (deranged halo repaired only by the one-rank exchange, as test_batched_partitioned_exchange);
    with and without the block-internal edges limited in p1v; even and odd L (the interior and
    boundary launches of b3h / c-horizontal in their level-pair forms)."""
    monkeypatch.setenv("FESOM2_P1V_B3H", internal)
    nx, ny, ntr = 64, 48, 2
    g = synth.make_mesh(nx, ny, nl)
    gtr = synth.make_tracer_fields(g, ntr)
    wants = [O.full_pass(g, t) for t in gtr]
    part = np.random.default_rng(9).integers(0, 2, g.N).astype(np.int32)
    locs = [partition.local_mesh(g, part, r) for r in range(2)]
    runs, plans, outs, pm = [], [], [], []
    L = g.L
    try:
        for m, _ in locs:
            dm = engine.DeviceMesh(m)
            runs.append((dm, engine.FctAleBatch(dm, synth.make_tracer_fields(m, ntr))))
        for _, e in runs:
            assert e.pre_comm_v() == 7, abi.last_error()
            e.sync()
            pm.append([e.download("plus").reshape(ntr, -1, L), e.download("minus").reshape(ntr, -1, L)])
        for r, (m, h) in enumerate(locs):
            for q in h.neighbors:
                src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
                for a in range(2):
                    pm[r][a][:, dst] = pm[q][a][:, src]
            cols = np.arange(m.N, m.N + m.H)
            nxt = np.roll(cols, -1)
            for a, name in enumerate(("plus", "minus")):
                stored = pm[r][a].copy()
                stored[:, cols] = pm[r][a][:, nxt]
                runs[r][1].upload(name, stored.reshape(-1))
            plans.append(make_plan(cols + 1, nxt + 1, nl))
        for (_, e), plan in zip(runs, plans):
            assert e.post_comm_h(comm, plan) == 9, abi.last_error()
        for _, e in runs:
            e.sync()
            outs.append({k: e.download(k) for k in ("del_v", "del_h", "adf_v")})
    finally:
        for plan in plans:
            dll().fesom2_halo_plan_free_(plan.ref)
        for dm, e in runs:
            e.free()
            dm.free()
    ms = [m for m, _ in locs]
    for k in range(ntr):
        for name, w in (("del_v", L), ("del_h", L), ("adf_v", nl)):
            got = partition.gather_owned(ms, lambda r: outs[r][name].reshape(ntr, -1)[k], w, g.N)
            assert np.array_equal(got, wants[k][name]), (name, k)


@pytest.mark.parametrize("shape", [{}, {"FESOM2_BATCH_GROUP_SHIFT": "0"},
                                   {"FESOM2_BATCH_GROUP_SHIFT": "-2", "FESOM2_BATCH_PATCH": "64"},
                                   {"FESOM2_BATCH_PATCH": "1"}, {"FESOM2_BATCH_GROUP": "6"},
                                   {"FESOM2_BATCH_GROUP": "5", "FESOM2_BATCH_PATCH": "300"},
                                   {"FESOM2_CACHE_ORDER": "1"}],
                         ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()) or "default")
@pytest.mark.parametrize("name,full", [("8k x 20", False), ("127k x 47", True)])
@pytest.mark.parametrize("internal", ["0", "1"])
def test_batched_plan_shapes(shape, name, full, internal, monkeypatch):
    """Batched calls run on a plan of their own (smaller patches, half-size blocks where they keep the
    lanes busy: the plan options FESOM2_BATCH_PATCH / FESOM2_BATCH_GROUP_SHIFT); the single-tracer
    plan is unchanged.
    Every shape is exact on every tracer, with and without the block-internal edges in p1v (whose
    lists follow the batched plan's block size)."""
    for k, v in dict(shape, FESOM2_P1V_B3H=internal).items():
        monkeypatch.setenv(k, v)
    m = synth.config_mesh(name, full_depth=full)
    tracers = synth.make_tracer_fields(m, 3)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        one, many = dm.info(), dm.info(batched=True)
        if internal == "1" and many["p1v_columns"]:  # (0: some block has too many internal edges)
            # default on these small partitions: the single plan's blocks (smaller ones only from 32M
            # wet cells, test_batched_plan_of_a_large_partition); FESOM2_BATCH_GROUP: exactly that many
            shift = int(shape.get("FESOM2_BATCH_GROUP_SHIFT", "0"))
            want = int(shape["FESOM2_BATCH_GROUP"]) if "FESOM2_BATCH_GROUP" in shape else \
                one["p1v_columns"] // 2 ** -shift
            assert many["p1v_columns"] == want, (one, many)
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        for k in range(3):
            check_tracer(m, e, k, O.full_pass(m, tracers[k]))
        # the fused batched pair on the same plan
        for name_ in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
            e.upload(name_)
        assert e.full_pass() == 9, abi.last_error()
        e.sync()
        for k in range(3):
            check_tracer(m, e, k, O.full_pass(m, tracers[k]))
    finally:
        e.free()
        dm.free()


def test_batched_plan_of_a_large_partition():
    """From 32M owned wet cells both plans take the largest column count below the natural one that
    keeps >= 90 % of a block's lanes busy: 1.2M x 80 (40 slots per column, 8 columns natural) -> 6
    columns (240 of 256 lanes), in row pairs (3 over 3); the batched plan with 4096-node patches,
    the single-tracer one with 16384."""
    m = synth.config_mesh("1.2M x 80", full_depth=True)
    dm = engine.DeviceMesh(m)
    try:
        one, many = dm.info(), dm.info(batched=True)
        assert one["p1v_columns"] == 6
        assert many["p1v_columns"] == 6
        # row-pair blocks (3 nodes of a patch row over the 3 below them): about half the interior
        # edges are block-internal (a single row of 8 columns: 29 %)
        assert one["internal_edges"] / one["interior_edges"] > 0.45
        assert many["internal_edges"] / many["interior_edges"] > 0.45
    finally:
        dm.free()


@pytest.mark.parametrize("ntr", [1, 3])
@pytest.mark.parametrize("mesh", ["odd L", "variable depth", "delaunay hilbert", "permuted"])
def test_large_partition_plan_on_small_meshes(mesh, ntr, monkeypatch):
    """The product's large-partition plan (6-column blocks in row pairs, the internal edges' raw
    flux stashed in LDS, the block-internal edges limited inside p1v) on meshes the 1.2M x 80 runs
    never reach: odd L (the k_p1<..., 52 | 256, true> form), variable depth, an unstructured
    Delaunay mesh with Hilbert numbering and a scattered numbering.  FESOM2_LARGE_CELLS=0 moves the
    32M-cell threshold so small meshes take that plan; split and fused pairs exact."""
    monkeypatch.setenv("FESOM2_LARGE_CELLS", "0")
    if mesh == "odd L":
        m = synth.make_mesh(64, 40, 48, full_depth=True)
    elif mesh == "variable depth":
        m = synth.make_mesh(64, 40, 81)
    elif mesh == "delaunay hilbert":
        m = synth.delaunay_mesh(3000, 48, numbering="hilbert")
    else:
        m = synth.permute_mesh(synth.make_mesh(64, 40, 48))
    tracers = synth.make_tracer_fields(m, ntr)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers) if ntr > 1 else engine.FctAle(dm, tracers[0])
    try:
        info = dm.info(batched=ntr > 1)
        assert info["internal_edges"] > 0, info
        # the largest column count below the natural one with >= 90 % of the lanes busy: 47 levels
        # (24 slots, 8 columns natural) -> 5, 80 levels (40 slots, 8 natural) -> 6
        assert info["p1v_columns"] == {47: 5, 80: 6}[m.L], info
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        wants = [O.full_pass(m, t) for t in tracers]
        got = {k: e.download(k).reshape(ntr, -1) for k in ("plus", "minus", "del_v", "del_h", "adf_v", "adf_h")}
        for k in range(ntr):
            assert_cols_equal(got["plus"][k][: m.N * m.L], wants[k]["plus"][: m.N * m.L], m.nlev_nod, m.L, m.N,
                              f"plus[{k}]")
            for name, n in (("adf_v", m.N * m.nl), ("del_v", m.N * m.L), ("del_h", m.N * m.L), ("adf_h", m.E * m.L)):
                bad = np.flatnonzero(got[name][k][:n] != wants[k][name][:n])
                assert bad.size == 0, f"{mesh} {name}[{k}]: {bad.size} differ, first at {bad[:5]}"
    finally:
        e.free()
        dm.free()


def test_batched_graph_after_prepare_only():
    """A batched pass captured right after fesom2_prepare_mesh_ (no eager call first): prepare builds
    the batched plans too (or shares the single-tracer one where the shapes resolve alike), so the
    capture builds nothing."""
    m = synth.config_mesh("8k x 20")
    tracers = synth.make_tracer_fields(m, 3)
    dm = engine.DeviceMesh(m)
    dm.prepare()
    e = engine.FctAleBatch(dm, tracers)
    graph = None
    try:
        with abi.Graph.capture(e.stream) as graph:
            assert e.pre_comm_v() == 7, abi.last_error()
            assert e.post_comm_h() == 9, abi.last_error()
        graph.launch(e.stream)
        e.sync()
        for k in range(3):
            check_tracer(m, e, k, O.full_pass(m, tracers[k]))
        # the same with the fused batched pair
        for name in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
            e.upload(name)
        graph.free()
        with abi.Graph.capture(e.stream) as graph:
            assert e.full_pass() == 9, abi.last_error()
        graph.launch(e.stream)
        e.sync()
        for k in range(3):
            check_tracer(m, e, k, O.full_pass(m, tracers[k]))
    finally:
        if graph is not None:
            graph.free()
        e.free()
        dm.free()


@pytest.mark.parametrize("env,expect", [(None, {1: 13, 2: 0, 6: 0}), ("0", {1: 0, 2: 0, 6: 0}),
                                        ("1", {1: 13, 2: 13, 6: 13})])
def test_pass_order_rule(env, expect, monkeypatch):
    """fesom2_pass_order_ reports the Infinity-Cache pass order the entries use: on 127k x 47 (one
    tracer's fct_adf_h 143 MB <= 192 MiB) for one tracer, off for two (286 MB) and six; the plan
    option FESOM2_CACHE_ORDER forces it either way.  8k x 20 keeps it for six tracers (23 MB)."""
    if env is not None:
        monkeypatch.setenv("FESOM2_CACHE_ORDER", env)
    else:
        monkeypatch.delenv("FESOM2_CACHE_ORDER", raising=False)
    m = synth.config_mesh("127k x 47", full_depth=True)
    dm = engine.DeviceMesh(m)
    try:
        assert {t: dm.pass_order(t) for t in expect} == expect
    finally:
        dm.free()
    if env is None:
        small = engine.DeviceMesh(synth.config_mesh("8k x 20"))
        try:
            assert small.pass_order(6) == 13
        finally:
            small.free()
