"""GPU: every BASELINE.json GPU configuration on the production path, exact against the oracle.

The benchmark times the direction-split pass (fct_ale_pre_comm_v_acc_ -> fct_ale_post_comm_h_acc_)
with the plan's automatic settings; these tests run exactly that, with no environment forcing, at
the configurations BASELINE.json names:

* config 1  127k x 47, 1 tracer, partitioned over 4 strips with the caller's halo exchange
            (FESOM2's own per-rank regime);
* config 2  1.2M x 80 full depth, 1 tracer (the bench default: block-internal edges limited inside
            p1v, 16384-node sorted patches, regular b3h packing -- all chosen by the plan);
* config 3  1.2M x 80, 6 tracers through the batched split entries;
* config 4  a 3-strip slice of the weak-scaling 9.6M x 80 geometry (1600 x 750 nodes = 1.2M per
            strip, the middle strip with two neighbours), phase 1 per strip, halo exchange, phase 2.

The oracle passes run in threads (the oracle's C calls release the GIL), one per tracer or strip.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import assert_cols_equal
from fesom2_amd import abi, engine, partition, synth

import oracle as O

pytestmark = pytest.mark.gpu

FIELDS = ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")


@pytest.fixture(scope="module", autouse=True)
def device():
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    abi.set_path("fused")
    yield


def pmap(fn, items):
    with ThreadPoolExecutor(max_workers=max(1, min(8, len(items)))) as ex:
        return list(ex.map(fn, items))


def check_owned(m, got, want, what):
    """plus/minus on the owned wet cells; fct_adf_v, del_v, del_h on the owned columns; fct_adf_h on
    every local edge."""
    L = m.L
    assert_cols_equal(got["plus"], want["plus"], m.nlev_nod, L, m.N, f"{what} plus")
    assert_cols_equal(got["minus"], want["minus"], m.nlev_nod, L, m.N, f"{what} minus")
    for k, n in (("adf_v", m.N * m.nl), ("del_v", m.N * L), ("del_h", m.N * L), ("adf_h", m.E * L)):
        g, w = got[k][:n], want[k][:n]
        bad = np.flatnonzero(g != w)
        assert bad.size == 0, f"{what} {k}: {bad.size} differ, first at {bad[:5]}: {g[bad[0]]!r} vs {w[bad[0]]!r}"


def test_config2_split_pass_1p2m_x_80_automatic_plan(monkeypatch):
    """BASELINE config 2, the bench's default step: the plan switches the block-internal edges on by
    itself at this size (>= 32M owned wet cells) -- asserted through fesom2_mesh_info_."""
    for k in ("FESOM2_P1V_B3H", "FESOM2_PATCH", "FESOM2_B3HP_REG", "FESOM2_P1V_INT_DMA"):
        monkeypatch.delenv(k, raising=False)
    m = synth.config_mesh("1.2M x 80", full_depth=True)
    f = synth.make_fields(m)
    dm = engine.DeviceMesh(m)
    e = None
    try:
        dm.prepare()
        info = dm.info()
        assert info["internal_edges"] > 0.2 * m.E, info  # automatic: block-internal edges in p1v
        assert info["union_columns"] == 0, info  # large partition: no cluster unions
        e = engine.FctAle(dm, f, copy=False)
        assert e.split_pass() == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k) for k in FIELDS}
    finally:
        if e is not None:
            e.free()
        dm.free()
    check_owned(m, got, O.full_pass(m, f), "1.2M x 80 split")


@pytest.mark.parametrize("name,ntr", [("1.2M x 80", 6), ("127k x 47", 6)])
def test_config3_batched_split_pass(name, ntr):
    """BASELINE config 3: 6 tracers batched through the split entries (fct_ale_pre_comm_v_acc_ /
    fct_ale_post_comm_h_acc_ with ntracers = 6), each tracer against its own oracle pass."""
    m = synth.config_mesh(name, full_depth=name == "1.2M x 80")
    tracers = synth.make_tracer_fields(m, ntr)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        info = dm.info(batched=True)
        if name == "127k x 47":  # small partition: cluster unions of 8-column row-pair blocks, capped
            assert info["union_columns"] == 8 and 8 < info["union_max"] <= 21, info
        else:
            assert info["union_columns"] == 0, info
        assert e.split_pass() == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k).reshape(ntr, -1) for k in FIELDS}
    finally:
        e.free()
        dm.free()
    wants = pmap(lambda t: O.full_pass(m, t), tracers)
    for k, want in enumerate(wants):
        check_owned(m, {n: got[n][k] for n in FIELDS}, want, f"{name} tracer {k}")


def test_fused_batched_entries_on_the_large_batched_plan():
    """The batched plan of a large partition marks the internal edges' first-endpoint EdgeRefs for
    p1v's LDS stash (DESIGN.md 3, row pairs + stash); the fused batched entries
    (fct_ale_pre_comm_batched_acc_ -> fct_ale_post_comm_c_batched_acc_) gather over the same
    records and must read past the marks: 2 tracers at 1.2M x 80, exact per tracer."""
    m = synth.config_mesh("1.2M x 80", full_depth=True)
    tracers = synth.make_tracer_fields(m, 2)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        assert e.full_pass(fused=True) == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k).reshape(2, -1) for k in FIELDS}
    finally:
        e.free()
        dm.free()
    wants = pmap(lambda t: O.full_pass(m, t), tracers)
    for k, want in enumerate(wants):
        check_owned(m, {n: got[n][k] for n in FIELDS}, want, f"fused batch tracer {k}")


def partitioned_split_pass(locs, fields):
    """Every strip's pre_comm_v on the GPU, the caller's exchange of fct_plus/fct_minus between the
    strips (FESOM's exchange_nod, here by the halo lists through host memory), every strip's
    post_comm_h.  Returns the downloaded outputs per strip."""
    runs = []
    try:
        for (m, _), f in zip(locs, fields):
            dm = engine.DeviceMesh(m)
            runs.append((dm, engine.FctAle(dm, f, copy=False)))
        for _, e in runs:
            assert e.pre_comm_v() == 7, abi.last_error()
        pm = []
        for (m, _), (_, e) in zip(locs, runs):
            e.sync()
            pm.append([e.download("plus").reshape(-1, m.L), e.download("minus").reshape(-1, m.L)])
        for r, (m, h) in enumerate(locs):
            for q in h.neighbors:
                src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
                for a in range(2):
                    pm[r][a][dst] = pm[q][a][src]
        for r, (_, e) in enumerate(runs):
            e.upload("plus", pm[r][0].reshape(-1))
            e.upload("minus", pm[r][1].reshape(-1))
            assert e.post_comm_h() == 9, abi.last_error()
        outs = []
        for _, e in runs:
            e.sync()
            outs.append({k: e.download(k) for k in FIELDS})
        return outs
    finally:
        for dm, e in runs:
            e.free()
            dm.free()


def test_config1_127k_x_47_partitioned_4_strips():
    """BASELINE config 1 as FESOM runs it: the 127k x 47 mesh (variable depth) over 4 strips, split
    pass per strip with the exchange between phases; owned results equal the single-domain oracle."""
    nx, ny, nl = synth.CONFIGS["127k x 47"]
    g = synth.config_mesh("127k x 47")
    want = O.full_pass(g, synth.make_fields(g))
    locs = [partition.local_mesh(g, partition.strip_parts(nx, ny, 4), r) for r in range(4)]
    outs = partitioned_split_pass(locs, [synth.make_fields(m) for m, _ in locs])
    ms = [m for m, _ in locs]
    L = g.L
    wet = np.arange(L)[None, :] < (g.nlev_nod[:, None] - 1)
    for k in ("plus", "minus"):
        got = partition.gather_owned(ms, lambda r: outs[r][k], L, g.N).reshape(-1, L)
        assert np.array_equal(got[wet], want[k].reshape(-1, L)[wet]), k
    for k in ("del_v", "del_h"):
        assert np.array_equal(partition.gather_owned(ms, lambda r: outs[r][k], L, g.N), want[k]), k
    assert np.array_equal(partition.gather_owned(ms, lambda r: outs[r]["adf_v"], g.nl, g.N), want["adf_v"])
    adf_h = want["adf_h"].reshape(-1, L)
    for (m, _), o in zip(locs, outs):
        assert np.array_equal(o["adf_h"].reshape(-1, L), adf_h[m.edge_gid])


def test_config4_weak_geometry_3_strips_of_1p2m_x_80():
    """BASELINE config 4's per-GPU problem: strips of 1600 x 750 nodes x 80 levels (the weak-scaling
    9.6M geometry is 8 of them), here 3 strips so the middle one has two neighbours.  Each strip
    against the oracle on its own local mesh with the same exchange (equal to the single-domain pass,
    tests/test_partition.py)."""
    nx, ny, nl = synth.CONFIGS["1.2M x 80"]
    world = 3
    g = synth.make_mesh(nx, ny * world, nl, full_depth=True)
    part = partition.strip_parts(nx, ny * world, world)
    locs = [partition.local_mesh(g, part, r) for r in range(world)]
    del g
    fields = [synth.make_fields(m) for m, _ in locs]
    assert all(m.N == nx * ny for m, _ in locs) and len(locs[1][1].neighbors) == 2
    outs = partitioned_split_pass(locs, fields)
    # the oracle per strip: phase 1, the same exchange, phase 2
    p1 = pmap(lambda r: O.pre_comm(locs[r][0], fields[r]), range(world))
    assert all(st == 5 for st, _ in p1)
    L = nl - 1
    for r, (m, h) in enumerate(locs):
        for q in h.neighbors:
            src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
            for k in ("plus", "minus"):
                p1[r][1][k].reshape(-1, L)[dst] = p1[q][1][k].reshape(-1, L)[src]
    wants = pmap(lambda r: O.post_comm(locs[r][0], fields[r], p1[r][1]["plus"], p1[r][1]["minus"]), range(world))
    for r, (m, _) in enumerate(locs):
        wants[r].update(plus=p1[r][1]["plus"], minus=p1[r][1]["minus"])
        check_owned(m, outs[r], wants[r], f"strip {r}")
