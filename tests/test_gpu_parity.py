"""GPU parity: the HIP engine, driven through the C-ABI, against the oracle.

The bar is exact equality (``==`` on every cell, i.e. max-abs error 0, which is inside the
north star's fp64 tolerance of 1e-12): the engine's edge->node sums are gathers in ascending edge
order, so they perform the same IEEE additions as reference.cpp, and the library is built with
-ffp-contract=off.  Meshes are the synthetic ones of SURVEY.md §8(d) (parity levels: element
levels uniform in [3, nl]; roofline levels: full depth) and a node/element/edge-permuted variant.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import assert_cols_equal
from fesom2_amd import abi, engine, synth

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def device():
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    abi.set_path("fused")
    yield
    abi.set_resident(False)
    abi.set_path("fused")


_MESHES = {}


def mesh(name, full_depth=False, perm=False):
    key = (name, full_depth, perm)
    if key not in _MESHES:
        m = synth.config_mesh(name, full_depth=full_depth)
        if perm:
            m = synth.permute_mesh(m)
        _MESHES[key] = (m, synth.make_fields(m))
    return _MESHES[key]


def run_pass(m, f, fused=True, path="fused", resident=True, vlimit=1):
    abi.set_resident(resident)
    abi.set_path(path)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f, vlimit=vlimit)
    try:
        st = e.full_pass(fused=fused)
        e.sync()
        out = {k: e.download(k) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")}
    finally:
        e.free()
        dm.free()
        abi.set_resident(True)
        abi.set_path("fused")
    return st, out


def check_pass(m, got, want):
    L = m.L
    assert_cols_equal(got["plus"], want["plus"], m.nlev_nod, L, m.N, "fct_plus")
    assert_cols_equal(got["minus"], want["minus"], m.nlev_nod, L, m.N, "fct_minus")
    for k in ("adf_v", "adf_h", "del_v", "del_h"):
        g, w = got[k], want[k]
        bad = np.flatnonzero(g != w)
        assert bad.size == 0, f"{k}: {bad.size} entries differ, first at {bad[:5]}: {g[bad[0]]!r} vs {w[bad[0]]!r}"


CASES = [("tiny", False, False), ("8k x 20", False, False), ("8k x 20", True, False),
         ("8k x 20", False, True), ("127k x 47", False, False)]


@pytest.mark.parametrize("name,full,perm", CASES)
@pytest.mark.parametrize("fused,path", [(True, "fused"), (False, "fused"), (False, "stepwise"), (False, "reference")])
def test_full_pass_matches_oracle(name, full, perm, fused, path):
    m, f = mesh(name, full, perm)
    want = O.full_pass(m, f)
    st, got = run_pass(m, f, fused=fused, path=path)
    assert st == 9
    check_pass(m, got, want)


@pytest.mark.parametrize("vlimit", [2, 3])
@pytest.mark.parametrize("path", ["fused", "stepwise"])
def test_vlimit_variants(vlimit, path):
    """vlimit 2/3 (docs/refactoring.md:113-148), which reference.cpp does not implement."""
    m, f = mesh("8k x 20")
    st, want = O.pre_comm(m, f, vlimit=vlimit, vlimit_ext=True)
    assert st == 5
    abi.set_path(path)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f, vlimit=vlimit)
    try:
        assert e.pre_comm() == 6
        e.sync()
        assert_cols_equal(e.download("plus"), want["plus"], m.nlev_nod, m.L, m.N, f"plus vlimit {vlimit}")
        assert_cols_equal(e.download("minus"), want["minus"], m.nlev_nod, m.L, m.N, f"minus vlimit {vlimit}")
    finally:
        e.free()
        dm.free()
        abi.set_path("fused")


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6])
def test_stepwise_alg_state_bisection(k, monkeypatch):
    """FESOM2_NUM_KERNELS=k stops phase 1 after step k with the reference's alg_state and
    materialised intermediates (src/fesom2-accelerate.cu:256-337)."""
    m, f = mesh("8k x 20")
    steps = O.pre_comm_steps(m, f)
    monkeypatch.setenv("FESOM2_NUM_KERNELS", str(k))
    abi.set_path("stepwise")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        assert e.pre_comm() == k
        e.sync()
        want = steps[k]
        NT = m.N + m.H
        if k in (1, 2):
            assert_cols_equal(e.download("ttf_max"), want["ttf_max"], m.nlev_nod, m.L, NT, "ttf_max")
            assert_cols_equal(e.download("ttf_min"), want["ttf_min"], m.nlev_nod, m.L, NT, "ttf_min")
        else:
            assert_cols_equal(e.download("ttf_max"), want["ttf_max"], m.nlev_nod, m.L, m.N, "ttf_max")
            assert_cols_equal(e.download("ttf_min"), want["ttf_min"], m.nlev_nod, m.L, m.N, "ttf_min")
        if k == 2:
            assert np.array_equal(e.download("UV_rhs"), want["UV"])
        if k >= 4:
            assert_cols_equal(e.download("plus"), want["plus"], m.nlev_nod, m.L, m.N, "plus")
            assert_cols_equal(e.download("minus"), want["minus"], m.nlev_nod, m.L, m.N, "minus")
    finally:
        e.free()
        dm.free()
        abi.set_path("fused")


def test_reference_transfer_semantics():
    """Non-resident mode keeps the reference's implicit copies: pre_comm uploads fct_LO and
    downloads fct_plus/minus (:268, :338-339); inter_comm downloads fct_adf_v (:355); post_comm
    uploads fct_plus/minus (:364-365) and downloads fct_adf_h (:378)."""
    m, f = mesh("8k x 20")
    want = O.full_pass(m, f)
    abi.set_resident(False)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        # poison the device copy of fct_LO: pre_comm must re-upload it from the host array
        e.upload("LO", np.full(e.host["LO"].size, 123.0))
        assert e.pre_comm() == 6
        e.sync()
        assert_cols_equal(e.host["plus"], want["plus"], m.nlev_nod, m.L, m.N, "host fct_plus")
        assert e.inter_comm() == 7
        # the caller's exchange writes the host arrays; post_comm must upload them again
        assert e.post_comm() == 8
        e.sync()
        assert np.array_equal(e.host["adf_v"], want["adf_v"])
        assert np.array_equal(e.host["adf_h"], want["adf_h"])
        assert e.c_step() == 9
        e.sync()
        assert np.array_equal(e.host["del_v"], want["del_v"])
        assert np.array_equal(e.host["del_h"], want["del_h"])
    finally:
        e.free()
        dm.free()
        abi.set_resident(True)


@pytest.mark.parametrize("name", ["8k x 20", "127k x 47"])
def test_producer_upload_mode_two_streams(name):
    """Round 5: a device-resident host that uploads the producer's fields (and its del_ttf) itself
    and takes back only del_ttf with fesom2_transfer_back_async_, two tracers on two streams from
    page-locked arrays (bench.py --transfers producer): every output equals the oracle's, del_ttf in
    the host arrays (which held the inputs before: the downloads replaced them); the host writes no
    pinned array while a transfer from it may be in flight, as FESOM2 would not."""
    from fesom2_amd import synth
    m, _ = mesh(name)
    tracers = synth.make_tracer_fields(m, 2)
    wants = [O.full_pass(m, t) for t in tracers]
    streamed = ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h")
    dm = engine.DeviceMesh(m)
    engines, pins = [], []
    try:
        for t in tracers:
            e = engine.FctAle(dm, t)
            engines.append(e)
        hosts = []
        for k, t in enumerate(tracers):
            h = {}
            for name_ in streamed:
                a, hp = abi.pinned(t[name_].size)
                a[:] = t[name_]
                pins.append(hp)
                h[name_] = a
            hosts.append(h)
        # the device copies start poisoned: only the in-step uploads may feed the pass
        for e in engines:
            for name_ in streamed:
                e.upload(name_, np.full(e.size(name_), 7.0))
        for e, h in zip(engines, hosts):
            for name_ in streamed:
                abi.transfer_var_async(e.h[name_], h[name_], e.stream, name_ in ("ttf", "adf_v", "adf_h"))
            assert e.pre_comm_v() == 7, abi.last_error()
            assert e.post_comm_h() == 9, abi.last_error()
            for name_ in ("del_v", "del_h"):
                abi.transfer_back_async(e.h[name_], h[name_], e.stream)
        for e in engines:
            e.sync()
        for k, (e, h) in enumerate(zip(engines, hosts)):
            n = m.N * m.L
            assert np.array_equal(h["del_v"][:n], wants[k]["del_v"][:n]), k
            assert np.array_equal(h["del_h"][:n], wants[k]["del_h"][:n]), k
            assert np.array_equal(e.download("adf_h"), wants[k]["adf_h"]), k
            assert_cols_equal(e.download("plus"), wants[k]["plus"], m.nlev_nod, m.L, m.N, f"plus[{k}]")
    finally:
        for e in engines:
            e.free()
        dm.free()
        for hp in pins:
            abi.free_pinned(hp)


def test_transfer_back_async_refuses_a_null_host_array():
    m, f = mesh("tiny")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        st = C.c_int(0)
        abi.dll().fesom2_transfer_back_async_(e.h["del_v"].ref, None, e.stream.ref, C.byref(st))
        assert st.value == 1 and "no host array" in abi.last_error()
    finally:
        e.free()
        dm.free()


def test_invalid_mesh_fails_loudly_without_launch():
    """An out-of-range edge node must be rejected on the host (alg_state 0), not faulted on."""
    m, f = mesh("tiny")
    import dataclasses
    bad = dataclasses.replace(m, edges=m.edges.copy())
    bad.edges[5] = m.N + 1000
    dm = engine.DeviceMesh(bad)
    e = engine.FctAle(dm, f)
    try:
        assert e.pre_comm() == 0
        assert "outside" in abi.last_error()
    finally:
        e.free()
        dm.free()


def test_repeat_is_deterministic():
    m, f = mesh("8k x 20", perm=True)
    _, a = run_pass(m, f)
    _, b = run_pass(m, f)
    for k in a:
        assert np.array_equal(a[k].view(np.uint64), b[k].view(np.uint64)), k


@pytest.mark.slow
def test_full_size_1p2m_x_80():
    """BASELINE config 2 at full size (1.2M nodes x 80 levels, full depth): exact vs the oracle."""
    m, f = mesh("1.2M x 80", full_depth=True)
    want = O.full_pass(m, f)
    st, got = run_pass(m, f)
    assert st == 9
    check_pass(m, got, want)


@pytest.mark.parametrize("name", ["tiny_16x8x10", "small_24x12x15"])
def test_golden_vectors_on_gpu(name):
    """The committed vectors made by the reference's own code (tests/golden/make_golden.py)."""
    from test_oracle import load_fixture
    m, f, want = load_fixture(name)
    st, got = run_pass(m, f)
    assert st == 9
    check_pass(m, got, want)


@pytest.mark.parametrize("kind,nranks", [("strips", 2), ("strips", 4), ("random", 3)])
def test_partitioned_pass_on_one_gpu(kind, nranks):
    """Halo meshes through the HIP engine: phase 1 per partition, the caller's exchange of
    fct_plus/fct_minus (here on the host, as the Fortran's exchange_nod does), fused phase 2.
    Owned results must equal the single-domain oracle exactly."""
    from fesom2_amd import partition
    nx, ny, nl = 64, 48, 21
    g = synth.make_mesh(nx, ny, nl)
    want = O.full_pass(g, synth.make_fields(g))
    if kind == "strips":
        part = partition.strip_parts(nx, ny, nranks)
    else:
        part = np.random.default_rng(3).integers(0, nranks, g.N).astype(np.int32)
    locs = [partition.local_mesh(g, part, r) for r in range(nranks)]
    runs = []
    try:
        for m, _ in locs:
            dm = engine.DeviceMesh(m)
            runs.append((dm, engine.FctAle(dm, synth.make_fields(m))))
        for _, e in runs:
            assert e.pre_comm() == 6
        pm = []
        for _, e in runs:
            e.sync()
            pm.append((e.download("plus").reshape(-1, g.L), e.download("minus").reshape(-1, g.L)))
        for r, (m, h) in enumerate(locs):
            for q in h.neighbors:
                src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
                pm[r][0][dst] = pm[q][0][src]
                pm[r][1][dst] = pm[q][1][src]
            runs[r][1].upload("plus", pm[r][0].reshape(-1))
            runs[r][1].upload("minus", pm[r][1].reshape(-1))
        for _, e in runs:
            assert e.post_comm_c() == 9
        outs = []
        for _, e in runs:
            e.sync()
            outs.append({k: e.download(k) for k in ("del_v", "del_h", "adf_v")})
    finally:
        for dm, e in runs:
            e.free()
            dm.free()
    ms = [m for m, _ in locs]
    for k in ("del_v", "del_h"):
        assert np.array_equal(partition.gather_owned(ms, lambda r: outs[r][k], g.L, g.N), want[k]), k
    assert np.array_equal(partition.gather_owned(ms, lambda r: outs[r]["adf_v"], g.nl, g.N), want["adf_v"])
    owned_plus = partition.gather_owned(ms, lambda r: pm[r][0].reshape(-1), g.L, g.N)
    assert_cols_equal(owned_plus, want["plus"], g.nlev_nod, g.L, g.N, "plus")


@pytest.mark.parametrize("ntr", [1, 3])
@pytest.mark.parametrize("kind", ["strips", "random", "delaunay"])
def test_partitioned_split_pass_with_cluster_unions(kind, ntr):
    """The default entry sequence on halo meshes at FESOM2's per-GPU depth class (nl - 1 <= 64, so
    the plans stage p1v's cluster unions in LDS, and the unions hold halo columns):
    fct_ale_pre_comm_v_acc_ per partition, the caller's exchange of fct_plus/fct_minus on the host,
    fct_ale_post_comm_h_acc_; 1 tracer and a batch of 3.  Owned results equal the single-domain
    oracle exactly."""
    from fesom2_amd import partition
    nl, nranks = 21, 3
    if kind == "delaunay":
        g = synth.delaunay_mesh(4000, nl)
        part = np.random.default_rng(11).integers(0, nranks, g.N).astype(np.int32)
    else:
        nx, ny = 64, 48
        g = synth.make_mesh(nx, ny, nl)
        part = (partition.strip_parts(nx, ny, nranks) if kind == "strips"
                else np.random.default_rng(3).integers(0, nranks, g.N).astype(np.int32))
    gtr = synth.make_tracer_fields(g, ntr)
    want = [O.full_pass(g, gtr[k]) for k in range(ntr)]
    locs = [partition.local_mesh(g, part, r) for r in range(nranks)]
    runs = []
    try:
        for m, _ in locs:
            dm = engine.DeviceMesh(m)
            assert dm.info(batched=ntr > 1)["union_columns"] > 0
            ftr = synth.make_tracer_fields(m, ntr)
            runs.append((dm, engine.FctAle(dm, ftr[0]) if ntr == 1 else engine.FctAleBatch(dm, ftr)))
        for _, e in runs:
            assert e.pre_comm_v() == 7, abi.last_error()
        pm = []
        for _, e in runs:
            e.sync()
            pm.append([e.download(k).reshape(ntr, -1, g.L) for k in ("plus", "minus")])
        for r, (m, h) in enumerate(locs):
            for q in h.neighbors:
                src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
                for a in range(2):
                    pm[r][a][:, dst] = pm[q][a][:, src]
            for a, name in enumerate(("plus", "minus")):
                runs[r][1].upload(name, pm[r][a].reshape(-1))
        for _, e in runs:
            assert e.post_comm_h() == 9, abi.last_error()
        outs = []
        for _, e in runs:
            e.sync()
            outs.append({k: e.download(k).reshape(ntr, -1) for k in ("del_v", "del_h", "adf_v")})
    finally:
        for dm, e in runs:
            e.free()
            dm.free()
    ms = [m for m, _ in locs]
    for t in range(ntr):
        for k in ("del_v", "del_h"):
            got = partition.gather_owned(ms, lambda r: outs[r][k][t], g.L, g.N)
            assert np.array_equal(got, want[t][k]), (k, t)
        got = partition.gather_owned(ms, lambda r: outs[r]["adf_v"][t], g.nl, g.N)
        assert np.array_equal(got, want[t]["adf_v"]), ("adf_v", t)
        owned_plus = partition.gather_owned(ms, lambda r: pm[r][0][t].reshape(-1), g.L, g.N)
        assert_cols_equal(owned_plus, want[t]["plus"], g.nlev_nod, g.L, g.N, "plus")


def test_reference_named_entries_run_on_gpu():
    """fct_ale_a1_reference_ .. fct_ale_pre_comm_ (reference .h:142, :225-235) on host arrays,
    executed by the HIP engine: same results as reference.cpp's CPU functions."""
    import ctypes as C
    from fesom2_amd.abi import arr, dll, dp, ip
    m, f = mesh("8k x 20")
    L, NT = m.L, m.N + m.H
    tmax, tmin, plus, minus = (np.zeros(NT * L) for _ in range(4))
    UV = np.zeros(2 * L * m.T)
    st = C.c_int(-1)
    dll().fct_ale_pre_comm_(C.byref(st), arr(tmax), arr(tmin), arr(plus), arr(minus), arr(f["ttf"]), arr(f["LO"]),
                            arr(f["adf_v"]), arr(f["adf_h"]), arr(UV), arr(f["area_inv"]), ip(m.N), ip(m.H),
                            ip(m.T), ip(m.E), ip(m.nl), arr(m.nlev_nod), arr(m.nlev_elem), arr(m.elem2D_nodes),
                            arr(m.nie_num), arr(m.nie), ip(m.dim), arr(m.edges), arr(m.edge_tri), ip(1), dp(1e-16),
                            dp(1e3), dp(1.0))
    assert st.value == 5
    want = O.pre_comm(m, f)[1]
    for k, v in (("ttf_max", tmax), ("ttf_min", tmin), ("plus", plus), ("minus", minus), ("UV", UV)):
        assert np.array_equal(v, want[k]), k


@pytest.mark.parametrize("name", ["tiny", "8k x 20", "127k x 47"])
@pytest.mark.parametrize("iterations", [2, 3])
@pytest.mark.parametrize("resident", [True, False])
@pytest.mark.parametrize("final", ["split", "fused"])
def test_iter_yn_iterations_match_oracle(name, iterations, resident, final):
    """iter_yn (docs/refactoring.md:227-290): iterations-1 rounds of fct_ale_post_comm_iter_acc_
    (LO update + remainder hand-over) then the final pass (direction-split or fused entries); every
    array equals the oracle's restatement of the Fortran (parity unpinned: no executable reference
    holds this branch)."""
    m, f = mesh(name)
    want = O.iterated_pass(m, f, iterations)
    abi.set_resident(resident)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        assert e.iterated_pass(iterations, final=final) == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h", "LO", "adf_v2",
                                          "adf_h2")}
    finally:
        abi.set_resident(True)
        e.free()
        dm.free()
    check_pass(m, got, want)
    for k in ("LO", "adf_v2", "adf_h2"):
        bad = np.flatnonzero(got[k] != want[k])
        assert bad.size == 0, f"{k}: {bad.size} differ, first at {bad[:5]}"


def test_iter_yn_batched():
    m = synth.config_mesh("8k x 20")
    tracers = synth.make_tracer_fields(m, 3)
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers)
    try:
        assert e.iterated_pass(2) == 9, abi.last_error()  # final pass: the batched split entries
        e.sync()
        for k in range(3):
            want = O.iterated_pass(m, tracers[k], 2)
            for name in ("LO", "adf_v", "adf_h", "del_v", "del_h", "adf_v2", "adf_h2"):
                assert np.array_equal(e.tracer(name, k), want[name]), (name, k)
    finally:
        e.free()
        dm.free()


def test_iter_yn_whole_array_swap_keeps_unassigned_levels():
    """Nonzero fct_adf_v2/fct_adf_h2 before the call: levels the iteration does not assign (nz=1,
    bottom interface, dry levels) reach fct_adf_v/fct_adf_h through the whole-array assignment."""
    m, f = mesh("8k x 20")
    st, p1 = O.pre_comm(m, f)
    rng = np.random.default_rng(5)
    v2, h2 = rng.standard_normal(f["adf_v"].size), rng.standard_normal(f["adf_h"].size)
    want = O.post_comm_iter(m, f, p1["plus"], p1["minus"], v2, h2)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        e._iter_buffers()
        e.upload("adf_v2", v2)
        e.upload("adf_h2", h2)
        assert e.pre_comm() == 6
        assert e.post_comm_iter() == 9, abi.last_error()
        e.sync()
        for k in ("LO", "adf_v", "adf_h", "adf_v2", "adf_h2"):
            got = e.download(k)
            bad = np.flatnonzero(got != want[k])
            assert bad.size == 0, f"{k}: {bad.size} differ, first at {bad[:5]}"
    finally:
        e.free()
        dm.free()


def test_sizes_beyond_int32():
    """The reference's int sizes stop at 2^31-1: a negative size is rejected (istat 1, no huge
    hipMalloc), and the int64 entries allocate the same kind of handle."""
    import ctypes as C
    from fesom2_amd.abi import arr, bp, dll, ip
    h = abi.Handle("neg")
    st = C.c_int(0)
    dll().alloc_var_(h.ref, None, ip(-5), bp(False), C.byref(st))
    assert st.value == 1 and not h and "< 0" in abi.last_error()
    a = np.arange(1000, dtype=np.float64)
    h8 = abi.Handle("i8")
    dll().fesom2_alloc_var_i8_(h8.ref, arr(a), C.byref(C.c_longlong(a.size)), bp(True), C.byref(st))
    assert st.value == 0 and h8
    dll().transfer_var_(h8.ref, arr(a))
    out = np.zeros_like(a)
    dll().fesom2_download_(h8.ref, arr(out), C.byref(st))
    assert st.value == 0 and np.array_equal(out, a)
    dll().fesom2_free_(h8.ref)


def run_split(m, f, vlimit=1):
    """The direction-split pass (bench default): fct_ale_pre_comm_v_acc_ -> fct_ale_post_comm_h_acc_."""
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f, vlimit=vlimit)
    try:
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        return {k: e.download(k) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")}
    finally:
        e.free()
        dm.free()


@pytest.mark.parametrize("nl", [3, 4, 5, 6, 48, 81, 129, 200])
@pytest.mark.parametrize("full", [False, True])
@pytest.mark.parametrize("mode", ["fused", "sequence", "split"])
def test_level_counts(nl, full, mode):
    """Level counts from the minimum to deep columns, odd and even L (one or two levels per thread,
    odd L in pairs with a one-level last slot on the split path, columns per block from 1 to 64,
    80-level columns and 128/199-level ones)."""
    m = synth.make_mesh(40, 14, nl, full_depth=full)
    f = synth.make_fields(m)
    if mode == "split":
        got = run_split(m, f)
    else:  # fused: pre_comm -> post_comm_c; sequence: pre_comm -> inter_comm -> post_comm -> c
        st, got = run_pass(m, f, fused=mode == "fused")
        assert st == 9
    check_pass(m, got, O.full_pass(m, f))


def degenerate_mesh(kind):
    """Shallow columns the synthetic generator never makes: "one_level" (nl = 2, a single level per
    column), "one_wet" (nl = 11 but every element has 2 levels: one wet cell per column, the rest of
    each column dry), "shallow_region" (a band of elements with 2 levels, so whole nodes have one wet
    level next to deep ones)."""
    import dataclasses
    if kind == "one_level":
        m = synth.make_mesh(16, 8, 3, full_depth=True)
        return dataclasses.replace(m, nl=2, nlev_elem=np.full_like(m.nlev_elem, 2), nlev_nod=np.full_like(m.nlev_nod, 2),
                                   name="16x8x1")
    m = synth.make_mesh(40, 14, 11, full_depth=kind == "one_wet")
    le = m.nlev_elem.copy()
    if kind == "one_wet":
        le[:] = 2
    else:
        le[: le.size // 3] = 2
    en = m.elem2D_nodes.reshape(-1, 3) - 1
    ln = np.zeros(m.N, np.int64)
    np.maximum.at(ln, en.reshape(-1), np.repeat(le, 3).astype(np.int64))
    return dataclasses.replace(m, nlev_elem=le.astype(np.int32), nlev_nod=ln.astype(np.int32), name=kind)


@pytest.mark.parametrize("kind", ["one_level", "one_wet", "shallow_region"])
@pytest.mark.parametrize("mode", ["split", "split_internal", "fused", "sequence", "stepwise", "vlimit2", "vlimit3"])
def test_degenerate_level_counts(kind, mode, monkeypatch):
    """Columns with one level or one wet cell: every path equals the oracle (b3v limits nz = 1 only,
    the a3 stencil has no interior levels, b1v reads the bottom interface)."""
    m = degenerate_mesh(kind)
    if kind == "shallow_region":
        assert (m.nlev_nod == 2).any() and (m.nlev_nod > 2).any()
    f = synth.make_fields(m)
    monkeypatch.setenv("FESOM2_P1V_B3H", "1" if mode == "split_internal" else "0")
    vl = int(mode[-1]) if mode.startswith("vlimit") else 1
    if mode.startswith("split") or mode.startswith("vlimit"):
        got = run_split(m, f, vlimit=vl)
    else:
        st, got = run_pass(m, f, fused=mode == "fused", path="stepwise" if mode == "stepwise" else "fused")
        assert st == 9, abi.last_error()
    check_pass(m, got, O.full_pass(m, f, vlimit=vl))


# plan options of the product library (read once when a mesh plan is built)
PLAN_OPTIONS = [{"FESOM2_P1V_B3H": "0"}, {"FESOM2_P1V_B3H": "1"}, {"FESOM2_PATCH": "64"}, {"FESOM2_PATCH": "0"},
                {"FESOM2_PATCH": "100", "FESOM2_P1V_B3H": "1"}, {"FESOM2_PATCH": "4096", "FESOM2_P1V_B3H": "1"},
                {"FESOM2_CACHE_ORDER": "0"}, {"FESOM2_CACHE_ORDER": "1", "FESOM2_P1V_B3H": "1"},
                # round 6: cluster unions off (the plain gather plan) / forced on with the large-partition
                # rules (row-pair blocks of 6 at L = 80, internal edges, stash) / with a patch size
                {"FESOM2_P1V_UNION": "0"}, {"FESOM2_P1V_UNION": "1", "FESOM2_LARGE_CELLS": "0"},
                {"FESOM2_P1V_UNION": "1", "FESOM2_PATCH": "100"}]


@pytest.mark.parametrize("nl", [3, 4, 5, 48, 81, 129])
@pytest.mark.parametrize("full", [False, True])
def test_internal_edges_level_counts_and_repeats(nl, full, monkeypatch):
    """FESOM2_P1V_B3H=1 (block-internal edges limited in p1v): three passes on the same plan, inputs
    re-uploaded before each, every one exact."""
    monkeypatch.setenv("FESOM2_P1V_B3H", "1")
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


@pytest.mark.parametrize("name", ["8k x 20", "127k x 47"])
def test_block_internal_edges(name, monkeypatch):
    """p1v limits the block-internal edges (both endpoints among one p1v block's columns) and b3h the
    rest: the plan reports them, the split pass stays exact, and a phase 2 other than
    fct_ale_post_comm_h_acc_ after fct_ale_pre_comm_v_acc_ fails loudly instead of limiting twice."""
    monkeypatch.setenv("FESOM2_P1V_B3H", "1")  # (automatic from 32M wet cells)
    m, f = mesh(name)
    dm = engine.DeviceMesh(m)
    info = dm.info()
    assert info["p1v_columns"] > 1 and 0 < info["internal_edges"] < info["interior_edges"] == m.E
    assert info["crossing_edges"] + info["internal_edges"] == info["interior_edges"]
    assert info["internal_edge_cells"] > info["internal_edges"]
    e = engine.FctAle(dm, f)
    try:
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_c() != 9 and "fct_ale_post_comm_h_acc_" in abi.last_error()
        for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
            e.upload(k)  # an upload clears the mark: the full fused pass runs again
        assert e.full_pass() == 9, abi.last_error()
        e.sync()
        check_pass(m, {k: e.download(k) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")},
                   O.full_pass(m, f))
    finally:
        e.free()
        dm.free()
    monkeypatch.setenv("FESOM2_P1V_B3H", "0")
    dm = engine.DeviceMesh(m)
    try:
        assert dm.info()["internal_edges"] == 0
    finally:
        dm.free()


@pytest.mark.parametrize("knobs", PLAN_OPTIONS, ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()))
@pytest.mark.parametrize("name,perm", [("8k x 20", False), ("8k x 20", True), ("127k x 47", False)])
def test_split_plan_options_match_oracle(knobs, name, perm, monkeypatch):
    """The plan options (block-internal edges in p1v or not, patch sizes incl. index order) are all
    exact on the direction-split pass."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    m, f = mesh(name, False, perm)
    check_pass(m, run_split(m, f), O.full_pass(m, f))


@pytest.mark.parametrize("name,full,perm", CASES + [("tiny", True, False)])
@pytest.mark.parametrize("resident", [True, False])
@pytest.mark.parametrize("internal", ["0", "1"])
def test_split_by_direction_matches_oracle(name, full, perm, resident, internal, monkeypatch):
    """fct_ale_pre_comm_v_acc_ (a1..b2 + b3v + cv) then fct_ale_post_comm_h_acc_ (b3h + ch): the
    same results as the reference sequence, every output exact (block-internal edges limited in p1v
    or all in b3h)."""
    monkeypatch.setenv("FESOM2_P1V_B3H", internal)
    m, f = mesh(name, full, perm)
    want = O.full_pass(m, f)
    abi.set_resident(resident)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        assert e.pre_comm_v() == 7, abi.last_error()
        assert e.post_comm_h() == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")}
    finally:
        abi.set_resident(True)
        e.free()
        dm.free()
    check_pass(m, got, want)


@pytest.mark.parametrize("vlimit", [2, 3])
@pytest.mark.parametrize("name,internal", [("8k x 20", "0"), ("8k x 20", "1"), ("127k x 47", "0"), ("127k x 47", "1")])
def test_split_by_direction_vlimit(vlimit, name, internal, monkeypatch):
    """vlimit 2/3 on the split path, with and without the block-internal edges limited in p1v (odd L
    runs in level pairs at every vlimit since round 3, so the plan's internal-edge lists match the
    vlimit-2/3 blocks too)."""
    monkeypatch.setenv("FESOM2_P1V_B3H", internal)
    m, f = mesh(name)
    st, p1 = O.pre_comm(m, f, vlimit=vlimit, vlimit_ext=True)
    want = O.post_comm(m, f, p1["plus"], p1["minus"])
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f, vlimit=vlimit)
    try:
        assert e.split_pass() == 9, abi.last_error()
        e.sync()
        for k in ("adf_v", "adf_h", "del_v", "del_h"):
            assert np.array_equal(e.download(k), want[k]), k
        assert_cols_equal(e.download("plus"), p1["plus"], m.nlev_nod, m.L, m.N, "plus")
        assert_cols_equal(e.download("minus"), p1["minus"], m.nlev_nod, m.L, m.N, "minus")
    finally:
        e.free()
        dm.free()


def test_graph_replay_matches_oracle():
    """A split pass captured into a hipGraph (fesom2_graph_begin_/end_) and replayed gives the eager
    results; a capture that would have to build a mesh plan fails cleanly."""
    m, f = mesh("127k x 47")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        assert e.pre_comm_v() == 7 and e.post_comm_h() == 9  # builds the plans
        for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
            e.upload(k)  # pristine inputs again
        e.sync()
        with abi.Graph.capture(e.stream) as g:
            assert e.pre_comm_v() == 7, abi.last_error()
            assert e.post_comm_h() == 9, abi.last_error()
        g.launch(e.stream)
        e.sync()
        got = {k: e.download(k) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")}
        g.free()
    finally:
        e.free()
        dm.free()
    check_pass(m, got, O.full_pass(m, f))
    # no plan yet for a fresh mesh: the capture refuses to build one
    m2, f2 = mesh("8k x 20", True)
    dm2 = engine.DeviceMesh(m2)
    e2 = engine.FctAle(dm2, f2)
    try:
        with abi.Graph.capture(e2.stream) as g2:
            assert e2.pre_comm_v() == 0
            assert "graph capture" in abi.last_error()
        g2.free()
    finally:
        e2.free()
        dm2.free()


@pytest.mark.parametrize("name,full", [("8k x 20", False), ("8k x 20", True), ("127k x 47", False), ("tiny", True)])
@pytest.mark.parametrize("resident", [True, False])
@pytest.mark.parametrize("internal", ["0", "1"])
@pytest.mark.parametrize("vlimit", [1, 2])
@pytest.mark.parametrize("bind", [False, True])
def test_reference_sequence_fast_mode(name, full, resident, internal, vlimit, bind, monkeypatch):
    """fesom2_set_path_(2): the unmodified reference sequence pre_comm -> inter_comm -> post_comm -> c
    with b3v (and the block-internal edges) done inside pre_comm -- and with c-vertical bound
    (fesom2_bind_c_vertical_) also cv there, the c-step c-horizontal only; every output exact, with
    the reference's transfer semantics too (inter_comm still hands the host the limited fct_adf_v)."""
    monkeypatch.setenv("FESOM2_P1V_B3H", internal)
    m, f = mesh(name, full)
    st, p1 = O.pre_comm(m, f, vlimit=vlimit, vlimit_ext=True)
    want = O.post_comm(m, f, p1["plus"], p1["minus"])
    abi.set_resident(resident)
    abi.set_path("reference")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f, vlimit=vlimit)
    if bind:
        e.bind_c_vertical()
    pristine = {k: e.host[k].copy() for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h")}
    try:
        for _ in range(2):  # twice on the same buffers: the marks are consumed every pass
            for k, v in pristine.items():
                e.host[k][:] = v  # (the reference transfers wrote the outputs into the host arrays)
                e.upload(k)
            assert e.pre_comm() == 6, abi.last_error()
            assert e.inter_comm() == 7, abi.last_error()
            assert e.post_comm() == 8, abi.last_error()
            assert e.c_step() == 9, abi.last_error()
            e.sync()
            for k in ("adf_v", "adf_h", "del_v", "del_h"):
                got = e.host[k] if not resident else e.download(k)
                assert np.array_equal(got, want[k]), k
    finally:
        abi.set_resident(True)
        abi.set_path("fused")
        e.free()
        dm.free()


def test_fast_mode_marks_refuse_other_phase_2():
    """After a fast-mode fct_ale_pre_comm_acc_ the fused phase 2 would limit fct_adf_v twice: it
    refuses; a second pre_comm without fresh fluxes refuses too."""
    m, f = mesh("8k x 20")
    abi.set_path("reference")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        assert e.pre_comm() == 6, abi.last_error()
        assert e.post_comm_c() != 9 and "fct_adf_v" in abi.last_error()
        assert e.pre_comm() != 6 and "upload" in abi.last_error()
    finally:
        abi.set_path("fused")
        e.free()
        dm.free()


def test_fast_mode_c_vertical_binding_checks():
    """A bound del_ttf_advvert that the c-step is not given is refused; unbinding restores the
    b3v-only pre_comm (and the full c-step)."""
    m, f = mesh("8k x 20")
    want = O.full_pass(m, f)
    abi.set_path("reference")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        e.bind_c_vertical()
        assert e.pre_comm() == 6 and e.inter_comm() == 7 and e.post_comm() == 8
        h = e.h
        e.h = dict(h, del_v=h["del_h"])  # the wrong del_ttf_advvert handle
        assert e.c_step() != 9 and "bound" in abi.last_error()
        e.h = h
        assert e.c_step() == 9, abi.last_error()
        e.sync()
        for k in ("del_v", "del_h", "adf_v", "adf_h"):
            assert np.array_equal(e.download(k), want[k]), k
        e.bind_c_vertical(False)
        for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
            e.upload(k)
        assert e.full_pass(fused=False) == 9, abi.last_error()
        e.sync()
        for k in ("del_v", "del_h", "adf_v", "adf_h"):
            assert np.array_equal(e.download(k), want[k]), k
    finally:
        abi.set_path("fused")
        e.free()
        dm.free()


def test_fast_mode_marks_refuse_a_split_pre_comm():
    """after a fast-mode fct_ale_pre_comm_acc_ (b3v, the internal edges and with the
    binding c-vertical done) the split entry fct_ale_pre_comm_v_acc_ and the batched/fused phase 1
    refuse the marked fluxes instead of limiting them a second time; fresh uploads clear the marks."""
    m, f = mesh("8k x 20", full_depth=True)
    want = O.full_pass(m, f)
    abi.set_path("reference")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        e.bind_c_vertical()
        assert e.pre_comm() == 6, abi.last_error()
        assert e.pre_comm_v() != 7 and "already hold a limited" in abi.last_error()
        abi.set_path("fused")
        assert e.pre_comm() != 6 and "already hold a limited" in abi.last_error()
        for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
            e.upload(k)
        assert e.split_pass() == 9, abi.last_error()
        e.sync()
        for k in ("del_v", "del_h", "adf_v", "adf_h"):
            assert np.array_equal(e.download(k), want[k]), k
    finally:
        abi.set_path("fused")
        e.bind_c_vertical(False)
        e.free()
        dm.free()


def test_fast_mode_c_step_checks_every_bound_field():
    """with c-vertical done in the fast-mode pre_comm, a c-step given other hnode /
    hnode_new / area handles than the bound ones is refused (c-vertical and c-horizontal would use
    different fields)."""
    m, f = mesh("8k x 20")
    abi.set_path("reference")
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        e.bind_c_vertical()
        assert e.pre_comm() == 6 and e.inter_comm() == 7 and e.post_comm() == 8, abi.last_error()
        h = e.h
        for k, other in (("hnode", "hnode_new"), ("hnode_new", "hnode"), ("area", "area_inv")):
            e.h = dict(h, **{k: h[other]})
            assert e.c_step() != 9 and "bound others" in abi.last_error(), k
        e.h = h
        assert e.c_step() == 9, abi.last_error()
    finally:
        abi.set_path("fused")
        e.bind_c_vertical(False)
        e.free()
        dm.free()


def test_kernel_timing_only_times_the_named_kernel():
    """fesom2_kernel_timing_only_ (bench.py --kernel-timing dominant): while a name is set only that
    kernel's launches get events; with None every launch of the split pass is timed again.  Results
    are unaffected by the timing."""
    m, f = mesh("8k x 20", full_depth=True)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f, copy=False)
    try:
        abi.kernel_timing(True)
        for only, want in (("fct_ale_p1v", {"fct_ale_p1v"}), (None, {"fct_ale_p1v", "fct_ale_b3_horizontal", "fct_ale_p2h"})):
            abi.kernel_timing_only(only)
            abi.kernel_timing_reset()
            for _ in range(3):
                for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
                    e.upload(k)  # pristine inputs for every pass
                assert e.split_pass() == 9, abi.last_error()
            e.sync()
            st = abi.kernel_stats()
            assert set(st) == want, st
            assert all(cnt == 3 and ms > 0 for cnt, ms in st.values()), st
        got = {k: e.download(k) for k in ("adf_v", "adf_h", "del_v", "del_h")}
    finally:
        abi.kernel_timing(False)
        abi.kernel_timing_only(None)
        e.free()
        dm.free()
    want = O.full_pass(m, f)
    for k, g in got.items():
        assert np.array_equal(g, want[k]), k


@pytest.mark.parametrize("path", ["split", "fused", "stepwise"])
def test_mesh_without_edges_matches_oracle(path):
    """The edge loops' empty case (myDim_edge2D = 0, a partition with no local edges): b1h, b3h and
    c-horizontal are no-ops, every launch over the edges has zero blocks, and the rest of the pass
    equals the oracle's (which the reference's loops admit, tests/test_oracle.py)."""
    import dataclasses
    m0, f0 = mesh("tiny")
    m = dataclasses.replace(m0, E=0)
    f = dict(f0, adf_h=np.zeros(0))
    want = O.full_pass(m, f)
    abi.set_path("fused" if path == "split" else path)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        st = e.split_pass() if path == "split" else e.full_pass(fused=path == "fused")
        e.sync()
        assert st == 9, abi.last_error()
        got = {k: e.download(k) for k in ("plus", "minus", "adf_v", "del_v", "del_h")}
    finally:
        e.free()
        dm.free()
        abi.set_path("fused")
    L = m.L
    for k in ("plus", "minus"):
        assert_cols_equal(got[k], want[k], m.nlev_nod, L, m.N, k)
    for k in ("adf_v", "del_v", "del_h"):
        assert np.array_equal(got[k][: want[k].size], want[k]), k


@pytest.mark.parametrize("seed", range(12))
def test_random_shapes_split_and_batched(seed):
    """Randomised shapes for the level-pair kernels (odd and even L from 2 to 63, shallow and full
    depth, grids whose node count is no multiple of a block): the direction-split pass of one tracer
    and a batch of two, each equal to the oracle.  Odd L exercises the pair loads that read one level
    past a column (into the next column, or the allocation pad after the last one)."""
    rng = np.random.default_rng(1000 + seed)
    nx, ny, nl = int(rng.integers(5, 40)), int(rng.integers(4, 30)), int(rng.integers(3, 65))
    vl = 1 + seed % 3  # vlimit 1, 2, 3 in turn
    m = synth.make_mesh(nx, ny, nl, seed=seed, full_depth=bool(seed % 2))
    tracers = synth.make_tracer_fields(m, 2)
    check_pass(m, run_split(m, tracers[0], vlimit=vl), O.full_pass(m, tracers[0], vlimit=vl))
    dm = engine.DeviceMesh(m)
    e = engine.FctAleBatch(dm, tracers, vlimit=vl)
    try:
        assert e.split_pass() == 9, abi.last_error()
        e.sync()
        got = {k: e.download(k).reshape(2, -1) for k in ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")}
    finally:
        e.free()
        dm.free()
    for t in range(2):
        check_pass(m, {k: v[t] for k, v in got.items()}, O.full_pass(m, tracers[t], vlimit=vl))


@pytest.mark.parametrize("nl,full", [(129, True), (129, False), (200, True), (200, False)])
def test_deep_columns_split_pass(nl, full, monkeypatch):
    """Deep columns (L = 128, 199): blocks of up to 832 threads, the LDS stencil and the internal-edge
    tail at that depth, odd and even L; the split pass with and without block-internal edges."""
    m = synth.make_mesh(24, 10, nl, seed=nl, full_depth=full)
    f = synth.make_fields(m)
    want = O.full_pass(m, f)
    for internal in ("0", "1"):
        monkeypatch.setenv("FESOM2_P1V_B3H", internal)  # a plan option: read when run_split builds the plan
        check_pass(m, run_split(m, f), want)
