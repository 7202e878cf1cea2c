"""GPU: the in-library RCCL halo exchange (fct_ale_exchange_acc_).

RCCL refuses two ranks on one device, so a one-GPU box cannot run the multi-rank exchange; here a
one-rank communicator exchanges with itself (grouped ncclSend/ncclRecv to rank 0 are legal), which
runs the whole pack -> send/recv -> unpack path with several neighbour slots and their buffer
offsets.  The multi-rank data flow itself (lists, ordering, equality with the single-domain pass) is
covered on the CPU by tests/test_partition.py (gloo, world_size 2) and on the GPU by
test_gpu_parity.py::test_partitioned_pass_on_one_gpu; bench.py --check verifies N > 1 runs.
"""
import ctypes as C

import numpy as np
import pytest

from fesom2_amd import abi
from fesom2_amd.abi import arr, dll, ip

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    abi.set_mpi_rank(0, 1)
    uid = (C.c_char * 128)()
    st = C.c_int(0)
    dll().fesom2_comm_unique_id_(uid, C.byref(st))
    abi.check(st, "fesom2_comm_unique_id_")
    h = abi.Handle("comm")
    dll().fesom2_comm_init_(h.ref, uid, ip(0), ip(1), C.byref(st))
    abi.check(st, "fesom2_comm_init_")
    yield h
    dll().fesom2_comm_free_(h.ref)


def make_buffer(values):
    h = abi.Handle("buf")
    st = C.c_int(0)
    dll().alloc_var_(h.ref, None, ip(values.size), abi.bp(False), C.byref(st))
    abi.check(st, "alloc_var_")
    dll().fesom2_upload_(h.ref, arr(values), C.byref(st))
    abi.check(st, "upload")
    return h


def download(h, n):
    out = np.empty(n)
    st = C.c_int(0)
    dll().fesom2_download_(h.ref, arr(out), C.byref(st))
    abi.check(st, "download")
    return out


def make_plan(ranks, send, recv, nl):
    h = abi.Handle("plan")
    st = C.c_int(0)
    sc = np.array([len(s) for s in send], np.int32)
    rc = np.array([len(r) for r in recv], np.int32)
    sn = np.ascontiguousarray(np.concatenate(send).astype(np.int32))
    rn = np.ascontiguousarray(np.concatenate(recv).astype(np.int32))
    dll().fesom2_halo_plan_(h.ref, ip(len(ranks)), arr(np.array(ranks, np.int32)), arr(sc), arr(sn), arr(rc),
                            arr(rn), ip(nl), C.byref(st))
    return h, st.value


def test_self_exchange_moves_columns(comm):
    L, ncol = 20, 40
    z = np.arange(L)
    plus = (np.arange(ncol)[:, None] * 1000.0 + z[None, :]).reshape(-1)
    minus = -plus - 0.5
    bp, bm = make_buffer(plus), make_buffer(minus)
    # two neighbour slots (both rank 0): columns (1-based) 1,2,3 -> 30,31,32 and 5,6 -> 38,39
    plan, st = make_plan([0, 0], [[1, 2, 3], [5, 6]], [[30, 31, 32], [38, 39]], L + 1)
    assert st == 0
    s = abi.Stream()
    try:
        ist = C.c_int(-1)
        dll().fct_ale_exchange_acc_(C.byref(ist), s.ref, comm.ref, plan.ref, bp.ref, bm.ref)
        assert ist.value == 0, abi.last_error()
        s.sync()
        gp = download(bp, plus.size).reshape(ncol, L)
        gm = download(bm, minus.size).reshape(ncol, L)
        want_p = plus.reshape(ncol, L).copy()
        want_m = minus.reshape(ncol, L).copy()
        for src, dst in ((0, 29), (1, 30), (2, 31), (4, 37), (5, 38)):
            want_p[dst] = want_p[src]
            want_m[dst] = want_m[src]
        assert np.array_equal(gp, want_p)
        assert np.array_equal(gm, want_m)
    finally:
        dll().fesom2_halo_plan_free_(plan.ref)
        dll().fesom2_free_(bp.ref)
        dll().fesom2_free_(bm.ref)
        s.free()


def test_exchange_rejects_out_of_range_columns(comm):
    L = 10
    bp, bm = make_buffer(np.zeros(5 * L)), make_buffer(np.zeros(5 * L))
    plan, st = make_plan([0], [[1]], [[9]], L + 1)  # column 9 does not exist in a 5-column buffer
    assert st == 0
    s = abi.Stream()
    try:
        ist = C.c_int(-1)
        dll().fct_ale_exchange_acc_(C.byref(ist), s.ref, comm.ref, plan.ref, bp.ref, bm.ref)
        assert ist.value == 1
        assert "holds" in abi.last_error()
    finally:
        dll().fesom2_halo_plan_free_(plan.ref)
        dll().fesom2_free_(bp.ref)
        dll().fesom2_free_(bm.ref)
        s.free()


def test_plan_rejects_bad_node_numbers():
    plan, st = make_plan([0], [[0]], [[1]], 11)  # node numbers are 1-based
    assert st == 1 and not plan


@pytest.mark.parametrize("kind", ["strips", "random"])
def test_overlapped_exchange_post_comm_c(comm, kind):
    """fct_ale_exchange_post_comm_c_acc_: exchange on the plan's stream, interior b3h + node kernel
    meanwhile, boundary part after the exchange event.  Each partition's halo columns are uploaded
    deranged (column c_j holds the true value of c_{j+1}); the one-rank plan sends c_j and receives
    into c_{j+1}, so the halo is only right once the exchange has landed -- boundary work that ran
    early would read wrong values.  Owned results must equal the single-domain oracle exactly."""
    import oracle as O
    from fesom2_amd import engine, partition, synth
    abi.set_resident(True)
    abi.set_path("fused")
    nx, ny, nl, nranks = 64, 48, 21, 2
    g = synth.make_mesh(nx, ny, nl)
    want = O.full_pass(g, synth.make_fields(g))
    part = (partition.strip_parts(nx, ny, nranks) if kind == "strips"
            else np.random.default_rng(5).integers(0, nranks, g.N).astype(np.int32))
    locs = [partition.local_mesh(g, part, r) for r in range(nranks)]
    runs, plans, outs = [], [], []
    try:
        for m, _ in locs:
            dm = engine.DeviceMesh(m)
            runs.append((dm, engine.FctAle(dm, synth.make_fields(m))))
        pm = []
        for _, e in runs:
            assert e.pre_comm() == 6
            e.sync()
            pm.append([e.download("plus").reshape(-1, g.L), e.download("minus").reshape(-1, g.L)])
        for r, (m, h) in enumerate(locs):
            for q in h.neighbors:  # the values the exchange must deliver
                src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
                for a in range(2):
                    pm[r][a][dst] = pm[q][a][src]
            cols = np.arange(m.N, m.N + m.H)
            assert cols.size > 1
            nxt = np.roll(cols, -1)
            for a, name in enumerate(("plus", "minus")):
                stored = pm[r][a].copy()
                stored[cols] = pm[r][a][nxt]  # c_j holds the value of c_{j+1}
                runs[r][1].upload(name, stored.reshape(-1))
            plan, st = make_plan([0], [cols + 1], [nxt + 1], g.nl)
            assert st == 0
            plans.append(plan)
        for (_, e), plan in zip(runs, plans):
            assert e.exchange_post_comm_c(comm, plan) == 9, abi.last_error()
        for _, e in runs:
            e.sync()
            outs.append({k: e.download(k) for k in ("del_v", "del_h", "adf_v", "plus")})
    finally:
        for plan in plans:
            dll().fesom2_halo_plan_free_(plan.ref)
        for dm, e in runs:
            e.free()
            dm.free()
    ms = [m for m, _ in locs]
    for r, (m, _) in enumerate(locs):  # the exchange restored the true halo
        assert np.array_equal(outs[r]["plus"].reshape(-1, g.L)[m.N:], pm[r][0][m.N:])
    for k in ("del_v", "del_h"):
        assert np.array_equal(partition.gather_owned(ms, lambda r: outs[r][k], g.L, g.N), want[k]), k
    assert np.array_equal(partition.gather_owned(ms, lambda r: outs[r]["adf_v"], g.nl, g.N), want["adf_v"])


@pytest.mark.parametrize("two", [False, True])
@pytest.mark.parametrize("ntr", [1, 3])
def test_exchange_nod_generic_fields(comm, two, ntr):
    """fesom2_exchange_nod_acc_: FESOM's exchange_nod for one or two (nl-1, nod) fields of ntr
    tracer blocks (ttf/LO before phase 1, del_ttf after c)."""
    L, ncol = 12, 30
    rng = np.random.default_rng(ntr + 10 * two)
    fa, fb = rng.standard_normal(ntr * ncol * L), rng.standard_normal(ntr * ncol * L)
    ha, hb = make_buffer(fa), make_buffer(fb)
    plan, st = make_plan([0], [[2, 4, 6]], [[28, 29, 30]], L + 1)
    assert st == 0
    s = abi.Stream()
    null = abi.Handle("none")
    try:
        ist = C.c_int(-1)
        dll().fesom2_exchange_nod_acc_(C.byref(ist), s.ref, comm.ref, plan.ref, ip(ntr), ip(ncol), ha.ref,
                                       hb.ref if two else null.ref)
        assert ist.value == 0, abi.last_error()
        s.sync()
        for h, f0, moved in ((ha, fa, True), (hb, fb, two)):
            got = download(h, f0.size).reshape(ntr, ncol, L)
            want = f0.reshape(ntr, ncol, L).copy()
            if moved:
                want[:, [27, 28, 29]] = want[:, [1, 3, 5]]
            assert np.array_equal(got, want)
    finally:
        dll().fesom2_halo_plan_free_(plan.ref)
        dll().fesom2_free_(ha.ref)
        dll().fesom2_free_(hb.ref)
        s.free()
