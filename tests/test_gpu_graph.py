"""GPU: hipGraph capture and replay of the entry points (fesom2_graph_begin_/end_/launch_/free_).

What a replay must keep from the eager calls, each checked against the oracle:
* the waits for the producers' upload events (transfer_var_async_ with record_event, reference
  src/fesom2-accelerate.cu:293/:316/:326): a captured stream may not wait on an event recorded
  outside the capture, so the library records the waits and issues them before every replay --
  the uploads here run on a second stream from pinned memory, launched without a host sync;
* the halo exchange inside fct_ale_post_comm_h_acc_ (fork onto the halo plan's stream, pack,
  grouped ncclSend/ncclRecv, unpack, join), twice in one graph with the same plan (two tracers of
  one time step, as FESOM2 calls fct_ale per tracer), on a one-rank communicator exchanging with
  itself into a deranged halo that only the exchange repairs;
* refusal to replay after a handle it captured has been freed, and per-stream capture state.
"""
import ctypes as C

import numpy as np
import pytest

from fesom2_amd import abi, engine, partition, synth
from fesom2_amd.abi import arr, dll, ip

import oracle as O
from test_gpu_halo import download, make_buffer, make_plan
from test_gpu_parity import check_pass

pytestmark = pytest.mark.gpu

OUT = ("plus", "minus", "adf_v", "adf_h", "del_v", "del_h")


@pytest.fixture(scope="module", autouse=True)
def device():
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    abi.set_path("fused")
    yield
    abi.set_resident(False)


@pytest.fixture(scope="module")
def comm():
    uid = (C.c_char * 128)()
    st = C.c_int(0)
    dll().fesom2_comm_unique_id_(uid, C.byref(st))
    abi.check(st, "fesom2_comm_unique_id_")
    h = abi.Handle("comm")
    dll().fesom2_comm_init_(h.ref, uid, ip(0), ip(1), C.byref(st))
    abi.check(st, "fesom2_comm_init_")
    yield h
    dll().fesom2_comm_free_(h.ref)


class Pinned:
    """A pinned host copy of ``a`` (allocate_pinned_doubles_), so H2D copies are truly async."""

    def __init__(self, a):
        self.ptr = C.c_void_p()
        st = C.c_int(0)
        dll().allocate_pinned_doubles_(C.byref(self.ptr), ip(a.size), C.byref(st))
        assert st.value == 0, "pinned allocation fell back to malloc"
        self.a = np.ctypeslib.as_array((C.c_double * a.size).from_address(self.ptr.value))
        self.a[:] = a

    def free(self):
        dll().fesom2_free_pinned_(C.byref(self.ptr))


def test_replay_waits_for_async_uploads():
    """Each replay is preceded by the producers' uploads of ttf / fct_adf_v / fct_adf_h on another
    stream (events recorded); the replay must see the new contents, i.e. wait for those events."""
    m = synth.config_mesh("127k x 47")
    f = synth.make_fields(m)
    want = O.full_pass(m, f)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    up = abi.Stream()
    pins = {k: Pinned(f[k]) for k in ("ttf", "adf_v", "adf_h")}
    g = None
    try:
        assert e.split_pass() == 9  # builds the plans
        e.sync()
        with abi.Graph.capture(e.stream) as g:
            assert e.pre_comm_v() == 7, abi.last_error()
            assert e.post_comm_h() == 9, abi.last_error()
        nuses, nwaits = g.info()
        assert nwaits == 3 and nuses >= 3  # ttf, fct_adf_v, fct_adf_h carry events
        for rep in range(2):
            for k in ("LO", "del_v", "del_h"):
                e.upload(k)  # synchronous
            for k, p in pins.items():  # the producer's uploads, async on `up`
                dll().transfer_var_async_(e.h[k].ref, C.cast(p.ptr, C.POINTER(C.c_double)), up.ref,
                                          abi.bp(True))
            g.launch(e.stream)  # no host synchronisation in between
            e.sync()
            up.sync()
            check_pass(m, {k: e.download(k) for k in OUT}, want)
    finally:
        if g is not None:
            g.free()
        up.sync()
        for p in pins.values():
            p.free()
        up.free()
        e.free()
        dm.free()


@pytest.mark.parametrize("internal", ["0", "1"])
def test_replay_with_halo_exchange_two_tracers(comm, internal, monkeypatch):
    """Two tracers of a partitioned mesh in ONE graph, each pre_comm_v -> post_comm_h(comm, plan) with
    the same halo plan (its stream and events reused twice in the capture).  Halo plus/minus are
    uploaded deranged before each replay; owned results must equal the single-domain oracle."""
    monkeypatch.setenv("FESOM2_P1V_B3H", internal)  # block-internal edges limited in p1v, or all in b3h
    nx, ny, nl, nranks, ntr = 64, 48, 21, 2, 2
    gm = synth.make_mesh(nx, ny, nl)
    gfields = synth.make_tracer_fields(gm, ntr)
    wants = [O.full_pass(gm, f) for f in gfields]
    part = partition.strip_parts(nx, ny, nranks)
    locs = [partition.local_mesh(gm, part, r) for r in range(nranks)]
    parts, plans, graphs = [], [], []
    try:
        for m, _ in locs:
            dm = engine.DeviceMesh(m)
            dm.prepare()  # both mesh plans (phase 1 and phase 2) before any capture
            s = abi.Stream()
            es = [engine.FctAle(dm, f, stream=s) for f in synth.make_tracer_fields(m, ntr)]
            parts.append((dm, s, es))
        # eager phase 1 for the owned plus/minus the exchange has to deliver (and the plans)
        pm = []
        for dm, s, es in parts:
            vals = []
            for e in es:
                assert e.pre_comm_v() == 7, abi.last_error()
            s.sync()
            for e in es:
                vals.append([e.download("plus").reshape(-1, gm.L), e.download("minus").reshape(-1, gm.L)])
            pm.append(vals)
        stored = []
        for r, (m, h) in enumerate(locs):
            for q in h.neighbors:
                src, dst = locs[q][1].send[r] - 1, h.recv[q] - 1
                for k in range(ntr):
                    for a in range(2):
                        pm[r][k][a][dst] = pm[q][k][a][src]
            cols = np.arange(m.N, m.N + m.H)
            nxt = np.roll(cols, -1)
            per_tr = []
            for k in range(ntr):
                pair = []
                for a in range(2):
                    x = pm[r][k][a].copy()
                    x[cols] = pm[r][k][a][nxt]  # c_j holds the value of c_{j+1}
                    pair.append(x.reshape(-1))
                per_tr.append(pair)
            stored.append(per_tr)
            plan, st = make_plan([0], [cols + 1], [nxt + 1], gm.nl)
            assert st == 0
            plans.append(plan)

        def reset(r):
            _, s, es = parts[r]
            for k, e in enumerate(es):
                for name in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
                    e.upload(name)
                e.upload("plus", stored[r][k][0])
                e.upload("minus", stored[r][k][1])

        for r, (dm, s, es) in enumerate(parts):
            reset(r)
            with abi.Graph.capture(s) as g:
                for e in es:
                    assert e.pre_comm_v() == 7, abi.last_error()
                    assert e.post_comm_h(comm, plans[r]) == 9, abi.last_error()
            graphs.append(g)
        outs = []
        for rep in range(2):
            if rep:
                for r in range(nranks):
                    reset(r)
            for (dm, s, es), g in zip(parts, graphs):
                g.launch(s)
            for dm, s, es in parts:
                s.sync()
            outs.append([[{k: e.download(k) for k in OUT} for e in es] for _, _, es in parts])
    finally:
        for g in graphs:
            g.free()
        for plan in plans:
            dll().fesom2_halo_plan_free_(plan.ref)
        for dm, s, es in parts:
            for e in es:
                e.free()
            s.free()
            dm.free()
    ms = [m for m, _ in locs]
    for out in outs:
        for k in range(ntr):
            want = wants[k]
            for r, (m, _) in enumerate(locs):  # the exchange restored the true halo
                assert np.array_equal(out[r][k]["plus"].reshape(-1, gm.L)[m.N:], pm[r][k][0][m.N:])
                got_h = out[r][k]["adf_h"].reshape(m.E, gm.L)
                assert np.array_equal(got_h, want["adf_h"].reshape(gm.E, gm.L)[m.edge_gid]), f"adf_h rank {r}"
            for name in ("del_v", "del_h"):
                got = partition.gather_owned(ms, lambda r: out[r][k][name], gm.L, gm.N)
                assert np.array_equal(got, want[name]), (name, k)
            got = partition.gather_owned(ms, lambda r: out[r][k]["adf_v"], gm.nl, gm.N)
            assert np.array_equal(got, want["adf_v"]), ("adf_v", k)


def test_launch_refuses_freed_handles(comm):
    """A graph over an RCCL self-exchange replays; once its halo plan or a buffer is freed it refuses."""
    L, ncol = 10, 12
    plus = np.arange(ncol * L, dtype=np.float64)
    for victim in ("plan", "buffer"):
        bp_, bm_ = make_buffer(plus), make_buffer(-plus)
        plan, st = make_plan([0], [[1, 2]], [[11, 12]], L + 1)
        assert st == 0
        s = abi.Stream()
        g = None
        try:
            with abi.Graph.capture(s) as g:
                ist = C.c_int(-1)
                dll().fct_ale_exchange_acc_(C.byref(ist), s.ref, comm.ref, plan.ref, bp_.ref, bm_.ref)
                assert ist.value == 0, abi.last_error()
            g.launch(s)
            s.sync()
            got = download(bp_, plus.size).reshape(ncol, L)
            assert np.array_equal(got[10:], plus.reshape(ncol, L)[:2])
            if victim == "plan":
                dll().fesom2_halo_plan_free_(plan.ref)
            else:
                dll().fesom2_free_(bm_.ref)
            st = C.c_int(0)
            dll().fesom2_graph_launch_(C.byref(st), g.ref, s.ref)
            assert st.value == 1 and "freed" in abi.last_error()
        finally:
            if g is not None:
                g.free()
            if plan:
                dll().fesom2_halo_plan_free_(plan.ref)
            for b in (bp_, bm_):
                if b:
                    dll().fesom2_free_(b.ref)
            s.free()


def test_capture_state_is_per_stream():
    """end on a stream that is not being captured fails; a second begin on the same thread fails
    without disturbing the first; an eager pass on another stream during an open capture runs (with
    its event waits) and matches the oracle; the capture then ends cleanly."""
    m = synth.config_mesh("8k x 20")
    f = synth.make_fields(m)
    want = O.full_pass(m, f)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    other = abi.Stream()
    try:
        assert e.split_pass() == 9
        e.sync()
        for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
            e.upload(k)
        st, g = C.c_int(0), abi.Graph()
        dll().fesom2_graph_end_(C.byref(st), other.ref, g.ref)
        assert st.value == 1 and not g
        dll().fesom2_graph_begin_(C.byref(st), other.ref)
        assert st.value == 0, abi.last_error()
        dll().fesom2_graph_begin_(C.byref(st), e.stream.ref)  # one open capture per thread
        assert st.value == 1
        assert e.split_pass() == 9, abi.last_error()  # eager, on e.stream (not captured)
        e.sync()
        # (downloads copy on the null stream, which would break the open capture: end it first)
        dll().fesom2_graph_end_(C.byref(st), other.ref, g.ref)
        assert st.value == 0, abi.last_error()
        check_pass(m, {k: e.download(k) for k in OUT}, want)
        g.launch(other)  # the empty graph
        other.sync()
        g.free()
    finally:
        e.free()
        dm.free()
        other.free()


def _split_outputs(e):
    return {k: e.download(k) for k in OUT}


def _reupload(e):
    for k in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h"):
        e.upload(k)


@pytest.mark.parametrize("captured", ["pre_comm_v", "post_comm_h"])
def test_half_pass_graph_with_eager_other_half(captured, monkeypatch):
    """fct_adf_h's internal-edge mark (host state) follows the replays: a graph holding only
    pre_comm_v leaves fct_adf_h marked after each launch, so an eager post_comm_h skips the edges p1v
    limited; a graph holding only post_comm_h checks before each launch that an eager pre_comm_v
    marked it (and refuses to run otherwise).  Three steps each, exact every time."""
    monkeypatch.setenv("FESOM2_P1V_B3H", "1")
    m = synth.config_mesh("8k x 20")
    f = synth.make_fields(m)
    want = O.full_pass(m, f)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    g = None
    try:
        assert dm.info()["internal_edges"] > 0
        assert e.split_pass() == 9, abi.last_error()  # plans
        _reupload(e)
        e.sync()
        if captured == "pre_comm_v":
            with abi.Graph.capture(e.stream) as g:
                assert e.pre_comm_v() == 7, abi.last_error()
            for _ in range(3):
                _reupload(e)
                g.launch(e.stream)
                assert e.post_comm_h() == 9, abi.last_error()
                e.sync()
                check_pass(m, _split_outputs(e), want)
        else:
            assert e.pre_comm_v() == 7, abi.last_error()  # marks fct_adf_h
            with abi.Graph.capture(e.stream) as g:
                assert e.post_comm_h() == 9, abi.last_error()
            e.sync()
            for step in range(3):
                if step:
                    _reupload(e)
                    assert e.pre_comm_v() == 7, abi.last_error()
                g.launch(e.stream)
                e.sync()
                check_pass(m, _split_outputs(e), want)
            # the mark was consumed by the last replay: another replay without pre_comm_v is refused
            with pytest.raises(abi.HipError, match="fct_adf_h"):
                g.launch(e.stream)
    finally:
        if g is not None:
            g.free()
        e.free()
        dm.free()


def test_graph_end_on_another_thread_does_not_block_plan_builds():
    """fesom2_graph_end_ from a thread other than the one that began the capture fails, but ends
    the HIP capture and unregisters it: later plan builds (which refuse to run while any capture is
    open) still work, and the opening thread can capture again."""
    import threading
    m = synth.config_mesh("tiny")
    f = synth.make_fields(m)
    dm = engine.DeviceMesh(m)
    e = engine.FctAle(dm, f)
    try:
        assert e.split_pass() == 9
        e.sync()
        st = C.c_int(0)
        dll().fesom2_graph_begin_(C.byref(st), e.stream.ref)
        assert st.value == 0, abi.last_error()
        result = {}

        def end_elsewhere():
            g = abi.Graph()
            s2 = C.c_int(0)
            dll().fesom2_graph_end_(C.byref(s2), e.stream.ref, g.ref)
            result["st"], result["graph"] = s2.value, bool(g)

        t = threading.Thread(target=end_elsewhere)
        t.start()
        t.join()
        assert result == {"st": 1, "graph": False}
        # a fresh mesh needs a plan build: not blocked by an orphaned capture
        m2 = synth.config_mesh("tiny", full_depth=True)
        dm2 = engine.DeviceMesh(m2)
        e2 = engine.FctAle(dm2, synth.make_fields(m2))
        try:
            assert e2.split_pass() == 9, abi.last_error()
            e2.sync()
        finally:
            e2.free()
            dm2.free()
        # and this thread can open and close a capture again
        with abi.Graph.capture(e.stream) as g:
            assert e.pre_comm_v() == 7
            assert e.post_comm_h() == 9
        g.free()
    finally:
        e.free()
        dm.free()
