"""Host driver: issues the C-ABI calls in the order FESOM2's Fortran ``fct_ale`` does.

Also the in-library halo (:class:`Halo`): RCCL communicator + halo plan from partition lists.

Call sequence (reference ``src/fesom2-accelerate.cu``)::

    transfer_mesh_ x7                      once per mesh      (:114-127)
    alloc_var_ / reserve_var_              once per field     (:129-141)
    transfer_var_async_(ttf, adf_v, adf_h) per step, events   (:163-168, waited on at :293/:316/:326)
    fct_ale_pre_comm_acc_                  a1..b2             (:258-340)
    [exchange_nod(fct_plus, fct_minus)]    host MPI, or fct_ale_exchange_acc_ (RCCL) here
    fct_ale_inter_comm_acc_                b3-vertical        (:342-356)
    fct_ale_post_comm_acc_                 b3-horizontal      (:358-379)
    fct_ale_c_acc_                         c-step (new; the reference leaves it to Fortran)

or, fused: ``fct_ale_pre_comm_acc_`` -> exchange -> ``fct_ale_post_comm_c_acc_``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .abi import arr, bp, check, dll, dp, ip

MESH_ARRAYS = ("nlev_nod", "nlev_elem", "elem2D_nodes", "nie_num", "nie", "edges", "edge_tri")
NODE_FIELDS = ("ttf", "LO", "hnode", "hnode_new", "del_v", "del_h", "plus", "minus")
NL_FIELDS = ("adf_v", "area", "area_inv")


class DeviceMesh:
    """Mesh connectivity uploaded with ``transfer_mesh_`` (int32, 1-based)."""

    def __init__(self, m):
        self.m = m
        self.h = {}
        self._host = {}
        for name in MESH_ARRAYS:
            a = np.ascontiguousarray(getattr(m, name), dtype=np.int32)
            self._host[name] = a  # the library keeps the host pointer, like Fortran's arrays
            h = abi.Handle(name)
            st = C.c_int(0)
            dll().transfer_mesh_(h.ref, arr(a), ip(max(a.size, 1)), C.byref(st))
            check(st, f"transfer_mesh_({name})")
            self.h[name] = h

    def prepare(self):
        m, h = self.m, self.h
        st = C.c_int(0)
        dll().fesom2_prepare_mesh_(C.byref(st), ip(m.N), ip(m.H), ip(m.T), ip(m.E), ip(m.nl), h["nlev_nod"].ref,
                                   h["nlev_elem"].ref, h["elem2D_nodes"].ref, h["nie_num"].ref, h["nie"].ref,
                                   ip(m.dim), h["edges"].ref, h["edge_tri"].ref)
        check(st, "fesom2_prepare_mesh_")

    def info(self, batched=False):
        """fesom2_mesh_info_: p1v block columns, interior edges, those crossing p1v blocks, the
        block-internal ones (limited inside p1v) and their edge cells -- of the single-tracer plan,
        or with ``batched`` of the plan calls with ntracers > 1 run on."""
        m, h = self.m, self.h
        st, n = C.c_int(0), C.c_int(14)
        out = (C.c_longlong * 14)()
        dll().fesom2_mesh_info_(C.byref(st), ip(m.N), ip(m.H), ip(m.T), ip(m.E), ip(m.nl), h["nlev_nod"].ref,
                                h["nlev_elem"].ref, h["elem2D_nodes"].ref, h["nie_num"].ref, h["nie"].ref,
                                ip(m.dim), h["edges"].ref, h["edge_tri"].ref, out, C.byref(n))
        check(st, "fesom2_mesh_info_")
        keys = ("p1v_columns", "interior_edges", "crossing_edges", "internal_edges", "internal_edge_cells")
        vals = list(out)[: n.value]
        d = dict(zip(keys, vals[5:10] if batched else vals[:5]))
        if n.value >= 14:  # the cluster unions (0 columns: none)
            d["union_columns"], d["union_max"] = vals[12:14] if batched else vals[10:12]
        return d

    def pass_order(self, ntracers=1):
        """fesom2_pass_order_: the Infinity-Cache pass order of a call of ``ntracers`` tracers
        (bits 1 / 4: phase 1 / the c-step's node kernel backwards, 8: b3h's flux stores
        cache-allocating; 0: off)."""
        m, h = self.m, self.h
        st, order = C.c_int(0), C.c_int(0)
        dll().fesom2_pass_order_(C.byref(st), ip(m.N), ip(m.H), ip(m.E), ip(m.nl), h["nlev_nod"].ref,
                                 h["nlev_elem"].ref, h["edges"].ref, h["edge_tri"].ref, ip(ntracers),
                                 C.byref(order))
        check(st, "fesom2_pass_order_")
        return order.value

    def free(self):
        for h in self.h.values():
            if h:
                dll().fesom2_free_(h.ref)
        self.h = {}


class FctAle:
    """Device state of one tracer on one (local) mesh, driven through the C-ABI.

    ``fields`` is the dict made by :func:`fesom2_amd.synth.make_fields` (host arrays, kept alive
    and bound as the handles' host pointers exactly like the Fortran arrays would be).
    """

    ntr = 1  # tracers per call (FctAleBatch: several)

    def __init__(self, dmesh: DeviceMesh, fields, stream=None, vlimit=1, flux_eps=1e-16, bignumber=1e3,
                 dt=1.0, copy=True):
        m = dmesh.m
        self.dm, self.m = dmesh, m
        self.stream = stream or abi.Stream()
        self.vlimit, self.eps, self.big, self.dt = vlimit, flux_eps, bignumber, dt
        NT, L, nl = m.N + m.H, m.L, m.nl
        # copy=False binds the caller's arrays (large meshes: no second host copy)
        self.host = {k: (np.array(v, dtype=np.float64) if copy else np.ascontiguousarray(v, dtype=np.float64))
                     for k, v in fields.items()}
        self.host.setdefault("plus", np.zeros(NT * L))
        self.host.setdefault("minus", np.zeros(NT * L))
        self.h = {}
        sizes = {k: NT * L for k in NODE_FIELDS}
        sizes.update({k: NT * nl for k in NL_FIELDS})
        sizes["adf_h"] = m.E * L
        events = {"ttf", "adf_v", "adf_h"}  # the buffers the reference waits on (:293, :316, :326)
        for name, n in sizes.items():
            a = self.host[name]
            assert a.size == n, (name, a.size, n)
            h = abi.Handle(name)
            check(abi.alloc_var(h, a, name in events), f"alloc_var_({name})")
            self.h[name] = h
            dll().transfer_var_(h.ref, arr(a))
        for name, n in (("ttf_max", NT * L), ("ttf_min", NT * L), ("UV_rhs", 2 * L * m.T)):
            h = abi.Handle(name)
            check(abi.reserve_var(h, n), f"reserve_var_({name})")
            self.h[name] = h

    # ------------------------------------------------------------------ phases (reference names)
    def pre_comm(self):
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_pre_comm_acc_(
            C.byref(st), self.stream.ref, h["ttf_max"].ref, h["ttf_min"].ref, h["plus"].ref, h["minus"].ref,
            h["ttf"].ref, h["LO"].ref, h["adf_v"].ref, h["adf_h"].ref, h["UV_rhs"].ref, h["area_inv"].ref,
            ip(m.N), ip(m.H), ip(m.T), ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref,
            d["elem2D_nodes"].ref, d["nie_num"].ref, d["nie"].ref, ip(m.dim), d["edges"].ref, d["edge_tri"].ref,
            ip(self.vlimit), dp(self.eps), dp(self.big), dp(self.dt))
        return st.value

    def inter_comm(self):
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_inter_comm_acc_(C.byref(st), self.stream.ref, h["plus"].ref, h["minus"].ref, h["adf_v"].ref,
                                      ip(m.N), ip(m.nl), d["nlev_nod"].ref)
        return st.value

    def post_comm(self):
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_post_comm_acc_(C.byref(st), self.stream.ref, h["plus"].ref, h["minus"].ref, h["adf_h"].ref,
                                     ip(m.E), ip(m.nl), d["nlev_elem"].ref, ip(m.dim), d["edges"].ref,
                                     d["edge_tri"].ref)
        return st.value

    def c_step(self):
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_c_acc_(C.byref(st), self.stream.ref, h["del_v"].ref, h["del_h"].ref, h["ttf"].ref, h["LO"].ref,
                             h["hnode"].ref, h["hnode_new"].ref, h["adf_v"].ref, h["adf_h"].ref, h["area"].ref,
                             ip(m.N), ip(m.H), ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref,
                             d["edges"].ref, d["edge_tri"].ref, dp(self.dt))
        return st.value

    def bind_c_vertical(self, on=True):
        """fesom2_bind_c_vertical_: in the fast mode (fesom2_set_path_(2)) pre_comm also does
        c-vertical on this tracer's del_ttf_advvert, and c_step only c-horizontal."""
        h, st, none = self.h, C.c_int(0), C.c_void_p()
        refs = [h[k].ref if on else C.byref(none) for k in ("del_v", "hnode", "hnode_new", "area")]
        dll().fesom2_bind_c_vertical_(C.byref(st), h["adf_v"].ref, *refs)
        check(st, "fesom2_bind_c_vertical_")

    def post_comm_c(self):
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_post_comm_c_acc_(
            C.byref(st), self.stream.ref, h["plus"].ref, h["minus"].ref, h["adf_v"].ref, h["adf_h"].ref,
            h["del_v"].ref, h["del_h"].ref, h["ttf"].ref, h["LO"].ref, h["hnode"].ref, h["hnode_new"].ref,
            h["area"].ref, ip(m.N), ip(m.H), ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref,
            d["edges"].ref, d["edge_tri"].ref, dp(self.dt))
        return st.value

    # ------------------------------------------------------------------ split by direction
    def pre_comm_v(self):
        """fct_ale_pre_comm_v_acc_: a1..b2 + b3v + cv (alg_state 7)."""
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_pre_comm_v_acc_(
            C.byref(st), self.stream.ref, ip(self.ntr), h["plus"].ref, h["minus"].ref, h["ttf"].ref, h["LO"].ref,
            h["adf_v"].ref, h["adf_h"].ref, h["area_inv"].ref, h["area"].ref, h["hnode"].ref, h["hnode_new"].ref,
            h["del_v"].ref, ip(m.N), ip(m.H), ip(m.T), ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref,
            d["elem2D_nodes"].ref, d["nie_num"].ref, d["nie"].ref, ip(m.dim), d["edges"].ref, d["edge_tri"].ref,
            ip(self.vlimit), dp(self.eps), dp(self.big), dp(self.dt))
        return st.value

    def post_comm_h(self, comm=None, plan=None):
        """fct_ale_post_comm_h_acc_: [exchange overlapped with the interior] + b3h + ch (alg_state 9)."""
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        none = C.c_void_p()
        dll().fct_ale_post_comm_h_acc_(
            C.byref(st), self.stream.ref, ip(self.ntr), comm.ref if comm else C.byref(none),
            plan.ref if plan else C.byref(none), h["plus"].ref, h["minus"].ref, h["adf_h"].ref, h["del_h"].ref,
            h["area"].ref, ip(m.N), ip(m.H), ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref,
            d["edges"].ref, d["edge_tri"].ref, dp(self.dt))
        return st.value

    def split_pass(self):
        """Single-domain pass through the direction-split entries (final alg_state, 9 on success)."""
        s1 = self.pre_comm_v()
        return self.post_comm_h() if s1 == 7 else s1

    def _iter_buffers(self):
        """fct_adf_v2 / fct_adf_h2 (zero-initialised, as FESOM allocates them) on first use."""
        for name, like in (("adf_v2", "adf_v"), ("adf_h2", "adf_h")):
            if name not in self.h:
                a = np.zeros_like(self.host[like])
                self.host[name] = a
                h = abi.Handle(name)
                check(abi.alloc_var(h, a), f"alloc_var_({name})")
                dll().transfer_var_(h.ref, arr(a))
                self.h[name] = h

    def post_comm_iter(self):
        """iter_yn phase 2 (fct_ale_post_comm_iter_acc_): LO updated, adf <- remainders."""
        self._iter_buffers()
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_post_comm_iter_acc_(
            C.byref(st), self.stream.ref, h["plus"].ref, h["minus"].ref, h["adf_v"].ref, h["adf_h"].ref,
            h["adf_v2"].ref, h["adf_h2"].ref, h["LO"].ref, h["hnode_new"].ref, h["area"].ref, ip(m.N), ip(m.H),
            ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref, d["edges"].ref, d["edge_tri"].ref,
            dp(self.dt))
        return st.value

    def iterated_pass(self, iterations, final="split"):
        """``iterations - 1`` iter_yn rounds then the final pass (final alg_state): the
        direction-split entries (``final="split"``, the fastest) or the fused pre_comm -> post_comm_c
        pair (``"fused"``).  The rounds hand over the LO update and the remainder fluxes only, so the
        final pass is an ordinary one on them."""
        for _ in range(iterations - 1):
            s1 = self.pre_comm()
            if s1 != 6:
                return s1
            s2 = self.post_comm_iter()
            if s2 != 9:
                return s2
        return self.split_pass() if final == "split" else self.full_pass()

    def exchange(self, comm, plan):
        """fct_ale_exchange_acc_: RCCL halo exchange of fct_plus/fct_minus on this stream."""
        st = C.c_int(-1)
        dll().fct_ale_exchange_acc_(C.byref(st), self.stream.ref, comm.ref, plan.ref, self.h["plus"].ref,
                                    self.h["minus"].ref)
        check(st, "fct_ale_exchange_acc_")

    def exchange_post_comm_c(self, comm, plan):
        """Exchange overlapped with the interior of the fused phase 2 (alg_state 9 on success)."""
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_exchange_post_comm_c_acc_(
            C.byref(st), self.stream.ref, comm.ref, plan.ref, h["plus"].ref, h["minus"].ref, h["adf_v"].ref,
            h["adf_h"].ref, h["del_v"].ref, h["del_h"].ref, h["ttf"].ref, h["LO"].ref, h["hnode"].ref,
            h["hnode_new"].ref, h["area"].ref, ip(m.N), ip(m.H), ip(m.E), ip(m.nl), d["nlev_nod"].ref,
            d["nlev_elem"].ref, d["edges"].ref, d["edge_tri"].ref, dp(self.dt))
        return st.value

    def full_pass(self, fused=True):
        """Single-domain pass (no halo): returns the final alg_state (9 on success)."""
        s1 = self.pre_comm()
        if s1 != 6:
            return s1
        if fused:
            return self.post_comm_c()
        s2 = self.inter_comm()
        s3 = self.post_comm()
        s4 = self.c_step()
        return s4 if (s2, s3) == (7, 8) else min(s2, s3)

    # ------------------------------------------------------------------ data movement
    def upload(self, name, a=None):
        a = self.host[name] if a is None else np.ascontiguousarray(a, dtype=np.float64)
        if a.size < self.size(name):
            raise ValueError(f"upload {name}: {a.size} doubles for a handle of {self.size(name)}")
        st = C.c_int(0)
        dll().fesom2_upload_(self.h[name].ref, arr(a), C.byref(st))
        check(st, f"upload {name}")

    def size(self, name):
        """Doubles the handle of ``name`` holds (its host array's size; kept by drop_host)."""
        sizes = getattr(self, "sizes", {})
        if name in sizes:
            return sizes[name]
        if name in self.host:
            return self.host[name].size
        return {"UV_rhs": 2 * self.m.L * self.m.T}.get(name, (self.m.N + self.m.H) * self.m.L)

    def drop_host(self):
        """Release the host copies of the fields (device-resident runs on large meshes): downloads
        keep working (sizes are kept), uploads then need an explicit array.  The library never reads
        the bound host pointers in resident mode (fesom2_set_resident_(1))."""
        self.sizes = {k: v.size for k, v in self.host.items()}
        self.host = {}

    def download(self, name, dtype=np.float64, out=None):
        """The handle's contents; into ``out`` (float64, contiguous, at least max(n, 1) doubles:
        e.g. a memory-mapped file) when given."""
        b = self.h[name]
        n = self.size(name)
        if out is None:
            out = np.empty(max(n, 1), dtype)  # every handle here holds exactly max(n, 1) doubles
        elif out.dtype != np.float64 or not out.flags.c_contiguous or out.size < max(n, 1):
            raise ValueError(f"download {name}: output buffer does not fit {max(n, 1)} doubles")
        st = C.c_int(0)
        dll().fesom2_download_(b.ref, arr(out), C.byref(st))
        check(st, f"download {name}")
        return out[:n]

    def sync(self):
        self.stream.sync()

    def free(self):
        for h in self.h.values():
            if h:
                dll().fesom2_free_(h.ref)
        self.h = {}


TRACER_FIELDS = ("ttf", "LO", "del_v", "del_h", "plus", "minus", "adf_v", "adf_h")
SHARED_FIELDS = ("area", "area_inv", "hnode", "hnode_new")


class FctAleBatch(FctAle):
    """``ntracers`` tracers on one mesh through the batched entry points
    (``fct_ale_pre_comm_batched_acc_`` / ``fct_ale_post_comm_c_batched_acc_``).

    ``tracers`` is a list of field dicts (:func:`fesom2_amd.synth.make_tracer_fields`); the mesh
    fields (area, area_inv, hnode, hnode_new) are taken from the first.  Per-tracer arrays are
    stacked tracer-slowest, i.e. Fortran ``(nl-1, nod, ntracers)``.
    """

    def __init__(self, dmesh: DeviceMesh, tracers, stream=None, vlimit=1, flux_eps=1e-16, bignumber=1e3, dt=1.0):
        m = dmesh.m
        self.dm, self.m, self.ntr = dmesh, m, len(tracers)
        self.stream = stream or abi.Stream()
        self.vlimit, self.eps, self.big, self.dt = vlimit, flux_eps, bignumber, dt
        NT, L = m.N + m.H, m.L
        self.host = {}
        for k in TRACER_FIELDS:
            parts = [np.asarray(t[k], np.float64) if k in t else np.zeros(NT * L) for t in tracers]
            self.host[k] = np.ascontiguousarray(np.concatenate(parts))
        for k in SHARED_FIELDS:
            self.host[k] = np.ascontiguousarray(tracers[0][k], dtype=np.float64).copy()
        self.h = {}
        events = {"ttf", "adf_v", "adf_h"}
        for name, a in self.host.items():
            h = abi.Handle(name)
            check(abi.alloc_var(h, a, name in events), f"alloc_var_({name})")
            self.h[name] = h
            dll().transfer_var_(h.ref, arr(a))

    def pre_comm(self):
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_pre_comm_batched_acc_(
            C.byref(st), self.stream.ref, ip(self.ntr), h["plus"].ref, h["minus"].ref, h["ttf"].ref, h["LO"].ref,
            h["adf_v"].ref, h["adf_h"].ref, h["area_inv"].ref, ip(m.N), ip(m.H), ip(m.T), ip(m.E), ip(m.nl),
            d["nlev_nod"].ref, d["nlev_elem"].ref, d["elem2D_nodes"].ref, d["nie_num"].ref, d["nie"].ref, ip(m.dim),
            d["edges"].ref, d["edge_tri"].ref, ip(self.vlimit), dp(self.eps), dp(self.big), dp(self.dt))
        return st.value

    def _phase2_args(self):
        m, h, d = self.m, self.h, self.dm.h
        return (h["plus"].ref, h["minus"].ref, h["adf_v"].ref, h["adf_h"].ref, h["del_v"].ref, h["del_h"].ref,
                h["ttf"].ref, h["LO"].ref, h["hnode"].ref, h["hnode_new"].ref, h["area"].ref, ip(m.N), ip(m.H),
                ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref, d["edges"].ref, d["edge_tri"].ref,
                dp(self.dt))

    def post_comm_c(self):
        st = C.c_int(-1)
        dll().fct_ale_post_comm_c_batched_acc_(C.byref(st), self.stream.ref, ip(self.ntr), *self._phase2_args())
        return st.value

    def exchange(self, comm, plan):
        st = C.c_int(-1)
        dll().fct_ale_exchange_batched_acc_(C.byref(st), self.stream.ref, comm.ref, plan.ref, ip(self.ntr),
                                            ip(self.m.N + self.m.H), self.h["plus"].ref, self.h["minus"].ref)
        check(st, "fct_ale_exchange_batched_acc_")

    def exchange_post_comm_c(self, comm, plan):
        st = C.c_int(-1)
        dll().fct_ale_exchange_post_comm_c_batched_acc_(C.byref(st), self.stream.ref, comm.ref, plan.ref,
                                                        ip(self.ntr), *self._phase2_args())
        return st.value

    def full_pass(self, fused=True):
        s1 = self.pre_comm()
        return self.post_comm_c() if s1 == 6 else s1

    def post_comm_iter(self):
        self._iter_buffers()
        m, h, d = self.m, self.h, self.dm.h
        st = C.c_int(-1)
        dll().fct_ale_post_comm_iter_batched_acc_(
            C.byref(st), self.stream.ref, ip(self.ntr), h["plus"].ref, h["minus"].ref, h["adf_v"].ref,
            h["adf_h"].ref, h["adf_v2"].ref, h["adf_h2"].ref, h["LO"].ref, h["hnode_new"].ref, h["area"].ref,
            ip(m.N), ip(m.H), ip(m.E), ip(m.nl), d["nlev_nod"].ref, d["nlev_elem"].ref, d["edges"].ref,
            d["edge_tri"].ref, dp(self.dt))
        return st.value

    def tracer(self, name, k):
        """Tracer k's slice of a downloaded per-tracer field."""
        a = self.download(name)
        n = a.size // self.ntr
        return a[k * n:(k + 1) * n]


class Halo:
    """RCCL communicator and halo plan of one rank (fesom2_comm_* / fesom2_halo_plan_).

    ``lists`` is a :class:`fesom2_amd.partition.Halo` (1-based local node numbers per neighbour);
    ``uid`` the 128-byte ncclUniqueId every rank got from rank 0.
    """

    def __init__(self, uid, rank, nranks, lists, nl):
        st = C.c_int(0)
        self.comm = abi.Handle("comm")
        dll().fesom2_comm_init_(self.comm.ref, uid, ip(rank), ip(nranks), C.byref(st))
        check(st, "fesom2_comm_init_")
        nb = list(lists.neighbors)
        sc = np.array([lists.send[q].size for q in nb], np.int32)
        rc = np.array([lists.recv[q].size for q in nb], np.int32)
        sn = np.ascontiguousarray(np.concatenate([lists.send[q] for q in nb] or [np.zeros(0, np.int32)]).astype(np.int32))
        rn = np.ascontiguousarray(np.concatenate([lists.recv[q] for q in nb] or [np.zeros(0, np.int32)]).astype(np.int32))
        self.plan = abi.Handle("halo")
        dll().fesom2_halo_plan_(self.plan.ref, ip(len(nb)), arr(np.array(nb, np.int32)), arr(sc), arr(sn), arr(rc),
                                arr(rn), ip(nl), C.byref(st))
        check(st, "fesom2_halo_plan_")

    def info(self):
        """The communicator's own view: {"rank", "nranks", "device"} (fesom2_comm_info_)."""
        st, r, n, d = C.c_int(0), C.c_int(-1), C.c_int(-1), C.c_int(-1)
        dll().fesom2_comm_info_(self.comm.ref, C.byref(r), C.byref(n), C.byref(d), C.byref(st))
        check(st, "fesom2_comm_info_")
        return {"rank": r.value, "nranks": n.value, "device": d.value}

    @staticmethod
    def unique_id():
        uid = (C.c_char * 128)()
        st = C.c_int(0)
        dll().fesom2_comm_unique_id_(uid, C.byref(st))
        check(st, "fesom2_comm_unique_id_")
        return uid

    def free(self):
        if self.plan:
            dll().fesom2_halo_plan_free_(self.plan.ref)
        if self.comm:
            dll().fesom2_comm_free_(self.comm.ref)
