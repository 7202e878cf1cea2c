"""ctypes front end of the FCT-ALE oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker.  It wraps:

* ``liboracle.so``  -- the C restatement in ``fct_ale_oracle.c`` (cites reference file:line per
  function), and
* ``_ref/libreference.so`` -- the reference's own ``src/reference.cpp`` built by ``oracle/Makefile``
  (dev container only; absent on a box without ``/root/reference`` unless the prebuilt .so
  travelled with the snapshot).

Arrays are numpy, Fortran layout flattened (see fct_ale_oracle.c header).
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_P = C.c_void_p
_I = C.c_int
_D = C.c_double


def _ptr(a):
    if a is None:
        return None
    assert a.flags.c_contiguous
    return a.ctypes.data_as(_P)


_lib = None
_ref = None


def lib():
    """The restatement (liboracle.so); built by ``make -C oracle`` / ``__graft_entry__.build()``."""
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run make -C oracle)")
        _lib = C.CDLL(path)
        _lib.oracle_pre_comm.restype = _I
        _lib.oracle_full_pass.restype = _I
    return _lib


def ref():
    """reference.cpp compiled from /root/reference (None if not available)."""
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libreference.so")
        if not os.path.exists(path):
            return None
        _ref = C.CDLL(path)
    return _ref


# --------------------------------------------------------------------------- restatement

def a1(n_nodes, nlev_nod, nl, tmax, tmin, LO, ttf):
    lib().oracle_a1(_I(n_nodes), _ptr(nlev_nod), _I(nl), _ptr(tmax), _ptr(tmin), _ptr(LO), _ptr(ttf))


def a2(n_elem, nlev_elem, nl, UV, elem2D_nodes, tmax, tmin, big):
    lib().oracle_a2(_I(n_elem), _ptr(nlev_elem), _I(nl), _ptr(UV), _ptr(elem2D_nodes), _ptr(tmax),
                    _ptr(tmin), _D(big))


def a3(n_nodes, nlev_nod, nl, tmax, tmin, LO, UV, plus, minus, adf_v, nie, nie_num, dim, vlimit=1):
    if vlimit == 1:
        lib().oracle_a3(_I(n_nodes), _ptr(nlev_nod), _I(nl), _ptr(tmax), _ptr(tmin), _ptr(LO), _ptr(UV),
                        _ptr(plus), _ptr(minus), _ptr(adf_v), _ptr(nie), _ptr(nie_num), _I(dim))
    else:
        lib().oracle_a3_vlimit23(_I(vlimit), _I(n_nodes), _ptr(nlev_nod), _I(nl), _ptr(tmax), _ptr(tmin),
                                 _ptr(LO), _ptr(UV), _ptr(plus), _ptr(minus), _ptr(adf_v), _ptr(nie),
                                 _ptr(nie_num), _I(dim))


def a4(n_nodes, nlev_nod, nlev_elem, nl, n_edges, plus, minus, adf_h, area_inv, tmax, tmin, edges,
       edge_tri, eps, dt):
    lib().oracle_a4(_I(n_nodes), _ptr(nlev_nod), _ptr(nlev_elem), _I(nl), _I(n_edges), _ptr(plus),
                    _ptr(minus), _ptr(adf_h), _ptr(area_inv), _ptr(tmax), _ptr(tmin), _ptr(edges),
                    _ptr(edge_tri), _D(eps), _D(dt))


def b3v(n_nodes, nlev_nod, nl, adf_v, plus, minus, adf_v2=None):
    lib().oracle_b3v(_I(n_nodes), _ptr(nlev_nod), _I(nl), _ptr(adf_v), _ptr(plus), _ptr(minus), _ptr(adf_v2))


def b3h(n_edges, nlev_elem, nl, edges, edge_tri, adf_h, plus, minus, adf_h2=None):
    lib().oracle_b3h(_I(n_edges), _ptr(nlev_elem), _I(nl), _ptr(edges), _ptr(edge_tri), _ptr(adf_h),
                     _ptr(plus), _ptr(minus), _ptr(adf_h2))


def cv(n_nodes, nlev_nod, nl, del_v, ttf, hnode, LO, hnode_new, adf_v, dt, area):
    lib().oracle_cv(_I(n_nodes), _ptr(nlev_nod), _I(nl), _ptr(del_v), _ptr(ttf), _ptr(hnode), _ptr(LO),
                    _ptr(hnode_new), _ptr(adf_v), _D(dt), _ptr(area))


def ch(n_edges, nlev_elem, nl, edges, edge_tri, del_h, adf_h, dt, area):
    lib().oracle_ch(_I(n_edges), _ptr(nlev_elem), _I(nl), _ptr(edges), _ptr(edge_tri), _ptr(del_h),
                    _ptr(adf_h), _D(dt), _ptr(area))


def lo_update(n_nodes, nlev_nod, n_edges, nlev_elem, nl, edges, edge_tri, LO, adf_v, adf_h, dt, area,
              hnode_new):
    lib().oracle_lo_update(_I(n_nodes), _ptr(nlev_nod), _I(n_edges), _ptr(nlev_elem), _I(nl),
                           _ptr(edges), _ptr(edge_tri), _ptr(LO), _ptr(adf_v), _ptr(adf_h), _D(dt),
                           _ptr(area), _ptr(hnode_new))


# --------------------------------------------------------------------------- whole phases

def pre_comm(m, f, vlimit=1, vlimit_ext=True, eps=1e-16, big=1e3, dt=1.0):
    """Phase 1 (a1..b2) on copies of the fields; returns (alg_state, dict of outputs).

    ``m`` is a mesh with attributes N, H, T, E, nl, dim, nlev_nod, nlev_elem, elem2D_nodes,
    nie_num, nie, edges, edge_tri; ``f`` a dict of fields (ttf, LO, adf_v, adf_h, area_inv).
    """
    L = m.nl - 1
    NT = m.N + m.H
    out = dict(ttf_max=np.zeros(NT * L), ttf_min=np.zeros(NT * L), plus=np.zeros(NT * L),
               minus=np.zeros(NT * L), UV=np.zeros(2 * L * m.T))
    st = lib().oracle_pre_comm(
        _ptr(out["ttf_max"]), _ptr(out["ttf_min"]), _ptr(out["plus"]), _ptr(out["minus"]),
        _ptr(f["ttf"]), _ptr(f["LO"]), _ptr(f["adf_v"]), _ptr(f["adf_h"]), _ptr(out["UV"]),
        _ptr(f["area_inv"]), _I(m.N), _I(m.H), _I(m.T), _I(m.E), _I(m.nl), _ptr(m.nlev_nod),
        _ptr(m.nlev_elem), _ptr(m.elem2D_nodes), _ptr(m.nie_num), _ptr(m.nie), _I(m.dim),
        _ptr(m.edges), _ptr(m.edge_tri), _I(vlimit), _D(eps), _D(big), _D(dt), _I(1 if vlimit_ext else 0))
    return st, out


def post_comm(m, f, plus, minus, dt=1.0):
    """Phase 2 (b3v, b3h, cv, ch) on copies; ``plus``/``minus`` must be valid on owned+halo."""
    adf_v = f["adf_v"].copy()
    adf_h = f["adf_h"].copy()
    del_v = f["del_v"].copy()
    del_h = f["del_h"].copy()
    b3v(m.N, m.nlev_nod, m.nl, adf_v, plus, minus)
    b3h(m.E, m.nlev_elem, m.nl, m.edges, m.edge_tri, adf_h, plus, minus)
    cv(m.N, m.nlev_nod, m.nl, del_v, f["ttf"], f["hnode"], f["LO"], f["hnode_new"], adf_v, dt, f["area"])
    ch(m.E, m.nlev_elem, m.nl, m.edges, m.edge_tri, del_h, adf_h, dt, f["area"])
    return dict(adf_v=adf_v, adf_h=adf_h, del_v=del_v, del_h=del_h)


def post_comm_iter(m, f, plus, minus, adf_v2, adf_h2, dt=1.0):
    """iter_yn phase 2 of one non-final iteration (docs/refactoring.md:204-290 with iter_yn true):
    b3v/b3h writing the remainders into copies of adf_v2/adf_h2, the LO update, then the Fortran's
    whole-array assignments fct_adf_h = fct_adf_h2, fct_adf_v = fct_adf_v2.  Returns LO, adf_v,
    adf_h, adf_v2, adf_h2 (parity unpinned: no executable reference holds this branch)."""
    adf_v, adf_h = f["adf_v"].copy(), f["adf_h"].copy()
    adf_v2, adf_h2 = adf_v2.copy(), adf_h2.copy()
    LO = f["LO"].copy()
    b3v(m.N, m.nlev_nod, m.nl, adf_v, plus, minus, adf_v2)
    b3h(m.E, m.nlev_elem, m.nl, m.edges, m.edge_tri, adf_h, plus, minus, adf_h2)
    lo_update(m.N, m.nlev_nod, m.E, m.nlev_elem, m.nl, m.edges, m.edge_tri, LO, adf_v, adf_h, dt, f["area"],
              f["hnode_new"])
    return dict(LO=LO, adf_v=adf_v2.copy(), adf_h=adf_h2.copy(), adf_v2=adf_v2, adf_h2=adf_h2)


def iterated_pass(m, f, iterations, dt=1.0, **kw):
    """FESOM2's iterative FCT on one domain: ``iterations - 1`` calls of fct_ale with iter_yn
    (each updating LO and handing the remainders on as the next antidiffusive fluxes), then the
    final non-iterative pass.  adf_v2/adf_h2 start at zero (FESOM allocates them zeroed)."""
    f = dict(f)
    adf_v2, adf_h2 = np.zeros_like(f["adf_v"]), np.zeros_like(f["adf_h"])
    for _ in range(iterations - 1):
        st, p1 = pre_comm(m, f, dt=dt, **kw)
        if st != 5:
            raise RuntimeError(f"oracle pre_comm stopped at alg_state {st}")
        r = post_comm_iter(m, f, p1["plus"], p1["minus"], adf_v2, adf_h2, dt=dt)
        f.update(LO=r["LO"], adf_v=r["adf_v"], adf_h=r["adf_h"])
        adf_v2, adf_h2 = r["adf_v2"], r["adf_h2"]
    out = full_pass(m, f, dt=dt, **kw)
    out.update(LO=f["LO"], adf_v2=adf_v2, adf_h2=adf_h2)
    return out


def full_pass(m, f, vlimit=1, eps=1e-16, big=1e3, dt=1.0):
    """Single-domain full pass a1..c; returns dict with plus, minus, adf_v, adf_h, del_v, del_h."""
    st, p1 = pre_comm(m, f, vlimit=vlimit, eps=eps, big=big, dt=dt)
    if st != 5:
        raise RuntimeError(f"oracle pre_comm stopped at alg_state {st}")
    out = post_comm(m, f, p1["plus"], p1["minus"], dt=dt)
    out.update(plus=p1["plus"], minus=p1["minus"], ttf_max=p1["ttf_max"], ttf_min=p1["ttf_min"], UV=p1["UV"])
    return out


def time_full_pass(m, f, budget_s=15.0, max_reps=50, keep=False):
    """Time the single-threaded oracle full pass (cpu_baseline leg of bench.py).  ``keep``: also
    return the last pass's outputs (bench.py checks the GPU against them)."""
    t_all = []
    out = None
    t0 = time.perf_counter()
    while len(t_all) < max_reps:
        t = time.perf_counter()
        out = full_pass(m, f)
        t_all.append(time.perf_counter() - t)
        if time.perf_counter() - t0 > budget_s:
            break
    return (min(t_all), len(t_all), out) if keep else (min(t_all), len(t_all))


# --------------------------------------------------------------------------- reference.cpp

def ref_pre_comm(m, f, eps=1e-16, big=1e3, dt=1.0):
    """Run reference.cpp a1..a4 exactly as its fct_ale_pre_comm_ sequences them
    (src/reference.cpp:289-304; vlimit 1).  Returns outputs dict, or None without _ref."""
    r = ref()
    if r is None:
        return None
    L = m.nl - 1
    NT = m.N + m.H
    tmax, tmin = np.zeros(NT * L), np.zeros(NT * L)
    plus, minus = np.zeros(NT * L), np.zeros(NT * L)
    UV = np.zeros(2 * L * m.T)
    ib = lambda v: C.byref(_I(v))
    db = lambda v: C.byref(_D(v))
    r.fct_ale_a1_reference_(ib(NT), _ptr(m.nlev_nod), ib(m.nl), _ptr(tmax), _ptr(tmin), _ptr(f["LO"]),
                            _ptr(f["ttf"]))
    r.fct_ale_a2_reference_(ib(m.T), _ptr(m.nlev_elem), ib(m.nl), _ptr(UV), _ptr(m.elem2D_nodes),
                            _ptr(tmax), _ptr(tmin), db(big))
    r.fct_ale_a3_reference_(ib(m.N), _ptr(m.nlev_nod), ib(m.nl), _ptr(tmax), _ptr(tmin), _ptr(f["LO"]),
                            _ptr(UV), _ptr(plus), _ptr(minus), _ptr(f["adf_v"]), _ptr(m.nie),
                            _ptr(m.nie_num), ib(m.dim))
    r.fct_ale_a4_reference_(ib(m.N), _ptr(m.nlev_nod), _ptr(m.nlev_elem), ib(m.nl), ib(m.E), _ptr(plus),
                            _ptr(minus), _ptr(f["adf_h"]), _ptr(f["area_inv"]), _ptr(tmax), _ptr(tmin),
                            _ptr(m.edges), _ptr(m.edge_tri), db(eps), db(dt))
    return dict(ttf_max=tmax, ttf_min=tmin, plus=plus, minus=minus, UV=UV)


def time_ref_pre_comm(m, f, reps=2):
    """Best wall time of reference.cpp's CPU path (a1..a4 = a1..b2, the whole of what the reference
    implements on the CPU), or None without _ref (bench.py's cpu_baseline, kind "reference")."""
    import time
    if ref() is None:
        return None
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        ref_pre_comm(m, f)
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    return best


def b1h(nlev_elem, nl, n_edges, plus, minus, adf_h, edges, edge_tri):
    lib().oracle_b1h(_ptr(nlev_elem), _I(nl), _I(n_edges), _ptr(plus), _ptr(minus), _ptr(adf_h), _ptr(edges),
                     _ptr(edge_tri))


def b2(n_nodes, nlev_nod, nl, plus, minus, area_inv, tmax, tmin, eps, dt):
    lib().oracle_b2(_I(n_nodes), _ptr(nlev_nod), _I(nl), _ptr(plus), _ptr(minus), _ptr(area_inv), _ptr(tmax),
                    _ptr(tmin), _D(eps), _D(dt))


def pre_comm_steps(m, f, eps=1e-16, big=1e3, dt=1.0, vlimit=1):
    """Phase 1 state after each reference step: {1: a1, 2: a2, 3: a3, 4: b1v, 5: b1h, 6: b2}."""
    L, NT = m.nl - 1, m.N + m.H
    tmax, tmin = np.zeros(NT * L), np.zeros(NT * L)
    plus, minus = np.zeros(NT * L), np.zeros(NT * L)
    UV = np.zeros(2 * L * m.T)
    snap = lambda: dict(ttf_max=tmax.copy(), ttf_min=tmin.copy(), plus=plus.copy(), minus=minus.copy(), UV=UV.copy())
    s = {}
    a1(NT, m.nlev_nod, m.nl, tmax, tmin, f["LO"], f["ttf"])
    s[1] = snap()
    a2(m.T, m.nlev_elem, m.nl, UV, m.elem2D_nodes, tmax, tmin, big)
    s[2] = snap()
    a3(m.N, m.nlev_nod, m.nl, tmax, tmin, f["LO"], UV, plus, minus, f["adf_v"], m.nie, m.nie_num, m.dim, vlimit)
    s[3] = s[4] = snap()  # the oracle's a3 includes b1-vertical (reference.cpp:393-399)
    b1h(m.nlev_elem, m.nl, m.E, plus, minus, f["adf_h"], m.edges, m.edge_tri)
    s[5] = snap()
    b2(m.N, m.nlev_nod, m.nl, plus, minus, f["area_inv"], tmax, tmin, eps, dt)
    s[6] = snap()
    return s
