"""GPU: the reference's C++ convenience entries a1 / a2 / a1+a2 on gpuMemory handles
(include/fesom2-accelerate-legacy.hpp; reference include/fesom2-accelerate.h:155-209,
src/fesom2-accelerate.cu:42-112) against a numpy restatement of the reference kernels they run
(kernels/fct_ale_a1.cu, kernels/fct_ale_a2.cu): one column stride maxLevels for every array, a1 over
z < nLevels(n) with fmax/fmin, a2 over z < nLevels(e) - 1 plus the (-1e3, +1e3) fill up to
maxLevels - 1.  (These kernels' conventions differ from src/reference.cpp's a1/a2, which the phase
path and the oracle follow; no executable reference runs them here -- they are CUDA -- so the pin is
this restatement of their ten lines each.)
"""
import ctypes as C

import numpy as np
import pytest

from fesom2_amd import abi, synth

pytestmark = pytest.mark.gpu


def a1_ref(stride, nlev, lo, ttf, tmax, tmin):
    for n, k in enumerate(nlev):  # kernels/fct_ale_a1.cu:2-15
        s = slice(n * stride, n * stride + k)
        tmax[s] = np.fmax(lo[s], ttf[s])
        tmin[s] = np.fmin(lo[s], ttf[s])


def a2_ref(stride, nlev_e, en, tmax, tmin, uv):
    uv = uv.reshape(-1, 2)
    for e, k in enumerate(nlev_e):  # kernels/fct_ale_a2.cu:2-25
        i = (en[3 * e: 3 * e + 3] - 1) * stride
        for z in range(stride + 1):
            if z < k - 1:
                uv[e * stride + z] = (np.fmax(np.fmax(tmax[i[0] + z], tmax[i[1] + z]), tmax[i[2] + z]),
                                      np.fmin(np.fmin(tmin[i[0] + z], tmin[i[1] + z]), tmin[i[2] + z]))
            elif z < stride - 1:
                uv[e * stride + z] = (-1.0e3, 1.0e3)


class Legacy:
    """Handles of one small problem (single stride = nl), host arrays bound, device arrays set."""

    def __init__(self, nx=16, ny=9, nl=9, seed=5):
        m = synth.make_mesh(nx, ny, nl, seed=seed)
        self.m, self.stride = m, nl
        rng = np.random.default_rng(seed)
        nn, ne = m.N, m.T
        self.host = {"lo": rng.standard_normal(nn * nl), "ttf": rng.standard_normal(nn * nl),
                     "tmax": np.full(nn * nl, 7.0), "tmin": np.full(nn * nl, -7.0),
                     "uv": np.full(2 * ne * nl, 3.0)}
        self.ints = {"nlev_nod": m.nlev_nod.astype(np.int32), "nlev_elem": m.nlev_elem.astype(np.int32),
                     "en": m.elem2D_nodes.astype(np.int32)}
        self.h = {}
        for k, a in self.ints.items():
            h, st = abi.Handle(k), C.c_int(0)
            abi.dll().transfer_mesh_(h.ref, abi.arr(a), abi.ip(a.size), C.byref(st))
            abi.check(st, f"transfer_mesh_({k})")
            self.h[k] = h
        for k, a in self.host.items():
            h = abi.Handle(k)
            abi.check(abi.alloc_var(h, a), f"alloc_var_({k})")
            abi.dll().transfer_var_(h.ref, abi.arr(a))  # initial device contents = the host arrays
            self.h[k] = h
        self.start = {k: v.copy() for k, v in self.host.items()}

    def g(self, k):
        return C.c_void_p(self.h[k].ptr.value)  # struct gpuMemory * = the handle's void*

    def free(self):
        for h in self.h.values():
            abi.dll().fesom2_free_(h.ref)


@pytest.fixture()
def prob():
    abi.set_mpi_rank(0, 1)
    p = Legacy()
    yield p
    p.free()


def stream_value(s):
    return C.c_void_p.from_address(s.ptr.value).value  # make_stream_'s handle holds a hipStream_t*


@pytest.mark.parametrize("sync", [True, False])
def test_a1_a2_accelerated_match_the_reference_kernels(prob, sync):
    lib = abi.legacy()
    s = abi.Stream()
    sv = None if sync else stream_value(s)
    p, st, m = prob, prob.stride, prob.m
    lib.fct_ale_a1_accelerated(st, m.N, p.g("nlev_nod"), p.g("tmax"), p.g("tmin"), p.g("lo"), p.g("ttf"), sync, sv)
    lib.fct_ale_a2_accelerated(st, m.T, p.g("nlev_elem"), p.g("en"), p.g("uv"), p.g("tmax"), p.g("tmin"), sync, sv)
    s.sync()
    w = {k: v.copy() for k, v in p.start.items()}
    a1_ref(st, p.ints["nlev_nod"], w["lo"], w["ttf"], w["tmax"], w["tmin"])
    a2_ref(st, p.ints["nlev_elem"], p.ints["en"], w["tmax"], w["tmin"], w["uv"])
    for k in ("tmax", "tmin", "uv"):
        assert np.array_equal(p.host[k], w[k]), k
    s.free()


def test_a1_a2_fused_entry_returns_uv_only(prob):
    """fct_ale_a1_a2_accelerated: a1 then a2 on the device; only UV_rhs comes back (src:91-112)."""
    lib = abi.legacy()
    p, st, m = prob, prob.stride, prob.m
    lib.fct_ale_a1_a2_accelerated(st, m.N, m.T, p.g("nlev_nod"), p.g("nlev_elem"), p.g("en"), p.g("tmax"),
                                  p.g("tmin"), p.g("lo"), p.g("ttf"), p.g("uv"), True, None)
    w = {k: v.copy() for k, v in p.start.items()}
    a1_ref(st, p.ints["nlev_nod"], w["lo"], w["ttf"], w["tmax"], w["tmin"])
    a2_ref(st, p.ints["nlev_elem"], p.ints["en"], w["tmax"], w["tmin"], w["uv"])
    assert np.array_equal(p.host["uv"], w["uv"])
    assert np.array_equal(p.host["tmax"], p.start["tmax"])  # not transferred back
    dev = np.empty_like(w["tmax"])
    st_ = C.c_int(0)
    abi.dll().fesom2_download_(p.h["tmax"].ref, abi.arr(dev), C.byref(st_))
    assert np.array_equal(dev, w["tmax"])


def test_legacy_entries_refuse_levels_beyond_the_stride(prob):
    """A column deeper than maxLevels (or an element node outside the arrays) is reported and nothing
    runs: the outputs keep their contents."""
    lib = abi.legacy()
    p, m = prob, prob.m
    lib.fct_ale_a1_accelerated(p.stride - 1, m.N, p.g("nlev_nod"), p.g("tmax"), p.g("tmin"), p.g("lo"), p.g("ttf"),
                               True, None)
    assert "exceeds maxLevels" in abi.last_error()
    assert np.array_equal(p.host["tmax"], p.start["tmax"])
    bad = p.ints["en"].copy()
    bad[4] = m.N + 1
    st = C.c_int(0)
    abi.dll().fesom2_upload_(p.h["en"].ref, abi.arr(bad), C.byref(st))
    lib.fct_ale_a2_accelerated(p.stride, m.T, p.g("nlev_elem"), p.g("en"), p.g("uv"), p.g("tmax"), p.g("tmin"),
                               True, None)
    assert "elementNodes" in abi.last_error()
    assert np.array_equal(p.host["uv"], p.start["uv"])


def test_legacy_check_waits_for_an_upload_on_another_stream(prob):
    """the index check is cached per (handle, serial, upload version), and the version is
    bumped when an upload is enqueued.  An upload of bad elementNodes on a second non-blocking stream,
    queued behind a 512 MB transfer, must still be seen by the next legacy call's check (it waits for
    the whole device on a cache miss): the call is refused and UV_rhs is never written."""
    lib = abi.legacy()
    p, m = prob, prob.m
    ne = p.ints["en"].size
    host, hp = abi.pinned((ne + 1) // 2)  # elementNodes as raw bytes in a pinned double array
    big, bhp = abi.pinned(64 << 20)
    hen, hbig, s2 = abi.Handle("en"), abi.Handle("big"), abi.Stream()
    try:
        host.view(np.int32)[:ne] = p.ints["en"]
        abi.check(abi.alloc_var(hen, host), "alloc_var_(en)")
        abi.check(abi.alloc_var(hbig, big), "alloc_var_(big)")
        abi.dll().transfer_var_(hen.ref, abi.arr(host))
        en = C.c_void_p(hen.ptr.value)
        lib.fct_ale_a2_accelerated(p.stride, m.T, p.g("nlev_elem"), en, p.g("uv"), p.g("tmax"), p.g("tmin"),
                                   True, None)
        w = {k: v.copy() for k, v in p.start.items()}
        a2_ref(p.stride, p.ints["nlev_elem"], p.ints["en"], w["tmax"], w["tmin"], w["uv"])
        assert np.array_equal(p.host["uv"], w["uv"])  # validated (and cached) with the good indices
        bad = p.ints["en"].copy()
        bad[4] = m.N + 1
        host.view(np.int32)[:ne] = bad
        abi.transfer_var_async(hbig, big, s2)  # keeps s2 busy for a few ms
        abi.transfer_var_async(hen, host, s2)
        p.host["uv"][:] = 11.0
        lib.fct_ale_a2_accelerated(p.stride, m.T, p.g("nlev_elem"), en, p.g("uv"), p.g("tmax"), p.g("tmin"),
                                   True, None)
        assert "elementNodes" in abi.last_error()
        assert np.all(p.host["uv"] == 11.0)
    finally:
        s2.sync()
        for h in (hen, hbig):
            abi.dll().fesom2_free_(h.ref)
        s2.free()
        abi.free_pinned(hp)
        abi.free_pinned(bhp)
