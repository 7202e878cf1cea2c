"""ctypes bindings of ``libfesom2-accelerate.so`` -- exactly the C-ABI of include/fesom2-accelerate.h.

This is the binding a maintainer of the reference's Python/kernel_tuner harness would use (the
reference declares the same entry points at ``include/fesom2-accelerate.h:128-236``).  Every
argument is passed by pointer, as gfortran does; device buffers are opaque ``void*`` handles
passed as ``void**``.

Loading fails loudly when the library is missing: there is no fallback path.
"""
from __future__ import annotations

import ctypes as C

from ._paths import engine_name, lib_path

# every exported symbol of include/fesom2-accelerate.h (checked by tests/test_abi.py)
EXPORTS = (
    "set_mpi_rank_", "transfer_mesh_", "alloc_var_", "reserve_var_", "allocate_pinned_doubles_",
    "transfer_var_", "transfer_var_async_", "make_stream_", "await_stream_",
    "fct_ale_pre_comm_acc_", "fct_ale_inter_comm_acc_", "fct_ale_post_comm_acc_",
    "fct_ale_a1_reference_", "fct_ale_a2_reference_", "fct_ale_a3_reference_", "fct_ale_a4_reference_",
    "fct_ale_pre_comm_",
    "fct_ale_c_acc_", "fct_ale_post_comm_c_acc_", "fesom2_set_resident_", "fesom2_set_path_",
    "fesom2_prepare_mesh_", "fesom2_download_", "fesom2_upload_", "fesom2_free_", "fesom2_free_stream_",
    "fesom2_free_pinned_", "fesom2_device_sync_", "fesom2_last_error", "fesom2_event_create_",
    "fesom2_event_record_", "fesom2_event_elapsed_", "fesom2_event_free_",
    "fesom2_kernel_timing_", "fesom2_kernel_timing_only_", "fesom2_kernel_timing_reset_", "fesom2_kernel_stats_",
    "fesom2_comm_unique_id_", "fesom2_comm_init_", "fesom2_comm_free_", "fesom2_comm_info_", "fesom2_halo_plan_",
    "fesom2_halo_plan_free_", "fct_ale_exchange_acc_", "fct_ale_exchange_post_comm_c_acc_",
    "fct_ale_pre_comm_batched_acc_", "fct_ale_post_comm_c_batched_acc_", "fct_ale_exchange_batched_acc_",
    "fct_ale_exchange_post_comm_c_batched_acc_", "fct_ale_post_comm_iter_acc_",
    "fct_ale_post_comm_iter_batched_acc_", "fesom2_exchange_nod_acc_",
    "fesom2_alloc_var_i8_", "fesom2_reserve_var_i8_", "fct_ale_pre_comm_v_acc_", "fct_ale_post_comm_h_acc_",
    "fesom2_graph_begin_", "fesom2_graph_end_", "fesom2_graph_launch_", "fesom2_graph_free_",
    "fesom2_graph_info_", "fesom2_mesh_info_", "fesom2_bind_c_vertical_", "fesom2_pass_order_",
    "fesom2_transfer_back_async_",
)

# the reference's C++ convenience entries (include/fesom2-accelerate-legacy.hpp: C linkage, plain
# values, `struct gpuMemory *` = the handle's void*, a hipStream_t stream)
LEGACY_EXPORTS = ("fct_ale_a1_accelerated", "fct_ale_a2_accelerated", "fct_ale_a1_a2_accelerated")

_dll = None


def dll():
    """The engine library (loaded once)."""
    global _dll
    if _dll is None:
        _dll = C.CDLL(lib_path(engine_name()))
        _dll.fesom2_last_error.restype = C.c_char_p
    return _dll


def ip(v):
    """int* argument."""
    return C.byref(C.c_int(int(v)))


def dp(v):
    """double* argument."""
    return C.byref(C.c_double(float(v)))


def bp(v):
    """bool* argument (C99 _Bool / Fortran logical(c_bool))."""
    return C.byref(C.c_bool(bool(v)))


def arr(a):
    """host array argument (numpy, contiguous)."""
    assert a.flags.c_contiguous, "host arrays must be contiguous"
    return a.ctypes.data_as(C.c_void_p)


def legacy():
    """The engine library with the argument types of the legacy C++ entries set."""
    lib = dll()
    vp, i, b = C.c_void_p, C.c_int, C.c_bool
    lib.fct_ale_a1_accelerated.argtypes = [i, i, vp, vp, vp, vp, vp, b, vp]
    lib.fct_ale_a2_accelerated.argtypes = [i, i, vp, vp, vp, vp, vp, b, vp]
    lib.fct_ale_a1_a2_accelerated.argtypes = [i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, b, vp]
    for name in LEGACY_EXPORTS:
        getattr(lib, name).restype = None
    return lib


def last_error():
    return dll().fesom2_last_error().decode()


class HipError(RuntimeError):
    pass


def check(istat, what):
    v = istat.value if hasattr(istat, "value") else istat
    if v != 0:
        raise HipError(f"{what} failed (istat={v}): {last_error()}")


def alloc_var(h, a, create_event=False):
    """alloc_var_ (int size), or fesom2_alloc_var_i8_ past 2^31-1 elements."""
    st = C.c_int(0)
    n = max(a.size, 1)
    if n < 2**31:
        dll().alloc_var_(h.ref, arr(a), ip(n), bp(create_event), C.byref(st))
    else:
        dll().fesom2_alloc_var_i8_(h.ref, arr(a), C.byref(C.c_longlong(n)), bp(create_event), C.byref(st))
    return st


def reserve_var(h, n, create_event=False):
    st = C.c_int(0)
    n = max(n, 1)
    if n < 2**31:
        dll().reserve_var_(h.ref, ip(n), bp(create_event), C.byref(st))
    else:
        dll().fesom2_reserve_var_i8_(h.ref, C.byref(C.c_longlong(n)), bp(create_event), C.byref(st))
    return st


class Handle:
    """A ``void*`` returned by the library; ``ref`` is the ``void**`` the entry points take."""

    def __init__(self, name=""):
        self.ptr = C.c_void_p()
        self.name = name

    @property
    def ref(self):
        return C.byref(self.ptr)

    def __bool__(self):
        return bool(self.ptr.value)


class Stream(Handle):
    def __init__(self):
        super().__init__("stream")
        st = C.c_int(0)
        dll().make_stream_(self.ref, C.byref(st))
        if st.value:
            raise HipError(f"make_stream_ fell back to the null stream: {last_error()}")

    def sync(self):
        st = C.c_int(0)
        dll().await_stream_(self.ref, C.byref(st))
        check(st, "await_stream_")

    def free(self):
        if self:
            dll().fesom2_free_stream_(self.ref)


class Event(Handle):
    def __init__(self):
        super().__init__("event")
        st = C.c_int(0)
        dll().fesom2_event_create_(self.ref, C.byref(st))
        check(st, "fesom2_event_create_")

    def record(self, stream):
        dll().fesom2_event_record_(self.ref, stream.ref)

    def elapsed_ms(self, later):
        ms = C.c_float(0)
        dll().fesom2_event_elapsed_(self.ref, later.ref, C.byref(ms))
        return ms.value

    def free(self):
        if self:
            dll().fesom2_event_free_(self.ref)


class Graph(Handle):
    """hipGraph of a captured call sequence: ``with Graph.capture(stream) as g: <entry calls>``,
    then ``g.launch(stream)`` replays it (device-resident mode, plans built beforehand)."""

    def __init__(self):
        super().__init__("graph")

    @classmethod
    def capture(cls, stream):
        return _Capture(cls(), stream)

    def launch(self, stream):
        st = C.c_int(0)
        dll().fesom2_graph_launch_(C.byref(st), self.ref, stream.ref)
        check(st, "fesom2_graph_launch_")

    def info(self):
        """(objects the replays check are alive, buffer events each replay waits for)."""
        nu, nw = C.c_int(0), C.c_int(0)
        dll().fesom2_graph_info_(self.ref, C.byref(nu), C.byref(nw))
        return nu.value, nw.value

    def free(self):
        if self:
            dll().fesom2_graph_free_(self.ref)


class _Capture:
    def __init__(self, graph, stream):
        self.graph, self.stream = graph, stream

    def __enter__(self):
        st = C.c_int(0)
        dll().fesom2_graph_begin_(C.byref(st), self.stream.ref)
        check(st, "fesom2_graph_begin_")
        return self.graph

    def __exit__(self, exc_type, exc, tb):
        st = C.c_int(0)
        dll().fesom2_graph_end_(C.byref(st), self.stream.ref, self.graph.ref)
        if exc_type is None:
            check(st, "fesom2_graph_end_")
        return False


def pinned(n):
    """A page-locked host array of n doubles (allocate_pinned_doubles_, as a FESOM2 host would
    allocate its transfer buffers) and its pointer (free with free_pinned)."""
    hp, st = C.c_void_p(), C.c_int(0)
    dll().allocate_pinned_doubles_(C.byref(hp), C.byref(C.c_int(int(max(n, 1)))), C.byref(st))
    if st.value or not hp.value:
        raise HipError(f"allocate_pinned_doubles_({n}) fell back to pageable memory: {last_error()}")
    import numpy as np
    return np.ctypeslib.as_array((C.c_double * int(max(n, 1))).from_address(hp.value))[:n], hp


def free_pinned(hp):
    dll().fesom2_free_pinned_(C.byref(hp))


def transfer_var_async(h, a, stream, record_event=False):
    """transfer_var_async_: rebind h's host array to ``a`` and enqueue its H2D on ``stream``."""
    dll().transfer_var_async_(h.ref, arr(a), stream.ref, bp(record_event))


def transfer_back_async(h, a, stream):
    """fesom2_transfer_back_async_: rebind h's host array to ``a`` and enqueue its D2H on ``stream``."""
    st = C.c_int(0)
    dll().fesom2_transfer_back_async_(h.ref, arr(a), stream.ref, C.byref(st))
    check(st, "fesom2_transfer_back_async_")


def set_resident(on):
    dll().fesom2_set_resident_(ip(1 if on else 0))


def set_path(path):
    """fesom2_set_path_: "fused" (0), "stepwise" (1), or "reference" (2: the reference entry
    sequence's fast mode, b3v inside fct_ale_pre_comm_acc_)."""
    code = {"fused": 0, "stepwise": 1, "reference": 2}.get(path, path)
    dll().fesom2_set_path_(ip(code))


def device_sync():
    st = C.c_int(0)
    dll().fesom2_device_sync_(C.byref(st))
    check(st, "fesom2_device_sync_")


def kernel_timing(on):
    """Enable/disable per-launch HIP-event timing inside the library."""
    dll().fesom2_kernel_timing_(ip(1 if on else 0))


def kernel_timing_only(name=None):
    """Time only the launches called ``name`` (None: every launch)."""
    dll().fesom2_kernel_timing_only_(name.encode() if name else None)


def kernel_timing_reset():
    dll().fesom2_kernel_timing_reset_()


def kernel_stats():
    """{kernel name: (launches, total ms)} accumulated while timing was enabled."""
    n = C.c_int(0)
    dll().fesom2_kernel_stats_(None, C.byref(n))
    buf = C.create_string_buffer(n.value + 1)
    n2 = C.c_int(n.value + 1)
    dll().fesom2_kernel_stats_(buf, C.byref(n2))
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split()
        out[name] = (int(cnt), float(ms))
    return out


def set_mpi_rank(rank, nranks):
    dll().set_mpi_rank_(ip(rank), ip(nranks))
