"""The Fortran host (``fesom2-accelerate_amd/fortran``): FESOM2's side of the drop-in.

``fct_ale_host`` is built with the image's amdflang from an ISO_C_BINDING module that declares the
reference's entry points (reference include/fesom2-accelerate.h:146-158) plus this library's
additions, and drives them in FESOM2's order.  CPU: the module and driver build
and bind exactly the exported C symbols.  GPU: the driver runs the reference sequence (reference
transfer semantics) and the device-resident split pass, and its host arrays equal the oracle's.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, assert_cols_equal
from fesom2_amd import synth

FDIR = os.path.join(ROOT, "fesom2-accelerate_amd", "fortran")
HOST = os.path.join(ROOT, "fesom2-accelerate_amd", "lib", "fct_ale_host")
LIB = os.path.join(ROOT, "fesom2-accelerate_amd", "lib", "libfesom2-accelerate.so")
ABI_NAMES = ("set_mpi_rank_", "transfer_mesh_", "alloc_var_", "reserve_var_", "transfer_var_",
             "transfer_var_async_", "make_stream_", "await_stream_")


def write_input(path, m, f, mode, vlimit=1, dt=1.0, eps=1e-16, big=1e3, tracers=None):
    """The driver's input file: int64 element count, then the elements, per array.  ``tracers``: a
    list of field dicts whose per-tracer arrays are written one after another (modes 1 and 2)."""
    with open(path, "wb") as fh:
        def put(a, typ):
            a = np.ascontiguousarray(a, dtype=typ).reshape(-1)
            fh.write(np.int64(a.size).tobytes())
            fh.write(a.tobytes())
        put([m.N, m.H, m.T, m.E, m.nl, m.dim, vlimit, mode], np.int32)
        for k in ("nlev_nod", "nlev_elem", "elem2D_nodes", "nie_num", "nie", "edges", "edge_tri"):
            put(getattr(m, k), np.int32)
        per_tracer = ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h")
        for k in ("ttf", "LO", "adf_v", "adf_h", "area", "area_inv", "hnode", "hnode_new", "del_v", "del_h"):
            put(np.concatenate([t[k] for t in tracers]) if tracers and k in per_tracer else f[k], np.float64)
        put([dt, eps, big], np.float64)


def read_output(path):
    with open(path, "rb") as fh:
        data = fh.read()
    pos, out = 0, []
    n = int(np.frombuffer(data, np.int64, 1, pos)[0])
    pos += 8
    states = np.frombuffer(data, np.int32, n, pos).tolist()
    pos += 4 * n
    for _ in range(6):
        n = int(np.frombuffer(data, np.int64, 1, pos)[0])
        pos += 8
        out.append(np.frombuffer(data, np.float64, n, pos).copy())
        pos += 8 * n
    return states, dict(zip(("plus", "minus", "adf_v", "adf_h", "del_v", "del_h"), out))


needs_flang = pytest.mark.skipif(shutil.which("amdflang") is None and not os.path.exists(HOST),
                                 reason="no amdflang and no prebuilt fct_ale_host")


@needs_flang
def test_fortran_host_builds_and_binds_the_abi():
    """The driver links against the library and every bind(C) name it uses is an exported symbol."""
    if shutil.which("amdflang"):
        subprocess.run(["make", "-C", FDIR], check=True, capture_output=True)
    assert os.path.exists(HOST)
    undef = subprocess.run(["nm", "-D", "--undefined-only", HOST], capture_output=True, text=True).stdout
    names = [ln.split()[-1] for ln in undef.splitlines() if ln.split()]
    used = {s for s in names if s.endswith("_") and (s.startswith(("fct_ale", "fesom2_")) or s in ABI_NAMES)}
    exported = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in exported.splitlines() if ln.split()}
    assert len(used) >= 16 and used <= exported, used - exported
    for name in ("fct_ale_pre_comm_acc_", "fct_ale_inter_comm_acc_", "fct_ale_post_comm_acc_", "fct_ale_c_acc_",
                 "fct_ale_pre_comm_v_acc_", "fct_ale_post_comm_h_acc_", "fesom2_graph_begin_", "fesom2_graph_launch_",
                 "fesom2_set_path_", "fesom2_bind_c_vertical_"):
        assert name in used


def test_input_format_header(tmp_path):
    """The writer lays out the header the driver reads first (CPU-only check of the format)."""
    m = synth.config_mesh("tiny")
    f = synth.make_fields(m)
    p = tmp_path / "in.bin"
    write_input(p, m, f, mode=1)
    raw = p.read_bytes()
    assert np.frombuffer(raw, np.int64, 1, 0)[0] == 8
    assert np.frombuffer(raw, np.int32, 8, 8).tolist() == [m.N, m.H, m.T, m.E, m.nl, m.dim, 1, 1]


@pytest.mark.gpu
@needs_flang
@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4], ids=["reference_sequence", "resident_split", "graph_replay",
                                                     "reference_sequence_fast_mode", "producer_uploads"])
@pytest.mark.parametrize("name", ["8k x 20", "127k x 47"])
def test_fortran_host_matches_oracle(tmp_path, mode, name):
    import oracle as O
    m = synth.config_mesh(name)
    f = synth.make_fields(m)
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    write_input(fin, m, f, mode)
    r = subprocess.run([HOST, str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    states, got = read_output(fout)
    assert states == ([6, 7, 8, 9] if mode in (0, 3) else [7, 9, -1, -1]), states  # mode 2: the captured calls
    want = O.full_pass(m, f)
    assert_cols_equal(got["plus"], want["plus"], m.nlev_nod, m.L, m.N, "fct_plus")
    assert_cols_equal(got["minus"], want["minus"], m.nlev_nod, m.L, m.N, "fct_minus")
    for k in ("adf_v", "adf_h", "del_v", "del_h"):
        assert np.array_equal(got[k], want[k]), k


@pytest.mark.gpu
@needs_flang
@pytest.mark.parametrize("mode", [1, 2, 4], ids=["resident_split", "graph_replay", "producer_uploads"])
@pytest.mark.parametrize("name", ["8k x 20", "127k x 47"])
def test_fortran_host_batched_tracers(tmp_path, mode, name):
    """FESOM2's tracer loop as one batched call from Fortran (BASELINE config 3's entry points):
    3 tracers in (nl-1, nod, ntracers) arrays through fct_ale_pre_comm_v_acc_ / fct_ale_post_comm_h_acc_
    with ntracers = 3, each tracer equal to its own oracle pass."""
    import oracle as O
    m = synth.config_mesh(name)
    tracers = synth.make_tracer_fields(m, 3)
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    write_input(fin, m, tracers[0], mode, tracers=tracers)
    r = subprocess.run([HOST, str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tracers  3" in r.stdout, r.stdout
    states, got = read_output(fout)
    assert states == [7, 9, -1, -1], states
    for t, f in enumerate(tracers):
        want = O.full_pass(m, f)
        part = {k: v.reshape(3, -1)[t] for k, v in got.items()}
        assert_cols_equal(part["plus"], want["plus"], m.nlev_nod, m.L, m.N, f"tracer {t} fct_plus")
        assert_cols_equal(part["minus"], want["minus"], m.nlev_nod, m.L, m.N, f"tracer {t} fct_minus")
        for k in ("adf_v", "adf_h", "del_v", "del_h"):
            assert np.array_equal(part[k], want[k]), (t, k)
