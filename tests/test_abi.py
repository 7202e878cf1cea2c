"""CPU: the C-ABI library builds, loads and exports exactly what include/fesom2-accelerate.h declares.

No compute call is made here (there is no GPU in the dev container); the parity of every entry point
is tested on the GPU in test_gpu_parity.py.  Also checks that the product library carries no CPU
implementation of the algorithm (no oracle symbols, no fallback path).
"""
import os
import re
import subprocess

import pytest

from fesom2_amd import abi
from fesom2_amd._paths import LIB_DIR, REPO_ROOT

HEADER = os.path.join(REPO_ROOT, "include", "fesom2-accelerate.h")
LIB = os.path.join(LIB_DIR, "libfesom2-accelerate.so")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_]+\s*\*?\s*([A-Za-z0-9_]+)\s*\(", txt, flags=re.M)))


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_header_declares_the_reference_entry_points():
    """Every entry point of the reference header (include/fesom2-accelerate.h:142-235) is kept."""
    ref = {"set_mpi_rank_", "transfer_mesh_", "alloc_var_", "reserve_var_", "allocate_pinned_doubles_",
           "transfer_var_", "transfer_var_async_", "make_stream_", "await_stream_", "fct_ale_pre_comm_acc_",
           "fct_ale_inter_comm_acc_", "fct_ale_post_comm_acc_", "fct_ale_a1_reference_", "fct_ale_a2_reference_",
           "fct_ale_a3_reference_", "fct_ale_a4_reference_", "fct_ale_pre_comm_"}
    assert ref <= set(header_functions())


def test_library_exports_every_declared_symbol():
    declared = set(header_functions())
    exported = exported_symbols()
    missing = declared - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    assert declared == set(abi.EXPORTS), "fesom2_amd.abi.EXPORTS out of sync with the header"


def test_library_loads_and_resolves_symbols():
    lib = abi.dll()
    for name in abi.EXPORTS:
        assert getattr(lib, name) is not None
    assert isinstance(abi.last_error(), str)


def test_no_cpu_fallback_in_the_product_library():
    syms = exported_symbols()
    assert not any(s.startswith("oracle_") for s in syms)
    undefined = subprocess.run(["nm", "-D", "--undefined-only", LIB], capture_output=True, text=True,
                               check=True).stdout
    assert "oracle" not in undefined
    # the kernels are compiled for gfx950 (the offload bundle names its target)
    with open(LIB, "rb") as fh:
        assert b"amdgcn-amd-amdhsa--gfx950" in fh.read()


def test_mode_switches_do_not_need_a_device():
    abi.set_resident(True)
    abi.set_resident(False)
    abi.set_path("stepwise")
    abi.set_path("fused")


def test_product_library_reads_only_the_plan_options():
    """The product library has no A/B knobs: the only environment variables it names are the plan
    options read when a mesh plan is built, and none of the measured-and-rejected
    variants deleted in round 4 (k_p2w, k_p2f, k_p1e, k_p1s, k_p2hf, k_b3h_n, k_p1p, k_p1t) is in it."""
    data = open(LIB, "rb").read()
    names = set(re.findall(rb"FESOM2_[A-Z0-9_]+", data))
    assert names <= {b"FESOM2_PATH", b"FESOM2_NUM_KERNELS", b"FESOM2_P1V_B3H", b"FESOM2_PATCH",
                     b"FESOM2_BATCH_PATCH", b"FESOM2_BATCH_GROUP_SHIFT", b"FESOM2_BATCH_GROUP",
                     b"FESOM2_CACHE_ORDER", b"FESOM2_LARGE_CELLS", b"FESOM2_P1V_UNION"}, names
    syms = subprocess.run(["nm", "-C", LIB], capture_output=True, text=True, check=True).stdout
    for k in ("k_p2w", "k_p2f", "k_p1e", "k_p1s", "k_p2hf", "k_b3h_n", "k_p1p", "k_p1t", "launch_p1_variant"):
        assert not re.search(rf"\b{k}\b", syms), k


def test_tuning_build_exports_the_same_abi():
    tuning = os.path.join(LIB_DIR, "libfesom2-accelerate-tuning.so")
    if not os.path.exists(tuning):
        pytest.skip("tuning build not made")
    out = subprocess.run(["nm", "-D", "--defined-only", tuning], capture_output=True, text=True, check=True).stdout
    assert set(header_functions()) <= {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_legacy_cpp_entries_are_declared_and_exported():
    """The reference's C++ convenience entries (reference include/fesom2-accelerate.h:155-209) are
    declared in include/fesom2-accelerate-legacy.hpp with C linkage and exported."""
    txt = open(os.path.join(REPO_ROOT, "include", "fesom2-accelerate-legacy.hpp")).read()
    declared = set(re.findall(r"^void\s+([A-Za-z0-9_]+)\s*\(", txt, flags=re.M))
    assert declared == set(abi.LEGACY_EXPORTS)
    assert declared <= exported_symbols()
    assert 'extern "C"' in txt and "hipStream_t stream = nullptr" in txt

