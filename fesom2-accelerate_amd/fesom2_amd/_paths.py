"""Locate the in-tree shared libraries (built by ``make -C fesom2-accelerate_amd``)."""
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # fesom2-accelerate_amd/
LIB_DIR = os.path.join(PKG_ROOT, "lib")
REPO_ROOT = os.path.dirname(PKG_ROOT)


ENGINE = "libfesom2-accelerate.so"


def engine_name():
    """The engine library to load: the product, or FESOM2_LIB_NAME (the tuning build,
    libfesom2-accelerate-tuning.so, for tools/sweep_env.sh and tests/test_gpu_tuning.py)."""
    return os.environ.get("FESOM2_LIB_NAME", ENGINE)


def lib_path(name):
    # FESOM2_LIB_DIR: another build of the libraries (A/B measurements of two versions)
    path = os.path.join(os.environ.get("FESOM2_LIB_DIR", LIB_DIR), name)
    if not os.path.exists(path):
        raise RuntimeError(
            f"{name} is not built ({path}); run `make -C fesom2-accelerate_amd` or __graft_entry__.build()")
    return path
