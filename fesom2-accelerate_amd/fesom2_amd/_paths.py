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


def code_object_hash(path=None):
    """sha256 (first 16 hex digits) of the device code objects in an engine library: the bytes of its
    ``.hip_fatbin`` ELF section, i.e. the gfx950 kernels of that build and nothing of its host code.
    profiles/pmc_traffic.py stamps every traffic*.json with the hash of the library it measured, and
    bench.py reports a file's PMC traffic only when the loaded library carries the same kernels."""
    import hashlib
    import struct

    path = path or lib_path(engine_name())
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        raise ValueError(f"{path}: not a little-endian ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sect(i):  # (name offset, file offset, size)
        b = shoff + i * shentsize
        name, = struct.unpack_from("<I", data, b)
        off, size = struct.unpack_from("<QQ", data, b + 0x18)
        return name, off, size

    _, stroff, _ = sect(shstrndx)
    for i in range(shnum):
        name, off, size = sect(i)
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    raise ValueError(f"{path}: no .hip_fatbin section")
