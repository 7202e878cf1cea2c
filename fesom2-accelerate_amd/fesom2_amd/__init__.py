"""fesom2_amd -- host side of the MI355X-native FCT-ALE engine.

The engine itself is the C-ABI shared library ``lib/libfesom2-accelerate.so`` (HIP kernels for
gfx950 behind the reference's ``fesom2-accelerate.h`` entry points).  This package is the Python
mirror of the reference's host usage: ctypes bindings of exactly those entry points
(:mod:`fesom2_amd.abi`), a driver that issues them in the order FESOM2's Fortran ``fct_ale`` does
(:mod:`fesom2_amd.engine`), deterministic synthetic meshes (:mod:`fesom2_amd.synth`) and the node
partition with halo lists for multi-GPU runs (:mod:`fesom2_amd.partition`).
"""
from . import abi, synth  # noqa: F401

__all__ = ["abi", "synth"]
