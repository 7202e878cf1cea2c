#!/usr/bin/env python3
"""Generate the golden FCT-ALE vectors from the reference's OWN code (dev container only).

* a1..a4 (phase 1): src/reference.cpp compiled from /root/reference by oracle/Makefile into
  oracle/_ref/libreference.so, called in the order of its fct_ale_pre_comm_ (reference.cpp:289-304).
* b3v, b3h, c_v, c_h (phase 2): the numpy ``reference()`` functions of the reference's tuning
  scripts kernels/fct_ale_b3_vertical.py:163-181, fct_ale_b3_horizontal.py:76-101,
  fct_ale_c_vertical.py:41-44, fct_ale_c_horizontal.py:53-71.  Those scripts import kernel_tuner
  (not installed, no network) at line 2, so a stub module is put in sys.modules first; bytecode
  writing is disabled so nothing is written under /root/reference.  They use one stride
  ``max_levels`` for every array, so inputs are re-laid out to that stride and results back.

Outputs (committed, data only):
  tests/golden/<name>.npz        inputs + outputs of small meshes, all arrays
  tests/golden/hashes.json       sha256 of every output of the 8k x 20 parity mesh

Run:  python tests/golden/make_golden.py      (needs /root/reference and ``make -C oracle``)
"""
import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "fesom2-accelerate_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from fesom2_amd import synth  # noqa: E402
import oracle as O  # noqa: E402

REF_KERNELS = "/root/reference/kernels"


def load_ref_module(fname):
    sys.modules.setdefault("kernel_tuner", types.SimpleNamespace(tune_kernel=None))
    spec = importlib.util.spec_from_file_location("ref_" + fname[:-3], os.path.join(REF_KERNELS, fname))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def restride(a, ncols, s_from, s_to):
    """(s_from, ncols) column-major -> (s_to, ncols), padding with zeros."""
    out = np.zeros(ncols * s_to)
    k = min(s_from, s_to)
    out.reshape(ncols, s_to)[:, :k] = np.asarray(a)[: ncols * s_from].reshape(ncols, s_from)[:, :k]
    return out


def reference_pass(m, f, dt=1.0):
    """Full pass with the reference's own code; returns dict of outputs in the library's layout."""
    L, nl = m.L, m.nl
    p1 = O.ref_pre_comm(m, f, dt=dt)
    if p1 is None:
        raise SystemExit("oracle/_ref/libreference.so missing: run make -C oracle (needs /root/reference)")
    b3v = load_ref_module("fct_ale_b3_vertical.py")
    b3h = load_ref_module("fct_ale_b3_horizontal.py")
    cv = load_ref_module("fct_ale_c_vertical.py")
    ch = load_ref_module("fct_ale_c_horizontal.py")
    plus, minus = p1["plus"], p1["minus"]
    # b3-vertical at stride nl (fct_adf_v is already (nl, nodes))
    adf_v = f["adf_v"].copy()
    b3v.reference(m.N, m.nlev_nod, nl, adf_v, restride(plus, m.N, L, nl), restride(minus, m.N, L, nl))
    # b3-horizontal at stride L (adf_h and plus/minus are (L, .))
    adf_h = f["adf_h"].copy()
    b3h.reference(m.E, m.edges, m.edge_tri, m.nlev_elem, L, adf_h, plus, minus, np.float64)
    # c-vertical at stride nl
    NT = m.N + m.H
    del_v = restride(f["del_v"], NT, L, nl)
    cv.reference(m.N, m.nlev_nod, nl, del_v, restride(f["ttf"], NT, L, nl), restride(f["hnode"], NT, L, nl),
                 restride(f["LO"], NT, L, nl), restride(f["hnode_new"], NT, L, nl), adf_v, dt, f["area"])
    # c-horizontal at stride nl
    del_h = restride(f["del_h"], NT, L, nl)
    ch.reference(m.E, m.edges, m.edge_tri, m.nlev_elem, nl, del_h, restride(adf_h, m.E, L, nl), dt, f["area"],
                 np.float64)
    out = dict(p1)
    out.update(adf_v=adf_v, adf_h=adf_h, del_v=restride(del_v, NT, nl, L), del_h=restride(del_h, NT, nl, L))
    return out


MESH_KEYS = ("elem2D_nodes", "edges", "edge_tri", "nie_num", "nie", "nlev_elem", "nlev_nod")
FIELD_KEYS = ("ttf", "LO", "adf_v", "adf_h", "area", "area_inv", "hnode", "hnode_new", "del_v", "del_h")
OUT_KEYS = ("ttf_max", "ttf_min", "UV", "plus", "minus", "adf_v", "adf_h", "del_v", "del_h")


def save_npz(name, m, f, out):
    arrays = {f"mesh_{k}": getattr(m, k) for k in MESH_KEYS}
    arrays.update({f"in_{k}": f[k] for k in FIELD_KEYS})
    arrays.update({f"out_{k}": out[k] for k in OUT_KEYS})
    arrays["sizes"] = np.array([m.nl, m.N, m.H, m.T, m.E, m.dim], np.int64)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    for name, (nx, ny, nl) in (("tiny_16x8x10", (16, 8, 11)), ("small_24x12x15", (24, 12, 16))):
        m = synth.make_mesh(nx, ny, nl)
        f = synth.make_fields(m)
        out = reference_pass(m, f)
        save_npz(name, m, f, out)
        print("wrote", name)
    m = synth.config_mesh("8k x 20")
    f = synth.make_fields(m)
    out = reference_pass(m, f)
    hashes = {"mesh": "8k x 20", "nx_ny_nl": list(synth.CONFIGS["8k x 20"]), "seed_mesh": 42, "seed_fields": 43,
              "inputs": {k: sha(f[k]) for k in FIELD_KEYS},
              "outputs": {k: sha(out[k]) for k in OUT_KEYS},
              "made_by": "tests/golden/make_golden.py (reference.cpp a1..a4 + reference numpy b3/c)"}
    with open(os.path.join(HERE, "hashes.json"), "w") as fh:
        json.dump(hashes, fh, indent=1)
    print("wrote hashes.json")


if __name__ == "__main__":
    main()
