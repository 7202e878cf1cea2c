"""CPU: the oracle against the reference (reference.cpp build + committed golden vectors).

The oracle (oracle/fct_ale_oracle.c) is the checker of every GPU parity test, so it is pinned first:
* bit-for-bit against src/reference.cpp compiled from /root/reference (oracle/_ref), when present;
* bit-for-bit against tests/golden/*.npz and tests/golden/hashes.json, which were produced by the
  reference's own code (reference.cpp for a1..a4, its numpy reference() functions for b3/c) by
  tests/golden/make_golden.py -- these travel with the repo, so the pin also holds on the GPU box.
"""
import dataclasses
import hashlib
import json
import os

import numpy as np
import pytest

from fesom2_amd import synth

import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load_fixture(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))  # allow_pickle=False (default)
    nl, N, H, T, E, dim = (int(v) for v in z["sizes"])
    m = synth.Mesh(nl=nl, N=N, H=H, T=T, E=E, dim=dim,
                   **{k: z["mesh_" + k] for k in ("elem2D_nodes", "edges", "edge_tri", "nie_num", "nie",
                                                  "nlev_elem", "nlev_nod")},
                   node_gid=np.arange(N + H, dtype=np.int64), edge_gid=np.arange(E, dtype=np.int64), name=name)
    f = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    out = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return m, f, out


@pytest.mark.parametrize("name", ["tiny_16x8x10", "small_24x12x15"])
def test_oracle_matches_golden_vectors(name):
    m, f, want = load_fixture(name)
    got = O.full_pass(m, f)
    for k, w in want.items():
        assert np.array_equal(got[k].view(np.uint64), w.view(np.uint64)), f"{name}: {k} differs"


def test_oracle_matches_golden_hashes_8k_x_20():
    h = json.load(open(os.path.join(GOLDEN, "hashes.json")))
    m = synth.config_mesh(h["mesh"])
    f = synth.make_fields(m)
    for k, v in h["inputs"].items():
        assert sha(f[k]) == v, f"synthetic input {k} is not bit-identical to the fixture's"
    got = O.full_pass(m, f)
    for k, v in h["outputs"].items():
        assert sha(got[k]) == v, f"oracle output {k} differs from the reference's"


MESHES = [("tiny", False, False), ("8k x 20", False, False), ("8k x 20", True, False), ("8k x 20", False, True)]


@pytest.mark.skipif(O.ref() is None, reason="oracle/_ref (reference.cpp build) not present")
@pytest.mark.parametrize("name,full,perm", MESHES)
def test_oracle_matches_reference_cpp(name, full, perm):
    m = synth.config_mesh(name, full_depth=full)
    if perm:
        m = synth.permute_mesh(m)
    f = synth.make_fields(m)
    st, got = O.pre_comm(m, f)
    assert st == 5
    want = O.ref_pre_comm(m, f)
    for k in ("ttf_max", "ttf_min", "plus", "minus", "UV"):
        assert np.array_equal(got[k].view(np.uint64), want[k].view(np.uint64)), k


@pytest.mark.skipif(O.ref() is None, reason="oracle/_ref (reference.cpp build) not present")
@pytest.mark.parametrize("npts,nl,full,numbering", [(3000, 21, False, "scipy"), (2000, 48, True, "scipy"),
                                                    (5000, 12, False, "scipy"), (4000, 21, False, "hilbert")])
def test_oracle_matches_reference_cpp_unstructured(npts, nl, full, numbering):
    """Delaunay meshes: node degrees 3..13 and scattered (or Hilbert-curve) numbering (the structured
    meshes have degree 6)."""
    m = synth.delaunay_mesh(npts, nl, full_depth=full, numbering=numbering)
    assert m.dim > 8
    f = synth.make_fields(m)
    st, got = O.pre_comm(m, f)
    assert st == 5
    want = O.ref_pre_comm(m, f)
    for k in ("ttf_max", "ttf_min", "plus", "minus", "UV"):
        assert np.array_equal(got[k].view(np.uint64), want[k].view(np.uint64)), k


def test_hilbert_numbering_is_a_renumbering():
    """synth.delaunay_mesh(numbering="hilbert") is the same triangulation with nodes along a Hilbert
    curve: same element/edge counts and degree histogram, edges between nearby numbers."""
    a = synth.delaunay_mesh(3000, 11)
    b = synth.delaunay_mesh(3000, 11, numbering="hilbert")
    assert (a.N, a.T, a.E, a.dim) == (b.N, b.T, b.E, b.dim)
    assert np.array_equal(np.sort(a.nie_num), np.sort(b.nie_num))
    e = b.edges.reshape(-1, 2).astype(np.int64)
    assert np.median(np.abs(e[:, 0] - e[:, 1])) < 16 < np.median(np.abs(np.diff(a.edges.reshape(-1, 2), axis=1)))
    # every element's nodes are its nod_in_elem2D entries' owners
    en = b.elem2D_nodes.reshape(-1, 3) - 1
    nie = b.nie.reshape(b.N, b.dim)
    for n in range(0, b.N, 97):
        els = nie[n, : b.nie_num[n]] - 1
        assert np.all(np.any(en[els] == n, axis=1))
    k = synth.hilbert_key(np.array([[(i + .5) / 4, (j + .5) / 4] for i in range(4) for j in range(4)]), bits=2)
    assert sorted(k) == list(range(16))


def test_vlimit_protocol_of_reference_cpp():
    """reference.cpp runs a3/a4 only for vlimit == 1 and reports alg_state 2 otherwise (:297-303)."""
    m = synth.config_mesh("tiny")
    f = synth.make_fields(m)
    for vl in (2, 3):
        st, _ = O.pre_comm(m, f, vlimit=vl, vlimit_ext=False)
        assert st == 2
        st, _ = O.pre_comm(m, f, vlimit=vl, vlimit_ext=True)
        assert st == 5


def test_limiter_is_active_on_synthetic_fields():
    """The synthetic scales must exercise b2/b3 (ratios below 1 in a good share of cells)."""
    m = synth.config_mesh("8k x 20")
    f = synth.make_fields(m)
    _, out = O.pre_comm(m, f)
    L = m.L
    wet = np.arange(L)[None, :] < (m.nlev_nod[:, None] - 1)
    plus = out["plus"].reshape(-1, L)[wet]
    assert 0.1 < np.mean(plus < 1.0) < 0.9
    assert plus.min() >= 0.0


def test_mesh_generator_conventions():
    m = synth.config_mesh("8k x 20")
    nx, ny, nl = synth.CONFIGS["8k x 20"]
    assert (m.N, m.T, m.E) == (nx * ny, 2 * nx * (ny - 1), 3 * nx * (ny - 1) + nx)
    en = m.elem2D_nodes.reshape(-1, 3) - 1
    # nlevels_nod2D = max over adjacent elements
    mx = np.zeros(m.N, np.int32)
    np.maximum.at(mx, en.reshape(-1), np.repeat(m.nlev_elem, 3))
    assert np.array_equal(mx, m.nlev_nod)
    assert m.nlev_elem.min() >= 3 and m.nlev_elem.max() <= nl
    # every edge's first element contains both endpoints; second is 0 only on the y boundary
    ed = m.edges.reshape(-1, 2) - 1
    et = m.edge_tri.reshape(-1, 2)
    assert (et[:, 0] > 0).all()
    for k in (0, 1):
        has = et[:, k] > 0
        tri = en[et[has, k] - 1]
        assert ((tri == ed[has, 0:1]).any(1) & (tri == ed[has, 1:2]).any(1)).all()
    # nod_in_elem2D lists exactly the adjacent elements
    nie = m.nie.reshape(-1, m.dim)
    cnt = np.bincount(en.reshape(-1), minlength=m.N)
    assert np.array_equal(cnt, m.nie_num)
    assert cnt.max() <= m.dim


def test_survey_config_sizes():
    """SURVEY.md §8 / BASELINE.md: 1.2M x 80 mesh has 2,396,800 elements and 3,596,800 edges."""
    m = synth.config_mesh("1.2M x 80", full_depth=True)
    assert (m.N, m.T, m.E, m.L) == (1_200_000, 2_396_800, 3_596_800, 80)
    assert m.cells == 96_000_000


def test_permuted_mesh_describes_the_same_problem():
    """Renumbering must not change the physics: per-global-id results agree up to the order of the
    edge sums (renumbered edges are added in a different order, so only rounding may differ)."""
    m = synth.config_mesh("tiny")
    p = synth.permute_mesh(m)
    a = O.full_pass(m, synth.make_fields(m))
    b = O.full_pass(p, synth.make_fields(p))
    L = m.L
    for k in ("plus", "minus", "del_v", "del_h"):
        A = a[k].reshape(-1, L)[p.node_gid]
        assert np.allclose(A, b[k].reshape(-1, L), rtol=1e-12, atol=1e-14), k
    assert np.allclose(a["adf_h"].reshape(-1, L)[p.edge_gid], b["adf_h"].reshape(-1, L), rtol=1e-12, atol=1e-14)


def test_empty_edge_set_and_minimum_levels():
    """Edge cases the reference's loops admit: no edges (b1h/b3h/ch are no-ops), nlevels = 3."""
    m = synth.make_mesh(4, 2, 3)
    f = synth.make_fields(m)
    st, out = O.pre_comm(dataclasses.replace(m, E=0), f)
    assert st == 5
    full = O.full_pass(m, f)
    assert np.isfinite(full["plus"]).all()


def _fortran_iter_phase2(m, f, plus, minus, adf_v2, adf_h2, dt=1.0):
    """docs/refactoring.md:204-290 with iter_yn true, transcribed statement by statement in plain
    Python floats (1-based Fortran loops shifted to 0-based)."""
    L, nl = m.L, m.nl
    av, ah = list(f["adf_v"]), list(f["adf_h"])
    av2, ah2, LO = list(adf_v2), list(adf_h2), list(f["LO"])
    P, M, area, hnn = list(plus), list(minus), list(f["area"]), list(f["hnode_new"])
    for n in range(m.N):
        a, b = n * nl, n * L
        ae = 1.0
        ae = min(ae, P[b]) if av[a] >= 0.0 else min(ae, M[b])
        av[a] = ae * av[a]
        for z in range(1, int(m.nlev_nod[n]) - 1):
            ae = 1.0
            if av[a + z] >= 0.0:
                ae = min(ae, M[b + z - 1]); ae = min(ae, P[b + z])
            else:
                ae = min(ae, P[b + z - 1]); ae = min(ae, M[b + z])
            av2[a + z] = (1.0 - ae) * av[a + z]
            av[a + z] = ae * av[a + z]
    ed, et = m.edges.reshape(-1, 2) - 1, m.edge_tri.reshape(-1, 2)
    lev = [max(int(m.nlev_elem[et[e, 0] - 1]) - 1, int(m.nlev_elem[et[e, 1] - 1]) - 1 if et[e, 1] > 0 else 0)
           for e in range(m.E)]
    for e in range(m.E):
        n1, n2 = ed[e]
        for z in range(lev[e]):
            i = e * L + z
            ae = 1.0
            if ah[i] >= 0.0:
                ae = min(ae, P[n1 * L + z]); ae = min(ae, M[n2 * L + z])
            else:
                ae = min(ae, M[n1 * L + z]); ae = min(ae, P[n2 * L + z])
            ah2[i] = (1.0 - ae) * ah[i]
            ah[i] = ae * ah[i]
    for n in range(m.N):
        for z in range(int(m.nlev_nod[n]) - 1):
            LO[n * L + z] = LO[n * L + z] + (av[n * nl + z] - av[n * nl + z + 1]) * dt / area[n * nl + z] / hnn[n * L + z]
    for e in range(m.E):
        n1, n2 = ed[e]
        for z in range(lev[e]):
            LO[n1 * L + z] = LO[n1 * L + z] + ah[e * L + z] * dt / area[n1 * nl + z] / hnn[n1 * L + z]
            LO[n2 * L + z] = LO[n2 * L + z] - ah[e * L + z] * dt / area[n2 * nl + z] / hnn[n2 * L + z]
    return dict(LO=np.array(LO), adf_v=np.array(av2), adf_h=np.array(ah2), adf_v2=np.array(av2), adf_h2=np.array(ah2))


def test_oracle_iter_yn_matches_fortran_transcription():
    """The C restatement of the iter_yn branch (oracle_b3v/b3h with adf2, oracle_lo_update) against
    a line-by-line Python transcription of the Fortran; nonzero initial adf_v2/adf_h2 check that
    unassigned levels are carried through the whole-array swap."""
    m = synth.config_mesh("tiny")
    f = synth.make_fields(m)
    st, p1 = O.pre_comm(m, f)
    assert st == 5
    rng = np.random.default_rng(11)
    v2, h2 = rng.standard_normal(f["adf_v"].size), rng.standard_normal(f["adf_h"].size)
    got = O.post_comm_iter(m, f, p1["plus"], p1["minus"], v2, h2)
    want = _fortran_iter_phase2(m, f, p1["plus"], p1["minus"], v2, h2)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    assert not np.array_equal(got["LO"], f["LO"])


def test_iterated_pass_with_one_iteration_is_the_plain_pass():
    m = synth.config_mesh("tiny")
    f = synth.make_fields(m)
    a, b = O.full_pass(m, f), O.iterated_pass(m, f, 1)
    for k in ("adf_v", "adf_h", "del_v", "del_h"):
        assert np.array_equal(a[k], b[k])
